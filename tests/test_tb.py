"""TensorBoard-compatible scalar sink (spprl/tb.py; rltoolkit/tensorboard_logger.py:173-364 scalar
methods): CRC-32C known answer, the TFRecord framing (both masked CRCs checked on read-back), the
reference's tags and step axes, corruption detection."""
import os

import pytest

from spprl.tb import TensorboardWriter, crc32c, read_scalars


def test_crc32c_known_answer():
    assert crc32c(b"123456789") == 0xE3069283  # the CRC-32C check value
    assert crc32c(b"") == 0


def test_scalar_events_round_trip(tmp_path):
    w = TensorboardWriter(str(tmp_path))
    w.log_running_return(3, 3000, 2, -12.5)
    w.log_test_return(3, 3000, 2, 4.25)
    w.log_loss(3, {"critic_1": 0.5, "actor": -1.0})
    w.log_acm_pretrain_loss(0.125, 0.25, 7)
    w.log_sac_alpha(3, 0.2)
    w.log_kl_div_updates(4, 4000, 3, 2.0)
    w.log_obs_mean_std(5, [1.0, 2.0], [3.0, 4.0])
    w.close()
    files = os.listdir(str(tmp_path))
    assert len(files) == 1 and files[0].startswith("events.out.tfevents.")
    got = read_scalars(w.path)
    exp = [(3, "1_Running_return/per_iterations", -12.5), (3000, "1_Running_return/per_frames", -12.5),
           (2, "1_Running_return/per_rollouts", -12.5), (3, "1_Test_return/per_iterations", 4.25),
           (3000, "1_Test_return/per_frames", 4.25), (2, "1_Test_return/per_rollouts", 4.25),
           (3, "Loss/Critic_1", 0.5), (3, "Loss/Actor", -1.0), (7, "Loss/pretrain_acm_train", 0.125),
           (7, "Loss/pretrain_acm_val", 0.25), (3, "SAC/Alpha_per_iterations", pytest.approx(0.2)),
           (4, "PPO/KL_updates_mean/per_iterations", 2.0), (4000, "PPO/KL_updates_mean/per_frames", 2.0),
           (3, "PPO/KL_updates_mean/per_rollouts", 2.0), (5, "Obs/mean/0", 1.0), (5, "Obs/std/0", 3.0),
           (5, "Obs/mean/1", 2.0), (5, "Obs/std/1", 4.0)]
    assert got == exp


def test_corrupted_record_is_detected(tmp_path):
    w = TensorboardWriter(str(tmp_path))
    w.add_scalar("x", 1.0, 1)
    w.close()
    with open(w.path, "r+b") as f:
        data = bytearray(f.read())
        data[-6] ^= 0xFF  # inside the last event's payload
        f.seek(0)
        f.write(data)
    with pytest.raises(ValueError):
        read_scalars(w.path)


def test_logging_after_close_reopens_the_event_file(tmp_path):
    """train() closes the writer on its last iteration (rl.py:229-235); a later train() or test log call
    appends to the same event file instead of failing."""
    w = TensorboardWriter(str(tmp_path))
    w.add_scalar("x", 1.0, 1)
    w.close()
    w.add_scalar("x", 2.0, 2)
    w.flush()
    w.close()
    assert read_scalars(w.path) == [(1, "x", 1.0), (2, "x", 2.0)]
