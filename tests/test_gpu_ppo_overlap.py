"""PPO_AcM's ACM update beside update(mem) (spprl/ppo_acm.py perform_iteration): the ACM epochs run on a side
stream while the critic steps and the actor epochs run on the main one, their persistent grids sized to leave
the ACM grid's workgroup slots free (sppOnpReserveWorkgroups).  The two updates touch disjoint networks and
data (the ACM trains on the already flushed ring; update(mem) never reads the ACM), so the overlapped
iteration must leave every network and every loss BIT-IDENTICAL to the serial order of the reference
(acm/on_policy.py:52-75: update(mem), then update_acm).  Multi-workgroup ACM steps (acm_batch_size 200: 4
workgroups) and persistent critic / actor kernels on a 1-GPU process; SPP_PPO_ACM_OVERLAP=0 is the serial
order.  The critic grid always leaves 64 slots free (kCriticSideSlots), so its row partition and summation
order are the same in both orders at any N (here 16,384 rows: 2 passes per workgroup)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

E, T = 2048, 8  # N = 16,384 critic rows: 2 passes of 64 rows on 128 workgroups in both orders
KW = dict(env_name="HalfCheetah-v2", batch_size=E * T, ppo_batch_size=512, max_ppo_epochs=3, acm_epochs=2,
          acm_batch_size=200, acm_update_freq=1, acm_pre_train_samples=E * 8, acm_pre_train_epochs=1,
          acm_ring_size=65536, n_envs=E, seed=5)


def _run(monkeypatch, overlap):
    import spprl

    monkeypatch.setenv("SPP_PPO_ACM_OVERLAP", "1" if overlap else "0")
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ag = spprl.PPO_AcM(device=dev, loop_seed=77, **KW)
    ag.pre_train()
    used = []
    for _ in range(3):
        used.append(ag._acm_side_stream() is not None)
        ag.perform_iteration(sync=False)
        ag.iteration += 1
    torch.cuda.synchronize()
    ag.acm.check_acm_sgd()
    ag.nets.check_actor_epochs()
    nets = [p.cpu().numpy().copy() for p in ag.nets.params] + [ag.acm.params[5].cpu().numpy().copy()]
    return used, nets, dict(ag.loss), ag.acm.acm_loss


def test_overlapped_acm_update_is_bit_identical_to_serial(monkeypatch):
    used1, nets1, loss1, acm1 = _run(monkeypatch, True)
    used0, nets0, loss0, acm0 = _run(monkeypatch, False)
    assert all(used1) and not any(used0)
    for a, b in zip(nets1, nets0):
        np.testing.assert_array_equal(a, b)
    for k in ("critic", "actor", "entropy", "kl", "dist", "policy"):
        assert loss1[k] == loss0[k], k
    assert acm1 == acm0
