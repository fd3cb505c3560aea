"""GPU: last_rollout (rltoolkit/buffer/replay_buffer.py:170-218, :335-383) against the oracle's
restatement of the reference walk (bit-exact indices and gathered values) on single-env episode
streams that exercise the time limit, early terminations, a ring wrap (Q6), the ts_idx == 0 case and
a buffer with one end; the native RCCL exchange (sppCommInitRank / sppAllReduceGrads) on a 1-rank
communicator (the sum over one rank is the identity, so grads must be unchanged bit for bit);
and the TensorBoard scalar sink wired into the fused training loop."""
import ctypes

import numpy as np
import pytest
import torch

import spprl
from spprl import _lib
from spprl._lib import call, ptr, stream_handle
from oracle.replay import OracleReplay

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _episodes(size, ob, aout, ac, ep_lens, seed):
    """Both rings driven by the reference's single-env loop (ddpg.py:182-223): reset obs, then per
    step add_acm_action + add_obs(next) + add_timestep(end at episode end)."""
    rng = np.random.RandomState(seed)
    rb = spprl.BufferAcMOffPolicy(size, ob, aout, ac, device=DEV)
    orb = OracleReplay(size, ob, aout, ac)
    for L in ep_lens:
        o = rng.randn(ob).astype(np.float32)
        prev = rb.add_obs(torch.from_numpy(o))
        assert prev == orb.add_obs(o)
        for t in range(L):
            a = rng.randn(aout).astype(np.float32)
            m = rng.randn(ac).astype(np.float32)
            r = float(np.float32(rng.randn()))
            no = rng.randn(ob).astype(np.float32)
            end = t == L - 1
            rb.add_acm_action(torch.from_numpy(m))
            orb.add_acm_action(m)
            nxt = rb.add_obs(torch.from_numpy(no))
            assert nxt == orb.add_obs(no)
            done = bool(end and rng.rand() < 0.5)  # terminal vs time-limit end
            rb.add_timestep(prev, nxt, torch.from_numpy(a), r, done, end)
            orb.add_timestep(prev, nxt, a, r, done, end)
            prev = nxt
    assert (rb.ts_idx, len(rb)) == (orb.ts_idx, len(orb))
    return rb, orb


@pytest.mark.parametrize("size,ep_lens", [(200, [5, 7, 3, 9]),          # plain
                                          (40, [6, 11, 4, 13, 8, 10]),   # obs ring wraps (Q6)
                                          (64, [63]),                    # one end in the buffer
                                          (30, [4, 9, 5, 6, 3])])
def test_last_rollout_matches_reference_walk(size, ep_lens):
    rb, orb = _episodes(size, 5, 5, 2, ep_lens, seed=size)
    m = rb.last_rollout()
    obs, act, rew, dones, acm, ts = orb.last_rollout()
    assert len(m) == len(rew)
    np.testing.assert_array_equal(m.obs.cpu().numpy(), obs[:-1])
    np.testing.assert_array_equal(m.next_obs.cpu().numpy(), obs[1:])
    np.testing.assert_array_equal(m.actions.cpu().numpy(), act)
    np.testing.assert_array_equal(m.rewards.cpu().numpy(), rew)
    np.testing.assert_array_equal(m.actions_acm.cpu().numpy(), acm)
    np.testing.assert_array_equal(m.end.cpu().numpy(), dones)
    assert m.rollouts_no == 1
    assert m.returns_rollouts[0] == pytest.approx(float(np.sum(rew.astype(np.float64))))


def test_last_rollout_needs_an_end():
    rb = spprl.BufferAcMOffPolicy(50, 3, 3, 1, device=DEV)
    s = rb.add_obs(torch.zeros(3))
    for _ in range(4):
        n = rb.add_obs(torch.ones(3))
        rb.add_timestep(s, n, torch.zeros(3), 0.0, False, False)
        s = n
    with pytest.raises(_lib.SppError):
        rb.last_rollout()


def test_replay_create_ex_validates_modes():
    h = ctypes.c_void_p()
    for args in ((4, 0, 0), (4, 1, 1), (0, 1, 0)):
        with pytest.raises(_lib.SppError):
            call("sppReplayCreateEx", ctypes.byref(h), 100, 3, 3, 1, *args, 0)
    call("sppReplayCreateEx", ctypes.byref(h), 100, 3, 3, 1, 8, 1, 0, 0)
    call("sppReplayDestroy", h)


def test_native_comm_allreduce_one_rank_is_identity():
    uid = ctypes.create_string_buffer(_lib.SPP_COMM_ID_BYTES)
    call("sppCommGetUniqueId", uid)
    comm = ctypes.c_void_p()
    call("sppCommInitRank", ctypes.byref(comm), 1, uid, 0, 0)
    try:
        ag = spprl.SAC_AcM(env_name="Hopper-v2", buffer_size=64, max_batch=64, device=DEV, seed=0)
        B, ob, aout, ac = 64, 11, 11, 3
        rng = np.random.RandomState(0)
        batch = (rng.randn(B, ob).astype(np.float32), rng.randn(B, ob).astype(np.float32),
                 rng.uniform(-1, 1, (B, aout)).astype(np.float32), rng.randn(B).astype(np.float32),
                 np.zeros(B, np.int8), rng.uniform(-1, 1, (B, ac)).astype(np.float32))
        ag.update(*batch, eps_next=rng.randn(B, aout).astype(np.float32),
                  eps_cur=rng.randn(B, aout).astype(np.float32))
        torch.cuda.synchronize()
        before = [t.clone() for t in (ag.bucket_critic, ag.bucket_actor, ag.bucket_acm)]
        for b in (_lib.SPP_BUCKET_CRITIC, _lib.SPP_BUCKET_ACTOR, _lib.SPP_BUCKET_ACM, _lib.SPP_BUCKET_ALL):
            call("sppAllReduceGrads", ag._h, b, 1, comm, stream_handle())
        torch.cuda.synchronize()
        for t0, t1 in zip(before, (ag.bucket_critic, ag.bucket_actor, ag.bucket_acm)):
            assert torch.equal(t0, t1)
    finally:
        call("sppCommDestroy", comm)


def test_training_loop_writes_tensorboard_scalars(tmp_path):
    from spprl.tb import read_scalars

    ag = spprl.SAC_AcM(env_name="Hopper-v2", n_envs=64, batch_size=512, iterations=6, buffer_size=20_000,
                       random_frames=128, update_freq=1, grad_steps=1, acm_update_freq=64, acm_update_batches=1,
                       acm_pre_train_samples=256, acm_pre_train_epochs=1, device=DEV, seed=0,
                       tensorboard_dir=str(tmp_path), debug_mode=True, env_spec=(11, 3, 1.0, 40))
    ag.pre_train()
    ag.train()
    tags = {t for _, t, _ in read_scalars(ag.tensorboard_writer.path)}
    assert {"Loss/Critic_1", "Loss/Critic_2", "Loss/Actor", "SAC/Alpha_per_iterations"} <= tags
    m = ag.replay_buffer.last_rollout()  # after real episodes of the loop
    assert len(m) >= 1 and bool(m.end[-1])


def test_native_comm_wrapper_drives_the_dp_update():
    from spprl.dp import NativeComm

    nc = NativeComm(0, 1, 0, lambda b: b)
    try:
        ag = spprl.SAC_AcM(env_name="Hopper-v2", buffer_size=64, max_batch=64, device=DEV, seed=0)
        ar = nc.allreduce_for(ag)
        for b in (ag.bucket_critic, ag.bucket_actor, ag.bucket_acm):
            ar(b)
        torch.cuda.synchronize()
    finally:
        nc.close()


def test_native_comm_attach_provides_the_statistics_exchange():
    """NativeComm.attach sets all three exchanges a data-parallel agent needs (gradient buckets,
    obs-statistics sums through sppCommAllReduceSum, host row counts); an explicit gradient exchange
    without a statistics exchange is refused (the replicas' normalisers would drift apart)."""
    from spprl.dp import NativeComm

    nc = NativeComm(0, 1, 0, lambda b: b)
    try:
        ag = spprl.SAC_AcM(env_name="Hopper-v2", buffer_size=64, max_batch=64, device=DEV, seed=0)
        nc.attach(ag)
        assert ag.allreduce is not None and ag.allreduce_sum is not None and ag.host_sum is not None
        for dt in (torch.float32, torch.float64, torch.int32, torch.int64):
            t = torch.arange(7, device=DEV).to(dt)
            nc.allreduce_sum(t)  # one rank: the sum is the identity
            torch.cuda.synchronize()
            assert torch.equal(t.cpu(), torch.arange(7).to(dt))
        assert nc.host_sum([3, 4]) == [3, 4] and nc.host_sum(9) == 9
        with pytest.raises(ValueError, match="allreduce_sum"):
            spprl.SAC_AcM(env_name="Hopper-v2", buffer_size=64, max_batch=64, device=DEV, seed=0,
                          allreduce=lambda b: None)
    finally:
        nc.close()


def test_host_synth_env_matches_device_dynamics_and_runs_the_loop():
    from spprl import HostSynthEnv, SynthVecEnv

    E, ob, ac = 256, 11, 3
    h = HostSynthEnv(E, ob, ac, max_episode_steps=5, seed=3, device=DEV)
    d = SynthVecEnv(E, ob, ac, max_episode_steps=5, seed=3, device=DEV)
    o = h.reset().clone()
    d.reset()
    d.obs.copy_(o)
    rng = np.random.RandomState(0)
    for t in range(5):
        a = torch.from_numpy(rng.uniform(-1, 1, (E, ac)).astype(np.float32)).to(DEV)
        ho, hr, hend, _ = h.step(a)
        do, dr, dend, _ = d.step(a)
        torch.testing.assert_close(ho, do, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(hr, dr, rtol=1e-5, atol=1e-5)
        assert (hend == dend).all() and bool(hend.all()) == (t == 4)
    ag = spprl.SAC_AcM(env_name="Hopper-v2", n_envs=E, batch_size=4 * E, iterations=2, buffer_size=20_000,
                       random_frames=E, update_freq=1, grad_steps=1, acm_update_freq=E, acm_update_batches=1,
                       device=DEV, seed=0, env=HostSynthEnv(E, ob, ac, max_episode_steps=3, seed=1, device=DEV))
    ag.train()
    torch.cuda.synchronize()
    assert len(ag.replay_buffer) == 8 * E and np.isfinite(ag.loss["critic_1"])
