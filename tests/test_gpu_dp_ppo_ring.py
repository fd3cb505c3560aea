"""Data-parallel PPO_AcM ACM regression with no per-batch collective (acm/acm.py:266-303,
acm/on_policy.py:78-82): the ACM ring is replicated -- every rank writes every rank's
transitions, in rank order, at the end of each iteration (ReplayBufferAcM.add_buffer,
replay_buffer.py:284-297) -- and every rank runs the same update_acm epochs (multi-workgroup
sppAcmSgd, one shared permutation stream) on its identical ring.

2 processes on one GPU over gloo (CUDA tensors), different env seeds per rank.  Checks:
  - after 2 iterations (pre-train, then ACM updates every iteration) both ranks' AcM parameters, ring
    contents and obs statistics are BIT-IDENTICAL;
  - the ring equals the union of the ranks' own transitions in rank order: each rank records the
    next-obs rows it produced in every flush (pre-train, each iteration); the ring's timestep rows
    are, flush by flush, rank 0's rows then rank 1's, bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rank_results import collect

pytestmark = pytest.mark.gpu

E, T, OB, AC = 64, 4, 17, 6
KW = dict(env_name="HalfCheetah-v2", batch_size=E * T, ppo_batch_size=128, max_ppo_epochs=2, acm_epochs=2,
          acm_batch_size=200, acm_update_freq=1, acm_pre_train_samples=2 * E * 8, acm_pre_train_epochs=1,
          acm_ring_size=8192, n_envs=E, seed=3)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ring(ag):
    rb = ag.replay_buffer
    n = len(rb)
    obs, nobs, act, rew, done, acm = rb.gather(torch.arange(n, device=ag.device))
    return n, torch.cat([obs, nobs, acm, rew[:, None]], 1).cpu().numpy()


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        import spprl

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        ag = spprl.PPO_AcM(device=dev, loop_seed=100 + 1000 * rank, **KW)
        assert ag.world == 2
        acm0 = ag.acm.params[5].cpu().clone()
        own = []
        flush = ag._flush_ring

        def recording_flush():  # this rank's own rows of each flush, then the real (replicating) flush
            rows = [r[1] for r in ag._ring_log if r[0] == "step"]
            if rows:
                own.append(torch.cat(rows).cpu().numpy())
            flush()

        ag._flush_ring = recording_flush
        ag.pre_train()
        for _ in range(2):
            ag.perform_iteration(sync=False)
            ag.iteration += 1
        torch.cuda.synchronize()
        n, ring = _ring(ag)
        rb = ag.replay_buffer
        q.put((rank, own, acm0.numpy(), ag.acm.params[5].cpu().numpy(), n, ring, rb.obs_mean.cpu().numpy(),
               rb.max_obs.cpu().numpy(), rb.min_obs.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def test_dp_ppo_replicated_acm_ring_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = collect(q, procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    own = {r: res[r][0] for r in res}
    a, b = res[0][1:], res[1][1:]
    np.testing.assert_array_equal(a[0], b[0])  # same initial AcM (same seed)
    assert a[2] == b[2]
    for x, y in zip(a[1:], b[1:]):
        np.testing.assert_array_equal(x, y)  # AcM after the epochs, ring, obs statistics
    n, ring = a[2], a[3]
    assert n == 2 * (KW["acm_pre_train_samples"] + 2 * E * T)
    assert len(own[0]) == len(own[1]) == 3  # pre-train + 2 iterations
    want = np.concatenate([blk for k in range(3) for blk in (own[0][k], own[1][k])])
    np.testing.assert_array_equal(ring[:, OB:2 * OB], want)
    assert not np.array_equal(own[0][1], own[1][1])  # different env seeds: different rows
