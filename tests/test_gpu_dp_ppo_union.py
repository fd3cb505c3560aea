"""Data-parallel PPO_AcM update on the replicated union batch (acm/on_policy.py:72-75,
algorithms/a2c/a2c.py:186-225, algorithms/ppo/ppo.py:152-192): each rank collects its own rollout [T][E], one
all-gather builds the union [T][world x E] (rank-major along the env axis), and every rank runs the persistent
critic steps (sppOnpCriticSteps) and actor epochs (sppOnpActorEpoch) on it -- no per-step gradient exchange.

2 processes on one GPU over gloo, different env seeds per rank.  Checks: after update(mem) both ranks' actor
and critic parameters are BIT-IDENTICAL, and equal -- bit for bit -- those of ONE process (no process group)
that runs update() on the concatenated batch with the same initial networks and permutation seed.
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

E, T = 64, 8
KW = dict(env_name="HalfCheetah-v2", batch_size=E * T, ppo_batch_size=256, max_ppo_epochs=3, acm_epochs=1,
          acm_batch_size=64, acm_update_freq=0, acm_pre_train_samples=1000, acm_pre_train_epochs=1,
          acm_ring_size=8192, critic_num_target_updates=2, num_critic_updates_per_target=3, kl_div_threshold=1e9,
          custom_loss=0.1, seed=3, dp_update="union")
MEM = ("obs", "act", "lp", "rew", "done", "end", "next_obs")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        import spprl

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        ag = spprl.PPO_AcM(device=dev, n_envs=E, loop_seed=100 + 1000 * rank, **KW)
        assert ag.dp and ag.world == 2 and ag.nets.allreduce is None
        assert ag.nets._critic_kernel_ok(2 * E * T) and ag.nets._epoch_kernel_ok(256)
        mem = ag.collect_batch()
        own = {k: mem[k].cpu().numpy() for k in MEM}
        ag.update(mem)
        torch.cuda.synchronize()
        q.put((rank, own, ag.nets.params[0].cpu().numpy(), ag.nets.params[1].cpu().numpy(), ag.nets.last_epochs,
               dict(ag.loss)))
    finally:
        dist.destroy_process_group()


def test_dp_ppo_update_on_union_equals_one_process():
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
    (own0, a0, c0, ep0, l0), (own1, a1, c1, ep1, l1) = res[0], res[1]
    np.testing.assert_array_equal(a0, a1)
    np.testing.assert_array_equal(c0, c1)
    assert ep0 == ep1 == KW["max_ppo_epochs"] and l0 == l1
    assert not np.array_equal(own0["obs"], own1["obs"])  # different env seeds: different shards
    # one process, no process group, the same networks and permutation seed, on the concatenated batch
    import spprl

    dev = torch.device("cuda", 0)
    one = spprl.PPO_AcM(device=dev, n_envs=2 * E, **dict(KW, batch_size=2 * E * T))
    assert not one.dp
    u = {k: torch.from_numpy(np.concatenate([own0[k], own1[k]], axis=1)).to(dev) for k in MEM}
    u["T"] = T
    one.update(u)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(one.nets.params[0].cpu().numpy(), a0)
    np.testing.assert_array_equal(one.nets.params[1].cpu().numpy(), c0)
    assert one.loss == l0
