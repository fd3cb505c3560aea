"""Data-parallel PPO_AcM with the sharded update (dp_update="shard"; acm/on_policy.py:72-75,
algorithms/a2c/a2c.py:186-225, algorithms/ppo/ppo.py:152-192): every rank updates on its own rollout and
all-reduces each critic step's and each clip-loss step's gradient (the global minibatch ppo_batch_size split over
the ranks), so the replicas stay bit-identical without any rollout exchange.

2 processes on one GPU over gloo, different env seeds per rank.  Checks:
  - after a whole update(mem) (critic targets, GAE, actor epochs with the KL stop) both ranks' actor and critic
    parameters, epochs run and losses are identical;
  - the critic's full-batch steps on two half batches with the averaged gradient track ONE process's critic steps
    on the union batch (the reference's mean-loss gradient of the union, a2c.py:209-219): the same gradient up to
    the summation order, so parameters within fp32 rounding plus the Adam first-step allowance.
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
          custom_loss=0.1, seed=3, dp_update="shard")


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
        assert ag.dp and ag.world == 2 and ag.nets.allreduce is not None and ag.nets.shards == 2
        assert not ag.nets._critic_kernel_ok(E * T) and not ag.nets._epoch_kernel_ok(128)
        mem = ag.collect_batch()
        n = mem["T"] * E
        shard = {k: mem[k].reshape(n, -1).cpu().numpy() for k in ("obs", "next_obs", "rew", "done")}
        c_init = ag.nets.params[1].clone()
        # the critic steps alone on this rank's half, from the initial critic (restored afterwards)
        nets = ag.nets
        obs, nobs = mem["obs"].reshape(n, -1), ag.normalize(mem["next_obs"].reshape(n, -1))
        m_init, v_init = nets.m[1].clone(), nets.v[1].clone()
        nets.update_critic(obs, nobs, mem["rew"].reshape(n), mem["done"].reshape(n).float())
        torch.cuda.synchronize()
        c_only = nets.params[1].cpu().numpy().copy()
        nobs_h = nobs.cpu().numpy()
        # back to the initial critic and Adam moments (the handle's step count moves on, alike on both ranks),
        # then the whole update
        nets.params[1].copy_(c_init)
        nets.m[1].copy_(m_init)
        nets.v[1].copy_(v_init)
        ag.update(mem)
        torch.cuda.synchronize()
        q.put((rank, shard, nobs_h, c_init.cpu().numpy(), c_only, ag.nets.params[0].cpu().numpy(),
               ag.nets.params[1].cpu().numpy(), ag.nets.last_epochs, dict(ag.loss)))
    finally:
        dist.destroy_process_group()


def test_dp_ppo_sharded_update_keeps_replicas_identical_and_critic_matches_union():
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
    (sh0, nx0, ci0, co0, a0, c0, ep0, l0), (sh1, nx1, ci1, co1, a1, c1, ep1, l1) = res[0], res[1]
    np.testing.assert_array_equal(a0, a1)
    np.testing.assert_array_equal(c0, c1)
    np.testing.assert_array_equal(co0, co1)
    assert ep0 == ep1 == KW["max_ppo_epochs"]
    assert l0["actor"] == l1["actor"] and l0["kl"] == l1["kl"]
    assert not np.array_equal(sh0["obs"], sh1["obs"])  # different env seeds: different shards
    np.testing.assert_array_equal(ci0, ci1)
    # one process, no process group: the same critic steps on the union batch
    import spprl

    dev = torch.device("cuda", 0)
    one = spprl.PPO_AcM(device=dev, n_envs=2 * E, **dict(KW, batch_size=2 * E * T))
    assert not one.dp
    one.nets.params[1].copy_(torch.from_numpy(ci0).to(dev))
    cat = lambda k: torch.from_numpy(np.concatenate([sh0[k], sh1[k]])).to(dev)  # noqa: E731
    one.nets.update_critic(cat("obs"), torch.from_numpy(np.concatenate([nx0, nx1])).to(dev),
                           cat("rew").reshape(-1), cat("done").reshape(-1).float())
    torch.cuda.synchronize()
    got, ref = co0, one.nets.params[1].cpu().numpy()
    steps = KW["critic_num_target_updates"] * KW["num_critic_updates_per_target"]
    d = np.abs(got - ref)
    assert d.max() <= 2 * steps * 3e-4 * 1.01, d.max()  # Adam's first steps: a sign flip costs <= 2 lr per step
    assert np.mean(d > 1e-5) < 5e-3, np.mean(d > 1e-5)
    assert np.abs(got - ci0).max() > 1e-4  # the critic did move
