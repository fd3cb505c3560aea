"""Data-parallel exchange of the SAC_AcM update, world size 2 over gloo on CPU.

Each rank runs the grads half of the update on its shard of the golden batch
(the oracle stands in for the device kernels, which need a GPU), averages the
flat buckets with ``spprl.dp.make_allreduce`` (the same callable bench.py hands
to ``SAC_AcM.update_from_replay_dp``), then applies.  Checks: the averaged
buckets equal the full-batch gradients, both replicas end bit-identical, and
the post-step parameters match a single-process full-batch update.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from golden_cases import sac_case

CASE = "sac_hopper_paper"
WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _make_oracle(cfg, params, norm, ob, aout, ac):
    from oracle.sac_acm import OracleSacAcm
    return OracleSacAcm(ob, aout, ac, acm_critic=cfg["acm_critic"], custom_loss=cfg["custom_loss"],
                        norm_closs=cfg["norm_closs"], norm=norm, acm_lim=np.ones(ac, np.float32), params=params)


def _flat(gs):
    return torch.cat([g.reshape(-1) for g in gs])


def _unflat(flat, like):
    out, o = [], 0
    for g in like:
        out.append(flat[o:o + g.numel()].view_as(g).clone())
        o += g.numel()
    return out


def _step(o, batch, e1, e2, allreduce):
    """update_from_replay_dp's exchange points, on the oracle."""
    obs, nobs, act, rew, done, acm = batch
    cg, _, _ = o.critic_grads(obs, nobs, act, rew, done, acm, e1)
    bucket = torch.cat([_flat(cg["critic_1"]), _flat(cg["critic_2"])])  # [critic_1 | critic_2]
    if allreduce is not None:
        allreduce(bucket)
    n1 = sum(g.numel() for g in cg["critic_1"])
    avg_c = {"critic_1": _unflat(bucket[:n1], cg["critic_1"]), "critic_2": _unflat(bucket[n1:], cg["critic_2"])}
    o.critic_apply(avg_c)
    g, ga, _, _ = o.actor_grads(obs, nobs, e2)
    bucket_a = torch.cat([_flat(g), ga.reshape(1).to(torch.float32)])  # [actor | alpha operand]
    if allreduce is not None:
        allreduce(bucket_a)
    o.actor_apply(_unflat(bucket_a[:-1], g), bucket_a[-1].to(torch.float64))
    return bucket, bucket_a


def _state(o):
    return {k: o.flat(k) for k in o.p} | {"log_alpha": np.array([o.log_alpha.item()])}


def _worker(rank, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from spprl.dp import make_allreduce, shard_batch
        cfg, fx, params, layouts, norm, steps = sac_case(CASE)
        ob, aout, ac, B = (int(v) for v in fx["dims"])
        b = shard_batch(B, WORLD)
        sl = slice(rank * b, (rank + 1) * b)
        o = _make_oracle(cfg, params, norm, ob, aout, ac)
        allreduce = make_allreduce()
        assert allreduce is not None
        buckets = []
        for batch, e1, e2 in steps:
            bc, ba = _step(o, tuple(x[sl] for x in batch), e1[sl], e2[sl], allreduce)
            buckets.append((bc.numpy(), ba.numpy()))
        st = _state(o)
        np.savez(os.path.join(out_dir, "rank%d.npz" % rank), **st,
                 **{"bc%d" % i: x[0] for i, x in enumerate(buckets)}, **{"ba%d" % i: x[1] for i, x in enumerate(buckets)})
    finally:
        dist.destroy_process_group()


def test_dp_world2_gloo_matches_full_batch(tmp_path):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, str(tmp_path))) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.is_alive():
            p.kill()
        assert p.exitcode == 0, "rank exited with %s" % p.exitcode
    r0 = dict(np.load(tmp_path / "rank0.npz"))
    r1 = dict(np.load(tmp_path / "rank1.npz"))
    # replicas bit-identical after the exchange
    for k in r0:
        assert np.array_equal(r0[k], r1[k]), k

    # single-process full-batch reference
    cfg, fx, params, layouts, norm, steps = sac_case(CASE)
    ob, aout, ac, B = (int(v) for v in fx["dims"])
    o = _make_oracle(cfg, params, norm, ob, aout, ac)
    for i, (batch, e1, e2) in enumerate(steps):
        bc, ba = _step(o, batch, e1, e2, None)
        for got, want in ((r0["bc%d" % i], bc.numpy()), (r0["ba%d" % i], ba.numpy())):
            scale = np.abs(want).max()
            assert np.abs(got - want).max() <= 1e-5 * scale
    full = _state(o)
    for k, want in full.items():
        d = np.abs(r0[k] - want)
        # Adam normalises the step: agreement to ~1e-6 except where a gradient
        # element sits at rounding level (sign may differ -> at most 2*lr*steps)
        assert np.mean(d > 1e-5) < 1e-3, (k, np.mean(d > 1e-5))
        assert d.max() <= 2 * 1e-3 * len(steps) + 1e-6, k


def test_make_allreduce_single_process_is_none():
    from spprl.dp import make_allreduce, shard_batch
    assert make_allreduce() is None
    assert shard_batch(409600, 8) == 51200
    with pytest.raises(ValueError):
        shard_batch(100, 3)


def _stats_worker(rank, port, shards, pivot, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=len(shards))
    from oracle.replay import dp_obs_stats

    def allreduce_sum(a):
        t = torch.from_numpy(np.ascontiguousarray(a))
        dist.all_reduce(t)
        return t.numpy()

    q.put((rank, dp_obs_stats(shards[rank], allreduce_sum, pivot)))
    dist.destroy_process_group()


def test_dp_obs_stats_protocol_gloo():
    """update_obs_mean_std over W=2 shards via all-reduced fp64 sums and radix-select
    histograms (the sppReplayObsStatsDP protocol, oracle form) equals numpy over the union."""
    rng = np.random.RandomState(4)
    shards = [(rng.standard_t(3, size=(n, 11)) * 2 + 1).astype(np.float32) for n in (3001, 4217)]
    pivot = rng.randn(11).astype(np.float32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stats_worker, args=(r, port, shards, pivot, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
    allx = np.concatenate(shards).astype(np.float64)
    for r in range(2):
        mean, std, p99, p1 = res[r]
        np.testing.assert_array_equal(p99, np.percentile(allx, 99, axis=0).astype(np.float32))
        np.testing.assert_array_equal(p1, np.percentile(allx, 1, axis=0).astype(np.float32))
        np.testing.assert_allclose(mean, allx.mean(0).astype(np.float32), rtol=1e-6)
        np.testing.assert_allclose(std, allx.std(0).astype(np.float32), rtol=1e-6)
    for a, b in zip(res[0], res[1]):
        np.testing.assert_array_equal(a, b)


def _ppo_worker(rank, port, q):
    """One data-parallel PPO_AcM actor step (OnPolicyNets.update_actor's exchange points):
    global advantage moments (sppAdvSums -> all-reduce -> sppAdvNormalizeGlobal, oracle form),
    per-rank half minibatch, gradient and loss/KL averaging with spprl.dp.make_allreduce."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from oracle import onpolicy as oo
        from spprl.dp import make_allreduce, make_allreduce_sum

        ob, aout, N = 17, 17, 512
        x, act, lp_old, adv, flat = _ppo_case(ob, aout, N)
        sl = slice(rank * N // WORLD, (rank + 1) * N // WORLD)
        a = torch.from_numpy(adv[sl].astype(np.float64))
        sums = torch.stack([a.sum(), (a * a).sum()])
        make_allreduce_sum()(sums)
        mean = sums[0] / N
        std = torch.sqrt(torch.clamp((sums[1] - sums[0] * mean) / (N - 1), min=0.0))
        an = ((a - mean) / (std.float() + 1.2e-7)).float().numpy()
        out, g = oo.actor_step(flat, ob, aout, np.ones(aout, np.float32), x[sl], act[sl], lp_old[sl], an)
        gt = torch.from_numpy(g)
        ot = torch.tensor([out["actor"], out["kl"]])
        ar = make_allreduce()
        ar(gt)
        ar(ot)
        q.put((rank, an, gt.numpy(), ot.numpy()))
    finally:
        dist.destroy_process_group()


def _ppo_case(ob, aout, N):
    from oracle import onpolicy as oo

    rng = np.random.RandomState(6)
    flat = oo.init_flat(oo.actor_layout(ob, aout), 3)
    x = rng.randn(N, ob).astype(np.float32)
    act, _ = oo.act(flat, ob, aout, np.ones(aout, np.float32), x, rng.randn(N, aout).astype(np.float32))
    lp_old = (rng.randn(N) * 0.1 - 20).astype(np.float32)
    adv = (rng.randn(N) * 3 + 1).astype(np.float32)
    return x, act.astype(np.float32), lp_old, adv, flat


def test_dp_ppo_actor_exchange_gloo():
    from oracle import onpolicy as oo

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ppo_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = dict((r, rest) for r, *rest in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(60)
    ob, aout, N = 17, 17, 512
    x, act, lp_old, adv, flat = _ppo_case(ob, aout, N)
    an = ((adv - adv.mean()) / (adv.std(ddof=1) + 1.2e-7)).astype(np.float32)  # AdvantageDataset
    np.testing.assert_allclose(np.concatenate([res[0][0], res[1][0]]), an, rtol=1e-5, atol=1e-6)
    out, g = oo.actor_step(flat, ob, aout, np.ones(aout, np.float32), x, act, lp_old, an)
    for r in range(WORLD):
        np.testing.assert_array_equal(res[r][1], res[0][1])  # replicas agree
        assert np.abs(res[r][1] - g).max() <= 1e-5 * np.abs(g).max()
        np.testing.assert_allclose(res[r][2], [out["actor"], out["kl"]], rtol=1e-5, atol=1e-6)


def _host_sum_worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from spprl.dp import make_host_allreduce_sum

        hs = make_host_allreduce_sum()
        # unequal shard lengths (resets advance the rings unevenly): the sum, on every rank
        q.put((rank, hs(1000 + 37 * rank), hs(2 ** 33 + rank)))
    finally:
        dist.destroy_process_group()


def test_host_row_count_exchange_gloo():
    """The DP obs statistics' global row count: host integers summed over the ranks (int64,
    no device tensor), identical on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_host_sum_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (a, b)) for r, a, b in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(60)
    for r in range(2):
        assert res[r] == (2037, 2 ** 34 + 1)


def test_make_host_allreduce_sum_single_process_is_none():
    from spprl.dp import make_host_allreduce_sum
    assert make_host_allreduce_sum() is None
