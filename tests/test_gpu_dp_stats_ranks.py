"""Global obs statistics across ranks through the product call (ReplayBuffer.update_obs_mean_std_dp,
replay_buffer.py:83-96 over the union of the shards): 2 processes on one GPU over
gloo (CUDA tensors), unequal shard lengths, the row count summed on the host (host_sum) or as a
device tensor.  Percentiles and running max / min bit-exact against numpy on the union; mean / std
rtol 1e-6 (fp64 sums in another order).  Exercises the fused step-0 exchange (moment sums and
top-byte counts in one fp64 all-reduce) and the later histogram all-reduces."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rank_results import collect


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shards(ob, kind="t3"):
    rng = np.random.RandomState(ob + 7)
    if kind == "skew":  # unequal, shifted shards: the union sample (equal rows per rank) mis-weights them, so
        # the brackets tend to miss and the raw-column rounds must carry the selection
        return [(rng.randn(n, ob) * s + m).astype(np.float32) for n, s, m in ((3000, 0.5, -4.0), (40000, 2.0, 3.0))]
    if kind == "ties":  # discrete values: long runs equal to the bracket bounds
        return [np.round(rng.randn(n, ob) * 3).astype(np.float32) for n in (9000, 12000)]
    return [(rng.standard_t(3, size=(n, ob)) * rng.uniform(0.5, 3, ob) + rng.randn(ob)).astype(np.float32)
            for n in (6000, 7321)]


def _worker(rank, port, ob, use_host, q, proto="stepwise", kind="t3", repeat=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        import spprl
        from spprl.dp import make_allgather, make_allreduce_sum, make_host_allreduce_sum

        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        rows = _shards(ob, kind)[rank]
        rb = spprl.BufferAcMOffPolicy(len(rows) + 8, ob, ob, 2, device=dev, min_max_denormalize=True)
        sl = rb.add_obs_batch(torch.from_numpy(np.concatenate([rows, rows[:1]])))
        n = len(rows)
        z = np.zeros(n, bool)
        rb.add_timestep_batch(sl[:n], sl[1:], torch.zeros(n, ob), np.zeros(n, np.float32), z, z, torch.zeros(n, 2))
        rb.obs_mean.zero_()  # replicated pivot
        ag, gathers = (make_allgather() if proto == "onepass" else None), [0]

        class CountingGather:  # the sample all-gather, counted
            def __init__(self, inner):
                self.world, self.rank = inner.world, inner.rank

            def __call__(self, *a):
                gathers[0] += 1
                return ag(*a)

        cg = CountingGather(ag) if ag is not None else None
        rb.update_obs_mean_std_dp(make_allreduce_sum(), host_sum=make_host_allreduce_sum() if use_host else None,
                                  allgather=cg)
        if repeat:  # a second call on the same shards (one-pass: reuses the union bracket, no all-gather)
            rb.update_obs_mean_std_dp(make_allreduce_sum(), host_sum=make_host_allreduce_sum() if use_host else None,
                                      allgather=cg)
            assert cg is None or gathers[0] == 1, gathers
        torch.cuda.synchronize()
        q.put((rank, rb.obs_mean.cpu().numpy(), rb.obs_std.cpu().numpy(), rb.max_obs.cpu().numpy(),
               rb.min_obs.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("ob,use_host,proto,kind,repeat", [(11, True, "stepwise", "t3", False),
                                                           (111, False, "stepwise", "t3", False),
                                                           (11, True, "onepass", "t3", False),
                                                           (111, True, "onepass", "t3", False),
                                                           (17, True, "onepass", "skew", False),
                                                           (11, True, "onepass", "ties", False),
                                                           (17, True, "onepass", "skew", True),
                                                           (111, False, "onepass", "t3", True)])
def test_dp_obs_stats_two_ranks_match_union(ob, use_host, proto, kind, repeat):
    """proto: the stepwise radix protocol or the one-pass sample-bracketed one (sppReplayObsStatsDP1);
    repeat: a second call on unchanged shards (bracket reuse) must give the same exact statistics."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, ob, use_host, q, proto, kind, repeat)) for r in range(2)]
    for p in procs:
        p.start()
    res = collect(q, procs, timeout=180)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    allx = np.concatenate(_shards(ob, kind)).astype(np.float64)
    for r in range(2):
        mean, std, mx, mn = res[r]
        np.testing.assert_array_equal(mx, np.percentile(allx, 99, axis=0).astype(np.float32))
        np.testing.assert_array_equal(mn, np.percentile(allx, 1, axis=0).astype(np.float32))
        np.testing.assert_allclose(mean, allx.mean(0).astype(np.float32), rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(std, allx.std(0).astype(np.float32), rtol=1e-6)
    for a, b in zip(res[0], res[1]):
        np.testing.assert_array_equal(a, b)
