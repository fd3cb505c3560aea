"""GPU parity of update_obs_mean_std (rltoolkit/buffer/replay_buffer.py:83-96) on the
single-device sample-bracketed path (csrc/stats.hip) against numpy on the same rows:
percentiles (np.percentile 'linear') bit-exact, mean / std within fp32 rounding of the fp64
result (rtol 2e-7), running max / min.  Cases cover the edge cases of the bracket: tiny and
sample-sized buffers, ties at the bounds, constant columns, heavy tails, wide observations,
a wrapped ring (obs_idx not in slot order) and a layout built so the stride sample misses the
tail (the exact raw-data fallback inside k_st_select)."""
import numpy as np
import pytest
import torch

import spprl

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _fill(rows, ac=3, extra=10):
    n, ob = rows.shape[0] - 1, rows.shape[1]
    rb = spprl.BufferAcMOffPolicy(n + extra, ob, ob, ac, device=DEV)
    slots = rb.add_obs_batch(torch.from_numpy(rows))
    rb.add_timestep_batch(slots[:n], slots[1:n + 1], torch.zeros(n, ob), np.zeros(n), np.zeros(n, bool),
                          np.zeros(n, bool), torch.zeros(n, ac))
    assert len(rb) == n
    return rb


def _check(rb, x, prev=None):
    rb.update_obs_mean_std()
    x = x.astype(np.float64)
    p99, p1 = np.percentile(x, 99, axis=0).astype(np.float32), np.percentile(x, 1, axis=0).astype(np.float32)
    if prev is not None:
        p99, p1 = np.maximum(p99, prev[0]), np.minimum(p1, prev[1])
    got = [t.cpu().numpy() for t in (rb.obs_mean, rb.obs_std, rb.max_obs, rb.min_obs)]
    np.testing.assert_array_equal(got[2], p99)
    np.testing.assert_array_equal(got[3], p1)
    np.testing.assert_allclose(got[0], x.mean(0).astype(np.float32), rtol=2e-7, atol=1e-30)
    np.testing.assert_allclose(got[1], x.std(0).astype(np.float32), rtol=2e-7, atol=1e-30)
    return got


@pytest.mark.parametrize("n,ob", [(11, 3), (100, 11), (16384, 11), (16385, 17), (300_001, 11), (150_000, 111)])
def test_obs_stats_exact_sizes(n, ob):
    rng = np.random.RandomState(n % 997 + ob)
    rows = (rng.standard_t(3, size=(n + 1, ob)) * rng.uniform(0.1, 5, ob) + rng.randn(ob)).astype(np.float32)
    _check(_fill(rows), rows[:n])


def test_obs_stats_ties_constant_and_discrete_columns():
    rng = np.random.RandomState(5)
    n, ob = 200_000, 6
    rows = np.empty((n + 1, ob), np.float32)
    rows[:, 0] = 3.0                                     # constant
    rows[:, 1] = rng.randint(-3, 4, n + 1)               # 7 values: ties at every bound
    rows[:, 2] = np.where(rng.rand(n + 1) < 0.985, 0.0, rng.randn(n + 1))  # mass at 0, sparse tail
    rows[:, 3] = rng.randn(n + 1) * 1e-30                # tiny magnitudes (denormal neighbourhood)
    rows[:, 4] = -np.abs(rng.standard_cauchy(n + 1))     # heavy one-sided tail
    rows[:, 5] = np.round(rng.randn(n + 1), 1)           # 0.1 grid
    _check(_fill(rows), rows[:n])


def test_obs_stats_fallback_when_sample_misses_tail():
    """Rows the stride sample ((2s+1) len / 2S) never visits carry the upper 2 %: every sample
    key is 0, the bracket is [0, 0] and the 99th-percentile ranks fall outside it."""
    n, ob = 100_000, 2
    S = 16384
    sampled = np.zeros(n, bool)
    sampled[((2 * np.arange(S) + 1) * n) // (2 * S)] = True
    rows = np.zeros((n + 1, ob), np.float32)
    free = np.flatnonzero(~sampled)
    rng = np.random.RandomState(1)
    pick = rng.choice(free, size=n // 50, replace=False)
    rows[pick, 0] = rng.uniform(1, 2, pick.size)
    rows[pick, 1] = -rng.uniform(1, 2, pick.size)
    _check(_fill(rows), rows[:n])


def test_obs_stats_wrapped_ring_and_running_extremes():
    """A ring that wrapped (Q6: obs_idx no longer in slot order) and a second update that keeps
    the running max / min (replay_buffer.py:93-96)."""
    rng = np.random.RandomState(9)
    size, ob = 50_000, 11
    rb = spprl.BufferAcMOffPolicy(size, ob, ob, 3, device=DEV)
    prev = rb.add_obs_batch(torch.from_numpy(rng.randn(1, ob).astype(np.float32)))
    for it in range(4):  # 4 x 20000 transitions into a 50000-slot ring: wraps
        E = 20_000
        obs = (rng.randn(E, ob) * (1 + it)).astype(np.float32)
        slots = rb.add_obs_batch(torch.from_numpy(obs))
        prevs = np.concatenate([prev[-1:], slots[:-1]])
        rb.add_timestep_batch(prevs, slots, torch.zeros(E, ob), np.zeros(E), np.zeros(E, bool), np.zeros(E, bool),
                              torch.zeros(E, 3))
        prev = slots
    n = len(rb)
    x = rb.gather(torch.arange(n))[0].cpu().numpy()  # obs[obs_idx[t]] (bit-exact gather)
    first = _check(rb, x)
    # one more obs slot (it overwrites the ring slot of the oldest live obs): running extremes hold
    rb.add_obs_batch(torch.zeros(1, ob))
    x = rb.gather(torch.arange(n))[0].cpu().numpy()
    _check(rb, x, prev=(first[2], first[3]))


def test_obs_stats_repeated_calls_reuse_bracket_and_follow_changes():
    """Calls on unchanged rows reuse the stored bracket (no sample / bracket launch: the ring
    generation is unchanged) and still match numpy; rows added after it (new generation) get a
    fresh bracket.  The bench's vector step makes ~4 such calls per step on the same rows."""
    rng = np.random.RandomState(13)
    n, ob = 120_000, 11
    rows = (rng.standard_t(4, size=(n + 1, ob)) * rng.uniform(0.5, 3, ob)).astype(np.float32)
    rb = _fill(rows, extra=n)
    first = _check(rb, rows[:n])
    again = _check(rb, rows[:n], prev=(first[2], first[3]))
    for a, b in zip(first, again):
        np.testing.assert_array_equal(a, b)
    # shift the distribution: a bracket of the old rows would miss the new percentiles
    more = (rng.standard_t(4, size=(n, ob)) * 10 + 50).astype(np.float32)
    slots = rb.add_obs_batch(torch.from_numpy(more))
    prevs = np.concatenate([[n], slots[:-1]])
    rb.add_timestep_batch(prevs, slots, torch.zeros(n, ob), np.zeros(n), np.zeros(n, bool), np.zeros(n, bool),
                          torch.zeros(n, 3))
    m = len(rb)
    x = rb.gather(torch.arange(m))[0].cpu().numpy()
    _check(rb, x, prev=(again[2], again[3]))


# ---------------------------------------------------------------- overflow paths at small sizes
# sppReplaySetObsStatsCaps lowers the per-workgroup candidate-list capacity and the per-(column, target)
# overflow list, so the overflow fallbacks (full lists -> raw-column selection) run at a few 100K rows.
def _stride_sample(n, S):
    step = n / (2.0 * S)  # exact: 2S is a power of two
    return np.minimum(((2 * np.arange(S) + 1) * step).astype(np.int64), n - 1)


def _tie_design(rng, S, n_rows, sample_pos):
    """Column values for the '== lo' trap of the 99th-percentile query: the sorted (union) sample is
    0.0 below rank 16,100, a block of 1.0 over ranks 16,100..16,199 (where the bracket's lower bound
    lands: rank 16,151 at 5 sigma, 16,164 at 4) and spread over (2, 3) above; the other rows of shard 0
    are 5,000 ties at 1.0, 20,000 candidates in (1.1, 1.9) and zeros.  The true 99th percentile is a
    candidate; a candidate count that loses the keys past a capped overflow list shifts the query into
    the '== lo' run and returns 1.0."""
    assert S == 16384
    vals = np.zeros(S, np.float32)
    vals[16100:16200] = 1.0
    vals[16200:] = 2.0 + (np.arange(S - 16200) + 1) / 200.0
    vals = vals[rng.permutation(S)]
    cols = [np.zeros(n, np.float32) for n in n_rows]
    free0 = np.setdiff1d(np.arange(n_rows[0]), sample_pos[0])
    pick = rng.choice(free0, 25_000, replace=False)
    cols[0][pick[:5000]] = 1.0
    cols[0][pick[5000:]] = rng.uniform(1.1, 1.9, 20_000)
    o = 0
    for r, pos in enumerate(sample_pos):
        cols[r][pos] = vals[o:o + pos.size]
        o += pos.size
    return cols


def test_obs_stats_overflowed_lists_small_caps():
    """N = 1: every list full at capacities (1 key per workgroup list, 16 overflow keys): the raw-column
    select carries every (column, target), bit-exact; the same rows again at full capacity agree."""
    rng = np.random.RandomState(31)
    n, ob = 300_000, 4
    rows = np.empty((n + 1, ob), np.float32)
    rows[:n, 0] = _tie_design(rng, 16384, [n], [_stride_sample(n, 16384)])[0]
    rows[n, 0] = 0.0
    rows[:, 1] = rng.standard_t(3, n + 1) * 2.0
    rows[:, 2] = rng.randint(-3, 4, n + 1)
    rows[:, 3] = rng.randn(n + 1)
    assert np.percentile(rows[:n, 0].astype(np.float64), 99) > 1.1  # the trap: p99 among the candidates
    rb = _fill(rows)
    from spprl import _lib

    _lib.call("sppReplaySetObsStatsCaps", rb._h, 1, 16)
    first = _check(rb, rows[:n])
    _lib.call("sppReplaySetObsStatsCaps", rb._h, 0, 0)
    again = _check(rb, rows[:n], prev=(first[2], first[3]))
    for a, b in zip(first, again):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("caps", [(1, 16), (0, 0)])
def test_obs_stats_one_pass_protocol_overflow_counts_every_candidate(caps):
    """The one-pass data-parallel protocol (sppReplayObsStatsDP1) with rank 0's candidate lists overflowing
    (caps (1, 16)): the exported candidate count must be the TRUE count (k_dp_reduce, stats.hip), else the
    99th-percentile rank of the _tie_design column falls into the '== lo' region and resolves to 1.0.
    Two shards (290K + 10K rows, the union sample weights them equally) against numpy on the union."""
    from spprl import _lib

    rng = np.random.RandomState(37)
    sizes, ob, W = [290_000, 10_000], 3, 2
    n_global = sum(sizes)
    pos = [_stride_sample(n, 8192) for n in sizes]
    col0 = _tie_design(rng, 16384, sizes, pos)
    data = []
    for r, n in enumerate(sizes):
        d = np.empty((n, ob), np.float32)
        d[:, 0] = col0[r]
        d[:, 1] = rng.standard_t(3, n) * (1 + r)
        d[:, 2] = np.round(rng.randn(n) * 2)
        data.append(d)
    allx = np.concatenate(data).astype(np.float64)
    assert np.percentile(allx[:, 0], 99) > 1.1
    shards = []
    for d in data:
        n = len(d)
        rb = spprl.BufferAcMOffPolicy(n + 8, ob, ob, 2, device=DEV, min_max_denormalize=True)
        sl = rb.add_obs_batch(torch.from_numpy(np.concatenate([d, d[:1]])))
        z = np.zeros(n, bool)
        rb.add_timestep_batch(sl[:n], sl[1:], torch.zeros(n, ob), np.zeros(n, np.float32), z, z, torch.zeros(n, 2))
        _lib.call("sppReplaySetObsStatsCaps", rb._h, *caps)
        shards.append(rb)
    Sl = _lib.load().sppReplayObsStatsDP1SampleRows(shards[0]._h, W, n_global)
    assert Sl == 8192
    pivot = torch.zeros(ob, device=DEV)
    st = _lib.stream_handle()
    bufs = [dict(samp=torch.zeros(W * ob * Sl, dtype=torch.int32, device=DEV),
                 exch=torch.zeros(12 * ob, dtype=torch.float64, device=DEV),
                 hist=torch.zeros(ob * 1024, dtype=torch.int32, device=DEV)) for _ in shards]
    for phase in range(7):
        for r, rb in enumerate(shards):
            b = bufs[r]
            _lib.call("sppReplayObsStatsDP1", rb._h, phase, W, r, _lib.ptr(pivot), _lib.ptr(b["samp"]),
                      _lib.ptr(b["exch"]), _lib.ptr(b["hist"]), n_global, _lib.ptr(rb.obs_mean), _lib.ptr(rb.obs_std),
                      _lib.ptr(rb.max_obs), _lib.ptr(rb.min_obs), 1, st)
        if phase == 0:
            allg = torch.cat([bufs[r]["samp"][r * ob * Sl:(r + 1) * ob * Sl] for r in range(W)])
            for b in bufs:
                b["samp"].copy_(allg)
        elif phase <= 5:
            k = "exch" if phase == 1 else "hist"
            tot = sum(b[k] for b in bufs)
            for b in bufs:
                b[k].copy_(tot)
    torch.cuda.synchronize()
    if caps[0]:  # rank 0's overflow flag was raised (the fallback under test really ran)
        assert float(bufs[0]["exch"][2 * ob + 4].item()) >= 1.0
    for rb in shards:
        np.testing.assert_array_equal(rb.max_obs.cpu().numpy(), np.percentile(allx, 99, axis=0).astype(np.float32))
        np.testing.assert_array_equal(rb.min_obs.cpu().numpy(), np.percentile(allx, 1, axis=0).astype(np.float32))
        np.testing.assert_allclose(rb.obs_mean.cpu().numpy(), allx.mean(0).astype(np.float32), rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(rb.obs_std.cpu().numpy(), allx.std(0).astype(np.float32), rtol=1e-6)
