"""GPU parity at BASELINE configs[2]'s timed shape: SPP-DDPG HalfCheetah-v2 with a 10M-transition HBM
replay ring (ob = 17, ac = 6; bench.py --config ddpg_hcheetah runs 8.2 statistics calls and one
819,200-sample staged update per vector step over it).

One ring of 1e7 live rows (built once per module) carries columns designed for the regimes that only a
ring this size reaches with the full candidate-list capacities:
  c0   every row but the stride sample's inside the sample's 99th-percentile bracket: ~1e7 candidates,
       every workgroup list and the 2^18-key overflow list full -> the raw-column select (both targets);
  c4   the upper 2 % on rows the stride sample never visits: a sample miss -> raw-column select;
  c7   c0's design for the 2-rank one-pass protocol's sample rows (S / W = 32,768 per rank);
  c9   ~150K candidates: more than the select's LDS (32,768), no overflow -> the global-list select;
  c1 / c8 ties (integers, a 0.1 grid), c3 constant, c6 denormal neighbourhood, heavy tails elsewhere.
Checked against numpy on the same rows (replay_buffer.py:83-96): np.percentile 'linear' bit-exact,
mean / std rtol 2e-7 (fp64 moments), running max / min; the one-pass data-parallel protocol over
(this ring, a 10K-row shard) against numpy on the union; and the staged random-row gather
(sppAgentStageFromReplay, replay_buffer.py:233-261) plus rbuffer_sample_acm (:404-430) from this ring
bit-exact against the explicit gather, through one DDPG_AcM update at B = 819,200 (ddpg_acm.py:147-201).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

import spprl  # noqa: E402
from spprl import _lib  # noqa: E402

DEV = torch.device("cuda:0")
N = 10_000_000
OB, AC = 17, 6
DDPG = dict(env_name="HalfCheetah-v2", gamma=0.95, actor_lr=5e-4, critic_lr=5e-4, acm_critic=True, custom_loss=1.0,
            norm_closs=False, min_max_denormalize=True, denormalize_actor_out=True, seed=4)


def sample_rows(n, S):
    """k_st_sample's stride sample: row ((2s + 1) n) / (2S) (exact here: 2S is a power of two)."""
    step = n / (2.0 * S)
    return np.minimum(((2 * np.arange(S) + 1) * step).astype(np.int64), n - 1)


def spread(rng, k):
    """k distinct values evenly over (-1, 1), in random order."""
    return (-1.0 + 2.0 * (np.arange(k) + 0.5) / k)[rng.permutation(k)]


def build_rows(seed=2024):
    rng = np.random.RandomState(seed)
    x = np.empty((N + 1, OB), np.float32)
    s1 = sample_rows(N, 65536)   # the N = 1 sample (len > 4M: S = 65,536)
    s2 = sample_rows(N, 32768)   # rank 0's sample in the 2-rank protocol (S / W)
    free = np.ones(N, bool)
    free[s1] = False
    free = np.flatnonzero(free)
    x[:, 0] = rng.uniform(0.978, 0.982, N + 1)
    x[s1, 0] = spread(rng, s1.size)
    x[:, 1] = rng.randint(-3, 4, N + 1)
    x[:, 2] = rng.standard_t(3, N + 1) * 2.5 + 0.3
    x[:, 3] = 3.0
    x[:, 4] = 0.0
    pick = rng.choice(free, N // 50, replace=False)
    x[pick, 4] = rng.uniform(1, 2, pick.size)
    x[:, 5] = -np.abs(rng.standard_cauchy(N + 1))
    x[:, 6] = rng.randn(N + 1) * 1e-30
    x[:, 7] = rng.uniform(0.978, 0.982, N + 1)
    x[s2, 7] = spread(rng, s2.size)
    x[:, 8] = np.round(rng.randn(N + 1), 1)
    x[:, 9] = rng.uniform(-1, 0.9, N + 1)
    band = rng.choice(free, 150_000, replace=False)
    x[band, 9] = rng.uniform(0.978, 0.982, band.size)
    x[s1, 9] = spread(rng, s1.size)
    for c in range(10, OB):
        x[:, c] = rng.standard_t(2 + c % 5, N + 1) * (0.2 + c) + (c - 13)
    return x


def numpy_stats(cols):
    """Per column (float64, one column at a time): mean, std (ddof 0), p99, p1 (np.percentile 'linear')."""
    out = np.zeros((4, len(cols)), np.float64)
    for c, col in enumerate(cols):
        v = col.astype(np.float64)
        out[0, c], out[1, c] = v.mean(), v.std()
        out[2, c], out[3, c] = np.percentile(v, [99, 1])
    return out


@pytest.fixture(scope="module")
def ring():
    x = build_rows()
    ag = spprl.DDPG_AcM(max_batch=819_200, buffer_size=N + 64, device=DEV, **DDPG)
    rb = ag.replay_buffer
    slots = rb.add_obs_batch(torch.from_numpy(x))
    assert slots[0] == 0 and slots[-1] == N
    torch.manual_seed(3)
    z = torch.zeros(N, dtype=torch.uint8, device=DEV)
    rb.add_timestep_batch(slots[:N], slots[1:], torch.randn(N, OB, device=DEV), torch.randn(N, device=DEV),
                          (torch.rand(N, device=DEV) < 0.05).to(torch.uint8), z,
                          torch.rand(N, AC, device=DEV) * 2 - 1)
    assert len(rb) == N
    want = numpy_stats([x[:N, c] for c in range(OB)])
    yield ag, rb, x, want
    del ag, rb


def _check(rb, want, first=None):
    got = [t.cpu().numpy() for t in (rb.obs_mean, rb.obs_std, rb.max_obs, rb.min_obs)]
    p99, p1 = want[2].astype(np.float32), want[3].astype(np.float32)
    if first is not None:
        p99, p1 = np.maximum(p99, first[2]), np.minimum(p1, first[3])
    np.testing.assert_array_equal(got[2], p99)
    np.testing.assert_array_equal(got[3], p1)
    np.testing.assert_allclose(got[0], want[0].astype(np.float32), rtol=2e-7, atol=1e-30)
    np.testing.assert_allclose(got[1], want[1].astype(np.float32), rtol=2e-7, atol=1e-30)
    return got


def test_obs_stats_10m_ring_exact_and_reused_bracket(ring):
    """update_obs_mean_std over the 1e7-row ring, then again on the unchanged rows (the bench's repeated calls
    reuse the stored bracket): both bit-exact against numpy."""
    ag, rb, x, want = ring
    # the designed columns really are in the regimes named above
    assert want[2, 0] > 0.978 and want[3, 0] > 0.978   # c0: both percentiles inside the overflowing band
    assert want[2, 4] > 1.0                           # c4: the p99 lies on rows the sample never visits
    assert 0.978 < want[2, 9] < 0.982                 # c9: among the ~150K candidates
    rb._have_minmax = False
    rb.update_obs_mean_std()
    torch.cuda.synchronize()
    first = _check(rb, want)
    rb.update_obs_mean_std()
    _check(rb, want, first=first)


def test_obs_stats_one_pass_protocol_with_10m_shard(ring):
    """sppReplayObsStatsDP1 over (the 1e7-row ring, a 10K-row shard) with the collectives emulated on one GPU:
    rank 0's c7 candidates overflow every list (raw-column rounds), the union sample weights the small shard
    like the large one.  Percentiles bit-exact on both ranks against numpy on the union."""
    ag, rb, x, _ = ring
    rng = np.random.RandomState(77)
    n1 = 10_000
    y = (rng.standard_t(4, size=(n1 + 1, OB)) * 1.5).astype(np.float32)
    y[:, 7] = spread(rng, n1 + 1)
    rb1 = spprl.BufferAcMOffPolicy(n1 + 8, OB, OB, AC, device=DEV, min_max_denormalize=True)
    sl = rb1.add_obs_batch(torch.from_numpy(y))
    z = np.zeros(n1, bool)
    rb1.add_timestep_batch(sl[:n1], sl[1:], torch.zeros(n1, OB), np.zeros(n1, np.float32), z, z, torch.zeros(n1, AC))
    shards = [rb, rb1]
    W, n_global = 2, N + n1
    Sl = _lib.load().sppReplayObsStatsDP1SampleRows(rb._h, W, n_global)
    assert Sl == 32768
    pivot = torch.from_numpy(rng.randn(OB).astype(np.float32)).to(DEV)
    outs = [[torch.zeros(OB, device=DEV) for _ in range(4)] for _ in shards]
    st = _lib.stream_handle()
    bufs = [dict(samp=torch.zeros(W * OB * Sl, dtype=torch.int32, device=DEV),
                 exch=torch.zeros(12 * OB, dtype=torch.float64, device=DEV),
                 hist=torch.zeros(OB * 1024, dtype=torch.int32, device=DEV)) for _ in shards]
    for phase in range(7):
        for r, b in enumerate(shards):
            o = outs[r]
            _lib.call("sppReplayObsStatsDP1", b._h, phase, W, r, _lib.ptr(pivot), _lib.ptr(bufs[r]["samp"]),
                      _lib.ptr(bufs[r]["exch"]), _lib.ptr(bufs[r]["hist"]), n_global, _lib.ptr(o[0]), _lib.ptr(o[1]),
                      _lib.ptr(o[2]), _lib.ptr(o[3]), 1, st)
        if phase == 0:
            allg = torch.cat([bufs[r]["samp"][r * OB * Sl:(r + 1) * OB * Sl] for r in range(W)])
            for b in bufs:
                b["samp"].copy_(allg)
        elif phase <= 5:
            k = "exch" if phase == 1 else "hist"
            tot = sum(b[k] for b in bufs)
            for b in bufs:
                b[k].copy_(tot)
    torch.cuda.synchronize()
    want = numpy_stats([np.concatenate([x[:N, c], y[:n1, c]]) for c in range(OB)])
    assert want[2, 7] > 0.978  # the union p99 of c7 lies inside rank 0's overflowing band
    for o in outs:
        got = [t.cpu().numpy() for t in o]
        np.testing.assert_array_equal(got[2], want[2].astype(np.float32))
        np.testing.assert_array_equal(got[3], want[3].astype(np.float32))
        np.testing.assert_allclose(got[0], want[0].astype(np.float32), rtol=1e-6, atol=1e-30)
        np.testing.assert_allclose(got[1], want[1].astype(np.float32), rtol=1e-6, atol=1e-30)


def test_staged_gather_and_update_from_10m_ring_bit_exact(ring):
    """The bench's staged path over the 10M ring (sppRandIndex -> sppAgentStageFromReplay -> DDPG_AcM critic /
    actor grads and Adam, B = rho E = 819,200) leaves the same parameters and losses, bit for bit, as the
    caller-batch update on the explicitly gathered tuples (a second agent with the same initial weights and
    normaliser); the ACM batch gather (sigma E = 419,430 rows) equals the explicit gather."""
    ag, rb, _, _ = ring
    B = 819_200
    rb.update_obs_mean_std()
    a2 = spprl.DDPG_AcM(max_batch=B, buffer_size=64, device=DEV, **DDPG)
    for net in ag.params:
        assert torch.equal(ag.params[net], a2.params[net]), net
    r2 = a2.replay_buffer
    for s, d in ((rb.min_obs, r2.min_obs), (rb.max_obs, r2.max_obs), (rb.obs_mean, r2.obs_mean),
                 (rb.obs_std, r2.obs_std)):
        d.copy_(s)
    r2._have_minmax = True
    st = _lib.stream_handle()
    idx = torch.empty(B, dtype=torch.int64, device=DEV)
    _lib.call("sppRandIndex", _lib.ptr(idx), B, len(rb), 91, 1, st)
    batch = rb.gather(idx)
    ag.update_from_replay_dp(idx)
    a2.update(*batch)
    torch.cuda.synchronize()
    ix = idx.cpu().numpy()
    assert ix.min() >= 0 and ix.max() < N and len(np.unique(ix)) > 0.9 * B
    for net in ag.params:
        np.testing.assert_array_equal(ag.params[net].cpu().numpy(), a2.params[net].cpu().numpy(), err_msg=str(net))
    assert ag.loss == a2.loss
    BA = 419_430
    ia = idx[:BA].flip(0).contiguous()
    xa = torch.empty(BA, 2 * OB, device=DEV)
    ya = torch.empty(BA, AC, device=DEV)
    _lib.call("sppReplayGatherAcm", rb._h, _lib.ptr(ia), BA, _lib.ptr(xa), _lib.ptr(ya), st)
    o, no, _, _, _, acm = rb.gather(ia)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(xa.cpu().numpy(), torch.cat([o, no], 1).cpu().numpy())
    np.testing.assert_array_equal(ya.cpu().numpy(), acm.cpu().numpy())
