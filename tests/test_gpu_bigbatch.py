"""GPU parity of the TIMED configuration: the update at the bench's batch sizes.

bench.py runs SAC_AcM / DDPG_AcM at B = rho*E = 409,600 (E = 4096 envs, rho = 100,
SURVEY.md §8d).  At that size the device path differs from the B <= 100 fixture
cases in ways only a large batch exercises:
  - split-K weight gradients over 2048-sample slabs (~200 slabs per job) and the
    fixed-order slab reduce ``k_dw_reduce``; the thin-job wave split;
  - grid-stride tile loops of the phase kernels over 12,800 tiles;
  - the replay stage (``k_replay_stage_fm``: random-row gather -> feature-major);
  - the device Philox eps (``k_eps_fm``) and indices (``k_rand_index``).
Each case runs the device step and the oracle (oracle/sac_acm.py, oracle/ddpg_acm.py,
float64 so its own summation error is negligible) on the same inputs and compares:
  fp32 path : losses rtol 1e-4; ||g - g_ref|| / ||g_ref|| < 2e-4 per network;
              post-Adam parameters |d| <= 2 lr (first Adam step moves by ~lr sign(g))
              with fewer than 0.2 % of weights beyond 1e-5
  bf16 MLP  : losses rtol 3e-2; gradient relative error < 6e-2 (bf16 operands,
              8-bit mantissa, fp32 accumulation)
Reference: acm/off_policy/sac_acm.py:89-162, ddpg_acm.py:147-201 (rltoolkit).
The sampler checks at the end cover sppRandIndex / sppRandNormal / sppSacAcmDrawEps
(range, uniformity, moments), which feed every timed step.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

import spprl  # noqa: E402
from spprl import _lib  # noqa: E402
from oracle.ddpg_acm import OracleDdpgAcm  # noqa: E402
from oracle.nets import Norm  # noqa: E402
from oracle.sac_acm import OracleSacAcm  # noqa: E402

DEV = torch.device("cuda:0")
F64 = torch.float64
SAC_NETS = {"actor": _lib.SPP_NET_ACTOR, "critic_1": _lib.SPP_NET_CRITIC1, "critic_2": _lib.SPP_NET_CRITIC2,
            "critic_1_targ": _lib.SPP_NET_CRITIC1_TARG, "critic_2_targ": _lib.SPP_NET_CRITIC2_TARG,
            "acm": _lib.SPP_NET_ACM}
DDPG_NETS = {"actor": _lib.SPP_NET_ACTOR, "critic": _lib.SPP_NET_CRITIC1, "actor_targ": _lib.SPP_NET_ACTOR_TARG,
             "critic_targ": _lib.SPP_NET_CRITIC1_TARG, "acm": _lib.SPP_NET_ACM}


def relerr(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def snapshot(ag, names):
    return {k: {n: v.numpy().copy() for n, v in ag.net_state(net).items()} for k, net in names.items()}


def random_batch(rng, B, ob, aout, ac):
    return (rng.randn(B, ob).astype(np.float32), rng.randn(B, ob).astype(np.float32),
            rng.uniform(-1, 1, (B, aout)).astype(np.float32), rng.randn(B).astype(np.float32),
            (rng.rand(B) < 0.05).astype(np.int8), rng.uniform(-1, 1, (B, ac)).astype(np.float32))


def set_minmax(ag, rng, ob):
    lo = -rng.uniform(0.5, 2, ob).astype(np.float32)
    hi = rng.uniform(0.5, 2, ob).astype(np.float32)
    rb = ag.replay_buffer
    rb.min_obs.copy_(torch.from_numpy(lo))
    rb.max_obs.copy_(torch.from_numpy(hi))
    rb._have_minmax = True
    return Norm(True, torch.from_numpy(lo), torch.from_numpy(hi))


def check_sac(ag, o, ol, grad_tol, loss_tol, params_check=True, params0=None):
    errs = {}
    for k in ("critic_1", "critic_2", "actor"):
        errs[k] = relerr(ag.grads[SAC_NETS[k]].cpu().numpy(), o.last["grads"][k])
    gl = ag.loss
    print("grad rel err", {k: "%.2e" % v for k, v in errs.items()},
          "losses", {k: (round(gl[k], 6), round(ol[k], 6)) for k in gl})
    for k, e in errs.items():
        assert e < grad_tol, (k, e)
    for k in gl:
        assert abs(gl[k] - ol[k]) <= loss_tol * abs(ol[k]) + 1e-6, (k, gl[k], ol[k])
    if params_check:
        assert ag.current_alpha() == pytest.approx(o.alpha, rel=1e-5)
        lr = 1e-3
        for k in ("actor", "critic_1", "critic_2", "critic_1_targ", "critic_2_targ"):
            got = ag.params[SAC_NETS[k]].cpu().numpy().astype(np.float64)
            want = o.flat(k).astype(np.float64)
            d = np.abs(got - want)
            assert d.max() <= 2 * lr * 1.01, (k, d.max())
            assert np.mean(d > 1e-5) < 2e-3, (k, np.mean(d > 1e-5))


# ------------------------------------------------------------------ caller-batch path
@pytest.mark.parametrize("env_name,ob,ac,B,bf16", [
    ("Hopper-v2", 11, 3, 65536, False),
    ("Hopper-v2", 11, 3, 409600, False),
    ("Ant-v2", 111, 8, 65536, True),
    ("Ant-v2", 111, 8, 409600, True),
    ("Ant-v2", 111, 8, 4096, False),    # fp32 Ant (bench config sac_ant): the widest phase kernels
    ("Ant-v2", 111, 8, 65536, False),
    ("Ant-v2", 111, 8, 4096, "acmc0"),  # fp32 Ant, critics on [s | a_d] (acm_critic=False)
    ("Ant-v2", 111, 8, 4096, "bf16_acmc0"),
])
def test_sac_acm_update_large_batch_matches_oracle(env_name, ob, ac, B, bf16):
    _sac_update_vs_oracle(env_name, ob, ac, B, bf16)


# ragged and minimal batches: Bp = B rounded up to 32 with dead samples in the last tile (B = 1: one live sample
# in the whole launch), a tile count below the grid, one live sample past a tile boundary
@pytest.mark.parametrize("env_name,ob,ac,B,bf16", [
    ("Hopper-v2", 11, 3, 1, False),
    ("Hopper-v2", 11, 3, 31, False),
    ("Hopper-v2", 11, 3, 33, False),
    ("Hopper-v2", 11, 3, 1001, False),
    ("Ant-v2", 111, 8, 33, True),
    ("Ant-v2", 111, 8, 1, "acmc0"),
])
def test_sac_acm_update_ragged_batches_match_oracle(env_name, ob, ac, B, bf16):
    # Adam's first step moves a parameter by ~lr whatever its gradient's size, so at a few samples the many
    # near-zero gradients make the post-step comparison a sign test; gradients and losses are compared instead
    _sac_update_vs_oracle(env_name, ob, ac, B, bf16, params_check=B >= 1000)


def _sac_update_vs_oracle(env_name, ob, ac, B, bf16, params_check=True):
    rng = np.random.RandomState(B % 1000 + ob)
    acmc = bf16 not in ("acmc0", "bf16_acmc0")
    bf16 = bf16 in (True, "bf16_acmc0")
    ag = spprl.SAC_AcM(env_name=env_name, acm_critic=acmc, custom_loss=0.2, norm_closs=False, min_max_denormalize=True,
                       denormalize_actor_out=True, gamma=0.99, max_batch=B, buffer_size=128, device=DEV, seed=3,
                       mlp_bf16=bf16)
    params = snapshot(ag, SAC_NETS)
    norm = set_minmax(ag, rng, ob)
    batch = random_batch(rng, B, ob, ob, ac)
    e1, e2 = rng.randn(B, ob).astype(np.float32), rng.randn(B, ob).astype(np.float32)
    ag.update(*batch, eps_next=e1, eps_cur=e2)
    torch.cuda.synchronize()
    o = OracleSacAcm(ob, ob, ac, acm_critic=acmc, custom_loss=0.2, norm_closs=False, norm=norm, actor_lim=1.0,
                     acm_lim=np.ones(ac, np.float32), gamma=0.99, params=params, dtype=F64)
    ol = o.update(*batch, e1, e2)
    if bf16:
        check_sac(ag, o, ol, grad_tol=6e-2, loss_tol=3e-2, params_check=False)
    else:
        check_sac(ag, o, ol, grad_tol=2e-4, loss_tol=1e-4, params_check=params_check)


@pytest.mark.parametrize("B", [1, 33, 65536, 409600, 819200])  # 819,200 = rho * E: the ddpg_hcheetah bench batch
def test_ddpg_acm_update_large_batch_matches_oracle(B):
    ob, ac = 17, 6
    rng = np.random.RandomState(B % 977)
    ag = spprl.DDPG_AcM(env_name="HalfCheetah-v2", gamma=0.95, actor_lr=5e-4, critic_lr=5e-4, acm_critic=True,
                        custom_loss=1.0, norm_closs=False, min_max_denormalize=True, denormalize_actor_out=True,
                        max_batch=B, buffer_size=64, device=DEV, seed=4)
    params = snapshot(ag, DDPG_NETS)
    norm = set_minmax(ag, rng, ob)
    batch = random_batch(rng, B, ob, ob, ac)
    ag.update(*batch)
    torch.cuda.synchronize()
    o = OracleDdpgAcm(ob, ob, ac, norm=norm, actor_lim=1.0, gamma=0.95, tau=0.005, params=params, dtype=F64)
    ol = o.update(*batch)
    gl = ag.loss
    for k in ("critic", "actor"):
        e = relerr(ag.grads[DDPG_NETS[k]].cpu().numpy(), o.last["grads"][k])
        print(k, "grad rel err %.2e" % e)
        assert e < 2e-4, (k, e)
    for k in ("critic", "actor", "ddpg", "dist"):
        assert abs(gl[k] - ol[k]) <= 1e-4 * abs(ol[k]) + 1e-6, (k, gl[k], ol[k])
    for k in ("actor", "critic"):
        if B < 1000:  # a few samples: post-Adam parameters are a sign test of near-zero gradients (see above)
            break
        d = np.abs(ag.params[DDPG_NETS[k]].cpu().numpy() - o.flat(k))
        assert d.max() <= 2 * 5e-4 * 1.01 and np.mean(d > 1e-5) < 2e-3, (k, d.max())


# ------------------------------------------------------------------ the bench's staged path
def _filled(ag, rng, n_rows, ob, ac):
    rb = ag.replay_buffer
    slots = rb.add_obs_batch(torch.from_numpy(rng.randn(n_rows + 1, ob).astype(np.float32)))
    rb.add_timestep_batch(slots[:n_rows], slots[1:], torch.from_numpy(rng.randn(n_rows, ob).astype(np.float32)),
                          rng.randn(n_rows).astype(np.float32), rng.rand(n_rows) < 0.05, rng.rand(n_rows) < 0.05,
                          torch.from_numpy(rng.uniform(-1, 1, (n_rows, ac)).astype(np.float32)))
    rb.update_obs_mean_std()
    return rb


@pytest.mark.parametrize("env_name,ob,ac,B,bf16", [("Hopper-v2", 11, 3, 409600, False),
                                                   ("Ant-v2", 111, 8, 409600, True)])
def test_staged_replay_update_with_device_draws_matches_oracle(env_name, ob, ac, B, bf16):
    """The exact sequence bench.py times per vector step (OffPolicyLoop._fused_make_update):
    sppRandIndex -> sppAgentStageFromReplay -> sppSacAcmDrawEps -> critic grads / apply ->
    actor grads / apply.  The device indices and eps are read back and replayed through the
    oracle on the gathered tuples."""
    rng = np.random.RandomState(11)
    n_rows = 200_000
    ag = spprl.SAC_AcM(env_name=env_name, acm_critic=True, custom_loss=0.2, norm_closs=False, min_max_denormalize=True,
                       denormalize_actor_out=True, gamma=0.99, max_batch=B, buffer_size=n_rows + 64, device=DEV,
                       seed=5, mlp_bf16=bf16)
    rb = _filled(ag, rng, n_rows, ob, ac)
    params = snapshot(ag, SAC_NETS)
    st = _lib.stream_handle()
    idx = torch.empty(B, dtype=torch.int64, device=DEV)
    _lib.call("sppRandIndex", _lib.ptr(idx), B, len(rb), 77, 5, st)
    _lib.call("sppAgentStageFromReplay", ag._h, rb._h, _lib.ptr(idx), B, st)
    _lib.call("sppSacAcmDrawEps", ag._h, 78, 3, st)
    eps = [torch.empty(B, ob, device=DEV) for _ in range(2)]
    for w in (0, 1):
        _lib.call("sppAgentReadEps", ag._h, w, _lib.ptr(eps[w]), st)
    batch = [t.cpu().numpy() for t in rb.gather(idx)]  # reference layout tuples (bit-exact gather)
    norm = Norm(True, rb.min_obs.cpu().clone(), rb.max_obs.cpu().clone())
    _lib.call("sppSacAcmCriticGrads", ag._h, None, None, _lib.ptr(ag._losses), st)
    _lib.call("sppSacAcmCriticApply", ag._h, st)
    _lib.call("sppSacAcmActorGrads", ag._h, None, _lib.ptr(ag._losses), st)
    _lib.call("sppSacAcmActorApply", ag._h, _lib.ptr(ag._losses), st)
    torch.cuda.synchronize()
    ix = idx.cpu().numpy()
    assert ix.min() >= 0 and ix.max() < len(rb)
    e1, e2 = eps[0].cpu().numpy(), eps[1].cpu().numpy()
    for e in (e1, e2):  # k_eps_fm draws: standard normal moments over 4.5e6 (11 dims) / 4.5e7 (111) values
        n = e.size
        assert abs(e.mean()) < 6 / np.sqrt(n) and abs(e.var() - 1) < 6 * np.sqrt(2.0 / n), (e.mean(), e.var())
    assert abs(np.corrcoef(e1.ravel()[:1 << 20], e2.ravel()[:1 << 20])[0, 1]) < 6 / np.sqrt(1 << 20)
    o = OracleSacAcm(ob, ob, ac, acm_critic=True, custom_loss=0.2, norm_closs=False, norm=norm, actor_lim=1.0,
                     acm_lim=np.ones(ac, np.float32), gamma=0.99, params=params, dtype=F64)
    ol = o.update(*batch, e1, e2)
    if bf16:
        check_sac(ag, o, ol, grad_tol=6e-2, loss_tol=3e-2, params_check=False)
    else:
        check_sac(ag, o, ol, grad_tol=2e-4, loss_tol=1e-4)


# ------------------------------------------------------------------ device samplers
@pytest.mark.parametrize("high", [3, 1 << 20, 999_983, 1_000_000, 10_000_000])
def test_rand_index_range_and_uniformity(high):
    from scipy import stats

    n = (1 << 22) + 5
    idx = torch.empty(n, dtype=torch.int64, device=DEV)
    _lib.call("sppRandIndex", _lib.ptr(idx), n, high, 1234, 9, _lib.stream_handle())
    x = idx.cpu().numpy()
    assert x.min() >= 0 and x.max() < high
    nb = min(high, 256)
    counts = np.bincount((x * nb) // high, minlength=nb)
    # equal-width bins of [0, high): expected mass proportional to the integers per bin
    edges = (np.arange(nb + 1) * high + nb - 1) // nb
    expected = np.diff(edges) / high * n
    p = stats.chisquare(counts, expected).pvalue
    assert p > 1e-4, p
    assert abs(x.mean() - (high - 1) / 2) < 6 * high / np.sqrt(12 * n)
    # consecutive draws uncorrelated; another counter gives another stream
    assert abs(np.corrcoef(x[:-1], x[1:])[0, 1]) < 6 / np.sqrt(n)
    _lib.call("sppRandIndex", _lib.ptr(idx), n, high, 1234, 10, _lib.stream_handle())
    y = idx.cpu().numpy()
    q = 1.0 / high
    assert np.mean(x == y) < q + 6 * np.sqrt(q * (1 - q) / n) + 1e-12


@pytest.mark.parametrize("n", [(1 << 22) + 3, 1001])
def test_rand_normal_moments(n):
    from scipy import stats

    out = torch.empty(n, device=DEV)
    _lib.call("sppRandNormal", _lib.ptr(out), n, 42, 1, _lib.stream_handle())
    x = out.cpu().numpy().astype(np.float64)
    assert np.isfinite(x).all()
    tol = 6 / np.sqrt(n)
    assert abs(x.mean()) < tol
    assert abs(x.var() - 1) < 6 * np.sqrt(2.0 / n)
    if n > 10000:
        assert abs(stats.skew(x)) < 6 * np.sqrt(6.0 / n)
        assert abs(stats.kurtosis(x)) < 6 * np.sqrt(24.0 / n)
        assert stats.kstest(x[: 1 << 20], "norm").pvalue > 1e-4
        assert abs(np.corrcoef(x[:-1], x[1:])[0, 1]) < tol
        assert np.abs(x).max() < 7.0  # u01 never returns 0: the Box-Muller radius is bounded (~5.7)


@pytest.mark.parametrize("n", [1, 5, 32768, 1_802_240, 14_417_920])
def test_rand_perm_is_a_uniform_permutation(n):
    """sppRandPerm (the epochs' shuffle: below 2^20 rows 64-bit Philox keys + a radix sort of (key, index), from
    2^20 a keyed Feistel bijection with cycle walking): a permutation of [0, n) (sorted = arange), reproducible
    for a (seed, offset), a different one for another offset; at n = 5 the 120 orders are equally likely over
    24,000 draws (chi-square) and every position's value is uniform; at the bench's sizes (the actor epoch's
    32,768 rows, the ACM rings' 1,802,240 and 14,417,920: the world-1 and world-8 shapes) the displacement of a
    value is uncorrelated with its index, and from 2^20 on (the Feistel path) the first 2^20 positions' values
    fall uniformly into 1,000 bins, consecutive positions' values are uncorrelated, and the fixed points are as
    few as a uniform permutation's (Poisson(1))."""
    from scipy import stats

    from spprl.perm import device_randperm

    p = device_randperm(n, 77, 0, DEV)
    x = p.cpu().numpy()
    np.testing.assert_array_equal(np.sort(x), np.arange(n))
    np.testing.assert_array_equal(device_randperm(n, 77, 0, DEV).cpu().numpy(), x)
    if n > 1:
        y = device_randperm(n, 77, n, DEV).cpu().numpy()
        assert not np.array_equal(x, y)
    if n == 5:
        draws = np.stack([device_randperm(5, 3, 5 * k, DEV).cpu().numpy() for k in range(24000)])
        code = (draws * (5 ** np.arange(5))).sum(1)
        _, counts = np.unique(code, return_counts=True)
        assert len(counts) == 120
        assert stats.chisquare(counts).pvalue > 1e-4
        for pos in range(5):
            assert stats.chisquare(np.bincount(draws[:, pos], minlength=5)).pvalue > 1e-4
    if n >= 32768:
        assert abs(np.corrcoef(np.arange(n), x)[0, 1]) < 6 / np.sqrt(n)
    if n >= 1 << 20:
        head = x[: 1 << 20]
        assert stats.chisquare(np.bincount(head * 1000 // n, minlength=1000)).pvalue > 1e-4
        assert abs(np.corrcoef(head[:-1], head[1:])[0, 1]) < 6 / np.sqrt(head.size)
        assert int((x == np.arange(n)).sum()) <= 12
        # the stream's scratch has grown to this n: a small permutation through the larger buffer
        np.testing.assert_array_equal(np.sort(device_randperm(7, 77, 0, DEV).cpu().numpy()), np.arange(7))


def test_rand_streams_do_not_alias():
    """Distinct (key, counter) pairs give unrelated streams (the loop derives one key per
    consumer: policy eps, indices, update eps, env resets)."""
    from spprl.dp import stream_key

    keys = {stream_key(0, t) for t in ("policy", "index", "update_eps", "env", "env_action")}
    assert len(keys) == 5
    n = 1 << 16
    a = torch.empty(n, device=DEV)
    b = torch.empty(n, device=DEV)
    _lib.call("sppRandNormal", _lib.ptr(a), n, stream_key(0, "policy"), 1, _lib.stream_handle())
    _lib.call("sppRandNormal", _lib.ptr(b), n, stream_key(0, "env"), 1, _lib.stream_handle())
    x, y = a.cpu().numpy(), b.cpu().numpy()
    assert abs(np.corrcoef(x, y)[0, 1]) < 6 / np.sqrt(n)
    assert not np.any(x == y)


@pytest.mark.parametrize("B", [1000, 65536])
def test_draw_eps_ragged_batch_law_and_determinism(B):
    """sppSacAcmDrawEps (k_eps_fm: 4 normals per philox block, hardware Box-Muller) on a batch whose
    padded width Bp is not B: standard normal law over the valid samples (moments, KS), the same
    (seed, counter) reproduces the draws bit for bit, EPS1 / EPS2 and the next counter are unrelated."""
    from scipy import stats

    ob = 11
    rng = np.random.RandomState(3)
    ag = spprl.SAC_AcM(env_name="Hopper-v2", max_batch=B, buffer_size=5000, device=DEV, seed=0)
    rb = _filled(ag, rng, 4000, ob, 3)
    st = _lib.stream_handle()
    idx = torch.randint(0, len(rb), (B,), device=DEV)
    _lib.call("sppAgentStageFromReplay", ag._h, rb._h, _lib.ptr(idx), B, st)

    def draw(counter):
        _lib.call("sppSacAcmDrawEps", ag._h, 91, counter, st)
        out = [torch.empty(B, ob, device=DEV) for _ in range(2)]
        for w in (0, 1):
            _lib.call("sppAgentReadEps", ag._h, w, _lib.ptr(out[w]), st)
        torch.cuda.synchronize()
        return [o.cpu().numpy().astype(np.float64) for o in out]

    e1, e2 = draw(7)
    r1, r2 = draw(7)
    n1, _ = draw(8)
    assert np.array_equal(e1, r1) and np.array_equal(e2, r2)
    for e in (e1, e2):
        x = e.ravel()
        n = x.size
        assert np.isfinite(x).all() and np.abs(x).max() < 7.0
        assert abs(x.mean()) < 6 / np.sqrt(n) and abs(x.var() - 1) < 6 * np.sqrt(2.0 / n)
        assert stats.kstest(x, "norm").pvalue > 1e-4
    for a, b in ((e1, e2), (e1, n1)):
        assert abs(np.corrcoef(a.ravel(), b.ravel())[0, 1]) < 6 / np.sqrt(a.size)
