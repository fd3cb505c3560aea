"""GPU parity: the HIP library (through the C-ABI) against the oracle and the
reference's golden vectors.  Tolerances (fp32 path, written per check):
  - per-sample MLP outputs / dense layers: rtol 2e-5, atol 2e-5 * scale
  - gradients: ||g_gpu - g_ref|| / ||g_ref|| < 2e-4 per network
  - losses: rtol 1e-4;  alpha: rtol 1e-5
  - replay indexing / gathers / obs statistics: bit-exact
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected on CPU boxes, skipped there
    pytest.skip("needs a GPU", allow_module_level=True)

import spprl  # noqa: E402
from spprl import _lib  # noqa: E402
from golden_cases import SAC_CASES, load, sac_case  # noqa: E402
from oracle import nets as onets  # noqa: E402
from oracle.acm import OracleAcmTrainer  # noqa: E402
from oracle.sac_acm import OracleSacAcm  # noqa: E402
from weights import fill_params  # noqa: E402

DEV = torch.device("cuda:0")


def relerr(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


# ------------------------------------------------------------------ MFMA tile layout
@pytest.mark.parametrize("K,N,act", [(11, 256, 1), (14, 256, 1), (22, 64, 2), (3, 256, 1), (3, 22, 0), (8, 64, 2), (17, 96, 1), (256, 256, 1), (256, 22, 0),
                                     (256, 1, 0), (64, 32, 2), (32, 3, 2), (111, 256, 1), (222, 64, 0)])
def test_dense_tile_matches_torch(K, N, act):
    torch.manual_seed(K * 1000 + N)
    B = 77
    x = torch.randn(B, K)
    W = torch.randn(N, K) / np.sqrt(K)
    b = torch.randn(N)
    y = torch.empty(B, N, device=DEV)
    xd, Wd, bd = x.to(DEV), W.to(DEV), b.to(DEV)  # keep the device copies alive across the call
    _lib.call("sppDebugDense", _lib.ptr(xd), _lib.ptr(Wd), _lib.ptr(bd), _lib.ptr(y), B, K, N, act,
              _lib.stream_handle())
    ref = x.double() @ W.double().T + b.double()
    if act == 1:
        ref = ref.clamp_min(0)
    elif act == 2:
        ref = torch.tanh(ref)
    np.testing.assert_allclose(y.cpu().numpy(), ref.numpy(), rtol=2e-5, atol=2e-5)


# ------------------------------------------------------------------ replay ring
def replay_from_fixture(fx, tag):
    p = "r%s_" % tag
    size, ob, aout, ac = (int(v) for v in fx[p + "dims"])
    rb = spprl.BufferAcMOffPolicy(size, ob, aout, ac, device=DEV)
    oi = si = 0
    states = []
    for kind, a, b in fx[p + "ops"]:
        if kind == 0:
            assert rb.add_obs(torch.from_numpy(fx[p + "obs"][oi])) == a
            oi += 1
        else:
            rb.add_acm_action(fx[p + "acm"][si])
            assert rb.add_obs(torch.from_numpy(fx[p + "obs"][oi])) == b
            oi += 1
            rb.add_timestep(a, b, fx[p + "act"][si], fx[p + "rew"][si], fx[p + "done"][si], fx[p + "end"][si])
            si += 1
            states.append((rb.obs_idx, rb.ts_idx, rb.current_len))
    return rb, p, states


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_replay_ring_sampling_and_stats_bit_exact(tag):
    fx = load("replay_ring")
    rb, p, states = replay_from_fixture(fx, tag)
    np.testing.assert_array_equal(np.array(states), fx[p + "states"])
    for s in (0, 5):
        q = p + "s%d_" % s
        np.random.seed(s)
        o, no, a, r, d, acm = rb.sample_batch(33)
        for got, key in ((o, "obs"), (no, "next_obs"), (a, "act"), (r, "rew"), (d, "done"), (acm, "acm")):
            np.testing.assert_array_equal(got.cpu().numpy(), fx[q + key], err_msg=key)
    np.random.seed(9)
    o, no, acm = rb.sample_acm_batch(17)
    np.testing.assert_array_equal(o.cpu().numpy(), fx[p + "acmb_obs"])
    np.testing.assert_array_equal(acm.cpu().numpy(), fx[p + "acmb_acm"])
    rb.update_obs_mean_std()
    got = np.stack([t.cpu().numpy() for t in (rb.obs_mean, rb.obs_std, rb.max_obs, rb.min_obs)])
    want = fx[p + "st1"]
    if np.isnan(want[2]).all():  # len <= 10: reference skips the update
        np.testing.assert_array_equal(got[:2], want[:2])
    else:
        np.testing.assert_array_equal(got, want)


def test_obs_stats_large_exact():
    rng = np.random.RandomState(7)
    N, ob = 200_000, 11
    rb = spprl.BufferAcMOffPolicy(N + 10, ob, ob, 3, device=DEV)
    obs = (rng.standard_t(3, size=(N + 1, ob)) * rng.uniform(0.1, 5, ob)).astype(np.float32)
    slots = rb.add_obs_batch(torch.from_numpy(obs))
    E = N
    rb.add_timestep_batch(slots[:E], slots[1:E + 1], torch.zeros(E, ob), np.zeros(E), np.zeros(E, bool),
                          np.zeros(E, bool), torch.zeros(E, 3))
    assert len(rb) == N
    rb.update_obs_mean_std()
    x = obs[:N].astype(np.float64)
    want = np.stack([x.mean(0), x.std(0), np.percentile(x, 99, axis=0), np.percentile(x, 1, axis=0)]).astype(
        np.float32)
    got = np.stack([t.cpu().numpy() for t in (rb.obs_mean, rb.obs_std, rb.max_obs, rb.min_obs)])
    np.testing.assert_array_equal(got[2:], want[2:])  # order statistics: exact
    np.testing.assert_allclose(got[:2], want[:2], rtol=2e-7, atol=0)  # fp64 sums, fp32 cast


# ------------------------------------------------------------------ SAC_AcM.update
def build_agent(cfg, fx, params, norm, B):
    ob, aout, ac = (int(v) for v in fx["dims"][:3])
    env_spec = (ob, ac, 1.0, 1000)
    ag = spprl.SAC_AcM(env_name="custom", env_spec=env_spec, gamma=float(fx["gamma"]), acm_critic=cfg["acm_critic"],
                       custom_loss=cfg["custom_loss"], norm_closs=cfg["norm_closs"],
                       min_max_denormalize=cfg["min_max"], denormalize_actor_out=cfg["min_max"],
                       alpha=float(fx["alpha0"]), max_batch=B, buffer_size=64, device=DEV)
    names = {"actor": _lib.SPP_NET_ACTOR, "critic_1": _lib.SPP_NET_CRITIC1, "critic_2": _lib.SPP_NET_CRITIC2,
             "critic_1_targ": _lib.SPP_NET_CRITIC1_TARG, "critic_2_targ": _lib.SPP_NET_CRITIC2_TARG,
             "acm": _lib.SPP_NET_ACM}
    for k, net in names.items():
        ag.load_net(net, params[k])
    rb = ag.replay_buffer
    rb.min_obs.copy_(norm.lo)
    rb.max_obs.copy_(norm.hi)
    rb.obs_mean.copy_(norm.mean)
    rb.obs_std.copy_(norm.std)
    rb._have_minmax = True
    return ag, names


@pytest.mark.parametrize("name", list(SAC_CASES))
def test_sac_acm_update_matches_oracle_and_reference(name):
    cfg, fx, params, layouts, norm, steps = sac_case(name)
    ob, aout, ac, B = (int(v) for v in fx["dims"])
    ag, names = build_agent(cfg, fx, params, norm, B)
    o = OracleSacAcm(ob, aout, ac, acm_critic=cfg["acm_critic"], custom_loss=cfg["custom_loss"],
                     norm_closs=cfg["norm_closs"], norm=norm, actor_lim=fx["actor_ac_lim"], acm_lim=fx["acm_ac_lim"],
                     gamma=float(fx["gamma"]), tau=float(fx["tau"]), alpha=float(fx["alpha0"]),
                     target_entropy=float(fx["target_entropy"]), params=params)
    for i, (batch, e1, e2) in enumerate(steps):
        ag.update(*batch, eps_next=e1, eps_cur=e2)
        ol = o.update(*batch, e1, e2)
        torch.cuda.synchronize()
        for k in ("critic_1", "critic_2", "actor"):
            g = ag.grads[names[k]].cpu().numpy()
            assert relerr(g, o.last["grads"][k]) < 2e-4, (k, relerr(g, o.last["grads"][k]))
        gl = ag.loss
        for k in ("critic_1", "critic_2", "actor"):
            assert gl[k] == pytest.approx(ol[k], rel=1e-4, abs=1e-6), k
            assert gl[k] == pytest.approx(float(fx["losses"][i][["critic_1", "critic_2", "actor"].index(k)]),
                                          rel=1e-4, abs=1e-6)
        if cfg["custom_loss"]:
            assert gl["sac"] == pytest.approx(ol["sac"], rel=1e-4, abs=1e-6)
            assert gl["dist"] == pytest.approx(ol["dist"], rel=1e-4, abs=1e-6)
    assert ag.current_alpha() == pytest.approx(float(fx["alpha"]), rel=1e-5)
    lr = 1e-3
    for k in ("actor", "critic_1", "critic_2", "critic_1_targ", "critic_2_targ"):
        got = ag.params[names[k]].cpu().numpy()
        want = fx["post_" + k]
        d = np.abs(got - want)
        # Adam's first steps move every weight by ~lr*sign(g): a weight whose gradient is at
        # rounding-noise level may take the other sign; require that to be rare and bounded.
        assert d.max() <= 2 * len(steps) * lr * 1.01, (k, d.max())
        assert np.mean(d > 1e-5) < 2e-3, (k, np.mean(d > 1e-5))


# ------------------------------------------------------------------ ACM regression + rollout action
def test_acm_regress_matches_oracle_and_reference():
    fx = load("acm_step")
    seed = int(fx["seed"])
    lay = onets.acm_layout(22, 3)
    params = fill_params(lay, seed)
    ag = spprl.SAC_AcM(env_name="Hopper-v2", acm_lr=1e-3, max_batch=128, buffer_size=64, device=DEV)
    ag.load_net(_lib.SPP_NET_ACM, params)
    o = OracleAcmTrainer(22, 3, lr=1e-3, ac_lim=fx["ac_lim"], params=params)
    rng = np.random.RandomState(seed)
    for i in range(3):
        x = (rng.randn(100, 22) * 1.2).astype(np.float32)
        y = rng.uniform(-1, 1, (100, 3)).astype(np.float32)
        loss = ag.batch_update_acm(x, y)
        ol = o.batch_update(x, y)
        torch.cuda.synchronize()
        assert relerr(ag.grads[_lib.SPP_NET_ACM].cpu().numpy(), o.last_grad) < 2e-4
        assert float(loss.item()) == pytest.approx(ol, rel=1e-5)
        assert float(loss.item()) == pytest.approx(float(fx["losses"][i]), rel=1e-4)
    got = ag.params[_lib.SPP_NET_ACM].cpu().numpy()
    d = np.abs(got - fx["post_acm"])
    assert d.max() < 6 * 1e-3 and np.mean(d > 1e-5) < 2e-3


def test_policy_act_matches_oracle():
    cfg, fx, params, layouts, norm, steps = sac_case("sac_hopper_paper")
    ob, aout, ac, B = (int(v) for v in fx["dims"])
    ag, names = build_agent(cfg, fx, params, norm, B)
    rng = np.random.RandomState(3)
    E = 300
    obs = (rng.randn(E, ob) * 1.3).astype(np.float32)
    eps = rng.randn(E, aout).astype(np.float32)
    noise = rng.randn(E, aout).astype(np.float32)
    tgt, env = ag.act(torch.from_numpy(obs), eps=torch.from_numpy(eps).to(DEV), noise=torch.from_numpy(noise).to(DEV),
                      mode=1, act_noise=0.1)
    torch.cuda.synchronize()
    P = {k: {n: torch.from_numpy(v) for n, v in params[k].items()} for k in params}
    lim = torch.as_tensor(fx["actor_ac_lim"])
    with torch.no_grad():
        a, _, _ = onets.sac_actor(P["actor"], torch.from_numpy(obs), lim, torch.from_numpy(eps))
        a = a + 0.1 * torch.from_numpy(noise) * lim
        a = torch.clamp(a, -1.1 * lim, 1.1 * lim)
        ad = norm.denormalize(a)
        c = onets.acm(P["acm"], torch.cat([torch.from_numpy(obs), ad], 1), torch.as_tensor(fx["acm_ac_lim"]))
    np.testing.assert_allclose(tgt.cpu().numpy(), ad.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(env.cpu().numpy(), c.numpy(), rtol=1e-4, atol=1e-5)


def test_staged_update_runs_and_is_finite():
    """Fused device path: replay gather + device eps; repeated steps stay finite and deterministic."""
    torch.manual_seed(0)
    outs = []
    for rep in range(2):
        ag = spprl.SAC_AcM(env_name="Hopper-v2", acm_critic=True, custom_loss=0.2, norm_closs=False,
                           min_max_denormalize=True, denormalize_actor_out=True, max_batch=4096, buffer_size=5000,
                           device=DEV, seed=1)
        rb = ag.replay_buffer
        rng = np.random.RandomState(0)
        obs = torch.from_numpy(rng.randn(3001, 11).astype(np.float32))
        slots = rb.add_obs_batch(obs)
        E = 3000
        rb.add_timestep_batch(slots[:E], slots[1:], torch.from_numpy(rng.randn(E, 11).astype(np.float32)),
                              rng.randn(E).astype(np.float32), rng.rand(E) < 0.05, rng.rand(E) < 0.05,
                              torch.from_numpy(rng.uniform(-1, 1, (E, 3)).astype(np.float32)))
        rb.update_obs_mean_std()
        for step in range(3):
            idx = torch.from_numpy(np.random.RandomState(step).randint(0, len(rb), 4000))
            ag.update_from_replay(idx, seed=123, counter=step)
        torch.cuda.synchronize()
        p = ag.params[_lib.SPP_NET_ACTOR].cpu().numpy()
        assert np.isfinite(p).all()
        assert all(np.isfinite(v) for v in ag.loss.values())
        outs.append(p)
    np.testing.assert_array_equal(outs[0], outs[1])


def _filled_agent(env_name, ob, ac, n_rows, seed=1, max_batch=4096):
    ag = spprl.SAC_AcM(env_name=env_name, acm_critic=True, custom_loss=0.2, norm_closs=False, min_max_denormalize=True,
                       denormalize_actor_out=True, max_batch=max_batch, buffer_size=n_rows + 64, device=DEV, seed=seed)
    rb = ag.replay_buffer
    rng = np.random.RandomState(0)
    slots = rb.add_obs_batch(torch.from_numpy(rng.randn(n_rows + 1, ob).astype(np.float32)))
    rb.add_timestep_batch(slots[:n_rows], slots[1:], torch.from_numpy(rng.randn(n_rows, ob).astype(np.float32)),
                          rng.randn(n_rows).astype(np.float32), rng.rand(n_rows) < 0.05, rng.rand(n_rows) < 0.05,
                          torch.from_numpy(rng.uniform(-1, 1, (n_rows, ac)).astype(np.float32)))
    rb.update_obs_mean_std()
    return ag


@pytest.mark.parametrize("env_name,ob,ac,B", [("Hopper-v2", 11, 3, 1000), ("Ant-v2", 111, 8, 613)])
def test_replay_staged_update_bit_exact_vs_explicit_batch(env_name, ob, ac, B):
    """sppAgentStageFromReplay (tiled random-row gather -> feature-major scratch, ragged last
    tile) feeds the same kernels as the caller-batch path: identical bits after a full step."""
    a1 = _filled_agent(env_name, ob, ac, 3000)
    a2 = _filled_agent(env_name, ob, ac, 3000)
    idx = torch.from_numpy(np.random.RandomState(5).randint(0, 3000, B)).to(DEV)
    rng = np.random.RandomState(9)
    e1 = torch.from_numpy(rng.randn(B, ob).astype(np.float32)).to(DEV)
    e2 = torch.from_numpy(rng.randn(B, ob).astype(np.float32)).to(DEV)
    st = _lib.stream_handle()
    _lib.call("sppAgentStageFromReplay", a1._h, a1.replay_buffer._h, _lib.ptr(idx), B, st)
    _lib.call("sppSacAcmCriticGrads", a1._h, None, _lib.ptr(e1), _lib.ptr(a1._losses), st)
    _lib.call("sppSacAcmCriticApply", a1._h, st)
    _lib.call("sppSacAcmActorGrads", a1._h, _lib.ptr(e2), _lib.ptr(a1._losses), st)
    _lib.call("sppSacAcmActorApply", a1._h, _lib.ptr(a1._losses), st)
    a2.update(*a2.replay_buffer.gather(idx), eps_next=e1, eps_cur=e2)
    torch.cuda.synchronize()
    for net in (_lib.SPP_NET_ACTOR, _lib.SPP_NET_CRITIC1, _lib.SPP_NET_CRITIC2):
        np.testing.assert_array_equal(a1.params[net].cpu().numpy(), a2.params[net].cpu().numpy())
    assert a1.loss == a2.loss


@pytest.mark.parametrize("env_name,ob,ac,B", [("Hopper-v2", 11, 3, 1000), ("Ant-v2", 111, 8, 613)])
def test_replay_gather_acm_bit_exact(env_name, ob, ac, B):
    ag = _filled_agent(env_name, ob, ac, 3000)
    rb = ag.replay_buffer
    idx = torch.from_numpy(np.random.RandomState(7).randint(0, 3000, B)).to(DEV)
    x = torch.empty(B, 2 * ob, device=DEV)
    y = torch.empty(B, ac, device=DEV)
    _lib.call("sppReplayGatherAcm", rb._h, _lib.ptr(idx), B, _lib.ptr(x), _lib.ptr(y), _lib.stream_handle())
    o, no, _, _, _, acm = rb.gather(idx)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(x.cpu().numpy(), torch.cat([o, no], 1).cpu().numpy())
    np.testing.assert_array_equal(y.cpu().numpy(), acm.cpu().numpy())


def test_synth_env_step_matches_numpy():
    E, ob, ac = 37, 111, 8
    rng = np.random.RandomState(3)
    A = (rng.randn(ob, ob) * 0.05).astype(np.float32)
    s = rng.randn(E, ob).astype(np.float32)
    a = rng.uniform(-1, 1, (E, ac)).astype(np.float32)
    dA, ds, da = (torch.from_numpy(v).to(DEV) for v in (A, s, a))
    ns = torch.empty(E, ob, device=DEV)
    r = torch.empty(E, device=DEV)
    _lib.call("sppSynthEnvStep", _lib.ptr(dA), _lib.ptr(ds), _lib.ptr(da), E, ob, ac, _lib.ptr(ns), _lib.ptr(r),
              _lib.stream_handle())
    ref = np.tanh(s.astype(np.float64) @ A.T.astype(np.float64)) + 0.1 * np.resize(a, (E, ac))[:, np.arange(ob) % ac]
    np.testing.assert_allclose(ns.cpu().numpy(), ref, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(r.cpu().numpy(), -np.square(a).sum(1) + ref[:, 0], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("ob,ranks", [(11, 2), (17, 3), (111, 2)])
def test_obs_stats_data_parallel_protocol_matches_union(ob, ranks):
    """sppReplayObsStatsDP over W shards, all-reduced in lockstep here on one GPU, equals the
    single-buffer statistics of the union of the shards (percentiles, max/min bit-exact;
    mean / std rtol 1e-6, the fp64 sums differ only in summation order / pivot)."""
    rng = np.random.RandomState(ob)
    sizes = [5000 + 997 * r for r in range(ranks)]
    data = [(rng.standard_t(3, size=(n, ob)) * rng.uniform(0.5, 3, ob) + rng.randn(ob)).astype(np.float32)
            for n in sizes]

    def buf(rows):
        rb = spprl.BufferAcMOffPolicy(len(rows) + 8, ob, ob, 2, device=DEV, min_max_denormalize=True)
        sl = rb.add_obs_batch(torch.from_numpy(np.concatenate([rows, rows[:1]])))
        n = len(rows)
        z = np.zeros(n, bool)
        rb.add_timestep_batch(sl[:n], sl[1:], torch.zeros(n, ob), np.zeros(n, np.float32), z, z,
                              torch.zeros(n, 2))
        return rb

    shards = [buf(d) for d in data]
    union = buf(np.concatenate(data))
    union.update_obs_mean_std()
    for rb in shards:
        rb.obs_mean.copy_(torch.from_numpy(rng.randn(ob).astype(np.float32)))  # any replicated pivot works
        rb._dp_hist = torch.zeros(_lib.load().sppReplayObsStatsDPHistSize(rb._h), dtype=torch.int32, device=DEV)
        rb._dp_sums = torch.zeros(ob, 2, dtype=torch.float64, device=DEV)
        rb._dp_pivot = torch.zeros(ob, device=DEV)
    pivot = shards[0].obs_mean.clone()
    for rb in shards:
        rb.obs_mean.copy_(pivot)
    n_global = sum(sizes)
    gens = [rb.obs_stats_dp_steps(n_global) for rb in shards]
    while True:
        steps = [next(g, None) for g in gens]
        if steps[0] is None:
            assert all(s is None for s in steps)
            break
        if steps[0] == 0:
            tot = sum(rb._dp_sums for rb in shards)
            for rb in shards:
                rb._dp_sums.copy_(tot)
        tot = sum(rb._dp_hist for rb in shards)
        for rb in shards:
            rb._dp_hist.copy_(tot)
    torch.cuda.synchronize()
    for rb in shards:
        np.testing.assert_array_equal(rb.max_obs.cpu().numpy(), union.max_obs.cpu().numpy())
        np.testing.assert_array_equal(rb.min_obs.cpu().numpy(), union.min_obs.cpu().numpy())
        np.testing.assert_allclose(rb.obs_mean.cpu().numpy(), union.obs_mean.cpu().numpy(), rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(rb.obs_std.cpu().numpy(), union.obs_std.cpu().numpy(), rtol=1e-6)
    allx = np.concatenate(data).astype(np.float64)
    np.testing.assert_array_equal(union.max_obs.cpu().numpy(), np.percentile(allx, 99, axis=0).astype(np.float32))
    np.testing.assert_array_equal(union.min_obs.cpu().numpy(), np.percentile(allx, 1, axis=0).astype(np.float32))


@pytest.mark.parametrize("env_name,ob,ac,bs", [("Hopper-v2", 11, 3, 100), ("HalfCheetah-v2", 17, 6, 64),
                                               ("HalfCheetah-v2", 17, 6, 129), ("Hopper-v2", 11, 3, 256),
                                               ("Hopper-v2", 11, 3, 700), ("HalfCheetah-v2", 17, 6, 1049),
                                               ("HalfCheetah-v2", 17, 6, 2500)])
def test_acm_persistent_sgd_matches_oracle(env_name, ob, ac, bs):
    """sppAcmSgd (K sequential AcM regression steps in one launch, parameters in LDS) against
    the oracle's AcMTrainer.batch_update sequence on the same replay batches (acm.py:246-264):
    losses rtol 1e-4; parameters after K Adam steps within 1e-5 * max(1, |p|) except for a
    few lr-sized flips of near-zero-moment coordinates.  bs 700 / 1049 (the PPO bench's scaled
    ACM batch) run the multi-workgroup form: each step over max(2, ceil(bs/64)) 4-wave workgroups whose gradients
    are summed behind one arrival barrier per step (its timeout flag must stay clear)."""
    ag = _filled_agent(env_name, ob, ac, 2000, seed=4)
    rb = ag.replay_buffer
    params = {k: v.numpy() for k, v in ag.net_state(_lib.SPP_NET_ACM).items()}
    o = OracleAcmTrainer(2 * ob, ac, lr=ag.acm_lr, ac_lim=ag.ac_lim.numpy(), params=params)
    K = 6
    idx = torch.from_numpy(np.random.RandomState(11).randint(0, 2000, K * bs)).to(DEV)
    loss = torch.zeros(1, device=DEV)
    xg = torch.empty(K * bs, 2 * ob, device=DEV)
    yg = torch.empty(K * bs, ac, device=DEV)
    _lib.call("sppReplayGatherAcm", rb._h, _lib.ptr(idx), K * bs, _lib.ptr(xg), _lib.ptr(yg), _lib.stream_handle())
    _lib.call("sppAcmSgd", ag._h, _lib.ptr(xg), _lib.ptr(yg), K, bs, _lib.ptr(loss), _lib.stream_handle())
    ol = 0.0
    for k in range(K):
        obs, nobs, _, _, _, acm = rb.gather(idx[k * bs:(k + 1) * bs])
        ol += o.batch_update(torch.cat([obs, nobs], 1).cpu().numpy(), acm.cpu().numpy())
    torch.cuda.synchronize()
    assert float(loss.item()) == pytest.approx(ol, rel=1e-4)
    got = ag.params[_lib.SPP_NET_ACM].cpu().numpy()
    ref = o.flat()
    d = np.abs(got - ref)
    assert np.mean(d > 1e-5 * np.maximum(1, np.abs(ref))) < 5e-3 and d.max() < 4 * K * ag.acm_lr
    steps = np.zeros(4, np.int64)
    _lib.call("sppAgentGetSteps", ag._h, steps.ctypes.data_as(__import__("ctypes").c_void_p))
    assert steps[3] == K
    flag = np.ones(1, np.int32)
    _lib.call("sppAcmSgdStatus", ag._h, flag.ctypes.data)
    assert flag[0] == 0


@pytest.mark.parametrize("bs,nrows,passes", [(1049, 3 * 1049 + 2, 0), (700, 2 * 700 + 650, 0), (64, 5 * 64 + 1, 0),
                                             (1049, 3 * 1049 + 2, 2), (2500, 2 * 2500 + 300, 4)])
def test_acm_sgd_epoch_ragged_last_batch_matches_oracle(bs, nrows, passes):
    """sppAcmSgdEpoch: one update_acm epoch (DataLoader batches of bs, drop_last=False: acm.py:270-297) in
    ONE launch, the ragged last batch included: at 3 x 1049 + 2 rows the last step has 2 rows, so 16 of
    its 17 workgroups hold none; its loss is that batch's own mean.  passes > 0 (sppSetAcmSgdPasses): each
    workgroup runs that many 64-row passes per step (1049 rows on 9 workgroups, 2500 on 10), summed before the
    exchange.  Same tolerance as above."""
    _lib.call("sppSetAcmSgdPasses", passes)
    try:
        _acm_epoch_case(bs, nrows)
    finally:
        _lib.call("sppSetAcmSgdPasses", 0)


def _acm_epoch_case(bs, nrows):
    ag = _filled_agent("HalfCheetah-v2", 17, 6, 4000, seed=8)
    rb = ag.replay_buffer
    params = {k: v.numpy() for k, v in ag.net_state(_lib.SPP_NET_ACM).items()}
    o = OracleAcmTrainer(34, 6, lr=ag.acm_lr, ac_lim=ag.ac_lim.numpy(), params=params)
    idx = torch.from_numpy(np.random.RandomState(12).randint(0, 4000, nrows)).to(DEV)
    loss = torch.zeros(1, device=DEV)
    xg = torch.empty(nrows, 34, device=DEV)
    yg = torch.empty(nrows, 6, device=DEV)
    _lib.call("sppReplayGatherAcm", rb._h, _lib.ptr(idx), nrows, _lib.ptr(xg), _lib.ptr(yg), _lib.stream_handle())
    _lib.call("sppAcmSgdEpoch", ag._h, _lib.ptr(xg), _lib.ptr(yg), nrows, bs, _lib.ptr(loss), _lib.stream_handle())
    x_all, y_all = xg.cpu().numpy(), yg.cpu().numpy()
    losses = [o.batch_update(x_all[s:s + bs], y_all[s:s + bs]) for s in range(0, nrows, bs)]
    torch.cuda.synchronize()
    assert float(loss.item()) == pytest.approx(sum(losses), rel=1e-4)
    got = ag.params[_lib.SPP_NET_ACM].cpu().numpy()
    ref = o.flat()
    d = np.abs(got - ref)
    assert np.mean(d > 1e-5 * np.maximum(1, np.abs(ref))) < 5e-3 and d.max() < 4 * len(losses) * ag.acm_lr
    steps = np.zeros(4, np.int64)
    _lib.call("sppAgentGetSteps", ag._h, steps.ctypes.data_as(__import__("ctypes").c_void_p))
    assert steps[3] == len(losses)
    flag = np.ones(1, np.int32)
    _lib.call("sppAcmSgdStatus", ag._h, flag.ctypes.data)
    assert flag[0] == 0


def test_acm_multi_workgroup_sgd_is_deterministic():
    """The multi-workgroup sppAcmSgd sums the workgroups' gradients in a fixed order: two agents with
    the same initial AcM and the same batches end bit-identical (what lets data-parallel ranks run
    the ACM epochs replicated, with no per-batch collective)."""
    bs, K = 1049, 20
    out = []
    for _ in range(2):
        ag = _filled_agent("HalfCheetah-v2", 17, 6, 4000, seed=9)
        rb = ag.replay_buffer
        idx = torch.from_numpy(np.random.RandomState(5).randint(0, 4000, K * bs)).to(DEV)
        xg = torch.empty(K * bs, 34, device=DEV)
        yg = torch.empty(K * bs, 6, device=DEV)
        loss = torch.zeros(1, device=DEV)
        _lib.call("sppReplayGatherAcm", rb._h, _lib.ptr(idx), K * bs, _lib.ptr(xg), _lib.ptr(yg),
                  _lib.stream_handle())
        _lib.call("sppAcmSgd", ag._h, _lib.ptr(xg), _lib.ptr(yg), K, bs, _lib.ptr(loss), _lib.stream_handle())
        torch.cuda.synchronize()
        out.append((ag.params[_lib.SPP_NET_ACM].cpu().clone(), float(loss.item())))
    assert torch.equal(out[0][0], out[1][0]) and out[0][1] == out[1][1]


@pytest.mark.parametrize("bs", [100, 160])
def test_update_acm_epochs_with_step_lr_match_oracle(bs, monkeypatch):
    """AcMTrainer.update_acm (acm.py:266-303, the pre-train epoch mode): shuffled epochs over every
    live row in batches of acm_batch_size with a ragged last batch, StepLR(step 1, gamma 0.5) stepped
    once per epoch, loss['acm'] = the last epoch's mean batch loss.  The oracle replays the same
    permutations (recorded from the loop's device_randperm) through AcMTrainer.batch_update with
    the scheduled lr.  bs = 100 runs the one-workgroup sppAcmSgd launches, bs = 160 the
    multi-workgroup form.  Tolerance as for the persistent SGD test, over all 3 x 21 (13) Adam steps."""
    import spprl.trainer as tr

    n = 2050
    ag = _filled_agent("Hopper-v2", 11, 3, n, seed=6)
    ag.acm_batch_size, ag.acm_scheduler_step, ag.acm_scheduler_gamma = bs, 1, 0.5
    perms = []
    real = tr.device_randperm

    def rec(*a, **k):
        p = real(*a, **k)
        perms.append(p.clone())
        return p

    monkeypatch.setattr(tr, "device_randperm", rec)
    rb = ag.replay_buffer
    params = {k: v.numpy() for k, v in ag.net_state(_lib.SPP_NET_ACM).items()}
    o = OracleAcmTrainer(22, 3, lr=ag.acm_lr, ac_lim=ag.ac_lim.numpy(), params=params)
    obs, nobs, _, _, _, acm = (t.cpu().numpy() for t in rb.gather(torch.arange(n, device=DEV)))
    x_all = np.concatenate([obs, nobs], 1)
    epochs = 3
    ag.update_acm(epochs, pretrain=True)
    torch.cuda.synchronize()
    assert len(perms) == epochs
    steps = 0
    for e, p in enumerate(perms):
        o.opt.lr = ag.acm_lr * 0.5 ** e
        p = p.cpu().numpy()
        losses = [o.batch_update(x_all[p[s:s + bs]], acm[p[s:s + bs]]) for s in range(0, n, bs)]
        steps += len(losses)
    assert ag.acm_loss == pytest.approx(np.mean(losses), rel=1e-4)
    got = ag.params[_lib.SPP_NET_ACM].cpu().numpy()
    ref = o.flat()
    d = np.abs(got - ref)
    assert np.mean(d > 1e-5 * np.maximum(1, np.abs(ref))) < 5e-3 and d.max() < 4 * steps * ag.acm_lr
    assert ag._acm_sched_epochs == epochs
    ss = np.zeros(4, np.int64)
    _lib.call("sppAgentGetSteps", ag._h, ss.ctypes.data_as(__import__("ctypes").c_void_p))
    assert ss[3] == steps


@pytest.mark.parametrize("env_name,ob,ac", [("Hopper-v2", 11, 3), ("Ant-v2", 111, 8)])
def test_sac_acm_update_bf16_mlp_within_bf16_tolerance(env_name, ob, ac):
    """mlp_bf16 (BASELINE configs[4]: bf16 MFMA MLP + fp32 targets): one SAC_AcM update against the
    fp32 oracle.  Tolerance stated for bf16 operands (8-bit mantissa, fp32 accumulation): losses
    rtol 3e-2, per-network gradient relative error < 6e-2; a wrong operand layout gives O(1)."""
    from oracle.nets import Norm

    B = 512
    rng = np.random.RandomState(1)
    ag = spprl.SAC_AcM(env_name=env_name, acm_critic=True, custom_loss=0.2, norm_closs=False, min_max_denormalize=True,
                       denormalize_actor_out=True, gamma=0.99, max_batch=B, buffer_size=128, device=DEV, seed=0,
                       mlp_bf16=True)
    names = {"actor": _lib.SPP_NET_ACTOR, "critic_1": _lib.SPP_NET_CRITIC1, "critic_2": _lib.SPP_NET_CRITIC2,
             "critic_1_targ": _lib.SPP_NET_CRITIC1_TARG, "critic_2_targ": _lib.SPP_NET_CRITIC2_TARG,
             "acm": _lib.SPP_NET_ACM}
    params = {k: {n: v.numpy() for n, v in ag.net_state(net).items()} for k, net in names.items()}
    lo = -rng.uniform(0.5, 2, ob).astype(np.float32)
    hi = rng.uniform(0.5, 2, ob).astype(np.float32)
    rb = ag.replay_buffer
    rb.min_obs.copy_(torch.from_numpy(lo))
    rb.max_obs.copy_(torch.from_numpy(hi))
    rb._have_minmax = True
    batch = (rng.randn(B, ob).astype(np.float32), rng.randn(B, ob).astype(np.float32),
             rng.uniform(-1, 1, (B, ob)).astype(np.float32), rng.randn(B).astype(np.float32),
             (rng.rand(B) < 0.1).astype(np.int8), rng.uniform(-1, 1, (B, ac)).astype(np.float32))
    e1, e2 = rng.randn(B, ob).astype(np.float32), rng.randn(B, ob).astype(np.float32)
    ag.update(*batch, eps_next=e1, eps_cur=e2)
    torch.cuda.synchronize()
    norm = Norm(True, torch.from_numpy(lo), torch.from_numpy(hi))
    o = OracleSacAcm(ob, ob, ac, acm_critic=True, custom_loss=0.2, norm_closs=False, norm=norm, actor_lim=1.0,
                     acm_lim=np.ones(ac, np.float32), gamma=0.99, params=params)
    ol = o.update(*batch, e1, e2)
    for k in ("critic_1", "critic_2", "actor"):
        err = relerr(ag.grads[names[k]].cpu().numpy(), o.last["grads"][k])
        assert err < 6e-2, (k, err)
    gl = ag.loss
    for k in ("critic_1", "critic_2", "actor"):
        assert abs(gl[k] - ol[k]) <= 3e-2 * abs(ol[k]) + 1e-3, (k, gl[k], ol[k])


@pytest.mark.parametrize("ob,ranks,kind", [(11, 2, "t3"), (17, 4, "t3"), (111, 3, "t3"), (11, 4, "skew"),
                                           (17, 2, "ties"), (11, 8, "t3")])
def test_obs_stats_one_pass_protocol_matches_union(ob, ranks, kind):
    """sppReplayObsStatsDP1 (the one-pass protocol) over W shards, its all-gather / all-reduces emulated here
    on one GPU between the phases, equals numpy on the union of the shards: percentiles and max/min
    bit-exact, mean / std rtol 1e-6, the same statistics on every shard.  "skew": unequal shifted shards,
    so the union sample (equal rows per shard) brackets the wrong place and the raw-column rounds must
    carry the selection; "ties": discrete values (long runs at the bracket bounds)."""
    rng = np.random.RandomState(ob + ranks)
    if kind == "skew":
        data = [(rng.randn(2000 * (1 + 5 * r), ob) * (0.5 + r) + 3.0 * r).astype(np.float32) for r in range(ranks)]
    elif kind == "ties":
        data = [np.round(rng.randn(7000 + 1000 * r, ob) * 2).astype(np.float32) for r in range(ranks)]
    else:
        data = [(rng.standard_t(3, size=(5000 + 997 * r, ob)) * rng.uniform(0.5, 3, ob) + rng.randn(ob))
                .astype(np.float32) for r in range(ranks)]

    def buf(rows):
        rb = spprl.BufferAcMOffPolicy(len(rows) + 8, ob, ob, 2, device=DEV, min_max_denormalize=True)
        sl = rb.add_obs_batch(torch.from_numpy(np.concatenate([rows, rows[:1]])))
        n = len(rows)
        z = np.zeros(n, bool)
        rb.add_timestep_batch(sl[:n], sl[1:], torch.zeros(n, ob), np.zeros(n, np.float32), z, z,
                              torch.zeros(n, 2))
        return rb

    shards = [buf(d) for d in data]
    pivot = torch.from_numpy(rng.randn(ob).astype(np.float32)).to(DEV)
    n_global = sum(len(d) for d in data)
    W = ranks
    Sl = _lib.load().sppReplayObsStatsDP1SampleRows(shards[0]._h, W, n_global)
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
        if phase == 0:  # all-gather: every rank's slot into every buffer
            allg = torch.cat([bufs[r]["samp"][r * ob * Sl:(r + 1) * ob * Sl] for r in range(W)])
            for b in bufs:
                b["samp"].copy_(allg)
        elif phase <= 5:  # all-reduce (sum)
            k = "exch" if phase == 1 else "hist"
            tot = sum(b[k] for b in bufs)
            for b in bufs:
                b[k].copy_(tot)
    torch.cuda.synchronize()
    allx = np.concatenate(data).astype(np.float64)
    for rb in shards:
        np.testing.assert_array_equal(rb.max_obs.cpu().numpy(), np.percentile(allx, 99, axis=0).astype(np.float32))
        np.testing.assert_array_equal(rb.min_obs.cpu().numpy(), np.percentile(allx, 1, axis=0).astype(np.float32))
        np.testing.assert_allclose(rb.obs_mean.cpu().numpy(), allx.mean(0).astype(np.float32), rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(rb.obs_std.cpu().numpy(), allx.std(0).astype(np.float32), rtol=1e-6)
