"""Pins the oracle (CPU restatement) against the golden vectors produced by the
reference itself (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from golden_cases import SAC_CASES, ddpg_case, ddpg_unbiased_case, load, sac_case
from oracle import nets
from oracle.acm import OracleAcmTrainer
from oracle.ddpg_acm import OracleDdpgAcm, make_unbiased_update
from oracle.ppo import clip_loss, gae_affine, gae_loop, q_val
from oracle.replay import OracleReplay
from oracle.rng import OracleMT
from oracle.sac_acm import OracleSacAcm
from weights import fill_params


def test_mt19937_randint_matches_numpy_golden():
    fx = load("mt19937_randint")
    for s, n, vals in zip(fx["seeds"], fx["ns"], fx["vals"]):
        got = OracleMT(int(s)).randint(int(n), vals.shape[0])
        np.testing.assert_array_equal(got, vals)
    mt = OracleMT(int(fx["seq_seed"]))
    for n, vals in zip(fx["seq_n"], fx["seq_vals"]):
        np.testing.assert_array_equal(mt.randint(int(n), len(vals)), vals)


def test_mt19937_randint_matches_installed_numpy():
    for seed, n in ((3, 977), (2**32 - 1, 2**32), (99, 1)):
        np.testing.assert_array_equal(OracleMT(seed).randint(n, 1000),
                                      np.random.RandomState(seed).randint(0, n, 1000))


def replay_from_fixture(fx, tag):
    p = "r%s_" % tag
    size, ob, aout, ac = (int(v) for v in fx[p + "dims"])
    rb = OracleReplay(size, ob, aout, ac)
    oi = si = 0
    states = []
    for kind, a, b in fx[p + "ops"]:
        if kind == 0:
            assert rb.add_obs(fx[p + "obs"][oi]) == a
            oi += 1
        else:
            rb.add_acm_action(fx[p + "acm"][si])
            assert rb.add_obs(fx[p + "obs"][oi]) == b
            oi += 1
            rb.add_timestep(a, b, fx[p + "act"][si], fx[p + "rew"][si], fx[p + "done"][si], fx[p + "end"][si])
            si += 1
            states.append((rb.obs_idx, rb.ts_idx, rb.current_len))
    return rb, p, states


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_replay_ring_and_sampling(tag):
    fx = load("replay_ring")
    rb, p, states = replay_from_fixture(fx, tag)
    np.testing.assert_array_equal(np.array(states), fx[p + "states"])
    L = rb.current_len
    np.testing.assert_array_equal(rb._obs_idx[:L], fx[p + "obs_idx"])
    np.testing.assert_array_equal(rb._next_obs_idx[:L], fx[p + "next_obs_idx"])
    for s in (0, 5):
        q = p + "s%d_" % s
        (o, no, a, r, d, acm), idx = rb.sample_batch(33, OracleMT(s))
        np.testing.assert_array_equal(idx, fx[q + "idx"])
        for got, key in ((o, "obs"), (no, "next_obs"), (a, "act"), (r, "rew"), (d, "done"), (acm, "acm")):
            np.testing.assert_array_equal(got, fx[q + key])
    (o, no, acm), _ = rb.sample_acm_batch(17, OracleMT(9))
    np.testing.assert_array_equal(o, fx[p + "acmb_obs"])
    np.testing.assert_array_equal(acm, fx[p + "acmb_acm"])
    for key in ("st1", "st2"):
        rb.update_obs_mean_std()
        nan = np.full(rb.ob, np.nan, np.float32)
        mx = nan if rb.max_obs is None else rb.max_obs
        mn = nan if rb.min_obs is None else rb.min_obs
        np.testing.assert_array_equal(np.stack([rb.obs_mean, rb.obs_std, mx, mn]), fx[p + key])
        rb._obs[rb._obs_idx[: rb.current_len]] *= 0.5


def test_q6_trace_from_survey():
    fx = load("replay_ring")
    rb, _, _ = replay_from_fixture(fx, "a")
    assert list(zip(rb._obs_idx[:8], rb._next_obs_idx[:8])) == [
        (0, 1), (2, 3), (3, 4), (4, 5), (6, 7), (7, 8), (8, 9), (9, 0)]
    assert len(rb) == 8


@pytest.mark.parametrize("name", list(SAC_CASES))
def test_sac_acm_update_matches_reference(name):
    cfg, fx, params, layouts, norm, steps = sac_case(name)
    ob, aout, ac, B = (int(v) for v in fx["dims"])
    o = OracleSacAcm(ob, aout, ac, acm_critic=cfg["acm_critic"], custom_loss=cfg["custom_loss"],
                     norm_closs=cfg["norm_closs"], norm=norm, actor_lim=fx["actor_ac_lim"],
                     acm_lim=fx["acm_ac_lim"], gamma=float(fx["gamma"]), tau=float(fx["tau"]),
                     alpha=float(fx["alpha0"]), target_entropy=float(fx["target_entropy"]), params=params)
    for i, (batch, e1, e2) in enumerate(steps):
        losses = o.update(*batch, e1, e2)
        np.testing.assert_allclose(o.last["y"].numpy(), fx["y"][i], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(o.last["logp"].numpy(), fx["logp"][i], rtol=1e-6, atol=1e-5)
        got = [losses[k] for k in ("critic_1", "critic_2", "actor", "sac", "dist")]
        np.testing.assert_allclose(got, fx["losses"][i], rtol=1e-6, atol=1e-7)
    for k in ("actor", "critic_1", "critic_2", "critic_1_targ", "critic_2_targ"):
        np.testing.assert_allclose(o.flat(k), fx["post_" + k], rtol=1e-6, atol=1e-7, err_msg=k)
    assert o.alpha == pytest.approx(float(fx["alpha"]), rel=1e-12)
    if "m_actor" in fx:
        for k in ("actor", "critic_1"):
            np.testing.assert_allclose(torch.cat([m.reshape(-1) for m in o.opt[k].m]).numpy(), fx["m_" + k],
                                       rtol=1e-5, atol=1e-9)
            np.testing.assert_allclose(torch.cat([v.reshape(-1) for v in o.opt[k].v]).numpy(), fx["v_" + k],
                                       rtol=1e-5, atol=1e-12)


def test_ddpg_acm_update_matches_reference():
    fx, params, layouts, norm, batches = ddpg_case()
    ob, aout, ac, B = (int(v) for v in fx["dims"])
    o = OracleDdpgAcm(ob, aout, ac, norm=norm, actor_lim=fx["actor_ac_lim"], gamma=float(fx["gamma"]),
                      tau=float(fx["tau"]), params=params)
    for i, batch in enumerate(batches):
        losses = o.update(*batch)
        np.testing.assert_allclose([losses[k] for k in ("critic", "actor", "ddpg", "dist")], fx["losses"][i],
                                   rtol=1e-6, atol=1e-7)
    for k in ("actor", "critic", "actor_targ", "critic_targ"):
        np.testing.assert_allclose(o.flat(k), fx["post_" + k], rtol=1e-6, atol=1e-7, err_msg=k)


def test_ddpg_acm_unbiased_make_update_matches_reference():
    """make_unbiased_update (ddpg_acm.py:59-73) over two cadences of the reference's ring: sampled indices,
    losses and post-step parameters (action = normalised next obs, acm_critic=False)."""
    fx, params, layouts, norm, replay = ddpg_unbiased_case()
    ob, aout, ac, B, gsteps, ufreq, size = (int(v) for v in fx["dims"])
    rb = OracleReplay(size, ob, aout, ac)
    replay(rb.add_obs, rb.add_acm_action, rb.add_timestep)
    params = dict(params, acm={n: np.zeros(s, np.float32) for n, s in nets.basic_acm_layout(2 * ob, ac)})
    o = OracleDdpgAcm(ob, aout, ac, acm_critic=False, custom_loss=0.3, norm_closs=True, norm=norm,
                      actor_lim=fx["actor_ac_lim"], gamma=float(fx["gamma"]), tau=float(fx["tau"]), params=params)
    for c, s in enumerate(fx["np_seeds"]):
        losses, idx = make_unbiased_update(o, rb, B, gsteps, OracleMT(int(s)), norm)
        np.testing.assert_array_equal(idx, fx["idx"][c])
        np.testing.assert_allclose([losses[k] for k in ("critic", "actor", "ddpg", "dist")], fx["losses"][c],
                                   rtol=1e-5, atol=1e-7)
    for k in ("actor", "critic", "actor_targ", "critic_targ"):
        np.testing.assert_allclose(o.flat(k), fx["post_" + k], rtol=1e-5, atol=1e-6, err_msg=k)
    # the branch matters: the biased update (action = the stored actor output) lands elsewhere
    o2 = OracleDdpgAcm(ob, aout, ac, acm_critic=False, custom_loss=0.3, norm_closs=True, norm=norm,
                       actor_lim=fx["actor_ac_lim"], gamma=float(fx["gamma"]), tau=float(fx["tau"]), params=params)
    (b_obs, b_nobs, b_act, b_rew, b_done, b_acm), _ = rb.sample_batch(B, OracleMT(int(fx["np_seeds"][0])))
    o2.update(norm.normalize(torch.from_numpy(b_obs)).numpy(), norm.normalize(torch.from_numpy(b_nobs)).numpy(),
              b_act, b_rew, b_done, b_acm)
    assert np.abs(o2.flat("critic") - fx["post_critic"]).max() > 1e-4


def test_sac_acm_unbiased_make_update_matches_reference():
    """SAC_AcM inherits DDPG_AcM.make_update (sac_acm.py:12, ddpg_acm.py:59-85): the unbiased branch over two
    cadences of the reference's ring (action = normalised next obs, acm_critic=False, z-score obs_norm), with the
    reference's injected rsample draws: sampled indices, losses, post-step parameters and alpha."""
    fx, params, layouts, norm, replay = ddpg_unbiased_case("sac_unbiased_hcheetah")
    ob, aout, ac, B, gsteps, ufreq, size = (int(v) for v in fx["dims"])
    rb = OracleReplay(size, ob, aout, ac)
    replay(rb.add_obs, rb.add_acm_action, rb.add_timestep)
    params = dict(params, acm={n: np.zeros(s, np.float32) for n, s in nets.acm_layout(2 * ob, ac)})
    o = OracleSacAcm(ob, aout, ac, acm_critic=False, custom_loss=0.3, norm_closs=True, norm=norm,
                     actor_lim=fx["actor_ac_lim"], gamma=float(fx["gamma"]), tau=float(fx["tau"]),
                     alpha=float(fx["alpha0"]), target_entropy=float(fx["target_entropy"]), params=params)
    for c, s in enumerate(fx["np_seeds"]):
        losses, idx = make_unbiased_update(o, rb, B, gsteps, OracleMT(int(s)), norm, eps=fx["eps"][c])
        np.testing.assert_array_equal(idx, fx["idx"][c])
        np.testing.assert_allclose([losses[k] for k in ("critic_1", "critic_2", "actor", "sac", "dist")],
                                   fx["losses"][c], rtol=1e-5, atol=1e-7)
    for k in ("actor", "critic_1", "critic_2", "critic_1_targ", "critic_2_targ"):
        np.testing.assert_allclose(o.flat(k), fx["post_" + k], rtol=1e-5, atol=1e-6, err_msg=k)
    assert o.alpha == pytest.approx(float(fx["alpha"]), rel=1e-10)


def test_acm_batch_update_matches_reference():
    fx = load("acm_step")
    seed = int(fx["seed"])
    lay = nets.acm_layout(22, 3)
    o = OracleAcmTrainer(22, 3, lr=1e-3, ac_lim=fx["ac_lim"], params=fill_params(lay, seed))
    rng = np.random.RandomState(seed)
    for i in range(3):
        x = (rng.randn(100, 22) * 1.2).astype(np.float32)
        y = rng.uniform(-1, 1, (100, 3)).astype(np.float32)
        assert o.batch_update(x, y) == pytest.approx(float(fx["losses"][i]), rel=1e-6)
    np.testing.assert_allclose(o.flat(), fx["post_acm"], rtol=1e-6, atol=1e-8)


def test_gae_and_clip_match_reference():
    fx = load("ppo_gae_clip")
    w = fx["w"]
    v_next = fx["next_obs"] @ w
    v = fx["obs"] @ w
    q = q_val(fx["rew"], fx["done"], v_next, float(fx["gamma"]))
    np.testing.assert_allclose(q, fx["q"], rtol=1e-6, atol=1e-6)
    delta = q - v
    adv = gae_loop(delta, fx["done"], fx["end"], v_next, float(fx["gamma"]), float(fx["lam"]))
    np.testing.assert_allclose(adv, fx["adv"], rtol=1e-5, atol=1e-5)
    adv2 = gae_affine(delta, fx["done"], fx["end"], v_next, float(fx["gamma"]), float(fx["lam"]))
    np.testing.assert_allclose(adv2, fx["adv"], rtol=1e-5, atol=1e-5)
    assert clip_loss(fx["clip_lp_old"], fx["clip_lp_new"], fx["clip_adv"]) == pytest.approx(
        float(fx["clip_loss"]), rel=1e-6)


def test_gae_reference_kat():
    """KAT of rltoolkit/algorithms/ppo/test/test_ppo.py:79-134 (gamma = lambda = 0.5)."""
    rew = np.array(list(range(10)) + [1, 2], np.float64)
    done = np.zeros(12)
    done[[3, 6, 11]] = 1
    end = done.copy()
    end[9] = 1
    obs = np.ones((12, 2)) * 5  # every obs 5 -> critic 10
    v = obs[:, 0] * 2
    q = q_val(rew, done, v, 0.5)
    np.testing.assert_array_equal(q, [5, 6, 7, 3, 9, 10, 6, 12, 13, 14, 6, 2])
    adv = gae_loop(q - v, done, end, v, 0.5, 0.5)
    np.testing.assert_almost_equal(adv, [-6.2969, -5.1875, -4.75, -7, -1.25, -1, -4, 3.1562, 4.625, 6.5, -6, -8],
                                   decimal=4)


@pytest.mark.parametrize("case", [
    ([-2.3, -5, -1.4, -1.5], [-2.3, -5, -1.4, -1.5], [1, 2.0, 3.0, 4.0], -2.5),
    ([-1.0], [-1.0], [-1.0], 1),
    ([-1.0], [-2.0], [-1.0], 0.8),
    ([-2.0], [-1.0], [1.0], -1.2),
    ([-1.0], [-2.0], [1.0], -0.3679),
])
def test_clip_loss_reference_kat(case):
    """KATs of rltoolkit/algorithms/ppo/test/test_ppo.py:34-76."""
    old, new, adv, want = case
    assert clip_loss(np.float32(old), np.float32(new), np.float32(adv)) == pytest.approx(want, rel=1e-4)


# ------------------------------------------------------------------ vanilla SAC (configs[0])
def test_vanilla_sac_update_matches_reference():
    from golden_cases import sac_vanilla_case
    from oracle.sac import OracleSac

    fx, params, steps = sac_vanilla_case()
    ob, ac, B = (int(v) for v in fx["dims"])
    assert float(fx["act_noise"]) == 0.1 and float(fx["tau"]) == 0.005  # quirk Q1
    assert int(fx["max_ep_len"]) == 1000  # quirk Q3: time-limit ends are not done
    o = OracleSac(ob, ac, ac_lim=fx["ac_lim"], gamma=float(fx["gamma"]), tau=float(fx["tau"]),
                  alpha=float(fx["alpha0"]), params=params)
    for i, (batch, e1, e2) in enumerate(steps):
        losses = o.update(*batch, e1, e2)
        np.testing.assert_allclose([losses[k] for k in ("critic_1", "critic_2", "actor")], fx["losses"][i],
                                   rtol=1e-6, atol=1e-7)
    for k in ("actor", "critic_1", "critic_2", "critic_1_targ", "critic_2_targ"):
        np.testing.assert_allclose(o.flat(k), fx["post_" + k], rtol=1e-6, atol=1e-7, err_msg=k)
    assert o.alpha == pytest.approx(float(fx["alpha"]), rel=1e-12)


# ------------------------------------------------------------------ on-policy (rows a21, a22, a24)
def test_onpolicy_actor_act_logprob_matches_reference():
    from golden_cases import onpolicy_case
    from oracle import onpolicy as oo

    fx = onpolicy_case()
    ob = fx["act_x"].shape[1]
    flat = fx["act_params"]
    sc = np.exp(flat[:ob].astype(np.float64))
    mu_ref = fx["act_mu"]
    eps = ((fx["act_a"] - mu_ref) / sc).astype(np.float32)  # the reference's normal draws, recovered
    a, lp = oo.act(flat, ob, ob, np.ones(ob, np.float32), fx["act_x"], eps)
    np.testing.assert_allclose(a, fx["act_a"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(lp, fx["act_lp"], rtol=1e-5, atol=1e-4)
    a, lp = oo.act(flat, ob, ob, np.ones(ob, np.float32), fx["act_x"], None)
    np.testing.assert_allclose(a, mu_ref, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(lp, fx["act_lp_det"], rtol=1e-6, atol=1e-5)


def test_onpolicy_update_critic_matches_reference():
    from golden_cases import onpolicy_case
    from oracle import onpolicy as oo
    from oracle.adam import OracleAdam

    fx = onpolicy_case()
    ob = fx["crit_obs"].shape[1]
    flat = torch.from_numpy(fx["crit_params0"].copy())
    opt = OracleAdam([flat], float(fx["crit_lr"]))
    g = float(fx["crit_gamma"])
    rew, done = torch.from_numpy(fx["crit_rew"]), torch.from_numpy(fx["crit_done"])
    total = 0.0
    for _ in range(10):
        with torch.no_grad():
            vn = oo.critic(oo._params(flat.numpy(), oo.critic_layout(ob)), torch.from_numpy(fx["crit_nobs"]))
        q = (rew + g * (1 - done) * vn.squeeze(-1)).numpy()
        for _ in range(10):
            loss, grad = oo.critic_step(flat.numpy(), ob, fx["crit_obs"], q)
            opt.step([torch.from_numpy(grad)])
            total += loss
    assert total / 100 == pytest.approx(float(fx["crit_loss"]), rel=1e-5)
    np.testing.assert_allclose(flat.numpy(), fx["crit_post"], rtol=1e-5, atol=1e-6)
    P = oo._params(flat.numpy(), oo.critic_layout(ob))
    with torch.no_grad():
        q = rew + g * (1 - done) * oo.critic(P, torch.from_numpy(fx["crit_nobs"])).squeeze(-1)
        adv = q - oo.critic(P, torch.from_numpy(fx["crit_obs"])).squeeze(-1)
    np.testing.assert_allclose(adv.numpy(), fx["crit_adv"], rtol=1e-5, atol=1e-5)


def test_onpolicy_ppo_acm_actor_step_matches_reference():
    from golden_cases import normalize_adv_ref, onpolicy_case
    from oracle import onpolicy as oo
    from oracle.adam import OracleAdam

    fx = onpolicy_case()
    ob = fx["crit_obs"].shape[1]
    adv = normalize_adv_ref(fx["ppo_adv"])
    out, g = oo.actor_step(fx["ppo_params0"], ob, ob, np.ones(ob, np.float32), fx["crit_obs"], fx["ppo_acts"],
                           fx["ppo_lp_old"], adv, eps_clip=float(fx["ppo_eps"]),
                           entropy_coef=float(fx["ppo_entropy_coef"]), next_obs=fx["crit_nobs"])
    policy = out["actor"] - float(fx["ppo_entropy_coef"]) * out["entropy"] + float(fx["ppo_custom_loss"]) * out["dist"]
    np.testing.assert_allclose([out["actor"], out["entropy"], policy, out["dist"]], fx["ppo_losses"], rtol=1e-5,
                               atol=1e-6)
    flat = torch.from_numpy(fx["ppo_params0"].copy())
    OracleAdam([flat], float(fx["ppo_lr"])).step([torch.from_numpy(g)])
    d = np.abs(flat.numpy() - fx["ppo_post"])
    assert d.max() < 1e-6, d.max()


def test_onpolicy_ppo_acm_actor_epochs_with_kl_stop_match_reference():
    """oracle.onpolicy.update_actor_epochs against the reference's multi-epoch update_actor_acm with the KL
    stop (tests/golden/ppo_epochs_hcheetah.npz): 4 epochs run, losses / 5, counter + 5, the per-epoch KLs."""
    from golden_cases import load, normalize_adv_ref
    from oracle import onpolicy as oo

    fx = load("ppo_epochs_hcheetah")
    ob = fx["obs"].shape[1]
    flat, losses, kls, cnt = oo.update_actor_epochs(
        fx["params0"], ob, ob, np.ones(ob, np.float32), fx["obs"], fx["acts"], fx["lp_old"],
        normalize_adv_ref(fx["adv"]), fx["nobs"], float(fx["lr"]), int(fx["max_epochs"]), float(fx["threshold"]),
        len(fx["obs"]), eps_clip=float(fx["eps"]), entropy_coef=float(fx["entropy_coef"]),
        custom_loss=float(fx["custom_loss"]))
    assert cnt == int(fx["counter"]) == 5 and len(kls) == 4
    np.testing.assert_allclose(kls, fx["kls"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose([losses[k] for k in ("actor", "entropy", "policy", "dist")], fx["losses"], rtol=1e-5,
                               atol=1e-6)
    d = np.abs(flat - fx["post"])
    lr = float(fx["lr"])
    assert d.max() <= 2 * lr * 4 * 1.01 and d.mean() < 0.01 * lr, (d.max(), d.mean())
