"""GPU parity of the on-policy (A2C / PPO) network kernels
against the oracle restatement of rltoolkit/basic_model.py Actor / Critic
(oracle/onpolicy.py) and the reference fixture tests/golden/onpolicy_hcheetah.npz (Actor.act,
A2C.update_critic, PPO_AcM.update_actor_acm run by the reference itself)."""
import numpy as np
import pytest
import torch

from oracle import onpolicy as oo

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
OB, AOUT = 17, 17


def relerr(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


@pytest.fixture(scope="module")
def nets():
    from spprl.onpolicy import OnPolicyNets
    n = OnPolicyNets(OB, AOUT, ac_lim=1.0, max_batch=5000, device=DEV, entropy_coef=0.01)
    return n


def _setup(nets, seed):
    a = oo.init_flat(oo.actor_layout(OB, AOUT), seed)
    a[:AOUT] += np.random.RandomState(seed).uniform(-0.3, 0.3, AOUT).astype(np.float32)
    c = oo.init_flat(oo.critic_layout(OB), seed + 1)
    nets.load_net(0, a)
    nets.load_net(1, c)
    return a, c


@pytest.mark.parametrize("N", [1, 77, 3000])
def test_value_and_critic_grad(nets, N):
    a, c = _setup(nets, 3)
    rng = np.random.RandomState(N)
    x = (rng.randn(N, OB) * 1.5).astype(np.float32)
    q = rng.randn(N).astype(np.float32)
    v = nets.value(x).cpu().numpy()
    with torch.no_grad():
        want = oo.critic(oo._params(c, oo.critic_layout(OB)), torch.from_numpy(x)).squeeze(-1).numpy()
    np.testing.assert_allclose(v, want, rtol=1e-5, atol=1e-5)
    from spprl import _lib
    xd, qd = torch.from_numpy(x).to(DEV), torch.from_numpy(q).to(DEV)
    loss = torch.zeros(1, device=DEV)
    _lib.call("sppOnpCriticGrads", nets._h, _lib.ptr(xd), _lib.ptr(qd), N, _lib.ptr(loss), _lib.stream_handle())
    torch.cuda.synchronize()
    l_ref, g_ref = oo.critic_step(c, OB, x, q)
    assert loss.item() == pytest.approx(l_ref, rel=1e-5)
    assert relerr(nets.grads[1].cpu().numpy(), g_ref) < 2e-5


def test_critic_full_batch_at_bench_size():
    """The ppo_hcheetah bench's critic full batch (A2C.update_critic on all N = T x E = 16 x 2048 = 32,768
    frames of an iteration, a2c.py:186-225): value and one gradient against the float64 oracle --
    loss rtol 1e-5, gradient relative error < 2e-5 (multi-workgroup partials and the dW reduction at the
    timed shape)."""
    from spprl import _lib
    from spprl.onpolicy import OnPolicyNets

    N = 32768
    n = OnPolicyNets(OB, AOUT, ac_lim=1.0, max_batch=N, device=DEV)
    a, c = _setup(n, 13)
    rng = np.random.RandomState(N)
    x = (rng.randn(N, OB) * 1.5).astype(np.float32)
    q = rng.randn(N).astype(np.float32)
    v = n.value(x).cpu().numpy()
    with torch.no_grad():
        want = oo.critic(oo._params(c, oo.critic_layout(OB), torch.float64),
                         torch.from_numpy(x).double()).squeeze(-1).numpy()
    np.testing.assert_allclose(v, want, rtol=1e-5, atol=1e-5)
    xd, qd = torch.from_numpy(x).to(DEV), torch.from_numpy(q).to(DEV)
    loss = torch.zeros(1, device=DEV)
    _lib.call("sppOnpCriticGrads", n._h, _lib.ptr(xd), _lib.ptr(qd), N, _lib.ptr(loss), _lib.stream_handle())
    torch.cuda.synchronize()
    l_ref, g_ref = oo.critic_step(c, OB, x, q, dtype=torch.float64)
    assert loss.item() == pytest.approx(l_ref, rel=1e-5)
    e = relerr(n.grads[1].cpu().numpy(), g_ref)
    print("N = %d: critic grad rel err %.2e" % (N, e))
    assert e < 2e-5, e


@pytest.mark.parametrize("N", [50, 300, 32768])
def test_critic_steps_kernel_matches_per_step_path_and_oracle(N):
    """sppOnpCriticSteps (A2C.update_critic's full-batch steps for one target in ONE launch: one workgroup at
    N = 50, 5 at N = 300, 256 workgroups x 2 passes of 64 rows at the bench's N = 32,768) against (a) the
    per-step path (sppOnpCriticGrads / Apply, five launches a step) and (b) the oracle's float64 steps with
    the same Adam (oracle.onpolicy.critic_steps): the summed loss rtol 1e-4; parameters within 2 lr per Adam
    step of the oracle (a sign flip of a near-zero gradient coordinate), mean far below that."""
    from spprl import _lib
    from spprl.onpolicy import OnPolicyNets

    K, lr = 10, 3e-4
    c0 = oo.init_flat(oo.critic_layout(OB), 31)
    rng = np.random.RandomState(N + 3)
    x = (rng.randn(N, OB) * 1.3).astype(np.float32)
    q = (rng.randn(N) * 0.7).astype(np.float32)
    xd, qd = torch.from_numpy(x).to(DEV), torch.from_numpy(q).to(DEV)
    res = []
    for one_launch in (True, False):
        n = OnPolicyNets(OB, AOUT, critic_lr=lr, max_batch=max(N, 512), device=DEV)
        n.load_net(1, c0)
        if not one_launch:
            n._critic_max_n = 0
        assert n._critic_kernel_ok(N) == one_launch
        total = torch.zeros(1, device=DEV)
        if one_launch:
            _lib.call("sppOnpCriticSteps", n._h, _lib.ptr(xd), _lib.ptr(qd), N, K, _lib.ptr(total),
                      _lib.stream_handle())
        else:
            for _ in range(K):
                total += n.critic_step(xd, qd)
        torch.cuda.synchronize()
        if one_launch:
            n.check_actor_epochs()  # (the shared timeout flag of the persistent launches)
        res.append((n.params[1].cpu().numpy().copy(), float(total.item())))
    flat, losses = oo.critic_steps(c0, OB, x, q, lr, K, dtype=torch.float64)
    for p, tot in res:
        assert tot == pytest.approx(sum(losses), rel=1e-4)
        d = np.abs(p - flat)
        print("N %d: loss %.6f (ref %.6f) |d|/lr max %.4f mean %.6f" % (N, tot, sum(losses), d.max() / lr,
                                                                       d.mean() / lr))
        assert d.max() <= 2 * lr * K * 1.01 and d.mean() <= 0.01 * lr, (d.max(), d.mean())


@pytest.mark.parametrize("N", [50, 1000, 32768])
def test_critic_step_grads_matches_phase_path_and_oracle(N):
    """sppOnpCriticStepGrads (the data-parallel critic step: the persistent kernel's reduced gradient of ONE step,
    written to the critic's gradient buffer, parameters and Adam state untouched; single workgroup at N = 50,
    multi-workgroup at 1,000 and the bench's 32,768) against sppOnpCriticGrads and the float64 oracle: loss rtol
    1e-5, gradient relative error < 2e-5, parameters bit-unchanged; then sppOnpCriticApply on either gradient gives
    parameters within fp32 rounding of each other."""
    from spprl import _lib
    from spprl.onpolicy import OnPolicyNets

    c0 = oo.init_flat(oo.critic_layout(OB), 41)
    rng = np.random.RandomState(N + 5)
    x = (rng.randn(N, OB) * 1.3).astype(np.float32)
    q = (rng.randn(N) * 0.7).astype(np.float32)
    xd, qd = torch.from_numpy(x).to(DEV), torch.from_numpy(q).to(DEV)
    l_ref, g_ref = oo.critic_step(c0, OB, x, q, dtype=torch.float64)
    out = {}
    for fn in ("sppOnpCriticStepGrads", "sppOnpCriticGrads"):
        n = OnPolicyNets(OB, AOUT, max_batch=max(N, 512), device=DEV)
        n.load_net(1, c0)
        loss = torch.zeros(1, device=DEV)
        if fn == "sppOnpCriticStepGrads":
            _lib.call(fn, n._h, _lib.ptr(xd), _lib.ptr(qd), N, _lib.ptr(loss), 1.0, _lib.stream_handle())
        else:
            _lib.call(fn, n._h, _lib.ptr(xd), _lib.ptr(qd), N, _lib.ptr(loss), _lib.stream_handle())
        torch.cuda.synchronize()
        n.check_actor_epochs()
        g = n.grads[1].cpu().numpy().copy()
        assert loss.item() == pytest.approx(l_ref, rel=1e-5), fn
        assert relerr(g, g_ref) < 2e-5, (fn, relerr(g, g_ref))
        np.testing.assert_array_equal(n.params[1].cpu().numpy(), c0)
        _lib.call("sppOnpCriticApply", n._h, _lib.stream_handle())
        torch.cuda.synchronize()
        out[fn] = (g, n.params[1].cpu().numpy().copy())
    (ga, pa), (gb, pb) = out["sppOnpCriticStepGrads"], out["sppOnpCriticGrads"]
    print("N %d: fused vs phase-path gradient rel err %.2e" % (N, relerr(ga, gb)))
    assert np.abs(pa - pb).max() <= 2 * 3e-4  # one Adam step: a sign flip of a near-zero coordinate costs <= 2 lr


@pytest.mark.parametrize("N", [1, 500, 2048])
def test_actor_grad_clip_entropy(nets, N):
    a, c = _setup(nets, 5)
    rng = np.random.RandomState(N + 1)
    x = (rng.randn(N, OB) * 1.2).astype(np.float32)
    act = rng.uniform(-1.2, 1.2, (N, AOUT)).astype(np.float32)
    lp_old = (rng.randn(N) * 2 - 10).astype(np.float32)
    with torch.no_grad():
        lp_cur = oo.actor_dist(oo._params(a, oo.actor_layout(OB, AOUT)), torch.from_numpy(x),
                               torch.ones(AOUT)).log_prob(torch.from_numpy(act)).numpy()
    lp_old = (lp_cur + rng.randn(N).astype(np.float32) * 0.2).astype(np.float32)  # ratios around 1 (both branches)
    adv = rng.randn(N).astype(np.float32)
    nxt = rng.randn(N, AOUT).astype(np.float32)
    from spprl import _lib
    t = lambda z: torch.from_numpy(np.ascontiguousarray(z)).to(DEV)  # noqa: E731
    xd, ad, ld, vd, nd = t(x), t(act), t(lp_old), t(adv), t(nxt)
    out = torch.zeros(4, device=DEV)
    _lib.call("sppOnpActorGrads", nets._h, _lib.ptr(xd), _lib.ptr(ad), _lib.ptr(ld), _lib.ptr(vd), _lib.ptr(nd), N,
              _lib.ptr(out), _lib.stream_handle())
    torch.cuda.synchronize()
    ref, g_ref = oo.actor_step(a, OB, AOUT, np.ones(AOUT, np.float32), x, act, lp_old, adv, entropy_coef=0.01,
                               next_obs=nxt)
    o = out.cpu().numpy()
    assert o[0] == pytest.approx(ref["actor"], rel=1e-4, abs=1e-6)
    assert o[1] == pytest.approx(ref["kl"], rel=1e-4, abs=1e-5)
    assert o[2] == pytest.approx(ref["dist"], rel=1e-5)
    assert o[3] == pytest.approx(ref["entropy"], rel=1e-5)
    g = nets.grads[0].cpu().numpy()
    assert relerr(g, g_ref) < 2e-4, relerr(g, g_ref)
    np.testing.assert_allclose(g[:AOUT], g_ref[:AOUT], rtol=1e-3, atol=1e-6)  # log_scale


@pytest.mark.parametrize("N", [40, 1000, 8388])
def test_actor_step_grads_matches_oracle_through_a_permutation(N):
    """sppOnpActorStepGrads (the data-parallel clip-loss step: the actor epoch kernel run for ONE minibatch whose
    rows are read through a permutation slice, gradient written to the actor's buffer instead of applied; one
    workgroup at N = 40, 16 at 1,000, 132 at the w8 rehearsal's 8,388-row shard) against the float64 oracle on the
    permuted rows: out4 as test_actor_grad_clip_entropy, gradient relative error < 2e-4, parameters untouched."""
    from spprl import _lib
    from spprl.onpolicy import OnPolicyNets

    n = OnPolicyNets(OB, AOUT, ac_lim=1.0, max_batch=max(2 * N, 512), device=DEV, entropy_coef=0.01)
    a, c = _setup(n, 7)
    M = 2 * N  # the rollout the permutation draws the minibatch from
    rng = np.random.RandomState(N + 9)
    x = (rng.randn(M, OB) * 1.2).astype(np.float32)
    act = rng.uniform(-1.2, 1.2, (M, AOUT)).astype(np.float32)
    with torch.no_grad():
        lp_cur = oo.actor_dist(oo._params(a, oo.actor_layout(OB, AOUT)), torch.from_numpy(x),
                               torch.ones(AOUT)).log_prob(torch.from_numpy(act)).numpy()
    lp_old = (lp_cur + rng.randn(M).astype(np.float32) * 0.2).astype(np.float32)
    adv = rng.randn(M).astype(np.float32)
    nxt = rng.randn(M, AOUT).astype(np.float32)
    idx = rng.permutation(M)[:N].astype(np.int64)
    t = lambda z: torch.from_numpy(np.ascontiguousarray(z)).to(DEV)  # noqa: E731
    dev = [t(z) for z in (x, act, lp_old, adv, nxt, idx)]  # (held: the launch reads them after the call returns)
    out = torch.zeros(4, device=DEV)
    _lib.call("sppOnpActorStepGrads", n._h, *[_lib.ptr(z) for z in dev], N, _lib.ptr(out), 1.0, _lib.stream_handle())
    torch.cuda.synchronize()
    n.check_actor_epochs()
    ref, g_ref = oo.actor_step(a, OB, AOUT, np.ones(AOUT, np.float32), x[idx], act[idx], lp_old[idx], adv[idx],
                               entropy_coef=0.01, next_obs=nxt[idx])
    o = out.cpu().numpy()
    assert o[0] == pytest.approx(ref["actor"], rel=1e-4, abs=1e-6)
    assert o[1] == pytest.approx(ref["kl"], rel=1e-4, abs=1e-5)
    assert o[2] == pytest.approx(ref["dist"], rel=1e-5)
    assert o[3] == pytest.approx(ref["entropy"], rel=1e-5)
    g = n.grads[0].cpu().numpy()
    assert relerr(g, g_ref) < 2e-4, relerr(g, g_ref)
    np.testing.assert_allclose(g[:AOUT], g_ref[:AOUT], rtol=1e-3, atol=1e-6)  # log_scale
    np.testing.assert_array_equal(n.params[0].cpu().numpy(), a)


def test_act_sample_and_deterministic(nets):
    a, c = _setup(nets, 9)
    rng = np.random.RandomState(4)
    x = rng.randn(333, OB).astype(np.float32)
    eps = rng.randn(333, AOUT).astype(np.float32)
    for e in (None, eps):
        act, lp = nets.act(x, e)
        want_a, want_lp = oo.act(a, OB, AOUT, np.ones(AOUT, np.float32), x, e)
        np.testing.assert_allclose(act.cpu().numpy(), want_a, rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(lp.cpu().numpy(), want_lp, rtol=1e-4, atol=1e-4)


def test_update_loops_run_and_improve(nets):
    """update_critic (10x10 full-batch steps) reduces the critic loss; update_actor runs its
    epochs with the KL stop and keeps parameters finite."""
    _setup(nets, 11)
    rng = np.random.RandomState(12)
    N = 2000
    obs = rng.randn(N, OB).astype(np.float32)
    nobs = rng.randn(N, OB).astype(np.float32)
    rew = rng.randn(N).astype(np.float32)
    done = (rng.rand(N) < 0.05).astype(np.float32)
    q0 = rew + 0.99 * (1 - done) * nets.value(nobs).cpu().numpy()
    l0 = 0.5 * np.mean((q0 - nets.value(obs).cpu().numpy()) ** 2)
    adv = nets.update_critic(obs, nobs, rew, done)
    assert nets.loss["critic"] < l0
    act, lp = nets.act(obs, rng.randn(N, AOUT).astype(np.float32))
    nets.max_ppo_epochs = 3
    kl = nets.update_actor(adv, obs, act, lp, generator=torch.Generator().manual_seed(0))
    assert np.isfinite(kl)
    assert all(torch.isfinite(p).all() for p in nets.params)


# ------------------------------------------------------------------ pinned by reference fixtures
# tests/golden/onpolicy_hcheetah.npz (make_golden.py gen_onpolicy): the reference's own Actor.act,
# A2C.update_critic and PPO_AcM.update_actor_acm on fixed inputs.
def _fx():
    from golden_cases import onpolicy_case

    return onpolicy_case()


def test_act_matches_reference_fixture():
    """basic_model.Actor.act (basic_model.py:32-51): sampled action and Independent-Normal log-prob,
    and the deterministic mean; the reference's normal draws are recovered from its sampled actions."""
    from spprl.onpolicy import OnPolicyNets

    fx = _fx()
    ob = fx["act_x"].shape[1]
    n = OnPolicyNets(ob, ob, ac_lim=1.0, max_batch=512, device=DEV)
    n.load_net(0, fx["act_params"])
    sc = np.exp(fx["act_params"][:ob].astype(np.float64))
    eps = ((fx["act_a"] - fx["act_mu"]) / sc).astype(np.float32)
    a, lp = n.act(fx["act_x"], eps)
    np.testing.assert_allclose(a.cpu().numpy(), fx["act_a"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(lp.cpu().numpy(), fx["act_lp"], rtol=1e-5, atol=2e-4)
    a, lp = n.act(fx["act_x"], None)
    np.testing.assert_allclose(a.cpu().numpy(), fx["act_mu"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(lp.cpu().numpy(), fx["act_lp_det"], rtol=1e-5, atol=2e-4)


def test_update_critic_matches_reference_fixture():
    """A2C.update_critic (a2c.py:186-225): 10 targets x 10 full-batch Adam steps on 0.5 * adv^2, then
    calculate_advantage.  100 sequential Adam steps: parameters within 5e-6 + 1e-4 relative."""
    from spprl.onpolicy import OnPolicyNets

    fx = _fx()
    ob = fx["crit_obs"].shape[1]
    n = OnPolicyNets(ob, ob, critic_lr=float(fx["crit_lr"]), gamma=float(fx["crit_gamma"]), max_batch=512, device=DEV)
    n.load_net(1, fx["crit_params0"])
    adv = n.update_critic(fx["crit_obs"], fx["crit_nobs"], fx["crit_rew"], fx["crit_done"])
    torch.cuda.synchronize()
    assert n.loss["critic"] == pytest.approx(float(fx["crit_loss"]), rel=1e-4)
    np.testing.assert_allclose(n.params[1].cpu().numpy(), fx["crit_post"], rtol=1e-4, atol=5e-6)
    np.testing.assert_allclose(adv.cpu().numpy(), fx["crit_adv"], rtol=1e-4, atol=1e-4)


def test_ppo_acm_actor_epoch_matches_reference_fixture():
    """PPO_AcM.update_actor_acm (acm/on_policy.py:164-216) with one epoch of one full-batch
    minibatch: normalised advantages, clip loss - entropy_coef * entropy, Adam step.  First Adam
    step moves each weight by ~lr * sign(g): |d| <= 2 lr, rare beyond 1e-6."""
    from spprl.onpolicy import OnPolicyNets

    fx = _fx()
    obs, nobs = fx["crit_obs"], fx["crit_nobs"]
    N, ob = obs.shape
    n = OnPolicyNets(ob, ob, actor_lr=float(fx["ppo_lr"]), ppo_epsilon=float(fx["ppo_eps"]),
                     entropy_coef=float(fx["ppo_entropy_coef"]), custom_loss=float(fx["ppo_custom_loss"]),
                     max_ppo_epochs=1, ppo_batch_size=N, normalize_adv=True, max_batch=512, device=DEV)
    n.load_net(0, fx["ppo_params0"])
    n.update_actor(fx["ppo_adv"], obs, fx["ppo_acts"], fx["ppo_lp_old"], nobs,
                   generator=torch.Generator().manual_seed(0))
    torch.cuda.synchronize()
    actor, entropy, policy, dist = (float(v) for v in fx["ppo_losses"])
    assert n.loss["actor"] == pytest.approx(actor, rel=1e-4, abs=1e-6)
    assert n.loss["entropy"] == pytest.approx(entropy, rel=1e-5)
    assert n.loss["policy"] == pytest.approx(policy, rel=1e-4, abs=1e-6)
    assert n.loss["dist"] == pytest.approx(dist, rel=1e-5)
    assert n.kl_div_updates_counter == 1
    d = np.abs(n.params[0].cpu().numpy() - fx["ppo_post"])
    lr = float(fx["ppo_lr"])
    assert d.max() <= 2 * lr * 1.01, d.max()
    assert np.mean(d > 1e-6) < 2e-3, np.mean(d > 1e-6)


def test_ppo_acm_actor_epochs_kl_stop_match_reference_fixture():
    """PPO_AcM.update_actor_acm over several epochs with the KL early stop (acm/on_policy.py:164-216,
    tests/golden/ppo_epochs_hcheetah.npz, make_golden.py gen_ppo_epochs): one full-batch minibatch per
    epoch; the reference's KL of each epoch is taken on the last minibatch's pre-step log-probs, the
    threshold sits between the 3rd and 4th epochs' KL, so 4 epochs run, the loop breaks at i = 4 and
    every loss is divided by i + 1 = 5; kl_div_updates_counter += 5.  Four sequential Adam steps at
    lr 3e-3: each weight within 2 lr per step of the reference (a sign flip of a near-zero gradient
    coordinate moves it by 2 lr), most far closer."""
    from golden_cases import load
    from spprl.onpolicy import OnPolicyNets

    fx = load("ppo_epochs_hcheetah")
    obs, nobs = fx["obs"], fx["nobs"]
    N, ob = obs.shape
    lr = float(fx["lr"])
    n = OnPolicyNets(ob, ob, actor_lr=lr, ppo_epsilon=float(fx["eps"]), entropy_coef=float(fx["entropy_coef"]),
                     custom_loss=float(fx["custom_loss"]), max_ppo_epochs=int(fx["max_epochs"]), ppo_batch_size=N,
                     kl_div_threshold=float(fx["threshold"]), normalize_adv=True, max_batch=512, device=DEV)
    n.load_net(0, fx["params0"])
    kl = n.update_actor(fx["adv"], obs, fx["acts"], fx["lp_old"], nobs, generator=torch.Generator().manual_seed(0))
    torch.cuda.synchronize()
    kls = fx["kls"]
    assert n.last_epochs == len(kls) == 4
    assert n.kl_div_updates_counter == int(fx["counter"]) == 5
    assert kl == pytest.approx(float(kls[-1]), rel=1e-4, abs=2e-5)
    actor, entropy, policy, dist = (float(v) for v in fx["losses"])
    assert n.loss["actor"] == pytest.approx(actor, rel=1e-4, abs=2e-6)
    assert n.loss["entropy"] == pytest.approx(entropy, rel=1e-5)
    assert n.loss["policy"] == pytest.approx(policy, rel=1e-4, abs=2e-6)
    assert n.loss["dist"] == pytest.approx(dist, rel=1e-5)
    d = np.abs(n.params[0].cpu().numpy() - fx["post"])
    print("epochs %d counter %d kl %.6f (ref %.6f); |d|/lr max %.4f mean %.5f frac>1e-5 %.4f" % (
        n.last_epochs, n.kl_div_updates_counter, kl, kls[-1], d.max() / lr, d.mean() / lr, np.mean(d > 1e-5)))
    assert d.max() <= 2 * lr * 4 * 1.01, d.max()
    assert d.mean() <= 0.02 * lr, d.mean()


@pytest.mark.parametrize("N,mb", [(2048, 512), (2000, 512), (2050, 512), (300, 64)])
def test_actor_epoch_kernel_matches_per_step_path_and_oracle(N, mb):
    """sppOnpActorEpoch (one launch per PPO epoch: every minibatch step's forward, clip-loss backward, weight
    gradients, fixed-order sum over the ceil(mb / 64) workgroups and Adam inside the kernel) against (a) the
    per-minibatch path (sppOnpActorGrads / Apply, six launches per step) and (b) the oracle's epoch loop
    (oracle.onpolicy.update_actor_epochs, on_policy.py:176-216) on the same permutations: 2 epochs, a ragged
    last minibatch (inside the same launch) for N = 2000 and 2050 (2 rows: 7 of its 8 workgroups hold none).  Losses / KL rtol 1e-4; parameters within 2 lr per Adam step of the oracle
    (a sign flip of a near-zero gradient coordinate), mean far below that."""
    from spprl.onpolicy import OnPolicyNets

    lr, ent, cl = 3e-4, 0.01, 0.1
    rng = np.random.RandomState(N + mb)
    a0 = oo.init_flat(oo.actor_layout(OB, AOUT), 21)
    a0[:AOUT] += rng.uniform(-0.3, 0.3, AOUT).astype(np.float32)
    x = (rng.randn(N, OB) * 1.2).astype(np.float32)
    act = rng.uniform(-1.1, 1.1, (N, AOUT)).astype(np.float32)
    nxt = rng.randn(N, AOUT).astype(np.float32)
    with torch.no_grad():
        lp_cur = oo.actor_dist(oo._params(a0, oo.actor_layout(OB, AOUT)), torch.from_numpy(x),
                               torch.ones(AOUT)).log_prob(torch.from_numpy(act)).numpy()
    lp_old = (lp_cur + 0.2 * rng.randn(N)).astype(np.float32)
    adv = rng.randn(N).astype(np.float32)
    adv = ((adv - adv.mean()) / adv.std()).astype(np.float32)  # already normalised (normalize_adv off)
    res = []
    for one_launch in (True, False):
        n = OnPolicyNets(OB, AOUT, ac_lim=1.0, actor_lr=lr, entropy_coef=ent, custom_loss=cl, max_ppo_epochs=2,
                         ppo_batch_size=mb, kl_div_threshold=1e9, normalize_adv=False, max_batch=max(N, 512),
                         device=DEV)
        n.load_net(0, a0)
        if not one_launch:
            n._epoch_max_bs = 0
        assert n._epoch_kernel_ok(mb) == one_launch
        kl = n.update_actor(adv, x, act, lp_old, nxt, generator=torch.Generator().manual_seed(7))
        torch.cuda.synchronize()
        if one_launch:
            n.check_actor_epochs()
        res.append((n.params[0].cpu().numpy().copy(), dict(n.loss), kl))
    g = torch.Generator().manual_seed(7)
    perms = [torch.randperm(N, generator=g).numpy() for _ in range(2)]
    flat, losses, kls, cnt = oo.update_actor_epochs(a0, OB, AOUT, np.ones(AOUT, np.float32), x, act, lp_old, adv, nxt,
                                                    lr, 2, 1e9, mb, entropy_coef=ent, custom_loss=cl, perms=perms)
    nsteps = 2 * -(-N // mb)
    for p, loss, kl in res:
        for k in ("actor", "entropy", "policy", "dist"):
            assert loss[k] == pytest.approx(losses[k], rel=1e-4, abs=1e-6), (k, loss[k], losses[k])
        assert kl == pytest.approx(kls[-1], rel=1e-3, abs=2e-6)
        d = np.abs(p - flat)
        print("N %d mb %d: |d|/lr max %.4f mean %.6f" % (N, mb, d.max() / lr, d.mean() / lr))
        assert d.max() <= 2 * lr * nsteps * 1.01 and d.mean() <= 0.01 * lr, (d.max(), d.mean())


def test_persistent_launch_timeouts_raise_in_the_product_path():
    """A multi-workgroup persistent launch whose arrival wait times out leaves invalid parameters: the product
    path (OnPolicyNets.update_critic / update_actor as PPO_AcM.update runs them, and the AcM epochs of
    update_acm) must raise SppError, not continue.  The timeout is forced with the spin-limit test hook
    (sppSetSgdSpinLimit(-1): every arrival wait gives up at once, as a co-residency miss would; a small positive
    limit is timing-dependent: the workgroups of a short epoch can all arrive before anyone's first poll)."""
    import spprl
    from spprl import _lib
    from spprl.onpolicy import OnPolicyNets

    N = 4096
    rng = np.random.RandomState(7)
    obs = torch.from_numpy((rng.randn(N, OB)).astype(np.float32)).to(DEV)
    nobs = torch.from_numpy((rng.randn(N, OB)).astype(np.float32)).to(DEV)
    rew = torch.from_numpy(rng.randn(N).astype(np.float32)).to(DEV)
    done = torch.zeros(N, device=DEV)
    act = torch.from_numpy(rng.uniform(-1, 1, (N, AOUT)).astype(np.float32)).to(DEV)
    lp = torch.from_numpy(rng.randn(N).astype(np.float32)).to(DEV)
    adv = torch.from_numpy(rng.randn(N).astype(np.float32)).to(DEV)
    # healthy: the same calls raise nothing
    n0 = OnPolicyNets(OB, AOUT, max_batch=N, ppo_batch_size=512, max_ppo_epochs=2, critic_num_target_updates=1,
                      num_critic_updates_per_target=3, device=DEV, seed=1)
    assert n0._critic_kernel_ok(N) and n0._epoch_kernel_ok(512)
    n0.update_critic(obs, nobs, rew, done)
    n0.update_actor(adv, obs, act, lp, nobs)
    try:
        _lib.call("sppSetSgdSpinLimit", -1)
        n1 = OnPolicyNets(OB, AOUT, max_batch=N, critic_num_target_updates=1, num_critic_updates_per_target=3,
                          device=DEV, seed=1)
        with pytest.raises(_lib.SppError, match="timed out"):
            n1.update_critic(obs, nobs, rew, done)
        n2 = OnPolicyNets(OB, AOUT, max_batch=N, ppo_batch_size=512, max_ppo_epochs=2, device=DEV, seed=1)
        with pytest.raises(_lib.SppError, match="timed out"):
            n2.update_actor(adv, obs, act, lp, nobs)
        # the AcM epochs (multi-workgroup sppAcmSgdEpoch, acm_batch_size > 64): raised at the next update_acm
        ag = spprl.SAC_AcM(env_name="HalfCheetah-v2", buffer_size=5000, max_batch=1024, acm_batch_size=1024,
                           device=DEV, seed=0)
        rb = ag.replay_buffer
        slots = rb.add_obs_batch(torch.randn(3001, 17, device=DEV))
        z = torch.zeros(3000, dtype=torch.uint8, device=DEV)
        rb.add_timestep_batch(slots[:-1], slots[1:], torch.randn(3000, 17, device=DEV), torch.randn(3000, device=DEV),
                              z, z, torch.rand(3000, 6, device=DEV))
        assert ag._acm_sgd_ok(1024)
        ag.update_acm(1)
        with pytest.raises(_lib.SppError, match="timed out"):
            ag.check_acm_sgd()
    finally:
        _lib.call("sppSetSgdSpinLimit", 0)
    torch.cuda.synchronize()
