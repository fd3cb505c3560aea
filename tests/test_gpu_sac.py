"""GPU parity of vanilla SAC (BASELINE.json configs[0], rltoolkit/algorithms/sac/sac.py) against the
reference-generated fixture tests/golden/sac_vanilla_hcheetah.npz (HalfCheetah dims, 2 updates of
B = 100) and the oracle (oracle/sac.py).  Tolerances as tests/test_gpu_parity.py: losses rtol 1e-4,
gradients relative error < 2e-4, post-Adam parameters within the first-step sign-flip allowance;
at B = 65,536 against the float64 oracle."""
import numpy as np
import pytest
import torch

import spprl
from spprl import _lib
from golden_cases import sac_vanilla_case
from oracle.sac import OracleSac, policy_act

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
NAMES = {"actor": _lib.SPP_NET_ACTOR, "critic_1": _lib.SPP_NET_CRITIC1, "critic_2": _lib.SPP_NET_CRITIC2,
         "critic_1_targ": _lib.SPP_NET_CRITIC1_TARG, "critic_2_targ": _lib.SPP_NET_CRITIC2_TARG}


def relerr(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def build(params, B, **kw):
    ag = spprl.SAC(env_name="HalfCheetah-v2", gamma=0.99, actor_lr=1e-3, critic_lr=1e-3, alpha_lr=1e-3, alpha=0.2,
                   max_batch=B, buffer_size=kw.pop("buffer_size", 64), device=DEV, **kw)
    for k, net in NAMES.items():
        if params is not None:
            ag.load_net(net, params[k])
    return ag


def test_vanilla_sac_update_matches_oracle_and_reference():
    fx, params, steps = sac_vanilla_case()
    ob, ac, B = (int(v) for v in fx["dims"])
    ag = build(params, B)
    assert ag.tau == 0.005 and ag.act_noise == 0.1 and ag.max_ep_len == 1000  # Q1, Q3
    assert ag.target_entropy == -6.0
    o = OracleSac(ob, ac, ac_lim=fx["ac_lim"], gamma=0.99, params=params)
    for i, (batch, e1, e2) in enumerate(steps):
        ag.update(*batch, eps_next=e1, eps_cur=e2)
        ol = o.update(*batch, e1, e2)
        torch.cuda.synchronize()
        for k in ("critic_1", "critic_2", "actor"):
            e = relerr(ag.grads[NAMES[k]].cpu().numpy(), o.last["grads"][k])
            assert e < 2e-4, (k, e)
        gl = ag.loss
        assert set(gl) == {"actor", "critic_1", "critic_2"}
        for j, k in enumerate(("critic_1", "critic_2", "actor")):
            assert gl[k] == pytest.approx(ol[k], rel=1e-4, abs=1e-6), k
            assert gl[k] == pytest.approx(float(fx["losses"][i][j]), rel=1e-4, abs=1e-6), k
    assert ag.current_alpha() == pytest.approx(float(fx["alpha"]), rel=1e-5)
    for k in NAMES:
        d = np.abs(ag.params[NAMES[k]].cpu().numpy() - fx["post_" + k])
        assert d.max() <= 2 * len(steps) * 1e-3 * 1.01, (k, d.max())
        assert np.mean(d > 1e-5) < 2e-3, (k, np.mean(d > 1e-5))


def test_vanilla_sac_large_batch_matches_float64_oracle():
    B, ob, ac = 65536, 17, 6
    ag = build(None, B, seed=7)
    params = {k: {n: v.numpy().copy() for n, v in ag.net_state(net).items()} for k, net in NAMES.items()}
    rng = np.random.RandomState(3)
    batch = (rng.randn(B, ob).astype(np.float32), rng.randn(B, ob).astype(np.float32),
             rng.uniform(-1, 1, (B, ac)).astype(np.float32), rng.randn(B).astype(np.float32),
             (rng.rand(B) < 0.05).astype(np.int8))
    e1, e2 = rng.randn(B, ac).astype(np.float32), rng.randn(B, ac).astype(np.float32)
    ag.update(*batch, eps_next=e1, eps_cur=e2)
    torch.cuda.synchronize()
    o = OracleSac(ob, ac, params=params, dtype=torch.float64)
    ol = o.update(*batch, e1, e2)
    for k in ("critic_1", "critic_2", "actor"):
        e = relerr(ag.grads[NAMES[k]].cpu().numpy(), o.last["grads"][k])
        assert e < 2e-4, (k, e)
        assert ag.loss[k] == pytest.approx(ol[k], rel=1e-4, abs=1e-6)


def test_vanilla_policy_act_matches_oracle():
    fx, params, steps = sac_vanilla_case()
    ag = build(params, 100)
    rng = np.random.RandomState(2)
    E, ob, ac = 300, 17, 6
    obs = (rng.randn(E, ob) * 1.3).astype(np.float32)
    eps = rng.randn(E, ac).astype(np.float32)
    noise = rng.randn(E, ac).astype(np.float32)
    P = {n: torch.from_numpy(v) for n, v in params["actor"].items()}
    t = lambda z: torch.from_numpy(z).to(DEV)  # noqa: E731
    tgt, env = ag.act(t(obs), eps=t(eps), noise=t(noise), mode=1)  # noise_action with act_noise 0.1 (Q1)
    torch.cuda.synchronize()
    want = policy_act(P, obs, 1.0, eps, noise, 0.1)
    np.testing.assert_allclose(env.cpu().numpy(), want, rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(tgt.cpu().numpy(), env.cpu().numpy())  # process_action is the identity
    assert np.abs(env.cpu().numpy()).max() <= 1.0
    _, env = ag.act(t(obs), mode=2, act_noise=0.0)  # test(): deterministic, no noise
    torch.cuda.synchronize()
    np.testing.assert_allclose(env.cpu().numpy(), policy_act(P, obs, 1.0, None, np.zeros_like(noise), 0.0),
                               rtol=1e-5, atol=1e-5)
    u = rng.uniform(-1, 1, (E, ac)).astype(np.float32)
    _, env = ag.act(t(obs), eps=t(u), mode=0)  # initial_act: the env's own sample, unchanged
    torch.cuda.synchronize()
    np.testing.assert_array_equal(env.cpu().numpy(), u)


def test_vanilla_sac_reference_schedule_loop():
    """configs[0] loop: 1 env, random frames, B=100 grad steps every 50 frames, time-limit ends
    stored as end but not done (Q3), obs stats per iteration."""
    ag = build(None, 100, seed=1, n_envs=1, batch_size=250, iterations=2, random_frames=100, update_freq=50,
               grad_steps=5, buffer_size=10_000, env_spec=(17, 6, 1.0, 120))
    ag.train()
    torch.cuda.synchronize()
    rb = ag.replay_buffer
    assert ag.stats_logger.frames == 2 * 360 and len(rb) == 720  # whole episodes of 120 frames
    obs, nobs, act, rew, done = rb.gather(torch.arange(len(rb)))
    assert int(done.sum()) == 0  # 6 episodes ended at the time limit: none of them is done
    for k, val in ag.loss.items():
        assert np.isfinite(val), k
    assert np.abs(act.cpu().numpy()).max() <= 1.0


def test_vanilla_sac_fused_loop_runs():
    E = 256
    ag = build(None, 100 * E, seed=2, n_envs=E, batch_size=2 * E, iterations=2, random_frames=E,
               buffer_size=100_000)
    ag.train()
    torch.cuda.synchronize()
    assert ag.stats_logger.frames == 4 * E
    for k, v in ag.loss.items():
        assert np.isfinite(v), k


@pytest.mark.parametrize("B", [1, 33, 100, 1000, 8192])
def test_vanilla_sac_team_kernels_match_float64_oracle(B, monkeypatch):
    """Small batches (at most one 32-sample tile per CU) run the team forms of the phase kernels
    (csrc/sac_team.h: one 4-wave workgroup per tile, layers split by output blocks); SPP_SAC_TEAM=0 forces the
    one-wave kernels.  Both against the float64 oracle at the same tolerance, and not bit-identical to each other
    (a different q / fc3 summation order: evidence the team kernels ran)."""
    ob, ac = 17, 6
    rng = np.random.RandomState(B)
    batch = (rng.randn(B, ob).astype(np.float32), rng.randn(B, ob).astype(np.float32),
             rng.uniform(-1, 1, (B, ac)).astype(np.float32), rng.randn(B).astype(np.float32),
             (rng.rand(B) < 0.1).astype(np.int8))
    e1, e2 = rng.randn(B, ac).astype(np.float32), rng.randn(B, ac).astype(np.float32)
    grads = {}
    for team in ("1", "0"):
        monkeypatch.setenv("SPP_SAC_TEAM", team)
        ag = build(None, B, seed=5)
        params = {k: {n: v.numpy().copy() for n, v in ag.net_state(net).items()} for k, net in NAMES.items()}
        ag.update(*batch, eps_next=e1, eps_cur=e2)
        torch.cuda.synchronize()
        o = OracleSac(ob, ac, params=params, dtype=torch.float64)
        ol = o.update(*batch, e1, e2)
        for k in ("critic_1", "critic_2", "actor"):
            g = ag.grads[NAMES[k]].cpu().numpy()
            e = relerr(g, o.last["grads"][k])
            assert e < 2e-4, (team, k, e)
            assert ag.loss[k] == pytest.approx(ol[k], rel=1e-4, abs=1e-6), (team, k)
            grads[team, k] = g
    assert any(not np.array_equal(grads["1", k], grads["0", k]) for k in ("critic_1", "critic_2", "actor"))
