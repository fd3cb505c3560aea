"""GPU parity of the DDPG_AcM device update with the
BasicAcM of the SPP-DDPG scripts, against the reference-generated fixture
tests/golden/ddpg_hcheetah_paper.npz (HalfCheetah dims, 2 update steps) and the
oracle (oracle/ddpg_acm.py)."""
import numpy as np
import pytest
import torch

import spprl
from spprl import _lib
from golden_cases import ddpg_case
from oracle import nets as onets
from oracle.ddpg_acm import OracleDdpgAcm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
NAMES = {"actor": _lib.SPP_NET_ACTOR, "critic": _lib.SPP_NET_CRITIC1, "actor_targ": _lib.SPP_NET_ACTOR_TARG,
         "critic_targ": _lib.SPP_NET_CRITIC1_TARG, "acm": _lib.SPP_NET_ACM}


def relerr(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def build(fx, params, norm, B):
    ob, aout, ac = (int(v) for v in fx["dims"][:3])
    ag = spprl.DDPG_AcM(env_name="custom", env_spec=(ob, ac, 1.0, 1000), gamma=float(fx["gamma"]), actor_lr=5e-4,
                        critic_lr=5e-4, tau=float(fx["tau"]), acm_critic=True, custom_loss=1.0, norm_closs=False,
                        min_max_denormalize=True, denormalize_actor_out=True, max_batch=B, buffer_size=64, device=DEV)
    for k, net in NAMES.items():
        ag.load_net(net, params[k])
    rb = ag.replay_buffer
    rb.min_obs.copy_(norm.lo)
    rb.max_obs.copy_(norm.hi)
    rb._have_minmax = True
    return ag


def test_ddpg_acm_update_matches_oracle_and_reference():
    fx, params, layouts, norm, batches = ddpg_case()
    ob, aout, ac, B = (int(v) for v in fx["dims"])
    ag = build(fx, params, norm, B)
    o = OracleDdpgAcm(ob, aout, ac, norm=norm, actor_lim=fx["actor_ac_lim"], gamma=float(fx["gamma"]),
                      tau=float(fx["tau"]), params=params)
    for i, batch in enumerate(batches):
        ag.update(*batch)
        ol = o.update(*batch)
        torch.cuda.synchronize()
        for k, net in (("critic", _lib.SPP_NET_CRITIC1), ("actor", _lib.SPP_NET_ACTOR)):
            g = ag.grads[net].cpu().numpy()
            assert relerr(g, o.last["grads"][k]) < 2e-4, (k, relerr(g, o.last["grads"][k]))
        gl = ag.loss
        for j, k in enumerate(("critic", "actor", "ddpg", "dist")):
            assert gl[k] == pytest.approx(ol[k], rel=1e-4, abs=1e-6), k
            assert gl[k] == pytest.approx(float(fx["losses"][i][j]), rel=1e-4, abs=1e-6), k
    lr = 5e-4
    for k in ("actor", "critic", "actor_targ", "critic_targ"):
        got = ag.params[NAMES[k]].cpu().numpy()
        want = fx["post_" + k]
        d = np.abs(got - want)
        scale = 1.0 if k in ("actor", "critic") else float(fx["tau"])
        assert d.max() <= 2 * len(batches) * lr * scale * 1.01 + 1e-6, (k, d.max())
        assert np.mean(d > 1e-5 * max(scale, 0.05)) < 2e-3, (k, np.mean(d > 1e-5))


def test_ddpg_policy_act_matches_oracle():
    fx, params, layouts, norm, batches = ddpg_case()
    ob, aout, ac, B = (int(v) for v in fx["dims"])
    ag = build(fx, params, norm, B)
    rng = np.random.RandomState(5)
    E = 200
    obs = (rng.randn(E, ob) * 1.3).astype(np.float32)
    noise = rng.randn(E, aout).astype(np.float32)
    tgt, env = ag.act(torch.from_numpy(obs), noise=torch.from_numpy(noise).to(DEV), mode=1, act_noise=0.1)
    torch.cuda.synchronize()
    P = {k: {n: torch.from_numpy(v) for n, v in params[k].items()} for k in params}
    lim = torch.as_tensor(fx["actor_ac_lim"])
    with torch.no_grad():
        a = onets.ddpg_actor(P["actor"], torch.from_numpy(obs), lim)
        a = torch.clamp(a + 0.1 * lim * torch.from_numpy(noise), -1.1 * lim, 1.1 * lim)  # ddpg_acm.py:40-50
        ad = norm.denormalize(a)
        c = onets.basic_acm(P["acm"], torch.cat([torch.from_numpy(obs), ad], 1))
    np.testing.assert_allclose(tgt.cpu().numpy(), ad.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(env.cpu().numpy(), c.numpy(), rtol=1e-4, atol=1e-5)


def test_basic_acm_regression_matches_torch():
    """AcMTrainer.batch_update (acm.py:246-258) on the BasicAcM: loss and every gradient
    (including the t / t1 output scales) against torch autograd of the oracle net."""
    fx, params, layouts, norm, batches = ddpg_case()
    ob, aout, ac, B = (int(v) for v in fx["dims"])
    ag = build(fx, params, norm, 300)
    rng = np.random.RandomState(8)
    x = (rng.randn(300, 2 * ob) * 1.2).astype(np.float32)
    y = rng.uniform(-1, 1, (300, ac)).astype(np.float32)
    # gradients only (no Adam step) through the split entry point
    xd, yd = torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV)
    loss = torch.zeros(1, device=DEV)
    _lib.call("sppAcmRegressGrads", ag._h, _lib.ptr(xd), _lib.ptr(yd), 300, _lib.ptr(loss), _lib.stream_handle())
    torch.cuda.synchronize()
    P = {n: torch.from_numpy(v).clone().requires_grad_(True) for n, v in params["acm"].items()}
    ref = torch.nn.functional.mse_loss(onets.basic_acm(P, torch.from_numpy(x)), torch.from_numpy(y))
    g = torch.autograd.grad(ref, list(P.values()))
    gflat = torch.cat([t.reshape(-1) for t in g]).numpy()
    assert loss.item() == pytest.approx(ref.item(), rel=1e-5)
    got = ag.grads[_lib.SPP_NET_ACM].cpu().numpy()
    assert relerr(got, gflat) < 2e-4, relerr(got, gflat)
    np.testing.assert_allclose(got[:1 + ac], gflat[:1 + ac], rtol=1e-3, atol=1e-6)  # t, t1


@pytest.mark.parametrize("B", [96, 4000])
def test_ddpg_acm_ant_dims_match_oracle(B):
    """SPP-DDPG Ant (train/spp_ddpg_ant.py: ob 111, ac 8, BasicAcM(222, 8)) kernel set: two updates
    and the policy act against the oracle from the agent's own initial parameters (no reference fixture
    exists at these dims: parity pinned through the oracle, which the HalfCheetah fixture pins)."""
    ob, ac = 111, 8
    ag = spprl.DDPG_AcM(env_name="Ant-v2", gamma=0.99, actor_lr=5e-4, critic_lr=5e-4, acm_critic=True,
                        custom_loss=1.0, norm_closs=False, min_max_denormalize=True, denormalize_actor_out=True,
                        max_batch=B, buffer_size=64, device=DEV, seed=11)
    params = {k: {n: v.numpy() for n, v in ag.net_state(net).items()} for k, net in NAMES.items()}
    rng = np.random.RandomState(B)
    lo = -rng.uniform(0.5, 2, ob).astype(np.float32)
    hi = rng.uniform(0.5, 2, ob).astype(np.float32)
    rb = ag.replay_buffer
    rb.min_obs.copy_(torch.from_numpy(lo))
    rb.max_obs.copy_(torch.from_numpy(hi))
    rb._have_minmax = True
    norm = onets.Norm(True, torch.from_numpy(lo), torch.from_numpy(hi))
    o = OracleDdpgAcm(ob, ob, ac, norm=norm, actor_lim=np.ones(ob, np.float32), gamma=0.99, tau=0.005,
                      params=params, dtype=torch.float64)  # float64: the oracle's own summation error negligible
    for _ in range(2):
        batch = (rng.randn(B, ob).astype(np.float32), rng.randn(B, ob).astype(np.float32),
                 rng.uniform(-1, 1, (B, ob)).astype(np.float32), rng.randn(B).astype(np.float32),
                 (rng.rand(B) < 0.1).astype(np.int8), rng.uniform(-1, 1, (B, ac)).astype(np.float32))
        ag.update(*batch)
        ol = o.update(*batch)
        torch.cuda.synchronize()
        for k, net in (("critic", _lib.SPP_NET_CRITIC1), ("actor", _lib.SPP_NET_ACTOR)):
            e = relerr(ag.grads[net].cpu().numpy(), o.last["grads"][k])
            assert e < 2e-4, (k, e)
        gl = ag.loss
        for k in ("critic", "actor", "ddpg", "dist"):
            assert gl[k] == pytest.approx(ol[k], rel=1e-4, abs=1e-6), k
