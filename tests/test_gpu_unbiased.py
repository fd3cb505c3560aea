"""unbiased_update of DDPG_AcM / SAC_AcM (rltoolkit/acm/off_policy/ddpg_acm.py:59-79: make_update samples
grad_steps batches and updates with action = next_obs) on the GPU path:
  * the reference cadence (E = 1, make_update over the MT19937 sample stream) against the reference's own
    make_update on the same ring and seeds (tests/golden/ddpg_unbiased_hcheetah.npz, obs_norm=True z-score,
    acm_critic=False, custom_loss with norm_closs): losses and post-step parameters;
  * the fused (staged) schedule: sppAgentStageFromReplay + sppAgentStagePost (obs normalised in place,
    action := next obs) leaves the same parameters, bit for bit, as the caller-batch update on the explicitly
    gathered, normalised tuples with action = next_obs (DDPG_AcM and SAC_AcM, whose eps draws are read back
    through sppAgentReadEps);
  * SAC_AcM's inherited make_update (sac_acm.py:12) against the reference's own SAC_AcM.make_update
    (tests/golden/sac_unbiased_hcheetah.npz: the same ring, seeds and injected rsample draws)."""
import numpy as np
import pytest
import torch

import spprl
from spprl import _lib
from golden_cases import ddpg_unbiased_case

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
NAMES = {"actor": _lib.SPP_NET_ACTOR, "critic": _lib.SPP_NET_CRITIC1, "actor_targ": _lib.SPP_NET_ACTOR_TARG,
         "critic_targ": _lib.SPP_NET_CRITIC1_TARG}


def build_ddpg(fx, params, norm, **kw):
    ob, aout, ac, B, gsteps, ufreq, size = (int(v) for v in fx["dims"])
    ag = spprl.DDPG_AcM(env_name="custom", env_spec=(ob, ac, 1.0, 1000), gamma=float(fx["gamma"]), actor_lr=5e-4,
                        critic_lr=5e-4, tau=float(fx["tau"]), acm_critic=False, custom_loss=0.3, norm_closs=True,
                        min_max_denormalize=False, denormalize_actor_out=True, obs_norm=True, unbiased_update=True,
                        update_batch_size=B, grad_steps=gsteps, update_freq=ufreq, buffer_size=size,
                        max_batch=kw.pop("max_batch", B), device=DEV, use_gpu=True, acm_val_buffer_size=None, **kw)
    for k, net in NAMES.items():
        ag.load_net(net, params[k])
    rb = ag.replay_buffer
    rb.obs_mean.copy_(norm.mean)
    rb.obs_std.copy_(norm.std)
    return ag


def fill(ag, replay):
    rb = ag.replay_buffer
    replay(rb.add_obs, rb.add_acm_action, rb.add_timestep)


def test_ddpg_unbiased_make_update_matches_reference_fixture():
    fx, params, _, norm, replay = ddpg_unbiased_case()
    ob, aout, ac, B, gsteps, ufreq, size = (int(v) for v in fx["dims"])
    ag = build_ddpg(fx, params, norm)
    assert ag.schedule == "reference" and ag.unbiased_update
    fill(ag, replay)
    ag.iteration = 0
    for c, s in enumerate(fx["np_seeds"]):
        ag.stats_logger.frames = ufreq * (c + 1)
        np.random.seed(int(s))
        ag.make_update()
        got = ag.loss
        for j, k in enumerate(("critic", "actor", "ddpg", "dist")):
            assert got[k] == pytest.approx(float(fx["losses"][c][j]), rel=1e-4, abs=1e-6), (c, k)
    torch.cuda.synchronize()
    lr, n = 5e-4, len(fx["np_seeds"]) * gsteps
    for k in ("actor", "critic", "actor_targ", "critic_targ"):
        got = ag.params[NAMES[k]].cpu().numpy()
        d = np.abs(got - fx["post_" + k])
        scale = 1.0 if k in ("actor", "critic") else float(fx["tau"])
        # Adam's first steps move a parameter by ~lr whatever the gradient's size: a gradient element within
        # rounding of zero may take the other sign (bounded by 2 lr per step), the rest agree to fp32 rounding
        assert d.max() <= 2 * n * lr * scale * 1.01 + 1e-6, (k, d.max())
        assert np.mean(d > 1e-5 * max(scale, 0.05)) < 2e-3, (k, np.mean(d > 1e-5))


@pytest.mark.parametrize("algo", ["ddpg", "sac"])
def test_unbiased_staged_update_equals_caller_batch(algo):
    fx, params, _, norm, replay = ddpg_unbiased_case()
    ob, aout, ac, B, gsteps, ufreq, size = (int(v) for v in fx["dims"])
    Bs = 300
    if algo == "ddpg":
        mk = lambda: build_ddpg(fx, params, norm, max_batch=Bs)  # noqa: E731
    else:
        def mk():
            ag = spprl.SAC_AcM(env_name="custom", env_spec=(ob, ac, 1.0, 1000), acm_critic=False, custom_loss=0.3,
                               norm_closs=True, min_max_denormalize=False, denormalize_actor_out=True, obs_norm=True,
                               unbiased_update=True, buffer_size=size, max_batch=Bs, device=DEV, seed=5)
            rb = ag.replay_buffer
            rb.obs_mean.copy_(norm.mean)
            rb.obs_std.copy_(norm.std)
            return ag
    a1, a2 = mk(), mk()
    for net in a1.params:
        a2.params[net].copy_(a1.params[net])
    fill(a1, replay)
    fill(a2, replay)
    idx = torch.from_numpy(np.random.RandomState(3).randint(0, len(a1.replay_buffer), Bs)).to(DEV)
    batch = a2.replay_buffer.gather(idx)  # normalised obs / next obs (obs_norm)
    batch[2] = batch[1]  # action = next_obs (ddpg_acm.py:67-73)
    if algo == "ddpg":
        a1.update_from_replay_dp(idx)
        a2.update(*batch)
    else:
        st = _lib.stream_handle()
        a1.update_from_replay_dp(idx, 77, 5)
        eps = [torch.empty(Bs, aout, device=DEV) for _ in range(2)]
        for w in range(2):
            _lib.call("sppAgentReadEps", a1._h, w, _lib.ptr(eps[w]), st)
        a2.update(*batch, eps_next=eps[0], eps_cur=eps[1])
    torch.cuda.synchronize()
    for net in a1.params:
        np.testing.assert_array_equal(a1.params[net].cpu().numpy(), a2.params[net].cpu().numpy(), err_msg=str(net))
    assert a1.loss == a2.loss
    # and the branch matters: the same staged step with unbiased_update off (action = the stored actor output)
    a3 = mk()
    a3.unbiased_update = False  # (mk() is deterministic: a3 starts from a1's initial parameters)
    fill(a3, replay)
    if algo == "ddpg":
        a3.update_from_replay_dp(idx)
    else:
        a3.update_from_replay_dp(idx, 77, 5)
    torch.cuda.synchronize()
    assert not torch.equal(a1.params[_lib.SPP_NET_CRITIC1], a3.params[_lib.SPP_NET_CRITIC1])


SAC_NAMES = {"actor": _lib.SPP_NET_ACTOR, "critic_1": _lib.SPP_NET_CRITIC1, "critic_2": _lib.SPP_NET_CRITIC2,
             "critic_1_targ": _lib.SPP_NET_CRITIC1_TARG, "critic_2_targ": _lib.SPP_NET_CRITIC2_TARG}


def test_sac_unbiased_make_update_matches_reference_fixture():
    """The reference cadence of SAC_AcM(unbiased_update=True): make_update's MT19937 index draws, the obs_norm
    gather and action = next obs, two SAC_AcM updates per cadence, with the reference's rsample draws injected
    into each update in call order.  Losses rtol 1e-4; parameters within the Adam first-step allowance."""
    fx, params, _, norm, replay = ddpg_unbiased_case("sac_unbiased_hcheetah")
    ob, aout, ac, B, gsteps, ufreq, size = (int(v) for v in fx["dims"])
    ag = spprl.SAC_AcM(env_name="custom", env_spec=(ob, ac, 1.0, 1000), gamma=float(fx["gamma"]), actor_lr=1e-3,
                       critic_lr=1e-3, alpha_lr=1e-3, alpha=float(fx["alpha0"]), acm_critic=False, custom_loss=0.3,
                       norm_closs=True, min_max_denormalize=False, denormalize_actor_out=True, obs_norm=True,
                       unbiased_update=True, update_batch_size=B, grad_steps=gsteps, update_freq=ufreq,
                       buffer_size=size, max_batch=B, device=DEV, seed=0)
    assert ag.schedule == "reference" and ag.unbiased_update
    for k, net in SAC_NAMES.items():
        ag.load_net(net, params[k])
    rb = ag.replay_buffer
    rb.obs_mean.copy_(norm.mean)
    rb.obs_std.copy_(norm.std)
    replay(rb.add_obs, rb.add_acm_action, rb.add_timestep)
    ag.iteration = 0
    queue = []
    orig = ag.update

    def update(*batch, **kw):  # the reference's rsample draws, two per update (eps_next, eps_cur)
        e1, e2 = queue.pop(0), queue.pop(0)
        return orig(*batch, eps_next=torch.from_numpy(e1).to(DEV), eps_cur=torch.from_numpy(e2).to(DEV), **kw)

    ag.update = update
    for c, s in enumerate(fx["np_seeds"]):
        ag.stats_logger.frames = ufreq * (c + 1)
        queue[:] = list(fx["eps"][c])
        np.random.seed(int(s))
        ag.make_update()
        assert not queue
        for j, k in enumerate(("critic_1", "critic_2", "actor", "sac", "dist")):
            assert ag.loss[k] == pytest.approx(float(fx["losses"][c][j]), rel=1e-4, abs=1e-6), (c, k)
    torch.cuda.synchronize()
    lr, n = 1e-3, len(fx["np_seeds"]) * gsteps
    for k, net in SAC_NAMES.items():
        got = ag.params[net].cpu().numpy()
        d = np.abs(got - fx["post_" + k])
        scale = 1.0 if not k.endswith("targ") else float(fx["tau"])
        assert d.max() <= 2 * n * lr * scale * 1.01 + 1e-6, (k, d.max())
        assert np.mean(d > 1e-5 * max(scale, 0.05)) < 2e-3, (k, np.mean(d > 1e-5))
    assert ag.current_alpha() == pytest.approx(float(fx["alpha"]), rel=1e-5)
