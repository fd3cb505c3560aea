"""Reference options of the off- and on-policy agents that round 6 brought onto the device path:

  * vanilla SAC with obs_norm=True (DDPG.__init__ ddpg.py:101-115 hands obs_norm to the plain ReplayBuffer, which
    z-scores every sampled obs / next obs, replay_buffer.py:246-249, with statistics that start as zeros / ones,
    :113-115): the reference's own make_update over two cadences (tests/golden/sac_vanilla_obsnorm_hcheetah.npz:
    initial statistics -- only the +-10 clip --, then after update_obs_mean_std), and the staged batch
    (sppAgentStagePost mode 2, z-score whatever the agent's min-max flag) equal to the caller batch bit for bit;
  * AcMTrainer's acm_ob_idx (acm/acm.py:94-99, 260-264): the ACM gather takes the listed ob columns of obs and
    next obs (sppReplaySetAcmColumns), bit-exact against the ring rows permuted on the host, for SAC_AcM and
    DDPG_AcM, and an ACM regression step on it equals one on the permuted batch;
  * PPO_AcM(obs_norm=True) is accepted and changes nothing computed (the ring's normalize is never called on
    the on-policy path).
"""
import numpy as np
import pytest
import torch

import spprl
from spprl import _lib
from golden_cases import load
from weights import fill_params
from oracle import nets

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
NAMES = {"actor": _lib.SPP_NET_ACTOR, "critic_1": _lib.SPP_NET_CRITIC1, "critic_2": _lib.SPP_NET_CRITIC2,
         "critic_1_targ": _lib.SPP_NET_CRITIC1_TARG, "critic_2_targ": _lib.SPP_NET_CRITIC2_TARG}


def _vanilla_case():
    fx = load("sac_vanilla_obsnorm_hcheetah")
    ob, ac = int(fx["dims"][0]), int(fx["dims"][1])
    seed = int(fx["seed"])
    layouts = {"actor": nets.sac_actor_layout(ob, ac), "critic_1": nets.critic_layout(ob + ac),
               "critic_2": nets.critic_layout(ob + ac), "critic_1_targ": nets.critic_layout(ob + ac),
               "critic_2_targ": nets.critic_layout(ob + ac)}
    params = {k: fill_params(lay, seed * 100 + i) for i, (k, lay) in enumerate(layouts.items())}
    return fx, params


def _vanilla_agent(fx, params, max_batch=None):
    ob, ac, B, gsteps, ufreq, size = (int(v) for v in fx["dims"])
    ag = spprl.SAC(env_name="HalfCheetah-v2", gamma=float(fx["gamma"]), actor_lr=1e-3, critic_lr=1e-3,
                   alpha_lr=1e-3, alpha=float(fx["alpha0"]), obs_norm=True, update_batch_size=B, grad_steps=gsteps,
                   update_freq=ufreq, buffer_size=size, max_batch=max_batch or B, device=DEV, seed=0)
    for k, net in NAMES.items():
        ag.load_net(net, params[k])
    rb = ag.replay_buffer
    oi = si = 0
    for kind, a, b in fx["ops"]:
        if kind == 0:
            assert rb.add_obs(fx["obs"][oi]) == a
            oi += 1
            continue
        assert rb.add_obs(fx["obs"][oi]) == b
        oi += 1
        rb.add_timestep(int(a), int(b), fx["act"][si], float(fx["rew"][si]), bool(fx["done"][si]), bool(fx["end"][si]))
        si += 1
    return ag


def test_vanilla_sac_obs_norm_make_update_matches_reference_fixture():
    """Two make_update cadences of the reference's vanilla SAC with obs_norm: the MT19937 index draws, the
    z-scored gather (initial zeros / ones statistics, then the device's update_obs_mean_std, which matches the
    reference's to fp32 rounding), two updates per cadence with the reference's rsample draws.  Losses rtol 1e-4,
    parameters within the Adam first-step allowance."""
    fx, params = _vanilla_case()
    ob, ac, B, gsteps, ufreq, size = (int(v) for v in fx["dims"])
    ag = _vanilla_agent(fx, params)
    rb = ag.replay_buffer
    assert ag.schedule == "reference" and rb.obs_norm and not rb.min_max_denormalize
    queue = []

    def staged_from_fixture(idx, key, ctr):  # the reference cadence's staged update, with the fixture's eps
        batch = rb.gather(idx)  # z-scored obs / next obs (obs_norm)
        e1, e2 = queue.pop(0), queue.pop(0)
        ag.update(*batch, eps_next=torch.from_numpy(e1).to(DEV), eps_cur=torch.from_numpy(e2).to(DEV))

    ag.update_from_replay = staged_from_fixture
    for c, s in enumerate(fx["np_seeds"]):
        if c == 1:
            ag.update_obs_stats()  # update_obs_mean_std (rl.py:93-112)
        np.testing.assert_allclose(rb.obs_mean.cpu().numpy(), fx["stats"][c][0], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(rb.obs_std.cpu().numpy(), fx["stats"][c][1], rtol=1e-6, atol=1e-6)
        ag.stats_logger.frames = ufreq * (c + 1)
        queue[:] = list(fx["eps"][c])
        np.random.seed(int(s))
        ag.make_update()
        assert not queue
        for j, k in enumerate(("critic_1", "critic_2", "actor")):
            assert ag.loss[k] == pytest.approx(float(fx["losses"][c][j]), rel=1e-4, abs=1e-6), (c, k)
    torch.cuda.synchronize()
    lr, n = 1e-3, len(fx["np_seeds"]) * gsteps
    for k, net in NAMES.items():
        d = np.abs(ag.params[net].cpu().numpy() - fx["post_" + k])
        scale = 1.0 if not k.endswith("targ") else float(fx["tau"])
        assert d.max() <= 2 * n * lr * scale * 1.01 + 1e-6, (k, d.max())
        assert np.mean(d > 1e-5 * max(scale, 0.05)) < 2e-3, (k, np.mean(d > 1e-5))
    assert ag.current_alpha() == pytest.approx(float(fx["alpha"]), rel=1e-5)


@pytest.mark.parametrize("stats", [False, True])
def test_vanilla_sac_obs_norm_staged_equals_caller_batch(stats):
    """sppAgentStageFromReplay + sppAgentStagePost(normalize = 2) -- the z-score of the ring's statistics although
    vanilla SAC's agent normaliser is min-max (its actor output's identity) -- leaves the parameters of the
    caller-batch update on the gathered, normalised tuples with the same eps, bit for bit."""
    fx, params = _vanilla_case()
    Bs = 120
    a1, a2 = _vanilla_agent(fx, params, Bs), _vanilla_agent(fx, params, Bs)
    if stats:
        a1.update_obs_stats()
        a2.update_obs_stats()
    idx = torch.from_numpy(np.random.RandomState(5).randint(0, len(a1.replay_buffer), Bs)).to(DEV)
    a1.update_from_replay_dp(idx, 91, 3)
    eps = [torch.empty(Bs, a1.ac_dim, device=DEV) for _ in range(2)]
    for w in range(2):
        _lib.call("sppAgentReadEps", a1._h, w, _lib.ptr(eps[w]), _lib.stream_handle())
    batch = a2.replay_buffer.gather(idx)
    raw = a2.replay_buffer
    raw.obs_norm = False
    unnorm = raw.gather(idx)
    raw.obs_norm = True
    assert not torch.equal(batch[0], unnorm[0])  # the normalisation ran (the clip at +-10 at least)
    a2.update(*batch, eps_next=eps[0], eps_cur=eps[1])
    torch.cuda.synchronize()
    for net in NAMES.values():
        np.testing.assert_array_equal(a1.params[net].cpu().numpy(), a2.params[net].cpu().numpy(), err_msg=str(net))
    assert a1.loss == a2.loss


@pytest.mark.parametrize("algo", ["sac", "ddpg"])
def test_acm_ob_idx_gather_takes_the_listed_columns(algo):
    """acm_cat(obs, next_obs) = [obs[:, idx] | next_obs[:, idx]] (acm.py:260-264) in every ACM gather, and an ACM
    regression step on it equals one on the host-permuted batch; lists the reference cannot run are refused."""
    ob, ac = 17, 6
    perm = list(np.random.RandomState(1).permutation(ob))
    perm[3] = perm[5]  # (repeats are a length-ob list too)
    Agent = spprl.SAC_AcM if algo == "sac" else spprl.DDPG_AcM
    kw = dict(env_name="HalfCheetah-v2", buffer_size=256, max_batch=128, device=DEV, seed=3)
    ag = Agent(acm_ob_idx=perm, **kw)
    ref = Agent(**kw)
    assert ag.acm_ob_idx == perm
    rng = np.random.RandomState(2)
    for a in (ag, ref):
        rb = a.replay_buffer
        r = np.random.RandomState(2)
        prev = rb.add_obs(r.randn(ob).astype(np.float32))
        for t in range(100):
            rb.add_acm_action(r.uniform(-1, 1, ac).astype(np.float32))
            nxt = rb.add_obs(r.randn(ob).astype(np.float32))
            rb.add_timestep(prev, nxt, r.uniform(-1, 1, ob).astype(np.float32), float(r.randn()), False, t % 25 == 24)
            prev = nxt
        a.params[_lib.SPP_NET_ACM].copy_(ref.params[_lib.SPP_NET_ACM])
    idx = torch.from_numpy(rng.randint(0, 100, 128)).to(DEV)
    x, y = torch.empty(128, 2 * ob, device=DEV), torch.empty(128, ac, device=DEV)
    x0, y0 = torch.empty_like(x), torch.empty_like(y)
    st = _lib.stream_handle()
    _lib.call("sppReplayGatherAcm", ag.replay_buffer._h, _lib.ptr(idx), 128, _lib.ptr(x), _lib.ptr(y), st)
    _lib.call("sppReplayGatherAcm", ref.replay_buffer._h, _lib.ptr(idx), 128, _lib.ptr(x0), _lib.ptr(y0), st)
    p = torch.tensor(perm, device=DEV)
    expect = torch.cat([x0[:, :ob][:, p], x0[:, ob:][:, p]], 1)
    assert torch.equal(x, expect) and torch.equal(y, y0)
    l1 = ag.batch_update_acm(x, y)
    l2 = ref.batch_update_acm(expect, y0)
    torch.cuda.synchronize()
    assert float(l1) == float(l2)
    assert torch.equal(ag.params[_lib.SPP_NET_ACM], ref.params[_lib.SPP_NET_ACM])
    with pytest.raises(ValueError):
        Agent(acm_ob_idx=[0, 1, 2], **kw)  # the reference's AcM would take ob + 3 inputs, acm_cat gives it 6
    with pytest.raises(ValueError):
        Agent(acm_ob_idx=list(range(ob - 1)) + [ob], **kw)


def test_ppo_acm_obs_norm_changes_nothing():
    """PPO_AcM(obs_norm=True): the flag reaches only ReplayBufferAcM.obs_norm, which the on-policy loop never
    reads -- one iteration with and without it leaves identical parameters."""
    kw = dict(env_name="HalfCheetah-v2", n_envs=32, batch_size=256, ppo_batch_size=128, max_ppo_epochs=2,
              acm_epochs=1, acm_batch_size=64, acm_update_freq=1, acm_pre_train_samples=512,
              acm_pre_train_epochs=1, acm_ring_size=2048, critic_num_target_updates=2,
              num_critic_updates_per_target=2, device=DEV, seed=4, loop_seed=9)
    out = []
    for flag in (False, True):
        ag = spprl.PPO_AcM(obs_norm=flag, **kw)
        ag.pre_train()
        ag.perform_iteration()
        torch.cuda.synchronize()
        out.append([t.cpu().numpy() for t in (ag.nets.params[0], ag.nets.params[1], ag.acm.params[5])])
    for a, b in zip(*out):
        np.testing.assert_array_equal(a, b)
