"""Rebuilds the inputs of the golden fixtures (tests/golden/make_golden.py)
from their numpy seeds, so fixtures only carry expected outputs."""
import os

import numpy as np
import torch

from weights import fill_params
from oracle import nets
from oracle.nets import Norm

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

SAC_CASES = {
    "sac_hopper_paper": dict(seed=1, acm_critic=True, custom_loss=0.2, norm_closs=False, min_max=True, steps=2),
    "sac_hopper_normcl": dict(seed=2, acm_critic=True, custom_loss=0.5, norm_closs=True, min_max=True, steps=1),
    "sac_hopper_plain": dict(seed=3, acm_critic=False, custom_loss=0.0, norm_closs=False, min_max=False, steps=1),
    "sac_hcheetah_paper": dict(seed=4, acm_critic=True, custom_loss=0.2, norm_closs=False, min_max=True, steps=1),
}


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz")))


def make_batch(rng, B, ob, aout, ac, done_p=0.15):
    obs = (rng.randn(B, ob) * 1.3).astype(np.float32)
    next_obs = (rng.randn(B, ob) * 1.3).astype(np.float32)
    act = rng.uniform(-1.2, 1.2, (B, aout)).astype(np.float32)
    rew = rng.randn(B).astype(np.float32)
    done = (rng.rand(B) < done_p).astype(np.int8)
    acm = rng.uniform(-1, 1, (B, ac)).astype(np.float32)
    return obs, next_obs, act, rew, done, acm


def sac_case(name):
    """Returns (cfg, fixture, params{net: {name: arr}}, norm, steps[list of (batch, eps1, eps2)])."""
    cfg = SAC_CASES[name]
    fx = load(name)
    ob, aout, ac, B = (int(v) for v in fx["dims"])
    seed = cfg["seed"]
    cin = ob + (ac if cfg["acm_critic"] else aout)
    layouts = {"actor": nets.sac_actor_layout(ob, aout), "critic_1": nets.critic_layout(cin),
               "critic_2": nets.critic_layout(cin), "critic_1_targ": nets.critic_layout(cin),
               "critic_2_targ": nets.critic_layout(cin), "acm": nets.acm_layout(2 * ob, ac)}
    params = {k: fill_params(lay, seed * 100 + i) for i, (k, lay) in enumerate(layouts.items())}
    rng = np.random.RandomState(seed)
    lo = -rng.uniform(0.5, 2.0, ob).astype(np.float32)
    hi = rng.uniform(0.5, 2.0, ob).astype(np.float32)
    mu = (rng.randn(ob) * 0.3).astype(np.float32)
    sd = rng.uniform(0.5, 1.5, ob).astype(np.float32)
    norm = Norm(cfg["min_max"], *(torch.from_numpy(v) for v in (lo, hi, mu, sd)))
    steps = []
    for _ in range(cfg["steps"]):
        batch = make_batch(rng, B, ob, aout, ac)
        e1 = rng.randn(B, aout).astype(np.float32)
        e2 = rng.randn(B, aout).astype(np.float32)
        steps.append((batch, e1, e2))
    return cfg, fx, params, layouts, norm, steps


def ddpg_case():
    from oracle.nets import basic_acm_layout, critic_layout, ddpg_actor_layout
    fx = load("ddpg_hcheetah_paper")
    ob, aout, ac, B = (int(v) for v in fx["dims"])
    seed = int(fx["seed"])
    layouts = {"actor": ddpg_actor_layout(ob, aout), "critic": critic_layout(ob + ac),
               "actor_targ": ddpg_actor_layout(ob, aout), "critic_targ": critic_layout(ob + ac),
               "acm": basic_acm_layout(2 * ob, ac)}
    params = {k: fill_params(lay, seed * 100 + i) for i, (k, lay) in enumerate(layouts.items())}
    rng = np.random.RandomState(seed)
    lo = -rng.uniform(0.5, 2.0, ob).astype(np.float32)
    hi = rng.uniform(0.5, 2.0, ob).astype(np.float32)
    norm = Norm(True, torch.from_numpy(lo), torch.from_numpy(hi))
    batches = [make_batch(rng, B, ob, aout, ac) for _ in range(2)]
    return fx, params, layouts, norm, batches


def sac_vanilla_case():
    """Vanilla SAC (HalfCheetah, configs[0]): (fixture, params, steps[(batch5, eps1, eps2)])."""
    fx = load("sac_vanilla_hcheetah")
    ob, ac, B = (int(v) for v in fx["dims"])
    seed = int(fx["seed"])
    layouts = {"actor": nets.sac_actor_layout(ob, ac), "critic_1": nets.critic_layout(ob + ac),
               "critic_2": nets.critic_layout(ob + ac), "critic_1_targ": nets.critic_layout(ob + ac),
               "critic_2_targ": nets.critic_layout(ob + ac)}
    params = {k: fill_params(lay, seed * 100 + i) for i, (k, lay) in enumerate(layouts.items())}
    rng = np.random.RandomState(seed)
    steps = []
    for _ in range(len(fx["losses"])):
        obs, next_obs, act, rew, done, _ = make_batch(rng, B, ob, ac, ac)
        act = np.clip(act, -1, 1)
        e1 = rng.randn(B, ac).astype(np.float32)
        e2 = rng.randn(B, ac).astype(np.float32)
        steps.append(((obs, next_obs, act, rew, done), e1, e2))
    return fx, params, steps


def onpolicy_case():
    """A2C / PPO_AcM fixture (tests/golden/onpolicy_hcheetah.npz): every input is stored."""
    return load("onpolicy_hcheetah")


def normalize_adv_ref(adv):
    """AdvantageDataset normalisation (advantage_dataset.py:8-12): torch.std is unbiased."""
    a = torch.as_tensor(adv)
    return ((a - a.mean()) / (a.std() + 1.2e-7)).numpy()


def ddpg_unbiased_case(name="ddpg_unbiased_hcheetah"):
    """DDPG_AcM / SAC_AcM (unbiased_update=True).make_update fixtures (tests/golden/ddpg_unbiased_hcheetah.npz,
    sac_unbiased_hcheetah.npz): (fixture, params, layouts, norm (z-score), ring ops replayer).  acm_critic=False:
    critics on (obs, actor output)."""
    from oracle.nets import critic_layout, ddpg_actor_layout
    fx = load(name)
    ob, aout, ac = (int(v) for v in fx["dims"][:3])
    seed = int(fx["seed"])
    if name.startswith("sac"):
        layouts = {"actor": nets.sac_actor_layout(ob, aout), "critic_1": critic_layout(ob + aout),
                   "critic_2": critic_layout(ob + aout), "critic_1_targ": critic_layout(ob + aout),
                   "critic_2_targ": critic_layout(ob + aout)}
    else:
        layouts = {"actor": ddpg_actor_layout(ob, aout), "critic": critic_layout(ob + aout),
                   "actor_targ": ddpg_actor_layout(ob, aout), "critic_targ": critic_layout(ob + aout)}
    params = {k: fill_params(lay, seed * 100 + i) for i, (k, lay) in enumerate(layouts.items())}
    mu, sd = fx["norm"]
    norm = Norm(False, mean=torch.from_numpy(mu), std=torch.from_numpy(sd))

    def replay(add_obs, add_acm_action, add_timestep):
        """Feed the fixture's ring writes (add_obs / add_acm_action / add_timestep) to a buffer."""
        oi = si = 0
        for kind, a, b in fx["ops"]:
            if kind == 0:
                assert add_obs(fx["obs"][oi]) == a
                oi += 1
                continue
            add_acm_action(fx["acm"][si])
            assert add_obs(fx["obs"][oi]) == b
            oi += 1
            add_timestep(int(a), int(b), fx["act"][si], float(fx["rew"][si]), bool(fx["done"][si]),
                         bool(fx["end"][si]))
            si += 1

    return fx, params, layouts, norm, replay
