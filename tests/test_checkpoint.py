"""Checkpoint interop (rltoolkit/rl.py:263-301, algorithms/sac/sac.py:287-309,
acm/off_policy/ddpg_acm.py:87-94).

CPU: the parameter-name layouts of every network and the top-level key order match the reference's
shipped checkpoints (tests/golden/ref_ckpt_keys.json, read by disassembling the reference's
/root/reference/models/*.pkl -- torch's weights-only loader refuses those files, so their tensors are
never loaded); save_params / load_params round trips; the loader refuses any pickle that names a
global outside the state-dict allowlist, without executing it.
GPU: SAC_AcM, vanilla SAC, DDPG_AcM and PPO_AcM save -> load into a differently seeded agent gives
bit-identical networks, normaliser state and actions."""
import collections
import json
import os
import pickle

import numpy as np
import pytest
import torch

from spprl import nets, onpolicy
from spprl.checkpoint import load_params, save_params

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_ckpt_keys.json")
TENSOR_KEYS = ("obs_mean", "obs_std", "min_obs", "max_obs")


def _names(layout):
    return [n for n, _ in layout]


def _expected(kind, ob, ac):
    if kind == "sac_acm":
        return {"actor": _names(nets.sac_actor_layout(ob, ac)), "critic_1": _names(nets.critic_layout(ob + ac)),
                "critic_2": _names(nets.critic_layout(ob + ac)), **{k: None for k in TENSOR_KEYS},
                "acm": _names(nets.acm_layout(2 * ob, ac))}
    if kind == "ddpg_acm":
        return {"actor": _names(nets.ddpg_actor_layout(ob, ac)), "critic": _names(nets.critic_layout(ob + ac)),
                **{k: None for k in TENSOR_KEYS}, "acm": _names(nets.basic_acm_layout(2 * ob, ac))}
    return {"actor": _names(onpolicy.actor_layout(ob, ob)), "critic": _names(onpolicy.critic_layout(ob)),
            **{k: None for k in TENSOR_KEYS}, "acm": _names(nets.acm_layout(2 * ob, ac))}


def _kind(fn):
    return "sac_acm" if "sac_acm" in fn else ("ddpg_acm" if "ddpg_acm" in fn else "ppo_acm")


@pytest.mark.parametrize("fn", sorted(json.load(open(GOLD))))
def test_param_layouts_match_reference_checkpoints(fn):
    ref = json.load(open(GOLD))[fn]
    exp = _expected(_kind(fn), 11, 3)
    assert list(ref) == list(exp), (fn, list(ref), list(exp))
    for k, v in exp.items():
        assert ref[k] == v, (fn, k)


def _rand_params(kind, ob, ac, seed=0):
    g = torch.Generator().manual_seed(seed)
    lay = {"sac_acm": {"actor": nets.sac_actor_layout(ob, ac), "critic_1": nets.critic_layout(ob + ac),
                       "critic_2": nets.critic_layout(ob + ac), "acm": nets.acm_layout(2 * ob, ac)}}[kind]
    out = {}
    for k in ("actor", "critic_1", "critic_2"):
        out[k] = collections.OrderedDict((n, torch.randn(s, generator=g)) for n, s in lay[k])
    out.update({k: torch.randn(ob, generator=g) for k in TENSOR_KEYS})
    out["acm"] = collections.OrderedDict((n, torch.randn(s, generator=g)) for n, s in lay["acm"])
    return out


def test_save_load_roundtrip_cpu(tmp_path):
    d = _rand_params("sac_acm", 11, 3)
    p = str(tmp_path / "ck.pkl")
    save_params(p, d)
    e = load_params(p)
    assert list(e) == list(d)
    for k, v in d.items():
        if isinstance(v, dict):
            assert isinstance(e[k], collections.OrderedDict) and list(e[k]) == list(v)
            for n in v:
                assert torch.equal(e[k][n], v[n])
        else:
            assert torch.equal(e[k], v)
    # the file is a plain pickle of the reference's structure (what the reference's pkl.load reads)
    with open(p, "rb") as f:
        assert f.read(2)[0] == 0x80


def test_loader_refuses_foreign_globals(tmp_path):
    p = str(tmp_path / "bad.pkl")
    with open(p, "wb") as f:
        pickle.dump({"actor": collections.Counter(a=1)}, f)  # a global outside the allowlist
    with pytest.raises(pickle.UnpicklingError):
        load_params(p)


# ------------------------------------------------------------------------------------------ GPU
def _equal_states(a, b):
    assert list(a) == list(b)
    for k in a:
        va, vb = a[k], b[k]
        if va is None or vb is None:
            assert va is None and vb is None, k
        elif isinstance(va, dict):
            assert list(va) == list(vb), k
            for n in va:
                assert torch.equal(torch.as_tensor(va[n]).cpu(), torch.as_tensor(vb[n]).cpu()), (k, n)
        else:
            assert torch.equal(torch.as_tensor(va).cpu(), torch.as_tensor(vb).cpu()), k


def _fill_stats(ag, ob, seed):
    rb = ag.replay_buffer
    rng = np.random.RandomState(seed)
    rows = rng.randn(300, ob).astype(np.float32)
    slots = rb.add_obs_batch(torch.from_numpy(rows).cuda())
    n = len(rows) - 1
    rb.add_timestep_batch(slots[:n], slots[1:], torch.zeros(n, ag.actor_output_dim), np.zeros(n), np.zeros(n, bool),
                          np.zeros(n, bool), torch.zeros(n, ag.ac_dim))
    rb.update_obs_mean_std()


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["sac_acm", "sac", "ddpg_acm"])
def test_offpolicy_checkpoint_roundtrip(algo, tmp_path):
    import spprl

    mk = {"sac_acm": lambda s: spprl.SAC_AcM(env_name="Hopper-v2", buffer_size=512, device="cuda:0", seed=s,
                                             min_max_denormalize=True),
          "sac": lambda s: spprl.SAC(env_name="HalfCheetah-v2", buffer_size=512, device="cuda:0", seed=s),
          "ddpg_acm": lambda s: spprl.DDPG_AcM(env_name="HalfCheetah-v2", buffer_size=512, device="cuda:0", seed=s,
                                               min_max_denormalize=True)}[algo]
    a, b = mk(0), mk(7)
    _fill_stats(a, a.ob_dim, 1)
    da = a.collect_params_dict()
    assert list(da) == list(_expected(algo if algo != "sac" else "sac_acm", a.ob_dim, a.ac_dim)) or algo == "sac"
    p = str(tmp_path / "ck.pkl")
    a.save(p)
    b.load(p)
    _equal_states(da, b.collect_params_dict())
    obs = torch.randn(64, a.ob_dim, device="cuda:0")
    eps = torch.randn(64, a.actor_output_dim, device="cuda:0")
    ta, ea = a.act(obs, eps=eps, mode=2, act_noise=0.0)
    tb, eb = b.act(obs, eps=eps, mode=2, act_noise=0.0)
    assert torch.equal(ta, tb) and torch.equal(ea, eb)


@pytest.mark.gpu
def test_ppo_acm_checkpoint_roundtrip(tmp_path):
    import spprl

    mk = lambda s: spprl.PPO_AcM(env_name="HalfCheetah-v2", n_envs=4, batch_size=64, iterations=1,
                                 ppo_batch_size=32, device="cuda:0", seed=s, env_spec=(17, 6, 1.0, 40))
    a, b = mk(0), mk(3)
    _fill_stats(a.acm, 17, 2)
    da = a.collect_params_dict()
    assert list(da) == list(_expected("ppo_acm", 17, 6))
    p = str(tmp_path / "ck.pkl")
    a.save(p)
    b.load(p)
    _equal_states(da, b.collect_params_dict())
