"""Golden-vector generator: runs the REFERENCE rltoolkit on CPU, in the build
container only (``/root/reference`` does not exist on the GPU box), and writes
small .npz fixtures next to this file.  The fixtures (inputs + expected
outputs) are data; no reference source is copied into the repository.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference pins gym 0.15 / mujoco-py / tensorboard, none of which exist
here, so a minimal stand-in for those *dependencies* is installed first
(SURVEY.md Appendix A): a synthetic fixed-shape env, a no-op SummaryWriter,
``np.int = int``.  Only the reference's own code paths under test run:
replay-ring indexing and sampling (rltoolkit/buffer/replay_buffer.py),
SAC_AcM / DDPG_AcM ``update`` (rltoolkit/acm/off_policy/*.py), AcMTrainer
``batch_update`` (rltoolkit/acm/acm.py:246-258), ``update_obs_mean_std``
(replay_buffer.py:83-96) and PPO ``calculate_gae`` / ``_clip_loss``
(rltoolkit/algorithms/ppo/ppo.py:117-150,194-204).

Gaussian draws inside ``Normal.rsample`` come from torch's CPU generator and
are not reproducible across implementations, so they are injected: the
generator replaces ``torch.distributions.normal._standard_normal`` with a
queue of seeded arrays that the tests regenerate.
"""
import os
import sys
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
os.makedirs("/tmp/spprl_golden", exist_ok=True)
sys.argv[0] = "/tmp/spprl_golden/gen.py"  # reference logger mkdirs next to argv[0]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from weights import fill_params  # noqa: E402

np.int = int  # reference targets numpy 1.18

# ---------------------------------------------------------------- dependency stand-ins
gym = types.ModuleType("gym")
spaces = types.ModuleType("gym.spaces")


class Box:
    def __init__(self, low, high, shape, seed=0):
        self.shape = shape
        self.low = np.full(shape, low, np.float32)
        self.high = np.full(shape, high, np.float32)
        self._rng = np.random.RandomState(seed)

    def sample(self):
        return self._rng.uniform(self.low, self.high).astype(np.float32)


class Discrete:
    def __init__(self, n):
        self.n = n


spaces.Box, spaces.Discrete, gym.spaces = Box, Discrete, spaces
SPECS = {"Pendulum-v0": (3, 1, 200), "Hopper-v2": (11, 3, 1000),
         "HalfCheetah-v2": (17, 6, 1000), "Ant-v2": (111, 8, 1000)}


class SynthEnv:
    def __init__(self, name, seed=0):
        ob, ac, T = SPECS[name]
        self.observation_space = Box(-np.inf, np.inf, (ob,))
        lim = 2.0 if name == "Pendulum-v0" else 1.0
        self.action_space = Box(-lim, lim, (ac,), seed)
        self._max_episode_steps = T


gym.make = lambda name: SynthEnv(name)
sys.modules["gym"] = gym
sys.modules["gym.spaces"] = spaces
tb = types.ModuleType("torch.utils.tensorboard")


class SummaryWriter:
    def __init__(self, *a, **k):
        pass

    def __getattr__(self, n):
        return lambda *a, **k: None


tb.SummaryWriter = SummaryWriter
sys.modules["torch.utils.tensorboard"] = tb
pvd = types.ModuleType("pyvirtualdisplay")
pvd.Display = object
sys.modules["pyvirtualdisplay"] = pvd
sys.path.insert(0, "/root/reference/rltoolkit")

from rltoolkit.acm.models.basic_acm import BasicAcM  # noqa: E402
from rltoolkit.acm.on_policy import PPO_AcM  # noqa: E402
from rltoolkit.algorithms import A2C, SAC  # noqa: E402
from rltoolkit.basic_model import Actor  # noqa: E402
from rltoolkit.buffer import MemoryAcM  # noqa: E402
from rltoolkit.acm.off_policy import DDPG_AcM, SAC_AcM  # noqa: E402
from rltoolkit.algorithms.ppo.ppo import PPO  # noqa: E402
from rltoolkit.buffer import BufferAcMOffPolicy, Memory  # noqa: E402

torch.set_num_threads(1)


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print("wrote", path, sum(a.size for a in arrays.values()), "values")


# ---------------------------------------------------------------- MT19937 randint
def gen_randint():
    out = {}
    cases = []
    for seed in (0, 1, 7, 12345, 2**31 - 1, 4294967295):
        for n in (1, 2, 3, 7, 100, 1000, 1024, 1025, 65537, 10**6, 10**7, 2**31 - 1):
            cases.append((seed, n))
    seeds = np.array([c[0] for c in cases], np.uint64)
    ns = np.array([c[1] for c in cases], np.int64)
    K = 257
    vals = np.zeros((len(cases), K), np.int64)
    for i, (s, n) in enumerate(cases):
        rs = np.random.RandomState(s)
        vals[i] = rs.randint(0, n, K)
    out.update(seeds=seeds, ns=ns, vals=vals)
    # interleaved draws from one stream (sample_batch called repeatedly)
    rs = np.random.RandomState(42)
    seq_n = np.array([100, 5000, 3, 999999, 100, 17], np.int64)
    seq = [rs.randint(0, n, 64) for n in seq_n]
    out.update(seq_seed=np.array(42), seq_n=seq_n, seq_vals=np.stack(seq))
    save("mt19937_randint.npz", **out)


# ---------------------------------------------------------------- replay ring (Q6)
def gen_replay():
    out = {}
    # (a) SURVEY Q6 trace: size 10, 5 episodes of 3 steps
    # (b) size 50, ragged episodes 1..9 steps, 40 episodes, ob=3, aout=3, ac=2
    for tag, size, ob, aout, ac, ep_lens, seed in (
        ("a", 10, 2, 2, 1, [3] * 5, 0),
        ("b", 50, 3, 3, 2, list(np.random.RandomState(3).randint(1, 10, 40)), 1),
        ("c", 64, 11, 11, 3, list(np.random.RandomState(4).randint(1, 30, 25)), 2),
    ):
        rng = np.random.RandomState(seed)
        buf = BufferAcMOffPolicy(size, ob, aout, acm_act_shape=ac)
        ops = []  # (kind, a, b): kind 0 = add_obs(reset), 1 = step
        obs_log, act_log, acm_log, rew_log, done_log, end_log = [], [], [], [], [], []
        states = []
        for L in ep_lens:
            o = rng.randn(1, ob).astype(np.float32)
            prev = buf.add_obs(torch.from_numpy(o))
            obs_log.append(o[0])
            ops.append((0, prev, -1))
            for t in range(L):
                acm = rng.uniform(-1, 1, ac).astype(np.float32)
                buf.add_acm_action(acm)
                a = torch.from_numpy(rng.randn(1, aout).astype(np.float32))
                o = rng.randn(1, ob).astype(np.float32)
                nxt = buf.add_obs(torch.from_numpy(o))
                r = float(rng.randn())
                end = t == L - 1
                done = bool(end and rng.rand() < 0.5)
                buf.add_timestep(prev, nxt, a, r, done, end)
                ops.append((1, prev, nxt))
                obs_log.append(o[0])
                act_log.append(a.numpy()[0])
                acm_log.append(acm)
                rew_log.append(r)
                done_log.append(done)
                end_log.append(end)
                states.append((buf.obs_idx, buf.ts_idx, buf.current_len))
                prev = nxt
        p = "r%s_" % tag
        out[p + "dims"] = np.array([size, ob, aout, ac])
        out[p + "ops"] = np.array(ops, np.int64)
        out[p + "obs"] = np.array(obs_log, np.float32)
        out[p + "act"] = np.array(act_log, np.float32)
        out[p + "acm"] = np.array(acm_log, np.float32)
        out[p + "rew"] = np.array(rew_log, np.float32)
        out[p + "done"] = np.array(done_log, np.bool_)
        out[p + "end"] = np.array(end_log, np.bool_)
        out[p + "states"] = np.array(states, np.int64)
        # last_rollout (replay_buffer.py:335-383) on the built ring, before the stats below scale _obs
        m = buf.last_rollout()
        out[p + "lr_obs"] = m.obs.numpy()
        out[p + "lr_next_obs"] = m.next_obs.numpy()
        out[p + "lr_act"] = torch.cat([torch.as_tensor(a).reshape(1, -1) for a in m._actions]).numpy().astype(np.float32)
        out[p + "lr_rew"] = np.array(m._rewards, np.float32)
        out[p + "lr_end"] = np.array(m._end, np.bool_)
        out[p + "lr_acm"] = np.stack([np.asarray(a, np.float32) for a in m.actions_acm])
        L = buf.current_len
        out[p + "obs_idx"] = buf._obs_idx[:L].astype(np.int64)
        out[p + "next_obs_idx"] = buf._next_obs_idx[:L].astype(np.int64)
        # sample_batch after np.random.seed(s)  (replay_buffer.py:233-261,385-398)
        for s in (0, 5):
            B = 33
            np.random.seed(s)
            o, no, a, r, d, acm = buf.sample_batch(B)
            np.random.seed(s)
            idx = np.random.randint(0, len(buf), B)
            q = p + "s%d_" % s
            out[q + "idx"] = idx.astype(np.int64)
            out[q + "obs"] = o.numpy()
            out[q + "next_obs"] = no.numpy()
            out[q + "act"] = a.numpy()
            out[q + "rew"] = r.numpy()
            out[q + "done"] = d.numpy()
            out[q + "acm"] = acm.numpy()
        # ACM regression batch (replay_buffer.py:404-430)
        np.random.seed(9)
        o, no, acm = buf.sample_acm_batch(17)
        out[p + "acmb_obs"], out[p + "acmb_next_obs"], out[p + "acmb_acm"] = (
            o.numpy(), no.numpy(), acm.numpy())
        # obs statistics (replay_buffer.py:83-96), twice for running max/min
        def stats():  # None (len <= 10: stats skipped) -> NaN row
            return np.stack([np.full(ob, np.nan, np.float32) if t is None else t.numpy()
                             for t in (buf.obs_mean, buf.obs_std, buf.max_obs, buf.min_obs)])

        buf.update_obs_mean_std()
        out[p + "st1"] = stats()
        buf._obs[buf._obs_idx[: buf.current_len]] *= 0.5
        buf.update_obs_mean_std()
        out[p + "st2"] = stats()
    save("replay_ring.npz", **out)


# ---------------------------------------------------------------- eps injection
class EpsQueue:
    def __init__(self):
        self.q = []

    def __call__(self, shape, dtype, device):
        e = self.q.pop(0)
        assert tuple(e.shape) == tuple(shape), (e.shape, shape)
        return torch.from_numpy(e).to(dtype)


EPS = EpsQueue()
torch.distributions.normal._standard_normal = EPS


def named_shapes(module):
    return [(k, tuple(v.shape)) for k, v in module.state_dict().items()]


def load(module, seed):
    vals = fill_params(named_shapes(module), seed)
    module.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})


def flat_params(module):
    return np.concatenate([v.detach().numpy().ravel() for v in module.state_dict().values()])


def make_batch(rng, B, ob, aout, ac, done_p=0.15):
    obs = (rng.randn(B, ob) * 1.3).astype(np.float32)
    next_obs = (rng.randn(B, ob) * 1.3).astype(np.float32)
    act = rng.uniform(-1.2, 1.2, (B, aout)).astype(np.float32)
    rew = rng.randn(B).astype(np.float32)
    done = (rng.rand(B) < done_p).astype(np.int8)
    acm = rng.uniform(-1, 1, (B, ac)).astype(np.float32)
    return obs, next_obs, act, rew, done, acm


# ---------------------------------------------------------------- SAC_AcM.update
SAC_VARIANTS = {
    # name: env, B, flags, steps, store_adam
    "sac_hopper_paper": ("Hopper-v2", 100, dict(acm_critic=True, custom_loss=0.2, norm_closs=False,
                                                 min_max_denormalize=True, denormalize_actor_out=True), 2, True),
    "sac_hopper_normcl": ("Hopper-v2", 37, dict(acm_critic=True, custom_loss=0.5, norm_closs=True,
                                                 min_max_denormalize=True, denormalize_actor_out=True), 1, False),
    "sac_hopper_plain": ("Hopper-v2", 64, dict(acm_critic=False, custom_loss=0.0,
                                                min_max_denormalize=False, denormalize_actor_out=False), 1, False),
    "sac_hcheetah_paper": ("HalfCheetah-v2", 45, dict(acm_critic=True, custom_loss=0.2, norm_closs=False,
                                                       min_max_denormalize=True, denormalize_actor_out=True), 1, False),
}


def gen_sac(name, env, B, flags, steps, store_adam, seed):
    torch.manual_seed(0)
    m = SAC_AcM(env_name=env, gamma=0.99, actor_lr=1e-3, critic_lr=1e-3, alpha_lr=1e-3, alpha=0.2,
                buffer_size=1000, acm_pre_train_samples=10, acm_val_buffer_size=None,
                update_batch_size=B, use_gpu=False, **flags)
    ob, aout, ac = m.ob_dim, m.actor_output_dim, m.ac_dim
    nets = {"actor": m._actor, "critic_1": m._critic_1, "critic_2": m._critic_2,
            "critic_1_targ": m.critic_1_targ, "critic_2_targ": m.critic_2_targ, "acm": m.acm}
    for i, (k, mod) in enumerate(nets.items()):
        load(mod, seed * 100 + i)
    rng = np.random.RandomState(seed)
    lo = -rng.uniform(0.5, 2.0, ob).astype(np.float32)
    hi = rng.uniform(0.5, 2.0, ob).astype(np.float32)
    mu = (rng.randn(ob) * 0.3).astype(np.float32)
    sd = rng.uniform(0.5, 1.5, ob).astype(np.float32)
    m.replay_buffer.min_obs, m.replay_buffer.max_obs = torch.from_numpy(lo), torch.from_numpy(hi)
    m.replay_buffer.obs_mean, m.replay_buffer.obs_std = torch.from_numpy(mu), torch.from_numpy(sd)
    out = dict(dims=np.array([ob, aout, ac, B]), seed=np.array(seed),
               norm=np.stack([lo, hi, mu, sd]), actor_ac_lim=m.actor_ac_lim.numpy().astype(np.float32),
               acm_ac_lim=np.asarray(m.acm.ac_lim, np.float32),
               log_alpha0=np.array(float(m.log_alpha)), alpha0=np.array(m.alpha),
               target_entropy=np.array(m.target_entropy), tau=np.array(m.tau), gamma=np.array(m.gamma))
    ys, logps = [], []
    orig_targ, orig_pi = m.compute_qfunc_targ, m.compute_pi_loss

    def targ(*a, **k):
        y = orig_targ(*a, **k)
        ys.append(y.detach().numpy().copy())
        return y

    def pi(obs, sa, slp, nobs):
        logps.append(slp.detach().numpy().copy())
        return orig_pi(obs, sa, slp, nobs)

    m.compute_qfunc_targ, m.compute_pi_loss = targ, pi
    losses = []
    for s in range(steps):
        obs, next_obs, act, rew, done, acm = make_batch(rng, B, ob, aout, ac)
        eps1 = rng.randn(B, aout).astype(np.float32)
        eps2 = rng.randn(B, aout).astype(np.float32)
        EPS.q = [eps1, eps2]
        m.update(torch.from_numpy(obs), torch.from_numpy(next_obs), torch.from_numpy(act),
                 torch.from_numpy(rew), torch.from_numpy(done), torch.from_numpy(acm))
        assert not EPS.q
        losses.append([m.loss.get(k, 0.0) for k in ("critic_1", "critic_2", "actor", "sac", "dist")])
    out["y"] = np.stack(ys)
    out["logp"] = np.stack(logps)
    out["losses"] = np.array(losses)
    out["log_alpha"] = np.array(float(m.log_alpha))
    out["alpha"] = np.array(m.alpha)
    for k, mod in nets.items():
        if k != "acm":
            out["post_" + k] = flat_params(mod)
    if store_adam:
        for k, opt, mod in (("actor", m.actor_optimizer, m._actor), ("critic_1", m.critic_1_optimizer, m._critic_1)):
            st = [opt.state[p] for p in mod.parameters()]
            out["m_" + k] = np.concatenate([s["exp_avg"].numpy().ravel() for s in st])
            out["v_" + k] = np.concatenate([s["exp_avg_sq"].numpy().ravel() for s in st])
    save(name + ".npz", **out)


# ---------------------------------------------------------------- DDPG_AcM.update
def gen_ddpg(seed=11):
    torch.manual_seed(0)
    env = "HalfCheetah-v2"
    m = DDPG_AcM(env_name=env, gamma=0.95, actor_lr=5e-4, critic_lr=5e-4, buffer_size=1000,
                 acm_pre_train_samples=10, acm_val_buffer_size=None, update_batch_size=50,
                 custom_loss=1.0, norm_closs=False, acm_critic=True, min_max_denormalize=True,
                 denormalize_actor_out=True, act_noise=0.05, use_gpu=False)
    m.acm = BasicAcM(34, 6, False)
    ob, aout, ac, B = m.ob_dim, m.actor_output_dim, m.ac_dim, 50
    nets = {"actor": m._actor, "critic": m._critic, "actor_targ": m.actor_targ,
            "critic_targ": m.critic_targ, "acm": m.acm}
    for i, (k, mod) in enumerate(nets.items()):
        load(mod, seed * 100 + i)
    rng = np.random.RandomState(seed)
    lo = -rng.uniform(0.5, 2.0, ob).astype(np.float32)
    hi = rng.uniform(0.5, 2.0, ob).astype(np.float32)
    m.replay_buffer.min_obs, m.replay_buffer.max_obs = torch.from_numpy(lo), torch.from_numpy(hi)
    out = dict(dims=np.array([ob, aout, ac, B]), seed=np.array(seed), norm=np.stack([lo, hi]),
               actor_ac_lim=m.actor_ac_lim.numpy().astype(np.float32), tau=np.array(m.tau),
               gamma=np.array(m.gamma))
    losses = []
    for s in range(2):
        obs, next_obs, act, rew, done, acm = make_batch(rng, B, ob, aout, ac)
        m.update(torch.from_numpy(obs), torch.from_numpy(next_obs), torch.from_numpy(act),
                 torch.from_numpy(rew), torch.from_numpy(done), torch.from_numpy(acm))
        losses.append([m.loss.get(k, 0.0) for k in ("critic", "actor", "ddpg", "dist")])
    out["losses"] = np.array(losses)
    for k, mod in nets.items():
        if k != "acm":
            out["post_" + k] = flat_params(mod)
    save("ddpg_hcheetah_paper.npz", **out)


# ---------------------------------------------------------------- AcMTrainer.batch_update
def gen_acm(seed=21):
    torch.manual_seed(0)
    m = SAC_AcM(env_name="Hopper-v2", acm_lr=1e-3, acm_pre_train_samples=10, acm_val_buffer_size=None,
                buffer_size=100, use_gpu=False)
    load(m.acm, seed)
    rng = np.random.RandomState(seed)
    xs, ys, ls = [], [], []
    for s in range(3):
        x = (rng.randn(100, 22) * 1.2).astype(np.float32)
        y = rng.uniform(-1, 1, (100, 3)).astype(np.float32)
        ls.append(m.batch_update(torch.from_numpy(x), torch.from_numpy(y)))
    out = dict(seed=np.array(seed), losses=np.array(ls), post_acm=flat_params(m.acm),
               ac_lim=np.asarray(m.acm.ac_lim, np.float32))
    save("acm_step.npz", **out)


# ---------------------------------------------------------------- PPO GAE / clip
def gen_ppo(seed=31):
    rng = np.random.RandomState(seed)
    buf = Memory()
    T = 0
    gam, lam = 0.99, 0.95
    for ep in range(6):
        L = int(rng.randint(1, 15))
        o = torch.from_numpy(rng.randn(1, 3).astype(np.float32))
        prev = buf.add_obs(o)
        for t in range(L):
            o = torch.from_numpy(rng.randn(1, 3).astype(np.float32))
            nxt = buf.add_obs(o)
            end = t == L - 1
            done = bool(end and rng.rand() < 0.5)
            buf.add_timestep(prev, nxt, np.zeros(1), np.zeros(1), float(rng.randn()), done, end)
            prev = nxt
            T += 1
        buf.end_rollout()
    buf.update_obs_mean_std()
    w = np.array([0.7, -1.1, 0.4], np.float32)

    def critic_func(obs, *a):
        if len(obs.shape) == 2:
            return obs @ torch.from_numpy(w)
        return (obs @ torch.from_numpy(w)).reshape(())

    ppo = PPO(env_name="Pendulum-v0", gamma=gam, gae_lambda=lam)
    ppo._critic = critic_func
    q = ppo.calculate_q_val(buf)
    adv = ppo.calculate_gae(buf, q)
    out = dict(obs=buf.norm_obs.numpy(), next_obs=buf.norm_next_obs.numpy(),
               rew=np.array(buf.rewards, np.float32), done=np.array(buf.done, np.float32),
               end=np.array(buf.end, np.float32), w=w, gamma=np.array(gam), lam=np.array(lam),
               q=q.numpy(), adv=adv.numpy())
    lp_old = rng.randn(64).astype(np.float32)
    lp_new = (lp_old + 0.3 * rng.randn(64)).astype(np.float32)
    A = rng.randn(64).astype(np.float32)
    ppo_e = PPO(env_name="Pendulum-v0", epsilon=0.2)
    cl = ppo_e._clip_loss(torch.from_numpy(lp_old), torch.from_numpy(lp_new), torch.from_numpy(A))
    out.update(clip_lp_old=lp_old, clip_lp_new=lp_new, clip_adv=A, clip_loss=np.array(cl.item()))
    save("ppo_gae_clip.npz", **out)


# ---------------------------------------------------------------- vanilla SAC.update (configs[0])
def gen_sac_vanilla(seed=41, B=100, steps=2):
    """SAC.update (rltoolkit/algorithms/sac/sac.py:218-280) at HalfCheetah dims: no ACM, the
    actor emits the env action (ac = 6), the critics take cat(obs, action)."""
    torch.manual_seed(0)
    m = SAC(env_name="HalfCheetah-v2", gamma=0.99, actor_lr=1e-3, critic_lr=1e-3, alpha_lr=1e-3, alpha=0.2,
            buffer_size=1000, update_batch_size=B, use_gpu=False)
    ob, ac = m.ob_dim, m.ac_dim
    nets = {"actor": m._actor, "critic_1": m._critic_1, "critic_2": m._critic_2,
            "critic_1_targ": m.critic_1_targ, "critic_2_targ": m.critic_2_targ}
    for i, (k, mod) in enumerate(nets.items()):
        load(mod, seed * 100 + i)
    rng = np.random.RandomState(seed)
    out = dict(dims=np.array([ob, ac, B]), seed=np.array(seed), ac_lim=m.ac_lim.numpy().astype(np.float32),
               alpha0=np.array(m.alpha), target_entropy=np.array(m.target_entropy), tau=np.array(m.tau),
               gamma=np.array(m.gamma), act_noise=np.array(m.act_noise),
               max_ep_len=np.array(m.max_ep_len if m.max_ep_len is not None else -1))
    losses = []
    for s in range(steps):
        obs, next_obs, act, rew, done, _ = make_batch(rng, B, ob, ac, ac)
        act = np.clip(act, -1, 1)
        EPS.q = [rng.randn(B, ac).astype(np.float32), rng.randn(B, ac).astype(np.float32)]
        m.update(torch.from_numpy(obs), torch.from_numpy(next_obs), torch.from_numpy(act), torch.from_numpy(rew),
                 torch.from_numpy(done))
        assert not EPS.q
        losses.append([m.loss[k] for k in ("critic_1", "critic_2", "actor")])
    out["losses"] = np.array(losses)
    out["log_alpha"] = np.array(float(m.log_alpha))
    out["alpha"] = np.array(m.alpha)
    for k, mod in nets.items():
        out["post_" + k] = flat_params(mod)
    save("sac_vanilla_hcheetah.npz", **out)


def gen_sac_vanilla_obsnorm(seed=43):
    """Vanilla SAC with obs_norm=True (configs[0]'s algorithm; DDPG.__init__ ddpg.py:101-115 gives the plain
    ReplayBuffer obs_norm): make_update (ddpg.py:231-237) over two cadences of the ring -- the first with the
    buffer's initial zeros / ones statistics (replay_buffer.py:113-115: only the +-10 clip, some obs beyond it),
    the second after update_obs_mean_std (rl.py:93-112, replay_buffer.py:83-96) -- each sample_batch z-scored
    (replay_buffer.py:246-249); rsample draws injected and stored."""
    torch.manual_seed(0)
    size, B, gsteps, ufreq = 400, 40, 2, 10
    m = SAC(env_name="HalfCheetah-v2", gamma=0.99, actor_lr=1e-3, critic_lr=1e-3, alpha_lr=1e-3, alpha=0.2,
            buffer_size=size, update_batch_size=B, grad_steps=gsteps, update_freq=ufreq, obs_norm=True,
            use_gpu=False)
    ob, ac = m.ob_dim, m.ac_dim
    nets = {"actor": m._actor, "critic_1": m._critic_1, "critic_2": m._critic_2,
            "critic_1_targ": m.critic_1_targ, "critic_2_targ": m.critic_2_targ}
    for i, (k, mod) in enumerate(nets.items()):
        load(mod, seed * 100 + i)
    rng = np.random.RandomState(seed)
    buf = m.replay_buffer
    assert buf.obs_norm and not buf.min_max_denormalize
    ops, obs_log, act_log, rew_log, done_log, end_log = [], [], [], [], [], []
    scale = (rng.uniform(0.5, 14.0, ob) * np.where(rng.rand(ob) < 0.5, -1, 1)).astype(np.float32)
    for L in rng.randint(5, 40, 9):  # ragged episodes, no wrap; columns of very different scales (some > 10)
        o = (rng.randn(1, ob) * scale + scale).astype(np.float32)
        prev = buf.add_obs(torch.from_numpy(o))
        obs_log.append(o[0])
        ops.append((0, prev, -1))
        for t in range(L):
            a = torch.from_numpy(rng.uniform(-1, 1, (1, ac)).astype(np.float32))
            o = (rng.randn(1, ob) * scale + scale).astype(np.float32)
            nxt = buf.add_obs(torch.from_numpy(o))
            r = float(rng.randn())
            end = t == L - 1
            done = bool(end and rng.rand() < 0.5)
            buf.add_timestep(prev, nxt, a, r, done, end)
            ops.append((1, prev, nxt))
            obs_log.append(o[0])
            act_log.append(a.numpy()[0])
            rew_log.append(r)
            done_log.append(done)
            end_log.append(end)
            prev = nxt
    out = dict(dims=np.array([ob, ac, B, gsteps, ufreq, size]), seed=np.array(seed), alpha0=np.array(m.alpha),
               target_entropy=np.array(m.target_entropy), tau=np.array(m.tau), gamma=np.array(m.gamma),
               ops=np.array(ops, np.int64), obs=np.array(obs_log, np.float32), act=np.array(act_log, np.float32),
               rew=np.array(rew_log, np.float32), done=np.array(done_log, np.bool_), end=np.array(end_log, np.bool_))
    losses, idxs, eps, stats, np_seeds = [], [], [], [], [401, 502]
    for c, s in enumerate(np_seeds):
        if c == 1:
            m.replay_buffer = m.update_obs_mean_std(m.replay_buffer)
            buf = m.replay_buffer
        stats.append(np.stack([buf.obs_mean.numpy(), buf.obs_std.numpy()]))
        m.stats_logger.frames = ufreq * (c + 1)
        assert m.update_condition()
        np.random.seed(s)
        idxs.append(np.stack([np.random.randint(0, len(buf), B) for _ in range(gsteps)]))
        e = [rng.randn(B, ac).astype(np.float32) for _ in range(2 * gsteps)]
        eps.append(np.stack(e))
        EPS.q = list(e)
        np.random.seed(s)
        m.make_update()
        assert not EPS.q
        losses.append([m.loss[k] for k in ("critic_1", "critic_2", "actor")])
    out.update(np_seeds=np.array(np_seeds), idx=np.stack(idxs), eps=np.stack(eps), stats=np.stack(stats),
               losses=np.array(losses), log_alpha=np.array(float(m.log_alpha)), alpha=np.array(m.alpha))
    for k, mod in nets.items():
        out["post_" + k] = flat_params(mod)
    save("sac_vanilla_obsnorm_hcheetah.npz", **out)


# ---------------------------------------------------------------- on-policy (A2C / PPO_AcM)
def onp_batch(rng, N, ob):
    obs = (rng.randn(N, ob) * 1.2).astype(np.float32)
    nobs = (rng.randn(N, ob) * 1.2).astype(np.float32)
    rew = rng.randn(N).astype(np.float32)
    done = (rng.rand(N) < 0.05).astype(np.float32)
    return obs, nobs, rew, done


def gen_onpolicy(seed=51):
    """Actor.act log-prob (basic_model.py:32-51), A2C.update_critic (a2c.py:186-225) and one
    PPO_AcM.update_actor_acm epoch over a single full-batch minibatch (acm/on_policy.py:164-216)."""
    out = {}
    ob = 17
    rng = np.random.RandomState(seed)
    # ---- Actor.act: sampled and deterministic actions, log-probs
    torch.manual_seed(seed)
    actor = Actor(ob, torch.ones(ob), ob, discrete=False)
    load(actor, seed * 100)
    with torch.no_grad():
        actor.log_scale.add_(torch.from_numpy(rng.uniform(-0.3, 0.3, ob).astype(np.float32)))
    x = (rng.randn(257, ob) * 1.3).astype(np.float32)
    a_s, lp_s = actor.act(torch.from_numpy(x))
    a_d, lp_d = actor.act(torch.from_numpy(x), deterministic=True)
    out.update(act_params=flat_params(actor), act_x=x, act_a=a_s.numpy(), act_lp=lp_s.detach().numpy(),
               act_mu=a_d.numpy(), act_lp_det=lp_d.detach().numpy())
    # ---- A2C.update_critic: 10 targets x 10 full-batch Adam steps on 0.5 * adv^2
    torch.manual_seed(seed + 1)
    a2c = A2C(env_name="HalfCheetah-v2", gamma=0.99, critic_lr=3e-4, use_gpu=False)
    load(a2c.critic, seed * 100 + 1)
    c0 = flat_params(a2c.critic)
    N = 300
    obs, nobs, rew, done = onp_batch(rng, N, ob)
    buf = Memory()
    prev = buf.add_obs(torch.from_numpy(obs[:1]))
    for i in range(N):  # one transition per rollout: obs_i -> next_obs_i
        if i:
            buf.new_rollout()
            prev = buf.add_obs(torch.from_numpy(obs[i:i + 1]))
        nxt = buf.add_obs(torch.from_numpy(nobs[i:i + 1]))
        buf.add_timestep(prev, nxt, torch.zeros(1, ob), torch.zeros(1), float(rew[i]), bool(done[i]), True)
    buf.end_rollout()
    assert np.array_equal(buf.norm_obs.numpy(), obs) and np.array_equal(buf.norm_next_obs.numpy(), nobs)
    adv = a2c.update_critic(buf)
    out.update(crit_params0=c0, crit_obs=obs, crit_nobs=nobs, crit_rew=rew, crit_done=done,
               crit_loss=np.array(a2c.loss["critic"]), crit_adv=adv.numpy(), crit_post=flat_params(a2c.critic),
               crit_lr=np.array(3e-4), crit_gamma=np.array(0.99))
    # ---- PPO_AcM.update_actor_acm: one epoch, one minibatch of the whole buffer
    torch.manual_seed(seed + 2)
    ppo = PPO_AcM(env_name="HalfCheetah-v2", gamma=0.99, actor_lr=3e-4, critic_lr=3e-4, custom_loss=0.1,
                  norm_closs=True, min_max_denormalize=True, denormalize_actor_out=True, ppo_batch_size=N,
                  max_ppo_epochs=1, entropy_coef=0.01, acm_pre_train_samples=10, use_gpu=False)
    load(ppo.actor, seed * 100 + 2)
    p0 = flat_params(ppo.actor)
    mem = MemoryAcM(min_max_denormalize=True)
    acts = rng.uniform(-1.1, 1.1, (N, ob)).astype(np.float32)
    with torch.no_grad():
        lp_cur = ppo.actor.get_actions_dist(torch.from_numpy(obs)).log_prob(torch.from_numpy(acts)).numpy()
    lp_old = (lp_cur + 0.2 * rng.randn(N)).astype(np.float32)
    adv_in = (rng.randn(N) * 2 + 0.5).astype(np.float32)
    prev = mem.add_obs(torch.from_numpy(obs[:1]))
    for i in range(N):
        if i:
            mem.new_rollout()
            prev = mem.add_obs(torch.from_numpy(obs[i:i + 1]))
        nxt = mem.add_obs(torch.from_numpy(nobs[i:i + 1]))
        mem.add_timestep(prev, nxt, torch.from_numpy(acts[i:i + 1]), torch.from_numpy(lp_old[i:i + 1]),
                         float(rew[i]), bool(done[i]), True)
    mem.end_rollout()
    ppo.update_actor_acm(torch.from_numpy(adv_in), mem)
    out.update(ppo_params0=p0, ppo_acts=acts, ppo_lp_old=lp_old, ppo_adv=adv_in, ppo_post=flat_params(ppo.actor),
               ppo_losses=np.array([ppo.loss[k] for k in ("actor", "entropy", "policy", "dist")]),
               ppo_lr=np.array(3e-4), ppo_eps=np.array(ppo.ppo_epsilon), ppo_entropy_coef=np.array(0.01),
               ppo_custom_loss=np.array(0.1))
    save("onpolicy_hcheetah.npz", **out)


def gen_ppo_epochs(seed=71, lr=3e-3, ent=0.05, N=300):
    """PPO_AcM.update_actor_acm over several epochs with the KL early stop (acm/on_policy.py:164-216): one
    full-batch minibatch per epoch (so the DataLoader's shuffle only reorders a mean), and a
    kl_div_threshold placed between the KLs of the 3rd and 4th epochs, read from utils.kl_divergence in a
    first run without the stop: epochs 0..3 run, the check at i = 4 breaks the loop, the losses are divided
    by i + 1 = 5 (one more than the epochs run) and kl_div_updates_counter grows by 5."""
    from rltoolkit import utils
    from rltoolkit.acm import on_policy as onp_mod

    ob = 17
    rng = np.random.RandomState(seed)
    obs, nobs, rew, done = onp_batch(rng, N, ob)
    acts = rng.uniform(-1.1, 1.1, (N, ob)).astype(np.float32)
    adv_in = (rng.randn(N) * 2 + 0.5).astype(np.float32)
    noise = (0.2 * rng.randn(N)).astype(np.float32)

    def run(thr, max_epochs):
        torch.manual_seed(seed + 2)
        ppo = PPO_AcM(env_name="HalfCheetah-v2", gamma=0.99, actor_lr=lr, critic_lr=3e-4, custom_loss=0.1,
                      norm_closs=True, min_max_denormalize=True, denormalize_actor_out=True, ppo_batch_size=N,
                      max_ppo_epochs=max_epochs, entropy_coef=ent, kl_div_threshold=thr, acm_pre_train_samples=10,
                      use_gpu=False)
        load(ppo.actor, seed * 100 + 2)
        p0 = flat_params(ppo.actor)
        with torch.no_grad():
            lp_cur = ppo.actor.get_actions_dist(torch.from_numpy(obs)).log_prob(torch.from_numpy(acts)).numpy()
        lp_old = (lp_cur + noise).astype(np.float32)
        mem = MemoryAcM(min_max_denormalize=True)
        prev = mem.add_obs(torch.from_numpy(obs[:1]))
        for i in range(N):
            if i:
                mem.new_rollout()
                prev = mem.add_obs(torch.from_numpy(obs[i:i + 1]))
            nxt = mem.add_obs(torch.from_numpy(nobs[i:i + 1]))
            mem.add_timestep(prev, nxt, torch.from_numpy(acts[i:i + 1]), torch.from_numpy(lp_old[i:i + 1]),
                             float(rew[i]), bool(done[i]), True)
        mem.end_rollout()
        kls = []
        real = utils.kl_divergence

        def rec(log_p, log_q):
            v = real(log_p, log_q)
            kls.append(v)
            return v

        onp_mod.utils.kl_divergence = rec
        try:
            ppo.update_actor_acm(torch.from_numpy(adv_in), mem)
        finally:
            onp_mod.utils.kl_divergence = real
        return ppo, kls, p0, lp_old

    _, kls, _, _ = run(1e9, 6)
    assert max(kls[:3]) + 2e-3 < kls[3], kls  # a crossing with margin on both sides
    thr = 0.5 * (max(kls[:3]) + kls[3])
    ppo, kls2, p0, lp_old = run(thr, 10)
    assert len(kls2) == 4 and ppo.kl_div_updates_counter == 5, (kls2, ppo.kl_div_updates_counter)
    print("ppo epochs: kl per epoch", [round(k, 5) for k in kls], "threshold", round(thr, 5))
    save("ppo_epochs_hcheetah.npz", params0=p0, obs=obs, nobs=nobs, acts=acts, lp_old=lp_old, adv=adv_in,
         post=flat_params(ppo.actor), losses=np.array([ppo.loss[k] for k in ("actor", "entropy", "policy", "dist")]),
         kls=np.array(kls2), counter=np.array(ppo.kl_div_updates_counter), threshold=np.array(thr),
         lr=np.array(lr), eps=np.array(ppo.ppo_epsilon), entropy_coef=np.array(ent), custom_loss=np.array(0.1),
         max_epochs=np.array(10))


# ---------------------------------------------------------------- normalizer KATs + reference checkpoint
def gen_interop(seed=61):
    """(1) MemoryMeta.normalize / denormalize (memory.py:76-127) and utils.standardize_and_clip /
    revert_standardization (utils.py:62-83) on the reference's own KAT inputs (buffer/test/test_memory.py:
    84-96 test_normalize, test/test_utils.py:9-43) and on a random batch in both modes; (2) a checkpoint
    written by the reference's own RL.save (rl.py:281-290; sac.py:287-296 + the ACM, ddpg_acm.py:87-90) from a
    SAC_AcM Hopper with random weights and normaliser, and the reference's deterministic test action on a
    batch of obs (ddpg.py:385-410: normalize -> noise_action(act_noise=0, deterministic=True) ->
    process_action)."""
    from rltoolkit import utils

    out = {}
    rng = np.random.RandomState(seed)
    # (1a) test_memory.py::test_normalize (z-score, clip 10)
    mem = Memory()
    mem.obs_std = torch.tensor([2.0, 20.0])
    mem.obs_mean = torch.tensor([2.5, 25.0])
    ex = torch.tensor([[i, 10 * i] for i in range(6)]).float()
    out["kat_mem_x"] = ex.numpy()
    out["kat_mem_y"] = mem.normalize(ex).numpy()
    ex2 = ex.clone()
    ex2[0, 0] = 1000
    out["kat_mem_x2"] = ex2.numpy()
    out["kat_mem_y2"] = mem.normalize(ex2).numpy()
    out["kat_mem_mean"], out["kat_mem_std"] = mem.obs_mean.numpy(), mem.obs_std.numpy()
    # (1b) test_utils.py fixture: obs = arange(20).reshape(4, 5).T, torch mean / std(ddof=1)
    obs = torch.tensor(np.arange(20).reshape(4, 5).T).float()
    mean, std = obs.mean(axis=0), obs.std(axis=0)
    st = utils.standardize_and_clip(obs, mean, std)
    out.update(kat_utl_x=obs.numpy(), kat_utl_mean=mean.numpy(), kat_utl_std=std.numpy(), kat_utl_stand=st.numpy(),
               kat_utl_revert=utils.revert_standardization(st, mean, std).numpy())
    # (1c) random batch, both modes, normalize and denormalize
    ob = 11
    x = (rng.randn(257, ob) * 3).astype(np.float32)
    x[0, :3] = [1e6, -1e6, 0.0]  # clipped in z-score mode
    lo = -rng.uniform(0.5, 2, ob).astype(np.float32)
    hi = rng.uniform(0.5, 2, ob).astype(np.float32)
    mu = rng.randn(ob).astype(np.float32)
    sd = rng.uniform(0.1, 3, ob).astype(np.float32)
    for mm in (True, False):
        m2 = Memory(min_max_denormalize=mm)
        m2.min_obs, m2.max_obs = torch.from_numpy(lo), torch.from_numpy(hi)
        m2.obs_mean, m2.obs_std = torch.from_numpy(mu), torch.from_numpy(sd)
        tag = "mm" if mm else "z"
        out["rnd_%s_norm" % tag] = m2.normalize(torch.from_numpy(x)).numpy()
        out["rnd_%s_denorm" % tag] = m2.denormalize(torch.from_numpy(x)).numpy()
    out.update(rnd_x=x, rnd_lo=lo, rnd_hi=hi, rnd_mean=mu, rnd_std=sd)
    # (2) reference-written checkpoint + the reference's deterministic test action
    torch.manual_seed(seed)
    ag = SAC_AcM(env_name="Hopper-v2", acm_critic=True, custom_loss=0.2, min_max_denormalize=True,
                 denormalize_actor_out=True, buffer_size=100)
    for net in (ag.actor, ag.critic_1, ag.critic_2, ag.acm):
        load(net, int(rng.randint(1 << 30)))
    rb = ag.replay_buffer
    rb.min_obs = torch.from_numpy(-rng.uniform(0.5, 2, ob).astype(np.float32))
    rb.max_obs = torch.from_numpy(rng.uniform(0.5, 2, ob).astype(np.float32))
    rb.obs_mean = torch.from_numpy(rng.randn(ob).astype(np.float32))
    rb.obs_std = torch.from_numpy(rng.uniform(0.5, 2, ob).astype(np.float32))
    path = os.path.join(HERE, "ref_sac_acm_hopper.pkl")
    ag.save(path)
    print("wrote", path)
    obs_raw = (rng.randn(64, ob) * 1.5).astype(np.float32)
    tgts, envs = [], []
    with torch.no_grad():
        for i in range(len(obs_raw)):
            o = ag.replay_buffer.normalize(torch.from_numpy(obs_raw[i:i + 1]))
            a = ag.noise_action(o, act_noise=0, deterministic=True)
            tgts.append(a.numpy()[0])
            envs.append(ag.process_action(a, o))
    out.update(ckpt_obs=obs_raw, ckpt_target=np.array(tgts, np.float32), ckpt_env_action=np.array(envs, np.float32),
               ckpt_obs_norm=np.array([int(rb.obs_norm)]))
    save("ref_interop.npz", **out)


# ---------------------------------------------------------------- DDPG_AcM.make_update, unbiased_update=True
def unbiased_ring(buf, rng, ob, aout, ac):
    """The unbiased-update fixtures' ring: z-score statistics, then 9 ragged episodes (no wrap) written through
    the reference buffer's add_obs / add_acm_action / add_timestep; returns the logged writes."""
    buf.obs_mean = torch.from_numpy((rng.randn(ob) * 0.3).astype(np.float32))
    buf.obs_std = torch.from_numpy(rng.uniform(0.5, 1.5, ob).astype(np.float32))
    ops, obs_log, act_log, acm_log, rew_log, done_log, end_log = [], [], [], [], [], [], []
    for L in rng.randint(5, 40, 9):  # ragged episodes, no wrap (size 400)
        o = (rng.randn(1, ob) * 1.4).astype(np.float32)
        prev = buf.add_obs(torch.from_numpy(o))
        obs_log.append(o[0])
        ops.append((0, prev, -1))
        for t in range(L):
            acm = rng.uniform(-1, 1, ac).astype(np.float32)
            buf.add_acm_action(acm)
            a = torch.from_numpy(rng.uniform(-1.2, 1.2, (1, aout)).astype(np.float32))
            o = (rng.randn(1, ob) * 1.4).astype(np.float32)
            nxt = buf.add_obs(torch.from_numpy(o))
            r = float(rng.randn())
            end = t == L - 1
            done = bool(end and rng.rand() < 0.5)
            buf.add_timestep(prev, nxt, a, r, done, end)
            ops.append((1, prev, nxt))
            obs_log.append(o[0])
            act_log.append(a.numpy()[0])
            acm_log.append(acm)
            rew_log.append(r)
            done_log.append(done)
            end_log.append(end)
            prev = nxt
    return dict(norm=np.stack([buf.obs_mean.numpy(), buf.obs_std.numpy()]), ops=np.array(ops, np.int64),
                obs=np.array(obs_log, np.float32), act=np.array(act_log, np.float32), acm=np.array(acm_log, np.float32),
                rew=np.array(rew_log, np.float32), done=np.array(done_log, np.bool_), end=np.array(end_log, np.bool_))


def gen_ddpg_unbiased(seed=81):
    """DDPG_AcM(unbiased_update=True).make_update (acm/off_policy/ddpg_acm.py:59-85) over two update
    cadences: each samples grad_steps batches from the ring (np.random.randint after np.random.seed) and
    updates with action = next_obs (normalised: obs_norm=True, z-score).  acm_critic=False, so the critic
    takes (obs, action) and the unbiased branch changes what it learns; custom_loss with norm_closs."""
    torch.manual_seed(0)
    env, size, B, gsteps, ufreq = "HalfCheetah-v2", 400, 40, 2, 10
    m = DDPG_AcM(env_name=env, unbiased_update=True, gamma=0.97, actor_lr=5e-4, critic_lr=5e-4, buffer_size=size,
                 acm_pre_train_samples=10, acm_val_buffer_size=None, update_batch_size=B, grad_steps=gsteps,
                 update_freq=ufreq, custom_loss=0.3, norm_closs=True, acm_critic=False, min_max_denormalize=False,
                 denormalize_actor_out=True, obs_norm=True, use_gpu=False)
    ob, aout, ac = m.ob_dim, m.actor_output_dim, m.ac_dim
    nets = {"actor": m._actor, "critic": m._critic, "actor_targ": m.actor_targ, "critic_targ": m.critic_targ}
    for i, (k, mod) in enumerate(nets.items()):
        load(mod, seed * 100 + i)
    rng = np.random.RandomState(seed)
    buf = m.replay_buffer
    out = dict(dims=np.array([ob, aout, ac, B, gsteps, ufreq, size]), seed=np.array(seed),
               actor_ac_lim=m.actor_ac_lim.numpy().astype(np.float32), tau=np.array(m.tau), gamma=np.array(m.gamma))
    out.update(unbiased_ring(buf, rng, ob, aout, ac))
    m.iteration = 0  # no ACM update in these cadences (ddpg_acm.py:52-57)
    losses, idxs, np_seeds = [], [], [101, 202]
    for c, s in enumerate(np_seeds):
        m.stats_logger.frames = ufreq * (c + 1)
        assert m.update_condition()
        np.random.seed(s)
        idxs.append(np.stack([np.random.randint(0, len(buf), B) for _ in range(gsteps)]))
        np.random.seed(s)
        m.make_update()
        losses.append([m.loss.get(k, 0.0) for k in ("critic", "actor", "ddpg", "dist")])
    out.update(np_seeds=np.array(np_seeds), idx=np.stack(idxs), losses=np.array(losses))
    for k, mod in nets.items():
        out["post_" + k] = flat_params(mod)
    save("ddpg_unbiased_hcheetah.npz", **out)


# ---------------------------------------------------------------- SAC_AcM.make_update, unbiased_update=True
def gen_sac_unbiased(seed=91):
    """SAC_AcM(unbiased_update=True).make_update -- DDPG_AcM.make_update inherited (acm/off_policy/ddpg_acm.py:
    59-85; SAC_AcM(DDPG_AcM), sac_acm.py:12) -- over two update cadences on the unbiased ring: each samples
    grad_steps batches (np.random.randint after np.random.seed) and updates with action = next_obs (normalised:
    obs_norm=True, z-score).  acm_critic=False (the critics take (obs, action)), custom_loss with norm_closs; the
    rsample draws of every update (two per update, in call order) are injected and stored."""
    torch.manual_seed(0)
    env, size, B, gsteps, ufreq = "HalfCheetah-v2", 400, 40, 2, 10
    m = SAC_AcM(env_name=env, unbiased_update=True, gamma=0.97, actor_lr=1e-3, critic_lr=1e-3, alpha_lr=1e-3,
                alpha=0.2, buffer_size=size, acm_pre_train_samples=10, acm_val_buffer_size=None, update_batch_size=B,
                grad_steps=gsteps, update_freq=ufreq, custom_loss=0.3, norm_closs=True, acm_critic=False,
                min_max_denormalize=False, denormalize_actor_out=True, obs_norm=True, use_gpu=False)
    assert m.unbiased_update
    ob, aout, ac = m.ob_dim, m.actor_output_dim, m.ac_dim
    nets = {"actor": m._actor, "critic_1": m._critic_1, "critic_2": m._critic_2,
            "critic_1_targ": m.critic_1_targ, "critic_2_targ": m.critic_2_targ}
    for i, (k, mod) in enumerate(nets.items()):
        load(mod, seed * 100 + i)
    rng = np.random.RandomState(seed)
    buf = m.replay_buffer
    out = dict(dims=np.array([ob, aout, ac, B, gsteps, ufreq, size]), seed=np.array(seed),
               actor_ac_lim=m.actor_ac_lim.numpy().astype(np.float32), tau=np.array(m.tau), gamma=np.array(m.gamma),
               alpha0=np.array(m.alpha), target_entropy=np.array(m.target_entropy))
    out.update(unbiased_ring(buf, rng, ob, aout, ac))
    m.iteration = 0  # no ACM update in these cadences (ddpg_acm.py:52-57)
    losses, idxs, eps, np_seeds = [], [], [], [201, 302]
    for c, s in enumerate(np_seeds):
        m.stats_logger.frames = ufreq * (c + 1)
        assert m.update_condition()
        np.random.seed(s)
        idxs.append(np.stack([np.random.randint(0, len(buf), B) for _ in range(gsteps)]))
        e = [rng.randn(B, aout).astype(np.float32) for _ in range(2 * gsteps)]
        eps.append(np.stack(e))
        EPS.q = list(e)
        np.random.seed(s)
        m.make_update()
        assert not EPS.q
        losses.append([m.loss.get(k, 0.0) for k in ("critic_1", "critic_2", "actor", "sac", "dist")])
    out.update(np_seeds=np.array(np_seeds), idx=np.stack(idxs), eps=np.stack(eps), losses=np.array(losses),
               log_alpha=np.array(float(m.log_alpha)), alpha=np.array(m.alpha))
    for k, mod in nets.items():
        out["post_" + k] = flat_params(mod)
    save("sac_unbiased_hcheetah.npz", **out)


GROUPS = {"interop": gen_interop, "randint": gen_randint, "replay": gen_replay, "ddpg": gen_ddpg, "acm": gen_acm, "ppo": gen_ppo,
          "sac_vanilla": gen_sac_vanilla, "onpolicy": gen_onpolicy, "ppo_epochs": gen_ppo_epochs,
          "ddpg_unbiased": gen_ddpg_unbiased, "sac_unbiased": gen_sac_unbiased,
          "sac_vanilla_obsnorm": gen_sac_vanilla_obsnorm}

if __name__ == "__main__":
    which = sys.argv[1:] or list(GROUPS) + ["sac"]
    for g in which:
        if g == "sac":
            for i, (name, (env, B, flags, steps, adam)) in enumerate(SAC_VARIANTS.items()):
                gen_sac(name, env, B, flags, steps, adam, seed=1 + i)
        else:
            GROUPS[g]()
