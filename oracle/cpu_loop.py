"""ORACLE (test infrastructure only; bench.py's cpu_baseline leg): the reference's per-frame
off-policy training loop, restated on the CPU with the oracle networks, to time the
reference's own N_CORES CPU path on the GPU box (where /root/reference does not exist).

One process = one single-threaded run (torch.set_num_threads(1), evals.py:22-26); the
reference runs N_CORES of them in a multiprocessing pool (train/spp_*.py).  Per frame it
does what DDPG.collect_batch_and_train (rltoolkit/algorithms/ddpg/ddpg.py:182-223) does:
  process_obs (torch tensor of the env obs)                 ddpg.py:358-369
  replay_buffer.normalize (identity unless obs_norm)        replay_buffer.py:77-81
  initial_act / noise_action (actor sample + act_noise, clip through numpy, denormalise)
                                                            ddpg_acm.py:40-50, off_policy.py:50-54, ddpg.py:171-180
  process_action (ACM forward, add_acm_action)              off_policy.py:89-106
  env.step (SURVEY Appendix A SynthEnv, numpy)
  add_obs / add_timestep (fp64 numpy ring)                  replay_buffer.py:56-75,133-137
  make_update: every update_freq frames, grad_steps x (sample_batch -> update)
                                                            ddpg.py:225-237, ddpg_acm.py:52-85
  ACM: every acm_update_freq frames, acm_update_batches x (sample_acm_batch -> batch_update)
                                                            acm.py:356-372
  per iteration (batch_size frames): update_obs_mean_std    ddpg.py:159-170, replay_buffer.py:83-96
The update itself is the oracle restatement (oracle/sac_acm.py, ddpg_acm.py, sac.py,
acm.py); the buffer is oracle/replay.py.  Gaussian draws come from numpy (the reference
uses torch's generator: same distribution, different stream).
"""
import time

import numpy as np
import torch
import torch.nn.functional as F

from . import nets
from .nets import Norm
from .replay import OracleReplay


class _NpMT:
    """np.random.randint on numpy's global-style legacy stream (replay_buffer.py:234)."""

    def __init__(self, seed):
        self.rs = np.random.RandomState(seed)

    def randint(self, high, n):
        return self.rs.randint(0, high, n)


class SynthEnv:
    """s' = tanh(A s) + 0.1 resize(a, ob), r = -|a|^2 + s'[0], T frames."""

    def __init__(self, ob, ac, T=1000, seed=0):
        self.rng = np.random.RandomState(seed)
        self.A = (self.rng.randn(ob, ob) * 0.05).astype(np.float32)
        self.ob, self.ac, self.T = ob, ac, T

    def reset(self):
        self.t = 0
        self.s = self.rng.randn(self.ob).astype(np.float32)
        return self.s.copy()

    def step(self, a):
        a = np.asarray(a, np.float32).reshape(-1)
        self.t += 1
        self.s = (np.tanh(self.A @ self.s) + 0.1 * np.resize(a, self.s.shape)).astype(np.float32)
        return self.s.copy(), float(-np.square(a).sum() + self.s[0]), self.t >= self.T, {}

    def sample(self):
        return self.rng.uniform(-1, 1, self.ac).astype(np.float32)


class _TorchAdam:
    """The reference's optimizer object, torch.optim.Adam (rl.py:62, ddpg.py:132-135, sac.py:107-110,
    acm.py:176-183; its single-tensor CPU path), stepping .grad: the baseline pays the reference's per-step
    optimizer host work.  The oracle's OracleAdam restates the same arithmetic for the parity tests but runs
    ~2.2 ms per SAC_AcM grad step faster (B = 100, one thread: reference update 12.96 ms, the port with
    OracleAdam 10.31 ms, with torch.optim.Adam 12.55 ms, tools/cpu_calibrate.py, profiles/r05/cpu_calibrate.txt)."""

    def __init__(self, params, lr):
        self.params = list(params)
        self.o = torch.optim.Adam(self.params, lr=lr)

    def step(self, grads):
        for p, g in zip(self.params, grads):
            p.grad = g
        self.o.step()
        self.o.zero_grad(set_to_none=True)


def _torch_adam(agent):
    """Swap the oracle's OracleAdam objects for _TorchAdam (same lr)."""
    if isinstance(getattr(agent, "opt", None), dict):
        for k, o in agent.opt.items():
            agent.opt[k] = _TorchAdam(o.params, o.lr)
    elif getattr(agent, "opt", None) is not None:
        agent.opt = _TorchAdam(agent.opt.params, agent.opt.lr)
    if getattr(agent, "opt_alpha", None) is not None:
        agent.opt_alpha = _TorchAdam(agent.opt_alpha.params, agent.opt_alpha.lr)


def _fill(layout, seed):
    from tests.golden.weights import fill_params

    return fill_params(layout, seed)


class CpuLoop:
    """algo: 'sac_acm' | 'ddpg_acm' | 'sac' (vanilla).  Hyper-parameters are the train/*.py ones."""

    def __init__(self, algo, ob, ac, *, update_batch_size=100, update_freq=50, grad_steps=50, acm_update_freq=1000,
                 acm_update_batches=100, acm_batch_size=100, batch_size=1000, buffer_size=1_000_000, prefill=0,
                 act_noise=None, seed=0):
        torch.set_num_threads(1)
        self.algo, self.ob, self.ac = algo, ob, ac
        self.B, self.update_freq, self.grad_steps = update_batch_size, update_freq, grad_steps
        self.acm_update_freq, self.acm_batches, self.acm_bs = acm_update_freq, acm_update_batches, acm_batch_size
        self.batch_size = batch_size
        self.rng = np.random.RandomState(seed)
        self.mt = _NpMT(seed)
        self.env = SynthEnv(ob, ac, seed=seed)
        vanilla = algo == "sac"
        aout = ac if vanilla else ob
        self.aout = aout
        self.rb = OracleReplay(buffer_size, ob, aout, ac)
        lo, hi = np.full(ob, -2.0, np.float32), np.full(ob, 2.0, np.float32)
        self.norm = Norm(True, torch.from_numpy(lo), torch.from_numpy(hi))
        if algo == "sac_acm":
            from .acm import OracleAcmTrainer
            from .sac_acm import OracleSacAcm

            lay = {"actor": nets.sac_actor_layout(ob, ob), "critic_1": nets.critic_layout(ob + ac),
                   "critic_2": nets.critic_layout(ob + ac), "critic_1_targ": nets.critic_layout(ob + ac),
                   "critic_2_targ": nets.critic_layout(ob + ac), "acm": nets.acm_layout(2 * ob, ac)}
            params = {k: _fill(v, i) for i, (k, v) in enumerate(lay.items())}
            self.agent = OracleSacAcm(ob, ob, ac, acm_critic=True, custom_loss=0.2, norm=self.norm,
                                      acm_lim=np.ones(ac, np.float32), gamma=0.99, params=params)
            self.acm = OracleAcmTrainer(2 * ob, ac, lr=1e-3, params=params["acm"])
            self.act_noise = 0.1 if act_noise is None else act_noise
        elif algo == "ddpg_acm":
            from .ddpg_acm import OracleDdpgAcm

            lay = {"actor": nets.ddpg_actor_layout(ob, ob), "critic": nets.critic_layout(ob + ac),
                   "actor_targ": nets.ddpg_actor_layout(ob, ob), "critic_targ": nets.critic_layout(ob + ac),
                   "acm": nets.basic_acm_layout(2 * ob, ac)}
            params = {k: _fill(v, i) for i, (k, v) in enumerate(lay.items())}
            self.agent = OracleDdpgAcm(ob, ob, ac, acm_critic=True, custom_loss=1.0, norm=self.norm, gamma=0.95,
                                       params=params)
            self.acm_p = {n: torch.as_tensor(v).clone().requires_grad_(True) for n, v in params["acm"].items()}
            self.acm_opt = torch.optim.Adam(self.acm_p.values(), lr=0.005)
            self.act_noise = 0.05 if act_noise is None else act_noise
        elif algo == "sac":
            from .sac import OracleSac

            lay = {"actor": nets.sac_actor_layout(ob, ac), "critic_1": nets.critic_layout(ob + ac),
                   "critic_2": nets.critic_layout(ob + ac), "critic_1_targ": nets.critic_layout(ob + ac),
                   "critic_2_targ": nets.critic_layout(ob + ac)}
            params = {k: _fill(v, i) for i, (k, v) in enumerate(lay.items())}
            self.agent = OracleSac(ob, ac, params=params)
            self.act_noise = 0.1  # Q1
            self.acm_batches = 0
        else:
            raise ValueError(algo)
        _torch_adam(self.agent)
        if getattr(self, "acm", None) is not None:
            _torch_adam(self.acm)
        self.frames = 0
        if prefill:
            self._prefill(prefill)

    def _prefill(self, n):
        """Replay rows as left by earlier training (N(0,1) obs), so sampling and the obs
        statistics run at the bench's buffer fill."""
        rb = self.rb
        o = self.rng.randn(n + 1, self.ob)
        rb._obs[:n + 1] = o
        rb._obs_idx[:n] = np.arange(n)
        rb._next_obs_idx[:n] = np.arange(1, n + 1)
        rb._actions[:n] = self.rng.randn(n, self.aout)
        rb._actions_acm[:n] = self.rng.uniform(-1, 1, (n, self.ac))
        rb._rewards[:n] = self.rng.randn(n)
        rb.obs_idx, rb.ts_idx, rb.current_len = n + 1, n, n

    # ------------------------------------------------------------------ per-frame pieces
    def _act(self, obs_t):
        P = self.agent.p
        lim = torch.ones(self.aout)
        with torch.no_grad():
            if self.algo == "ddpg_acm":
                a = nets.ddpg_actor(P["actor"], obs_t, lim)
            else:
                a, _, _ = nets.sac_actor(P["actor"], obs_t, lim, torch.randn(1, self.aout))
            if self.algo == "sac":  # DDPG.noise_action: + act_noise N(0,1), clip to the env limit
                a = a + self.act_noise * torch.randn(self.aout)
                return np.clip(a.cpu(), -1.0, 1.0), None
            a = a + self.act_noise * torch.randn(self.aout) * lim  # DDPG_AcM.noise_action
            a = torch.as_tensor(np.clip(a.cpu(), -1.1, 1.1))
            a = self.norm.denormalize(a)
            x = torch.cat([obs_t, a], 1)
            if self.algo == "ddpg_acm":
                c = nets.basic_acm(self.acm_p, x)
            else:
                c = nets.acm(P["acm"], x, torch.ones(self.ac))
            return a, c.cpu().numpy()[0]

    def _update(self):
        batch, _ = self.rb.sample_batch(self.B, self.mt)
        tens = [torch.as_tensor(b) for b in batch]  # sample_batch -> torch tensors (replay_buffer.py:248-260)
        if self.algo == "sac":
            self.agent.update(*tens[:5], self.rng.randn(self.B, self.aout).astype(np.float32),
                              self.rng.randn(self.B, self.aout).astype(np.float32))
        elif self.algo == "sac_acm":
            self.agent.update(*tens, self.rng.randn(self.B, self.aout).astype(np.float32),
                              self.rng.randn(self.B, self.aout).astype(np.float32))
        else:
            self.agent.update(*tens)

    def _acm_step(self):
        (o, no, acm), _ = self.rb.sample_acm_batch(self.acm_bs, self.mt)
        x = torch.cat([torch.as_tensor(o), torch.as_tensor(no)], 1)
        y = torch.as_tensor(acm)
        if self.algo == "ddpg_acm":
            loss = F.mse_loss(nets.basic_acm(self.acm_p, x), y)
            self.acm_opt.zero_grad()
            loss.backward()
            self.acm_opt.step()
        else:
            self.acm.batch_update(x, y)

    def _obs_stats(self):
        x = self.rb._obs[self.rb._obs_idx[:len(self.rb)]]  # MetaReplayBuffer.obs (gathered, fp64)
        x.mean(axis=0), x.std(axis=0), np.percentile(x, 99, axis=0), np.percentile(x, 1, axis=0)

    def run(self, seconds):
        """Frames per second of the reference loop over at least ``seconds`` of wall time."""
        rb = self.rb
        obs = self.env.reset()
        prev = rb.add_obs(obs)
        n = 0
        t0 = time.perf_counter()
        while True:
            obs_t = torch.tensor(obs, dtype=torch.float32).unsqueeze(0)  # process_obs
            a, c = self._act(obs_t)
            if c is not None:
                rb.add_acm_action(c)
                env_a = c
            else:
                env_a = a.numpy()[0]
            obs, r, end, _ = self.env.step(env_a)
            done = False if (self.algo == "sac" and self.env.t == self.env.T) else end  # Q3
            nxt = rb.add_obs(torch.tensor(obs, dtype=torch.float32).unsqueeze(0).numpy())
            rb.add_timestep(prev, nxt, np.asarray(a).reshape(-1), r, done, end)
            prev = nxt
            self.frames += 1
            n += 1
            if len(rb) > self.B and self.frames % self.update_freq == 0:
                for _ in range(self.grad_steps):
                    self._update()
            if self.acm_batches and self.frames % self.acm_update_freq == 0:
                for _ in range(self.acm_batches):
                    self._acm_step()
            if self.frames % self.batch_size == 0:
                self._obs_stats()
            if end:
                obs = self.env.reset()
                prev = rb.add_obs(obs)
            el = time.perf_counter() - t0
            if el >= seconds and self.frames % self.update_freq == 0:
                return n / el, n, el
