"""ORACLE (test infrastructure only; bench.py's cpu_baseline leg for ppo_hcheetah): the reference's
PPO_AcM training iteration, restated on the CPU with the oracle networks, to time the reference's
N_CORES CPU path (train/spp_ppo_hcheetah.py: one 1-thread process per hyper-parameter run) on the GPU
box, where /root/reference does not exist.

One iteration (AcMOnPolicyTrainer.perform_iteration, rltoolkit/acm/on_policy.py:52-79):
  collect_batch        batch_size frames of single-env episodes (a2c.py:141-181): normalize obs,
                       Actor.act (basic_model.py:32-51), process_action = denormalize + AcM act
                       (on_policy.py:31-50), env.step, Memory adds
  update_critic        critic_num_target_updates x num_critic_updates_per_target full-batch steps
                       of 0.5 mean((q - V)^2) with Adam (a2c.py:186-225)
  calculate_gae        the per-sample reverse loop (ppo.py:117-150)
  update_actor_acm     <= max_ppo_epochs shuffled epochs of ppo_batch_size minibatches: clip loss +
                       custom_loss * mse(actions, next_obs), Adam; KL stop (on_policy.py:164-216)
  replay add_buffer    the ACM ring (fp64 numpy, oracle/replay.py)
  update_acm           every acm_update_freq iterations: acm_epochs shuffled epochs over the ring in
                       acm_batch_size batches (acm.py:266-303)
  update_obs_mean_std  on the ring (replay_buffer.py:83-96)
Networks: oracle/onpolicy.py (Actor / Critic, 64 hidden) and oracle/nets.py (AcM); the
optimisers are torch.optim.Adam on the same tensors, as the reference's nn.Modules use them.
"""
import time

import numpy as np
import torch
import torch.nn.functional as F

from . import nets, onpolicy
from .cpu_loop import SynthEnv
from .nets import Norm
from .replay import OracleReplay


def _tensors(flat, layout):
    out, o = {}, 0
    for n, shape in layout:
        k = int(np.prod(shape))
        out[n] = torch.as_tensor(flat[o:o + k].reshape(shape)).clone().requires_grad_(True)
        o += k
    return out


class PpoCpuLoop:
    """train/spp_ppo_hcheetah.py hyper-parameters (HalfCheetah dims: ob 17, ac 6)."""

    def __init__(self, ob=17, ac=6, *, batch_size=2000, gamma=0.99, lr=3e-4, ppo_batch_size=512, max_ppo_epochs=10,
                 kl_div_threshold=0.1, custom_loss=0.1, critic_target_updates=10, critic_updates_per_target=10,
                 acm_epochs=5, acm_batch_size=64, acm_update_freq=3, acm_lr=3e-4, ring=110_000, prefill=100_000,
                 ep_len=1000, seed=0):
        torch.set_num_threads(1)
        self.ob, self.ac, self.aout = ob, ac, ob
        self.batch_size, self.gamma = batch_size, gamma
        self.ppo_bs, self.max_epochs, self.kl_thr, self.custom_loss = ppo_batch_size, max_ppo_epochs, kl_div_threshold, custom_loss
        self.c_targets, self.c_updates = critic_target_updates, critic_updates_per_target
        self.acm_epochs, self.acm_bs, self.acm_freq = acm_epochs, acm_batch_size, acm_update_freq
        self.rng = np.random.RandomState(seed)
        self.env = SynthEnv(ob, ac, T=ep_len, seed=seed)
        self.actor = _tensors(onpolicy.init_flat(onpolicy.actor_layout(ob, ob), seed), onpolicy.actor_layout(ob, ob))
        self.critic = _tensors(onpolicy.init_flat(onpolicy.critic_layout(ob), seed + 1), onpolicy.critic_layout(ob))
        acm_lay = nets.acm_layout(2 * ob, ac)
        self.acm = _tensors(onpolicy.init_flat(acm_lay, seed + 2), acm_lay)
        self.a_opt = torch.optim.Adam(self.actor.values(), lr=lr)
        self.c_opt = torch.optim.Adam(self.critic.values(), lr=lr)
        self.m_opt = torch.optim.Adam(self.acm.values(), lr=acm_lr)
        self.lim = torch.ones(ob)
        self.acm_lim = torch.ones(ac)
        self.rb = OracleReplay(ring, ob, ob, ac)
        rb = self.rb
        rb._obs[:prefill + 1] = self.rng.randn(prefill + 1, ob)  # the ring after ACM pre-training
        rb._obs_idx[:prefill] = np.arange(prefill)
        rb._next_obs_idx[:prefill] = np.arange(1, prefill + 1)
        rb._actions_acm[:prefill] = self.rng.uniform(-1, 1, (prefill, ac))
        rb.obs_idx, rb.ts_idx, rb.current_len = prefill + 1, prefill, prefill
        self.mean, self.std = np.zeros(ob, np.float32), np.ones(ob, np.float32)
        self.norm = Norm(True, torch.full((ob,), -2.0), torch.full((ob,), 2.0))
        self.iteration = 1

    # ------------------------------------------------------------------ collect_batch (a2c.py:141-181)
    def _collect(self):
        obs_l, nobs_l, act_l, lp_l, acm_l, rew_l, done_l, end_l = [], [], [], [], [], [], [], []
        while len(rew_l) < self.batch_size:
            obs = self.env.reset()
            end = False
            while not end:
                x = torch.as_tensor((obs - self.mean) / self.std, dtype=torch.float32).unsqueeze(0)
                with torch.no_grad():
                    dist = onpolicy.actor_dist(self.actor, x, self.lim)
                    a = dist.sample()
                    lp = dist.log_prob(a)
                    ad = self.norm.denormalize(a)
                    c = nets.acm(self.acm, torch.cat([x, ad], 1), self.acm_lim)
                nobs, r, end, _ = self.env.step(c.numpy()[0])
                obs_l.append(x[0])
                act_l.append(a[0])
                lp_l.append(lp[0])
                acm_l.append(c[0].numpy())
                rew_l.append(r)
                done_l.append(float(end and self.env.t < self.env.T))
                end_l.append(end)
                nobs_l.append(torch.as_tensor((nobs - self.mean) / self.std, dtype=torch.float32))
                obs = nobs
        return (torch.stack(obs_l), torch.stack(nobs_l), torch.stack(act_l), torch.stack(lp_l), np.stack(acm_l),
                torch.tensor(rew_l, dtype=torch.float32), torch.tensor(done_l), np.array(end_l))

    # ------------------------------------------------------------------ update_critic (a2c.py:186-225)
    def _update_critic(self, obs, nobs, rew, done):
        for _ in range(self.c_targets):
            with torch.no_grad():
                q = rew + self.gamma * (1 - done) * onpolicy.critic(self.critic, nobs).squeeze(-1)
            for _ in range(self.c_updates):
                loss = 0.5 * (q - onpolicy.critic(self.critic, obs).squeeze(-1)).pow(2).mean()
                self.c_opt.zero_grad()
                loss.backward()
                self.c_opt.step()
        with torch.no_grad():
            v = onpolicy.critic(self.critic, obs).squeeze(-1)
            vn = onpolicy.critic(self.critic, nobs).squeeze(-1)
        return v, vn

    # ------------------------------------------------------------------ calculate_gae (ppo.py:117-150)
    def _gae(self, rew, v, vn, done, end, lam=0.95):
        deltas = rew + self.gamma * (1 - done) * vn - v
        adv = torch.zeros_like(rew)
        gae = 0.0
        disc = self.gamma * lam
        for i in range(len(deltas) - 1, -1, -1):
            if done[i]:
                gae = 0.0
            elif end[i]:
                gae = vn[i].item()
            gae = gae * disc + deltas[i].item()
            adv[i] = gae
        return adv

    # ------------------------------------------------------------------ update_actor_acm (on_policy.py:164-216)
    def _update_actor(self, adv, obs, nobs, act, lp_old):
        adv = (adv - adv.mean()) / (adv.std() + 1e-8)
        n = len(adv)
        kl = 0.0
        for _ in range(self.max_epochs):
            if kl >= self.kl_thr:
                break
            perm = torch.from_numpy(self.rng.permutation(n))
            for s in range(0, n, self.ppo_bs):
                i = perm[s:s + self.ppo_bs]
                dist = onpolicy.actor_dist(self.actor, obs[i], self.lim)
                lp = dist.log_prob(act[i])
                ratio = torch.exp(lp - lp_old[i])
                A = adv[i]
                loss = -(torch.min(ratio * A, torch.clamp(ratio, 0.8, 1.2) * A)).mean()
                loss = loss + self.custom_loss * F.mse_loss(act[i], nobs[i])
                self.a_opt.zero_grad()
                loss.backward()
                self.a_opt.step()
            kl = (lp_old[i] - lp.detach()).mean().item()

    # ------------------------------------------------------------------ update_acm (acm.py:266-303)
    def _update_acm(self):
        rb = self.rb
        n = len(rb)
        o = torch.as_tensor(rb._obs[rb._obs_idx[:n]], dtype=torch.float32)
        no = torch.as_tensor(rb._obs[rb._next_obs_idx[:n]], dtype=torch.float32)
        x_all = torch.cat([o, no], 1)
        y_all = torch.as_tensor(rb._actions_acm[:n], dtype=torch.float32)
        for _ in range(self.acm_epochs):
            perm = torch.from_numpy(self.rng.permutation(n))
            for s in range(0, n, self.acm_bs):
                i = perm[s:s + self.acm_bs]
                loss = F.mse_loss(nets.acm(self.acm, x_all[i], self.acm_lim), y_all[i])
                self.m_opt.zero_grad()
                loss.backward()
                self.m_opt.step()

    def iterate(self):
        obs, nobs, act, lp, acm, rew, done, end = self._collect()
        v, vn = self._update_critic(obs, nobs, rew, done)
        adv = self._gae(rew, v, vn, done, end)
        self._update_actor(adv, obs, nobs, act, lp)
        rb = self.rb
        prev = rb.add_obs(obs[0].numpy())
        for t in range(len(rew)):  # ReplayBufferAcM.add_buffer
            rb.add_acm_action(acm[t])
            nxt = rb.add_obs(nobs[t].numpy())
            rb.add_timestep(prev, nxt, act[t].numpy(), float(rew[t]), bool(done[t]), bool(end[t]))
            prev = nxt
        if self.acm_freq and self.iteration % self.acm_freq == 0:
            self._update_acm()
        x = rb._obs[rb._obs_idx[:len(rb)]]  # update_obs_mean_std
        self.mean, self.std = x.mean(0).astype(np.float32), (x.std(0) + 1e-8).astype(np.float32)
        np.percentile(x, 99, axis=0), np.percentile(x, 1, axis=0)
        self.iteration += 1
        return len(rew)

    def run(self, iterations=None):
        """Frames per second over ``iterations`` (default: one ACM update cycle, acm_update_freq
        iterations, so the ACM epochs are amortised at the reference's cadence)."""
        iterations = iterations or max(1, self.acm_freq)
        t0 = time.perf_counter()
        n = sum(self.iterate() for _ in range(iterations))
        el = time.perf_counter() - t0
        return n / el, n, el
