"""ORACLE (test infrastructure only): one SAC_AcM grad step, restated.

Follows rltoolkit/acm/off_policy/sac_acm.py (reference @ v0):
  compute_qfunc_targ :30-58   y = r + g(1-d)(min(Q1t,Q2t)(s', ACM(s', denorm a')) - alpha logpi')
  compute_pi_loss    :60-87   mean(alpha logpi - min(Q1,Q2)(s, ACM(s, denorm a))) + c*MSE
  update             :89-162  critic_1 step, critic_2 step, actor step, polyak, alpha step
and rltoolkit/algorithms/sac/sac.py:186-216 (update_target_q, compute_alpha_loss).
Quirks kept: Q1 tau is always config.TAU; Q4 target entropy = -env ac_dim and
alpha loss exp(log_alpha)*(...); log_alpha is float64 (sac.py:107-109); the
ACM is frozen during the update (grad flows to its input only).
Gaussian eps of both rsample calls are inputs (eps_next, eps_cur).
"""
import numpy as np
import torch
import torch.nn.functional as F

from . import nets
from .adam import OracleAdam


class OracleSacAcm:
    def __init__(self, ob, aout, ac, *, acm_critic=True, custom_loss=0.2, norm_closs=False,
                 norm=None, actor_lim=1.0, acm_lim=1.0, gamma=0.99, tau=0.005, actor_lr=1e-3,
                 critic_lr=1e-3, alpha_lr=1e-3, alpha=0.2, target_entropy=None, params=None, dtype=torch.float32):
        # dtype=torch.float64 gives a clean reference for the large-batch parity tests (the
        # device path is fp32; at B = 409,600 its summation order differs from torch's)
        self.dt = dtype
        self.ob, self.aout, self.ac = ob, aout, ac
        self.acm_critic, self.custom_loss, self.norm_closs = acm_critic, custom_loss, norm_closs
        self.norm = norm
        self.actor_lim = torch.as_tensor(actor_lim, dtype=dtype)
        self.acm_lim = torch.as_tensor(acm_lim, dtype=dtype)
        self.gamma, self.tau = gamma, tau
        self.target_entropy = float(-ac if target_entropy is None else target_entropy)
        cin = ob + (ac if acm_critic else aout)
        self.layouts = {"actor": nets.sac_actor_layout(ob, aout), "critic_1": nets.critic_layout(cin),
                        "critic_2": nets.critic_layout(cin), "critic_1_targ": nets.critic_layout(cin),
                        "critic_2_targ": nets.critic_layout(cin), "acm": nets.acm_layout(2 * ob, ac)}
        self.p = {}
        for k, lay in self.layouts.items():
            trainable = k in ("actor", "critic_1", "critic_2")
            self.p[k] = {n: torch.as_tensor(params[k][n]).to(dtype).clone()
                         .requires_grad_(trainable) for n, _ in lay}
        self.opt = {"actor": OracleAdam(self.p["actor"].values(), actor_lr),
                    "critic_1": OracleAdam(self.p["critic_1"].values(), critic_lr),
                    "critic_2": OracleAdam(self.p["critic_2"].values(), critic_lr)}
        self.log_alpha = torch.tensor(np.log(alpha), requires_grad=True)  # float64, sac.py:107
        self.alpha = alpha
        self.opt_alpha = OracleAdam([self.log_alpha], alpha_lr)
        self.last = {}

    def _acm(self, x):
        return nets.acm(self.p["acm"], x, self.acm_lim)

    def _t(self, a, dt=None):
        return torch.as_tensor(np.asarray(a)).to(self.dt if dt is None else dt)

    def critic_grads(self, obs, next_obs, action, reward, done, acm_action, eps_next):
        """compute_qfunc_targ (sac_acm.py:30-58) + both critic losses (:97-131).
        Returns ({critic_k: [grad tensors]}, losses, y)."""
        t = self._t
        obs, next_obs, action, reward = t(obs), t(next_obs), t(action), t(reward)
        done, acm_action, eps_next = t(done, torch.int8), t(acm_action), t(eps_next)
        P, losses = self.p, {}
        with torch.no_grad():
            a2, lp2, _ = nets.sac_actor(P["actor"], next_obs, self.actor_lim, eps_next)
            a2 = self.norm.denormalize(a2)
            if self.acm_critic:
                a2 = self._acm(torch.cat([next_obs, a2], axis=1))
            q1t = nets.sac_critic(P["critic_1_targ"], next_obs, a2)
            q2t = nets.sac_critic(P["critic_2_targ"], next_obs, a2)
            y = reward + self.gamma * (1 - done) * (torch.min(q1t, q2t) - self.alpha * lp2)
        if self.acm_critic:
            action = acm_action
        grads = {}
        for k in ("critic_1", "critic_2"):
            q = nets.sac_critic(P[k], obs, action)
            loss = F.mse_loss(q, y)
            losses[k] = loss.item()
            grads[k] = list(torch.autograd.grad(loss, list(P[k].values())))
        return grads, losses, y

    def critic_apply(self, grads):
        for k in ("critic_1", "critic_2"):
            self.opt[k].step(grads[k])

    def actor_grads(self, obs, next_obs, eps_cur):
        """compute_pi_loss (sac_acm.py:60-87) against the updated critics and the alpha-loss
        gradient operand (sac.py:201-216).  Returns ([actor grads], alpha_grad, losses, logp)."""
        t = self._t
        obs, next_obs, eps_cur = t(obs), t(next_obs), t(eps_cur)
        P, losses = self.p, {}
        a, lp, _ = nets.sac_actor(P["actor"], obs, self.actor_lim, eps_cur)
        ad = self.norm.denormalize(a)
        ca = self._acm(torch.cat([obs, ad], axis=1)) if self.acm_critic else ad
        q = torch.min(nets.sac_critic(P["critic_1"], obs, ca), nets.sac_critic(P["critic_2"], obs, ca))
        loss = (self.alpha * lp - q).mean()
        losses["sac"], losses["dist"] = 0.0, 0.0
        if self.custom_loss:
            losses["sac"] = loss.item()
            if self.norm_closs:
                target, pred = self.norm.normalize(next_obs), a
            else:
                target, pred = next_obs, ad
            dist = F.mse_loss(pred, target)
            losses["dist"] = dist.item()
            loss = loss + self.custom_loss * dist
        losses["actor"] = loss.item()
        g = list(torch.autograd.grad(loss, list(P["actor"].values())))
        lpd = lp.detach()
        alpha_loss = (self.log_alpha.exp() * (-lpd - self.target_entropy)).mean()
        losses["alpha_loss"] = alpha_loss.item()
        (ga,) = torch.autograd.grad(alpha_loss, [self.log_alpha])
        return g, ga, losses, lpd

    def actor_apply(self, g, alpha_grad):
        """Actor Adam step, polyak (sac.py:186-199, two roundings), alpha Adam step."""
        P = self.p
        self.opt["actor"].step(g)
        with torch.no_grad():
            for c, tg in (("critic_1", "critic_1_targ"), ("critic_2", "critic_2_targ")):
                for n in P[c]:
                    P[tg][n].mul_(1 - self.tau)
                    P[tg][n].add_(self.tau * P[c][n])
        self.opt_alpha.step([alpha_grad])
        self.alpha = self.log_alpha.exp().item()

    def update(self, obs, next_obs, action, reward, done, acm_action, eps_next, eps_cur):
        """SAC_AcM.update (sac_acm.py:89-162) = critic_grads, critic_apply, actor_grads, actor_apply."""
        cg, losses, y = self.critic_grads(obs, next_obs, action, reward, done, acm_action, eps_next)
        self.critic_apply(cg)
        g, ga, l2, lpd = self.actor_grads(obs, next_obs, eps_cur)
        losses.update(l2)
        self.actor_apply(g, ga)
        flat = lambda gs: torch.cat([x.detach().reshape(-1) for x in gs]).numpy()  # noqa: E731
        self.last = {"y": y, "logp": lpd, "grads": {"critic_1": flat(cg["critic_1"]), "critic_2": flat(cg["critic_2"]),
                                                    "actor": flat(g)}}
        return losses

    def flat(self, k):
        return nets.flatten(self.p[k]).numpy()
