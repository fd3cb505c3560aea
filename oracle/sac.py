"""ORACLE (test infrastructure only): one vanilla SAC grad step (BASELINE configs[0]).

Follows rltoolkit/algorithms/sac/sac.py (reference @ v0):
  compute_qfunc_targ :138-161  y = r + g(1-d)(min(Q1t,Q2t)(s', a') - alpha logpi'),  a' ~ pi(s')
  compute_pi_loss    :163-184  mean(alpha logpi - min(Q1,Q2)(s, a))
  update             :218-280  critic_1 step, critic_2 step, actor step, polyak, alpha step
The math is SAC_AcM's with no ACM, the critics fed the actor's action directly, no custom
loss, and an identity denormalisation; it is restated on top of OracleSacAcm with exactly
that configuration (min-max denormalisation over [-1, 1] is mid 0 + x * delta 1, exact).
Quirks: Q1 tau = config.TAU and act_noise = config.ACT_NOISE whatever is passed
(sac.py:17-24 forwards neither to DDPG), Q4 target entropy = -ac_dim.
"""
import numpy as np
import torch

from . import nets
from .nets import Norm
from .sac_acm import OracleSacAcm


class OracleSac(OracleSacAcm):
    def __init__(self, ob, ac, *, ac_lim=1.0, gamma=0.99, tau=0.005, actor_lr=1e-3, critic_lr=1e-3, alpha_lr=1e-3,
                 alpha=0.2, params=None, dtype=torch.float32):
        params = dict(params)
        params.setdefault("acm", {n: np.zeros(s, np.float32) for n, s in nets.acm_layout(2 * ob, ac)})
        ident = Norm(True, -torch.ones(ac, dtype=dtype), torch.ones(ac, dtype=dtype))
        super().__init__(ob, ac, ac, acm_critic=False, custom_loss=0.0, norm_closs=False, norm=ident,
                         actor_lim=ac_lim, acm_lim=1.0, gamma=gamma, tau=tau, actor_lr=actor_lr, critic_lr=critic_lr,
                         alpha_lr=alpha_lr, alpha=alpha, target_entropy=-float(ac), params=params, dtype=dtype)

    def update(self, obs, next_obs, action, reward, done, eps_next, eps_cur):
        """SAC.update (sac.py:218-280); the batch has no ACM action."""
        B = np.asarray(obs).shape[0]
        return super().update(obs, next_obs, action, reward, done, np.zeros((B, self.ac), np.float32), eps_next,
                              eps_cur)


def policy_act(p, obs, ac_lim, eps, noise, act_noise):
    """DDPG.noise_action (ddpg.py:171-176) with the SAC actor: a ~ pi(s) (tanh-squashed, * ac_lim),
    a += act_noise * N(0, 1), clip to [-ac_lim, ac_lim]; process_action is the identity."""
    lim = torch.as_tensor(ac_lim, dtype=torch.float32)
    with torch.no_grad():
        a, _, _ = nets.sac_actor(p, torch.as_tensor(obs), lim, None if eps is None else torch.as_tensor(eps))
        a = a + act_noise * torch.as_tensor(noise)
        return torch.max(torch.min(a, lim), -lim).numpy()
