"""ORACLE (test infrastructure only): one DDPG_AcM grad step, restated.

Follows rltoolkit/acm/off_policy/ddpg_acm.py (reference @ v0):
  compute_qfunc_targ :100-123  y = r + g(1-d) Qt(s', ACM(s', denorm mu_t(s')))
  compute_pi_loss    :125-145  -Q(s, ACM(s, denorm mu(s))).mean() + c*MSE
  update             :147-201  critic step, actor step, polyak on critic AND actor targets
polyak: rltoolkit/algorithms/ddpg/ddpg.py:273-284.  The SPP-DDPG scripts inject
BasicAcM (train/spp_ddpg_hcheetah.py:124) — ``acm_kind`` selects it.
"""
import numpy as np
import torch
import torch.nn.functional as F

from . import nets
from .adam import OracleAdam


class OracleDdpgAcm:
    def __init__(self, ob, aout, ac, *, acm_critic=True, custom_loss=1.0, norm_closs=False, norm=None,
                 actor_lim=1.0, acm_lim=1.0, acm_kind="basic", gamma=0.95, tau=0.005, actor_lr=5e-4,
                 critic_lr=5e-4, params=None, dtype=torch.float32):
        self.dt = dtype  # float64: clean reference for the large-batch parity tests
        self.acm_critic, self.custom_loss, self.norm_closs, self.norm = acm_critic, custom_loss, norm_closs, norm
        self.actor_lim = torch.as_tensor(actor_lim, dtype=dtype)
        self.acm_lim = torch.as_tensor(acm_lim, dtype=dtype)
        self.acm_kind, self.gamma, self.tau = acm_kind, gamma, tau
        cin = ob + (ac if acm_critic else aout)
        acm_lay = nets.basic_acm_layout(2 * ob, ac) if acm_kind == "basic" else nets.acm_layout(2 * ob, ac)
        self.layouts = {"actor": nets.ddpg_actor_layout(ob, aout), "critic": nets.critic_layout(cin),
                        "actor_targ": nets.ddpg_actor_layout(ob, aout), "critic_targ": nets.critic_layout(cin),
                        "acm": acm_lay}
        self.p = {k: {n: torch.as_tensor(params[k][n]).to(dtype).clone()
                      .requires_grad_(k in ("actor", "critic")) for n, _ in lay}
                  for k, lay in self.layouts.items()}
        self.opt = {"actor": OracleAdam(self.p["actor"].values(), actor_lr),
                    "critic": OracleAdam(self.p["critic"].values(), critic_lr)}

    def _acm(self, x):
        if self.acm_kind == "basic":
            return nets.basic_acm(self.p["acm"], x)
        return nets.acm(self.p["acm"], x, self.acm_lim)

    def update(self, obs, next_obs, action, reward, done, acm_action):
        t = lambda a, dt=self.dt: torch.as_tensor(np.asarray(a)).to(dt)  # noqa: E731
        obs, next_obs, action, reward = t(obs), t(next_obs), t(action), t(reward)
        done, acm_action = t(done, torch.int8), t(acm_action)
        P, losses = self.p, {}
        with torch.no_grad():
            na = self.norm.denormalize(nets.ddpg_actor(P["actor_targ"], next_obs, self.actor_lim))
            if self.acm_critic:
                na = self._acm(torch.cat([next_obs, na], axis=1))
            y = reward + self.gamma * (1 - done) * nets.ddpg_critic(P["critic_targ"], next_obs, na)
        if self.acm_critic:
            action = acm_action
        lq = F.mse_loss(nets.ddpg_critic(P["critic"], obs, action), y)
        losses["critic"] = lq.item()
        gq = torch.autograd.grad(lq, list(P["critic"].values()))
        self.opt["critic"].step(gq)
        a = nets.ddpg_actor(P["actor"], obs, self.actor_lim)
        ad = self.norm.denormalize(a)
        ca = self._acm(torch.cat([obs, ad], axis=1)) if self.acm_critic else ad
        loss = -nets.ddpg_critic(P["critic"], obs, ca).mean()
        losses["ddpg"], losses["dist"] = 0.0, 0.0
        if self.custom_loss:
            losses["ddpg"] = loss.item()
            target, pred = (self.norm.normalize(next_obs), a) if self.norm_closs else (next_obs, ad)
            dist = F.mse_loss(pred, target)
            losses["dist"] = dist.item()
            loss = loss + self.custom_loss * dist
        losses["actor"] = loss.item()
        ga = torch.autograd.grad(loss, list(P["actor"].values()))
        self.opt["actor"].step(ga)
        flat = lambda gs: torch.cat([x.reshape(-1) for x in gs]).numpy()  # noqa: E731
        self.last = {"y": y, "grads": {"critic": flat(gq), "actor": flat(ga)}}
        with torch.no_grad():
            for c, tg in (("critic", "critic_targ"), ("actor", "actor_targ")):
                for n in P[c]:
                    P[tg][n].mul_(1 - self.tau)
                    P[tg][n].add_(self.tau * P[c][n])
        return losses

    def flat(self, k):
        return nets.flatten(self.p[k]).numpy()


def make_unbiased_update(oracle, ring, B, grad_steps, mt, norm=None, eps=None):
    """DDPG_AcM.make_unbiased_update (acm/off_policy/ddpg_acm.py:59-73): grad_steps batches of
    sample_batch (replay_buffer.py:233-261, 385-398; with obs_norm the buffer normalises obs and next obs,
    :247-249), each updated with action = next_obs.  ``ring`` is an OracleReplay, ``mt`` its index stream,
    ``norm`` the buffer's normaliser when obs_norm (None: raw obs); ``eps`` (SAC_AcM, which inherits this
    make_update: sac_acm.py:12) the rsample draws of each update in call order, [2 grad_steps][B][aout].  Returns
    the last step's losses and the sampled indices [grad_steps][B]."""
    losses, idxs = None, []
    for _ in range(grad_steps):
        (obs, next_obs, _, rew, done, acm), idx = ring.sample_batch(B, mt)
        if norm is not None:
            obs = norm.normalize(torch.from_numpy(obs)).numpy()
            next_obs = norm.normalize(torch.from_numpy(next_obs)).numpy()
        k = len(idxs)
        extra = () if eps is None else (eps[2 * k], eps[2 * k + 1])
        losses = oracle.update(obs, next_obs, next_obs, rew, done, acm, *extra)
        idxs.append(idx)
    return losses, np.stack(idxs)
