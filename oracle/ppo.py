"""ORACLE (test infrastructure only): PPO advantage pieces, restated.

  calculate_q_val  rltoolkit/algorithms/a2c/a2c.py:247-265   q = r + g(1-d) V(s')
  calculate_gae    rltoolkit/algorithms/ppo/ppo.py:117-150   reverse scan with done reset
                   and end (truncation) bootstrap gae = V(s') (Q10)
  _clip_loss       rltoolkit/algorithms/ppo/ppo.py:194-204
The scan is also given in its affine form a_t = b_t + c_t a_{t+1}
(b_t = delta_t + [end & !done] gl V(s'_t), c_t = [!done & !end] gl), the
formulation the device scan uses.
"""
import numpy as np
import torch


def q_val(rew, done, v_next, gamma):
    return rew + gamma * (1 - done) * v_next


def gae_loop(delta, done, end, v_next, gamma, lam):
    adv = np.empty_like(delta)
    disc = gamma * lam
    gae = 0.0
    for i in range(len(delta) - 1, -1, -1):
        if done[i]:
            gae = 0.0
        elif end[i]:
            gae = float(v_next[i])
        gae = gae * disc + delta[i]
        adv[i] = gae
    return adv


def gae_affine(delta, done, end, v_next, gamma, lam):
    gl = gamma * lam
    done = np.asarray(done, bool)
    end = np.asarray(end, bool)
    b = delta + np.where(end & ~done, gl * v_next, 0.0)
    c = np.where(~done & ~end, gl, 0.0)
    out = np.empty_like(delta)
    acc = 0.0
    for i in range(len(delta) - 1, -1, -1):
        acc = b[i] + c[i] * acc
        out[i] = acc
    return out


def clip_loss(lp_old, lp_new, adv, eps=0.2):
    lp_old, lp_new, adv = (torch.as_tensor(np.asarray(x)) for x in (lp_old, lp_new, adv))
    ratio = torch.exp(lp_new - lp_old)
    clipped = torch.clamp(ratio, 1 - eps, 1 + eps)
    return -(torch.min(ratio * adv, clipped * adv)).mean().item()
