"""ORACLE (test infrastructure only): functional forwards of the reference MLPs.

Parameters are dicts ``{state_dict key: tensor}`` in state_dict order.
  sac_actor     rltoolkit/algorithms/sac/models.py:24-54   (SAC_Actor.forward, continuous)
  sac_critic    rltoolkit/algorithms/sac/models.py:81-91   (SAC_Critic.forward)
  ddpg_actor    rltoolkit/algorithms/ddpg/models.py:17-22  (Actor.forward)
  ddpg_critic   rltoolkit/algorithms/ddpg/models.py:39-44  (Critic.forward)
  acm           rltoolkit/basic_model.py:118-126           (AcM.forward, continuous)
  basic_acm     rltoolkit/acm/models/basic_acm.py:20-24    (BasicAcM.forward)
  denormalize / normalize  rltoolkit/buffer/memory.py:76-127, utils.py:62-73
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

LOG2 = float(np.log(2))
LOG_SQRT_2PI = math.log(math.sqrt(2 * math.pi))


def lin(x, p, name):
    return F.linear(x, p[name + ".weight"], p[name + ".bias"])


def sac_actor(p, x, lim, eps=None):
    """Returns (action, logprob, u).  eps=None -> deterministic (action = tanh(mu)*lim)."""
    h = torch.relu(lin(x, p, "fc1"))
    h = torch.relu(lin(h, p, "fc2"))
    mu = lin(h, p, "fc_prob")
    ls = torch.clamp(lin(h, p, "fc_scale"), -20, 2)
    scale = torch.exp(ls)
    u = mu if eps is None else mu + eps * scale
    var = scale ** 2
    lp = (-((u - mu) ** 2) / (2 * var) - scale.log() - LOG_SQRT_2PI).sum(axis=-1)
    corr = 2 * (LOG2 - u - F.softplus(-2 * u)).sum(axis=1)
    lp = lp - corr
    return torch.tanh(u) * lim, lp, u


def sac_critic(p, obs, ac):
    x = torch.cat((obs, ac), dim=-1)
    x = torch.relu(lin(x, p, "fc1"))
    x = torch.relu(lin(x, p, "fc2"))
    return torch.squeeze(lin(x, p, "fc3"), -1)


ddpg_critic = sac_critic


def ddpg_actor(p, x, lim):
    h = torch.relu(lin(x, p, "fc1"))
    h = torch.relu(lin(h, p, "fc2"))
    return torch.tanh(lin(h, p, "fc3")) * lim


def acm(p, x, lim):
    x = torch.tanh(lin(x, p, "fc1"))
    x = torch.tanh(lin(x, p, "fc2"))
    return torch.tanh(lin(x, p, "fc3")) * lim


def basic_acm(p, x):
    h = torch.tanh(lin(x, p, "fc1"))
    h1 = torch.tanh(lin(h, p, "fc2") + p["t"] * lin(x, p, "fc21"))
    return torch.tanh(lin(h1, p, "fc3")) * p["t1"]


class Norm:
    """Replay-buffer normalizer state: min/max (min_max_denormalize) or mean/std."""

    def __init__(self, min_max, lo=None, hi=None, mean=None, std=None):
        self.min_max, self.lo, self.hi, self.mean, self.std = min_max, lo, hi, mean, std

    def denormalize(self, x):
        if self.min_max:
            mid = (self.hi + self.lo) / 2
            delta = (self.hi - self.lo) / 2
            return mid + x * delta
        return (self.std + 1e-8) * x + self.mean

    def normalize(self, x):
        if self.min_max:
            mid = (self.hi + self.lo) / 2
            return (x - mid) / (self.hi - mid + 1e-8)
        return torch.clamp((x - self.mean) / (self.std + 1e-8), -10, 10)


# state_dict layouts (name, shape) — the flat parameter order shared with the device library
def sac_actor_layout(ob, aout, H=256):
    return [("fc1.weight", (H, ob)), ("fc1.bias", (H,)), ("fc2.weight", (H, H)), ("fc2.bias", (H,)),
            ("fc_prob.weight", (aout, H)), ("fc_prob.bias", (aout,)),
            ("fc_scale.weight", (aout, H)), ("fc_scale.bias", (aout,))]


def critic_layout(inp, H=256):
    return [("fc1.weight", (H, inp)), ("fc1.bias", (H,)), ("fc2.weight", (H, H)), ("fc2.bias", (H,)),
            ("fc3.weight", (1, H)), ("fc3.bias", (1,))]


def ddpg_actor_layout(ob, aout, H=256):
    return [("fc1.weight", (H, ob)), ("fc1.bias", (H,)), ("fc2.weight", (H, H)), ("fc2.bias", (H,)),
            ("fc3.weight", (aout, H)), ("fc3.bias", (aout,))]


def acm_layout(inp, ac):
    return [("fc1.weight", (64, inp)), ("fc1.bias", (64,)), ("fc2.weight", (32, 64)), ("fc2.bias", (32,)),
            ("fc3.weight", (ac, 32)), ("fc3.bias", (ac,))]


def basic_acm_layout(inp, ac):
    return [("t", (1,)), ("t1", (ac,)), ("fc1.weight", (100, inp)), ("fc1.bias", (100,)),
            ("fc2.weight", (50, 100)), ("fc2.bias", (50,)), ("fc21.weight", (50, inp)),
            ("fc21.bias", (50,)), ("fc3.weight", (ac, 50)), ("fc3.bias", (ac,))]


def flatten(p):
    return torch.cat([v.detach().reshape(-1) for v in p.values()])


def unflatten(flat, layout, requires_grad=False):
    out, o = {}, 0
    flat = torch.as_tensor(flat, dtype=torch.float32)
    for name, shape in layout:
        n = int(np.prod(shape))
        out[name] = flat[o:o + n].reshape(shape).clone().requires_grad_(requires_grad)
        o += n
    return out
