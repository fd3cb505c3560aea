"""Flat parameter layouts of the hot-path networks (state_dict order) and
nn.Linear-style initialisation.

Each network lives in ONE contiguous float32 device buffer; the device library
addresses layers by these offsets.  Layouts follow the reference modules:
  SAC_Actor   rltoolkit/algorithms/sac/models.py:8-22   fc1, fc2, fc_prob, fc_scale
  SAC_Critic  rltoolkit/algorithms/sac/models.py:72-80  fc1, fc2, fc3
  AcM         rltoolkit/basic_model.py:108-117          fc1 (->64), fc2 (->32), fc3 (->ac)
  DDPG Actor  rltoolkit/algorithms/ddpg/models.py:5-22  fc1, fc2, fc3 (->aout, tanh*lim)
  BasicAcM    rltoolkit/acm/models/basic_acm.py:11-21   t, t1, fc1 (->100), fc2 (->50), fc21 (->50), fc3
"""
import math

import torch

H = 256


def sac_actor_layout(ob, aout):
    return [("fc1.weight", (H, ob)), ("fc1.bias", (H,)), ("fc2.weight", (H, H)), ("fc2.bias", (H,)),
            ("fc_prob.weight", (aout, H)), ("fc_prob.bias", (aout,)),
            ("fc_scale.weight", (aout, H)), ("fc_scale.bias", (aout,))]


def critic_layout(inp):
    return [("fc1.weight", (H, inp)), ("fc1.bias", (H,)), ("fc2.weight", (H, H)), ("fc2.bias", (H,)),
            ("fc3.weight", (1, H)), ("fc3.bias", (1,))]


def acm_layout(inp, ac):
    return [("fc1.weight", (64, inp)), ("fc1.bias", (64,)), ("fc2.weight", (32, 64)), ("fc2.bias", (32,)),
            ("fc3.weight", (ac, 32)), ("fc3.bias", (ac,))]


def ddpg_actor_layout(ob, aout):
    return [("fc1.weight", (H, ob)), ("fc1.bias", (H,)), ("fc2.weight", (H, H)), ("fc2.bias", (H,)),
            ("fc3.weight", (aout, H)), ("fc3.bias", (aout,))]


def basic_acm_layout(inp, ac):
    # module parameters t, t1 precede the submodules' in named_parameters / state_dict
    return [("t", (1,)), ("t1", (ac,)), ("fc1.weight", (100, inp)), ("fc1.bias", (100,)),
            ("fc2.weight", (50, 100)), ("fc2.bias", (50,)), ("fc21.weight", (50, inp)), ("fc21.bias", (50,)),
            ("fc3.weight", (ac, 50)), ("fc3.bias", (ac,))]


def numel(layout):
    return sum(math.prod(s) for _, s in layout)


def views(flat, layout):
    """{name: view into the flat buffer} (state_dict-like)."""
    out, o = {}, 0
    for name, shape in layout:
        n = math.prod(shape)
        out[name] = flat[o:o + n].view(shape)
        o += n
    return out


def linear_init_(flat, layout, generator=None):
    """nn.Linear.reset_parameters: weight and bias ~ U(-1/sqrt(fan_in), 1/sqrt(fan_in))."""
    v = views(flat, layout)
    fan_in = None
    with torch.no_grad():
        for name, shape in layout:
            if name in ("t", "t1"):  # BasicAcM output scales start at 1 (basic_acm.py:20-21)
                v[name].fill_(1.0)
                continue
            if name.endswith("weight"):
                fan_in = shape[1]
            bound = 1.0 / math.sqrt(fan_in)
            t = torch.empty(shape).uniform_(-bound, bound, generator=generator)
            v[name].copy_(t.to(flat.device))
    return flat


def load_state(flat, layout, state):
    """Copy a state_dict-like mapping into the flat buffer."""
    v = views(flat, layout)
    with torch.no_grad():
        for name, _ in layout:
            v[name].copy_(torch.as_tensor(state[name], dtype=torch.float32).reshape(v[name].shape))
    return flat


def state_dict(flat, layout):
    return {k: t.detach().cpu().clone() for k, t in views(flat, layout).items()}
