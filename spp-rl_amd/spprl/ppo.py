"""PPO advantage / loss pieces on the MI355X library.

Mirrors rltoolkit's on-policy helpers with device tensors in and out:
  calculate_q_val + calculate_gae   rltoolkit/algorithms/a2c/a2c.py:247-265,
                                    rltoolkit/algorithms/ppo/ppo.py:117-150
  clip_loss (+ kl_divergence)       ppo.py:194-204, utils.py:48-59
  normalize_advantages              algorithms/ppo/advantage_dataset.py:8-12
The reference walks one rollout buffer (E = 1); here E lockstep envs are
time-major [T][E] streams, each scanned independently.
"""
import torch

from . import _lib
from ._lib import call, ptr, stream_handle


def _dev(x, dtype):
    return x.to(dtype=dtype).contiguous()


def calculate_gae(rew, v, v_next, done, end, gamma, gae_lambda, mode=-1, with_q=True):
    """Returns (q_val, advantage) for time-major [T] or [T, E] device tensors.
    mode 0 = exact sequential per stream, 1 = wavefront-shuffle scan, -1 = auto."""
    _lib.load()
    shape = rew.shape
    T = shape[0]
    E = 1 if rew.dim() == 1 else shape[1]
    rew, v, v_next = (_dev(x, torch.float32) for x in (rew, v, v_next))
    done, end = (_dev(x != 0, torch.uint8) for x in (done, end))
    adv = torch.empty_like(rew)
    q = torch.empty_like(rew) if with_q else None
    call("sppGaeScan", ptr(rew), ptr(v), ptr(v_next), ptr(done), ptr(end), T, E, float(gamma), float(gae_lambda),
         int(mode), ptr(q), ptr(adv), stream_handle())
    return q, adv


def clip_loss(lp_old, lp_new, adv, eps=0.2, with_grad=True):
    """PPO._clip_loss forward on device; returns (loss[0-dim], kl[0-dim], d loss / d lp_new or None)."""
    _lib.load()
    lp_old, lp_new, adv = (_dev(x, torch.float32).reshape(-1) for x in (lp_old, lp_new, adv))
    B = lp_old.numel()
    out = torch.empty(2, device=lp_old.device)
    grad = torch.empty_like(lp_new) if with_grad else None
    call("sppPpoClipLoss", ptr(lp_old), ptr(lp_new), ptr(adv), B, float(eps), ptr(grad), ptr(out), stream_handle())
    return out[0], out[1], grad


def normalize_advantages(adv):
    """(A - mean) / (std + 1.2e-7) (AdvantageDataset, normalize_adv=True)."""
    _lib.load()
    a = _dev(adv, torch.float32)
    out = torch.empty_like(a)
    call("sppAdvNormalize", ptr(a), a.numel(), ptr(out), stream_handle())
    return out
