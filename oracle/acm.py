"""ORACLE (test infrastructure only): AcMTrainer.batch_update, restated.

rltoolkit/acm/acm.py:246-258 — y_pred = ACM(x); loss = MSE(y_pred, y); Adam step.
Batch assembly: acm_cat (acm.py:260-264) = cat(obs[:, idx], next_obs[:, idx]).
"""
import numpy as np
import torch
import torch.nn.functional as F

from . import nets
from .adam import OracleAdam


class OracleAcmTrainer:
    def __init__(self, inp, ac, lr=3e-3, ac_lim=1.0, params=None):
        self.layout = nets.acm_layout(inp, ac)
        self.p = {n: torch.as_tensor(params[n], dtype=torch.float32).clone().requires_grad_(True)
                  for n, _ in self.layout}
        self.lim = torch.as_tensor(ac_lim, dtype=torch.float32)
        self.opt = OracleAdam(self.p.values(), lr)

    def batch_update(self, x, y):
        x = torch.as_tensor(np.asarray(x), dtype=torch.float32)
        y = torch.as_tensor(np.asarray(y), dtype=torch.float32)
        if y.dim() < 2:
            y = y.reshape(len(y), -1)
        loss = F.mse_loss(nets.acm(self.p, x, self.lim), y)
        g = torch.autograd.grad(loss, list(self.p.values()))
        self.last_grad = torch.cat([t.reshape(-1) for t in g]).numpy()
        self.opt.step(g)
        return loss.item()

    def flat(self):
        return nets.flatten(self.p).numpy()


def acm_cat(obs, next_obs, idx=None):
    obs, next_obs = np.asarray(obs), np.asarray(next_obs)
    if idx is not None:
        obs, next_obs = obs[:, idx], next_obs[:, idx]
    return np.concatenate([obs, next_obs], axis=1)
