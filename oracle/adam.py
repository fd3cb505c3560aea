"""ORACLE (test infrastructure only): torch.optim.Adam step, restated.

Third-party algorithm (torch 1.3.1 pinned by the reference, 2.10 here; the
golden vectors come from the installed 2.10 single-tensor CPU path):
  m <- lerp(m, g, 1-b1); v <- v*b2 + (1-b2) g^2
  p <- p - lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
Used by every optimizer of the hot path (rltoolkit/rl.py:62, ddpg.py:132-135,
sac.py:107-110, acm.py:176-183); betas (0.9, 0.999), eps 1e-8, no weight decay.
"""
import torch


class OracleAdam:
    def __init__(self, params, lr, betas=(0.9, 0.999), eps=1e-8):
        self.params = list(params)
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.t = 0

    @torch.no_grad()
    def step(self, grads):
        self.t += 1
        bc1 = 1 - self.b1 ** self.t
        bc2s = (1 - self.b2 ** self.t) ** 0.5
        step_size = self.lr / bc1
        for p, g, m, v in zip(self.params, grads, self.m, self.v):
            if g is None:
                g = torch.zeros_like(p)
            m.lerp_(g, 1 - self.b1)
            v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            denom = (v.sqrt() / bc2s).add_(self.eps)
            p.addcdiv_(m, denom, value=-step_size)
