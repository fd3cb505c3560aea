"""Micro-run of update_obs_mean_std for rocprofv3 (kernel breakdown): python tools/stats_prof.py [n] [ob] [reps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "spp-rl_amd"))
import spprl  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
ob = int(sys.argv[2]) if len(sys.argv) > 2 else 11
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
dev = torch.device("cuda:0")
rb = spprl.BufferAcMOffPolicy(n + 10, ob, ob, 3, device=dev)
obs = torch.randn(n + 1, ob, device=dev)
slots = rb.add_obs_batch(obs)
rb.add_timestep_batch(slots[:n], slots[1:], torch.zeros(n, ob, device=dev), torch.zeros(n, device=dev),
                      torch.zeros(n, dtype=torch.uint8, device=dev), torch.zeros(n, dtype=torch.uint8, device=dev),
                      torch.zeros(n, 3, device=dev))
for _ in range(3):
    rb.update_obs_mean_std()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(reps):
    rb.update_obs_mean_std()
e.record()
torch.cuda.synchronize()
print("n=%d ob=%d: %.4f ms per update_obs_mean_std" % (n, ob, s.elapsed_time(e) / reps))
