"""Region timing of the SAC phase kernels (profiling build: python spp-rl_amd/build.py --prof).
Usage: SPPRL_LIB=spp-rl_amd/spprl/libspprl_prof.so python tools/region_prof.py"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "spp-rl_amd"), REPO]
import torch  # noqa: E402

import spprl  # noqa: E402
from spprl import _lib  # noqa: E402

NAMES = {0: "tile start", 1: "actor L1", 2: "actor L2", 3: "actor heads", 4: "squash", 5: "ACM + target input",
         6: "targ1 L1", 7: "targ1 L2", 8: "targ2 L1", 9: "targ2 L2", 10: "y + critic input", 11: "critic L1",
         12: "critic L2", 13: "delta2 staging", 14: "critic W2T", 15: "tile end",
         20: "dense_lds prologue | A: delta staging (nodense)", 21: "dense_lds loop | A: W2T (nodense)",
         22: "dense_lds epilogue | A: W1Ta (nodense)",
         23: "dense prologue | A: ACM bwd input (nodense)", 24: "dense mfma | A: ACM W3T (nodense)",
         25: "dense epilogue | A: ACM W2T (nodense)",
         26: "A: tile start", 27: "A: actor trunk", 28: "A: squash", 29: "A: ACM fwd", 19: "A: q min",
         30: "A: critics L1 (fwd)", 31: "A: critics L2 (fwd)", 16: "A: ACM bwd", 17: "A: heads bwd", 18: "A: trunk bwd"}


def main():
    """argv[1]: hopper (default) | ant_bf16 (build with --prof --bf16-only)"""
    dev = torch.device("cuda", 0)
    E, B = 4096, 409600
    cfg = sys.argv[1] if len(sys.argv) > 1 else "hopper"
    env, ob, ac, bf = {"hopper": ("Hopper-v2", 11, 3, False), "ant_bf16": ("Ant-v2", 111, 8, True)}[cfg]
    ag = spprl.SAC_AcM(env_name=env, acm_critic=True, custom_loss=0.2, norm_closs=False,
                       min_max_denormalize=True, denormalize_actor_out=True, max_batch=B, buffer_size=200_000,
                       device=dev, seed=0, mlp_bf16=bf)
    rb = ag.replay_buffer
    n = 150_000
    slots = rb.add_obs_batch(torch.randn(n + 1, ob, device=dev))
    rb.add_timestep_batch(slots[:n], slots[1:], torch.randn(n, ob, device=dev), torch.randn(n, device=dev),
                          torch.zeros(n, dtype=torch.uint8, device=dev), torch.zeros(n, dtype=torch.uint8, device=dev),
                          torch.rand(n, ac, device=dev) * 2 - 1)
    rb.update_obs_mean_std()
    idx = torch.randint(0, n, (B,), device=dev)
    buf = (ctypes.c_ulonglong * 64)()
    for it in range(4):
        if it == 1:
            _lib.call("sppDebugReadProf", buf, 1)
        ag.update_from_replay_dp(idx, 1, it)
    torch.cuda.synchronize()
    _lib.call("sppDebugReadProf", buf, 0)
    t = np.array(buf[:32], np.float64)
    tiles = 3 * (B // 32)
    tot = t.sum()
    print("%s: both phases, cycles per tile (%d tiles per phase): total %.0f" % (cfg, tiles, tot / tiles))
    for k in [k for k in NAMES if t[k] > 0]:
        print("  %2d %-20s %9.0f  %5.1f%%" % (k, NAMES[k], t[k] / tiles, 100 * t[k] / tot))


if __name__ == "__main__":
    main()
