"""Region timing of the persistent MLP SGD kernel (k_mlp_sgd<34, 32, 6, 0>) at the PPO HalfCheetah AcM shape
(AcM in 34, out 6; argv[1] = batch rows, 1049 = the bench's).  Profiling build:
python spp-rl_amd/build.py --prof --hopper-only --hcheetah, then
SPPRL_LIB=spp-rl_amd/spprl/libspprl_prof.so python tools/sgd_prof.py [bs]"""
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "spp-rl_amd"), REPO]
import torch  # noqa: E402

import spprl  # noqa: E402
from spprl import _lib  # noqa: E402

NAMES = {0: "stage rows, prefetch", 1: "fc1", 2: "fc2, fc3, loss, dz2", 3: "dz1", 4: "gradient tiles, bias sums",
         5: "canonical staging", 6: "slab stores, barrier 1", 7: "shard reduce, Adam, publish",
         8: "barrier 2, reload", 9: "  dW pair MFMAs", 10: "  dW pair stores"}


def main():
    dev = torch.device("cuda", 0)
    ob, ac, K = 17, 6, 400
    bs = int(sys.argv[1]) if len(sys.argv) > 1 else 1049  # > 64: the multi-workgroup form
    ag = spprl.SAC_AcM(env_name="HalfCheetah-v2", max_batch=max(4096, bs), buffer_size=40_000, device=dev, seed=0)
    rb = ag.replay_buffer
    n = 20_000
    slots = rb.add_obs_batch(torch.randn(n + 1, ob, device=dev))
    rb.add_timestep_batch(slots[:n], slots[1:], torch.randn(n, ob, device=dev), torch.randn(n, device=dev),
                          torch.zeros(n, dtype=torch.uint8, device=dev), torch.zeros(n, dtype=torch.uint8, device=dev),
                          torch.rand(n, ac, device=dev) * 2 - 1)
    idx = torch.randint(0, n, (K * bs,), device=dev)
    x = torch.empty(K * bs, 2 * ob, device=dev)
    y = torch.empty(K * bs, ac, device=dev)
    loss = torch.zeros(1, device=dev)
    st = _lib.stream_handle()
    _lib.call("sppReplayGatherAcm", rb._h, _lib.ptr(idx), K * bs, _lib.ptr(x), _lib.ptr(y), st)
    _lib.call("sppAcmSgd", ag._h, _lib.ptr(x), _lib.ptr(y), K, bs, _lib.ptr(loss), st)  # warm-up
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 64)()
    _lib.call("sppDebugReadProf", buf, 1)
    t0 = time.perf_counter()
    _lib.call("sppAcmSgd", ag._h, _lib.ptr(x), _lib.ptr(y), K, bs, _lib.ptr(loss), st)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    _lib.call("sppDebugReadProf", buf, 1)
    G = -(-bs // 64)
    v = np.array(buf[:32], dtype=np.float64) / (4 * K * G)  # waves 0..3 of every workgroup recorded
    tot = v.sum()
    print("k_mlp_sgd<34, 32, 6, 0>: %d steps of %d in %.3f ms (%.2f us/step); cycles per step per wave: %.0f"
          % (K, bs, el * 1e3, el * 1e6 / K, tot))
    for k in range(11):
        print("  %2d %-20s %8.0f  %5.1f%%" % (k, NAMES[k], v[k], 100 * v[k] / tot))


if __name__ == "__main__":
    main()
