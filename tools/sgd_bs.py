"""Timing of one persistent AcM SGD launch at the PPO bench's batch: python tools/sgd_bs.py [bs] [steps]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "spp-rl_amd"), REPO]
import torch  # noqa: E402

import spprl  # noqa: E402
from spprl import _lib  # noqa: E402

bs = int(sys.argv[1]) if len(sys.argv) > 1 else 1049
K = int(sys.argv[2]) if len(sys.argv) > 2 else 400
dev = torch.device("cuda", 0)
ob, ac = 17, 6
ag = spprl.SAC_AcM(env_name="HalfCheetah-v2", max_batch=max(4096, bs), buffer_size=20_000, device=dev, seed=0)
x = torch.randn(K * bs, 2 * ob, device=dev)
y = torch.rand(K * bs, ac, device=dev) * 2 - 1
loss = torch.zeros(1, device=dev)
st = _lib.stream_handle()
for _ in range(2):
    _lib.call("sppAcmSgd", ag._h, _lib.ptr(x), _lib.ptr(y), K, bs, _lib.ptr(loss), st)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    _lib.call("sppAcmSgd", ag._h, _lib.ptr(x), _lib.ptr(y), K, bs, _lib.ptr(loss), st)
torch.cuda.synchronize()
el = (time.perf_counter() - t0) / 3
print("lib=%s bs=%d: %.2f us per SGD step (%d steps, loss %.5f)" % (os.environ.get("SPPRL_LIB", "default"), bs,
                                                                    el * 1e6 / K, K, float(loss)))
