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

NAMES = {0: "prefetch issue", 1: "fc1", 2: "d3 stores, b3 sums", 11: "fc2", 12: "fc3", 13: "head", 3: "dz2, dz1, image barrier", 4: "dW loop exit",
         5: "bias sums, scalars, barrier", 14: "slab drain, arrival 1 wait", 6: "shard fetch + sum",
         7: "Adam, publish, next rows", 15: "publish drain, arrival 2 wait", 8: "reload",
         9: "  dW pair MFMAs", 10: "  dW pair stores"}


def report(name, K, G, el, buf):
    v = np.array(buf[:32], dtype=np.float64) / (4 * K * G)  # waves 0..3 of every workgroup recorded
    tot = v.sum()
    print("%s: %d steps in %.3f ms (%.2f us/step); cycles per step per wave: %.0f" % (name, K, el * 1e3, el * 1e6 / K, tot))
    for k in (0, 1, 11, 12, 13, 2, 3, 4, 5, 14, 6, 7, 15, 8, 9, 10):
        print("  %2d %-28s %8.0f  %5.1f%%" % (k, NAMES[k], v[k], 100 * v[k] / tot))


def actor(dev):
    """The PPO actor epoch (k_mlp_sgd<17, 64, 17, 1>): 32,768 rows in 512-row minibatches (8 workgroups)."""
    from spprl.onpolicy import OnPolicyNets
    N, mb = 32768, 512
    n = OnPolicyNets(17, 17, ac_lim=1.0, max_batch=N, device=dev, seed=0)
    x = torch.randn(N, 17, device=dev)
    act = torch.rand(N, 17, device=dev) * 2 - 1
    lp = torch.randn(N, device=dev) - 20
    adv = torch.randn(N, device=dev)
    perm = torch.randperm(N, device=dev)
    outs = torch.empty(N // mb, 4, device=dev)
    st = _lib.stream_handle()
    args = [n._h] + [_lib.ptr(t) for t in (x, act, lp, adv, act, perm)] + [N, mb, _lib.ptr(outs), st]
    _lib.call("sppOnpActorEpoch", *args)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 64)()
    _lib.call("sppDebugReadProf", buf, 1)
    t0 = time.perf_counter()
    _lib.call("sppOnpActorEpoch", *args)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    _lib.call("sppDebugReadProf", buf, 1)
    report("k_mlp_sgd<17, 64, 17, 1> (actor epoch, 512-row steps)", N // mb, mb // 64, el, buf)


def main():
    dev = torch.device("cuda", 0)
    if len(sys.argv) > 1 and sys.argv[1] == "actor":
        return actor(dev)
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
    report("k_mlp_sgd<34, 32, 6, 0> (%d-row steps)" % bs, K, -(-bs // 64), el, buf)


if __name__ == "__main__":
    main()
