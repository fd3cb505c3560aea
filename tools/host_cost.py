"""Host-side cost (no synchronisation) of the per-epoch calls of the PPO_AcM loop: device permutations
(sppRandPerm vs torch.randperm) and the ACM epoch launch path, to find what holds the host behind the GPU."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "spp-rl_amd"), REPO]
import torch  # noqa: E402

from spprl.perm import device_randperm  # noqa: E402


def t_host(fn, reps=20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / reps * 1e6, (t2 - t0) / reps * 1e6


def main():
    dev = torch.device("cuda", 0)
    for n in (32768, 1802240):
        device_randperm(n, 1, 0, dev)
        torch.randperm(n, device=dev)
        print("n %8d  sppRandPerm host %.1f us (with GPU %.1f us)   torch.randperm host %.1f us (with GPU %.1f us)" % (
            (n,) + t_host(lambda: device_randperm(n, 1, 0, dev)) + t_host(lambda: torch.randperm(n, device=dev))))
    x = torch.empty(1802240, 34, device=dev)
    print("torch.empty 245 MB host %.1f us" % t_host(lambda: torch.empty(1802240, 34, device=dev))[0])
    print("x /= 3 host %.1f us" % t_host(lambda: x.div_(3.0))[0])


if __name__ == "__main__":
    main()
