"""Device permutations for the shuffled epochs (DataLoader(shuffle=True): rltoolkit/acm/acm.py:275,
acm/on_policy.py:176-190) through sppRandPerm: Philox keys + a radix sort, stream-ordered with no host
synchronisation (torch.randperm on the device stalls the stream between its kernels).  The permutation is a
function of (seed, offset) only.  One scratch buffer per (device, stream), grown to the largest n seen (a
growing ACM ring asks for a new n every update; concurrent streams never share one)."""
import torch

from . import _lib
from ._lib import call, ptr, stream_handle

_scratch = {}


def device_randperm(n, seed, offset, device):
    """A uniform random permutation of [0, n) as an int64 device tensor (counters offset .. offset + n - 1 of
    the seed's Philox stream)."""
    n = int(n)
    out = torch.empty(n, dtype=torch.int64, device=device)
    if n == 0:
        return out
    st = stream_handle()
    key = (str(device), int(st.value or 0))  # (the stream's handle value: one buffer per stream)
    nb = int(_lib.load().sppRandPermScratchBytes(n))
    buf = _scratch.get(key)
    if buf is None or buf.numel() < nb:
        buf = torch.empty(nb, dtype=torch.uint8, device=device)
        _scratch[key] = buf
    call("sppRandPerm", ptr(out), n, int(seed) & (2**64 - 1), int(offset) & (2**64 - 1), ptr(buf), buf.numel(), st)
    return out
