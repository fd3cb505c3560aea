"""Host time per C-ABI entry point over a bench run: wraps every libspprl function that spprl._lib.call
reaches with a wall-clock timer.  Usage: python tools/call_probe.py <bench.py args>"""
import os
import sys
import time
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "spp-rl_amd"))
from spprl import _lib  # noqa: E402

T = defaultdict(lambda: [0.0, 0])


class Proxy:
    def __init__(self, lib):
        self._l = lib

    def __getattr__(self, name):
        f = getattr(self._l, name)

        def w(*a):
            t0 = time.perf_counter()
            r = f(*a)
            d = T[name]
            d[0] += time.perf_counter() - t0
            d[1] += 1
            return r
        return w


_lib._lib = Proxy(_lib.load())
sys.argv = ["bench.py"] + sys.argv[1:]
import bench  # noqa: E402

bench.main()
tot = sum(v[0] for v in T.values())
print("C-ABI host time %.1f ms over %d calls" % (tot * 1e3, sum(v[1] for v in T.values())), file=sys.stderr)
for k, (t, n) in sorted(T.items(), key=lambda kv: -kv[1][0])[:25]:
    print("%10.1f ms %7d x %8.1f us  %s" % (t * 1e3, n, t / n * 1e6, k), file=sys.stderr)
