"""Collect per-rank results of spawned multi-process tests without hanging on a dead rank."""
import queue
import time


def collect(q, procs, timeout=240):
    """{rank: rest} from the (rank, *rest) tuples the workers put on q; fails as soon as a worker
    exits non-zero (a rank that died would otherwise leave the test waiting for the full timeout)."""
    res, t0 = {}, time.time()
    while len(res) < len(procs):
        try:
            r = q.get(timeout=5)
            res[r[0]] = r[1:]
        except queue.Empty:
            assert all(p.exitcode in (None, 0) for p in procs), "a rank died: exit codes %s" % [
                p.exitcode for p in procs]
            assert time.time() - t0 < timeout, "ranks did not report within %d s" % timeout
    return res
