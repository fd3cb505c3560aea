"""Device occupancy of a rocprofv3 kernel trace: over the last fraction of the run (the timed steps), the
span, the union of kernel intervals (busy), the idle gaps, and per-kernel totals.  A busy / span well below
1 means the host (launch issue, Python) or a synchronisation gates the step, not the kernels.
Usage: python tools/trace_busy.py gpurun_out/prof_X/run_kernel_trace.csv [tail_fraction=0.5] [top=15]"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    t0 = iv[0][0] + (iv[-1][1] - iv[0][0]) * (1 - frac)
    iv = [x for x in iv if x[0] >= t0]
    span = iv[-1][1] - iv[0][0]
    busy, cur_s, cur_e = 0, iv[0][0], iv[0][1]
    gaps = []
    per = defaultdict(lambda: [0, 0])
    for s, e, n in iv:
        per[n][0] += e - s
        per[n][1] += 1
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    gaps.sort()
    print("window %.3f ms, %d dispatches: busy %.3f ms (%.1f %%), idle %.3f ms in %d gaps (median %.1f us, "
          "p90 %.1f us)" % (span / 1e6, len(iv), busy / 1e6, 100.0 * busy / span, (span - busy) / 1e6, len(gaps),
                            gaps[len(gaps) // 2] / 1e3 if gaps else 0, gaps[int(len(gaps) * 0.9)] / 1e3 if gaps else 0))
    for n, (t, c) in sorted(per.items(), key=lambda kv: -kv[1][0])[:top]:
        print("  %8.3f ms %6d x %7.1f us  %s" % (t / 1e6, c, t / c / 1e3, n[:90]))


if __name__ == "__main__":
    main()
