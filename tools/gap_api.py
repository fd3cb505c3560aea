"""Device-idle gaps of a rocprofv3 kernel trace attributed to the host: for each gap (> 50 us, last 60 % of the
run), the HIP API calls overlapping it (the host was blocked in them) and the time the host spent outside any HIP
call (Python).  Usage: gap_api.py KERNEL_TRACE.csv HIP_API_TRACE.csv"""
import bisect
import csv
import sys
from collections import defaultdict

krows = list(csv.DictReader(open(sys.argv[1])))
hrows = list(csv.DictReader(open(sys.argv[2])))
kv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].replace("void ", "")[:50],
             int(r.get("Correlation_Id", 0) or 0)) for r in krows)
api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"], int(r.get("Correlation_Id", 0) or 0))
             for r in hrows)
launch_of = {c: (s, e, f) for s, e, f, c in api}
t0 = kv[0][0] + (kv[-1][1] - kv[0][0]) * 0.4
kv = [x for x in kv if x[0] >= t0]
api_starts = [a[0] for a in api]
gaps = []
cur_e, prev = kv[0][1], kv[0][2]
for s, e, n, c in kv[1:]:
    if s > cur_e + 50000:
        gaps.append((cur_e, s, prev, n, c))
    if e > cur_e:
        cur_e, prev = e, n
tot = sum(b - a for a, b, *_ in gaps)
print("gaps > 50 us in window: %d, total %.1f ms (window %.1f ms)" % (len(gaps), tot / 1e6, (kv[-1][1] - t0) / 1e6))
blocked = defaultdict(float)
outside = 0.0
lat = []
bykind = defaultdict(lambda: [0.0, 0, defaultdict(float)])
for a, b, pn, nn, c in gaps:
    i = max(0, bisect.bisect_left(api_starts, a) - 200)
    cov = []
    for s, e, f, _ in api[i:]:
        if s > b:
            break
        if e > a:
            ov = min(e, b) - max(s, a)
            if ov > 0:
                cov.append((max(s, a), min(e, b), f))
    # union of API coverage of the gap
    cov.sort()
    u, ce = 0, a
    for s, e, f in cov:
        if e > ce:
            u += e - max(s, ce)
            ce = e
        blocked[f] += (e - s) / 1e3
    outside += (b - a - u) / 1e3
    L = launch_of.get(c)
    lat.append(((b - a) / 1e3, (L[0] - a) / 1e3 if L else None, L[2] if L else "?"))
    k = bykind[(pn[:34], nn[:40])]
    k[0] += (b - a) / 1e3
    k[1] += 1
    for s, e, f in cov:
        k[2][f] += (e - s) / 1e3
print("host outside HIP calls during gaps: %.1f ms" % (outside / 1e3))
print("HIP calls overlapping gaps (us, summed):")
for f, t in sorted(blocked.items(), key=lambda kv: -kv[1])[:15]:
    print("  %10.1f  %s" % (t, f))
print("gap kinds (kernel before -> after): total us, count, top overlapping calls")
for (p, n), (t, cnt, fs) in sorted(bykind.items(), key=lambda kv: -kv[1][0])[:20]:
    top = ", ".join("%s %.0f" % (f, v) for f, v in sorted(fs.items(), key=lambda kv: -kv[1])[:3])
    print("%9.1f %4d  %-34s -> %-40s | %s" % (t, cnt, p, n, top))
print("largest gaps: (us, launch API start after gap start us, launch fn)")
for g in sorted(lat, key=lambda x: -x[0])[:15]:
    print("  %9.1f  %s  %s" % g)
