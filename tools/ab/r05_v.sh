#!/bin/bash
# Round-5 GPU call V: where the PPO iteration leaves the device idle: kernel trace of the plain PPO line, gaps summed
# by the kernel that precedes them (tools/trace_busy.py for the totals).
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r05v; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 $R/bench.py \
    --config ppo_hcheetah --steps 9 --warmup 3 --no-cpu-baseline --no-pmc --no-rocprof > $O/bench.log 2>&1 \
    || { tail -5 $O/bench.log; exit 1; }
F=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_busy.py $F 0.6 8
python3 - $F <<'PY'
import csv, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].replace("void ", "")[:60]) for r in rows)
t0 = iv[0][0] + (iv[-1][1] - iv[0][0]) * 0.4
iv = [x for x in iv if x[0] >= t0]
gap_by = defaultdict(lambda: [0.0, 0])
cur_e, prev = iv[0][1], iv[0][2]
for s, e, n in iv[1:]:
    if s > cur_e:
        g = (s - cur_e) / 1e3
        gap_by[(prev, n)][0] += g
        gap_by[(prev, n)][1] += 1
    if e > cur_e:
        cur_e, prev = e, n
print("idle gaps by (kernel before -> kernel after), top 20 by total us:")
for (a, b), (t, c) in sorted(gap_by.items(), key=lambda kv: -kv[1][0])[:20]:
    print("%9.1f us %5d x  %-40s -> %s" % (t, c, a[:40], b[:50]))
PY
