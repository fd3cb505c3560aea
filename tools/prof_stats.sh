#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run -> gpurun_out/prof/run_kernel_stats.csv
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv \
  -- python3 $R/bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof.log 2>&1
python3 - <<'PY'
import csv, os
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
rows = list(csv.DictReader(open(R + "/gpurun_out/prof/run_kernel_stats.csv")))
for r in rows[:25]:
    print("%8.3f ms x%4s  %5.1f%%  %s" % (float(r["AverageNs"]) / 1e6, r["Calls"], float(r["Percentage"]), r["Name"][:90]))
PY
python3 - <<'PY'
import csv, os
from collections import defaultdict
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
# per-grid breakdown of the multi-launch kernels (e.g. the three k_dw launches of a step)
d = defaultdict(list)
for r in csv.DictReader(open(R + "/gpurun_out/prof/run_kernel_trace.csv")):
    n = r["Kernel_Name"]
    if n.startswith("spp::k_dw"):
        d[(n[:20], r.get("Grid_Size", r.get("Grid_Size_X", "?")))].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, v in sorted(d.items()):
    print("%-22s grid %-8s x%3d  avg %.3f ms" % (k[0], k[1], len(v), sum(v) / len(v)))
PY
