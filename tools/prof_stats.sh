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
