#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/stats_prof.py ${ARGS} > $R/gpurun_out/stats_prof.log 2>&1
cat $R/gpurun_out/stats_prof.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_stats -o run --output-format csv -- python3 $R/tools/stats_prof.py ${ARGS} > /dev/null 2>&1
python3 - <<'PY'
import csv, os
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
for r in list(csv.DictReader(open(R + "/gpurun_out/prof_stats/run_kernel_stats.csv")))[:12]:
    print("%9.4f ms x%5s  %5.1f%%  %s" % (float(r["AverageNs"]) / 1e6, r["Calls"], float(r["Percentage"]), r["Name"][:80]))
PY
