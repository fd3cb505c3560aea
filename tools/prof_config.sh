#!/bin/bash
# rocprofv3 kernel stats for one bench config: CONFIG=ddpg_hcheetah bash tools/prof_config.sh
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
C=${CONFIG:-sac_hopper}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$C -o run --output-format csv \
  -- python3 $R/bench.py --config $C --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-pmc > $R/gpurun_out/prof_$C.log 2>&1
python3 - $C <<'PY'
import csv, os, sys
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
rows = list(csv.DictReader(open(R + "/gpurun_out/prof_%s/run_kernel_stats.csv" % sys.argv[1])))
print("==", sys.argv[1])
for r in rows[:22]:
    print("%8.3f ms x%4s  %5.1f%%  %s" % (float(r["AverageNs"]) / 1e6, r["Calls"], float(r["Percentage"]), r["Name"][:90]))
PY
