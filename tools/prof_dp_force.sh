#!/bin/bash
# rocprofv3 kernel stats of bench.py's DP code as a one-rank RCCL job (env:// rendezvous, no launcher)
R=${GRAFT_REPO_ROOT:-/root/repo}
C=${CONFIG:-sac_hopper}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
export SPP_DP_FORCE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29581 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_dp_$C -o run --output-format csv \
  -- python3 $R/bench.py --config $C --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-pmc > $R/gpurun_out/prof_dp_$C.log 2>&1 || { tail -20 $R/gpurun_out/prof_dp_$C.log; exit 1; }
python3 - $C <<'PY'
import csv, os, sys
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
rows = list(csv.DictReader(open(R + "/gpurun_out/prof_dp_%s/run_kernel_stats.csv" % sys.argv[1])))
print("== DP-forced", sys.argv[1])
for r in rows[:26]:
    print("%8.3f ms x%5s  %5.1f%%  total %8.3f ms  %s" % (float(r["AverageNs"]) / 1e6, r["Calls"], float(r["Percentage"]),
          float(r["TotalDurationNs"]) / 1e6, r["Name"][:80]))
PY
