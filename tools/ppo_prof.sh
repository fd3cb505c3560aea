#!/bin/bash
# PPO config: bench line + rocprofv3 kernel stats (gpurun_out/prof_ppo)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
timeout -k 10 300 python -u bench.py --config ppo_hcheetah > gpurun_out/bench_ppo.log 2>&1; tail -1 gpurun_out/bench_ppo.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ppo -o run --output-format csv -- python3 $R/bench.py --config ppo_hcheetah --steps 3 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_ppo.log 2>&1
python3 - <<'PY'
import csv, os
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
rows = list(csv.DictReader(open(R + "/gpurun_out/prof_ppo/run_kernel_stats.csv")))
for r in rows[:16]:
    print("%8.3f ms x%6s  %5.1f%%  %s" % (float(r["AverageNs"]) / 1e6, r["Calls"], float(r["Percentage"]), r["Name"][:80]))
PY
