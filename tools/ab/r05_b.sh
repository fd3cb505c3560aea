#!/bin/bash
# Round-5 GPU call B: kernel traces of the PPO line, plain against DP-forced (one-rank RCCL, bench.py's N > 1 code,
# started with the rank env set directly: no launcher under the profiler), device occupancy and per-kernel totals.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p $R/gpurun_out/r05b
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/r05b
A="--config ppo_hcheetah --steps 9 --warmup 3 --no-cpu-baseline --no-pmc --no-rocprof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_plain -o run --output-format csv -- python3 $R/bench.py $A \
  > $O/plain.log 2>&1 &&
python3 $R/tools/trace_busy.py $O/prof_plain/run_kernel_trace.csv 0.6 25 > $O/busy_plain.txt &&
SPP_DP_FORCE=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29575 timeout -k 10 300 \
  rocprofv3 --kernel-trace --stats -d $O/prof_dp -o run --output-format csv -- python3 $R/bench.py --gpus 1 $A \
  > $O/dp.log 2>&1 &&
python3 $R/tools/trace_busy.py $O/prof_dp/run_kernel_trace.csv 0.6 25 > $O/busy_dp.txt &&
head -8 $O/busy_plain.txt $O/busy_dp.txt
