#!/bin/bash
# bench every config (1 GPU); stops at the first failure
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py ${ARGS} > gpurun_out/bench_sac_hopper.log 2>&1; tail -1 gpurun_out/bench_sac_hopper.log
timeout -k 10 300 python -u bench.py --config ddpg_hcheetah --cpu-seconds 5 ${ARGS} > gpurun_out/bench_ddpg_hcheetah.log 2>&1; tail -1 gpurun_out/bench_ddpg_hcheetah.log
timeout -k 10 300 python -u bench.py --config sac_ant --cpu-seconds 5 ${ARGS} > gpurun_out/bench_sac_ant.log 2>&1; tail -1 gpurun_out/bench_sac_ant.log
