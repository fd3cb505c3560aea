#!/bin/bash
# bench every config (1 GPU); stops at the first failure. CONFIGS="sac_hopper sac_ant_bf16" to pick.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
for C in ${CONFIGS:-sac_hopper ddpg_hcheetah sac_ant sac_ant_bf16 ppo_hcheetah vanilla_sac_hcheetah}; do
  X="--cpu-seconds 5"; [ $C = sac_hopper ] && X=""
  timeout -k 10 400 python -u bench.py --config $C $X ${ARGS} > gpurun_out/bench_$C.log 2>&1
  tail -1 gpurun_out/bench_$C.log
done
