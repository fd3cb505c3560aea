#!/bin/bash
# Round-end measurement set (1 GPU): full GPU suite, every bench config (with PMC traffic and the CPU
# baselines), rocprofv3 kernel stats of the main configs. Stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
TMO=700 bash tools/gpu_tests.sh
bash tools/bench_all.sh
for C in sac_hopper sac_ant_bf16 ddpg_hcheetah; do CONFIG=$C STEPS=10 bash tools/prof_config.sh; done
