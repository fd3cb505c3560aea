#!/bin/bash
# bench.py runs on the box, each under its own time limit: CONFIGS="sac_hopper vanilla_sac_hcheetah" EXTRA="--no-pmc"
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
for c in ${CONFIGS:-sac_hopper}; do
  timeout -k 10 ${TMO:-600} python -u bench.py --config $c ${EXTRA} > gpurun_out/bench_$c.log 2>&1 || { tail -30 gpurun_out/bench_$c.log; exit 1; }
  tail -1 gpurun_out/bench_$c.log
done
