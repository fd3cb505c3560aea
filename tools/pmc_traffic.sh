#!/bin/bash
# HBM traffic per kernel launch: two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE),
# each over a short bench run; summary -> gpurun_out/pmc_traffic.json (gfx950 FETCH_SIZE x2 correction,
# MI355X_MICROARCH.md "HBM").
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_$c -o run --output-format csv \
     -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --config ${BENCH_CONFIG:-sac_hopper} > $R/gpurun_out/pmc_$c.log 2>&1
done
python3 $R/tools/pmc_summarize.py $R/gpurun_out
