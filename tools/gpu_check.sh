#!/bin/bash
# GPU validation: parity tests, smoke, bench, rocprof stats. Each step time-limited; stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
tail -1 gpurun_out/bench.log
if [ -n "$PROF" ]; then bash tools/prof_stats.sh; fi
