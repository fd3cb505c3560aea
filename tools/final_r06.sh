# Round-6 end GPU evidence (gpurun -- 'STAGE=tests bash tools/final_r06.sh', 'STAGE=bench CONFIGS="..." ...'):
# the full GPU suite + smoke, or full bench lines (rocprof child, PMC passes, CPU baseline) per config.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/final06
case "$STAGE" in
  tests)
    timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final06/gpu_tests.log 2>&1; rc=$?
    tail -3 gpurun_out/final06/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > gpurun_out/final06/smoke.log 2>&1; rc=$?
    tail -2 gpurun_out/final06/smoke.log; exit $rc;;
  bench)
    for C in $CONFIGS; do
      X="--cpu-seconds 5"; [ "$C" = sac_hopper ] && X=""
      timeout -k 10 700 python -u bench.py --config $C $X --trace-dir gpurun_out/final06 > gpurun_out/final06/bench_$C.log 2>&1 || exit $?
      tail -1 gpurun_out/final06/bench_$C.log | cut -c1-240
    done;;
esac
