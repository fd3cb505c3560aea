# bf16 two-tile critic phase: parity (bf16 tests) then the Ant bf16 line with its rocprof child
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}; O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bigbatch.py tests/test_gpu_multistep.py tests/test_gpu_parity.py -k "bf16 or Ant or bigbatch or multistep" > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --config sac_ant_bf16 --no-cpu-baseline --no-pmc --trace-dir $O > $O/bench_ant_bf16.log 2>&1 || exit $?
grep '"metric"' $O/bench_ant_bf16.log | cut -c1-400
head -12 $O/steady_kernel_stats_sac_ant_bf16.csv
