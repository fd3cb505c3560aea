set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_onpolicy.py "tests/test_gpu_parity.py::test_acm_persistent_sgd_matches_oracle" "tests/test_gpu_parity.py::test_acm_multi_workgroup_sgd_is_deterministic" "tests/test_gpu_parity.py::test_update_acm_epochs_with_step_lr_match_oracle" tests/test_gpu_dp_ppo_ring.py tests/test_gpu_ppo.py -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/gpu_sgd.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|\|d\|/lr|Error|assert" gpurun_out/gpu_sgd.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config ppo_hcheetah --no-cpu-baseline > gpurun_out/bench_ppo.log 2>&1 && tail -1 gpurun_out/bench_ppo.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ppo -o run --output-format csv -- python3 $R/bench.py --config ppo_hcheetah --steps 6 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_ppo.log 2>&1
python3 $R/tools/trace_busy.py $R/gpurun_out/prof_ppo/run_kernel_trace.csv 0.6 16
