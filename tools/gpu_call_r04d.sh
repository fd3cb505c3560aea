# re-run of the stepwise DP statistics tests, then bench lines (PPO, SAC Hopper, DDPG HalfCheetah)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp_stats_ranks.py "tests/test_gpu_parity.py::test_obs_stats_data_parallel_protocol_matches_union" tests/test_gpu_stats.py -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/gpu_dpstats.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_dpstats.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config ppo_hcheetah --no-cpu-baseline --no-pmc > gpurun_out/bench_ppo.log 2>&1 && tail -1 gpurun_out/bench_ppo.log | cut -c1-1200
timeout -k 10 300 python -u bench.py --config sac_hopper --no-cpu-baseline --no-pmc --no-rocprof > gpurun_out/bench_hopper.log 2>&1 && tail -1 gpurun_out/bench_hopper.log | cut -c1-600
timeout -k 10 300 python -u bench.py --config ddpg_hcheetah --no-cpu-baseline --no-pmc --no-rocprof > gpurun_out/bench_ddpg.log 2>&1 && tail -1 gpurun_out/bench_ddpg.log | cut -c1-600
