# full GPU suite, then quick bench lines (PPO, SAC Hopper) and a PPO kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/gpu_full.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_full.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config ppo_hcheetah --no-cpu-baseline --no-pmc > gpurun_out/bench_ppo.log 2>&1 && tail -1 gpurun_out/bench_ppo.log | cut -c1-900
timeout -k 10 300 python -u bench.py --config sac_hopper --no-cpu-baseline --no-pmc --no-rocprof > gpurun_out/bench_hopper.log 2>&1 && tail -1 gpurun_out/bench_hopper.log | cut -c1-700
