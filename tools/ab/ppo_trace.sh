# PPO kernel trace of the timed iterations + device occupancy (gpurun -- bash tools/ab/ppo_trace.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ppo -o run --output-format csv -- python3 $R/bench.py --config ppo_hcheetah --steps 6 --warmup 3 --no-cpu-baseline --no-pmc --no-rocprof > $R/gpurun_out/prof_ppo.log 2>&1 || exit $?
python3 $R/tools/trace_busy.py $R/gpurun_out/prof_ppo/run_kernel_trace.csv 0.6 22
