set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
echo "== A/B: old capped candidate count (expect caps0 FAIL, caps1 pass)"
SPPRL_LIB=$R/spp-rl_amd/spprl/libspprl_oldncd.so timeout -k 10 300 python -u -m pytest "tests/test_gpu_stats.py::test_obs_stats_one_pass_protocol_overflow_counts_every_candidate" -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/ab_oldncd.log 2>&1; echo "old lib pytest rc=$?"
grep -E "PASSED|FAILED|Mismatch|x: |y: " gpurun_out/ab_oldncd.log | head -12
echo "== SGD region profile"
SPPRL_LIB=$R/spp-rl_amd/spprl/libspprl_prof.so timeout -k 10 120 python -u tools/sgd_prof.py 64 > gpurun_out/sgd_prof_64.txt 2>&1 && cat gpurun_out/sgd_prof_64.txt
SPPRL_LIB=$R/spp-rl_amd/spprl/libspprl_prof.so timeout -k 10 120 python -u tools/sgd_prof.py 1049 > gpurun_out/sgd_prof_1049.txt 2>&1 && cat gpurun_out/sgd_prof_1049.txt
echo "== PPO trace"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ppo -o run --output-format csv -- python3 $R/bench.py --config ppo_hcheetah --steps 3 --warmup 3 --no-cpu-baseline --no-pmc --no-rocprof > $R/gpurun_out/prof_ppo.log 2>&1
tail -1 $R/gpurun_out/prof_ppo.log | cut -c1-300
python3 $R/tools/trace_busy.py $R/gpurun_out/prof_ppo/run_kernel_trace.csv 0.5 20
