# region timing of k_mlp_sgd (baseline profiling build), then the SGD parity tests and the PPO bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
for L in prof_base prof; do for BS in 1049 64; do echo "== $L $BS"; SPPRL_LIB=$R/spp-rl_amd/spprl/libspprl_$L.so timeout -k 10 120 python -u tools/sgd_prof.py $BS || exit $?; done; done 2>&1 | tee gpurun_out/sgd_prof.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_onpolicy.py -m gpu -x -q --timeout 200 --timeout-method thread -k "sgd or epoch or acm" > gpurun_out/gpu_sgd_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_sgd_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config ppo_hcheetah --no-cpu-baseline --no-pmc > gpurun_out/bench_ppo.log 2>&1 && tail -1 gpurun_out/bench_ppo.log | cut -c1-300 && tail -1 gpurun_out/bench_ppo.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['roofline'])"
