# granule hand-off SGD: parity tests (SGD, actor epochs, DP replicated ring), PPO bench, region timing
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_onpolicy.py tests/test_gpu_dp_ppo_ring.py -m gpu -x -q --timeout 200 --timeout-method thread -k "sgd or epoch or acm or ring" > gpurun_out/gpu_sgd_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_sgd_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config ppo_hcheetah --no-cpu-baseline --no-pmc --no-rocprof > gpurun_out/bench_ppo.log 2>&1 && tail -1 gpurun_out/bench_ppo.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step']); print(d['roofline'])" || exit $?
if false; then for BS in 1049 64; do SPPRL_LIB=$R/spp-rl_amd/spprl/libspprl_prof.so timeout -k 10 120 python -u tools/sgd_prof.py $BS || exit $?; done 2>&1 | tee gpurun_out/sgd_prof.log; fi
