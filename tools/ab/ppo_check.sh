# PPO path check: SGD / critic / permutation parity tests and the PPO bench line (gpurun -- bash tools/ab/ppo_check.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo_overlap.py tests/test_gpu_onpolicy.py tests/test_gpu_parity.py tests/test_gpu_dp_ppo_ring.py tests/test_gpu_bigbatch.py -m gpu -x -q -s --timeout 200 --timeout-method thread -k "sgd or epoch or acm or ring or critic or onpolicy or actor or act or rand_perm or overlap" > gpurun_out/gpu_sgd_tests.log 2>&1; rc=$?
grep -E "^N [0-9]+:|passed|failed" gpurun_out/gpu_sgd_tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config ppo_hcheetah --no-cpu-baseline --no-pmc --no-rocprof > gpurun_out/bench_ppo.log 2>&1 && tail -1 gpurun_out/bench_ppo.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['us_per_sgd_step'], d['losses'])"
