set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out/r06a
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_obs_norm.py tests/test_gpu_unbiased.py tests/test_gpu_dp_ppo_union.py tests/test_gpu_dp_ppo_ring.py tests/test_gpu_ppo.py tests/test_gpu_ppo_overlap.py > gpurun_out/r06a/tests.log 2>&1; rc=$?
tail -15 gpurun_out/r06a/tests.log
[ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/r06a VARIANTS="w1 w8 w8u" PROF="w8" bash tools/r06_ppo.sh
