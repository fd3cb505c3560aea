set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out/r06a
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_dp_ppo_shard.py > gpurun_out/r06a/tests2.log 2>&1; rc=$?
tail -3 gpurun_out/r06a/tests2.log
[ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/r06a VARIANTS="w8 w8u" PROF="w8" bash tools/ppo_scaling.sh
