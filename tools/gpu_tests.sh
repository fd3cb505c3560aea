#!/bin/bash
# Run a subset (or all) of the GPU tests on the box: TESTS="tests/x.py -k y" bash tools/gpu_tests.sh
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 ${TMO:-900} python -u -m pytest ${TESTS:-tests} ${K:+-k "$K"} -m gpu -x -v -s --timeout ${PER_TEST:-300} --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
grep -E "PASSED|FAILED|ERROR|grad rel err|passed|failed" gpurun_out/gpu_tests.log | tail -80
