#!/bin/bash
# Round-5 GPU call K: the dW / update / on-policy parity tests on the working-tree library (grouped dW reduce).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/r05k; O=gpurun_out/r05k
timeout -k 10 1000 python -u -m pytest tests/test_gpu_multistep.py tests/test_gpu_bigbatch.py tests/test_gpu_sac.py tests/test_gpu_ddpg.py \
    tests/test_gpu_dp_sac_union.py tests/test_gpu_onpolicy.py tests/test_gpu_parity.py tests/test_gpu_ppo.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -n 3 $O/tests.log; exit $rc
