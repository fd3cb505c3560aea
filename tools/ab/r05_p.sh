#!/bin/bash
# Round-5 GPU call P: SAC_AcM / DDPG_AcM updates at ragged and minimal batches (B = 1, 31, 33, 1001) against the
# float64 oracle, with the rest of the big-batch file.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/r05p; O=gpurun_out/r05p
timeout -k 10 900 python -u -m pytest tests/test_gpu_bigbatch.py -m gpu -v --timeout 300 --timeout-method thread \
    > $O/tests.log 2>&1; rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -n 40; exit $rc
