#!/bin/bash
# Round-5 GPU call O: the plain-C host of the C-ABI (examples/c_host/sac_acm_step, built in the container by
# spp-rl_amd/build.py) against the Python host on the same SAC_AcM state and data.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/r05o; O=gpurun_out/r05o
timeout -k 10 300 python -u -m pytest tests/test_gpu_c_host.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > $O/tests.log 2>&1; rc=$?; tail -n 30 $O/tests.log; exit $rc
