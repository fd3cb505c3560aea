#!/bin/bash
# Round-5 GPU call H: obs-statistics kernel timings (tools/stats_bench.hip: DDPG 1e7 x 17, Hopper 1e6 x 11; a repeated
# call = pass + select), then the RCCL one-rank tests (exchange overlap on / off, plain vs DP-forced).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/r05h; O=gpurun_out/r05h
hipcc --offload-arch=gfx950 -O3 -std=c++17 -o $O/stats_bench tools/stats_bench.hip || exit 1
timeout -k 10 120 $O/stats_bench 10000000 17 20 > $O/stats_ddpg.txt 2>&1; rc=$?; cat $O/stats_ddpg.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 $O/stats_bench 1000000 11 50 > $O/stats_hopper.txt 2>&1; rc=$?; cat $O/stats_hopper.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_dp_rccl.py -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/dp_tests.log 2>&1; rc=$?; tail -n 8 $O/dp_tests.log; exit $rc
