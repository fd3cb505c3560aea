#!/bin/bash
# Round-5 GPU call I: obs-statistics select A/B (abbin/stats_old = HEAD, abbin/stats_new = working tree; built
# in the container from tools/stats_bench.hip), then the statistics parity tests on the working-tree library.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/r05i; O=gpurun_out/r05i
for k in 1 2; do for v in old new; do
  timeout -k 10 120 abbin/stats_$v 10000000 17 30 > $O/ddpg_$v$k.txt 2>&1 || exit $?
  timeout -k 10 120 abbin/stats_$v 1000000 11 100 > $O/hopper_$v$k.txt 2>&1 || exit $?
  echo "== $v $k"; grep -hE "^select|pass\+sel|p99" $O/ddpg_$v$k.txt $O/hopper_$v$k.txt
done; done
timeout -k 10 900 python -u -m pytest tests/test_gpu_stats.py tests/test_gpu_ring10m.py tests/test_gpu_dp_stats_ranks.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $O/stats_tests.log 2>&1; rc=$?; tail -n 4 $O/stats_tests.log; exit $rc
