#!/bin/bash
# Root-cause A/B of the round-2 "wrong values under VGPR spills" finding: the spilling one-kernel
# Ant actor phase (worktree of 8f1cc8c^ at _old) against the same source with a compiler memory
# barrier at each cross-lane LDS hand-over (_old2, tools' xlane patch).  Same test, same seed.
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
for t in _old _old2; do
  cd $R/$t
  timeout -k 10 300 python -u -m pytest tests/test_gpu_bigbatch.py -m gpu -x -v -s --timeout 240 --timeout-method thread \
    -k "Ant-v2-111-8-4096-False or Ant-v2-111-8-4096-acmc0" > $R/gpurun_out/xlane_$t.log 2>&1
  echo "== $t rc=$?"
  grep -E "PASSED|FAILED|Error|assert|loss" $R/gpurun_out/xlane_$t.log | head -12
done
