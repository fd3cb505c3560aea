#!/bin/bash
# Round-5 GPU call J: the grouped fixed-order dW reduce (k_dw_reduce) A/B: the bench's steady-state rocprof
# kernel summary with the HEAD library (libspprl_head.so) and with the working tree's.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/r05j; O=gpurun_out/r05j
for v in head new; do for C in sac_hopper ddpg_hcheetah; do
  if [ $v = head ]; then L=$R/spp-rl_amd/spprl/libspprl_head.so; else L=""; fi
  mkdir -p $O/$v
  SPPRL_LIB=$L timeout -k 10 400 python bench.py --config $C --no-cpu-baseline --no-pmc --trace-dir $O/$v \
      > $O/$v/$C.json 2> $O/$v/$C.err || exit $?
  python3 - $O/$v/steady_kernel_stats_$C.csv "$C $v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "dw" in r["Name"]: print(sys.argv[2], r["Name"][:40], r["Calls"], r["AverageNs"])
PY
done; done
