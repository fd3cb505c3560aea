#!/bin/bash
# Round-5 GPU call S: the LDS-staged bf16 weight-gradient kernel (k_dw_big16) A/B on the SAC Ant bf16 line (bench
# rocprof child: steady per-kernel summary), default library vs -DSPP_DW_BIG16=0; then the bf16 parity tests.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/r05s; O=gpurun_out/r05s
for v in new nobig16; do
  if [ $v = new ]; then L=""; else L=$R/spp-rl_amd/spprl/libspprl_$v.so; fi
  mkdir -p $O/$v
  SPPRL_LIB=$L timeout -k 10 400 python bench.py --config sac_ant_bf16 --no-cpu-baseline --no-pmc --trace-dir $O/$v \
      > $O/$v/ant_bf16.json 2> $O/$v/ant_bf16.err || { tail -5 $O/$v/ant_bf16.err; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'],d['kernels_ms_per_launch'])" $O/$v/ant_bf16.json $v
  python3 - $O/$v/steady_kernel_stats_sac_ant_bf16.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "dw" in r["Name"]: print(sys.argv[2], r["Name"][:40], r["Calls"], r["AverageNs"])
PY
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_multistep.py tests/test_gpu_bigbatch.py tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -n 3 $O/tests.log; exit $rc
