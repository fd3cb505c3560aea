#!/bin/bash
# Round-5 GPU call T: fp32 weight gradients of every job up to 256 x 256 on the LDS-staged k_dw_big (default) vs the
# round-4 routing (-DSPP_DW_LDS_MID=0: only 256 x 256 jobs there, the rest in k_dw), per fp32 config (bench rocprof
# child: steady per-kernel summary); then the dW / update parity tests on the default library.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/r05t; O=gpurun_out/r05t
for C in sac_hopper ddpg_hcheetah sac_ant; do for v in new nomid; do
  if [ $v = new ]; then L=""; else L=$R/spp-rl_amd/spprl/libspprl_$v.so; fi
  mkdir -p $O/$v
  SPPRL_LIB=$L timeout -k 10 400 python bench.py --config $C --no-cpu-baseline --no-pmc --trace-dir $O/$v \
      > $O/$v/$C.json 2> $O/$v/$C.err || { tail -5 $O/$v/$C.err; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'])" $O/$v/$C.json "$C $v"
  python3 - $O/$v/steady_kernel_stats_$C.csv "$C $v" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
n = int(rows[0]["Calls"])
print("   ", sys.argv[2], [(r["Name"][5:20], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6 / n, 3)) for r in rows if "k_dw" in r["Name"]])
PY
done; done
timeout -k 10 900 python -u -m pytest tests/test_gpu_multistep.py tests/test_gpu_bigbatch.py tests/test_gpu_ddpg.py tests/test_gpu_sac.py \
    tests/test_gpu_parity.py tests/test_gpu_ring10m.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -n 3 $O/tests.log; exit $rc
