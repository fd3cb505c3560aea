#!/bin/bash
# A/B: default operand-store cache policy vs nt (libspprl_nt.so), short bench runs.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
for c in sac_ant_bf16 sac_hopper; do
  for v in default nt; do
    if [ $v = nt ]; then export SPPRL_LIB=$R/spp-rl_amd/spprl/libspprl_nt.so; else unset SPPRL_LIB; fi
    timeout -k 10 240 python bench.py --config $c --steps 60 --warmup 5 --no-cpu-baseline --no-pmc \
      > gpurun_out/ab_${c}_$v.json 2> gpurun_out/ab_${c}_$v.err || { tail -5 gpurun_out/ab_${c}_$v.err; exit 1; }
    python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d['value'],d['kernels_ms_per_launch'])" gpurun_out/ab_${c}_$v.json
  done
done
