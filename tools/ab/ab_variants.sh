#!/bin/bash
# A/B of library variants (tools/build_variant.py TAG ...): short bench runs per config and variant,
# printing env-steps/s and the HBM kernels' per-call times.
#   VARIANTS="default stagev1" CONFIGS="sac_ant_bf16 sac_hopper" bash tools/ab/ab_variants.sh
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
for c in ${CONFIGS:-sac_ant_bf16 sac_hopper}; do
  for v in ${VARIANTS:-default}; do
    if [ $v = default ]; then unset SPPRL_LIB; else export SPPRL_LIB=$R/spp-rl_amd/spprl/libspprl_$v.so; fi
    timeout -k 10 240 python bench.py --config $c --steps ${STEPS:-60} --warmup 5 --no-cpu-baseline --no-pmc --no-rocprof \
      > gpurun_out/ab_${c}_$v.json 2> gpurun_out/ab_${c}_$v.err || { tail -5 gpurun_out/ab_${c}_$v.err; exit 1; }
    python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d['value'],d['ms_per_step'],{k:v['ms'] for k,v in d['hbm_kernels'].items()})" gpurun_out/ab_${c}_$v.json
  done
done
