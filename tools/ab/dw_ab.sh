#!/bin/bash
# k_dw per-dispatch durations per library variant (rocprofv3 kernel trace of a short bench run):
#   VARIANTS="default dwr32" CONFIG=sac_hopper bash tools/ab/dw_ab.sh
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
C=${CONFIG:-sac_hopper}
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-default}; do
  if [ $v = default ]; then unset SPPRL_LIB; else export SPPRL_LIB=$R/spp-rl_amd/spprl/libspprl_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/dwab_${C}_$v -o run --output-format csv \
    -- python3 $R/bench.py --config $C --steps 6 --warmup 2 --no-cpu-baseline --no-pmc --no-rocprof > $R/gpurun_out/dwab_${C}_$v.log 2>&1
  echo "== $C $v"
  python3 $R/tools/trace_kernels.py $R/gpurun_out/dwab_${C}_$v/run_kernel_trace.csv "k_dw<" k_sac_critic_phase k_ddpg_critic_phase
done
