#!/bin/bash
# rocprofv3 kernel-trace stats of the plain bench and of bench.py's N > 1 code on one rank (SPP_DP_FORCE=1,
# process group from env:// without a launcher), same config
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/profdp; export TMPDIR=/tmp
C=${CONFIG:-sac_hopper}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profdp/plain -o run -- python bench.py --config $C \
  --steps 50 --warmup 5 --no-cpu-baseline --no-pmc --no-rocprof > gpurun_out/profdp/plain_$C.log 2>&1 || exit 1
SPP_DP_FORCE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29573 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 timeout -k 10 300 \
  rocprofv3 --kernel-trace --stats -d gpurun_out/profdp/dp -o run -- python bench.py --config $C --steps 50 --warmup 5 \
  --no-cpu-baseline --no-pmc --no-rocprof > gpurun_out/profdp/dp_$C.log 2>&1 || exit 1
tail -1 gpurun_out/profdp/plain_$C.log | cut -c1-200; tail -1 gpurun_out/profdp/dp_$C.log | cut -c1-200
