#!/bin/bash
# bench.py's N > 1 code as a one-rank RCCL job (SPP_DP_FORCE=1) beside the plain N = 1 run, same
# config: the difference is the cost of the DP exchange code at N = 1 (stepwise global obs
# statistics, bucket all-reduces, host row-count exchange), RCCL latency across GPUs excluded.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
C=${CONFIG:-sac_hopper}
SPP_DP_FORCE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 1 --config $C --steps ${STEPS:-100} --warmup 10 \
  --no-cpu-baseline --no-pmc > gpurun_out/dp_force_$C${TAG}.log 2>&1 || { tail -20 gpurun_out/dp_force_$C${TAG}.log; exit 1; }
python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print('dp-forced' + sys.argv[3], sys.argv[2], d['value'], d['ms_per_step'], d['kernels_ms_per_launch'])" gpurun_out/dp_force_$C${TAG}.log $C "${TAG}"
