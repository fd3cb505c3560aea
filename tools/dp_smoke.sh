#!/bin/bash
# 2-rank data-parallel rehearsal on ONE GPU: both ranks on cuda:0 over gloo (CUDA tensors),
# exercising bench.py's whole N>1 path (gradient buckets, global obs statistics, max-over-ranks timing).
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
for c in ${CONFIGS:-sac_hopper}; do
SPP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --envs 1024 --config $c \
  > gpurun_out/dp_smoke_$c.log 2>&1 || { tail -30 gpurun_out/dp_smoke_$c.log; exit 1; }
tail -1 gpurun_out/dp_smoke_$c.log | cut -c1-400
done
