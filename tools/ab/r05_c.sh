#!/bin/bash
# DP-forced PPO: is the lost ACM overlap a hardware-queue collision between the ACM side stream and the main
# stream once the NCCL process group's streams exist?  Same run with GPU_MAX_HW_QUEUES 4 (box default) and 8.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/r05c; O=gpurun_out/r05c
A="--config ppo_hcheetah --steps 30 --warmup 6 --no-cpu-baseline --no-pmc --no-rocprof"
for Q in 4 8; do
  GPU_MAX_HW_QUEUES=$Q SPP_DP_FORCE=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=2958$Q \
    timeout -k 10 300 python bench.py --gpus 1 $A > $O/dp_q$Q.json 2> $O/dp_q$Q.err || { tail -5 $O/dp_q$Q.err; exit 1; }
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py $A > $O/plain_q$Q.json 2> $O/plain_q$Q.err || { tail -5 $O/plain_q$Q.err; exit 1; }
  for f in dp_q$Q plain_q$Q; do
    python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[1],d['value'],d['ms_per_step'])" $O/$f.json
  done
done
