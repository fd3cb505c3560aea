#!/bin/bash
# Round-5 GPU call Q: bench.py's N > 1 code as a one-rank RCCL job (SPP_DP_FORCE=1, native communicator) for SAC
# Hopper and DDPG HalfCheetah, exchange overlap on (default) and off (SPP_DP_OVERLAP=0), beside the plain lines.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/r05q; O=gpurun_out/r05q
P=29611
for C in sac_hopper ddpg_hcheetah; do
  timeout -k 10 300 python bench.py --config $C --steps 100 --warmup 10 --no-cpu-baseline --no-pmc --no-rocprof \
      > $O/${C}_plain.json 2> $O/${C}_plain.err || exit $?
  for ov in 1 0; do
    P=$((P+1))
    SPP_DP_FORCE=1 SPP_DP_OVERLAP=$ov timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port $P bench.py --gpus 1 --config $C --steps 100 --warmup 10 \
        --no-cpu-baseline --no-pmc --no-rocprof > $O/${C}_dp_ov$ov.json 2> $O/${C}_dp_ov$ov.err || exit $?
  done
  for v in plain dp_ov1 dp_ov0; do
    python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'],d.get('param_checksum'))" $O/${C}_$v.json "$C $v"
  done
done
