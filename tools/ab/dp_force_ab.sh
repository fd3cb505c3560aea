#!/bin/bash
# DP-forced overhead per config: the plain N = 1 bench against bench.py's N > 1 code run as a one-rank RCCL
# job (SPP_DP_FORCE=1): one-pass obs statistics over libspprl's communicator (the default), the same over
# torch.distributed, and the stepwise statistics protocol.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
for C in ${CONFIGS:-sac_hopper sac_ant_bf16 ddpg_hcheetah}; do
  timeout -k 10 300 python bench.py --config $C --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline --no-pmc \
    --no-rocprof > gpurun_out/dpab_plain_$C.log 2>&1 || { tail -20 gpurun_out/dpab_plain_$C.log; exit 1; }
  for P in onepass torchcomm stepwise; do
    case $P in
      onepass) E="SPP_DP_STATS=onepass"; A="--dp-comm native" ;;
      torchcomm) E="SPP_DP_STATS=onepass"; A="--dp-comm torch" ;;
      stepwise) E="SPP_DP_STATS=stepwise"; A="--dp-comm native" ;;
    esac
    env $E SPP_DP_FORCE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 1 --config $C --steps ${STEPS:-100} --warmup 10 \
      --no-cpu-baseline --no-pmc --no-rocprof $A > gpurun_out/dpab_${P}_$C.log 2>&1 || { tail -20 gpurun_out/dpab_${P}_$C.log; exit 1; }
  done
  for T in plain onepass torchcomm stepwise; do
    python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" gpurun_out/dpab_${T}_$C.log $C $T
  done
done
