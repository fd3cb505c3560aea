#!/bin/bash
# Round-5 GPU call E: full -m gpu suite, the default bench (sac_hopper, full fields), the PPO plain / DP-forced pair
# (8 HW queues now set by bench.py), and the Ant bf16 line.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/r05e; O=gpurun_out/r05e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
tail -2 $O/gpu_tests.log &&
timeout -k 10 600 python bench.py > $O/bench_sac_hopper.json 2> $O/bench_sac_hopper.err && tail -c 400 $O/bench_sac_hopper.json &&
timeout -k 10 300 python bench.py --config ppo_hcheetah --steps 60 --warmup 6 --no-cpu-baseline --no-pmc --no-rocprof \
  > $O/ppo_plain.json 2> $O/ppo_plain.err &&
SPP_DP_FORCE=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29591 timeout -k 10 300 \
  python bench.py --gpus 1 --config ppo_hcheetah --steps 60 --warmup 6 --no-cpu-baseline --no-pmc --no-rocprof \
  > $O/ppo_dpforce.json 2> $O/ppo_dpforce.err &&
timeout -k 10 300 python bench.py --config sac_ant_bf16 --steps 100 --warmup 10 --no-cpu-baseline --no-pmc --no-rocprof \
  > $O/ant_bf16.json 2> $O/ant_bf16.err &&
for f in ppo_plain ppo_dpforce ant_bf16; do
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[1],d['value'],d['ms_per_step'],d['roofline'].get('frac'))" $O/$f.json
done
