#!/bin/bash
# Round-5 GPU call D: the 8-wave (two waves per SIMD) AcM kernel: its parity / PPO tests, the PPO line, and the
# hardware-queue test of the DP-forced overlap (tools/ab/r05_c.sh).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/r05d; O=gpurun_out/r05d
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ppo_overlap.py tests/test_gpu_dp_ppo_ring.py \
  tests/test_gpu_dp_ppo_union.py tests/test_gpu_onpolicy.py tests/test_trainer.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1 && tail -2 $O/tests.log &&
timeout -k 10 300 python bench.py --config ppo_hcheetah --steps 60 --warmup 6 --no-cpu-baseline --no-pmc --no-rocprof \
  > $O/ppo.json 2> $O/ppo.err &&
python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print('ppo',d['value'],d['ms_per_step'],d['roofline'].get('us_per_sgd_step'),d['roofline']['kernel'][:60])" $O/ppo.json &&
bash tools/ab/r05_c.sh
