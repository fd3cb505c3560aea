#!/bin/bash
# Round-5 GPU call A: the full -m gpu suite, the bf16 fc3-fusion A/B (critic-phase time), and the PPO lines:
# plain, DP-forced (one-rank RCCL through bench.py's N > 1 code: the replicated union update), and the
# one-GPU rehearsal of a world-8 rank's work.  Every step has its own time limit; the first failure ends it.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/r05a
O=gpurun_out/r05a
step() { echo "== $1"; }
step tests && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/gpu_tests.log 2>&1 && tail -3 $O/gpu_tests.log &&
step ab_fuse3 && for v in default nofuse3; do
  if [ $v = default ]; then unset SPPRL_LIB; else export SPPRL_LIB=$R/spp-rl_amd/spprl/libspprl_$v.so; fi
  timeout -k 10 300 python bench.py --config sac_ant_bf16 --steps 100 --warmup 10 --no-cpu-baseline --no-pmc \
    --no-rocprof > $O/ab_fuse3_$v.json 2> $O/ab_fuse3_$v.err || { tail -5 $O/ab_fuse3_$v.err; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d['value'],d['ms_per_step'],d['kernels_ms_per_launch'])" $O/ab_fuse3_$v.json
done && unset SPPRL_LIB &&
step ppo_plain && timeout -k 10 300 python bench.py --config ppo_hcheetah --steps 60 --warmup 6 --no-cpu-baseline \
    --no-pmc --no-rocprof > $O/ppo_plain.json 2> $O/ppo_plain.err && tail -c 600 $O/ppo_plain.json &&
step ppo_dpforce && SPP_DP_FORCE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29573 bench.py --gpus 1 --config ppo_hcheetah --steps 60 --warmup 6 \
    --no-cpu-baseline --no-pmc --no-rocprof > $O/ppo_dpforce.json 2> $O/ppo_dpforce.err && tail -c 600 $O/ppo_dpforce.json &&
step ppo_world8 && timeout -k 10 400 python bench.py --config ppo_hcheetah --rehearse-world 8 --steps 9 --warmup 3 \
    --no-cpu-baseline --no-pmc --no-rocprof > $O/ppo_world8.json 2> $O/ppo_world8.err && tail -c 900 $O/ppo_world8.json
