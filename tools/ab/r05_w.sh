#!/bin/bash
# Round-5 GPU call W: the PPO host loop: on-policy parity tests, the plain PPO line (actor-epoch permutations drawn up
# front), then a host-side profile (cProfile) of the bench loop: where the host spends the iteration while the
# device idles (tools/ab/r05_v.sh's kernel trace: ~16 % device idle).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/r05w; O=gpurun_out/r05w
timeout -k 10 600 python -u -m pytest tests/test_gpu_onpolicy.py tests/test_gpu_ppo_overlap.py tests/test_gpu_dp_ppo_union.py \
    tests/test_gpu_ppo.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -n 2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config ppo_hcheetah --steps 60 --warmup 6 --no-cpu-baseline --no-pmc --no-rocprof \
    > $O/ppo_plain.json 2> $O/ppo_plain.err || { tail -5 $O/ppo_plain.err; exit 1; }
python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print('ppo', d['value'],d['ms_per_step'],d['roofline']['us_per_sgd_step'])" $O/ppo_plain.json
timeout -k 10 400 python -m cProfile -o $O/ppo.prof bench.py --config ppo_hcheetah --steps 12 --warmup 3 \
    --no-cpu-baseline --no-pmc --no-rocprof > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 - $O/ppo.prof > $O/prof.txt <<'PY'
import pstats, sys
p = pstats.Stats(sys.argv[1])
p.sort_stats("tottime").print_stats(30)
p.sort_stats("cumulative").print_stats(40)
PY
