#!/bin/bash
# Round-5 GPU call: host profile (cProfile) of the vanilla SAC configs[0] loop (reference schedule).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r05hp; mkdir -p $O
timeout -k 10 400 python -m cProfile -o $O/v.prof bench.py --config vanilla_sac_hcheetah --steps 1000 --warmup 100 \
    --no-cpu-baseline --no-pmc --no-rocprof > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 - $O/v.prof > $O/prof.txt <<'PY'
import pstats, sys
p = pstats.Stats(sys.argv[1])
p.sort_stats("tottime").print_stats(35)
p.sort_stats("cumulative").print_stats(60)
PY
