#!/bin/bash
# Round-5 GPU call N: rocprofv3 --kernel-trace --stats over the default bench command (sac_hopper, 20 timed steps;
# the bench's own rocprof / PMC children off, so the stats cover this one process), for profiles/r05/final/.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r05n; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py \
    --steps 20 --warmup 3 --no-cpu-baseline --no-pmc --no-rocprof > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
head -8 $O/kernel_stats.csv | cut -c1-200; grep '^{' $O/bench.log | tail -n 1 | cut -c1-300
