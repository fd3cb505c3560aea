#!/bin/bash
# Round-5 GPU call U: obs-statistics pass A/B for wide rows (ob > 64): rows in flight per lane (SPP_ST_UNROLL_W) and
# pass workgroups per CU (SPP_ST_WPE), tools/stats_bench.hip builds in abbin/ (made in the container).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/r05u; O=gpurun_out/r05u
for v in w4_4 w6_3 w8_3 w8_2 w12_2 w4_4; do
  for shape in "1000000 111 50" "1000000 11 50" "10000000 17 20"; do
    set -- $shape
    timeout -k 10 120 abbin/stats_$v $1 $2 $3 > $O/${v}_$2.txt 2>&1 || { cat $O/${v}_$2.txt; exit 1; }
    echo "$v ob=$2 $(grep -E '^pass ' $O/${v}_$2.txt | tr -s ' ') | $(grep -E '^select' $O/${v}_$2.txt | tr -s ' ') | $(grep p99 $O/${v}_$2.txt | awk '{print $NF}')"
  done
done
