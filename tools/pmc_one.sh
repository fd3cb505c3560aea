#!/bin/bash
# usage: pmc_one.sh <kernel-regex> "<counters pass 1>" ["<counters pass 2>" ...]
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
re=$1; shift
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "$re" -d $R/gpurun_out/pmc1_$i -o run --output-format csv \
     -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc1_$i.log 2>&1
done
python3 - "$i" <<'PY'
import csv, collections, os, sys
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for i in range(1, int(sys.argv[1]) + 1):
    for r in csv.DictReader(open(R + "/gpurun_out/pmc1_%d/run_counter_collection.csv" % i)):
        agg[(r["Kernel_Name"][:60], r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print("   %-28s %.4g (n=%d)" % (c, sum(v) / len(v), len(v)))
PY
