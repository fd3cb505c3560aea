#!/bin/bash
# Wave-state breakdown of the kernels of a short bench run (one rocprofv3 --pmc pass of 8 SQ-block
# counters): WAIT_ANY (s_waitcnt / barrier), WAIT_INST_ANY (issue stalls: MFMA dependency, pipe,
# instruction fetch), ACTIVE_INST_ANY, instruction mix and L1I hits / misses.
# Summary -> gpurun_out/pmc_sq.txt.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
   SQ_INSTS_VALU SQ_INSTS_MFMA SQC_ICACHE_HITS SQC_ICACHE_MISSES \
   -d $R/gpurun_out/pmc_sq -o run --output-format csv \
   -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --config ${BENCH_CONFIG:-sac_hopper} > $R/gpurun_out/pmc_sq.log 2>&1
python3 - "$R/gpurun_out/pmc_sq" > $R/gpurun_out/pmc_sq.txt <<'EOF'
import csv, glob, os, sys
from collections import defaultdict
tot = defaultdict(lambda: defaultdict(float))
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "?").replace("void ", "").split("(")[0][:60]
        tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:12]:
    w = c.get("SQ_WAVE_CYCLES", 0) or 1
    ic = (c.get("SQC_ICACHE_HITS", 0) + c.get("SQC_ICACHE_MISSES", 0)) or 1
    print("%-60s wave_qcyc %.3g  wait %.1f%%  issue_stall %.1f%%  active %.1f%%  valu %.3g  mfma %.3g  "
          "icache_miss %.2f%% (%.3g)" % (
              k, w, 100 * c["SQ_WAIT_ANY"] / w, 100 * c["SQ_WAIT_INST_ANY"] / w, 100 * c["SQ_ACTIVE_INST_ANY"] / w,
              c["SQ_INSTS_VALU"], c["SQ_INSTS_MFMA"], 100 * c.get("SQC_ICACHE_MISSES", 0) / ic,
              c.get("SQC_ICACHE_MISSES", 0)))
EOF
cat $R/gpurun_out/pmc_sq.txt
