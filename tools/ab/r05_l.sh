#!/bin/bash
# Round-5 GPU call L: SQ wave-state and instruction-mix counters of the phase kernels (two rocprofv3 --pmc passes
# of <= 8 SQ counters each, every pass its own run) for the bf16 Ant and the fp32 Hopper configs.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r05l; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM"
for C in sac_ant_bf16 sac_hopper; do
  for p in 1 2; do
    if [ $p = 1 ]; then PC=$P1; else PC=$P2; fi
    timeout -s KILL 240 rocprofv3 --pmc $PC -d $O/${C}_p$p -o run --output-format csv \
      -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-rocprof --config $C \
      > $O/${C}_p$p.log 2>&1 || { tail -5 $O/${C}_p$p.log; exit 1; }
  done
done
python3 - $O > $O/summary.txt <<'PY'
import csv, glob, os, sys
from collections import defaultdict
for C in ("sac_ant_bf16", "sac_hopper"):
    tot = defaultdict(lambda: defaultdict(float))
    for p in (1, 2):
        for f in glob.glob(os.path.join(sys.argv[1], "%s_p%d" % (C, p), "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r.get("Kernel_Name", "?").replace("void ", "").split("(")[0][:48]
                key = r["Counter_Name"] + ("" if r["Counter_Name"] != "SQ_WAVE_CYCLES" else "_p%d" % p)
                tot[name][key] += float(r["Counter_Value"])
    print("==", C)
    for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES_p1", 0))[:6]:
        w = c.get("SQ_WAVE_CYCLES_p1", 0) or 1
        m = c.get("SQ_INSTS_MFMA", 0) or 1
        print("%-48s wait %.1f%%  issue_stall %.1f%%  active %.1f%% | per MFMA: valu %.2f lds %.2f salu %.2f vmem_rd %.2f "
              "vmem_wr %.2f smem %.2f | lds_bank_conflict/lds %.3f" % (
                  k, 100 * c["SQ_WAIT_ANY"] / w, 100 * c["SQ_WAIT_INST_ANY"] / w, 100 * c["SQ_ACTIVE_INST_ANY"] / w,
                  c["SQ_INSTS_VALU"] / m, c["SQ_INSTS_LDS"] / m, c["SQ_INSTS_SALU"] / m, c.get("SQ_INSTS_VMEM_RD", 0) / m,
                  c.get("SQ_INSTS_VMEM_WR", 0) / m, c.get("SQ_INSTS_SMEM", 0) / m,
                  c.get("SQ_LDS_BANK_CONFLICT", 0) / max(1.0, c.get("SQ_ACTIVE_INST_LDS", 1.0))))
PY
cat $O/summary.txt
