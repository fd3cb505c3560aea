#!/bin/bash
# Round-5 GPU call R: kernel trace of the one-rank RCCL rehearsal (SPP_DP_FORCE=1) with the exchange overlap on,
# to find what the overlap serialises (bench.py run directly under rocprofv3 with the rank environment exported).
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r05r; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29655 SPP_DP_FORCE=1 SPP_DP_OVERLAP=${OV:-1}
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof$OV -o run --output-format csv -- python3 $R/bench.py --gpus 1 \
    --config sac_hopper --steps 12 --warmup 3 --no-cpu-baseline --no-pmc --no-rocprof > $O/bench$OV.log 2>&1 \
    || { tail -5 $O/bench$OV.log; exit 1; }
F=$(find $O/prof$OV -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_busy.py $F 0.5 12
python3 - $F <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print("columns:", list(rows[0].keys()))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60], r.get("Queue_Id", "?"),
             r.get("Stream_Id", "?")) for r in rows)
# one step in the middle of the timed window: from a critic-phase start to the next
cs = [i for i, x in enumerate(iv) if "k_sac_critic_phase" in x[2]]
a, b = cs[len(cs) // 2], cs[len(cs) // 2 + 1]
t0 = iv[a][0]
for s, e, n, q, st in iv[a:b + 1]:
    print("%9.1f %8.1f  q%s s%s  %s" % ((s - t0) / 1e3, (e - s) / 1e3, q, st, n))
PY
