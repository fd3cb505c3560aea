# Round-6 GPU call E: (1) the DP exchange-beside-compute order re-measured with bench.py's 8 hardware queues: SAC
# Hopper one-rank RCCL rehearsal (SPP_DP_FORCE=1) with SPP_DP_OVERLAP=0 / 1 beside the plain line, and a kernel trace
# of the overlapped run with each kernel's queue; (2) PPO's N > 1 code path (sharded update, per-step exchange) as a
# one-rank RCCL job beside the plain line; (3) the Ant bf16 line on the default (one-tile) library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r06e; mkdir -p $O
B="python -u bench.py --no-cpu-baseline --no-pmc --no-rocprof"
timeout -k 10 300 $B --config sac_hopper --steps 100 --warmup 10 > $O/hopper_plain.json 2> $O/hopper_plain.err || exit $?
for ov in 0 1; do
  SPP_DP_FORCE=1 SPP_DP_OVERLAP=$ov timeout -k 10 300 $B --config sac_hopper --steps 100 --warmup 10 \
      > $O/hopper_dp_ov$ov.json 2> $O/hopper_dp_ov$ov.err || exit $?
done
for v in plain dp_ov0 dp_ov1; do
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'],d.get('param_checksum'))" $O/hopper_$v.json "hopper $v"
done
(cd /tmp && export TMPDIR=/tmp SPP_DP_FORCE=1 SPP_DP_OVERLAP=1 && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/kt_ov1 -o run \
    --output-format csv -- python3 $R/bench.py --config sac_hopper --steps 12 --warmup 3 --no-cpu-baseline --no-pmc \
    --no-rocprof > $R/$O/kt_ov1.log 2>&1) || exit $?
F=$(find $O/kt_ov1 -name "*kernel_trace.csv" | head -1)
python3 tools/trace_busy.py $F 0.5 12 > $O/trace_ov1_busy.txt
python3 - $F > $O/trace_ov1_step.txt <<'PY'
import csv, sys
from collections import Counter
rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60], r.get("Queue_Id", "?"),
             r.get("Stream_Id", "?")) for r in rows)
cs = [i for i, x in enumerate(iv) if "k_sac_critic_phase" in x[2]]
a, b = cs[len(cs) // 2], cs[len(cs) // 2 + 1]
t0 = iv[a][0]
print("one step of the overlapped DP-forced run (us from the critic phase start, duration, queue, stream):")
for s, e, n, q, st in iv[a:b + 1]:
    print("%9.1f %8.1f  q%s s%s  %s" % ((s - t0) / 1e3, (e - s) / 1e3, q, st, n))
print("queues over the whole trace:", Counter(x[3] for x in iv))
PY
head -5 $O/trace_ov1_step.txt; tail -1 $O/trace_ov1_step.txt
timeout -k 10 400 $B --config ppo_hcheetah --steps 12 --warmup 3 > $O/ppo_plain.json 2> $O/ppo_plain.err || exit $?
SPP_DP_FORCE=1 timeout -k 10 400 $B --config ppo_hcheetah --steps 12 --warmup 3 > $O/ppo_dp.json 2> $O/ppo_dp.err || exit $?
for v in plain dp; do
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'],d['config'].get('update_batch','')[:90])" $O/ppo_$v.json "ppo $v"
done
timeout -k 10 600 python -u bench.py --config sac_ant_bf16 --no-cpu-baseline --no-pmc --no-rocprof > $O/ant_bf16.json 2>$O/ant_bf16.err || exit $?
grep '"metric"' $O/ant_bf16.json | cut -c1-160
