#!/bin/bash
# Round-5 end: quick lines of the other configs on the final library (no CPU baseline / PMC / rocprof child).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r05chk; mkdir -p $O
for C in sac_ant_bf16 sac_ant ddpg_hcheetah; do
  timeout -k 10 400 python bench.py --config $C --no-cpu-baseline --no-pmc --no-rocprof > $O/$C.json 2> $O/$C.err \
      || { tail -5 $O/$C.err; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'])" $O/$C.json $C
done
