#!/bin/bash
# Round-5 GPU call: configs[0] as R independent runs sharing the GPU (bench.py --replicas), R = 1, 4, 8, 15.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r05rep; mkdir -p $O
for N in ${NS:-4 8 15}; do
  timeout -k 10 400 python bench.py --config vanilla_sac_hcheetah --replicas $N --no-cpu-baseline --no-pmc --no-rocprof \
      > $O/rep$N.json 2> $O/rep$N.err || { tail -5 $O/rep$N.err; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print('replicas',sys.argv[2],d['value'],d['ms_per_step'],d['replicas']['per_replica_value'])" $O/rep$N.json $N
done
