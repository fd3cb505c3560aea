#!/bin/bash
# Round-5 GPU call Y: the small-batch team kernels of vanilla SAC (csrc/sac_team.h): parity, then the configs[0]
# line with the team kernels (default) and with SPP_SAC_TEAM=0 (the one-wave kernels), same library.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r05y; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sac.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > $O/tests.log 2>&1; rc=$?; tail -n 12 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for T in 1 0 1 0; do
  SPP_SAC_TEAM=$T timeout -k 10 300 python bench.py --config vanilla_sac_hcheetah --no-cpu-baseline --no-pmc --no-rocprof \
      > $O/bench_team$T.json 2> $O/bench_team$T.err || { tail -5 $O/bench_team$T.err; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);r=d['roofline'];print('team',sys.argv[2],d['value'],d['ms_per_step'],{k:v for k,v in r.items() if 'ms' in k})" $O/bench_team$T.json $T
done
