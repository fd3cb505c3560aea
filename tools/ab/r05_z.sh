#!/bin/bash
# Round-5 GPU call Z: vanilla SAC reference schedule with the sampled indices uploaded through pinned memory
# (async) instead of a pageable copy (a stream sync per grad step): parity, then the configs[0] line.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r05z; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_sac.py tests/test_gpu_parity.py tests/test_gpu_unbiased.py tests/test_gpu_stats.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -n 3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --config vanilla_sac_hcheetah --no-cpu-baseline --no-pmc --no-rocprof \
      > $O/bench$i.json 2> $O/bench$i.err || { tail -5 $O/bench$i.err; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print('vanilla',d['value'],d['ms_per_step'])" $O/bench$i.json
done
