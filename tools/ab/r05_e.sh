#!/bin/bash
# Round-5 GPU call: both rsample draws in one k_eps_fm launch: staged-update parity, then configs[0] and the headline.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sac.py tests/test_gpu_bigbatch.py tests/test_gpu_c_host.py \
    tests/test_gpu_multistep.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -n 2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for C in vanilla_sac_hcheetah sac_hopper; do
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --no-pmc --no-rocprof > $O/$C.json 2> $O/$C.err \
      || { tail -5 $O/$C.err; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'])" $O/$C.json $C
done
