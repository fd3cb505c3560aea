#!/bin/bash
# Round-5 GPU call M: the 2-wave AcM SGD form (-DSPP_ACM_WV=2: 32 rows per workgroup, 33 workgroups per 1049-row
# step) against the default 4-wave form, on the PPO line (HIP events around each ACM epoch launch), then the ACM
# parity tests on the variant library.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/r05m; O=gpurun_out/r05m
for v in default wv2 default wv2; do
  if [ $v = default ]; then L=""; else L=$R/spp-rl_amd/spprl/libspprl_$v.so; fi
  SPPRL_LIB=$L timeout -k 10 300 python bench.py --config ppo_hcheetah --steps 30 --warmup 3 --no-cpu-baseline --no-pmc \
      --no-rocprof > $O/ppo_$v.json 2> $O/ppo_$v.err || { tail -5 $O/ppo_$v.err; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);r=d['roofline'];print(sys.argv[2],d['value'],d['ms_per_step'],r['us_per_sgd_step'],r['kernel'][:40])" $O/ppo_$v.json $v
done
SPPRL_LIB=$R/spp-rl_amd/spprl/libspprl_wv2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ppo_overlap.py \
    tests/test_gpu_dp_ppo_ring.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -n 3 $O/tests.log; exit $rc
