#!/bin/bash
# Round-5 GPU call G: bf16 LDS-input layer A/B (weight ring depth, output-block chains) on the SAC Ant bf16
# line per library (HIP events, no rocprof / PMC), then the bf16 GPU tests on the variant library.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/r05g; O=gpurun_out/r05g
for v in ${VARIANTS:-default obc}; do
  if [ $v = default ]; then L=""; else L=spp-rl_amd/spprl/libspprl_$v.so; fi
  SPPRL_LIB=$L timeout -k 10 300 python bench.py --config sac_ant_bf16 --no-cpu-baseline --no-pmc --no-rocprof \
      > $O/ant_$v.json 2> $O/ant_$v.err || exit $?
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['avg_launch_ms'])" $O/ant_$v.json $v
done
SPPRL_LIB=spp-rl_amd/spprl/libspprl_obc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_multistep.py tests/test_gpu_bigbatch.py tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $O/obc_tests.log 2>&1; rc=$?; tail -n 3 $O/obc_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_dp_rccl.py -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/dp_tests.log 2>&1; rc=$?; tail -n 8 $O/dp_tests.log; exit $rc
