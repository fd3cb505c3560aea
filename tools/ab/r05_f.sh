#!/bin/bash
# Round-5 GPU call F: the timestep-record replay layout: full -m gpu suite (ring / sampling / last_rollout /
# staged-update parity, the new DP SAC union test), then the default bench line (hbm_kernels).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out/r05f; O=gpurun_out/r05f
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -m5 -B2 -A25 "FAILED\|Error" $O/gpu_tests.log | head -80; exit $rc; }
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench_sac_hopper.json 2> $O/bench_sac_hopper.err &&
python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac']);print(d['hbm_kernels']);print(d.get('pmc_bytes_per_launch'))" $O/bench_sac_hopper.json
