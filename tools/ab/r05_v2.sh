#!/bin/bash
# Round-5 GPU call X: host side of the PPO iteration's device idle: kernel + HIP API trace of the plain PPO line;
# for every device-idle gap > 50 us, the HIP API calls the host was inside during it (tools/gap_api.py).
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/r05v2; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --hip-trace -d $O/prof -o run --output-format csv -- python3 $R/bench.py \
    --config vanilla_sac_hcheetah --steps 800 --warmup 100 --no-cpu-baseline --no-pmc --no-rocprof > $O/bench.log 2>&1 \
    || { tail -5 $O/bench.log; exit 1; }
ls $O/prof/*/ 2>/dev/null | head -20
K=$(find $O/prof -name "*kernel_trace.csv" | head -1); H=$(find $O/prof -name "*hip_api_trace.csv" | head -1)
python3 $R/tools/gap_api.py $K $H > $O/gaps.txt && head -c 6000 $O/gaps.txt
gzip -k $K $H
