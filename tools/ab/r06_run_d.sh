# (1) bf16 two-tile critic phase with the first layers one tile at a time: region profile + Ant bf16 line + parity;
# (2) the SGD arrival counter sharded over 8 lines: SGD / on-policy parity + PPO w1 / w8 lines
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}; O=gpurun_out/r06d; mkdir -p $O
SPPRL_LIB=spp-rl_amd/spprl/libspprl_prof.so timeout -k 10 300 python -u tools/region_prof.py ant_bf16 > $O/region_prof.txt 2>&1 || exit $?
head -18 $O/region_prof.txt
timeout -k 10 600 python -u bench.py --config sac_ant_bf16 --no-cpu-baseline --no-pmc --trace-dir $O > $O/bench_ant_bf16.log 2>&1 || exit $?
grep '"metric"' $O/bench_ant_bf16.log | cut -c1-200
head -4 $O/steady_kernel_stats_sac_ant_bf16.csv
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bigbatch.py tests/test_gpu_multistep.py tests/test_gpu_parity.py tests/test_gpu_onpolicy.py tests/test_gpu_ppo.py tests/test_gpu_ppo_overlap.py -k "bf16 or Ant or acm or sgd or critic or actor or ppo" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
B="python -u bench.py --config ppo_hcheetah --no-cpu-baseline --no-pmc --no-rocprof --steps 12 --warmup 3"
for V in w1 w8; do
  X=""; [ $V = w8 ] && X="--rehearse-world 8"
  timeout -k 10 400 $B $X > $O/ppo_$V.log 2>&1 || exit $?
  echo "$V $(grep '"metric"' $O/ppo_$V.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["us_per_sgd_step"])')"
done
