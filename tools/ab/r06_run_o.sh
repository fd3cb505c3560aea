# Round-6 GPU call O: the data-parallel critic step through the persistent kernel's gradient-only launch
# (sppOnpCriticStepGrads) -- on-policy / DP PPO tests, then the PPO w8 rehearsal and the DP-forced w1 line with the
# fused step (default) against the phase-kernel path (SPP_ONP_FUSED_GRADS=0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r06o; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_onpolicy.py \
  tests/test_gpu_dp_ppo_shard.py tests/test_gpu_dp_ppo_union.py tests/test_gpu_dp_ppo_ring.py tests/test_gpu_ppo_overlap.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2; grep "fused vs" $O/tests.log
B="python -u bench.py --config ppo_hcheetah --no-cpu-baseline --no-pmc --no-rocprof --steps 15 --warmup 3"
for fz in 1 0 1 0; do
  SPP_ONP_FUSED_GRADS=$fz timeout -k 10 400 $B --rehearse-world 8 > $O/w8_f$fz.json 2> $O/w8_f$fz.err || exit $?
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'],d['roofline'].get('us_per_sgd_step'))" $O/w8_f$fz.json "w8 fused=$fz" | tee -a $O/ab.txt
done
for fz in 1 0; do
  SPP_DP_FORCE=1 SPP_ONP_FUSED_GRADS=$fz timeout -k 10 400 $B > $O/w1dp_f$fz.json 2> $O/w1dp_f$fz.err || exit $?
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'])" $O/w1dp_f$fz.json "w1 DP-forced fused=$fz" | tee -a $O/ab.txt
done
