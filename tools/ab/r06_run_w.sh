# Round-6 GPU call W: the fused data-parallel steps write their gradients times 1 / ranks (no per-step mul
# launch after the all-reduce): on-policy / DP PPO tests, then the w8 rehearsal and the DP-forced w1 line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r06w; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_onpolicy.py \
  tests/test_gpu_dp_ppo_shard.py tests/test_gpu_dp_ppo_union.py tests/test_gpu_dp_ppo_ring.py tests/test_gpu_ppo_overlap.py \
  tests/test_gpu_parity.py tests/test_gpu_dp_rccl.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="python -u bench.py --config ppo_hcheetah --no-cpu-baseline --no-pmc --no-rocprof --steps 15 --warmup 3"
timeout -k 10 400 $B --rehearse-world 8 > $O/w8.json 2> $O/w8.err || exit $?
SPP_DP_FORCE=1 timeout -k 10 400 $B > $O/w1dp.json 2> $O/w1dp.err || exit $?
for t in w8 w1dp; do
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'],d['roofline'].get('us_per_sgd_step'))" $O/$t.json "$t" | tee -a $O/ab.txt
done
