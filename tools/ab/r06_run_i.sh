# Round-6 GPU call I: the SGD shard reduce summed while loading (SPP_SGD_PRED=1, now the default): the persistent
# SGD's parity tests (AcM, on-policy critic / actor, PPO ring / overlap) and the PPO line at w1 and the w8 rehearsal.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r06i; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_onpolicy.py tests/test_gpu_dp_ppo_ring.py tests/test_gpu_ppo_overlap.py tests/test_gpu_dp_ppo_shard.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
B="python -u bench.py --config ppo_hcheetah --no-cpu-baseline --no-pmc --no-rocprof --steps 12 --warmup 3"
timeout -k 10 400 $B > $O/ppo_w1.json 2> $O/ppo_w1.err || exit $?
timeout -k 10 400 $B --rehearse-world 8 > $O/ppo_w8.json 2> $O/ppo_w8.err || exit $?
for w in w1 w8; do
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'],d['roofline'].get('us_per_sgd_step'))" $O/ppo_$w.json "ppo $w" | tee -a $O/ppo.txt
done
