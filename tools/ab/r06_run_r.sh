# Round-6 GPU call R: sppRandPerm's Feistel path for n >= 2^20 (the ACM rings' epoch permutations): permutation /
# parity tests, then the PPO w8 rehearsal twice and the w1 line (against profiles/r06/ppo/ab_prep_ahead_and_fused_actor.txt
# runs B: 65.9 / 65.7 ms, w1 45.24 ms, the same code with the radix-sort permutation).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r06r; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bigbatch.py \
  tests/test_gpu_parity.py tests/test_gpu_ppo_overlap.py tests/test_gpu_dp_ppo_ring.py tests/test_gpu_onpolicy.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="python -u bench.py --config ppo_hcheetah --no-cpu-baseline --no-pmc --no-rocprof --steps 15 --warmup 3"
for t in w8_1 w8_2 w1; do
  X="--rehearse-world 8"; [ $t = w1 ] && X=""
  timeout -k 10 400 $B $X > $O/$t.json 2> $O/$t.err || exit $?
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'],d['roofline'].get('us_per_sgd_step'))" $O/$t.json "$t" | tee -a $O/ab.txt
done
