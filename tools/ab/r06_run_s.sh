# Round-6 GPU call S: the ACM epochs' rows prepared ahead on a prep stream (SPP_ACM_PREP_AHEAD=1) now that the
# ring's permutation is one O(n) launch, against the serial order: PPO w8 rehearsal alternating twice, w1 once each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r06s; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ppo_overlap.py \
  tests/test_gpu_dp_ppo_ring.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
SPP_ACM_PREP_AHEAD=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_ppo_overlap.py tests/test_gpu_dp_ppo_ring.py tests/test_gpu_parity.py -k "acm or ppo or ring" \
  > $O/tests_prep.log 2>&1 || { tail -30 $O/tests_prep.log; exit 1; }
tail -1 $O/tests.log; tail -1 $O/tests_prep.log
B="python -u bench.py --config ppo_hcheetah --no-cpu-baseline --no-pmc --no-rocprof --steps 15 --warmup 3"
for t in w8_p1_a w8_p0_a w8_p1_b w8_p0_b w1_p1 w1_p0; do
  X="--rehearse-world 8"; case $t in w1*) X="";; esac
  P=0; case $t in *p1*) P=1;; esac
  SPP_ACM_PREP_AHEAD=$P timeout -k 10 400 $B $X > $O/$t.json 2> $O/$t.err || exit $?
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'],d['roofline'].get('us_per_sgd_step'))" $O/$t.json "$t" | tee -a $O/ab.txt
done
