# Round-6 GPU call T: the ACM epochs' rows read from the replay ring inside the persistent kernel
# (sppAcmSgdEpochRing, SPP_ACM_RING=1, the default) against the gathered form (SPP_ACM_RING=0): parity tests
# (ring = gathered bit for bit), then the PPO w8 rehearsal and w1 alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r06t; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_ppo_overlap.py tests/test_gpu_dp_ppo_ring.py tests/test_gpu_onpolicy.py tests/test_gpu_obs_norm.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="python -u bench.py --config ppo_hcheetah --no-cpu-baseline --no-pmc --no-rocprof --steps 15 --warmup 3"
for t in w8_r1_a w8_r0_a w8_r1_b w8_r0_b w1_r1 w1_r0; do
  X="--rehearse-world 8"; case $t in w1*) X="";; esac
  RG=0; case $t in *r1*) RG=1;; esac
  SPP_ACM_RING=$RG timeout -k 10 400 $B $X > $O/$t.json 2> $O/$t.err || exit $?
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'],d['roofline'].get('us_per_sgd_step'))" $O/$t.json "$t" | tee -a $O/ab.txt
done
