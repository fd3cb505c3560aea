# Round-6 GPU call P: (1) the ACM epochs' permutations + row gathers prepared ahead on a prep stream
# (SPP_ACM_PREP_AHEAD=1, the default) against the serial order; (2) the data-parallel clip-loss steps through the
# epoch kernel's gradient-only launch (sppOnpActorStepGrads) beside the fused critic step (SPP_ONP_FUSED_GRADS=0:
# the phase-kernel paths).  ACM / on-policy / DP PPO tests, then the w8 rehearsal (A default, B prep off, C fused
# off) alternating twice and the w1 line (A, B).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r06p; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_ppo_overlap.py tests/test_gpu_dp_ppo_ring.py tests/test_gpu_dp_ppo_shard.py tests/test_gpu_onpolicy.py \
  tests/test_gpu_dp_ppo_union.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="python -u bench.py --config ppo_hcheetah --no-cpu-baseline --no-pmc --no-rocprof --steps 15 --warmup 3"
run() {  # tag, env..., then extra bench args after --
  tag=$1; shift
  env "$@" timeout -k 10 400 $B $EXTRA > $O/$tag.json 2> $O/$tag.err || return $?
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'],d['roofline'].get('us_per_sgd_step'))" $O/$tag.json "$tag" | tee -a $O/ab.txt
}
export EXTRA="--rehearse-world 8"
for i in 1 2; do
  run w8_A_$i SPP_ACM_PREP_AHEAD=1 || exit $?
  run w8_B_$i SPP_ACM_PREP_AHEAD=0 || exit $?
  run w8_C_$i SPP_ONP_FUSED_GRADS=0 || exit $?
done
export EXTRA=""
run w1_A SPP_ACM_PREP_AHEAD=1 || exit $?
run w1_B SPP_ACM_PREP_AHEAD=0 || exit $?
