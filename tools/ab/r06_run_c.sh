# region profiles of the bf16 critic phase (two-tile vs one-tile prof builds) + the ACM passes A/B (PPO w1 / w8)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}; O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "acm_sgd_epoch_ragged" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for L in prof prof_old; do
  SPPRL_LIB=spp-rl_amd/spprl/libspprl_$L.so timeout -k 10 300 python -u tools/region_prof.py ant_bf16 > $O/region_$L.txt 2>&1 || exit $?
  cat $O/region_$L.txt
done
B="python -u bench.py --config ppo_hcheetah --no-cpu-baseline --no-pmc --no-rocprof --steps 12 --warmup 3"
for V in "w1 1" "w1 2" "w8 1" "w8 2" "w8 4"; do
  set -- $V; X=""; [ $1 = w8 ] && X="--rehearse-world 8"
  timeout -k 10 400 $B $X --acm-passes $2 > $O/ppo_$1_p$2.log 2>&1 || exit $?
  echo "$V $(grep '"metric"' $O/ppo_$1_p$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["us_per_sgd_step"], d["roofline"]["kernel"][:60])')"
done
