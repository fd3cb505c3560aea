# Round-6 GPU call K: the ACM SGD with the shard's Adam spread one element per thread and branch-free row prefetch
# (variant acm2) against the default: tools/sgd_bs.py at w1 / w8 (alternating twice), the SGD parity tests on the
# variant, and the Hopper phase kernels' top-level region profile (nodense profiling library).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r06k; mkdir -p $O
L=spp-rl_amd/spprl
for v in default acm2 default acm2; do
  lib=$L/libspprl.so; [ $v != default ] && lib=$L/libspprl_$v.so
  for bs in 1049 8389; do
    SPPRL_LIB=$lib timeout -k 10 120 python -u tools/sgd_bs.py $bs 400 2>&1 | grep "us per" | sed "s/^/$v /" | tee -a $O/sgd_bs.txt || exit $?
  done
done
SPPRL_LIB=$L/libspprl_acm2.so timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_onpolicy.py tests/test_gpu_dp_ppo_ring.py tests/test_gpu_ppo_overlap.py \
  tests/test_gpu_dp_ppo_shard.py > $O/tests_acm2.log 2>&1 || { tail -30 $O/tests_acm2.log; exit 1; }
tail -2 $O/tests_acm2.log
SPPRL_LIB=$L/libspprl_prof.so timeout -k 10 300 python -u tools/region_prof.py > $O/region_hopper_nodense.txt 2>&1 || exit $?
cat $O/region_hopper_nodense.txt
