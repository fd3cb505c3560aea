# Round-6 GPU call M: the ACM SGD's weight-gradient pair stores issued under the next pair's MFMAs (variant dwd,
# SPP_SGD_DWDELAY=1) against the default: tools/sgd_bs.py at w1 / w8 alternating twice, SGD parity tests on dwd.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r06m; mkdir -p $O
L=spp-rl_amd/spprl
for v in default dwd default dwd; do
  lib=$L/libspprl.so; [ $v != default ] && lib=$L/libspprl_$v.so
  for bs in 1049 8389; do
    SPPRL_LIB=$lib timeout -k 10 120 python -u tools/sgd_bs.py $bs 400 2>&1 | grep "us per" | sed "s/^/$v /" | tee -a $O/sgd_bs.txt || exit $?
  done
done
SPPRL_LIB=$L/libspprl_dwd.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_onpolicy.py > $O/tests_dwd.log 2>&1 || { tail -30 $O/tests_dwd.log; exit 1; }
tail -2 $O/tests_dwd.log
