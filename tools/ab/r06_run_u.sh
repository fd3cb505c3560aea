# Round-6 GPU call U: the persistent SGD's tanh as one rational approximation (variant ftanh, SPP_SGD_FAST_TANH=1;
# <= 5 ulp on the float grid) against the two-branch form: SGD / on-policy / PPO parity and fixture tests on the
# variant, tools/sgd_bs.py at w1 / w8 alternating, PPO w1 line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r06u; mkdir -p $O
L=spp-rl_amd/spprl
SPPRL_LIB=$L/libspprl_ftanh.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_onpolicy.py tests/test_gpu_ppo_overlap.py tests/test_gpu_dp_ppo_shard.py \
  tests/test_gpu_dp_ppo_ring.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in default ftanh default ftanh; do
  lib=$L/libspprl.so; [ $v != default ] && lib=$L/libspprl_$v.so
  for bs in 1049 8389; do
    SPPRL_LIB=$lib timeout -k 10 120 python -u tools/sgd_bs.py $bs 400 2>&1 | grep "us per" | sed "s/^/$v /" | tee -a $O/sgd_bs.txt || exit $?
  done
done
B="python -u bench.py --config ppo_hcheetah --no-cpu-baseline --no-pmc --no-rocprof --steps 15 --warmup 3"
for v in ftanh default; do
  lib=$L/libspprl.so; [ $v != default ] && lib=$L/libspprl_$v.so
  SPPRL_LIB=$lib timeout -k 10 400 $B > $O/w1_$v.json 2> $O/w1_$v.err || exit $?
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'],d['roofline'].get('us_per_sgd_step'))" $O/w1_$v.json "w1 $v" | tee -a $O/ab.txt
done
