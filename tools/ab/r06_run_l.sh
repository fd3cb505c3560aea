# Round-6 GPU call L: the critic phase's fused fc3 weight gradient with 16-B LDS reads (variant f3, ks_sac_hopper.hip)
# against the default, SAC Hopper line alternating twice; the Hopper parity tests on the variant.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r06l; mkdir -p $O
L=spp-rl_amd/spprl
B="python -u bench.py --config sac_hopper --no-cpu-baseline --no-pmc --no-rocprof --steps 100 --warmup 10"
for v in default f3 default f3; do
  lib=$L/libspprl.so; [ $v != default ] && lib=$L/libspprl_$v.so
  SPPRL_LIB=$lib timeout -k 10 300 $B > $O/hopper_$v.json 2> $O/hopper_$v.err || exit $?
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);r=d['roofline'];print(sys.argv[2],d['value'],d['ms_per_step'],r['frac'],r.get('avg_launch_ms'))" $O/hopper_$v.json "hopper $v" | tee -a $O/ab.txt
done
SPPRL_LIB=$L/libspprl_f3.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "hopper or Hopper" > $O/tests_f3.log 2>&1 || { tail -30 $O/tests_f3.log; exit 1; }
tail -2 $O/tests_f3.log
