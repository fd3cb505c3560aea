# Round-6 GPU call G: the ACM SGD step's hand-offs, A/B on variant libraries (tools/build_variant.py, api.hip only):
# counter shard stride 4 KB (sg_s4k), no sleep in the poll (sg_ns), 16 shards 4 KB apart (sg_16), the published
# parameters in 8 / 16 replicas (sg_rep8 / sg_rep16).  tools/sgd_bs.py: one isolated launch of 400 steps at the w1
# (1049 rows, 17 workgroups) and w8 (8389 rows, 132 workgroups) batch; then the PPO line (w1, w8 rehearsal) on the
# default and the replicated-publish libraries.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r06g; mkdir -p $O
L=spp-rl_amd/spprl
for v in default sg_s4k sg_ns sg_16 sg_rep8 sg_rep16 default; do
  lib=$L/libspprl.so; [ $v != default ] && lib=$L/libspprl_$v.so
  for bs in 1049 8389; do
    SPPRL_LIB=$lib timeout -k 10 120 python -u tools/sgd_bs.py $bs 400 2>&1 | grep "us per" | sed "s/^/$v /" | tee -a $O/sgd_bs.txt || exit $?
  done
done
B="python -u bench.py --config ppo_hcheetah --no-cpu-baseline --no-pmc --no-rocprof --steps 12 --warmup 3"
for v in default sg_rep8; do
  lib=$L/libspprl.so; [ $v != default ] && lib=$L/libspprl_$v.so
  SPPRL_LIB=$lib timeout -k 10 400 $B > $O/ppo_w1_$v.json 2> $O/ppo_w1_$v.err || exit $?
  SPPRL_LIB=$lib timeout -k 10 400 $B --rehearse-world 8 > $O/ppo_w8_$v.json 2> $O/ppo_w8_$v.err || exit $?
  for w in w1 w8; do
    python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'],d['roofline'].get('us_per_sgd_step'))" $O/ppo_${w}_$v.json "ppo $w $v" | tee -a $O/ppo.txt
  done
done
