# Round-6 PPO_AcM scaling evidence (gpurun -- 'VARIANTS="..." PROF="..." bash tools/ppo_scaling.sh'):
#   w1            world-1 line, minibatch 512 x s (the cadence rule)       w1_512   the round-5 minibatch 512
#   w8 / w8u      world-8 rehearsal, sharded update / union update          w8_512   union, minibatch 512 (round 5)
# PROF: kernel-trace breakdowns (tools/ppo_breakdown.py) over 6 whole iterations (two ACM cycles).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=${OUT:-gpurun_out/r06_ppo}; mkdir -p $O
args() {
  case $1 in
    w1) echo "";; w1_512) echo "--ppo-minibatch 512";;
    w8) echo "--rehearse-world 8 --ppo-dp shard";; w8u) echo "--rehearse-world 8 --ppo-dp union";;
    w8_512) echo "--rehearse-world 8 --ppo-dp union --ppo-minibatch 512";;
  esac
}
B="python -u bench.py --config ppo_hcheetah --no-cpu-baseline --no-pmc --no-rocprof"
for V in $VARIANTS; do
  timeout -k 10 400 $B $(args $V) --steps ${STEPS:-15} --warmup 3 > $O/bench_$V.log 2>&1 || exit $?
  tail -1 $O/bench_$V.log | cut -c1-200
done
for V in $PROF; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d $R/$O/kt_$V -o run \
    --output-format csv -- python3 $R/bench.py --config ppo_hcheetah --no-cpu-baseline --no-pmc --no-rocprof \
    $(args $V) --steps 7 --warmup 3 > $R/$O/kt_$V.log 2>&1) || exit $?
  f=$(find $O/kt_$V -name 'run_kernel_trace.csv' | head -1)
  python3 tools/ppo_breakdown.py $f 3 6 > $O/breakdown_$V.txt || exit $?
  cat $O/breakdown_$V.txt
done
