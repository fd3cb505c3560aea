# Round-6 GPU call V: bench.py's N > 1 code as a one-rank RCCL job (SPP_DP_FORCE=1) beside the plain lines on the
# final library: SAC Hopper (serial exchange) and PPO HalfCheetah (sharded update with the fused steps).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r06v; mkdir -p $O
B="python -u bench.py --no-cpu-baseline --no-pmc --no-rocprof"
run() { tag=$1; shift; env "$@" timeout -k 10 400 $B $ARGS > $O/$tag.json 2> $O/$tag.err || return $?
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(sys.argv[2],d['value'],d['ms_per_step'],d.get('param_checksum'))" $O/$tag.json "$tag" | tee -a $O/ab.txt; }
export ARGS="--config sac_hopper --steps 100 --warmup 10"
run hopper_plain SPP_X=0 || exit $?
run hopper_dp SPP_DP_FORCE=1 || exit $?
export ARGS="--config ppo_hcheetah --steps 15 --warmup 3"
run ppo_plain SPP_X=0 || exit $?
run ppo_dp SPP_DP_FORCE=1 || exit $?
