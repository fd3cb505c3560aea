# Round-6 GPU call H: the ACM SGD shard reduce summed while loading (SPP_SGD_PRED=1: sg_pred; with the replicated
# publish: sg_pred_rep8) against the default, tools/sgd_bs.py at the w1 / w8 batches, alternating twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=gpurun_out/r06h; mkdir -p $O
L=spp-rl_amd/spprl
for v in default sg_pred sg_pred_rep8 default sg_pred sg_pred_rep8; do
  lib=$L/libspprl.so; [ $v != default ] && lib=$L/libspprl_$v.so
  for bs in 1049 8389; do
    SPPRL_LIB=$lib timeout -k 10 120 python -u tools/sgd_bs.py $bs 400 2>&1 | grep "us per" | sed "s/^/$v /" | tee -a $O/sgd_bs.txt || exit $?
  done
done
