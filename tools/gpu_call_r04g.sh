# region timing of k_mlp_sgd: baseline and current profiling builds
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
for L in prof; do for BS in 1049 64; do echo "== $L $BS"; SPPRL_LIB=$R/spp-rl_amd/spprl/libspprl_$L.so timeout -k 10 120 python -u tools/sgd_prof.py $BS || exit $?; done; done 2>&1 | tee gpurun_out/sgd_prof.log
