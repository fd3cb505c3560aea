# region timing of k_mlp_sgd (current profiling build)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
for BS in 1049 512; do SPPRL_LIB=$R/spp-rl_amd/spprl/libspprl_prof.so timeout -k 10 120 python -u tools/sgd_prof.py $BS || exit $?; done 2>&1 | tee gpurun_out/sgd_prof.log
