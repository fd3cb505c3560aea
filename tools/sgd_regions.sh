# region timing of k_mlp_sgd, AcM and actor epoch (profiling build: build.py --prof --hopper-only --hcheetah)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
for BS in 1049 actor; do SPPRL_LIB=$R/spp-rl_amd/spprl/libspprl_prof.so timeout -k 10 120 python -u tools/sgd_prof.py $BS || exit $?; done 2>&1 | tee gpurun_out/sgd_prof.log
