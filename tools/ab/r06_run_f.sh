# Round-6 GPU call F: region timing of the multi-workgroup ACM SGD step (k_mlp_sgd<34, 32, 6, 0>) at the w1 (1049
# rows, 17 workgroups) and world-8 (8389 rows, 132 workgroups) shapes, on the profiling library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; O=${OUT:-gpurun_out/r06f}; mkdir -p $O
for bs in 1049 8389; do
  SPPRL_LIB=spp-rl_amd/spprl/libspprl_prof.so timeout -k 10 120 python -u tools/sgd_prof.py $bs > $O/sgd_prof_$bs.txt 2>&1 || exit $?
  cat $O/sgd_prof_$bs.txt
done
