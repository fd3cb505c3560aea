// Weight-gradient GEMMs (dw.hip) in their own translation unit: the operand-type x tile-shape
// instantiations of k_dw compile in parallel with the phase-kernel sets.
#include "dw.hip"

namespace spp {
void launch_dw_kernels(const DwJob* jobs, const int* item_job, const int* item_split, int nitems, int nlds,
                       int njobs, int64_t max_elems, bool bf16, hipStream_t st) {
  if (nlds > 0)
    hipLaunchKernelGGL(bf16 ? k_dw_big16 : k_dw_big, dim3(nlds), dim3(kDwThreads), 0, st, jobs, item_job, item_split);
  if (nitems > nlds)
    hipLaunchKernelGGL(bf16 ? k_dw<true> : k_dw<false>, dim3(nitems - nlds), dim3(kDwThreads), 0, st, jobs,
                       item_job + nlds, item_split + nlds);
  hipLaunchKernelGGL(k_dw_reduce, dim3(cdiv(max_elems, 256), njobs), dim3(256), 0, st, jobs);
}
}  // namespace spp
