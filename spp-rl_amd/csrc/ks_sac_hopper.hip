// SAC_AcM phase kernels instantiated for Hopper-v2.
#ifndef SPP_SINGLE_TU
#define SPP_KSET_TU
#endif
#include "kset.h"

namespace spp {
bool kset_sac_hopper(int ob, int aout, int ac, bool acmc, KernelSet* ks) {
  SPP_KSET_CASE(make_kset, 11, 11, 3)
  return false;
}
}  // namespace spp
