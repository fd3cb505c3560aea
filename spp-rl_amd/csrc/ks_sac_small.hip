// SAC_AcM phase kernels instantiated for Pendulum-v0 (tests).
#ifndef SPP_SINGLE_TU
#define SPP_KSET_TU
#endif
#include "kset.h"

namespace spp {
bool kset_sac_small(int ob, int aout, int ac, bool acmc, KernelSet* ks) {
  SPP_KSET_CASE(make_kset, 3, 3, 1)
  return false;
}
}  // namespace spp
