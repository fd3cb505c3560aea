// SAC_AcM phase kernels instantiated for Ant-v2/v3.
#ifndef SPP_SINGLE_TU
#define SPP_KSET_TU
#endif
#include "kset.h"

namespace spp {
bool kset_sac_ant(int ob, int aout, int ac, bool acmc, KernelSet* ks) {
  SPP_KSET_CASE(make_kset, 111, 111, 8)
  return false;
}
}  // namespace spp
