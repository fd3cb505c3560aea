// DDPG_AcM phase kernels: HalfCheetah-v2 (SPP-DDPG, train/spp_ddpg_hcheetah.py) and Hopper-v2.
#ifndef SPP_SINGLE_TU
#define SPP_KSET_TU
#endif
#include "kset.h"

namespace spp {
bool kset_ddpg(int ob, int aout, int ac, bool acmc, KernelSet* ks) {
  SPP_KSET_CASE(make_dkset, 17, 17, 6)
  SPP_KSET_CASE(make_dkset, 11, 11, 3)
  return false;
}
}  // namespace spp
