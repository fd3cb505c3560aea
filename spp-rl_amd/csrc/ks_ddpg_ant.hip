// DDPG_AcM phase kernels: Ant-v2 (SPP-DDPG Ant, train/spp_ddpg_ant.py: BasicAcM(222, 8)).
#ifndef SPP_SINGLE_TU
#define SPP_KSET_TU
#endif
#include "kset.h"

namespace spp {
bool kset_ddpg_ant(int ob, int aout, int ac, bool acmc, KernelSet* ks) {
  SPP_KSET_CASE(make_dkset, 111, 111, 8)
  return false;
}
}  // namespace spp
