// SAC_AcM phase kernels with bf16 MFMA MLP layers (Cfg::BF): Hopper-v2 and Ant
// (BASELINE.json configs[4]: "bf16 MFMA MLP + fp32 targets").
#ifndef SPP_SINGLE_TU
#define SPP_KSET_TU
#endif
#include "kset.h"

namespace spp {
template <int OB, int AOUT, int AC, bool ACMC>
KernelSet make_kset_bf16() {
  return make_kset<OB, AOUT, AC, ACMC, true>();
}
bool kset_sac_bf16(int ob, int aout, int ac, bool acmc, KernelSet* ks) {
  SPP_KSET_CASE(make_kset_bf16, 11, 11, 3)
  SPP_KSET_CASE(make_kset_bf16, 111, 111, 8)
  return false;
}
}  // namespace spp
