// Vanilla SAC phase kernels (BASELINE.json configs[0], rltoolkit/algorithms/sac/sac.py):
// HalfCheetah-v2, the actor emits the 6-dim env action, critics on cat(obs, action).
#ifndef SPP_SINGLE_TU
#define SPP_KSET_TU
#endif
#include "kset.h"

namespace spp {
bool kset_sac_vanilla(int ob, int aout, int ac, bool acmc, KernelSet* ks) {
  if (acmc || aout != ac) return false;
  if (ob == 17 && ac == 6) {
    *ks = make_kset<17, 6, 6, false>();
    using C = Cfg<17, 6, 6, false>;
    ks->critic_team = k_sac_critic_team<C>;
    ks->actor_team = k_sac_actor_team<C>;
    ks->act_team = k_policy_act_team<C>;
    return true;
  }
  return false;
}
}  // namespace spp
