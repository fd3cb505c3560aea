// Kernel-set table: dims -> phase-kernel instantiations.  Each config family is
// instantiated in its own translation unit (ks_*.hip) so the library builds in
// parallel; api.hip only holds the function pointers.
#pragma once
#include "sac.hip"
#include "sac_bf.h"
#include "ddpg.hip"
#include "sac_team.h"

namespace spp {

struct KernelSet {
  void (*critic)(SacArgs);
  void (*actor)(SacArgs, AcmScratch);
  void (*actor_heads)(SacArgs, AcmScratch);  // wide heads: second kernel of the actor phase
  void (*act)(SacArgs, ActArgs);
  void (*acmreg)(SacArgs, AcmRegArgs);
  // DDPG_AcM
  void (*dcritic)(SacArgs, BAcmScratch);
  void (*dactor)(SacArgs, BAcmScratch);
  void (*dact)(SacArgs, ActArgs, BAcmScratch);
  void (*dreg)(SacArgs, BAcmRegArgs);
  // small-batch (team) forms of the SAC phases: one 4-wave workgroup per 32-sample tile (sac_team.h);
  // null where the shapes have none
  void (*critic_team)(SacArgs);
  void (*actor_team)(SacArgs, AcmScratch);
  void (*act_team)(SacArgs, ActArgs);  // plain handles' rollout action
};

template <int OB, int AOUT, int AC, bool ACMC, bool BF = false>
KernelSet make_kset() {
  using C = Cfg<OB, AOUT, AC, ACMC, BF>;
  void (*heads)(SacArgs, AcmScratch) = nullptr;
  if constexpr (C::NB_PAIR > 2) heads = k_sac_actor_heads<C>;
  void (*critic)(SacArgs) = k_sac_critic_phase<C>;
#if SPP_BF16_TWO_TILES
  if constexpr (C::BF && C::ACMC && !C::F3) critic = k_sac_critic_phase2<C>;  // two tiles per wave (sac_bf.h)
#endif
  return {critic, k_sac_actor_phase<C>, heads, k_policy_act<C>, k_acm_regress<C>,
          nullptr, nullptr, nullptr, nullptr};
}
template <int OB, int AOUT, int AC, bool ACMC>
KernelSet make_dkset() {
  using D = DCfg<OB, AOUT, AC, ACMC>;
  return {nullptr, nullptr, nullptr, nullptr, nullptr,
          k_ddpg_critic_phase<D>, k_ddpg_actor_phase<D>, k_ddpg_policy_act<D>, k_bacm_regress<D>};
}

#define SPP_KSET_CASE(mk, o, a, c)                                     \
  if (ob == o && aout == a && ac == c) {                               \
    *ks = acmc ? mk<o, a, c, true>() : mk<o, a, c, false>();           \
    return true;                                                       \
  }

bool kset_sac_hopper(int ob, int aout, int ac, bool acmc, KernelSet* ks);    // ks_sac_hopper.hip
bool kset_sac_hcheetah(int ob, int aout, int ac, bool acmc, KernelSet* ks);  // ks_sac_hcheetah.hip
bool kset_sac_ant(int ob, int aout, int ac, bool acmc, KernelSet* ks);       // ks_sac_ant.hip
bool kset_sac_small(int ob, int aout, int ac, bool acmc, KernelSet* ks);     // ks_sac_small.hip
bool kset_ddpg(int ob, int aout, int ac, bool acmc, KernelSet* ks);          // ks_ddpg.hip
bool kset_ddpg_ant(int ob, int aout, int ac, bool acmc, KernelSet* ks);      // ks_ddpg_ant.hip
bool kset_sac_bf16(int ob, int aout, int ac, bool acmc, KernelSet* ks);      // ks_sac_bf16.hip
bool kset_sac_vanilla(int ob, int aout, int ac, bool acmc, KernelSet* ks);   // ks_sac_vanilla.hip

}  // namespace spp
