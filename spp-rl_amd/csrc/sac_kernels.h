// Device-side argument blocks shared by the SAC_AcM kernels and the host API.
#pragma once
#include "mlp.h"

namespace spp {

// Packed (fragment-image) views of one network, produced by the pack kernels.
// W2 / Wh / W2T / W1Ta (256-input layers) are ib-major images for dense_lds;
// the others are ob-major images for dense.  t* are offsets of the network's
// bias (and critic fc3 weight) vectors in the per-workgroup LDS table.
struct ActorDev {
  const float4 *W1, *W2, *Wh, *W2T, *WhT;
  int tb1, tb2, tbh;
  const float4* WhP;  // bf16 sets: the heads in pairing output order (MAP_PAIR, ib-major; k_sac_critic_phase2)
};
struct CriticDev {
  const float4 *W1, *W2, *W2T, *W1Ta;
  int tb1, tb2, tw3;
  const float* b3;  // canonical scalar
};
struct AcmDev {
  const float4 *W1, *W2, *W3, *W3T, *W2T, *W1Ta;
  int tb1, tb2, tb3;
};

// BasicAcM (rltoolkit/acm/models/basic_acm.py:11-27): fc1 in->100, fc2 100->50,
// fc21 in->50 (skip), fc3 50->ac; h1 = tanh(fc2(h) + t*fc21(x)); out = tanh(fc3(h1))*t1.
struct BAcmDev {
  const float4 *W1, *W21, *W2, *W3, *W3T, *W2T, *W1Ta, *W21Ta;
  int tb1, tb21, tb2, tb3;
  const float *t, *t1;  // canonical scalar / [ac] (frozen during the agent update)
};

// LDS table segment: tbl[off + i] = i < n ? src[i] : 0 for i < npad.
struct TabSeg {
  const float* src;
  int n, npad, off, pad_;
};
constexpr int kTabSegs = 28;
constexpr int kTabMax = 6144;  // floats (24 KiB)

// Feature-major ("unit-major") scratch: X[f][Bp], zero padded beyond B.
struct SacArgs {
  int B, Bp;
  float inv_B;
  // staged batch
  const float *S, *S2, *ACT, *AENV, *R, *DN;  // DN = done as float
  const float *EPS1, *EPS2;                   // [aout][Bp]
  // normaliser + limits
  int min_max;
  const float *lo, *hi, *mean, *std;
  const float *actor_lim, *acm_lim;
  float gamma, custom_loss;
  int norm_closs;
  const float* alpha;  // device scalar (python float self.alpha)
  ActorDev actor;
  CriticDev critic[2], targ[2];
  AcmDev acm;
  BAcmDev bacm;       // DDPG_AcM's ACM
  ActorDev actor_targ;  // DDPG target actor
  // critic-phase outputs (weight-gradient operands)
  float *H1[2], *H2[2], *D1[2], *D2[2], *DQ[2];
  // actor-phase outputs
  float *AH1, *AH2, *AD1, *AD2, *ADH;
  float *part;  // per-tile partial sums [ntiles][8]
  // SAC critic phase: per-wave partials of the fused fc3 weight gradient, [waves][w3p_stride] per critic
  float* W3P[2];
  int64_t w3p_stride;
  // per-workgroup LDS constant table (biases, critic fc3 weights; then the limits and the
  // normaliser vectors at t_lim / t_alim / t_n0 / t_n1: lo, hi or mean, std)
  TabSeg seg[kTabSegs];
  int nseg;
  int t_lim, t_alim, t_n0, t_n1;
};

constexpr int kParts = 8;

}  // namespace spp
