// Device-side argument blocks shared by the SAC_AcM kernels and the host API.
#pragma once
#include "mlp.h"

namespace spp {

// Packed (fragment-image) views of one network, produced by the pack kernels.
struct ActorDev {
  const float4 *W1, *W2, *Wh, *W2T, *WhT;
  const float *b1P, *b2P, *bhP;  // packed bias images
};
struct CriticDev {
  const float4 *W1, *W2, *W2T, *W1Ta;
  const float *b1P, *b2P, *w3P;
  const float* b3;  // canonical scalar
};
struct AcmDev {
  const float4 *W1, *W2, *W3, *W3T, *W2T, *W1Ta;
  const float *b1P, *b2P, *b3P;
};

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
  // critic-phase outputs (weight-gradient operands)
  float *H1[2], *H2[2], *D1[2], *D2[2], *DQ[2];
  // actor-phase outputs
  float *AH1, *AH2, *AD1, *AD2, *ADH;
  float *part;  // per-tile partial sums [ntiles][8]
};

constexpr int kParts = 8;

}  // namespace spp
