// Persistent minibatch SGD of a 3-layer tanh MLP on the fp32 matrix cores: many sequential Adam steps in ONE
// launch, the parameters held in LDS images for the whole launch.  Two heads:
//   HEAD 0  AcMTrainer (rltoolkit/basic_model.py:108-132, acm/acm.py:246-303, 356-372):
//           IN -> 64 -> H2 (tanh) -> OUT, out = tanh(fc3) * lim, loss = mse(out, y); x / y rows contiguous
//   HEAD 1  PPO_AcM.update_actor_acm's minibatch steps (acm/on_policy.py:176-207, ppo.py:194-204; the
//           Gaussian Actor of basic_model.py:7-51): IN -> 64 -> 64 (tanh) -> OUT, mu = tanh(fc3) * lim,
//           log_prob of the stored actions under Normal(mu, exp(log_scale)), clip loss - ent_coef * entropy;
//           rows gathered through the epoch's permutation; per step {actor loss, KL, dist, entropy} out.
//
// One step of bs rows runs on G = ceil(bs / 64) workgroups of 4 waves (64 rows each); wave w = (sample block
// sb = w & 1, unit block hb = w >> 1).  Every layer, delta and weight gradient is a v_mfma_f32_32x32x2_f32
// tile from LDS images laid out conflict-free (odd row strides):
//   X [64 samples][SX]   the step's inputs (+ a constant-1 column IN: b1's gradient is dW1's column IN)
//   H1L / D1L [64 units][65], H2L / D2L [H2][65], D3L / LSL [32][65]  activations and deltas ([unit][sample])
//   W1 [64][SW1], W2 [H2][65], W3 [32][H2 + 1]  parameters (row = output unit; rows >= OUT zero)
// The step's gradient is staged in canonical (state_dict) order in LDS.  G = 1: Adam in place.  G > 1: a
// reduce-scatter with sharded Adam -- each workgroup writes its gradient slab (write-through sc1 stores), one
// arrival barrier, workgroup g sums ITS 1/G of the slab over the G slabs in a fixed order and applies Adam to
// that shard (its Adam moments live in its registers for the whole launch), publishes the new parameters,
// a second arrival barrier, every workgroup reloads the parameters into its LDS images.  The shard's G slab
// chunks are fetched by all 256 threads at once into LDS (one memory round trip, not G dependent ones) and
// summed from there; the reload issues all of its loads before the first LDS write.  Sums in a fixed order:
// every workgroup (and every data-parallel replica running the same launch) holds identical parameters.
// Adam follows torch.optim.Adam's operation order (IEEE divide / sqrt), as k_adam.
#pragma once
// (included by api.hip after sgd.hip: AcmSgdArgs' slab helpers and the bounded arrival barrier)

namespace spp {

constexpr int kMlR = 64;      // rows per workgroup and step
constexpr int kMlTH = 256;    // 4 waves
constexpr int kMlS = 65;      // row stride of the [unit][sample] images
constexpr int kMlMaxWG = 512;  // workgroups per step (bs <= 32,768)
constexpr int kMlSlabMax = 8192;  // slab floats per workgroup (>= MlCfg::SLAB)

struct MlpSgdArgs {
  // rows
  const float* x;        // HEAD 0: [nsteps * bs][IN] contiguous; HEAD 1: normalised obs [n][IN] (through idx)
  const float* y;        // HEAD 0: targets [nsteps * bs][OUT]; HEAD 1: actions [n][OUT]
  const float* nxt;      // HEAD 1: next obs [n][OUT] (the dist loss, data only)
  const float* lp_old;   // HEAD 1: [n]
  const float* adv;      // HEAD 1: normalised advantages [n]
  const int64_t* idx;    // HEAD 1: row of step k's r-th sample = idx[k * bs + r]
  int nsteps, bs, bsl;   // bsl: rows per workgroup (G > 1)
  int bs_last;           // rows of the last step (<= bs: an epoch's ragged last minibatch in the same launch)
  float* params;         // canonical flat parameters (state_dict order)
  float* m;              // Adam exp_avg
  float* v;              // Adam exp_avg_sq
  float lr;
  int64_t step0;         // Adam steps already taken
  const float* lim;      // [OUT]
  float eps_clip, ent_coef;
  float* loss_sum;       // HEAD 0: += sum over steps of the batch loss
  float* out;            // HEAD 1: [nsteps][4] actor loss, KL, dist, entropy
  float* slab;           // G > 1: [2][G][slab floats] gradient slabs (step parity)
  float* pbuf;           // G > 1: [param floats] the new parameters of each step
  int* ctr;              // arrival counter (zeroed per launch)
  int* err;              // set to 1 if an arrival wait timed out
};

template <int IN, int H2, int OUT, int HEAD>
struct MlCfg {
  static_assert(H2 == 32 || H2 == 64, "H2");
  static_assert(OUT >= 1 && OUT <= 32, "OUT");
  static constexpr int NKS1 = (IN + 1) / 2;        // fc1 k-steps (pairs of inputs)
  static constexpr int NIB1 = (IN + 1 + 31) / 32;  // dW1 input blocks (input IN: the constant 1)
  static constexpr int SX = ((2 * NKS1 > 32 * NIB1 ? 2 * NKS1 : 32 * NIB1)) | 1;
  static constexpr int SW1 = (2 * NKS1) | 1;
  static constexpr int SW3 = H2 + 1;
  static constexpr int NB2 = H2 / 32;              // unit blocks of layer 2
  static constexpr int NKS3 = (OUT + 1) / 2;       // k-steps over fc3's outputs (dz2)
  static constexpr int NTILE = 2 * NIB1 + 2 * NB2 + NB2;  // dW1 | dW2 | dW3
  static constexpr int TPW = (NTILE + 3) / 4;
  // canonical layout: [log_scale (HEAD 1)] fc1.weight fc1.bias fc2.weight fc2.bias fc3.weight fc3.bias
  static constexpr int O_W1 = HEAD ? OUT : 0;
  static constexpr int O_B1 = O_W1 + 64 * IN;
  static constexpr int O_W2 = O_B1 + 64;
  static constexpr int O_B2 = O_W2 + H2 * 64;
  static constexpr int O_W3 = O_B2 + H2;
  static constexpr int O_B3 = O_W3 + OUT * H2;
  static constexpr int NP = O_B3 + OUT;                 // parameters
  // scalar partials (HEAD 0: loss; HEAD 1: min-term, KL, dist) in ONE float4 after the parameters
  static constexpr int O_SC = (NP + 3) / 4 * 4;
  static constexpr int NPS = O_SC + 4;                  // slab floats
  static constexpr int NP4 = NPS / 4;
  static constexpr int SLAB = (NPS + 63) / 64 * 64;     // slab stride (floats)
  static constexpr int K4 = (NP4 + kMlTH - 1) / kMlTH;  // float4 slots per thread (G = 1: all of them)
  static constexpr int NXP = (kMlR * IN + kMlTH - 1) / kMlTH, NYP = (kMlR * OUT + kMlTH - 1) / kMlTH;
  static_assert(NPS <= 64 * kMlS * 2, "gradient staging fits the H1L | D1L alias");
  // G > 1: the shard's G slab chunks are staged in the same alias, at most NP4 + G - 1 float4
  static constexpr int RED4 = 64 * kMlS * 2 / 4;
  static constexpr int MAXG = RED4 - NP4 + 1 < kMlMaxWG ? RED4 - NP4 + 1 : kMlMaxWG;
  static constexpr int RLC = HEAD ? 4 : 8;  // slab float4 loads in flight per thread (register budget)
  static constexpr int NL = (NP4 + kMlTH - 1) / kMlTH;   // reloaded float4 per thread
  static_assert(SLAB <= kMlSlabMax, "slab");
};

__device__ __forceinline__ constexpr int ml_ru(int r) { return (r & 3) + 8 * (r >> 2); }
__device__ __forceinline__ f32x16 ml_mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

template <class C>
__device__ __forceinline__ void ml_tile(int t, int& layer, int& r0, int& c0) {
  if (t < 2 * C::NIB1) {
    layer = 0; r0 = 32 * (t & 1); c0 = 32 * (t >> 1);
  } else if (t < 2 * C::NIB1 + 2 * C::NB2) {
    const int q = t - 2 * C::NIB1;
    layer = 1; r0 = 32 * (q >> 1); c0 = 32 * (q & 1);
  } else {
    layer = 2; r0 = 0; c0 = 32 * (t - 2 * C::NIB1 - 2 * C::NB2);
  }
}

template <int IN, int H2, int OUT, int HEAD, bool MW>
__global__ __launch_bounds__(kMlTH, 1) void k_mlp_sgd(MlpSgdArgs a) {
  using C = MlCfg<IN, H2, OUT, HEAD>;
  constexpr int SX = C::SX, SW1 = C::SW1, SW3 = C::SW3, S = kMlS, R = kMlR, NP = C::NP;
  __shared__ float X[R * SX];
  __shared__ __attribute__((aligned(16))) float H1D1[2 * 64 * S];  // H1L | D1L; then the step's gradient
  __shared__ float H2L[H2 * S], D2L[H2 * S], D3L[32 * S];
  __shared__ float LSL[HEAD ? 32 * S : 1];
  __shared__ float W1[64 * SW1], W2[H2 * S], W3[32 * SW3];
  __shared__ float B1[64], B2[H2], B3[32], LS[32];
  __shared__ float Y[R * OUT];
  __shared__ float LPO[HEAD ? R : 1], ADV[HEAD ? R : 1];
  __shared__ int64_t IDX[HEAD ? 2 * R : 1];
  __shared__ float SCP[4][4];       // per wave: scalar partials
  __shared__ float adam_s[2][2];
  __shared__ int s_dead;
  float* const H1L = H1D1;
  float* const D1L = H1D1 + 64 * S;
  float* const GR = H1D1;  // staging alias (after the gradient tiles)
  const int t = threadIdx.x, w = t >> 6, lane = t & 63, h = lane >> 5, l32 = lane & 31;
  const int sb = w & 1, hb = w >> 1;
  const int G = MW ? (int)gridDim.x : 1, g = MW ? (int)blockIdx.x : 0;
  const int r0 = MW ? g * a.bsl : 0;
  auto step_rows = [&](int st) { return st == a.nsteps - 1 ? a.bs_last : a.bs; };  // the step's batch
  auto wg_rows = [&](int st) {  // this workgroup's rows of step st (<= 64)
    return MW ? max(0, min(a.bsl, step_rows(st) - r0)) : step_rows(st);
  };
  if (t == 0) s_dead = 0;
  // ---- the canonical element c (< NP) of the parameters inside the LDS images
  auto pref = [&](int c) -> float& {
    if (HEAD && c < C::O_W1) return LS[c];
    if (c < C::O_B1) { const int q = c - C::O_W1; return W1[(q / IN) * SW1 + q % IN]; }
    if (c < C::O_W2) return B1[c - C::O_B1];
    if (c < C::O_B2) { const int q = c - C::O_W2; return W2[(q >> 6) * S + (q & 63)]; }
    if (c < C::O_W3) return B2[c - C::O_B2];
    if (c < C::O_B3) { const int q = c - C::O_W3; return W3[(q / H2) * SW3 + q % H2]; }
    return B3[c - C::O_B3];
  };
  // ---- parameter images (zero padding)
  for (int i = t; i < 64 * SW1; i += kMlTH) W1[i] = 0.f;
  for (int i = t; i < H2 * S; i += kMlTH) W2[i] = 0.f;
  for (int i = t; i < 32 * SW3; i += kMlTH) W3[i] = 0.f;
  if (t < 32) { B3[t] = 0.f; LS[t] = 0.f; }
  for (int i = t; i < 32 * S; i += kMlTH) {
    D3L[i] = 0.f;  // rows >= OUT stay zero
    if constexpr (HEAD) LSL[i] = 0.f;
  }
  for (int i = t; i < R * SX; i += kMlTH) X[i] = 0.f;  // padding columns / rows past bs stay zero
  __syncthreads();
  for (int c = t; c < NP; c += kMlTH) pref(c) = a.params[c];
  // ---- Adam moments of the owned float4 slots: slot f = f0 + t + 256 k (this workgroup's shard)
  const int C4 = (C::NP4 + G - 1) / G, f0 = g * C4, f1 = min(f0 + C4, C::NP4);
  const int c4n = max(f1 - f0, 0);  // this shard's float4 slots
  // (MW: G >= 2, so a shard holds at most ceil(NP4 / 2) slots)
  constexpr int K4 = MW ? ((C::NP4 + 1) / 2 + kMlTH - 1) / kMlTH : C::K4;
  float mom[K4][4], vel[K4][4];
#pragma unroll
  for (int k = 0; k < K4; ++k)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = f0 + t + kMlTH * k, c = 4 * f + i;
      const bool own = f < f1 && c < NP;
      mom[k][i] = own ? a.m[c] : 0.f;
      vel[k][i] = own ? a.v[c] : 0.f;
    }
  double pw1 = 0.0, pw2 = 0.0;  // beta1^t, beta2^t of the next step (thread kMlTH - 1: pow once, then products)
  auto adam_scalars = [&](int st) {
    if (st == 0) {
      pw1 = pow(0.9, (double)(a.step0 + 1));
      pw2 = pow(0.999, (double)(a.step0 + 1));
    } else {
      pw1 *= 0.9;
      pw2 *= 0.999;
    }
    adam_s[st & 1][0] = (float)(-((double)a.lr / (1.0 - pw1)));
    adam_s[st & 1][1] = (float)sqrt(1.0 - pw2);
  };
  // ---- register prefetch of one step's rows (HEAD 1: through the step's indices in IDX)
  float xp[C::NXP], yp[C::NYP], lpp = 0.f, advp = 0.f, dsum = 0.f;
  auto row_of = [&](int st, int r) -> int64_t {
    if constexpr (HEAD) return IDX[(st & 1) * R + r];
    else return (int64_t)st * a.bs + r0 + r;
  };
  auto prefetch = [&](int st) {
    const bool live = st < a.nsteps;
    const int bs = wg_rows(st);
#pragma unroll
    for (int k = 0; k < C::NXP; ++k) {
      const int i = t + kMlTH * k, r = i / IN;
      xp[k] = (live && i < bs * IN) ? a.x[row_of(st, r) * IN + i % IN] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < C::NYP; ++k) {
      const int i = t + kMlTH * k, r = i / OUT;
      const bool ok = live && i < bs * OUT;
      yp[k] = ok ? a.y[row_of(st, r) * OUT + i % OUT] : 0.f;
      if constexpr (HEAD) {  // the dist loss is data only: its per-step sum is taken here
        const float e = ok ? yp[k] - a.nxt[row_of(st, r) * OUT + i % OUT] : 0.f;
        dsum = fmaf(e, e, dsum);
      }
    }
    if constexpr (HEAD) {
      lpp = (live && t < bs) ? a.lp_old[row_of(st, t)] : 0.f;
      advp = (live && t < bs) ? a.adv[row_of(st, t)] : 0.f;
    }
  };
  auto load_idx = [&](int st) {  // HEAD 1: step st's row indices -> IDX[st & 1]
    if constexpr (HEAD)
      if (t < R) IDX[(st & 1) * R + t] = (st < a.nsteps && t < wg_rows(st)) ? a.idx[(int64_t)st * a.bs + r0 + t] : 0;
  };
  load_idx(0);
  if (t == kMlTH - 1) adam_scalars(0);
  __syncthreads();
  prefetch(0);
  load_idx(1);
  SPP_TP_INIT();
  float loss_acc = 0.f;  // HEAD 0: the scalar slot's owner sums the steps' losses  // HEAD 0: sum over steps (the scalar shard's owner)
  const float lo = 1.f - a.eps_clip, hi = 1.f + a.eps_clip;
  for (int st = 0; st < a.nsteps; ++st) {
    const int bsg = step_rows(st), bs = wg_rows(st);
    const float inv_bs = 1.f / (float)bsg;
    // ---- the step's rows into LDS (rows >= bs: zeros)
#pragma unroll
    for (int k = 0; k < C::NXP; ++k) {
      const int i = t + kMlTH * k;
      if (i < R * IN) X[(i / IN) * SX + (i % IN)] = xp[k];
    }
    if (t < R) X[t * SX + IN] = t < bs ? 1.f : 0.f;  // the bias input
#pragma unroll
    for (int k = 0; k < C::NYP; ++k) {
      const int i = t + kMlTH * k;
      if (i < R * OUT) Y[i] = yp[k];
    }
    if constexpr (HEAD) {
      if (t < R) {
        LPO[t] = lpp;
        ADV[t] = advp;
      }
    }
    const float dist_step = dsum;
    dsum = 0.f;
    __syncthreads();  // (also: IDX[(st + 1) & 1] written)
    prefetch(st + 1);
    load_idx(st + 2);  // IDX[st & 1]: its last reader was prefetch(st), issued a step ago
    SPP_TP(0);
    // ---- fc1: block (hb, sb) of h1 = tanh(W1 x + b1)
    f32x16 h1r;
    {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = B1[32 * hb + ml_ru(r) + 4 * h];
      const float* pa = W1 + (32 * hb + l32) * SW1 + h;
      const float* pb = X + (32 * sb + l32) * SX + h;
#pragma unroll
      for (int ks = 0; ks < C::NKS1; ++ks) acc = ml_mfma(pa[2 * ks], pb[2 * ks], acc);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        h1r[r] = tanhf(acc[r]);
        H1L[(32 * hb + ml_ru(r) + 4 * h) * S + 32 * sb + l32] = h1r[r];
      }
    }
    __syncthreads();
    SPP_TP(1);
    // ---- fc2: block (hb, sb) of h2 = tanh(W2 h1 + b2) (H2 = 32: waves hb = 0)
    f32x16 h2r;
    const bool l2w = hb < C::NB2;
    if (l2w) {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = B2[32 * hb + ml_ru(r) + 4 * h];
      const float* pa = W2 + (32 * hb + l32) * S + h;
      const float* pb = H1L + h * S + 32 * sb + l32;
#pragma unroll 8
      for (int ks = 0; ks < 32; ++ks) acc = ml_mfma(pa[2 * ks], pb[2 * ks * S], acc);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        h2r[r] = tanhf(acc[r]);
        H2L[(32 * hb + ml_ru(r) + 4 * h) * S + 32 * sb + l32] = h2r[r];
      }
    }
    // H2 = 64: fc3 of sample block sb reads both unit blocks; H2 = 32: the same wave's other lanes (a compiler
    // memory barrier keeps their reads below these stores)
    if constexpr (H2 == 64) __syncthreads();
    else asm volatile("" ::: "memory");
    // ---- fc3 and the head (waves hb = 0): D3L = d loss / d z3
    if (hb == 0) {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int u = ml_ru(r) + 4 * h;
        acc[r] = u < OUT ? B3[u] : 0.f;
      }
      const float* pa = W3 + l32 * SW3 + h;
      const float* pb = H2L + h * S + 32 * sb + l32;
#pragma unroll 8
      for (int ks = 0; ks < H2 / 2; ++ks) acc = ml_mfma(pa[2 * ks], pb[2 * ks * S], acc);
      const int sm = 32 * sb + l32;
      const bool valid = sm < bs;
      if constexpr (HEAD == 0) {
        float lpart = 0.f;
        const float inv_n = 1.f / (float)(bsg * OUT);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int u = ml_ru(r) + 4 * h;
          if (u < OUT) {
            const float th = tanhf(acc[r]), lm = a.lim[u];
            const float e = th * lm - Y[sm * OUT + u];
            float d = 0.f;
            if (valid) {
              lpart = fmaf(e, e, lpart);
              d = 2.f * e * inv_n * lm * (1.f - th * th);
            }
            D3L[u * S + sm] = d;
          }
        }
        lpart = wave_sum(lpart);
        if (lane == 0) SCP[w][0] = lpart;
      } else {
        // log_prob of the stored action (torch Normal: -(a-mu)^2/(2 var) - log(scale) - log(sqrt(2 pi)), summed)
        float th[16], dd[16], lp = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int u = ml_ru(r) + 4 * h;
          th[r] = 0.f;
          dd[r] = 0.f;
          if (u < OUT) {
            const float sc = expf(LS[u]);
            th[r] = tanhf(acc[r]);
            const float mu = fmul_rn(th[r], a.lim[u]);
            dd[r] = fsub_rn(Y[sm * OUT + u], mu);
            lp += fsub_rn(fsub_rn(fdiv_rn(-fmul_rn(dd[r], dd[r]), 2.f * fmul_rn(sc, sc)), logf(sc)), kLogSqrt2PiO);
          }
        }
        lp += __shfl_xor(lp, 32, 64);
        // clip objective (ppo.py:194-204) and its gradient wrt lp_new (torch minimum / clamp rules)
        float mterm = 0.f, kl = 0.f, glp = 0.f;
        if (valid) {
          const float lpo = LPO[sm], A = ADV[sm];
          const float rt = expf(fsub_rn(lp, lpo));
          const float rc = fminf(fmaxf(rt, lo), hi);
          const float u1 = fmul_rn(rt, A), u2 = fmul_rn(rc, A);
          mterm = fminf(u1, u2);
          kl = fsub_rn(lpo, lp);
          const float wu = u1 < u2 ? 1.f : (u1 == u2 ? 0.5f : 0.f);
          const float pass = (rt >= lo && rt <= hi) ? 1.f : 0.f;
          glp = -(wu * A * rt + (1.f - wu) * A * pass * rt) * inv_bs;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int u = ml_ru(r) + 4 * h;
          if (u < OUT) {
            const float sc = expf(LS[u]);
            const float var = fmul_rn(sc, sc);
            const float gmu = glp * dd[r] / var;
            LSL[u * S + sm] = glp * (dd[r] * dd[r] / var - 1.f);
            D3L[u * S + sm] = gmu * a.lim[u] * (1.f - th[r] * th[r]);
          }
        }
        const float sm_ = wave_sum(h == 0 ? mterm : 0.f), sk = wave_sum(h == 0 ? kl : 0.f);
        if (lane == 0) {
          SCP[w][0] = sm_;
          SCP[w][1] = sk;
        }
      }
    }
    if constexpr (H2 == 64) __syncthreads();  // dz2 block (hb, sb) reads sample block sb's D3L
    else asm volatile("" ::: "memory");
    // ---- dz2 = (W3^T dz3) * (1 - h2^2), block (hb, sb)
    if (l2w) {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      const float* pa = W3 + h * SW3 + 32 * hb + l32;
      const float* pb = D3L + h * S + 32 * sb + l32;
#pragma unroll
      for (int ks = 0; ks < C::NKS3; ++ks) acc = ml_mfma(pa[2 * ks * SW3], pb[2 * ks * S], acc);
#pragma unroll
      for (int r = 0; r < 16; ++r) D2L[(32 * hb + ml_ru(r) + 4 * h) * S + 32 * sb + l32] = acc[r] * (1.f - h2r[r] * h2r[r]);
    }
    __syncthreads();
    SPP_TP(2);
    // ---- dz1 = (W2^T dz2) * (1 - h1^2), block (hb, sb)
    {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      const float* pa = W2 + h * S + 32 * hb + l32;
      const float* pb = D2L + h * S + 32 * sb + l32;
#pragma unroll 8
      for (int ks = 0; ks < H2 / 2; ++ks) acc = ml_mfma(pa[2 * ks * S], pb[2 * ks * S], acc);
#pragma unroll
      for (int r = 0; r < 16; ++r) D1L[(32 * hb + ml_ru(r) + 4 * h) * S + 32 * sb + l32] = acc[r] * (1.f - h1r[r] * h1r[r]);
    }
    __syncthreads();
    SPP_TP(3);
    // ---- weight-gradient tiles over the 64 samples: tile q = w + 4k
    f32x16 gt[C::TPW];
#pragma unroll
    for (int k = 0; k < C::TPW; ++k) {
      const int q = w + 4 * k;
#pragma unroll
      for (int r = 0; r < 16; ++r) gt[k][r] = 0.f;
      if (q < C::NTILE) {
        int layer, rr, cc;
        ml_tile<C>(q, layer, rr, cc);
        if (layer == 0) {
          const float* pa = D1L + (rr + l32) * S + h;
          const float* pb = X + h * SX + cc + l32;
#pragma unroll 8
          for (int ks = 0; ks < 32; ++ks) gt[k] = ml_mfma(pa[2 * ks], pb[2 * ks * SX], gt[k]);
        } else {
          const float* pa = layer == 1 ? D2L + (rr + l32) * S + h : D3L + l32 * S + h;
          const float* pb = (layer == 1 ? H1L : H2L) + (cc + l32) * S + h;
#pragma unroll 8
          for (int ks = 0; ks < 32; ++ks) gt[k] = ml_mfma(pa[2 * ks], pb[2 * ks], gt[k]);
        }
      }
    }
    // b2 / b3 (and log_scale) gradients: row sums over the 64 samples
    float bg = 0.f;
    {
      const float* row = t < H2 ? D2L + t * S : (t < H2 + OUT ? D3L + (t - H2) * S : LSL + (t - H2 - OUT) * S);
      if (t < H2 + OUT * (HEAD ? 2 : 1)) {
#pragma unroll 16
        for (int s2 = 0; s2 < R; ++s2) bg += row[s2];
      }
      if (HEAD && g == 0 && t >= H2 + OUT && t < H2 + 2 * OUT) bg -= a.ent_coef;  // - ent_coef * d entropy / d ls
    }
    __syncthreads();  // every read of the activations is done: H1L | D1L becomes the gradient staging area
    SPP_TP(4);
    // ---- the step's gradient in canonical order -> GR[0 .. NP), scalars -> GR[NP ..]
#pragma unroll
    for (int k = 0; k < C::TPW; ++k) {
      const int q = w + 4 * k;
      if (q < C::NTILE) {
        int layer, rr, cc;
        ml_tile<C>(q, layer, rr, cc);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = rr + ml_ru(e) + 4 * h, col = cc + l32;
          int c = -1;
          if (layer == 0) c = col < IN ? C::O_W1 + row * IN + col : (col == IN ? C::O_B1 + row : -1);
          else if (layer == 1) c = C::O_W2 + row * 64 + col;
          else c = row < OUT ? C::O_W3 + row * H2 + col : -1;
          if (c >= 0) GR[c] = gt[k][e];
        }
      }
    }
    if (t < H2) GR[C::O_B2 + t] = bg;
    else if (t < H2 + OUT) GR[C::O_B3 + t - H2] = bg;
    else if (HEAD && t < H2 + 2 * OUT) GR[t - H2 - OUT] = bg;
    if (t < 4) GR[C::O_SC + t] = t == 0 ? SCP[0][0] + SCP[1][0] : (HEAD && t == 1 ? SCP[0][1] + SCP[1][1] : 0.f);
    if constexpr (HEAD) {  // the dist partials of every thread (this step's rows)
      const float ds = wave_sum(dist_step);
      if (lane == 0) SCP[w][2] = ds;
    }
    if (t < C::O_SC - NP) GR[NP + t] = 0.f;
    __syncthreads();
    if constexpr (HEAD) {
      if (t == 0) GR[C::O_SC + 2] = SCP[0][2] + SCP[1][2] + SCP[2][2] + SCP[3][2];
      __syncthreads();
    }
    // ---- exchange (G > 1) and Adam on this workgroup's shard
    float entropy = 0.f;
    if (HEAD && g == 0 && t == 0) {  // of the parameters this step's forward used (before the update)
      double ent = 0.0;
      for (int j = 0; j < OUT; ++j) ent += 0.5 + 0.91893853320467274178 + (double)LS[j];
      entropy = (float)ent;
    }
    SPP_TP(5);
    const auto all = sgd_rsrc(a.slab + (int64_t)(st & 1) * G * C::SLAB);  // (G = 1: unused)
    if constexpr (MW) {
      const auto mine = sgd_rsrc(a.slab + ((int64_t)(st & 1) * G + g) * C::SLAB);
      for (int f = t; f < C::NP4; f += kMlTH) {
        const float4 v4 = *reinterpret_cast<const float4*>(GR + 4 * f);
        slab_st4(mine, 4 * f, v4);
      }
      sgd_arrive_wait_wt(a.ctr, G * (2 * st + 1), a.err, &s_dead);
      // this shard's chunk of every slab -> the alias, [q][c4n] (G > 1: the staged gradient is dead)
      const int nit = c4n * G;
      for (int i0 = 0; i0 < nit; i0 += C::RLC * kMlTH) {  // (G = 17, 64-wide AcM: one round)
        float4 ld[C::RLC];
#pragma unroll
        for (int k = 0; k < C::RLC; ++k) {
          const int i = i0 + t + kMlTH * k;
          if (i < nit) {
            const int q = i / c4n;
            ld[k] = slab_ld4(all, q * C::SLAB + 4 * (f0 + i - q * c4n));
          }
        }
#pragma unroll
        for (int k = 0; k < C::RLC; ++k) {
          const int i = i0 + t + kMlTH * k;
          if (i < nit) reinterpret_cast<float4*>(H1D1)[i] = ld[k];
        }
      }
      __syncthreads();
    }
    SPP_TP(6);
    const float neg_step = adam_s[st & 1][0], bc2s = adam_s[st & 1][1];
    if (t == kMlTH - 1) adam_scalars(st + 1);
    const float omb1 = 0.1f, b2c = 0.999f, omb2 = 0.001f, eps = 1e-8f;
    const auto pub = sgd_rsrc(a.pbuf);
#pragma unroll
    for (int k = 0; k < K4; ++k) {
      const int f = f0 + t + kMlTH * k;
      if (f < f1) {
        float4 gg4;
        if constexpr (MW) {
          const float4* red = reinterpret_cast<const float4*>(H1D1) + (f - f0);
          gg4 = make_float4(0.f, 0.f, 0.f, 0.f);
          for (int q = 0; q < G; ++q) {
            const float4 x4 = red[q * c4n];
            gg4.x += x4.x; gg4.y += x4.y; gg4.z += x4.z; gg4.w += x4.w;
          }
        } else {
          gg4 = *reinterpret_cast<const float4*>(GR + 4 * f);
        }
        const float gv[4] = {gg4.x, gg4.y, gg4.z, gg4.w};
        float nv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = 4 * f + i;
          if (c < NP) {  // torch.optim.Adam (k_adam's operation order)
            float& p = pref(c);
            const float gi = gv[i];
            mom[k][i] = fadd_rn(mom[k][i], fmul_rn(omb1, fsub_rn(gi, mom[k][i])));
            vel[k][i] = fadd_rn(fmul_rn(vel[k][i], b2c), fmul_rn(fmul_rn(omb2, gi), gi));
            const float denom = fadd_rn(fdiv_rn(sqrtf(vel[k][i]), bc2s), eps);
            p = fadd_rn(p, fmul_rn(neg_step, fdiv_rn(mom[k][i], denom)));
            nv[i] = p;
          }
        }
        if (4 * f == C::O_SC) {  // the scalar partials (the shard holding them)
          if constexpr (HEAD == 0) {
            loss_acc += gv[0] * (1.f / (float)(bsg * OUT));
          } else {
            a.out[(int64_t)st * 4 + 0] = (float)(-(double)gv[0] / (double)bsg);
            a.out[(int64_t)st * 4 + 1] = (float)((double)gv[1] / (double)bsg);
            a.out[(int64_t)st * 4 + 2] = (float)((double)gv[2] / ((double)bsg * OUT));
          }
        }
        if constexpr (MW) slab_st4(pub, 4 * f, make_float4(nv[0], nv[1], nv[2], nv[3]));
      }
    }
    if (HEAD && g == 0 && t == 0) a.out[(int64_t)st * 4 + 3] = entropy;
    SPP_TP(7);
    if constexpr (MW) {
      sgd_arrive_wait_wt(a.ctr, G * (2 * st + 2), a.err, &s_dead);
      float4 rv[C::NL];
#pragma unroll
      for (int k = 0; k < C::NL; ++k) {  // (this shard's values are already in the images)
        const int f = t + kMlTH * k;
        if (f < C::NP4 && (f < f0 || f >= f1)) rv[k] = slab_ld4(pub, 4 * f);
      }
#pragma unroll
      for (int k = 0; k < C::NL; ++k) {
        const int f = t + kMlTH * k;
        if (f < C::NP4 && (f < f0 || f >= f1)) {
          const float vv[4] = {rv[k].x, rv[k].y, rv[k].z, rv[k].w};
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (4 * f + i < NP) pref(4 * f + i) = vv[i];
        }
      }
    }
    __syncthreads();
    SPP_TP(8);
  }
  SPP_TP_FLUSH();
  // ---- write back: parameters (workgroup 0, from its images), moments (each shard's owner)
  if (g == 0)
    for (int c = t; c < NP; c += kMlTH) a.params[c] = pref(c);
#pragma unroll
  for (int k = 0; k < K4; ++k)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = f0 + t + kMlTH * k, c = 4 * f + i;
      if (f < f1 && c < NP) {
        a.m[c] = mom[k][i];
        a.v[c] = vel[k][i];
      }
    }
  constexpr int fsc = C::O_SC / 4;  // the scalar slot: owned by thread (fsc - f0) % kMlTH of its shard
  if (HEAD == 0 && fsc >= f0 && fsc < f1 && (fsc - f0) % kMlTH == t) *a.loss_sum += loss_acc;
}

}  // namespace spp
