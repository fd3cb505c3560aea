// Persistent minibatch SGD of a 3-layer tanh MLP on the fp32 matrix cores: many sequential Adam steps in ONE
// launch, the parameters held in LDS images for the whole launch.  Two heads:
//   HEAD 0  AcMTrainer (rltoolkit/basic_model.py:108-132, acm/acm.py:246-303, 356-372):
//           IN -> 64 -> H2 (tanh) -> OUT, out = tanh(fc3) * lim, loss = mse(out, y); x / y rows contiguous
//   HEAD 1  PPO_AcM.update_actor_acm's minibatch steps (acm/on_policy.py:176-207, ppo.py:194-204; the
//           Gaussian Actor of basic_model.py:7-51): IN -> 64 -> 64 (tanh) -> OUT, mu = tanh(fc3) * lim,
//           log_prob of the stored actions under Normal(mu, exp(log_scale)), clip loss - ent_coef * entropy;
//           rows gathered through the epoch's permutation; per step {actor loss, KL, dist, entropy} out.
//   HEAD 2  A2C.update_critic's full-batch steps (a2c.py:186-225; the Critic of basic_model.py:55-76):
//           IN -> 64 -> 64 (tanh) -> 1 (linear), loss = 0.5 mean((q - V)^2); x / q rows contiguous.  A step's
//           rows may exceed 64 per workgroup: each workgroup runs ceil(rows / 64) passes of 64 and adds the
//           passes' gradients before the exchange.
//
// One step of bs rows runs on G = ceil(bs / 64) workgroups of 4 waves; wave w owns 16 of the workgroup's 64
// rows (image column 16 w + n, n = lane & 15) through every layer.  Forward and backward are
// v_mfma_f32_16x16x4_f32 tiles with units on the rows and the wave's samples on the columns: a result tile
// (lane (q = lane >> 4, n), register i = unit 4q + i of sample n) is the next layer's B operand as it stands
// (k-step (T, j) of lane group q = unit 16T + 4q + j), so activations and deltas stay in registers from
// layer to layer and the waves never wait for each other until the weight gradient.  fc1's bias is a
// column of W1 against a constant-1 input row.  The activations and deltas are also written to
// [unit][64 sample] LDS images (row stride 68: the result-layout stores hit 64 distinct banks); the weight
// gradients dW = delta . act^T are 16x16 tiles over all 64 samples (sample 16q + ks on k-step ks), spread
// over the 4 waves, two tiles in flight per wave; b2 / b3 / log_scale gradients are 16-lane row sums of the
// delta registers (per wave), added over the waves in a fixed order.
//
// The step's gradient is staged in canonical (state_dict) order in LDS.  G = 1: Adam in place.  G > 1: a
// reduce-scatter with sharded Adam -- each workgroup writes its gradient slab (write-through sc1 stores), one
// arrival barrier, workgroup g sums ITS 1/G of the slab over the G slabs in a fixed order and applies Adam to
// that shard (its Adam moments live in its registers for the whole launch, one element per thread), publishes
// the new parameters, a second arrival barrier, every workgroup reloads the parameters into its LDS images.  The
// shard's G slab chunks are fetched by all 256 threads at once (one memory round trip, not G dependent ones):
// thread (group pg, slot j) sums slabs pg, pg + P, ... of slot j as they arrive, and Adam adds the P group sums
// in order (round 6: the w8 ACM step 18.8 -> 15.5 us against one thread per slot summing all G; Adam one
// element per thread instead of one float4: 15.5 -> 15.2 us, w1 13.2 -> 12.8 us; profiles/r06/acm_step/).  The
// reload issues all of its loads before the first LDS write.  Sums in a fixed order: every workgroup (and every
// data-parallel replica running the same launch) holds identical parameters.
// Adam follows torch.optim.Adam's operation order (IEEE divide / sqrt), as k_adam.
#pragma once
// (included by api.hip after sgd.hip: the slab helpers and the bounded arrival barrier)

namespace spp {

constexpr int kMlR = 64;          // rows per workgroup and step of the 4-wave form (4 waves x 16; WV waves: 16 WV)
constexpr int kMlTH = 256;        // threads of the 4-wave form (WV waves: 64 WV)
constexpr int kMlRS = 68;         // row stride of the 4-wave form's [unit][64 sample] images (WV waves: 16 WV + 4)
constexpr int kMlMaxWG = 512;     // workgroups per step (bs <= 32,768)
constexpr int kMlSlabMax = 8192;  // slab floats per workgroup (>= MlCfg::SLAB)

struct MlpSgdArgs {
  // rows
  const float* x;        // HEAD 0: [nsteps * bs][IN] contiguous; HEAD 1: normalised obs [n][IN] (through idx);
                         // HEAD 2: [bs][IN], the same full batch every step (bs_last = bs)
  const float* y;        // HEAD 0: targets [nsteps * bs][OUT]; HEAD 1: actions [n][OUT]; HEAD 2: q [bs]
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
  float* loss_sum;       // HEAD 0 / 2: += sum over steps of the batch loss
  float* out;            // HEAD 1: [nsteps][4] actor loss, KL, dist, entropy
  float* slab;           // G > 1: [2][G][slab floats] gradient slabs (step parity)
  float* pbuf;           // G > 1: [param floats] the new parameters of each step
  int* ctr;              // arrival counter (zeroed per launch)
  int* err;              // set to 1 if an arrival wait timed out
  int spin;              // polls before an arrival wait times out (sppSetSgdSpinLimit; 0: the default)
  float* gout;           // non-null: ONE step's reduced gradient (canonical order) goes here instead of Adam --
                         // the data-parallel per-step path, whose caller all-reduces it and applies Adam
  float gscale;          // (gout) the gradient and the HEAD 1 partials are written times gscale (1 / ranks: the
                         // caller's all-reduce is then a plain sum)
};

template <int IN, int H2, int OUT, int HEAD, int WV = 4>
struct MlCfg {
  static_assert(WV == 2 || WV == 4 || WV == 8, "2, 4 or 8 waves per workgroup");
  static constexpr int R = 16 * WV;                 // rows per workgroup and step (16 per wave)
  static constexpr int TH = 64 * WV;                // threads
  static constexpr int RS = R + 4;                  // image row stride (result-layout stores: 64 distinct banks)
  static_assert(H2 == 32 || H2 == 64, "H2");
  static_assert(OUT >= 1 && OUT <= 32, "OUT");
  static constexpr int KQ1 = (IN + 1 + 3) / 4;     // fc1 k-steps (the inputs and the constant-1 row)
  static constexpr int SW1 = 4 * (KQ1 | 1);        // W1 row stride (odd multiple of 4: conflict-free A reads)
  static constexpr int NIT1 = (IN + 1 + 15) / 16;  // dW1 column tiles (inputs + the bias column)
  static constexpr int XTR = 16 * NIT1 > 4 * KQ1 ? 16 * NIT1 : 4 * KQ1;  // rows of the transposed input image
  static constexpr int NB2 = H2 / 16;              // layer-2 unit tiles
  static constexpr int NO = (OUT + 15) / 16;       // output tiles
  static constexpr int SW2 = 68;                   // W2 row stride (64 h1 units + 4)
  static constexpr int SW3 = H2 + 4;               // W3 row stride
  static constexpr int NT1 = 4 * NIT1, NT2 = NB2 * 4, NT3 = NO * NB2, NT = NT1 + NT2 + NT3;  // dW tiles
  static constexpr int IMGR = 128 + 2 * H2 + 16 * NO;  // image rows: H1, D1, H2, D2, D3
  static constexpr int NBP = H2 + 16 * NO + (HEAD == 1 ? 16 * NO : 0);  // per-wave bias partials: b2, b3 (, ls)
  // canonical layout: [log_scale (HEAD 1)] fc1.weight fc1.bias fc2.weight fc2.bias fc3.weight fc3.bias
  static constexpr int O_W1 = HEAD == 1 ? OUT : 0;
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
  static constexpr int K4 = (NP4 + TH - 1) / TH;  // float4 slots per thread (G = 1: all of them)
  static constexpr int NXP = (R * IN + TH - 1) / TH, NYP = (R * OUT + TH - 1) / TH;
  static_assert(SLAB <= kMlSlabMax && SLAB > NPS, "slab (and its dump word at NPS)");
  // G > 1: the shard's G slab chunks are staged in the image region, at most NP4 + G - 1 float4
  static constexpr int RED4 = IMGR * RS / 4;
  static constexpr int MAXG = RED4 - NP4 + 1 < kMlMaxWG ? RED4 - NP4 + 1 : kMlMaxWG;
  static constexpr int RLC = HEAD == 1 ? 4 : 8;  // slab float4 loads in flight per thread (register budget)
  static constexpr int NL = (NP4 + TH - 1) / TH;   // reloaded float4 per thread
};

__device__ __forceinline__ f32x4 ml_mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// tanh without branches.  Default (round 6, SPP_SGD_FAST_TANH=1): one odd 13 / 6 rational on the clamped range,
// <= 5 ulp of tanh on a dense float grid; ACM step 12.97 -> 12.7 us (w1), 15.2 -> 15.0 us (w8),
// profiles/r06/acm_step/ab_fast_tanh.txt.  0: |x| < 0.625 the odd polynomial of ocml's tanhf, else
// 1 - 2 / (e^{2|x|} + 1) with e^{2|x|} = 2^h (1 + l ln 2) from the split product 2|x| log2(e) = h + l (v_exp_f32,
// v_rcp_f32), both computed.  Either is within the SGD's fp32 tolerance (tests/test_gpu_parity.py,
// test_gpu_onpolicy.py, the reference PPO fixtures)
#ifndef SPP_SGD_FAST_TANH
#define SPP_SGD_FAST_TANH 1
#endif
__device__ __forceinline__ float ml_tanh(float x) {
#if SPP_SGD_FAST_TANH
  // one odd rational approximation on the clamped range (13 / 6 degrees, the minimax form of Eigen's fast float
  // tanh), its quotient through v_rcp_f32: no branch pair, half the issue cost of the two-branch form
  const float xc = fminf(fmaxf(x, -7.90531110763549805f), 7.90531110763549805f);
  const float x2 = xc * xc;
  float p = fmaf(x2, -2.76076847742355e-16f, 2.00018790482477e-13f);
  p = fmaf(x2, p, -8.60467152213735e-11f);
  p = fmaf(x2, p, 5.12229709037114e-08f);
  p = fmaf(x2, p, 1.48572235717979e-05f);
  p = fmaf(x2, p, 6.37261928875436e-04f);
  p = fmaf(x2, p, 4.89352455891786e-03f);
  p *= xc;
  float q = fmaf(x2, 1.19825839466702e-06f, 1.18534705686654e-04f);
  q = fmaf(x2, q, 2.26843463243900e-03f);
  q = fmaf(x2, q, 4.89352518554385e-03f);
  const float r = p * __builtin_amdgcn_rcpf(q);
  return fabsf(x) < 0.0004f ? x : r;
#else
  const float ax = fabsf(x);
  const float t2 = ax + ax;
  const float h = t2 * 1.44269504088896341f;
  const float l = fmaf(t2, 1.44269504088896341f, -h) + t2 * 1.925963033500e-8f;
  const float e = __builtin_amdgcn_exp2f(h) * fmaf(l, 0.693147180559945309f, 1.f);
  const float big = fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
  const float x2 = x * x;
  float p = fmaf(x2, -0.00570002059f, 0.0206340719f);
  p = fmaf(x2, p, -0.0537379310f);
  p = fmaf(x2, p, 0.133314162f);
  p = fmaf(x2, p, -0.333332807f);
  const float small = fmaf(x2, ax * p, ax);
  return copysignf(ax < 0.625f ? small : big, x);
#endif
}
// sum over the 16 lanes of a lane's DPP row (row_ror 8, 4, 2, 1: every lane ends with a row sum; callers take
// lane 0 of the row, so the order is fixed)
template <int CTRL>
__device__ __forceinline__ float ml_dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float ml_row16_sum(float v) {
  v += ml_dpp<0x128>(v);
  v += ml_dpp<0x124>(v);
  v += ml_dpp<0x122>(v);
  v += ml_dpp<0x121>(v);
  return v;
}
// sum over the wave: the 4 row sums (lanes 0, 16, 32, 48) added in a fixed order (uniform result)
__device__ __forceinline__ float ml_wave_sum(float v) {
  v = ml_row16_sum(v);
  const int b = __builtin_bit_cast(int, v);
  auto lane_v = [&](int l) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, l)); };
  return (lane_v(0) + lane_v(16)) + (lane_v(32) + lane_v(48));
}

// LDS words addressed by 32-bit offsets held in registers (ds_write with a VGPR address, no generic pointer)
typedef __attribute__((address_space(3))) float ml_lds_f;
__device__ __forceinline__ uint32_t lds_off(float* p) { return (uint32_t)(uintptr_t)(ml_lds_f*)p; }
__device__ __forceinline__ void lds_st(uint32_t off, float v) { *(ml_lds_f*)(uintptr_t)off = v; }

// WV = 8: two waves per SIMD (128 rows per workgroup, half the workgroups of a step): every latency of one
// wave's chain (LDS reads, dependent MFMAs, tanh) overlaps the other wave's work; <= 256 registers per wave.
// MP (HEAD 0, G > 1): a step's rows per workgroup may exceed R, run as passes of R rows whose gradients add up in
// the canonical LDS staging before the exchange (as HEAD 2): fewer workgroups meet at each step's two hand-offs.
template <int IN, int H2, int OUT, int HEAD, bool MW, int WV = 4, bool MP = false>
__global__ __launch_bounds__(64 * WV, 1) void k_mlp_sgd(MlpSgdArgs a) {
  using C = MlCfg<IN, H2, OUT, HEAD, WV>;
  constexpr int TH = C::TH;
  constexpr bool GAUSS = HEAD == 1, VALUE = HEAD == 2;
  static_assert(!MP || (MW && HEAD == 0), "passes: the multi-workgroup AcM form");
  // G > 1, one pass per step: every gradient element goes to this workgroup's slab as soon as it is final
  // (write-through stores issued under the remaining tiles' MFMAs), not through the canonical LDS staging
  constexpr bool DIRECT = MW && !VALUE && !MP;
  static_assert(!VALUE || OUT == 1, "value head");
  constexpr int RS = C::RS, R = C::R, NP = C::NP, SW1 = C::SW1, SW2 = C::SW2, SW3 = C::SW3, NB2 = C::NB2,
                NO = C::NO;
  __shared__ __attribute__((aligned(16))) float IMG[C::IMGR * RS];  // H1 | D1 | H2 | D2 | D3; G > 1: the slab chunks
  __shared__ __attribute__((aligned(16))) float XT[C::XTR * RS];    // [input][sample]; row IN = 1 (rows < bs)
  // the step's gradient, canonical order (+ dump words at NPS, NPS + 1); the direct-store form (DIRECT) keeps
  // only the dump word (its gradient goes straight to the slab)
  constexpr int GRN = DIRECT ? 4 : C::NPS + 4, GRD = DIRECT ? 1 : C::NPS + 1;
  __shared__ __attribute__((aligned(16))) float GR[GRN];
  __shared__ __attribute__((aligned(16))) float W1[64 * SW1];       // [unit][input]; column IN = b1
  __shared__ __attribute__((aligned(16))) float W2[H2 * SW2];
  __shared__ __attribute__((aligned(16))) float W3[16 * NO * SW3];  // rows >= OUT zero
  __shared__ float B2[H2], B3[16 * NO], LS[32], LIM[32];
  __shared__ float Y[R * OUT];
  __shared__ float LPO[GAUSS ? R : 1], ADV[GAUSS ? R : 1];
  __shared__ int64_t IDX[GAUSS ? 2 * R : 1];
  __shared__ float BP[WV][C::NBP];   // per wave: bias (and log_scale) gradient partials over its 16 samples
  __shared__ float SCP[WV][4];       // per wave: scalar partials
  __shared__ float GT[GAUSS ? WV : 1][3][32];  // HEAD 1, per wave: scale, variance, log(scale) of the step's log_scale
  __shared__ float adam_s[2][2];
  __shared__ int s_dead;
  float* const H1I = IMG;
  float* const D1I = IMG + 64 * RS;
  float* const H2I = IMG + 128 * RS;
  float* const D2I = H2I + H2 * RS;
  float* const D3I = D2I + H2 * RS;
  const int t = threadIdx.x, lane = t & 63, q = lane >> 4, n = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);  // wave-uniform: the tile choices below are scalar
  const int col = 16 * w + n;  // this lane's sample (image column)
  const int G = MW ? (int)gridDim.x : 1, g = MW ? (int)blockIdx.x : 0;
  const int r0 = MW ? g * a.bsl : 0;
  auto step_rows = [&](int st) { return st == a.nsteps - 1 ? a.bs_last : a.bs; };  // the step's batch
  auto wg_rows = [&](int st) {  // this workgroup's rows of step st
    return MW ? max(0, min(a.bsl, step_rows(st) - r0)) : step_rows(st);
  };
  // passes of <= 64 rows: pass p = step p / nsub, rows [64 (p % nsub), +64) of the workgroup's rows
  const int nsub = (MW && (VALUE || MP)) ? (a.bsl + R - 1) / R : 1;  // (else one pass: the host keeps bsl <= R)
  auto pass_rows = [&](int p) {
    const int st = p / nsub;
    return st < a.nsteps ? max(0, min(R, wg_rows(st) - R * (p - st * nsub))) : 0;
  };
  if (t == 0) s_dead = 0;
  // ---- the canonical element c (< NP) of the parameters inside the LDS images
  auto pref = [&](int c) -> float& {
    if (GAUSS && c < C::O_W1) return LS[c];
    if (c < C::O_B1) { const int e = c - C::O_W1; return W1[(e / IN) * SW1 + e % IN]; }
    if (c < C::O_W2) return W1[(c - C::O_B1) * SW1 + IN];
    if (c < C::O_B2) { const int e = c - C::O_W2; return W2[(e >> 6) * SW2 + (e & 63)]; }
    if (c < C::O_W3) return B2[c - C::O_B2];
    if (c < C::O_B3) { const int e = c - C::O_W3; return W3[(e / H2) * SW3 + e % H2]; }
    return B3[c - C::O_B3];
  };
  // ---- images (zero padding)
  for (int i = t; i < 64 * SW1; i += TH) W1[i] = 0.f;
  for (int i = t; i < H2 * SW2; i += TH) W2[i] = 0.f;
  for (int i = t; i < 16 * NO * SW3; i += TH) W3[i] = 0.f;
  for (int i = t; i < C::XTR * RS; i += TH) XT[i] = 0.f;  // rows > IN stay zero
  if (t < 16 * NO) B3[t] = 0.f;
  if (t < 32) {
    LS[t] = 0.f;
    LIM[t] = t < OUT ? a.lim[t] : 0.f;
  }
  __syncthreads();
  for (int c = t; c < NP; c += TH) pref(c) = a.params[c];
  // ---- Adam moments of the owned float4 slots: slot f = f0 + t + 256 k (this workgroup's shard)
  const int C4 = (C::NP4 + G - 1) / G, f0 = g * C4, f1 = min(f0 + C4, C::NP4);
  const int c4n = max(f1 - f0, 0);  // this shard's float4 slots
  // (SPP_SGD_PRED) partial-sum groups of the shard reduce: as many as the threads cover, at most G
  const int npg = max(1, min(G, TH / max(c4n, 1)));
  // ---- Adam moments of the owned elements: element c = e0 + t + TH k of the shard [e0, e1) (one element per
  // thread and k: the shard's Adam is spread over the workgroup's threads, not its float4 slots)
  const int e0 = 4 * f0, e1 = min(4 * f1, NP);
  // (MW: G >= 2, so a shard holds at most 4 ceil(NP4 / 2) elements)
  constexpr int KE = MW ? (4 * ((C::NP4 + 1) / 2) + TH - 1) / TH : (NP + TH - 1) / TH;
  float mom[KE], vel[KE];
#pragma unroll
  for (int k = 0; k < KE; ++k) {
    const int c = e0 + t + TH * k;
    const bool own = c < e1;
    mom[k] = own ? a.m[c] : 0.f;
    vel[k] = own ? a.v[c] : 0.f;
  }
  double pw1 = 0.0, pw2 = 0.0;  // beta1^t, beta2^t of the next step (thread TH - 1: pow once, then products)
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
  // ---- register prefetch of one pass's rows (HEAD 1: through the step's indices in IDX)
  float xp[C::NXP], yp[C::NYP], nxp[GAUSS ? C::NYP : 1], lpp = 0.f, advp = 0.f;
  auto row_of = [&](int p, int r) -> int64_t {
    if constexpr (GAUSS) return IDX[(p & 1) * R + r];
    else {
      const int st = p / nsub;
      return (VALUE ? 0 : (int64_t)st * a.bs) + r0 + R * (p - st * nsub) + r;  // (HEAD 2: the same batch)
    }
  };
  auto prefetch = [&](int p) {
    const int bs = pass_rows(p);
    const bool live = bs > 0;
    if constexpr (!GAUSS) {  // HEAD 0 / 2: the pass's rows are contiguous, element i of the block at row 0 + i
      // (buffer loads ranged to the pass's rows: past them, and for a dead pass, the hardware returns 0 -- no
      // per-element branch)
      const float* xb = a.x + (live ? row_of(p, 0) * IN : 0);
      const float* yb = a.y + (live ? row_of(p, 0) * OUT : 0);
      const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xb), (short)0, live ? 4 * bs * IN : 0,
                                                        0x00020000);
      const auto yr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(yb), (short)0, live ? 4 * bs * OUT : 0,
                                                        0x00020000);
#pragma unroll
      for (int k = 0; k < C::NXP; ++k)
        xp[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, 4u * (uint32_t)(t + TH * k), 0, 0));
#pragma unroll
      for (int k = 0; k < C::NYP; ++k)
        yp[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(yr, 4u * (uint32_t)(t + TH * k), 0, 0));
      return;
    }
#pragma unroll
    for (int k = 0; k < C::NXP; ++k) {
      const int i = t + TH * k, r = i / IN;
      xp[k] = (live && i < bs * IN) ? a.x[row_of(p, r) * IN + i % IN] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < C::NYP; ++k) {
      const int i = t + TH * k, r = i / OUT;
      const bool ok = live && i < bs * OUT;
      yp[k] = ok ? a.y[row_of(p, r) * OUT + i % OUT] : 0.f;
      // the dist loss is data only: its per-step sum is taken when the rows are staged (not here, where it
      // would wait for these loads instead of leaving them in flight under the step)
      if constexpr (GAUSS) nxp[k] = ok ? a.nxt[row_of(p, r) * OUT + i % OUT] : 0.f;
    }
    if constexpr (GAUSS) {
      lpp = (live && t < bs) ? a.lp_old[row_of(p, t)] : 0.f;
      advp = (live && t < bs) ? a.adv[row_of(p, t)] : 0.f;
    }
  };
  auto load_idx = [&](int p) {  // HEAD 1 (one pass per step): step p's row indices -> IDX[p & 1]
    if constexpr (GAUSS)
      if (t < R) IDX[(p & 1) * R + t] = t < pass_rows(p) ? a.idx[(int64_t)p * a.bs + r0 + t] : 0;
  };
  // ---- a prefetched step's rows into LDS: inputs transposed (rows >= bs: zeros), the constant-1 row
  float dist_next = 0.f;
  auto stage = [&](int p) {
#pragma unroll
    for (int k = 0; k < C::NXP; ++k) {
      const int i = t + TH * k;
      if (i < R * IN) XT[(i % IN) * RS + i / IN] = xp[k];
    }
    if (t < R) XT[IN * RS + t] = t < pass_rows(p) ? 1.f : 0.f;
#pragma unroll
    for (int k = 0; k < C::NYP; ++k) {
      const int i = t + TH * k;
      if (i < R * OUT) Y[i] = yp[k];
    }
    if constexpr (GAUSS) {
      if (t < R) {
        LPO[t] = lpp;
        ADV[t] = advp;
      }
    }
    if constexpr (GAUSS) {
      float dsum = 0.f;
#pragma unroll
      for (int k = 0; k < C::NYP; ++k) {
        const float e = yp[k] - nxp[k];  // (rows past the batch: 0 - 0)
        dsum = fmaf(e, e, dsum);
      }
      dist_next = dsum;
    }
  };
  load_idx(0);
  if (t == TH - 1) adam_scalars(0);
  __syncthreads();
  prefetch(0);
  load_idx(1);
  stage(0);
  __syncthreads();
  // G > 1: the LDS image word of each canonical element this thread reloads after the publish (slot
  // f = t + 256 k, element i; elements past the parameters -> a dump word), resolved once for the launch
  uint32_t roff[MW ? C::NL : 1][4];
#pragma unroll
  for (int k = 0; k < (MW ? C::NL : 1); ++k)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = 4 * (t + TH * k) + i;
      roff[k][i] = lds_off(c < NP ? &pref(c) : &GR[GRD]);
    }
  SPP_TP_INIT();
  float loss_acc = 0.f;  // HEAD 0 / 2: sum over steps of the batch loss (the scalar slot's owner)
  const float lo = 1.f - a.eps_clip, hi = 1.f + a.eps_clip;
  int p = 0;  // pass
  for (int st = 0; st < a.nsteps; ++st) {
    const int bsg = step_rows(st);
    const float inv_bs = 1.f / (float)bsg;
    const auto mine = sgd_rsrc(a.slab + ((int64_t)(st & 1) * G + g) * C::SLAB);  // (G > 1) this step's slab
    float dist_step = 0.f;
   for (int sb = 0; sb < nsub; ++sb, ++p) {
    const int bs = pass_rows(p);
    dist_step = dist_next;
    prefetch(p + 1);  // (IDX[(p + 1) & 1]: written a pass ago, behind the last pass's barrier)
    load_idx(p + 2);  // IDX[p & 1]: its last reader was prefetch(p), issued a pass ago
    SPP_TP(0);
    const bool svalid = col < bs;
    auto acc_to = [&](float& dst, float v) { dst = sb ? dst + v : v; };  // passes of one step add up
    // ---- fc1: h1 = tanh(W1 [x; 1]), 4 unit tiles of this wave's 16 samples
    f32x4 h1r[4];
    {
      f32x4 acc[4];
#pragma unroll
      for (int T = 0; T < 4; ++T) acc[T] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < C::KQ1; ++ks) {
        const float xb = XT[(4 * ks + q) * RS + col];
#pragma unroll
        for (int T = 0; T < 4; ++T) acc[T] = ml_mfma16(W1[(16 * T + n) * SW1 + 4 * ks + q], xb, acc[T]);
      }
#pragma unroll
      for (int T = 0; T < 4; ++T)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          h1r[T][i] = ml_tanh(acc[T][i]);
          H1I[(16 * T + 4 * q + i) * RS + col] = h1r[T][i];
        }
    }
    SPP_TP(1);
    // ---- fc2: h2 = tanh(W2 h1 + b2); k-step (T, j) of lane group q = h1 unit 16T + 4q + j (h1r[T][j])
    f32x4 h2r[NB2];
    {
      f32x4 acc[NB2];
#pragma unroll
      for (int T2 = 0; T2 < NB2; ++T2)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[T2][i] = B2[16 * T2 + 4 * q + i];
#pragma unroll
      for (int T = 0; T < 4; ++T)
#pragma unroll
        for (int T2 = 0; T2 < NB2; ++T2) {
          const float4 w4 = *reinterpret_cast<const float4*>(W2 + (16 * T2 + n) * SW2 + 16 * T + 4 * q);
          acc[T2] = ml_mfma16(w4.x, h1r[T][0], acc[T2]);
          acc[T2] = ml_mfma16(w4.y, h1r[T][1], acc[T2]);
          acc[T2] = ml_mfma16(w4.z, h1r[T][2], acc[T2]);
          acc[T2] = ml_mfma16(w4.w, h1r[T][3], acc[T2]);
        }
#pragma unroll
      for (int T2 = 0; T2 < NB2; ++T2)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          h2r[T2][i] = ml_tanh(acc[T2][i]);
          H2I[(16 * T2 + 4 * q + i) * RS + col] = h2r[T2][i];
        }
    }
    SPP_TP(11);
    // ---- fc3 and the head: d3r = d loss / d z3 (rows >= OUT zero)
    f32x4 d3r[NO];
    {
      f32x4 acc[NO];
#pragma unroll
      for (int T3 = 0; T3 < NO; ++T3)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[T3][i] = B3[16 * T3 + 4 * q + i];
#pragma unroll
      for (int T = 0; T < NB2; ++T)
#pragma unroll
        for (int T3 = 0; T3 < NO; ++T3) {
          const float4 w4 = *reinterpret_cast<const float4*>(W3 + (16 * T3 + n) * SW3 + 16 * T + 4 * q);
          acc[T3] = ml_mfma16(w4.x, h2r[T][0], acc[T3]);
          acc[T3] = ml_mfma16(w4.y, h2r[T][1], acc[T3]);
          acc[T3] = ml_mfma16(w4.z, h2r[T][2], acc[T3]);
          acc[T3] = ml_mfma16(w4.w, h2r[T][3], acc[T3]);
        }
      SPP_TP(12);
      if constexpr (HEAD == 0) {
        float lpart = 0.f;
        const float inv_n = 1.f / (float)(bsg * OUT);
#pragma unroll
        for (int T3 = 0; T3 < NO; ++T3)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int u = 16 * T3 + 4 * q + i;
            float d = 0.f;
            if (u < OUT) {
              const float th = ml_tanh(acc[T3][i]), lm = LIM[u];
              const float e = th * lm - Y[col * OUT + u];
              if (svalid) {
                lpart = fmaf(e, e, lpart);
                d = 2.f * e * inv_n * lm * (1.f - th * th);
              }
            }
            d3r[T3][i] = d;
          }
        lpart = ml_wave_sum(lpart);
        if (lane == 0) acc_to(SCP[w][0], lpart);
      } else if constexpr (VALUE) {  // value head: v = z3 (linear), loss 0.5 (q - v)^2 (a2c.py:209-219)
        float lpart = 0.f;
        const float inv_n = 1.f / (float)bsg;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float d = 0.f;
          if (q == 0 && i == 0 && svalid) {
            const float e = fsub_rn(Y[col], acc[0][i]);
            lpart = 0.5f * e * e;
            d = -e * inv_n;
          }
          d3r[0][i] = d;
        }
        lpart = ml_wave_sum(lpart);
        if (lane == 0) acc_to(SCP[w][0], lpart);
      } else {
        // log_prob of the stored action (torch Normal: -(a-mu)^2/(2 var) - log(scale) - log(sqrt(2 pi)), summed
        // over the outputs: this lane's registers, then the sample's 4 lane groups).  The per-output scale terms
        // once per wave and step (the same values every use: scale = exp(log_scale), its square and log)
        if (lane < OUT) {
          const float sc = expf(LS[lane]);
          GT[w][0][lane] = sc;
          GT[w][1][lane] = fmul_rn(sc, sc);
          GT[w][2][lane] = logf(sc);
        }
        SPP_XLANE_SYNC();
        float th[NO][4], dd[NO][4], lp = 0.f;
#pragma unroll
        for (int T3 = 0; T3 < NO; ++T3)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int u = 16 * T3 + 4 * q + i;
            th[T3][i] = 0.f;
            dd[T3][i] = 0.f;
            if (u < OUT) {
              th[T3][i] = ml_tanh(acc[T3][i]);
              const float mu = fmul_rn(th[T3][i], LIM[u]);
              dd[T3][i] = fsub_rn(Y[col * OUT + u], mu);
              lp += fsub_rn(fsub_rn(fdiv_rn(-fmul_rn(dd[T3][i], dd[T3][i]), 2.f * GT[w][1][u]), GT[w][2][u]),
                            kLogSqrt2PiO);
            }
          }
        lp += __shfl_xor(lp, 16, 64);
        lp += __shfl_xor(lp, 32, 64);
        // clip objective (ppo.py:194-204) and its gradient wrt lp_new (torch minimum / clamp rules)
        float mterm = 0.f, kl = 0.f, glp = 0.f;
        if (svalid) {
          const float lpo = LPO[col], A = ADV[col];
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
        for (int T3 = 0; T3 < NO; ++T3)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int u = 16 * T3 + 4 * q + i;
            float d = 0.f, lsg = 0.f;
            if (u < OUT) {
              const float var = GT[w][1][u];
              const float gmu = glp * dd[T3][i] / var;
              lsg = glp * (dd[T3][i] * dd[T3][i] / var - 1.f);
              d = gmu * LIM[u] * (1.f - th[T3][i] * th[T3][i]);
            }
            d3r[T3][i] = d;
            lsg = ml_row16_sum(lsg);  // the log_scale gradient over this wave's 16 samples
            if (n == 0 && u < OUT) acc_to(BP[w][H2 + 16 * NO + u], lsg);
          }
        const float sm_ = ml_wave_sum(q == 0 ? mterm : 0.f), sk = ml_wave_sum(q == 0 ? kl : 0.f);
        if (lane == 0) {
          acc_to(SCP[w][0], sm_);
          acc_to(SCP[w][1], sk);
        }
      }
      SPP_TP(13);
#pragma unroll
      for (int T3 = 0; T3 < NO; ++T3)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          D3I[(16 * T3 + 4 * q + i) * RS + col] = d3r[T3][i];
          const float s = ml_row16_sum(d3r[T3][i]);  // b3's gradient over this wave's samples
          if (n == 0) acc_to(BP[w][H2 + 16 * T3 + 4 * q + i], s);
        }
    }
    SPP_TP(2);
    // ---- dz2 = (W3^T dz3) * (1 - h2^2); k-step (T3, j) = output 16 T3 + 4q + j
    f32x4 d2r[NB2];
    {
#pragma unroll
      for (int T2 = 0; T2 < NB2; ++T2) d2r[T2] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int T3 = 0; T3 < NO; ++T3)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int T2 = 0; T2 < NB2; ++T2)
            d2r[T2] = ml_mfma16(W3[(16 * T3 + 4 * q + j) * SW3 + 16 * T2 + n], d3r[T3][j], d2r[T2]);
#pragma unroll
      for (int T2 = 0; T2 < NB2; ++T2)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          d2r[T2][i] *= 1.f - h2r[T2][i] * h2r[T2][i];
          D2I[(16 * T2 + 4 * q + i) * RS + col] = d2r[T2][i];
          const float s = ml_row16_sum(d2r[T2][i]);  // b2's gradient over this wave's samples
          if (n == 0) acc_to(BP[w][16 * T2 + 4 * q + i], s);
        }
    }
    // ---- dz1 = (W2^T dz2) * (1 - h1^2)
    {
      f32x4 acc[4];
#pragma unroll
      for (int T = 0; T < 4; ++T) acc[T] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int T2 = 0; T2 < NB2; ++T2)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int T = 0; T < 4; ++T)
            acc[T] = ml_mfma16(W2[(16 * T2 + 4 * q + j) * SW2 + 16 * T + n], d2r[T2][j], acc[T]);
#pragma unroll
      for (int T = 0; T < 4; ++T)
#pragma unroll
        for (int i = 0; i < 4; ++i) D1I[(16 * T + 4 * q + i) * RS + col] = acc[T][i] * (1.f - h1r[T][i] * h1r[T][i]);
    }
    __syncthreads();  // the images hold all 64 samples
    SPP_TP(3);
    // ---- weight gradients: 16x16 tiles over the R samples (k-step ks of lane group q = sample (R/4) q + ks),
    // tiles w, w + WV, ... of this wave two at a time; each finished tile goes to GR in canonical order
    auto tile_rows = [&](int tt, const float*& ar, const float*& br, int& layer, int& mt, int& nt) {
      if (tt < C::NT1) {
        layer = 0; mt = tt / C::NIT1; nt = tt - mt * C::NIT1;
        ar = D1I; br = XT;
      } else if (tt < C::NT1 + C::NT2) {
        const int u = tt - C::NT1;
        layer = 1; mt = u >> 2; nt = u & 3;
        ar = D2I; br = H1I;
      } else {
        const int u = tt - C::NT1 - C::NT2;
        layer = 2; mt = u / NB2; nt = u - mt * NB2;
        ar = D3I; br = H2I;
      }
      ar += (16 * mt + n) * RS + (R / 4) * q;
      br += (16 * nt + n) * RS + (R / 4) * q;
    };
    // (elements outside the parameters -- dW1's padding columns, dW3's rows >= OUT -- go to the dump word
    // GR[NPS]: every lane stores, no divergent branch)
    auto tile_store = [&](const f32x4& acc, int layer, int mt, int nt) {
      const int row0 = 16 * mt + 4 * q, cu = 16 * nt + n;
      int c0, dc;
      if (layer == 0) {
        c0 = cu < IN ? C::O_W1 + row0 * IN + cu : C::O_B1 + row0;
        dc = cu < IN ? IN : 1;
      } else if (layer == 1) {
        c0 = C::O_W2 + row0 * 64 + cu;
        dc = 64;
      } else {
        c0 = C::O_W3 + row0 * H2 + cu;
        dc = H2;
      }
      const bool col_ok = layer != 0 || cu <= IN;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool ok = col_ok && (layer != 2 || row0 + i < OUT);
        if constexpr (DIRECT) slab_st1(mine, ok ? c0 + i * dc : C::NPS, acc[i]);
        else acc_to(GR[ok ? c0 + i * dc : C::NPS], acc[i]);
      }
    };
    for (int tt = w; tt < C::NT; tt += 2 * WV) {  // (wave-uniform; a missing second tile repeats the first)
      const bool two = tt + WV < C::NT;
      const float *a0, *b0, *a1, *b1;
      int l0, m0, n0, l1, m1, n1;
      tile_rows(tt, a0, b0, l0, m0, n0);
      tile_rows(two ? tt + WV : tt, a1, b1, l1, m1, n1);
      f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
      float4 x0 = reinterpret_cast<const float4*>(a0)[0], y0 = reinterpret_cast<const float4*>(b0)[0];
      float4 x1 = reinterpret_cast<const float4*>(a1)[0], y1 = reinterpret_cast<const float4*>(b1)[0];
      constexpr int NCQ = R / 16;  // float4 groups of a lane group's R / 4 samples
#pragma unroll
      for (int cq = 0; cq < NCQ; ++cq) {
        float4 nx0, ny0, nx1, ny1;
        if (cq < NCQ - 1) {  // the next 4 samples' operands in flight under this group's MFMAs
          nx0 = reinterpret_cast<const float4*>(a0)[cq + 1];
          ny0 = reinterpret_cast<const float4*>(b0)[cq + 1];
          nx1 = reinterpret_cast<const float4*>(a1)[cq + 1];
          ny1 = reinterpret_cast<const float4*>(b1)[cq + 1];
        }
        c0 = ml_mfma16(x0.x, y0.x, c0);
        c1 = ml_mfma16(x1.x, y1.x, c1);
        c0 = ml_mfma16(x0.y, y0.y, c0);
        c1 = ml_mfma16(x1.y, y1.y, c1);
        c0 = ml_mfma16(x0.z, y0.z, c0);
        c1 = ml_mfma16(x1.z, y1.z, c1);
        c0 = ml_mfma16(x0.w, y0.w, c0);
        c1 = ml_mfma16(x1.w, y1.w, c1);
        if (cq < NCQ - 1) {
          x0 = nx0; y0 = ny0; x1 = nx1; y1 = ny1;
        }
      }
      SPP_TP(9);
      tile_store(c0, l0, m0, n0);
      if (two) tile_store(c1, l1, m1, n1);
      SPP_TP(10);
    }
    SPP_TP(4);
    if (sb + 1 < nsub) {  // the step's next pass: its rows into LDS once every wave is done with this one's
      __syncthreads();
      stage(p + 1);
      __syncthreads();
    }
   }  // passes
    // ---- bias (and log_scale) gradients: the waves' partials in a fixed order; scalars -> GR[O_SC ..]
    {
      auto wsum = [&](int j) {  // waves in order
        float v = BP[0][j];
#pragma unroll
        for (int k = 1; k < WV; ++k) v += BP[k][j];
        return v;
      };
      auto scsum = [&](int j) {
        float v = SCP[0][j];
#pragma unroll
        for (int k = 1; k < WV; ++k) v += SCP[k][j];
        return v;
      };
      auto put = [&](int c, float v) {
        if constexpr (DIRECT) slab_st1(mine, c, v);
        else GR[c] = v;
      };
      if (t < H2) put(C::O_B2 + t, wsum(t));
      else if (t < H2 + OUT) put(C::O_B3 + t - H2, wsum(t));
      else if (GAUSS && t >= 128 && t < 128 + OUT) {  // - ent_coef * d entropy / d log_scale (once: workgroup 0)
        const int u = t - 128;
        const float s = wsum(H2 + 16 * NO + u);
        put(u, (g == 0) ? s - a.ent_coef : s);
      }
      // scalars (HEAD 1's dist partial at O_SC + 2 is written below, after its reduction)
      if (t < 4 && !(GAUSS && t == 2))
        put(C::O_SC + t, t == 0 ? scsum(0) : (GAUSS && t == 1 ? scsum(1) : 0.f));
      if (t >= 192 && t - 192 < C::O_SC - NP) put(NP + t - 192, 0.f);
    }
    if constexpr (GAUSS) {  // the dist partials of every thread (this step's rows)
      const float ds = ml_wave_sum(dist_step);
      if (lane == 0) SCP[w][2] = ds;
    }
    __syncthreads();
    if constexpr (GAUSS) {
      if (t == 0) {
        float ds = SCP[0][2];
#pragma unroll
        for (int k = 1; k < WV; ++k) ds += SCP[k][2];
        if constexpr (DIRECT) slab_st1(mine, C::O_SC + 2, ds);
        else GR[C::O_SC + 2] = ds;
      }
      __syncthreads();
    }
    // ---- exchange (G > 1) and Adam on this workgroup's shard
    float entropy = 0.f;
    if (GAUSS && g == 0 && t == 0) {  // of the parameters this step's forward used (before the update)
      double ent = 0.0;
      for (int j = 0; j < OUT; ++j) ent += 0.5 + 0.91893853320467274178 + (double)LS[j];
      entropy = (float)ent;
    }
    SPP_TP(5);
    const auto all = sgd_rsrc(a.slab + (int64_t)(st & 1) * G * C::SLAB);  // (G = 1: unused)
    if constexpr (MW) {
      if constexpr (!DIRECT)  // (HEAD 2, MP: the passes' sums staged in GR)
        for (int f = t; f < C::NP4; f += TH) {
          const float4 v4 = *reinterpret_cast<const float4*>(GR + 4 * f);
          slab_st4(mine, 4 * f, v4);
        }
      // the next step's Adam scalars (thread 255's double-precision powers) while lane 0 polls
      sgd_arrive_wait_wt(a.ctr, G * (2 * st + 1), a.err, &s_dead, a.spin, [&] {
        if (t == TH - 1) adam_scalars(st + 1);
      });
      SPP_TP(14);
#if SPP_SGD_PRED
      // this shard's chunk of every slab, summed on the way in: item u = (group pg, slot j) adds the slabs
      // pg, pg + P, ... of slot j in that order (all of a thread's loads in flight at once) -> the image region
      // [pg][c4n]; Adam adds the P group sums in order (a fixed order: every workgroup and replica the same)
      for (int u = t; u < npg * c4n; u += TH) {
        const int pg = u / c4n, j = u - pg * c4n;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int s0 = pg; s0 < G; s0 += npg * C::RLC) {
          float4 ld[C::RLC];
#pragma unroll
          for (int k = 0; k < C::RLC; ++k) {
            const int src = s0 + npg * k;
            if (src < G) ld[k] = slab_ld4(all, src * C::SLAB + 4 * (f0 + j));
          }
#pragma unroll
          for (int k = 0; k < C::RLC; ++k)
            if (s0 + npg * k < G) {
              acc.x += ld[k].x; acc.y += ld[k].y; acc.z += ld[k].z; acc.w += ld[k].w;
            }
        }
        reinterpret_cast<float4*>(IMG)[u] = acc;
      }
#else
      // this shard's chunk of every slab -> the image region, [p][c4n] (the images are dead until the next step)
      const int nit = c4n * G;
      for (int i0 = 0; i0 < nit; i0 += C::RLC * TH) {  // (G = 17, 64-wide AcM: one round)
        float4 ld[C::RLC];
#pragma unroll
        for (int k = 0; k < C::RLC; ++k) {
          const int i = i0 + t + TH * k;
          if (i < nit) {
            const int src = i / c4n;
            ld[k] = slab_ld4(all, src * C::SLAB + 4 * (f0 + i - src * c4n));
          }
        }
#pragma unroll
        for (int k = 0; k < C::RLC; ++k) {
          const int i = i0 + t + TH * k;
          if (i < nit) reinterpret_cast<float4*>(IMG)[i] = ld[k];
        }
      }
#endif
      __syncthreads();
    }
    SPP_TP(6);
    const float neg_step = adam_s[st & 1][0], bc2s = adam_s[st & 1][1];
    if (!MW && t == TH - 1) adam_scalars(st + 1);  // (G > 1: computed during the arrival wait)
    const float omb1 = 0.1f, b2c = 0.999f, omb2 = 0.001f, eps = 1e-8f;
    const auto pub = sgd_rsrc(a.pbuf);
#pragma unroll
    for (int k = 0; k < KE; ++k) {
      const int c = e0 + t + TH * k;
      if (c < e1) {
        float gi;
        if constexpr (MW) {  // the shard's partial sums in order (SPP_SGD_PRED: npg group sums; else the G slabs)
          const float* red = IMG + (c - e0);
          gi = 0.f;
          for (int src = 0; src < (SPP_SGD_PRED ? npg : G); ++src) gi += red[src * 4 * c4n];
        } else {
          gi = GR[c];
        }
        if (a.gout) {  // gradient-only launch: the reduced gradient out, the parameters untouched
          a.gout[c] = gi * a.gscale;
          continue;
        }
        float& pv = pref(c);
        if (c < NP) {  // torch.optim.Adam (k_adam's operation order)
          mom[k] = fadd_rn(mom[k], fmul_rn(omb1, fsub_rn(gi, mom[k])));
          vel[k] = fadd_rn(fmul_rn(vel[k], b2c), fmul_rn(fmul_rn(omb2, gi), gi));
          const float denom = fadd_rn(fdiv_rn(sqrtf(vel[k]), bc2s), eps);
          pv = fadd_rn(pv, fmul_rn(neg_step, fdiv_rn(mom[k], denom)));
        }
        if constexpr (MW)
#pragma unroll
          for (int rep = 0; rep < kSgdPubReps; ++rep) slab_st1(pub, rep * kMlSlabMax + c, pv);
      }
    }
    // the scalar partials (the shard holding slot O_SC; elements past the parameters, not in e1's range)
    if (C::O_SC >= e0 && C::O_SC < 4 * f1 && t < 3) {
      float gv = 0.f;
      if constexpr (MW)
        for (int src = 0; src < (SPP_SGD_PRED ? npg : G); ++src) gv += IMG[src * 4 * c4n + (C::O_SC - e0) + t];
      else
        gv = GR[C::O_SC + t];
      if constexpr (!GAUSS) {  // (HEAD 2: the partials are 0.5 e^2; OUT = 1)
        if (t == 0) loss_acc += gv * (1.f / (float)(bsg * OUT));
      } else {
        const double d = t == 0 ? -(double)bsg : (t == 1 ? (double)bsg : (double)bsg * OUT);
        a.out[(int64_t)st * 4 + t] = (float)((double)gv / d) * (a.gout ? a.gscale : 1.f);
      }
    }
    if (GAUSS && g == 0 && t == 0) a.out[(int64_t)st * 4 + 3] = entropy * (a.gout ? a.gscale : 1.f);
    // the next step's rows into LDS while the other workgroups publish (XT, Y, LPO, ADV: last read by this
    // step's head and dW tiles, before the gradient staging barrier)
    stage(p);
    SPP_TP(7);
    if constexpr (MW) {
     if (!a.gout) {  // (a gradient-only launch is one step: nothing published, nothing to reload)
      sgd_arrive_wait_wt(a.ctr, G * (2 * st + 2), a.err, &s_dead, a.spin);
      SPP_TP(15);
      float4 rv[C::NL];
#pragma unroll
      for (int k = 0; k < C::NL; ++k) {  // (this shard's own slots reload the values it published)
        rv[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (t + TH * k < C::NP4) rv[k] = slab_ld4(pub, (g % kSgdPubReps) * kMlSlabMax + 4 * (t + TH * k));
      }
#pragma unroll
      for (int k = 0; k < C::NL; ++k) {
        lds_st(roff[k][0], rv[k].x);
        lds_st(roff[k][1], rv[k].y);
        lds_st(roff[k][2], rv[k].z);
        lds_st(roff[k][3], rv[k].w);
      }
     }
    }
    __syncthreads();
    SPP_TP(8);
  }
  SPP_TP_FLUSH();
  // ---- write back: parameters (workgroup 0, from its images), moments (each shard's owner)
  if (a.gout) {  // (gradient-only: nothing changed; the loss sum below still goes out)
    if (!GAUSS && C::O_SC >= e0 && C::O_SC < 4 * f1 && t == 0) *a.loss_sum += loss_acc;
    return;
  }
  if (g == 0)
    for (int c = t; c < NP; c += TH) a.params[c] = pref(c);
#pragma unroll
  for (int k = 0; k < KE; ++k) {
    const int c = e0 + t + TH * k;
    if (c < e1) {
      a.m[c] = mom[k];
      a.v[c] = vel[k];
    }
  }
  // the loss sum: thread 0 of the shard holding the scalar slot
  if (!GAUSS && C::O_SC >= e0 && C::O_SC < 4 * f1 && t == 0) *a.loss_sum += loss_acc;
}

}  // namespace spp
