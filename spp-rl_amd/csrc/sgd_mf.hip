// AcM regression SGD on the fp32 matrix cores: sppAcmSgd's sequential minibatch steps (acm/acm.py:246-258,
// 266-303) with every layer of the 64-32 AcM MLP as v_mfma_f32_32x32x2_f32 tiles.
//
// One step, one workgroup of 4 waves per kMfR = 64 rows of the step's batch (several workgroups per step
// above 64 rows: per-step gradients summed over them in a fixed order through write-through slabs, as
// k_acm_sgd).  Wave w = (sample block sb = w & 1, unit block hb = w >> 1).  MFMA operands come from LDS
// images laid out so every read is bank-conflict free (odd row strides, or lanes on consecutive columns):
//   X   [64 samples][SX]       the step's inputs (zero padding columns / rows)
//   H1L [64 units][65]         tanh(fc1), written in the D layout ([unit][sample]), read as B (fc2) and B (dW2)
//   H2L [32 units][65], D3L [8][65], D2L [32][65], D1L [64][65]   likewise for h2 and the deltas
//   W1 [64][SW1], W2 [32][65], W3 [8][33]   the parameters (row = output unit), b1 / b2 / b3
// Forward: fc1 by all 4 waves (their (hb, sb) block), fc2 / fc3 / dz3 / dz2 by waves sb = 0, 1 (hb = 0),
// dz1 by all 4.  Weight gradients: 2 * NIB1 tiles of dW1 (unit block x input block), 2 of dW2, 1 of dW3
// (rows < AC), each over the 64 samples (32 k-steps), dealt to the 4 waves; b1's gradient is dW1's column
// IN (X carries a constant-1 input there), b2 / b3's are row sums of dz2 / dz3 by wave 3.  The wave that
// computes a gradient tile owns its Adam state (16 moments per lane per tile, in registers) and writes the
// updated weights back into the LDS image.
#pragma once
// (included by api.hip after sgd.hip: AcmSgdArgs, the slab helpers, the arrival barrier)

namespace spp {

constexpr int kMfR = 64;    // rows per workgroup and step
constexpr int kMfTH = 256;  // 4 waves
constexpr int kMfS = 65;    // row stride of the [unit][sample] images
constexpr int kMfSlab = 8192;   // floats per workgroup slab (>= MfCfg::NSLAB)
constexpr int kMfMaxWG = 512;   // batches up to 32,768 rows

template <int IN, int AC>
struct MfCfg {
  static constexpr int NKS1 = (IN + 1) / 2;           // fc1 k-steps (pairs of inputs)
  static constexpr int NIB1 = (IN + 1 + 31) / 32;     // dW1 input blocks (input IN: the constant 1, b1's gradient)
  static constexpr int SX = (2 * NKS1 > 32 ? 2 * NKS1 : 32) + 1;  // odd, >= 33: dW1 reads inputs 0..32 NIB1-1
  static constexpr int SX2 = 32 * NIB1 + 1 > SX ? 32 * NIB1 + 1 : SX;
  static constexpr int SW1 = (2 * NKS1) | 1;
  static constexpr int NTILE = 2 * NIB1 + 3;          // dW1 | dW2 (2) | dW3
  static constexpr int TPW = (NTILE + 3) / 4;         // tiles per wave (at most)
  static constexpr int NB = 32 + AC;                  // thread-owned bias parameters (b2 | b3); b1 rides on dW1
  static constexpr int NSLAB = 1024 * NTILE + NB + 1; // floats per workgroup slab (+ loss)
  static_assert(AC <= 8, "AcM output <= 8");
  static_assert(NSLAB <= kMfSlab, "gradient slab");
};

__device__ __forceinline__ constexpr int mf_ru(int r) { return (r & 3) + 8 * (r >> 2); }
__device__ __forceinline__ f32x16 mf_mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
// tile t of the step's gradient -> (layer, first row, first column); rows of dW3 past AC are padding
template <class C>
__device__ __forceinline__ void mf_tile(int t, int& layer, int& r0, int& c0) {
  if (t < 2 * C::NIB1) {
    layer = 0; r0 = 32 * (t & 1); c0 = 32 * (t >> 1);
  } else if (t < 2 * C::NIB1 + 2) {
    layer = 1; r0 = 0; c0 = 32 * (t - 2 * C::NIB1);
  } else {
    layer = 2; r0 = 0; c0 = 0;
  }
}

template <int IN, int AC, bool MW>
__global__ __launch_bounds__(kMfTH, 1) void k_acm_sgd_mf(AcmSgdArgs a) {
  using C = MfCfg<IN, AC>;
  constexpr int SX = C::SX2, SW1 = C::SW1, S = kMfS, R = kMfR;
  __shared__ float X[R * SX];
  __shared__ float H1L[64 * S], D1L[64 * S], H2L[32 * S], D2L[32 * S], D3L[8 * S];
  __shared__ float W1[64 * SW1], W2[32 * S], W3[8 * 33];
  __shared__ float B1[64], B2[32], B3[8];
  __shared__ float Y[R * AC];
  __shared__ float LP[2];               // per sample block: loss partials
  __shared__ float adam_s[2][2];
  __shared__ int s_dead;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63, h = lane >> 5, l32 = lane & 31;
  const int sb = w & 1, hb = w >> 1;
  const bool bown = w == 3 && lane < MfCfg<IN, AC>::NB;  // owner of bias parameter `lane` of [b2 | b3]
  const int bsg = a.bs;
  const int r0 = MW ? (int)blockIdx.x * a.bsl : 0;
  const int bs = MW ? min(a.bsl, bsg - r0) : bsg;  // this workgroup's rows (<= 64)
  const float inv_n = 1.f / (float)(bsg * AC);
  if (t == 0) s_dead = 0;
  double pw1 = 0.0, pw2 = 0.0;  // beta1^t, beta2^t of the next step (thread kMfTH - 1; pow once, then products)
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
  // ---- parameters -> LDS images (zero padding), Adam moments of the owned elements -> registers
  for (int i = t; i < 64 * SW1; i += kMfTH) {
    const int u = i / SW1, c = i % SW1;
    W1[i] = c < IN ? a.params[u * IN + c] : 0.f;
  }
  for (int i = t; i < 32 * S; i += kMfTH) {
    const int u = i / S, c = i % S;
    W2[i] = c < 64 ? a.params[64 * IN + 64 + u * 64 + c] : 0.f;
  }
  for (int i = t; i < 8 * 33; i += kMfTH) {
    const int u = i / 33, c = i % 33;
    W3[i] = (u < AC && c < 32) ? a.params[64 * IN + 64 + 32 * 64 + 32 + u * 32 + c] : 0.f;
  }
  if (t < 64) B1[t] = a.params[64 * IN + t];
  if (t < 32) B2[t] = a.params[64 * IN + 64 + 32 * 64 + t];
  if (t < 8) B3[t] = t < AC ? a.params[64 * IN + 64 + 32 * 64 + 32 + AC * 32 + t] : 0.f;
  for (int i = t; i < 8 * S; i += kMfTH) D3L[i] = 0.f;  // rows >= AC stay zero
  // canonical flat index of tile element (tile q, register e) of this lane, or -1
  auto canon = [&](int q, int e) -> int {
    int layer, rr, cc;
    mf_tile<C>(q, layer, rr, cc);
    const int row = rr + mf_ru(e) + 4 * h, col = cc + l32;
    if (layer == 0) return col < IN ? row * IN + col : (col == IN ? 64 * IN + row : -1);
    if (layer == 1) return 64 * IN + 64 + row * 64 + col;
    return row < AC ? 64 * IN + 64 + 32 * 64 + 32 + row * 32 + col : -1;
  };
  auto bcanon = [&](int j) -> int {  // bias parameter j of [b2 | b3]
    if (j < 32) return 64 * IN + 64 + 32 * 64 + j;
    return 64 * IN + 64 + 32 * 64 + 32 + AC * 32 + (j - 32);
  };
  float mom[C::TPW][16], vel[C::TPW][16];
#pragma unroll
  for (int k = 0; k < C::TPW; ++k) {
    const int q = w + 4 * k;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int c = q < C::NTILE ? canon(q, e) : -1;
      mom[k][e] = c >= 0 ? a.m[c] : 0.f;
      vel[k][e] = c >= 0 ? a.v[c] : 0.f;
    }
  }
  float bm = 0.f, bv = 0.f;
  if (bown) {
    bm = a.m[bcanon(lane)];
    bv = a.v[bcanon(lane)];
  }
  // register prefetch of one step's rows
  constexpr int NXP = (R * IN + kMfTH - 1) / kMfTH, NYP = (R * AC + kMfTH - 1) / kMfTH;
  float xp[NXP], yp[NYP];
  auto prefetch = [&](int st) {
    const float* xs = a.x + ((int64_t)st * bsg + r0) * IN;
    const float* ys = a.y + ((int64_t)st * bsg + r0) * AC;
#pragma unroll
    for (int k = 0; k < NXP; ++k) {
      const int i = t + kMfTH * k;
      xp[k] = (st < a.nsteps && i < bs * IN) ? xs[i] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < NYP; ++k) {
      const int i = t + kMfTH * k;
      yp[k] = (st < a.nsteps && i < bs * AC) ? ys[i] : 0.f;
    }
  };
  // zero X once: padding columns and rows past bs stay zero (rows past bs are rewritten with zeros)
  for (int i = t; i < R * SX; i += kMfTH) X[i] = 0.f;
  float loss_acc = 0.f;
  prefetch(0);
  if (t == kMfTH - 1) adam_scalars(0);
  __syncthreads();
  SPP_TP_INIT();
  for (int st = 0; st < a.nsteps; ++st) {
    // ---- the step's rows into LDS (rows >= bs: xp / yp are zero)
#pragma unroll
    for (int k = 0; k < NXP; ++k) {
      const int i = t + kMfTH * k;
      if (i < R * IN) X[(i / IN) * SX + (i % IN)] = xp[k];
    }
    if (t < R) X[t * SX + IN] = t < bs ? 1.f : 0.f;  // the bias input (dW1 column IN = b1's gradient)
#pragma unroll
    for (int k = 0; k < NYP; ++k) {
      const int i = t + kMfTH * k;
      if (i < R * AC) Y[i] = yp[k];
    }
    prefetch(st + 1);
    __syncthreads();
    SPP_TP(0);
    // ---- fc1: block (hb, sb) of h1 = tanh(W1 x + b1)
    f32x16 h1r;
    {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = B1[32 * hb + mf_ru(r) + 4 * h];
      const float* pa = W1 + (32 * hb + l32) * SW1 + h;
      const float* pb = X + (32 * sb + l32) * SX + h;
#pragma unroll
      for (int ks = 0; ks < C::NKS1; ++ks) acc = mf_mfma(pa[2 * ks], pb[2 * ks], acc);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        h1r[r] = tanhf(acc[r]);
        H1L[(32 * hb + mf_ru(r) + 4 * h) * S + 32 * sb + l32] = h1r[r];
      }
    }
    __syncthreads();
    SPP_TP(1);
    float lpart = 0.f;
    if (hb == 0) {
      // ---- fc2: h2 = tanh(W2 h1 + b2) for sample block sb
      f32x16 h2r;
      {
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = B2[mf_ru(r) + 4 * h];
        const float* pa = W2 + l32 * S + h;
        const float* pb = H1L + h * S + 32 * sb + l32;
#pragma unroll 8
        for (int ks = 0; ks < 32; ++ks) acc = mf_mfma(pa[2 * ks], pb[2 * ks * S], acc);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          h2r[r] = tanhf(acc[r]);
          H2L[(mf_ru(r) + 4 * h) * S + 32 * sb + l32] = h2r[r];
        }
      }
      // ---- fc3, loss, dz3 = d loss / d z3 (rows < AC: registers 0..3 of the two lane halves)
      {
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = r < 4 ? B3[mf_ru(r) + 4 * h] : 0.f;
        const float* pa = W3 + (l32 < 8 ? l32 : 0) * 33 + h;
        const float* pb = H2L + h * S + 32 * sb + l32;
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) acc = mf_mfma(l32 < AC ? pa[2 * ks] : 0.f, pb[2 * ks * S], acc);
        const int sm = 32 * sb + l32;
        const bool valid = sm < bs;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int u = r + 4 * h;
          float d = 0.f;
          if (u < AC) {
            const float th = tanhf(acc[r]), lim = a.lim[u];
            const float e = th * lim - Y[sm * AC + u];
            if (valid) {
              lpart = fmaf(e, e, lpart);
              d = 2.f * e * inv_n * lim * (1.f - th * th);
            }
            D3L[u * S + sm] = d;
          }
        }
      }
      // ---- dz2 = (W3^T dz3) * (1 - h2^2)
      {
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
        const float* pa = W3 + h * 33 + l32;
        const float* pb = D3L + h * S + 32 * sb + l32;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) acc = mf_mfma(pa[2 * ks * 33], pb[2 * ks * S], acc);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d = acc[r] * (1.f - h2r[r] * h2r[r]);
          D2L[(mf_ru(r) + 4 * h) * S + 32 * sb + l32] = d;
        }
      }
      lpart = wave_sum(lpart);
      if (lane == 0) LP[sb] = lpart;
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
      for (int ks = 0; ks < 16; ++ks) acc = mf_mfma(pa[2 * ks * S], pb[2 * ks * S], acc);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float d = acc[r] * (1.f - h1r[r] * h1r[r]);
        D1L[(32 * hb + mf_ru(r) + 4 * h) * S + 32 * sb + l32] = d;
      }
    }
    __syncthreads();
    SPP_TP(3);
    // ---- weight-gradient tiles over the 64 samples: tile q = w + 4k
    f32x16 g[C::TPW];
#pragma unroll
    for (int k = 0; k < C::TPW; ++k) {
      const int q = w + 4 * k;
#pragma unroll
      for (int r = 0; r < 16; ++r) g[k][r] = 0.f;
      if (q < C::NTILE) {
        int layer, rr, cc;
        mf_tile<C>(q, layer, rr, cc);
        const float* pa;
        const float* pb;
        int sbs;  // B stride between consecutive samples
        if (layer == 0) {
          pa = D1L + (rr + l32) * S + h;
          pb = X + h * SX + cc + l32;
          sbs = SX;
        } else if (layer == 1) {
          pa = D2L + l32 * S + h;
          pb = H1L + (cc + l32) * S + h;
          sbs = 1;
        } else {
          pa = D3L + (l32 < 8 ? l32 : 0) * S + h;
          pb = H2L + l32 * S + h;
          sbs = 1;
        }
        const bool arow = layer != 2 || l32 < 8;
        if (layer == 0) {
#pragma unroll 8
          for (int ks = 0; ks < 32; ++ks) g[k] = mf_mfma(pa[2 * ks], pb[2 * ks * sbs], g[k]);
        } else {
#pragma unroll 8
          for (int ks = 0; ks < 32; ++ks) g[k] = mf_mfma(arow ? pa[2 * ks] : 0.f, pb[2 * ks], g[k]);
        }
      }
    }
    // b2 / b3 gradients: row sums of dz2 / dz3 over the 64 samples (wave 3: it has the fewest tiles)
    float bg = 0.f;  // bias owners: the gradient of their parameter
    if (bown) {
      const float* row = lane < 32 ? D2L + lane * S : D3L + (lane - 32) * S;
#pragma unroll 16
      for (int s2 = 0; s2 < R; ++s2) bg += row[s2];
    }
    __syncthreads();  // LP complete; bias sums done
    SPP_TP(4);
    float ls_part = LP[0] + LP[1];
    if constexpr (MW) {
      const int G = gridDim.x;
      const auto mine = sgd_rsrc(a.slab + ((int64_t)(st & 1) * G + blockIdx.x) * kMfSlab);
#pragma unroll
      for (int k = 0; k < C::TPW; ++k) {
        const int q = w + 4 * k;
        if (q < C::NTILE)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            slab_st4(mine, 1024 * q + 16 * lane + 4 * i,
                     make_float4(g[k][4 * i], g[k][4 * i + 1], g[k][4 * i + 2], g[k][4 * i + 3]));
      }
      if (bown) slab_st1(mine, 1024 * C::NTILE + lane, bg);
      if (t == 0) slab_st1(mine, C::NSLAB - 1, ls_part);
      const int nsync = G > kSgdTwoLevel ? 2 : 1;
      sgd_arrive_wait_wt(a.ctr, G * nsync * st + G, a.err, &s_dead);
      const auto all = sgd_rsrc(a.slab + (int64_t)(st & 1) * G * kMfSlab);
      if (G > kSgdTwoLevel) {
        const auto red = sgd_rsrc(a.slab + (int64_t)2 * G * kMfSlab + (int64_t)(st & 1) * kMfSlab);
        // workgroup g sums quads [g * chunk, (g + 1) * chunk) of the slab over the G slabs (16-B sc1 loads)
        constexpr int NQ4 = (C::NSLAB + 3) / 4;
        const int chunk = (NQ4 + G - 1) / G;
        const int e1 = min((int)(blockIdx.x + 1) * chunk, NQ4);
        for (int e = (int)blockIdx.x * chunk + t; e < e1; e += kMfTH) {
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          for (int gg = 0; gg < G; ++gg) {
            const float4 x = slab_ld4(all, gg * kMfSlab + 4 * e);
            v.x += x.x; v.y += x.y; v.z += x.z; v.w += x.w;
          }
          slab_st4(red, 4 * e, v);
        }
        sgd_arrive_wait_wt(a.ctr, G * nsync * st + 2 * G, a.err, &s_dead);
#pragma unroll
        for (int k = 0; k < C::TPW; ++k) {
          const int q = w + 4 * k;
          if (q < C::NTILE)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float4 v = slab_ld4(red, 1024 * q + 16 * lane + 4 * i);
              g[k][4 * i] = v.x; g[k][4 * i + 1] = v.y; g[k][4 * i + 2] = v.z; g[k][4 * i + 3] = v.w;
            }
        }
        if (bown) bg = slab_ld1(red, 1024 * C::NTILE + lane);
        ls_part = slab_ld1(red, C::NSLAB - 1);
      } else {
#pragma unroll
        for (int k = 0; k < C::TPW; ++k) {
          const int q = w + 4 * k;
          if (q < C::NTILE) {
            float4 acc[4] = {};
            for (int gg = 0; gg < G; ++gg)
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const float4 v = slab_ld4(all, gg * kMfSlab + 1024 * q + 16 * lane + 4 * i);
                acc[i].x += v.x; acc[i].y += v.y; acc[i].z += v.z; acc[i].w += v.w;
              }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              g[k][4 * i] = acc[i].x; g[k][4 * i + 1] = acc[i].y; g[k][4 * i + 2] = acc[i].z; g[k][4 * i + 3] = acc[i].w;
            }
          }
        }
        if (bown) {
          float v = 0.f;
          for (int gg = 0; gg < G; ++gg) v += slab_ld1(all, gg * kMfSlab + 1024 * C::NTILE + lane);
          bg = v;
        }
        if (t == 0) {
          float v = 0.f;
          for (int gg = 0; gg < G; ++gg) v += slab_ld1(all, gg * kMfSlab + C::NSLAB - 1);
          ls_part = v;
        }
      }
    }
    if (t == 0) loss_acc += ls_part * inv_n;
    SPP_TP(5);
    // ---- Adam (torch.optim.Adam, k_adam's operation order) on the owned elements; new weights -> LDS
    const float omb1 = 0.1f, b2c = 0.999f, omb2 = 0.001f, eps = 1e-8f;
    const float neg_step = adam_s[st & 1][0], bc2s = adam_s[st & 1][1];
    __syncthreads();  // every wave is done reading the weights of this step (dz1 read W2)
    if (t == kMfTH - 1) adam_scalars(st + 1);
    auto adam = [&](float gg, float& m, float& v, float& p) {
      m = fadd_rn(m, fmul_rn(omb1, fsub_rn(gg, m)));
      v = fadd_rn(fmul_rn(v, b2c), fmul_rn(fmul_rn(omb2, gg), gg));
      const float denom = fadd_rn(fdiv_rn(sqrtf(v), bc2s), eps);
      p = fadd_rn(p, fmul_rn(neg_step, fdiv_rn(m, denom)));
    };
#pragma unroll
    for (int k = 0; k < C::TPW; ++k) {
      const int q = w + 4 * k;
      if (q < C::NTILE) {
        int layer, rr, cc;
        mf_tile<C>(q, layer, rr, cc);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = rr + mf_ru(e) + 4 * h, col = cc + l32;
          float* p = layer == 0 ? (col < IN ? W1 + row * SW1 + col : (col == IN ? B1 + row : nullptr))
                                : (layer == 1 ? W2 + row * S + col : (row < AC ? W3 + row * 33 + col : nullptr));
          if (p) adam(g[k][e], mom[k][e], vel[k][e], *p);
        }
      }
    }
    if (bown) adam(bg, bm, bv, lane < 32 ? B2[lane] : B3[lane - 32]);
    __syncthreads();
    SPP_TP(6);
  }
  SPP_TP_FLUSH();
  if (MW && blockIdx.x != 0) return;  // every workgroup holds the same parameters and moments
  // ---- write back parameters and moments (canonical layout)
#pragma unroll
  for (int k = 0; k < C::TPW; ++k) {
    const int q = w + 4 * k;
    if (q < C::NTILE) {
      int layer, rr, cc;
      mf_tile<C>(q, layer, rr, cc);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int c = canon(q, e);
        if (c >= 0) {
          const int row = rr + mf_ru(e) + 4 * h, col = cc + l32;
          a.params[c] = layer == 0 ? (col < IN ? W1[row * SW1 + col] : B1[row])
                                   : (layer == 1 ? W2[row * S + col] : W3[row * 33 + col]);
          a.m[c] = mom[k][e];
          a.v[c] = vel[k][e];
        }
      }
    }
  }
  if (bown) {
    const int c = bcanon(lane);
    a.params[c] = lane < 32 ? B2[lane] : B3[lane - 32];
    a.m[c] = bm;
    a.v[c] = bv;
  }
  if (t == 0) *a.loss_sum += loss_acc;
}

}  // namespace spp
