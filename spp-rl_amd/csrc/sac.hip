// SAC_AcM per-sample kernels (gfx950).  One wave = 32 samples; one workgroup
// = 4 waves (one per SIMD), each with a private 32 KiB LDS image [256][32]
// (rows 192..255 double as the SMALL image of the 64-wide ACM layers), plus a
// 16 KiB per-workgroup table of bias / fc3 vectors shared by the 4 waves.
//
//  k_sac_critic_phase   rltoolkit/acm/off_policy/sac_acm.py:30-58 (targets) and
//                       :114-131 (both critics' forward + backward) -> per-sample
//                       operands of the critic weight gradients
//  k_sac_actor_phase    sac_acm.py:60-87 + :137-145 (actor loss through the
//                       frozen ACM and both updated critics) -> actor grad operands
//  k_policy_act         ddpg_acm.py:40-50, off_policy.py:50-54, :89-106 (rollout)
//  k_acm_regress        acm.py:246-258 (ACM regression forward + backward)
#pragma once
#include "sac_kernels.h"

namespace spp {

constexpr float kLog2 = 0.69314718055994530942f;
constexpr float kLogSqrt2Pi = 0.91893853320467274178f;  // math.log(math.sqrt(2*pi))

template <int OB_, int AOUT_, int AC_, bool ACMC_, bool BF_ = false>
struct Cfg {
  static constexpr int OB = OB_, AOUT = AOUT_, AC = AC_;
  static constexpr bool ACMC = ACMC_;
  static constexpr bool BF = BF_;  // bf16 MFMA MLP layers (fp32 accumulation, epilogues and targets)
  // the critics' fc3 weight gradient fused into k_sac_critic_phase (else h2 / dq go to HBM for a k_dw job);
  // bf16 sets: SPP_BF16_FUSE3 (api.hip's build_dw makes the same choice through sac_fuse3())
  static constexpr bool F3 = !BF_ || SPP_BF16_FUSE3;
  static constexpr int NB_OB = blocks_of(OB);
  static constexpr int NB_AOUT = blocks_of(AOUT);
  static constexpr int NB_H2 = blocks_of(2 * AOUT);      // heads output blocks (natural rows mu | logsig)
  static constexpr int NB_PAIR = (AOUT + 15) / 16;        // heads in pairing layout
  static constexpr int CA = ACMC ? AC : AOUT;             // critic action-input width
  static constexpr int NB_CA = blocks_of(CA);
  static constexpr int NB_CIN = NB_OB + NB_CA;
  static constexpr int NB_ACMIN = NB_OB + NB_AOUT;
  static constexpr uint64_t RV_X = rv_nat(OB, NB_OB);
  static constexpr uint64_t RV_H = rv_nat(256, 8);
  static constexpr uint64_t RV_CIN = rv_cat(OB, NB_OB, CA, NB_CA);
  static constexpr uint64_t RV_ACMIN = rv_cat(OB, NB_OB, AOUT, NB_AOUT);
  static constexpr uint64_t RV_Z1 = rv_nat(64, 2);
  static constexpr uint64_t RV_Z2 = rv_nat(32, 1);
  static constexpr uint64_t RV_AC = rv_nat(AC, 1);
  static constexpr uint64_t RV_CA = rv_nat(CA, NB_CA);
  static constexpr uint64_t RV_PAIR = rv_pair(AOUT, NB_PAIR);
  static_assert(AC <= 32, "env action dim <= 32");
  static_assert(2 * AOUT <= 256 && OB + AOUT <= 256, "dims");
};

constexpr int kWavesPerWG = 4;

constexpr int kLdsPerWave = 256 * 32;  // BIG [256][32] floats
constexpr int kSmallRow = 192;         // SMALL [64][32] = BIG rows 192..255

// Fill the per-workgroup LDS constant table (all threads), then barrier.
__device__ __forceinline__ void load_table(const SacArgs& p, float* tbl) {
  for (int s = 0; s < p.nseg; ++s) {
    const TabSeg g = p.seg[s];
    for (int i = threadIdx.x; i < g.npad; i += blockDim.x) tbl[g.off + i] = i < g.n ? g.src[i] : 0.f;
  }
  __syncthreads();
}
// Natural-order table vector at (block ob, register q) of this lane half.
__device__ __forceinline__ float tval(const float* t, int ob, int q, int h4) { return t[32 * ob + ru(q) + h4]; }
// All 16 table values of output block ob for this lane half (v[q] = tval(t, ob, q, h4)) as 4
// broadcast ds_read_b128, read before any use: an LDS read inside a select is turned into a
// branch with its own wait, i.e. one LDS round trip per element.
__device__ __forceinline__ void tvals(const float* t, int ob, int h4, float (&v)[16]) {
  const float4* p = reinterpret_cast<const float4*>(t + 32 * ob + h4);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float4 x = p[2 * k];
    v[4 * k + 0] = x.x;
    v[4 * k + 1] = x.y;
    v[4 * k + 2] = x.z;
    v[4 * k + 3] = x.w;
  }
}

__device__ __forceinline__ void setbits(uint64_t& lo, uint64_t& hi, int ob, uint32_t bits) {
  if (ob < 4) lo |= (uint64_t)bits << (16 * ob);
  else hi |= (uint64_t)bits << (16 * (ob - 4));
  asm volatile("" : "+v"(lo), "+v"(hi));  // materialise now: no sinking of 16 live floats per block
}
__device__ __forceinline__ bool getbit(uint64_t lo, uint64_t hi, int ob, int q) {
  const uint64_t w = ob < 4 ? (lo >> (16 * ob)) : (hi >> (16 * (ob - 4)));
  return (w >> q) & 1;
}

// memory.py:107-121 (denormalize) and :76-87 / utils.py:62-73 (normalize, force=True)
// TB: read the kernel's LDS table T (make_args puts the limits at t_lim / t_alim and the
// normaliser vectors at t_n0 / t_n1) instead of the global arrays (per-slot global loads are one
// round trip each).  Every kernel set reads the table (TB = true); the global form stays for
// reference.
template <bool TB>
__device__ __forceinline__ float nv0(const SacArgs& p, const float* T, int j) {
  if constexpr (TB) return T[p.t_n0 + j];
  else return p.min_max ? p.lo[j] : p.mean[j];
}
template <bool TB>
__device__ __forceinline__ float nv1(const SacArgs& p, const float* T, int j) {
  if constexpr (TB) return T[p.t_n1 + j];
  else return p.min_max ? p.hi[j] : p.std[j];
}
template <bool TB>
__device__ __forceinline__ float denorm(const SacArgs& p, const float* T, int j, float x) {
  const float n0 = nv0<TB>(p, T, j), n1 = nv1<TB>(p, T, j);
  if (p.min_max) {  // n0 = lo, n1 = hi
    const float mid = fadd_rn(n1, n0) * 0.5f, delta = fsub_rn(n1, n0) * 0.5f;
    return fadd_rn(mid, fmul_rn(x, delta));
  }
  return fadd_rn(fmul_rn(fadd_rn(n1, 1e-8f), x), n0);  // n0 = mean, n1 = std
}
template <bool TB>
__device__ __forceinline__ float denorm_scale(const SacArgs& p, const float* T, int j) {
  const float n0 = nv0<TB>(p, T, j), n1 = nv1<TB>(p, T, j);
  if (p.min_max) return fsub_rn(n1, n0) * 0.5f;
  return fadd_rn(n1, 1e-8f);
}
template <bool TB>
__device__ __forceinline__ float normalize(const SacArgs& p, const float* T, int j, float x) {
  const float n0 = nv0<TB>(p, T, j), n1 = nv1<TB>(p, T, j);
  if (p.min_max) {
    const float mid = fadd_rn(n1, n0) * 0.5f;
    return fdiv_rn(fsub_rn(x, mid), fadd_rn(fsub_rn(n1, mid), 1e-8f));
  }
  return fminf(fmaxf(fdiv_rn(fsub_rn(x, n0), fadd_rn(n1, 1e-8f)), -10.f), 10.f);
}
template <bool TB>
__device__ __forceinline__ float actor_lim(const SacArgs& p, const float* T, int j) {
  if constexpr (TB) return T[p.t_lim + j];
  else return p.actor_lim[j];
}
template <bool TB>
__device__ __forceinline__ float acm_lim(const SacArgs& p, const float* T, int u) {
  if constexpr (TB) return T[p.t_alim + u];
  else return p.acm_lim[u];
}
__device__ __forceinline__ float softplus_t(float x) {  // torch softplus(beta=1, threshold=20)
  return x > 20.f ? x : log1pf(expf(x));
}

// Transcendentals of the squash / log-prob epilogues.  F (the bf16 kernel sets, BASELINE configs[4]:
// bf16 MLP): the hardware forms (v_exp_f32 / v_log_f32 / v_rcp_f32, ~1 ulp), far inside the bf16
// tolerance; these epilogues are VALU-latency bound on the 111-wide Ant heads.  fp32 sets: libm.
template <bool F>
__device__ __forceinline__ float t_exp(float x) {
  if constexpr (F) return __expf(x);
  else return expf(x);
}
template <bool F>
__device__ __forceinline__ float t_rcp(float x) {
  if constexpr (F) return __builtin_amdgcn_rcpf(x);
  else return 1.f / x;
}
template <bool F>
__device__ __forceinline__ float t_tanh(float x) {
  if constexpr (F) return 1.f - 2.f * __builtin_amdgcn_rcpf(__expf(2.f * x) + 1.f);
  else return tanhf(x);
}
template <bool F>
__device__ __forceinline__ float t_softplus(float x) {
  if constexpr (F) return x > 20.f ? x : __logf(1.f + __expf(x));
  else return softplus_t(x);
}

// Pairing-layout tile of the actor heads from the LDS image rows [0, 2*AOUT)
// pairing layout: block ib, register r<8 (mu) / r+8 (logsig), half h -> j = 16*ib + 8*h + r
template <class C>
__device__ __forceinline__ void load_pair(f32x16 (&t)[C::NB_PAIR], const float* lds) {
  SPP_XLANE_SYNC();
  const int lane = lane_id(), h8 = 8 * (lane >> 5);
  const float* pl = lds + h8 * 32 + (lane & 31);
#pragma unroll
  for (int ib = 0; ib < C::NB_PAIR; ++ib)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int j0 = 16 * ib + (r & 7);
      t[ib][r] = (j0 + h8 < C::AOUT) ? pl[((r < 8) ? j0 : C::AOUT + j0) * 32] : 0.f;
    }
}

// Concatenated input tile: blocks [0, NB0) natural from global X (F0 units),
// blocks [NB0, NB0+NB1) natural from the LDS image rows [0, F1).
template <int NB0, int NB1>
__device__ __forceinline__ void load_cat_gl(f32x16 (&t)[NB0 + NB1], const float* X, int nbytes, int F0, int ld4,
                                            uint32_t vo, const float* lds, int F1) {
  SPP_XLANE_SYNC();
  const int lane = lane_id(), h4 = 4 * (lane >> 5);
  const float* l = lds + h4 * 32 + (lane & 31);
  f32x16 g[NB0];
  gm_load<NB0>(g, X, nbytes, F0, ld4, vo);
#pragma unroll
  for (int ib = 0; ib < NB0; ++ib) t[ib] = g[ib];
#pragma unroll
  for (int ib = 0; ib < NB1; ++ib)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int u0 = 32 * ib + ru(r);
      t[NB0 + ib][r] = (u0 + h4 < F1) ? l[u0 * 32] : 0.f;
    }
}
// Concatenated input tile from two global feature-major arrays.
template <int NB0, int NB1>
__device__ __forceinline__ void load_cat_gg(f32x16 (&t)[NB0 + NB1], const float* X0, int F0, const float* X1, int F1,
                                            int ld4, uint32_t vo) {
  f32x16 g0[NB0], g1[NB1];
  gm_load<NB0>(g0, X0, F0 * ld4, F0, ld4, vo);
  gm_load<NB1>(g1, X1, F1 * ld4, F1, ld4, vo);
#pragma unroll
  for (int ib = 0; ib < NB0; ++ib) t[ib] = g0[ib];
#pragma unroll
  for (int ib = 0; ib < NB1; ++ib) t[NB0 + ib] = g1[ib];
}

// Per-tile lane context: LDS images, sample column offsets.
// Global 2-D arrays X[row][ld] are addressed through buffer resources:
// byte offset row*ld4 (wave-uniform soffset) + vo (this lane's column, voffset).
struct Lane {
  int h, s, h4;
  float* img;             // BIG image base of this wave
  const float* tbl;       // per-workgroup LDS table
  int b, ld4;             // sample index, row stride in bytes
  uint32_t vo, vp;        // 4*(4h*ld + b) (natural layout), 4*(8h*ld + b) (pairing layout)
  float *bl, *sl;         // BIG / SMALL image at this lane: image[urow*32] = unit (urow + 4h), sample s
  float* pl;              // BIG at the pairing offset: pl[j0*32] = row j0 + 8h
};
__device__ __forceinline__ Lane make_lane(float* big, float* small, const float* tbl, int ld, int b) {
  Lane L;
  L.img = big;
  L.tbl = tbl;
  int lane = lane_id();
  asm volatile("" : "+v"(lane));  // keep lane-derived values inside the tile loop (no LICM + spill)
  int ld4 = 4 * ld;
  asm volatile("" : "+s"(ld4));   // likewise the row strides (no hoisted per-row offsets)
  L.h = lane >> 5;
  L.s = lane & 31;
  L.h4 = 4 * L.h;
  L.ld4 = ld4;
  L.b = b;
  L.vo = (uint32_t)(L.h4 * ld4 + 4 * b);
  L.vp = (uint32_t)(8 * L.h * ld4 + 4 * b);
  L.bl = big + L.h4 * 32 + L.s;
  L.sl = small + L.h4 * 32 + L.s;
  L.pl = big + 8 * L.h * 32 + L.s;
  return L;
}

// Actor trunk: x -> relu(L1) -> relu(L2) -> heads into LDS rows [0, NHR): SAC
// (mu | logsig), NHR = 2*AOUT; DDPG fc3 pre-activation, NHR = AOUT (NBH blocks).
// ST: store h1 / h2 feature-major (H1g, H2g).  Returns the ReLU masks.
template <class C, bool ST, int NBH = C::NB_H2, int NHR = 2 * C::AOUT>
__device__ __forceinline__ void actor_trunk(const ActorDev& A, const float* X, int xbytes, const Lane& L, float* H1g,
                                            float* H2g,
                                            uint64_t& m1lo, uint64_t& m1hi, uint64_t& m2lo, uint64_t& m2hi) {
  {
    f32x16 x[C::NB_OB];
    gm_load<C::NB_OB>(x, X, xbytes, C::OB, L.ld4, L.vo);
    const rsrc_t hr = rsrc(H1g);
    dense<C::NB_OB, C::RV_X, C::BF>(A.W1, 8, x, L.tbl + A.tb1, [&](int ob, const f32x16& acc) {
      uint32_t bits = 0;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ur = 32 * ob + ru(q);
        const float v = fmaxf(acc[q], 0.f);
        L.bl[ur * 32] = v;
        if constexpr (ST) op_st<C::BF>(hr, ur, L.ld4, L.vo, v);
        bits |= (uint32_t)(v > 0.f) << q;
      }
      setbits(m1lo, m1hi, ob, bits);
    });
  }
  SPP_TP(1);
  {
    const rsrc_t hr = rsrc(H2g);
    dense_lds<8, C::BF>(A.W2, L.img, L.tbl + A.tb2, [&](int ob, const f32x16& acc) {
      uint32_t bits = 0;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ur = 32 * ob + ru(q);
        const float v = fmaxf(acc[q], 0.f);
        L.bl[ur * 32] = v;
        if constexpr (ST) op_st<C::BF>(hr, ur, L.ld4, L.vo, v);
        bits |= (uint32_t)(v > 0.f) << q;
      }
      setbits(m2lo, m2hi, ob, bits);
    });
  }
  SPP_TP(2);
  {
    dense_lds<NBH, C::BF>(A.Wh, L.img, L.tbl + A.tbh, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ur = 32 * ob + ru(q);
        if (ur + L.h4 < NHR) L.bl[ur * 32] = acc[q];
      }
    });
  }
  SPP_TP(3);
}

// ACM forward (basic_model.py:118-126): in [s | a_d] -> tanh 64 -> tanh 32 -> tanh(ac)*lim.
// ST: store z1 / z2 / t3 feature-major; output c into SMALL rows [0, AC).
template <class C, bool ST>
__device__ __forceinline__ void acm_forward(const SacArgs& p, const f32x16 (&xin)[C::NB_ACMIN], const Lane& L,
                                            float* Z1g, float* Z2g, float* T3g) {
  float* small = L.sl - L.h4 * 32 - L.s;
  const rsrc_t z1r = rsrc(Z1g), z2r = rsrc(Z2g), t3r = rsrc(T3g);
  dense<C::NB_ACMIN, C::RV_ACMIN, C::BF>(p.acm.W1, 2, xin, L.tbl + p.acm.tb1, [&](int ob, const f32x16& acc) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ur = 32 * ob + ru(q);
      const float v = tanhf(acc[q]);
      L.sl[ur * 32] = v;
      if constexpr (ST) fm_st(z1r, ur, L.ld4, L.vo, v);
    }
  });
  f32x16 z1[2];
  lds_load<2>(z1, small);
  dense<2, C::RV_Z1, C::BF>(p.acm.W2, 1, z1, L.tbl + p.acm.tb2, [&](int ob, const f32x16& acc) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float v = tanhf(acc[q]);
      L.sl[ru(q) * 32] = v;
      if constexpr (ST) fm_st(z2r, ru(q), L.ld4, L.vo, v);
    }
  });
  f32x16 z2[1];
  lds_load<1>(z2, small);
  float limv[16];  // before the layer: a load behind the epilogue's buffer stores waits per element
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int u = ru(q) + L.h4;
    limv[q] = acm_lim<true>(p, L.tbl, u < C::AC ? u : 0);
  }
  dense<1, C::RV_Z2, C::BF>(p.acm.W3, 1, z2, L.tbl + p.acm.tb3, [&](int ob, const f32x16& acc) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int u = ru(q) + L.h4;
      if (u < C::AC) {
        const float t = tanhf(acc[q]);
        L.sl[ru(q) * 32] = t * limv[q];
        if constexpr (ST) fm_st(t3r, ru(q), L.ld4, L.vo, t);
      }
    }
  });
}

// Critic forward through L2 with q = w3 . relu(h2) + b3 reduced per sample.
// ST: store h1 / h2 feature-major.
// H2L: h2 goes to the wave's LDS image (the caller's fused layer-3 weight gradient reads it there) instead
// of to HBM.
template <class C, bool ST, int R = 30, bool H2L = false>
__device__ __forceinline__ float critic_forward(const CriticDev& Q, const f32x16 (&xin)[C::NB_CIN], const Lane& L,
                                                float* H1g, float* H2g, uint64_t& m1lo, uint64_t& m1hi,
                                                uint64_t& m2lo, uint64_t& m2hi) {
  const rsrc_t h1r = rsrc(H1g), h2r = rsrc(H2g);
  dense<C::NB_CIN, C::RV_CIN, C::BF>(Q.W1, 8, xin, L.tbl + Q.tb1, [&](int ob, const f32x16& acc) {
    uint32_t bits = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ur = 32 * ob + ru(q);
      const float v = fmaxf(acc[q], 0.f);
      L.bl[ur * 32] = v;
      if constexpr (ST) op_st<C::BF>(h1r, ur, L.ld4, L.vo, v);
      bits |= (uint32_t)(v > 0.f) << q;
    }
    setbits(m1lo, m1hi, ob, bits);
  });
  SPP_TP(R);
  float qp = 0.f;
  const float* w3 = L.tbl + Q.tw3;
  dense_lds<8, C::BF>(Q.W2, L.img, L.tbl + Q.tb2, [&](int ob, const f32x16& acc) {
    uint32_t bits = 0;
    float tv[16];
    tvals(w3, ob, L.h4, tv);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float v = fmaxf(acc[q], 0.f);
      if constexpr (H2L) L.bl[(32 * ob + ru(q)) * 32] = v;  // the image's h1 reads are done (dense_lds)
      else if constexpr (ST) op_st<C::BF>(h2r, 32 * ob + ru(q), L.ld4, L.vo, v);
      qp = fmaf(v, tv[q], qp);
      bits |= (uint32_t)(v > 0.f) << q;
    }
    setbits(m2lo, m2hi, ob, bits);
  });
  SPP_TP(R + 1);
  return qp + __shfl_xor(qp, 32, 64) + *Q.b3;
}

// Squash (sac/models.py:37-52) of the pairing-layout heads tile with eps [aout][Bp].
// Writes a_d = denormalize(tanh(u)*lim) into LDS rows [0, AOUT); returns logpi.
template <class C, bool BRF = false>
__device__ __forceinline__ float squash_write(const SacArgs& p, const f32x16 (&hd)[C::NB_PAIR],
                                              const float* __restrict__ EPS, const Lane& L) {
  float lp = 0.f, corr = 0.f;
  const int h8 = 8 * L.h;
  // all eps reads first (one latency for the block, not one per output).  The loads may be
  // issued for every lane, so they go through a resource bounded to the [AOUT][Bp] array:
  // the pairing layout's unused slots (j >= AOUT) read 0 instead of past the array.
  const rsrc_t er = rsrc_n(EPS, C::AOUT * L.ld4);
  float ev[C::NB_PAIR][8];
#pragma unroll
  for (int ib = 0; ib < C::NB_PAIR; ++ib)
#pragma unroll
    for (int r = 0; r < 8; ++r) ev[ib][r] = 16 * ib + r < C::AOUT ? fm_ldb(er, 16 * ib + r, L.ld4, L.vp) : 0.f;
  // BRF (critic phase): no per-slot branch (a branch holding a table load and its use costs one
  // LDS round trip per slot); slots j >= AOUT compute on index 0 and are dropped.  The actor
  // phase keeps the branches (its branch-free live ranges spill).
  constexpr bool kBranchFree = BRF;
#pragma unroll
  for (int ib = 0; ib < C::NB_PAIR; ++ib)
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int j0 = 16 * ib + r;
      if (j0 >= C::AOUT) continue;  // no lane holds a slot of this row (unrolled: folded away)
      const int j = j0 + h8;
      const bool ok = j < C::AOUT;
      if (kBranchFree || ok) {
        const int jj = ok ? j : 0;
        constexpr bool F = C::BF;
        const float mu = hd[ib][r];
        const float ls = fminf(fmaxf(hd[ib][r + 8], -20.f), 2.f);
        const float sc = t_exp<F>(ls);
        const float e = ev[ib][r];
        const float u = fadd_rn(mu, fmul_rn(e, sc));
        float lpj;
        if constexpr (F) {  // Normal(mu, sc).log_prob(u) with u - mu = e sc, log sc = ls
          lpj = -0.5f * e * e - ls - kLogSqrt2Pi;
        } else {  // the reference's operation order
          const float d = fsub_rn(u, mu);
          const float var = fmul_rn(sc, sc);
          lpj = fsub_rn(fsub_rn(fdiv_rn(-fmul_rn(d, d), 2.f * var), logf(sc)), kLogSqrt2Pi);
        }
        const float cj = 2.f * fsub_rn(fsub_rn(kLog2, u), t_softplus<F>(-2.f * u));
        lp += ok ? lpj : 0.f;
        corr += ok ? cj : 0.f;
        const float a = fmul_rn(t_tanh<F>(u), actor_lim<true>(p, L.tbl, jj));
        const float ad = denorm<true>(p, L.tbl, jj, a);
        if (ok) L.pl[j0 * 32] = ad;
      }
    }
  SPP_XLANE_SYNC();
  const float tot = lp + __shfl_xor(lp, 32, 64);
  const float tc = corr + __shfl_xor(corr, 32, 64);
  return fsub_rn(tot, tc);
}

// ============================================================================ critic phase
template <class C>
__global__ __launch_bounds__(256, 1) void k_sac_critic_phase(SacArgs p) {
  __shared__ __attribute__((aligned(16))) float smem[kWavesPerWG * kLdsPerWave];
  __shared__ __attribute__((aligned(16))) float tbl[kTabMax];
  __shared__ __attribute__((aligned(16))) float s_dq[kWavesPerWG][32];  // the tile's d loss / dq, for the fused layer-3 weight gradient
  SPP_TP_INIT();
  load_table(p, tbl);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* big = smem + w * kLdsPerWave;
  float* small = big + kSmallRow * 32;
  const int ntiles = p.Bp / 32;
  const int ld = p.Bp;
  const float alpha = *p.alpha;
  float w3a[4] = {0.f, 0.f, 0.f, 0.f}, w3b[4] = {0.f, 0.f, 0.f, 0.f}, b3a = 0.f, b3b = 0.f;  // fused fc3 grads
  for (int tile = blockIdx.x * kWavesPerWG + w; tile < ntiles; tile += gridDim.x * kWavesPerWG) {
    const Lane L = make_lane(big, small, tbl, ld, tile * 32 + (lane & 31));
    const int b = L.b;
    const bool valid = b < p.B;
    uint64_t d0 = 0, d1 = 0, d2 = 0, d3 = 0;
    // ---- target action: a' ~ pi(s'), a'_d, logpi'   (sac_acm.py:44-45)
    SPP_TP(0);
    actor_trunk<C, false>(p.actor, p.S2, C::OB * L.ld4, L, nullptr, nullptr, d0, d1, d2, d3);
    float lp2;
    {
      f32x16 hd[C::NB_PAIR];
      load_pair<C>(hd, big);
      lp2 = squash_write<C, true>(p, hd, p.EPS1, L);
    }
    SPP_TP(4);
    // ---- critic-target input: [s' | ACM(s', a'_d)] or [s' | a'_d]   (:46-48)
    f32x16 tin[C::NB_CIN];
    if constexpr (C::ACMC) {
      f32x16 xin[C::NB_ACMIN];
      load_cat_gl<C::NB_OB, C::NB_AOUT>(xin, p.S2, C::OB * L.ld4, C::OB, L.ld4, L.vo, big, C::AOUT);
      acm_forward<C, false>(p, xin, L, nullptr, nullptr, nullptr);
      load_cat_gl<C::NB_OB, C::NB_CA>(tin, p.S2, C::OB * L.ld4, C::OB, L.ld4, L.vo, small, C::AC);
    } else {
      load_cat_gl<C::NB_OB, C::NB_CA>(tin, p.S2, C::OB * L.ld4, C::OB, L.ld4, L.vo, big, C::AOUT);
    }
    // ---- soft-min twin target (:50-56)
    SPP_TP(5);
    const float q1t = critic_forward<C, false, 6>(p.targ[0], tin, L, nullptr, nullptr, d0, d1, d2, d3);
    const float q2t = critic_forward<C, false, 8>(p.targ[1], tin, L, nullptr, nullptr, d0, d1, d2, d3);
    const float notdone = 1.f - p.DN[b];
    const float y = fadd_rn(p.R[b], fmul_rn(p.gamma * notdone, fsub_rn(fminf(q1t, q2t), alpha * lp2)));
    // ---- both critics: forward, MSE grad, backward to weight-gradient operands (:117-131)
    float lq0 = 0.f, lq1 = 0.f;
#pragma unroll 1
    for (int i = 0; i < 2; ++i) {
      uint64_t m1lo = 0, m1hi = 0, m2lo = 0, m2hi = 0;
      f32x16 xin[C::NB_CIN];
      load_cat_gg<C::NB_OB, C::NB_CA>(xin, p.S, C::OB, C::ACMC ? p.AENV : p.ACT, C::CA, L.ld4, L.vo);
      const CriticDev& Q = p.critic[i];
      SPP_TP(10);
      const float q = critic_forward<C, true, 11, C::F3>(Q, xin, L, p.H1[i], C::F3 ? nullptr : p.H2[i], m1lo, m1hi,
                                                        m2lo, m2hi);
      const float diff = fsub_rn(q, y);
      const float dq = valid ? fmul_rn(2.f * diff, p.inv_B) : 0.f;  // d mse / dq
      const float lqi = (valid && L.h == 0) ? diff * diff : 0.f;
      if (i == 0) lq0 = lqi; else lq1 = lqi;
      if constexpr (!C::F3) {
        if (L.h == 0) p.DQ[i][b] = dq;  // (h2 is stored by critic_forward: the k_dw job dW3 = dq . h2^T)
      } else {
      // fc3's weight gradient, fused (sac_acm.py:117-131; dW3 = dq . h2^T, db3 = sum dq): h2 is in the image;
      // lane l sums units l + 64k over the tile's 32 samples (rotated column order: conflict-free rows)
      // into registers that carry over the wave's tiles; the per-wave partials are reduced in a fixed order
      // by k_dw_reduce (no h2 / dq written to HBM and read back)
      if (L.h == 0) s_dq[w][L.s] = dq;
      SPP_XLANE_SYNC();
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int u = lane + 64 * k;
        const float* row = big + u * 32;
        float acc = 0.f;
#pragma unroll 8
        for (int j = 0; j < 32; ++j) {
          const int s2 = (j + u) & 31;
          acc = fmaf(row[s2], s_dq[w][s2], acc);
        }
        if (i == 0) w3a[k] += acc;
        else w3b[k] += acc;
      }
      const float dsum = wave_sum(L.h == 0 ? dq : 0.f);
      if (i == 0) b3a += dsum;
      else b3b += dsum;
      SPP_XLANE_SYNC();  // the image rows are rewritten by the delta2 staging below
      }
      // delta2 = dq * w3 * relu'(h2): staged through the LDS image, stored feature-major
      const rsrc_t d2r = rsrc(p.D2[i]);
      const float* w3 = tbl + Q.tw3;
#pragma unroll 1
      for (int ob = 0; ob < 8; ++ob) {
        float tv[16];
        tvals(w3, ob, L.h4, tv);
#pragma unroll
        for (int q2 = 0; q2 < 16; ++q2) {
          const int ur = 32 * ob + ru(q2);
          const float v = getbit(m2lo, m2hi, ob, q2) ? dq * tv[q2] : 0.f;
          L.bl[ur * 32] = v;
          op_st<C::BF>(d2r, ur, L.ld4, L.vo, v);
        }
      }
      SPP_TP(13);
      // delta1 = (W2^T delta2) * relu'(h1)
      const rsrc_t d1r = rsrc(p.D1[i]);
      dense_lds<8, C::BF>(Q.W2T, big, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
        for (int q2 = 0; q2 < 16; ++q2)
          op_st<C::BF>(d1r, 32 * ob + ru(q2), L.ld4, L.vo, getbit(m1lo, m1hi, ob, q2) ? acc[q2] : 0.f);
      });
    }
    SPP_TP(14);
    const float s0 = wave_sum(lq0), s1 = wave_sum(lq1);
    if (lane == 0) {
      p.part[tile * kParts + 0] = s0;
      p.part[tile * kParts + 1] = s1;
    }
    SPP_TP(15);
  }
  // this wave's fc3 partials [256 weights | bias] per critic (every wave writes, tiles or not)
  if constexpr (C::F3) {
    const int64_t wg = (int64_t)blockIdx.x * kWavesPerWG + w;
    float* o0 = p.W3P[0] + wg * p.w3p_stride;
    float* o1 = p.W3P[1] + wg * p.w3p_stride;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o0[lane + 64 * k] = w3a[k];
      o1[lane + 64 * k] = w3b[k];
    }
    if (lane == 0) {
      o0[256] = b3a;
      o1[256] = b3b;
    }
  }
  SPP_TP_FLUSH();
}

// ============================================================================ actor phase
// Scratch for the frozen-ACM backward (feature-major, same-lane re-read).
struct AcmScratch {
  float *Z1, *Z2, *T3;
  // wide heads (NB_PAIR > 2): the actor phase runs as two kernels; the first hands the second
  // d loss / d a_d [AOUT][Bp] (GAD) and the trunk's ReLU masks [tile][4][64 lanes] (MASK)
  float* GAD;
  uint64_t* MASK;
};

template <class C>
__global__ __launch_bounds__(256, 1) void k_sac_actor_phase(SacArgs p, AcmScratch z) {
  __shared__ float smem[kWavesPerWG * kLdsPerWave];
  __shared__ __attribute__((aligned(16))) float tbl[kTabMax];
  SPP_TP_INIT();
  load_table(p, tbl);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* big = smem + w * kLdsPerWave;
  float* small = big + kSmallRow * 32;
  const int ntiles = p.Bp / 32;
  const int ld = p.Bp;
  const float alpha = *p.alpha;
  for (int tile = blockIdx.x * kWavesPerWG + w; tile < ntiles; tile += gridDim.x * kWavesPerWG) {
    const Lane L = make_lane(big, small, tbl, ld, tile * 32 + (lane & 31));
    const int b = L.b;
    const bool valid = b < p.B;
    const float g_lp = valid ? alpha * p.inv_B : 0.f;  // d loss / d logpi_b
    // ---- a, logpi = actor(s)  (sac_acm.py:137)
    uint64_t a1lo = 0, a1hi = 0, a2lo = 0, a2hi = 0;
    SPP_TP(26);
    actor_trunk<C, true>(p.actor, p.S, C::OB * L.ld4, L, p.AH1, p.AH2, a1lo, a1hi, a2lo, a2hi);
    SPP_TP(27);  // actor trunk
    f32x16 hd[C::NB_PAIR];
    load_pair<C>(hd, big);
    const float lp = squash_write<C>(p, hd, p.EPS2, L);  // a_d -> big rows [0, AOUT)
    SPP_TP(28);  // squash
    // Wide heads (Ant): park mu / raw log-std in the ADH rows the heads backward overwrites
    // (same lane, same element), instead of keeping NB_PAIR tiles live through the critics.
    constexpr bool kParkHeads = C::NB_PAIR > 2;
    if constexpr (kParkHeads) {
#pragma unroll
      for (int ib = 0; ib < C::NB_PAIR; ++ib)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int j0 = 16 * ib + r;
          if (j0 + 8 * L.h < C::AOUT) {
            fm_st(rsrc(p.ADH), j0, L.ld4, L.vp, hd[ib][r]);
            fm_st(rsrc(p.ADH), C::AOUT + j0, L.ld4, L.vp, hd[ib][r + 8]);
          }
        }
    }
    // ---- critic input [s | ACM(s, a_d)] or [s | a_d]  (:67-72)
    f32x16 cin[C::NB_CIN];
    if constexpr (C::ACMC) {
      f32x16 xin[C::NB_ACMIN];
      load_cat_gl<C::NB_OB, C::NB_AOUT>(xin, p.S, C::OB * L.ld4, C::OB, L.ld4, L.vo, big, C::AOUT);
      acm_forward<C, true>(p, xin, L, z.Z1, z.Z2, z.T3);
      load_cat_gl<C::NB_OB, C::NB_CA>(cin, p.S, C::OB * L.ld4, C::OB, L.ld4, L.vo, small, C::AC);
    } else {
      load_cat_gl<C::NB_OB, C::NB_CA>(cin, p.S, C::OB * L.ld4, C::OB, L.ld4, L.vo, big, C::AOUT);
    }
    SPP_TP(29);  // ACM forward
    // ---- q = min(Q1, Q2)(s, c)  (:73-75), masks kept for the backward
    uint64_t ma0 = 0, ma1 = 0, ma2 = 0, ma3 = 0, mb0 = 0, mb1 = 0, mb2 = 0, mb3 = 0;
    const float q1 = critic_forward<C, false>(p.critic[0], cin, L, nullptr, nullptr, ma0, ma1, ma2, ma3);
    const float q2 = critic_forward<C, false>(p.critic[1], cin, L, nullptr, nullptr, mb0, mb1, mb2, mb3);
    const float qmin = fminf(q1, q2);
    // torch.minimum backward: ties split the gradient in half
    const float gq = valid ? -p.inv_B : 0.f;
    const float dqa = q1 < q2 ? gq : (q1 == q2 ? 0.5f * gq : 0.f);
    const float dqb = q2 < q1 ? gq : (q1 == q2 ? 0.5f * gq : 0.f);
    SPP_TP(19);  // q min (the critic layers themselves: slots 30, 31)
    // ---- back through both critics to their action input
    f32x16 dca[C::NB_CA];
#pragma unroll
    for (int ib = 0; ib < C::NB_CA; ++ib) dca[ib] = zero16();
#pragma unroll 1
    for (int i = 0; i < 2; ++i) {
      const CriticDev& Q = p.critic[i];
      const uint64_t k0 = i ? mb0 : ma0, k1 = i ? mb1 : ma1, k2 = i ? mb2 : ma2, k3 = i ? mb3 : ma3;
      const float dqi = i ? dqb : dqa;
      const float* w3 = tbl + Q.tw3;
#pragma unroll 1
      for (int ob = 0; ob < 8; ++ob) {
        float tv[16];
        tvals(w3, ob, L.h4, tv);
#pragma unroll
        for (int q = 0; q < 16; ++q) L.bl[(32 * ob + ru(q)) * 32] = getbit(k2, k3, ob, q) ? dqi * tv[q] : 0.f;
      }
      SPP_TPN(20);  // delta staging
      dense_lds<8, C::BF>(Q.W2T, big, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
        for (int q = 0; q < 16; ++q) L.bl[(32 * ob + ru(q)) * 32] = getbit(k0, k1, ob, q) ? acc[q] : 0.f;
      });
      SPP_TPN(21);  // W2T
      dense_lds<C::NB_CA, C::BF>(Q.W1Ta, big, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
        for (int ib = 0; ib < C::NB_CA; ++ib)
          if (ib == ob) dca[ib] += acc;
      });
      SPP_TPN(22);  // W1Ta
    }
    SPP_TP(31);  // critics backward
    // ---- through the frozen ACM to d a_d  (basic_model.py:118-126 backward)
    if constexpr (C::ACMC) {
      // Every scratch value of the three layers is requested up front: buffer loads cannot be
      // moved across the epilogues' LDS stores (no alias proof), so loads issued inside an
      // epilogue run as one round trip each.
      // (Wide-head configs keep the per-element loads: their registers are taken.)
      constexpr bool kPre = !kParkHeads;
      float t3v[16], limv[16], z2v[16], z1v[2][16];
      const rsrc_t t3r = rsrc_n(z.T3, C::AC * L.ld4);  // rows >= AC read 0
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int u = ru(q) + L.h4;
        t3v[q] = fm_ldb(t3r, ru(q), L.ld4, L.vo);
        limv[q] = acm_lim<true>(p, L.tbl, u < C::AC ? u : 0);
      }
      if constexpr (kPre) {
#pragma unroll
        for (int q = 0; q < 16; ++q) z2v[q] = fm_ld(rsrc(z.Z2), ru(q), L.ld4, L.vo);
#pragma unroll
        for (int ob = 0; ob < 2; ++ob)
#pragma unroll
          for (int q = 0; q < 16; ++q) z1v[ob][q] = fm_ld(rsrc(z.Z1), 32 * ob + ru(q), L.ld4, L.vo);
      }
      auto z2at = [&](int q) {
        if constexpr (kPre) return z2v[q];
        else return fm_ld(rsrc(z.Z2), ru(q), L.ld4, L.vo);
      };
      auto z1at = [&](int ob, int q) {
        if constexpr (kPre) return ob ? z1v[1][q] : z1v[0][q];
        else return fm_ld(rsrc(z.Z1), 32 * ob + ru(q), L.ld4, L.vo);
      };
      f32x16 dp3[1];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int u = ru(q) + L.h4;
        const float t = t3v[q];
        dp3[0][q] = u < C::AC ? dca[0][q] * limv[q] * (1.f - t * t) : 0.f;
      }
      SPP_TPN(23);  // ACM bwd input
      dense<1, C::RV_AC, C::BF>(p.acm.W3T, 1, dp3, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const float zz = z2at(q);
          L.sl[ru(q) * 32] = acc[q] * (1.f - zz * zz);
        }
      });
      SPP_TPN(24);  // ACM W3T
      f32x16 dp2[1];
      lds_load<1>(dp2, small);
      dense<1, C::RV_Z2, C::BF>(p.acm.W2T, 2, dp2, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const float zz = z1at(ob, q);
          L.sl[(32 * ob + ru(q)) * 32] = acc[q] * (1.f - zz * zz);
        }
      });
      SPP_TPN(25);  // ACM W2T
      f32x16 dp1[2];
      lds_load<2>(dp1, small);
      dense<2, C::RV_Z1, C::BF>(p.acm.W1Ta, C::NB_AOUT, dp1, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int ur = 32 * ob + ru(q);
          if (ur + L.h4 < C::AOUT) L.bl[ur * 32] = acc[q];
        }
      });
    } else {
#pragma unroll
      for (int ib = 0; ib < C::NB_CA; ++ib)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int ur = 32 * ib + ru(q);
          if (ur + L.h4 < C::AOUT) L.bl[ur * 32] = dca[ib][q];
        }
    }
    SPP_TP(16);  // ACM backward
    if constexpr (kParkHeads) {
      // Wide heads: the heads and trunk backward run in k_sac_actor_heads (a second kernel with
      // the whole register file: in one kernel the live ranges spill to scratch, and spilled
      // phase kernels have returned wrong results).  Hand over d a_d and the masks.
      const rsrc_t gr = rsrc(z.GAD);
#pragma unroll
      for (int ib = 0; ib < C::NB_AOUT; ++ib)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int ur = 32 * ib + ru(q);
          if (ur + L.h4 < C::AOUT) fm_st(gr, ur, L.ld4, L.vo, L.bl[ur * 32]);
        }
      uint64_t* mk = z.MASK + (int64_t)tile * 4 * 64 + lane;
      mk[0] = a1lo;
      mk[64] = a1hi;
      mk[128] = a2lo;
      mk[192] = a2hi;
      const float ps = wave_sum((valid && L.h == 0) ? fsub_rn(alpha * lp, qmin) : 0.f);
      const float pl = wave_sum((valid && L.h == 0) ? lp : 0.f);
      if (lane == 0) {
        p.part[tile * kParts + 2] = ps;
        p.part[tile * kParts + 4] = pl;
      }
      continue;
    }
    // ---- heads backward in the pairing layout (squash, denorm, custom loss, logpi)
    float sac_part = (valid && L.h == 0) ? fsub_rn(alpha * lp, qmin) : 0.f;
    float dist_part = 0.f;
    const float cl_scale = valid ? p.custom_loss * 2.f * p.inv_B / (float)C::AOUT : 0.f;
    const int h8 = 8 * L.h;
    {
      // Branch-free over the pairing slots: every lane loads through resources bounded to the
      // arrays (slots j >= AOUT read 0) and computes; results of those slots are dropped.  Per-slot
      // branches would put each load and its use in one block, i.e. one round trip per slot.
      const rsrc_t adhr = rsrc_n(p.ADH, 2 * C::AOUT * L.ld4);
      const rsrc_t epsr = rsrc_n(p.EPS2, C::AOUT * L.ld4);
      const rsrc_t s2r = rsrc_n(p.S2, C::OB * L.ld4);
      const bool closs = p.custom_loss != 0.f;
      SPP_XLANE_SYNC();  // d loss / d a_d was written in the natural layout (other lanes' rows)
  #pragma unroll
      for (int ib = 0; ib < C::NB_PAIR; ++ib)
  #pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int j0 = 16 * ib + r;
          const int j = j0 + h8;
          const bool ok = j < C::AOUT;
          const int jj = ok ? j : 0;
          const float mu = kParkHeads ? fm_ldb(adhr, j0, L.ld4, L.vp) : hd[ib][r];
          const float lsr = kParkHeads ? fm_ldb(adhr, C::AOUT + j0, L.ld4, L.vp) : hd[ib][r + 8];
          const float e = fm_ldb(epsr, j0, L.ld4, L.vp);
          const float s2 = closs ? fm_ldb(s2r, j0, L.ld4, L.vp) : 0.f;
          const float ls = fminf(fmaxf(lsr, -20.f), 2.f);
          const float sc = expf(ls);
          const float u = fadd_rn(mu, fmul_rn(e, sc));
          const float d = fsub_rn(u, mu);
          const float t = tanhf(u);
          const float lim = actor_lim<true>(p, L.tbl, jj);
          const float a = fmul_rn(t, lim);
          float g_ad = L.pl[j0 * 32];  // from the critics through the ACM
          float g_a = 0.f;
          if (closs) {
            if (p.norm_closs) {
              const float df = fsub_rn(a, normalize<true>(p, L.tbl, jj, s2));
              g_a += cl_scale * df;
              dist_part += (valid && ok) ? df * df : 0.f;
            } else {
              const float df = fsub_rn(denorm<true>(p, L.tbl, jj, a), s2);
              g_ad += cl_scale * df;
              dist_part += (valid && ok) ? df * df : 0.f;
            }
          }
          g_a += g_ad * denorm_scale<true>(p, L.tbl, jj);
          const float var = fmul_rn(sc, sc);
          const float sig_m2u = 1.f / (1.f + expf(2.f * u));  // sigmoid(-2u)
          const float gu = g_a * lim * (1.f - t * t) + g_lp * (-d / var + 2.f - 4.f * sig_m2u);
          const float gmu = gu + g_lp * d / var;
          const float gsc = gu * e + g_lp * (d * d / (var * sc) - 1.f / sc);
          const float gls = (lsr >= -20.f && lsr <= 2.f) ? gsc * sc : 0.f;
          hd[ib][r] = ok ? gmu : 0.f;
          hd[ib][r + 8] = ok ? gls : 0.f;
        }
      // stores after all of the loop's loads (a buffer store would order every later load behind it)
  #pragma unroll
      for (int ib = 0; ib < C::NB_PAIR; ++ib)
  #pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int j0 = 16 * ib + r;
          if (j0 + h8 < C::AOUT) {
            fm_st(rsrc(p.ADH), j0, L.ld4, L.vp, hd[ib][r]);
            fm_st(rsrc(p.ADH), C::AOUT + j0, L.ld4, L.vp, hd[ib][r + 8]);
          }
        }
    }
    SPP_TP(17);  // heads backward
    // ---- dh2 = Wh^T dheads * relu'(h2); dh1 = W2^T dh2 * relu'(h1)
    dense<C::NB_PAIR, C::RV_PAIR, C::BF>(p.actor.WhT, 8, hd, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ur = 32 * ob + ru(q);
        const float v = getbit(a2lo, a2hi, ob, q) ? acc[q] : 0.f;
        L.bl[ur * 32] = v;
        op_st<C::BF>(rsrc(p.AD2), ur, L.ld4, L.vo, v);
      }
    });
    {
      dense_lds<8, C::BF>(p.actor.W2T, big, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
        for (int q = 0; q < 16; ++q)
          op_st<C::BF>(rsrc(p.AD1), 32 * ob + ru(q), L.ld4, L.vo, getbit(a1lo, a1hi, ob, q) ? acc[q] : 0.f);
      });
    }
    SPP_TP(18);  // trunk backward
    const float ps = wave_sum(sac_part);
    const float pd = wave_sum(dist_part);
    const float pl = wave_sum((valid && L.h == 0) ? lp : 0.f);
    if (lane == 0) {
      p.part[tile * kParts + 2] = ps;
      p.part[tile * kParts + 3] = pd;
      p.part[tile * kParts + 4] = pl;
    }
  }
  SPP_TP_FLUSH();
}

// ============================================================================ actor phase, wide heads
// k_sac_actor_heads: the heads backward (squash, denormalisation, custom loss, logpi, in the
// pairing layout) and the trunk backward of the actor phase for wide heads (Ant), after
// k_sac_actor_phase handed over d loss / d a_d (z.GAD) and the trunk's ReLU masks (z.MASK).  One
// pairing block at a time: the block's parked heads, eps, targets and d a_d are requested together
// (one round trip per block), the limit / normaliser vectors come from the LDS table, and the
// results stay in registers (the WhT layer's input tile) until every load has been issued.
template <class C>
__global__ __launch_bounds__(256, 1) void k_sac_actor_heads(SacArgs p, AcmScratch z) {
  __shared__ float smem[kWavesPerWG * kLdsPerWave];
  __shared__ __attribute__((aligned(16))) float tbl[kTabMax];
  SPP_TP_INIT();
  load_table(p, tbl);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* big = smem + w * kLdsPerWave;
  float* small = big + kSmallRow * 32;
  const int ntiles = p.Bp / 32;
  const int ld = p.Bp;
  const float alpha = *p.alpha;
  for (int tile = blockIdx.x * kWavesPerWG + w; tile < ntiles; tile += gridDim.x * kWavesPerWG) {
    const Lane L = make_lane(big, small, tbl, ld, tile * 32 + (lane & 31));
    const bool valid = L.b < p.B;
    const float g_lp = valid ? alpha * p.inv_B : 0.f;
    const uint64_t* mk = z.MASK + (int64_t)tile * 4 * 64 + lane;
    const uint64_t a1lo = mk[0], a1hi = mk[64], a2lo = mk[128], a2hi = mk[192];
    float dist_part = 0.f;
    const float cl_scale = valid ? p.custom_loss * 2.f * p.inv_B / (float)C::AOUT : 0.f;
    const rsrc_t adhr = rsrc_n(p.ADH, 2 * C::AOUT * L.ld4);
    const rsrc_t epsr = rsrc_n(p.EPS2, C::AOUT * L.ld4);
    const rsrc_t s2r = rsrc_n(p.S2, C::OB * L.ld4);
    const rsrc_t gr = rsrc_n(z.GAD, C::AOUT * L.ld4);
    const bool closs = p.custom_loss != 0.f;
    const int h8 = 8 * L.h;
    // one pairing block per iteration (not unrolled: a block's loads and math stay within the
    // iteration); results go to the LDS image in the pairing layout (rows j / AOUT + j)
#pragma unroll 1
    for (int ib = 0; ib < C::NB_PAIR; ++ib) {
      float mu[8], lsr[8], ev[8], s2v[8], gv[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int j0 = 16 * ib + r;
        mu[r] = fm_ldb(adhr, j0, L.ld4, L.vp);
        lsr[r] = fm_ldb(adhr, C::AOUT + j0, L.ld4, L.vp);
        ev[r] = fm_ldb(epsr, j0, L.ld4, L.vp);
        s2v[r] = closs ? fm_ldb(s2r, j0, L.ld4, L.vp) : 0.f;
        gv[r] = fm_ldb(gr, j0, L.ld4, L.vp);
      }
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int j0 = 16 * ib + r;
        const int j = j0 + h8;
        const bool ok = j < C::AOUT;
        const int jj = ok ? j : 0;
        constexpr bool F = C::BF;
        const float e = ev[r];
        const float ls = fminf(fmaxf(lsr[r], -20.f), 2.f);
        const float sc = t_exp<F>(ls);
        const float u = fadd_rn(mu[r], fmul_rn(e, sc));
        const float d = fsub_rn(u, mu[r]);
        const float t = t_tanh<F>(u);
        const float lim = actor_lim<true>(p, L.tbl, jj);
        const float a = fmul_rn(t, lim);
        float g_ad = gv[r];  // from the critics through the ACM
        float g_a = 0.f;
        if (closs) {
          if (p.norm_closs) {
            const float df = fsub_rn(a, normalize<true>(p, L.tbl, jj, s2v[r]));
            g_a += cl_scale * df;
            dist_part += (valid && ok) ? df * df : 0.f;
          } else {
            const float df = fsub_rn(denorm<true>(p, L.tbl, jj, a), s2v[r]);
            g_ad += cl_scale * df;
            dist_part += (valid && ok) ? df * df : 0.f;
          }
        }
        g_a += g_ad * denorm_scale<true>(p, L.tbl, jj);
        const float var = fmul_rn(sc, sc);
        const float ivar = t_rcp<F>(var), isc = t_rcp<F>(sc);
        const float sig_m2u = t_rcp<F>(1.f + t_exp<F>(2.f * u));  // sigmoid(-2u)
        const float gu = g_a * lim * (1.f - t * t) + g_lp * (-d * ivar + 2.f - 4.f * sig_m2u);
        const float gmu = gu + g_lp * d * ivar;
        const float gsc = gu * e + g_lp * (d * d * ivar * isc - isc);
        const float gls = (lsr[r] >= -20.f && lsr[r] <= 2.f) ? gsc * sc : 0.f;
        if (ok) {  // slot j >= AOUT would land on row AOUT + j' of a valid slot's log-std
          L.pl[j0 * 32] = gmu;
          L.pl[(C::AOUT + j0) * 32] = gls;
        }
      }
    }
    f32x16 hd[C::NB_PAIR];
    load_pair<C>(hd, big);
    // the heads' gradient operands (dW of fc_prob / fc_scale), after every load above
#pragma unroll
    for (int ib = 0; ib < C::NB_PAIR; ++ib)
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int j0 = 16 * ib + r;
        if (j0 + h8 < C::AOUT) {
          fm_st(rsrc(p.ADH), j0, L.ld4, L.vp, hd[ib][r]);
          fm_st(rsrc(p.ADH), C::AOUT + j0, L.ld4, L.vp, hd[ib][r + 8]);
        }
      }
    SPP_TP(17);  // heads backward
    // ---- dh2 = Wh^T dheads * relu'(h2); dh1 = W2^T dh2 * relu'(h1)
    dense<C::NB_PAIR, C::RV_PAIR, C::BF>(p.actor.WhT, 8, hd, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ur = 32 * ob + ru(q);
        const float v = getbit(a2lo, a2hi, ob, q) ? acc[q] : 0.f;
        L.bl[ur * 32] = v;
        op_st<C::BF>(rsrc(p.AD2), ur, L.ld4, L.vo, v);
      }
    });
    dense_lds<8, C::BF>(p.actor.W2T, big, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q = 0; q < 16; ++q)
        op_st<C::BF>(rsrc(p.AD1), 32 * ob + ru(q), L.ld4, L.vo, getbit(a1lo, a1hi, ob, q) ? acc[q] : 0.f);
    });
    SPP_TP(18);  // trunk backward
    const float pd = wave_sum(dist_part);
    if (lane == 0) p.part[tile * kParts + 3] = pd;
  }
  SPP_TP_FLUSH();
}

// ============================================================================ rollout action
struct ActArgs {
  int E, mode, denorm_out;
  float act_noise;
  const float *obs, *eps, *noise;  // row-major [E][ob], [E][aout]
  float *target_out, *env_out;     // [E][aout], [E][ac]
  int plain;  // vanilla SAC (sac.py + DDPG.noise_action, ddpg.py:171-176): no ACM, env action = actor action
};

template <class C>
__global__ __launch_bounds__(256, 1) void k_policy_act(SacArgs p, ActArgs a) {
  __shared__ float smem[kWavesPerWG * kLdsPerWave];
  __shared__ __attribute__((aligned(16))) float tbl[kTabMax];
  load_table(p, tbl);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* big = smem + w * kLdsPerWave;
  float* small = big + kSmallRow * 32;
  const int ntiles = (a.E + 31) / 32;
  for (int tile = blockIdx.x * kWavesPerWG + w; tile < ntiles; tile += gridDim.x * kWavesPerWG) {
    const int e = tile * 32 + (lane & 31);
    const bool valid = e < a.E;
    const int er = valid ? e : 0;
    // row-major obs: element (unit u, env e) = obs[e*OB + u] -> ld = 1, offset 4h + e*OB
    Lane L = make_lane(big, small, tbl, 1, er * C::OB);
    const bool use_actor = a.mode == 1 || a.mode == 2;
    if (use_actor) {
      uint64_t d0 = 0, d1 = 0, d2 = 0, d3 = 0;
      actor_trunk<C, false>(p.actor, a.obs, a.E * C::OB * 4, L, nullptr, nullptr, d0, d1, d2, d3);
    }
    f32x16 hd[C::NB_PAIR];
    if (use_actor) load_pair<C>(hd, big);
    const int h8 = 8 * L.h;
#pragma unroll
    for (int ib = 0; ib < C::NB_PAIR; ++ib)
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int j0 = 16 * ib + r;
        const int j = j0 + h8;
        if (j < C::AOUT) {
          const float lim = actor_lim<true>(p, L.tbl, j);
          float act;
          if (a.plain && (a.mode == 0 || a.mode == 3)) {
            act = valid ? a.eps[er * C::AOUT + j] : 0.f;  // action_space.sample() drawn by the caller (ddpg.py:178-180)
          } else if (a.plain) {  // DDPG.noise_action: a + act_noise * N(0,1), clip to [-lim, lim]
            const float mu = hd[ib][r];
            float u = mu;
            if (a.mode == 1 && a.eps) {
              const float ls = fminf(fmaxf(hd[ib][r + 8], -20.f), 2.f);
              u = fadd_rn(mu, fmul_rn(valid ? a.eps[er * C::AOUT + j] : 0.f, expf(ls)));
            }
            act = fmul_rn(tanhf(u), lim);
            if (a.mode == 1 && a.noise) act = fadd_rn(act, a.act_noise * (valid ? a.noise[er * C::AOUT + j] : 0.f));
            act = fminf(fmaxf(act, -lim), lim);
          } else if (a.mode == 0) {
            act = valid ? lim * a.eps[er * C::AOUT + j] : 0.f;  // off_policy.py:50-54
          } else if (a.mode == 3) {
            act = valid ? a.eps[er * C::AOUT + j] : 0.f;  // caller's action (on-policy process_action)
          } else {
            const float mu = hd[ib][r];
            float u = mu;
            if (a.mode == 1 && a.eps) {
              const float ls = fminf(fmaxf(hd[ib][r + 8], -20.f), 2.f);
              u = fadd_rn(mu, fmul_rn(valid ? a.eps[er * C::AOUT + j] : 0.f, expf(ls)));
            }
            act = fmul_rn(tanhf(u), lim);
            if (a.mode == 1 && a.noise) act += fmul_rn(a.act_noise * (valid ? a.noise[er * C::AOUT + j] : 0.f), lim);
            act = fminf(fmaxf(act, -1.1f * lim), 1.1f * lim);  // ddpg_acm.py:43-45
          }
          if (a.denorm_out && !a.plain) act = denorm<true>(p, L.tbl, j, act);
          L.pl[j0 * 32] = act;
          if (valid) a.target_out[er * C::AOUT + j] = act;
          if (valid && a.plain) a.env_out[er * C::AOUT + j] = act;  // process_action: identity (ddpg.py:371-384)
        }
      }
    if (a.plain) continue;
    // env action = ACM(cat(obs, a))  (off_policy.py:89-106)
    f32x16 xin[C::NB_ACMIN];
    load_cat_gl<C::NB_OB, C::NB_AOUT>(xin, a.obs, a.E * C::OB * 4, C::OB, L.ld4, L.vo, big, C::AOUT);
    acm_forward<C, false>(p, xin, L, nullptr, nullptr, nullptr);
    if (L.h == 0 && valid)
      for (int u = 0; u < C::AC; ++u) a.env_out[er * C::AC + u] = small[u * 32 + L.s];
  }
}

// ============================================================================ ACM regression
// acm.py:246-258: forward + MSE backward; writes the dW operands feature-major.
struct AcmRegArgs {
  int B, Bp;
  const float *x, *y;                   // row-major [B][2ob], [B][ac]
  float *XT, *Z1, *Z2, *P1, *P2, *P3;  // feature-major [.][Bp]
  float* part;                          // [ntiles]
};

template <class C>
__global__ __launch_bounds__(256, 1) void k_acm_regress(SacArgs p, AcmRegArgs g) {
  __shared__ float smem[kWavesPerWG * kLdsPerWave];
  __shared__ __attribute__((aligned(16))) float tbl[kTabMax];
  load_table(p, tbl);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* big = smem + w * kLdsPerWave;
  float* small = big + kSmallRow * 32;
  const int ntiles = g.Bp / 32;
  const int ld = g.Bp;
  constexpr int IN = 2 * C::OB;
  constexpr int NB_IN = blocks_of(IN);
  constexpr uint64_t RV_IN = rv_nat(IN, NB_IN);
  for (int tile = blockIdx.x * kWavesPerWG + w; tile < ntiles; tile += gridDim.x * kWavesPerWG) {
    const Lane L = make_lane(big, small, tbl, ld, tile * 32 + (lane & 31));
    const int b = L.b;
    const bool valid = b < g.B;
    const int br = valid ? b : 0;
    f32x16 xin[NB_IN];
#pragma unroll
    for (int ib = 0; ib < NB_IN; ++ib)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ur = 32 * ib + ru(r);
        const int u = ur + L.h4;
        xin[ib][r] = (u < IN && valid) ? g.x[br * IN + u] : 0.f;
      }
    // stores after all loads (a buffer store orders every later load behind it)
#pragma unroll
    for (int ib = 0; ib < NB_IN; ++ib)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ur = 32 * ib + ru(r);
        if (ur + L.h4 < IN) fm_st(rsrc(g.XT), ur, L.ld4, L.vo, xin[ib][r]);
      }
    dense<NB_IN, RV_IN, C::BF>(p.acm.W1, 2, xin, tbl + p.acm.tb1, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ur = 32 * ob + ru(q);
        const float v = tanhf(acc[q]);
        L.sl[ur * 32] = v;
        fm_st(rsrc(g.Z1), ur, L.ld4, L.vo, v);
      }
    });
    f32x16 z1[2];
    lds_load<2>(z1, small);
    dense<2, C::RV_Z1, C::BF>(p.acm.W2, 1, z1, tbl + p.acm.tb2, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const float v = tanhf(acc[q]);
        L.sl[ru(q) * 32] = v;
        fm_st(rsrc(g.Z2), ru(q), L.ld4, L.vo, v);
      }
    });
    f32x16 z2[1];
    lds_load<1>(z2, small);
    float lsum = 0.f;
    f32x16 p3[1];
    const float sc = 2.f / ((float)g.B * (float)C::AC);
    float limv[16], yv[16];  // requested before the layer (see above)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int u = ru(q) + L.h4;
      const int uu = u < C::AC ? u : 0;
      limv[q] = acm_lim<true>(p, L.tbl, uu);
      yv[q] = g.y[br * C::AC + uu];
    }
    dense<1, C::RV_Z2, C::BF>(p.acm.W3, 1, z2, tbl + p.acm.tb3, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int u = ru(q) + L.h4;
        float v = 0.f;
        if (u < C::AC && valid) {
          const float t = tanhf(acc[q]);
          const float lim = limv[q];
          const float df = fsub_rn(fmul_rn(t, lim), yv[q]);
          lsum += df * df;
          v = sc * df * lim * (1.f - t * t);
        }
        p3[0][q] = v;
        if (u < C::AC) fm_st(rsrc(g.P3), ru(q), L.ld4, L.vo, v);
      }
    });
    dense<1, C::RV_AC, C::BF>(p.acm.W3T, 1, p3, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const float zz = z2[0][q];
        const float v = acc[q] * (1.f - zz * zz);
        L.sl[ru(q) * 32] = v;
        fm_st(rsrc(g.P2), ru(q), L.ld4, L.vo, v);
      }
    });
    f32x16 p2[1];
    lds_load<1>(p2, small);
    dense<1, C::RV_Z2, C::BF>(p.acm.W2T, 2, p2, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ur = 32 * ob + ru(q);
        const float zz = ob == 0 ? z1[0][q] : z1[1][q];
        fm_st(rsrc(g.P1), ur, L.ld4, L.vo, acc[q] * (1.f - zz * zz));
      }
    });
    const float ls = wave_sum(lsum);
    if (lane == 0) g.part[tile] = ls;
  }
}

#ifndef SPP_KSET_TU  // non-template kernels live in the api.hip translation unit only
// ============================================================================ staging
// Row-major caller batch (sample_batch layout) -> feature-major padded scratch.
struct StageArgs {
  int B, Bp, ob, aout, ac;
  const float *obs, *next_obs, *act, *rew, *acm;
  const int8_t* done;
  const float *eps1, *eps2;  // [B][aout] or NULL
  float *S, *S2, *ACT, *AENV, *R, *DN, *EPS1, *EPS2;
};
__global__ void k_stage_batch(StageArgs a) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.Bp) return;
  const bool v = b < a.B;
  const int64_t ld = a.Bp;
  for (int f = 0; f < a.ob; ++f) {
    a.S[f * ld + b] = v ? a.obs[b * a.ob + f] : 0.f;
    a.S2[f * ld + b] = v ? a.next_obs[b * a.ob + f] : 0.f;
  }
  for (int f = 0; f < a.aout; ++f) {
    if (a.act) a.ACT[f * ld + b] = v ? a.act[b * a.aout + f] : 0.f;
    if (a.eps1) a.EPS1[f * ld + b] = v ? a.eps1[b * a.aout + f] : 0.f;
    if (a.eps2) a.EPS2[f * ld + b] = v ? a.eps2[b * a.aout + f] : 0.f;
  }
  for (int f = 0; f < a.ac; ++f) a.AENV[f * ld + b] = v ? a.acm[b * a.ac + f] : 0.f;
  a.R[b] = v ? a.rew[b] : 0.f;
  a.DN[b] = v ? (float)a.done[b] : 0.f;
}

// Caller eps [B][aout] -> feature-major [aout][Bp] (zero padded).
__global__ void k_eps_copy_fm(const float* eps, float* E, int aout, int B, int Bp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)aout * Bp) return;
  const int64_t j = i / Bp, b = i % Bp;
  E[i] = b < B ? eps[b * aout + j] : 0.f;
}

// Feature-major [aout][Bp] -> row-major [B][aout] (read-back of the staged eps).
__global__ void k_eps_read_fm(const float* E, float* eps, int aout, int B, int Bp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)aout * B) return;
  const int64_t b = i / aout, j = i % aout;
  eps[i] = E[j * Bp + b];
}

// Device-side Gaussian eps straight into the feature-major layout (zero padded).
// Box-Muller with the hardware transcendentals (v_log_f32, v_sqrt_f32, v_sin/cos_f32 of 2 pi v in
// revolutions): the policy noise needs the N(0, 1) law, not libm-exact values.
__device__ __forceinline__ void box_muller_hw(uint32_t a, uint32_t b, float& n0, float& n1) {
  const float u = u01(a), v = u01(b);
  const float r = __builtin_amdgcn_sqrtf(-2.f * 0.69314718055994531f * __builtin_amdgcn_logf(u));
  n0 = r * __builtin_amdgcn_cosf(v);
  n1 = r * __builtin_amdgcn_sinf(v);
}
// eps [aout][Bp] (padding columns b >= B zero): one philox block -> 4 normals -> one 16-B store
// (Bp is a multiple of 32, so a quad never crosses a row).
__global__ void k_eps_fm(float* E, int aout, int B, int Bp, uint64_t seed, uint64_t ctr, float* E2, uint64_t ctr2) {
  if (blockIdx.y) {  // (a second array in the same launch: the update's two rsample draws)
    E = E2;
    ctr = ctr2;
  }
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // quad index; aout * Bp < 2^31 (host check)
  if (4 * i >= aout * Bp) return;
  const u32x4 r = philox(seed, ctr, (uint64_t)i);
  float4 v;
  box_muller_hw(r.x, r.y, v.x, v.y);
  box_muller_hw(r.z, r.w, v.z, v.w);
  const int col = (4 * i) % Bp;
  v.x = col < B ? v.x : 0.f;
  v.y = col + 1 < B ? v.y : 0.f;
  v.z = col + 2 < B ? v.z : 0.f;
  v.w = col + 3 < B ? v.w : 0.f;
  *reinterpret_cast<float4*>(E + 4 * (int64_t)i) = v;
}

#endif  // SPP_KSET_TU

// ============================================================================ debug dense
// One layer on a [B][K] row-major batch with a natural bias b (NULL -> 0).
// K <= 224: register-input dense (ob-major image); K == 256: dense_lds from the
// LDS image (ib-major image), NBO compile-time.  KQ > 0 (NBI == 1): only the first
// KQ register quads of the input block carry units, as in the 3..24-wide first layers.
template <int NBI, int NBO, int KQ = 0>
__global__ __launch_bounds__(64) void k_debug_dense(const float4* Wf, const float* bias, const float* x, float* y,
                                                    int B, int K, int N, int act) {
  __shared__ float img[256 * 32];
  __shared__ __attribute__((aligned(16))) float tb[256];
  const int lane = threadIdx.x & 63, h = lane >> 5, s = lane & 31;
  for (int i = lane; i < 256; i += 64) tb[i] = (bias && i < N) ? bias[i] : 0.f;
  const int64_t b = (int64_t)blockIdx.x * 32 + s;
  f32x16 in[NBI];
#pragma unroll
  for (int ib = 0; ib < NBI; ++ib)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int u = 32 * ib + unit_of(r, h);
      in[ib][r] = (u < K && b < B) ? x[b * K + u] : 0.f;
      img[(32 * ib + ru(r) + 4 * h) * 32 + s] = in[ib][r];
    }
  __syncthreads();
  auto epi = [&](int ob, const f32x16& acc) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int u = 32 * ob + unit_of(q, h);
      float v = acc[q];
      if (act == 1) v = fmaxf(v, 0.f);
      if (act == 2) v = tanhf(v);
      if (u < N && b < B) y[b * N + u] = v;
    }
  };
  if constexpr (NBI == 8)
    dense_lds<NBO>(Wf, img, tb, epi);  // tb holds zeros without a bias
  else
    dense<NBI, KQ ? (uint64_t)KQ : rv_nat(32 * NBI, NBI)>(Wf, (N + 31) / 32, in, tb, epi);
}

}  // namespace spp
