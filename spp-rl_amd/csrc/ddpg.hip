// DDPG_AcM per-sample kernels (gfx950), same tile machinery as sac.hip.
//
//  k_ddpg_critic_phase  rltoolkit/acm/off_policy/ddpg_acm.py:100-123 (targets through the
//                       target actor, the frozen BasicAcM and the target critic) and :174-185
//                       (critic forward + MSE backward) -> critic weight-gradient operands
//  k_ddpg_actor_phase   ddpg_acm.py:125-145 + :187-196 (-Q(s, ACM(s, denorm mu(s))) + c*MSE,
//                       backward through the updated critic, the BasicAcM and the actor)
//  k_bacm_regress       AcMTrainer.batch_update (rltoolkit/acm/acm.py:246-258) for BasicAcM
//
// BasicAcM image rows (per-wave LDS image): h (fc1, 100 units) at rows 128..227 then
// h1 (50 units) at rows 128..191; the output c goes to the SMALL rows 192.. .
#pragma once
#include "sac.hip"

namespace spp {

template <int OB_, int AOUT_, int AC_, bool ACMC_>
struct DCfg : Cfg<OB_, AOUT_, AC_, ACMC_> {
  using Base = Cfg<OB_, AOUT_, AC_, ACMC_>;
  static constexpr uint64_t RV_AOUT = rv_nat(AOUT_, Base::NB_AOUT);
  static constexpr uint64_t RV_B100 = rv_nat(100, 4);
  static constexpr uint64_t RV_B50 = rv_nat(50, 2);
};
constexpr int kBacmRow = 128;

// Feature-major scratch of the BasicAcM activations kept for its backward.
struct BAcmScratch {
  float *H, *H1, *R3;  // tanh(fc1) [100], tanh(fc2 + t fc21) [50], tanh(fc3) [ac]
};

// BasicAcM forward (basic_acm.py:23-27) on the input tile [s | a] -> c into SMALL rows [0, AC).
template <class C, bool ST>
__device__ __forceinline__ void bacm_forward(const SacArgs& p, const f32x16 (&xin)[C::NB_ACMIN], const Lane& L,
                                             const BAcmScratch& z) {
  const BAcmDev& B = p.bacm;
  float* bimg = L.img + kBacmRow * 32;
  float* bl = L.bl + kBacmRow * 32;
  const float t = *B.t;
  // fc21(x) (with bias), kept in registers for the sum with fc2(h)
  f32x16 s21[2];
  dense<C::NB_ACMIN, C::RV_ACMIN>(B.W21, 2, xin, L.tbl + B.tb21, [&](int ob, const f32x16& acc) {
    if (ob == 0) s21[0] = acc;
    else s21[1] = acc;
  });
  const rsrc_t hr = rsrc(z.H), h1r = rsrc(z.H1), r3r = rsrc(z.R3);
  dense<C::NB_ACMIN, C::RV_ACMIN>(B.W1, 4, xin, L.tbl + B.tb1, [&](int ob, const f32x16& acc) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ur = 32 * ob + ru(q);
      const float v = tanhf(acc[q]);
      bl[ur * 32] = v;
      if constexpr (ST) fm_st(hr, ur, L.ld4, L.vo, v);
    }
  });
  f32x16 hin[4];
  lds_load<4>(hin, bimg);
  dense<4, C::RV_B100>(B.W2, 2, hin, L.tbl + B.tb2, [&](int ob, const f32x16& acc) {
    const f32x16 sk = ob == 0 ? s21[0] : s21[1];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ur = 32 * ob + ru(q);
      const float v = tanhf(fadd_rn(acc[q], fmul_rn(t, sk[q])));  // fc2(h) + t * fc21(x)
      bl[ur * 32] = v;
      if constexpr (ST) fm_st(h1r, ur, L.ld4, L.vo, v);
    }
  });
  f32x16 h1in[2];
  lds_load<2>(h1in, bimg);
  dense<2, C::RV_B50>(B.W3, 1, h1in, L.tbl + B.tb3, [&](int ob, const f32x16& acc) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int u = ru(q) + L.h4;
      if (u < C::AC) {
        const float r = tanhf(acc[q]);
        L.sl[ru(q) * 32] = fmul_rn(r, B.t1[u]);
        if constexpr (ST) fm_st(r3r, ru(q), L.ld4, L.vo, r);
      }
    }
  });
}

// BasicAcM backward from dc (natural tile, units < AC) to d a (the action part of
// its input, units < AOUT), written to BIG rows [0, AOUT).
template <class C>
__device__ __forceinline__ void bacm_backward(const SacArgs& p, const f32x16& dc, const Lane& L,
                                              const BAcmScratch& z) {
  const BAcmDev& B = p.bacm;
  float* bimg = L.img + kBacmRow * 32;
  float* bl = L.bl + kBacmRow * 32;
  const float t = *B.t;
  const rsrc_t hr = rsrc(z.H), h1r = rsrc(z.H1), r3r = rsrc_n(z.R3, C::AC * L.ld4);
  // All scratch values requested up front: a buffer load issued inside an epilogue is ordered
  // behind the epilogue's stores (no alias proof against LDS), i.e. one round trip per element.
  float r3v[16], t1v[16], h1v[2][16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int u = ru(q) + L.h4;
    r3v[q] = fm_ldb(r3r, ru(q), L.ld4, L.vo);  // rows >= AC read 0
    t1v[q] = B.t1[u < C::AC ? u : 0];
  }
#pragma unroll
  for (int ob = 0; ob < 2; ++ob)
#pragma unroll
    for (int q = 0; q < 16; ++q) h1v[ob][q] = fm_ld(h1r, 32 * ob + ru(q), L.ld4, L.vo);
  f32x16 du3[1];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int u = ru(q) + L.h4;
    const float r = r3v[q];
    du3[0][q] = u < C::AC ? dc[q] * t1v[q] * (1.f - r * r) : 0.f;
  }
  // dz = (W3^T du3) * (1 - h1^2) -> BasicAcM rows
  dense<1, C::RV_AC>(B.W3T, 2, du3, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float h1 = ob ? h1v[1][q] : h1v[0][q];
      bl[(32 * ob + ru(q)) * 32] = acc[q] * (1.f - h1 * h1);
    }
  });
  float hv[4][16];
#pragma unroll
  for (int ob = 0; ob < 4; ++ob)
#pragma unroll
    for (int q = 0; q < 16; ++q) hv[ob][q] = fm_ld(hr, 32 * ob + ru(q), L.ld4, L.vo);
  f32x16 dz[2];
  lds_load<2>(dz, bimg);
  // du1 = (W2^T dz) * (1 - h^2) -> BIG rows [0, 128)
  dense<2, C::RV_B50>(B.W2T, 4, dz, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float h = ob == 0 ? hv[0][q] : (ob == 1 ? hv[1][q] : (ob == 2 ? hv[2][q] : hv[3][q]));
      L.bl[(32 * ob + ru(q)) * 32] = acc[q] * (1.f - h * h);
    }
  });
  f32x16 du1[4];
  lds_load<4>(du1, L.img);
  // d a = W1a^T du1 + t * W21a^T dz  (the two uses of x in basic_acm.py:25-26)
  f32x16 da[C::NB_AOUT];
#pragma unroll
  for (int ib = 0; ib < C::NB_AOUT; ++ib) da[ib] = zero16();
  dense<4, C::RV_B100>(B.W1Ta, C::NB_AOUT, du1, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
    for (int ib = 0; ib < C::NB_AOUT; ++ib)
      if (ib == ob) da[ib] = acc;
  });
  dense<2, C::RV_B50>(B.W21Ta, C::NB_AOUT, dz, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
    for (int ib = 0; ib < C::NB_AOUT; ++ib)
      if (ib == ob)
#pragma unroll
        for (int q = 0; q < 16; ++q) da[ib][q] += t * acc[q];
  });
#pragma unroll
  for (int ib = 0; ib < C::NB_AOUT; ++ib)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ur = 32 * ib + ru(q);
      if (ur + L.h4 < C::AOUT) L.bl[ur * 32] = da[ib][q];
    }
}

// Deterministic actor head (ddpg/models.py:17-22): a = tanh(fc3) * lim, a_d = denormalize(a)
// (natural tile of the fc3 pre-activation in BIG rows [0, AOUT)); a_d overwrites those rows.
template <class C, bool BRF = false>
__device__ __forceinline__ void ddpg_head(const SacArgs& p, const Lane& L, f32x16 (&u)[C::NB_AOUT]) {
  lds_load<C::NB_AOUT>(u, L.img);
#pragma unroll
  for (int ib = 0; ib < C::NB_AOUT; ++ib)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ur = 32 * ib + ru(q), j = ur + L.h4;
      const bool ok = j < C::AOUT;
      if (BRF || ok) {  // BRF: no per-unit branch around the table loads (one round trip each)
        const int jj = ok ? j : 0;
        const float ad = denorm<true>(p, L.tbl, jj, fmul_rn(tanhf(u[ib][q]), actor_lim<true>(p, L.tbl, jj)));
        if (ok) L.bl[ur * 32] = ad;
      }
    }
}

// ============================================================================ critic phase
template <class C>
__global__ __launch_bounds__(256, 1) void k_ddpg_critic_phase(SacArgs p, BAcmScratch z) {
  __shared__ float smem[kWavesPerWG * kLdsPerWave];
  __shared__ __attribute__((aligned(16))) float tbl[kTabMax];
  __shared__ float s_dq[kWavesPerWG][32];  // the tile's d loss / dq, for the fused fc3 weight gradient
  // this wave's fused fc3 gradient partials [256 | bias], in LDS.  Narrow observations only: in the 111-dim
  // ACM instantiation the fused loop spills VGPRs to scratch, so that one keeps the (DQ, H2) k_dw job.
  constexpr bool kFuse3 = C::OB <= 32;
  __shared__ float s_w3[kWavesPerWG][257];
  load_table(p, tbl);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* big = smem + w * kLdsPerWave;
  float* small = big + kSmallRow * 32;
  const int ntiles = p.Bp / 32;
#pragma unroll
  for (int k = 0; k < 4; ++k) s_w3[w][lane + 64 * k] = 0.f;
  if (lane == 0) s_w3[w][256] = 0.f;
  for (int tile = blockIdx.x * kWavesPerWG + w; tile < ntiles; tile += gridDim.x * kWavesPerWG) {
    const Lane L = make_lane(big, small, tbl, p.Bp, tile * 32 + (lane & 31));
    const int b = L.b;
    const bool valid = b < p.B;
    uint64_t d0 = 0, d1 = 0, d2 = 0, d3 = 0;
    // ---- a' = mu_targ(s'), a'_d = denormalize(a')   (ddpg_acm.py:114-115)
    actor_trunk<C, false, C::NB_AOUT, C::AOUT>(p.actor_targ, p.S2, C::OB * L.ld4, L, nullptr, nullptr, d0, d1, d2, d3);
    {
      f32x16 u[C::NB_AOUT];
      ddpg_head<C, true>(p, L, u);
    }
    // ---- critic-target input [s' | ACM(s', a'_d)] or [s' | a'_d]   (:116-118)
    f32x16 tin[C::NB_CIN];
    if constexpr (C::ACMC) {
      f32x16 xin[C::NB_ACMIN];
      load_cat_gl<C::NB_OB, C::NB_AOUT>(xin, p.S2, C::OB * L.ld4, C::OB, L.ld4, L.vo, big, C::AOUT);
      bacm_forward<C, false>(p, xin, L, z);
      load_cat_gl<C::NB_OB, C::NB_CA>(tin, p.S2, C::OB * L.ld4, C::OB, L.ld4, L.vo, small, C::AC);
    } else {
      load_cat_gl<C::NB_OB, C::NB_CA>(tin, p.S2, C::OB * L.ld4, C::OB, L.ld4, L.vo, big, C::AOUT);
    }
    // ---- y = r + gamma (1 - d) Q_targ   (:119-121)
    const float qt = critic_forward<C, false>(p.targ[0], tin, L, nullptr, nullptr, d0, d1, d2, d3);
    const float notdone = 1.f - p.DN[b];
    const float y = fadd_rn(p.R[b], fmul_rn(fmul_rn(p.gamma, notdone), qt));
    // ---- critic forward, MSE grad, backward to the weight-gradient operands (:174-185)
    uint64_t m1lo = 0, m1hi = 0, m2lo = 0, m2hi = 0;
    f32x16 xin[C::NB_CIN];
    load_cat_gg<C::NB_OB, C::NB_CA>(xin, p.S, C::OB, C::ACMC ? p.AENV : p.ACT, C::CA, L.ld4, L.vo);
    const CriticDev& Q = p.critic[0];
    const float q = critic_forward<C, true, 30, kFuse3>(Q, xin, L, p.H1[0], p.H2[0], m1lo, m1hi, m2lo, m2hi);
    const float diff = fsub_rn(q, y);
    const float dq = valid ? fmul_rn(2.f * diff, p.inv_B) : 0.f;
    const float lq = (valid && L.h == 0) ? diff * diff : 0.f;
    if constexpr (kFuse3) {
      // fc3's weight gradient, fused as in k_sac_critic_phase (h2 in the image; per-wave partials)
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
        s_w3[w][u] += acc;  // (each lane owns its units)
      }
      const float dsum = wave_sum(L.h == 0 ? dq : 0.f);
      if (lane == 0) s_w3[w][256] += dsum;
      SPP_XLANE_SYNC();  // the image rows are rewritten by the delta2 staging below
    } else if (L.h == 0) {
      p.DQ[0][b] = dq;  // the fc3 job of k_dw reads (DQ, H2)
    }
    const rsrc_t d2r = rsrc(p.D2[0]);
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
        fm_st(d2r, ur, L.ld4, L.vo, v);
      }
    }
    const rsrc_t d1r = rsrc(p.D1[0]);
    dense_lds<8>(Q.W2T, big, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q2 = 0; q2 < 16; ++q2)
        fm_st(d1r, 32 * ob + ru(q2), L.ld4, L.vo, getbit(m1lo, m1hi, ob, q2) ? acc[q2] : 0.f);
    });
    const float s0 = wave_sum(lq);
    if (lane == 0) p.part[tile * kParts + 0] = s0;
  }
  if constexpr (kFuse3) {  // this wave's fc3 partials [256 weights | bias]
    float* o0 = p.W3P[0] + ((int64_t)blockIdx.x * kWavesPerWG + w) * p.w3p_stride;
#pragma unroll
    for (int k = 0; k < 4; ++k) o0[lane + 64 * k] = s_w3[w][lane + 64 * k];
    if (lane == 0) o0[256] = s_w3[w][256];
  }
}

// ============================================================================ actor phase
template <class C>
__global__ __launch_bounds__(256, 1) void k_ddpg_actor_phase(SacArgs p, BAcmScratch z) {
  __shared__ float smem[kWavesPerWG * kLdsPerWave];
  __shared__ __attribute__((aligned(16))) float tbl[kTabMax];
  load_table(p, tbl);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* big = smem + w * kLdsPerWave;
  float* small = big + kSmallRow * 32;
  const int ntiles = p.Bp / 32;
  for (int tile = blockIdx.x * kWavesPerWG + w; tile < ntiles; tile += gridDim.x * kWavesPerWG) {
    const Lane L = make_lane(big, small, tbl, p.Bp, tile * 32 + (lane & 31));
    const int b = L.b;
    const bool valid = b < p.B;
    // ---- a = mu(s), a_d   (ddpg_acm.py:126-127)
    uint64_t a1lo = 0, a1hi = 0, a2lo = 0, a2hi = 0;
    actor_trunk<C, true, C::NB_AOUT, C::AOUT>(p.actor, p.S, C::OB * L.ld4, L, p.AH1, p.AH2, a1lo, a1hi, a2lo, a2hi);
    f32x16 u[C::NB_AOUT];
    ddpg_head<C>(p, L, u);
    // Wide heads (Ant): park the fc3 pre-activation in the ADH rows the heads backward overwrites
    // (same lane, same element) instead of keeping NB_AOUT tiles live through the critic section.
    constexpr bool kParkHeads = C::NB_AOUT > 2;
    const rsrc_t adhr = rsrc(p.ADH);
    if constexpr (kParkHeads) {
#pragma unroll
      for (int ib = 0; ib < C::NB_AOUT; ++ib)
#pragma unroll
        for (int q2 = 0; q2 < 16; ++q2) {
          const int ur = 32 * ib + ru(q2);
          if (ur + L.h4 < C::AOUT) fm_st(adhr, ur, L.ld4, L.vo, u[ib][q2]);
        }
    }
    // ---- critic input [s | ACM(s, a_d)] or [s | a_d]   (:128-132)
    f32x16 cin[C::NB_CIN];
    if constexpr (C::ACMC) {
      f32x16 xin[C::NB_ACMIN];
      load_cat_gl<C::NB_OB, C::NB_AOUT>(xin, p.S, C::OB * L.ld4, C::OB, L.ld4, L.vo, big, C::AOUT);
      bacm_forward<C, true>(p, xin, L, z);
      load_cat_gl<C::NB_OB, C::NB_CA>(cin, p.S, C::OB * L.ld4, C::OB, L.ld4, L.vo, small, C::AC);
    } else {
      load_cat_gl<C::NB_OB, C::NB_CA>(cin, p.S, C::OB * L.ld4, C::OB, L.ld4, L.vo, big, C::AOUT);
    }
    // ---- loss = -Q(s, c).mean()   (:133)
    uint64_t k0 = 0, k1 = 0, k2 = 0, k3 = 0;
    const CriticDev& Q = p.critic[0];
    const float q = critic_forward<C, false>(Q, cin, L, nullptr, nullptr, k0, k1, k2, k3);
    const float dqv = valid ? -p.inv_B : 0.f;
    // ---- back through the critic to its action input
    const float* w3 = tbl + Q.tw3;
#pragma unroll 1
    for (int ob = 0; ob < 8; ++ob) {
      float tv[16];
      tvals(w3, ob, L.h4, tv);
#pragma unroll
      for (int q2 = 0; q2 < 16; ++q2) L.bl[(32 * ob + ru(q2)) * 32] = getbit(k2, k3, ob, q2) ? dqv * tv[q2] : 0.f;
    }
    dense_lds<8>(Q.W2T, big, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q2 = 0; q2 < 16; ++q2) L.bl[(32 * ob + ru(q2)) * 32] = getbit(k0, k1, ob, q2) ? acc[q2] : 0.f;
    });
    f32x16 dca[C::NB_CA];
#pragma unroll
    for (int ib = 0; ib < C::NB_CA; ++ib) dca[ib] = zero16();
    dense_lds<C::NB_CA>(Q.W1Ta, big, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int ib = 0; ib < C::NB_CA; ++ib)
        if (ib == ob) dca[ib] = acc;
    });
    // ---- through the frozen ACM to d a_d (BIG rows [0, AOUT))
    if constexpr (C::ACMC) {
      bacm_backward<C>(p, dca[0], L, z);
    } else {
#pragma unroll
      for (int ib = 0; ib < C::NB_CA; ++ib)
#pragma unroll
        for (int q2 = 0; q2 < 16; ++q2) {
          const int ur = 32 * ib + ru(q2);
          if (ur + L.h4 < C::AOUT) L.bl[ur * 32] = dca[ib][q2];
        }
    }
    // ---- heads backward (tanh * lim, denormalize, custom loss; :134-143)
    float ddpg_part = (valid && L.h == 0) ? -q : 0.f;
    float dist_part = 0.f;
    const float cl_scale = valid ? p.custom_loss * 2.f * p.inv_B / (float)C::AOUT : 0.f;
    // Branch-free over the units, loads through array-bounded resources (rows >= AOUT read 0),
    // stores after the loop: per-unit branches or interleaved stores cost a round trip per unit.
    const rsrc_t s2r = rsrc_n(p.S2, C::OB * L.ld4);
    const bool closs = p.custom_loss != 0.f;
    if constexpr (kParkHeads) {
#pragma unroll
      for (int ib = 0; ib < C::NB_AOUT; ++ib)
#pragma unroll
        for (int q2 = 0; q2 < 16; ++q2) u[ib][q2] = fm_ld(adhr, 32 * ib + ru(q2), L.ld4, L.vo);
    }
#pragma unroll
    for (int ib = 0; ib < C::NB_AOUT; ++ib)
#pragma unroll
      for (int q2 = 0; q2 < 16; ++q2) {
        const int ur = 32 * ib + ru(q2), j = ur + L.h4;
        const bool ok = j < C::AOUT;
        const int jj = ok ? j : 0;
        const float s2 = closs ? fm_ldb(s2r, ur, L.ld4, L.vo) : 0.f;
        const float t = tanhf(u[ib][q2]);
        const float lim = actor_lim<true>(p, L.tbl, jj);
        const float a = fmul_rn(t, lim);
        float g_ad = L.bl[ur * 32];
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
        u[ib][q2] = ok ? g_a * lim * (1.f - t * t) : 0.f;
      }
#pragma unroll
    for (int ib = 0; ib < C::NB_AOUT; ++ib)
#pragma unroll
      for (int q2 = 0; q2 < 16; ++q2) {
        const int ur = 32 * ib + ru(q2);
        if (ur + L.h4 < C::AOUT) fm_st(adhr, ur, L.ld4, L.vo, u[ib][q2]);
      }
    // ---- dh2 = fc3^T du * relu'(h2); dh1 = W2^T dh2 * relu'(h1)
    const rsrc_t ad2r = rsrc(p.AD2), ad1r = rsrc(p.AD1);
    dense<C::NB_AOUT, C::RV_AOUT>(p.actor.WhT, 8, u, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q2 = 0; q2 < 16; ++q2) {
        const int ur = 32 * ob + ru(q2);
        const float v = getbit(a2lo, a2hi, ob, q2) ? acc[q2] : 0.f;
        L.bl[ur * 32] = v;
        fm_st(ad2r, ur, L.ld4, L.vo, v);
      }
    });
    dense_lds<8>(p.actor.W2T, big, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q2 = 0; q2 < 16; ++q2)
        fm_st(ad1r, 32 * ob + ru(q2), L.ld4, L.vo, getbit(a1lo, a1hi, ob, q2) ? acc[q2] : 0.f);
    });
    const float pq = wave_sum(ddpg_part);
    const float pd = wave_sum(dist_part);
    if (lane == 0) {
      p.part[tile * kParts + 2] = pq;
      p.part[tile * kParts + 3] = pd;
    }
  }
}

// ============================================================================ rollout action (DDPG)
// DDPG_AcM.noise_action (ddpg_acm.py:40-50) + process_action (off_policy.py:89-106):
// mode 1: a = clip(tanh(fc3)*lim + act_noise*lim*noise, +-1.1 lim); mode 2: deterministic;
// mode 0 random: a = lim * eps.  a_d = denormalize(a) if denorm_out; env action = ACM(s, a_d).
template <class C>
__global__ __launch_bounds__(256, 1) void k_ddpg_policy_act(SacArgs p, ActArgs a, BAcmScratch z) {
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
    Lane L = make_lane(big, small, tbl, 1, er * C::OB);
    f32x16 u[C::NB_AOUT];
    if (a.mode != 0) {
      uint64_t d0 = 0, d1 = 0, d2 = 0, d3 = 0;
      actor_trunk<C, false, C::NB_AOUT, C::AOUT>(p.actor, a.obs, a.E * C::OB * 4, L, nullptr, nullptr, d0, d1, d2,
                                                 d3);
      lds_load<C::NB_AOUT>(u, big);
    }
#pragma unroll
    for (int ib = 0; ib < C::NB_AOUT; ++ib)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ur = 32 * ib + ru(q), j = ur + L.h4;
        if (j < C::AOUT) {
          const float lim = actor_lim<true>(p, L.tbl, j);
          float act;
          if (a.mode == 0) {
            act = valid ? lim * a.eps[er * C::AOUT + j] : 0.f;
          } else {
            act = fmul_rn(tanhf(u[ib][q]), lim);
            if (a.mode == 1 && a.noise) act += fmul_rn(a.act_noise * (valid ? a.noise[er * C::AOUT + j] : 0.f), lim);
            act = fminf(fmaxf(act, -1.1f * lim), 1.1f * lim);
          }
          if (a.denorm_out) act = denorm<true>(p, L.tbl, j, act);
          L.bl[ur * 32] = act;
          if (valid) a.target_out[er * C::AOUT + j] = act;
        }
      }
    f32x16 xin[C::NB_ACMIN];
    load_cat_gl<C::NB_OB, C::NB_AOUT>(xin, a.obs, a.E * C::OB * 4, C::OB, L.ld4, L.vo, big, C::AOUT);
    bacm_forward<C, false>(p, xin, L, z);
    if (L.h == 0 && valid)
      for (int u2 = 0; u2 < C::AC; ++u2) a.env_out[er * C::AC + u2] = small[u2 * 32 + L.s];
  }
}

// ============================================================================ BasicAcM regression
// acm.py:246-258 with BasicAcM: MSE(ACM(x), y) forward + backward to the weight-gradient
// operands (incl. the t / t1 scale gradients, reduced per tile).
constexpr int kBParts = 16;  // per-tile partials: loss, dt, dt1[ac <= 14]
struct BAcmRegArgs {
  int B, Bp;
  const float *x, *y;                            // row-major [B][2ob], [B][ac]
  float *XT, *H, *H1, *S21, *P1, *PZ, *PZ21, *P3;  // feature-major [.][Bp]
  float* part;                                   // [ntiles][kBParts]
};

template <class C>
__global__ __launch_bounds__(256, 1) void k_bacm_regress(SacArgs p, BAcmRegArgs g) {
  static_assert(C::AC + 2 <= kBParts, "BasicAcM regression partials");
  __shared__ float smem[kWavesPerWG * kLdsPerWave];
  __shared__ __attribute__((aligned(16))) float tbl[kTabMax];
  load_table(p, tbl);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* big = smem + w * kLdsPerWave;
  float* small = big + kSmallRow * 32;
  const int ntiles = g.Bp / 32;
  constexpr int IN = 2 * C::OB;
  constexpr int NB_IN = blocks_of(IN);
  constexpr uint64_t RV_IN = rv_nat(IN, NB_IN);
  const BAcmDev& B = p.bacm;
  for (int tile = blockIdx.x * kWavesPerWG + w; tile < ntiles; tile += gridDim.x * kWavesPerWG) {
    const Lane L = make_lane(big, small, tbl, g.Bp, tile * 32 + (lane & 31));
    const int b = L.b;
    const bool valid = b < g.B;
    const int br = valid ? b : 0;
    const float t = *B.t;
    const rsrc_t xtr = rsrc(g.XT), hr = rsrc(g.H), h1r = rsrc(g.H1), s21r = rsrc(g.S21), p1r = rsrc(g.P1),
                 pzr = rsrc(g.PZ), pz21r = rsrc(g.PZ21), p3r = rsrc(g.P3);
    f32x16 xin[NB_IN];
#pragma unroll
    for (int ib = 0; ib < NB_IN; ++ib)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ur = 32 * ib + ru(r);
        const int u = ur + L.h4;
        xin[ib][r] = (u < IN && valid) ? g.x[br * IN + u] : 0.f;
      }
#pragma unroll
    for (int ib = 0; ib < NB_IN; ++ib)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ur = 32 * ib + ru(r);
        if (ur + L.h4 < IN) fm_st(xtr, ur, L.ld4, L.vo, xin[ib][r]);
      }
    float* bl = L.bl + kBacmRow * 32;
    float* bimg = big + kBacmRow * 32;
    f32x16 s21[2];
    dense<NB_IN, RV_IN>(B.W21, 2, xin, tbl + B.tb21, [&](int ob, const f32x16& acc) {
      if (ob == 0) s21[0] = acc;
      else s21[1] = acc;
#pragma unroll
      for (int q = 0; q < 16; ++q) fm_st(s21r, 32 * ob + ru(q), L.ld4, L.vo, acc[q]);
    });
    dense<NB_IN, RV_IN>(B.W1, 4, xin, tbl + B.tb1, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ur = 32 * ob + ru(q);
        const float v = tanhf(acc[q]);
        bl[ur * 32] = v;
        fm_st(hr, ur, L.ld4, L.vo, v);
      }
    });
    f32x16 hin[4];
    lds_load<4>(hin, bimg);
    f32x16 h1t[2];
    dense<4, C::RV_B100>(B.W2, 2, hin, tbl + B.tb2, [&](int ob, const f32x16& acc) {
      const f32x16 sk = ob == 0 ? s21[0] : s21[1];
      f32x16 v;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        v[q] = tanhf(fadd_rn(acc[q], fmul_rn(t, sk[q])));
        bl[(32 * ob + ru(q)) * 32] = v[q];
        fm_st(h1r, 32 * ob + ru(q), L.ld4, L.vo, v[q]);
      }
      if (ob == 0) h1t[0] = v;
      else h1t[1] = v;
    });
    f32x16 h1in[2];
    lds_load<2>(h1in, bimg);
    float lsum = 0.f;
    float dt1[C::AC];
#pragma unroll
    for (int k = 0; k < C::AC; ++k) dt1[k] = 0.f;
    f32x16 p3[1];
    const float sc = 2.f / ((float)g.B * (float)C::AC);
    float t1v[16], yv[16];  // before the layer (loads behind the epilogue's stores serialise)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int u = ru(q) + L.h4;
      const int uu = u < C::AC ? u : 0;
      t1v[q] = B.t1[uu];
      yv[q] = g.y[br * C::AC + uu];
    }
    dense<2, C::RV_B50>(B.W3, 1, h1in, tbl + B.tb3, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int u = ru(q) + L.h4;
        float v = 0.f;
        if (u < C::AC && valid) {
          const float r = tanhf(acc[q]);
          const float t1 = t1v[q];
          const float df = fsub_rn(fmul_rn(r, t1), yv[q]);
          lsum += df * df;
          const float dout = sc * df;
#pragma unroll
          for (int k = 0; k < C::AC; ++k)
            if (k == u) dt1[k] += dout * r;
          v = dout * t1 * (1.f - r * r);
        }
        p3[0][q] = v;
        if (u < C::AC) fm_st(p3r, ru(q), L.ld4, L.vo, v);
      }
    });
    // dz = (W3^T du3) * (1 - h1^2); dt = sum dz * fc21(x)
    float dts = 0.f;
    dense<1, C::RV_AC>(B.W3T, 2, p3, nullptr, [&](int ob, const f32x16& acc) {
      const f32x16 hv = ob == 0 ? h1t[0] : h1t[1];
      const f32x16 sk = ob == 0 ? s21[0] : s21[1];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ur = 32 * ob + ru(q);
        const float v = (ur + L.h4 < 50) ? acc[q] * (1.f - hv[q] * hv[q]) : 0.f;
        bl[ur * 32] = v;
        fm_st(pzr, ur, L.ld4, L.vo, v);
        fm_st(pz21r, ur, L.ld4, L.vo, fmul_rn(t, v));  // grad of fc21's output: t * dz
        dts += v * sk[q];
      }
    });
    f32x16 dz[2];
    lds_load<2>(dz, bimg);
    dense<2, C::RV_B50>(B.W2T, 4, dz, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ur = 32 * ob + ru(q);
        const float hh = ob == 0 ? hin[0][q] : (ob == 1 ? hin[1][q] : (ob == 2 ? hin[2][q] : hin[3][q]));
        fm_st(p1r, ur, L.ld4, L.vo, (ur + L.h4 < 100) ? acc[q] * (1.f - hh * hh) : 0.f);
      }
    });
    const float ls = wave_sum(lsum);
    const float dtt = wave_sum(dts);
    if (lane == 0) {
      g.part[tile * kBParts + 0] = ls;
      g.part[tile * kBParts + 1] = dtt;
    }
#pragma unroll
    for (int k = 0; k < C::AC; ++k) {
      const float s = wave_sum(dt1[k]);
      if (lane == 0) g.part[tile * kBParts + 2 + k] = s;
    }
  }
}

}  // namespace spp
