// Small-batch ("team") forms of the SAC phase kernels (gfx950), for batches of at most one 32-sample tile
// per CU (BASELINE.json configs[0]: vanilla SAC, B = 100, rltoolkit/algorithms/sac/sac.py:218-280).
//
// k_sac_critic_phase / k_sac_actor_phase give each 32-sample tile to ONE wave, which runs every layer of the
// phase as a serial chain of 32x32x2 f32 MFMAs; at B = 100 that is 4 waves on 4 SIMDs of one CU, and the
// phase is that chain's length (MFMA-bound: ~8 layer-equivalents x 1,024 MFMAs x 64 cycles).  Here a tile
// gets a workgroup: its 4 waves (one per SIMD) share the tile's LDS image, and each 256-wide layer is split
// by output blocks -- wave w computes blocks 2w, 2w+1 (units 64w .. 64w+63) -- with a workgroup barrier
// between a layer's last image read and its first image write, and another before the next layer reads.
// The per-sample work (squash, log-prob, targets, losses, the 1-block heads) is computed by every wave on
// the same values in the same order, so every wave holds the same scalars and the barrier sequence is
// uniform; HBM writes of replicated values are made by wave 0 only.  Each tile runs on its own CU, one tile
// per workgroup (grid = min(tiles, CUs), api.hip's sac_grid).
//
// Same math as the one-wave kernels (sac.hip); the summation order of the q reduction and of the fused fc3
// weight gradient differs (wave-partials in fixed order), so results agree within fp32 rounding, not bit
// for bit.  Vanilla-SAC shapes only (no ACM in the critic input, fp32, heads <= 2 pairing blocks).
#pragma once
#include "sac.hip"

namespace spp {

__device__ __forceinline__ void team_sync() { __syncthreads(); }

// This wave's NOW output blocks ob0 .. ob0+NOW-1 of a 256-input layer (input: the team's LDS image, all 8
// input blocks) whose ib-major image has NBT output blocks: Wf[((ib*NBT + ob)*4 + rq)*64 + lane].  Weight
// chunks stream one input block ahead.  The team synchronises after the MFMAs (every wave's image reads
// are done), then epi(ob, acc) may overwrite the image.
template <int NOW, int NBT, bool BIAS, typename Epi>
__device__ __forceinline__ void dense_lds_team(const float4* __restrict__ Wf, int ob0, const float* img,
                                               const float* biasL, Epi&& epi) {
  const int lane = lane_id();
  const int h = lane >> 5;
  const float* l = img + 4 * h * 32 + (lane & 31);
  const rsrc_t wr = rsrc(Wf);
  const uint32_t l16 = 16u * lane;
  f32x16 acc[NOW];
#pragma unroll
  for (int j = 0; j < NOW; ++j) {
    if constexpr (BIAS) acc[j] = bias_tile(biasL, ob0 + j, h);
    else acc[j] = zero16();
  }
  float4 cur[NOW][4];
  f32x16 x;
#pragma unroll
  for (int j = 0; j < NOW; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) cur[j][q] = wfrag(wr, l16, ((ob0 + j) * 4 + q) * 1024);
#pragma unroll
  for (int r = 0; r < 16; ++r) x[r] = l[ru(r) * 32];
#pragma unroll
  for (int ib = 0; ib < 8; ++ib) {
    float4 nxt[NOW][4];
    f32x16 xn;
    if (ib + 1 < 8) {
#pragma unroll
      for (int j = 0; j < NOW; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) nxt[j][q] = wfrag(wr, l16, (((ib + 1) * NBT + ob0 + j) * 4 + q) * 1024);
#pragma unroll
      for (int r = 0; r < 16; ++r) xn[r] = l[(32 * (ib + 1) + ru(r)) * 32];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < NOW; ++j) {
        acc[j] = mfma(cur[j][q].x, x[4 * q + 0], acc[j]);
        acc[j] = mfma(cur[j][q].y, x[4 * q + 1], acc[j]);
        acc[j] = mfma(cur[j][q].z, x[4 * q + 2], acc[j]);
        acc[j] = mfma(cur[j][q].w, x[4 * q + 3], acc[j]);
      }
    if (ib + 1 < 8) {
#pragma unroll
      for (int j = 0; j < NOW; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) cur[j][q] = nxt[j][q];
      x = xn;
    }
  }
  team_sync();
#pragma unroll
  for (int j = 0; j < NOW; ++j) epi(ob0 + j, acc[j]);
}

// This wave's 2 output blocks of a register-input layer with 8 output blocks (ob-major image, sac.hip's
// dense); the epilogue may write the image: the caller has synchronised after the team's last image read.
template <int NBI, uint64_t RV, typename Epi>
__device__ __forceinline__ void dense_team(const float4* __restrict__ Wf, int ob0, const f32x16 (&in)[NBI],
                                           const float* biasL, Epi&& epi) {
  dense<NBI, RV>(Wf + (size_t)ob0 * NBI * 4 * 64, 2, in, biasL + 32 * ob0,
                 [&](int j, const f32x16& acc) { epi(ob0 + j, acc); });
}
template <int NBI, uint64_t RV, typename Epi>
__device__ __forceinline__ void dense_team(const float4* __restrict__ Wf, int ob0, const f32x16 (&in)[NBI],
                                           decltype(nullptr), Epi&& epi) {
  dense<NBI, RV>(Wf + (size_t)ob0 * NBI * 4 * 64, 2, in, nullptr,
                 [&](int j, const f32x16& acc) { epi(ob0 + j, acc); });
}

// Actor trunk (sac.hip actor_trunk), team form: h1 / h2 split by blocks (masks of the wave's own blocks only),
// heads (one block) computed by every wave from the full h2 image and written to rows [0, 2*AOUT) by wave 0.
// Returns with the heads in the image, team-synchronised.
template <class C, bool ST>
__device__ __forceinline__ void actor_trunk_team(const ActorDev& A, const float* X, int xbytes, const Lane& L,
                                                 int w, float* H1g, float* H2g, uint64_t& m1lo, uint64_t& m1hi,
                                                 uint64_t& m2lo, uint64_t& m2hi) {
  static_assert(C::NB_H2 == 1, "team heads: one output block");
  const int ob0 = 2 * w;
  {
    f32x16 x[C::NB_OB];
    gm_load<C::NB_OB>(x, X, xbytes, C::OB, L.ld4, L.vo);
    const rsrc_t hr = rsrc(H1g);
    dense_team<C::NB_OB, C::RV_X>(A.W1, ob0, x, L.tbl + A.tb1, [&](int ob, const f32x16& acc) {
      uint32_t bits = 0;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ur = 32 * ob + ru(q);
        const float v = fmaxf(acc[q], 0.f);
        L.bl[ur * 32] = v;
        if constexpr (ST) fm_st_op(hr, ur, L.ld4, L.vo, v);
        bits |= (uint32_t)(v > 0.f) << q;
      }
      setbits(m1lo, m1hi, ob, bits);
    });
  }
  team_sync();
  {
    const rsrc_t hr = rsrc(H2g);
    dense_lds_team<2, 8, true>(A.W2, ob0, L.img, L.tbl + A.tb2, [&](int ob, const f32x16& acc) {
      uint32_t bits = 0;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ur = 32 * ob + ru(q);
        const float v = fmaxf(acc[q], 0.f);
        L.bl[ur * 32] = v;
        if constexpr (ST) fm_st_op(hr, ur, L.ld4, L.vo, v);
        bits |= (uint32_t)(v > 0.f) << q;
      }
      setbits(m2lo, m2hi, ob, bits);
    });
  }
  team_sync();
  dense_lds_team<1, 1, true>(A.Wh, 0, L.img, L.tbl + A.tbh, [&](int, const f32x16& acc) {
    if (w == 0) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ur = ru(q);
        if (ur + L.h4 < 2 * C::AOUT) L.bl[ur * 32] = acc[q];
      }
    }
  });
  team_sync();
}

// Critic forward through L2 (sac.hip critic_forward), team form: returns q (every wave the same value; the
// per-wave partials of w3 . relu(h2) summed in wave order through red).  H2L: h2 of the wave's own blocks
// goes to the image (the fused fc3 weight gradient reads it there).  Caller: the image is free to write.
template <class C, bool ST, bool H2L>
__device__ __forceinline__ float critic_forward_team(const CriticDev& Q, const f32x16 (&xin)[C::NB_CIN],
                                                     const Lane& L, int w, float* H1g, float* H2g,
                                                     float (*red)[64], uint64_t& m1lo, uint64_t& m1hi,
                                                     uint64_t& m2lo, uint64_t& m2hi) {
  const int ob0 = 2 * w;
  const rsrc_t h1r = rsrc(H1g), h2r = rsrc(H2g);
  dense_team<C::NB_CIN, C::RV_CIN>(Q.W1, ob0, xin, L.tbl + Q.tb1, [&](int ob, const f32x16& acc) {
    uint32_t bits = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ur = 32 * ob + ru(q);
      const float v = fmaxf(acc[q], 0.f);
      L.bl[ur * 32] = v;
      if constexpr (ST) fm_st_op(h1r, ur, L.ld4, L.vo, v);
      bits |= (uint32_t)(v > 0.f) << q;
    }
    setbits(m1lo, m1hi, ob, bits);
  });
  team_sync();
  float qp = 0.f;
  const float* w3 = L.tbl + Q.tw3;
  dense_lds_team<2, 8, true>(Q.W2, ob0, L.img, L.tbl + Q.tb2, [&](int ob, const f32x16& acc) {
    uint32_t bits = 0;
    float tv[16];
    tvals(w3, ob, L.h4, tv);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float v = fmaxf(acc[q], 0.f);
      if constexpr (H2L) L.bl[(32 * ob + ru(q)) * 32] = v;
      else if constexpr (ST) fm_st_op(h2r, 32 * ob + ru(q), L.ld4, L.vo, v);
      qp = fmaf(v, tv[q], qp);
      bits |= (uint32_t)(v > 0.f) << q;
    }
    setbits(m2lo, m2hi, ob, bits);
  });
  const int lane = lane_id();
  red[w][lane] = qp;
  team_sync();
  const float s = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
  return s + __shfl_xor(s, 32, 64) + *Q.b3;
}

// ============================================================================ critic phase, team form
template <class C>
__global__ __launch_bounds__(256, 1) void k_sac_critic_team(SacArgs p) {
  static_assert(!C::ACMC && !C::BF && C::F3 && C::NB_PAIR == 1, "team critic phase: vanilla fp32 shapes");
  __shared__ float img[kLdsPerWave];
  __shared__ __attribute__((aligned(16))) float tbl[kTabMax];
  __shared__ float red[kWavesPerWG][64];
  __shared__ float s_dq[kWavesPerWG][32];
  load_table(p, tbl);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int ob0 = 2 * w;
  const int ntiles = p.Bp / 32;
  const int ld = p.Bp;
  const float alpha = *p.alpha;
  float w3a = 0.f, w3b = 0.f, b3a = 0.f, b3b = 0.f;  // fused fc3 grads of unit 64w + lane (bias: wave 0)
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const Lane L = make_lane(img, img + kSmallRow * 32, tbl, ld, tile * 32 + (lane & 31));
    const int b = L.b;
    const bool valid = b < p.B;
    uint64_t d0 = 0, d1 = 0, d2 = 0, d3 = 0;
    // ---- target action a' ~ pi(s'), logpi'   (sac.py:230-236)
    actor_trunk_team<C, false>(p.actor, p.S2, C::OB * L.ld4, L, w, nullptr, nullptr, d0, d1, d2, d3);
    float lp2;
    {
      f32x16 hd[C::NB_PAIR];
      load_pair<C>(hd, img);
      team_sync();
      lp2 = squash_write<C, true>(p, hd, p.EPS1, L);  // every wave writes the same a'_d rows
    }
    team_sync();
    f32x16 tin[C::NB_CIN];
    load_cat_gl<C::NB_OB, C::NB_CA>(tin, p.S2, C::OB * L.ld4, C::OB, L.ld4, L.vo, img, C::AOUT);
    team_sync();
    // ---- soft-min twin target (sac.py:237-241)
    const float q1t = critic_forward_team<C, false, false>(p.targ[0], tin, L, w, nullptr, nullptr, red, d0, d1, d2, d3);
    const float q2t = critic_forward_team<C, false, false>(p.targ[1], tin, L, w, nullptr, nullptr, red, d0, d1, d2, d3);
    const float notdone = 1.f - p.DN[b];
    const float y = fadd_rn(p.R[b], fmul_rn(p.gamma * notdone, fsub_rn(fminf(q1t, q2t), alpha * lp2)));
    // ---- both critics: forward, MSE grad, backward to the weight-gradient operands (sac.py:243-252)
    float lq0 = 0.f, lq1 = 0.f;
#pragma unroll 1
    for (int i = 0; i < 2; ++i) {
      uint64_t m1lo = 0, m1hi = 0, m2lo = 0, m2hi = 0;
      f32x16 xin[C::NB_CIN];
      load_cat_gg<C::NB_OB, C::NB_CA>(xin, p.S, C::OB, p.ACT, C::CA, L.ld4, L.vo);
      const CriticDev& Q = p.critic[i];
      const float q = critic_forward_team<C, true, true>(Q, xin, L, w, p.H1[i], nullptr, red, m1lo, m1hi, m2lo, m2hi);
      const float diff = fsub_rn(q, y);
      const float dq = valid ? fmul_rn(2.f * diff, p.inv_B) : 0.f;
      const float lqi = (valid && L.h == 0) ? diff * diff : 0.f;
      if (i == 0) lq0 = lqi; else lq1 = lqi;
      // fc3 weight gradient of this wave's units (dW3 = dq . h2^T, db3 = sum dq): h2 rows 64w .. 64w+63 are
      // this wave's own image rows
      if (L.h == 0) s_dq[w][L.s] = dq;
      SPP_XLANE_SYNC();
      {
        const int u = 64 * w + lane;
        const float* row = img + u * 32;
        float acc = 0.f;
#pragma unroll 8
        for (int j = 0; j < 32; ++j) {
          const int s2 = (j + u) & 31;
          acc = fmaf(row[s2], s_dq[w][s2], acc);
        }
        if (i == 0) w3a += acc; else w3b += acc;
      }
      const float dsum = wave_sum(L.h == 0 ? dq : 0.f);
      if (i == 0) b3a += dsum; else b3b += dsum;
      SPP_XLANE_SYNC();  // own rows rewritten below
      // delta2 = dq * w3 * relu'(h2), own blocks, staged in the image and stored feature-major
      const rsrc_t d2r = rsrc(p.D2[i]);
      const float* w3 = tbl + Q.tw3;
#pragma unroll 1
      for (int k = 0; k < 2; ++k) {
        const int ob = ob0 + k;
        float tv[16];
        tvals(w3, ob, L.h4, tv);
#pragma unroll
        for (int q2 = 0; q2 < 16; ++q2) {
          const int ur = 32 * ob + ru(q2);
          const float v = getbit(m2lo, m2hi, ob, q2) ? dq * tv[q2] : 0.f;
          L.bl[ur * 32] = v;
          fm_st_op(d2r, ur, L.ld4, L.vo, v);
        }
      }
      team_sync();
      // delta1 = (W2^T delta2) * relu'(h1), own blocks
      const rsrc_t d1r = rsrc(p.D1[i]);
      dense_lds_team<2, 8, false>(Q.W2T, ob0, img, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
        for (int q2 = 0; q2 < 16; ++q2)
          fm_st_op(d1r, 32 * ob + ru(q2), L.ld4, L.vo, getbit(m1lo, m1hi, ob, q2) ? acc[q2] : 0.f);
      });
    }
    const float s0 = wave_sum(lq0), s1 = wave_sum(lq1);
    if (w == 0 && lane == 0) {
      p.part[tile * kParts + 0] = s0;
      p.part[tile * kParts + 1] = s1;
    }
  }
  // this wave's fc3 partials [256 weights | bias] per critic: unit 64w + lane, zeros elsewhere
  const int64_t wg = (int64_t)blockIdx.x * kWavesPerWG + w;
  float* o0 = p.W3P[0] + wg * p.w3p_stride;
  float* o1 = p.W3P[1] + wg * p.w3p_stride;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    o0[lane + 64 * k] = k == w ? w3a : 0.f;
    o1[lane + 64 * k] = k == w ? w3b : 0.f;
  }
  if (lane == 0) {
    o0[256] = w == 0 ? b3a : 0.f;
    o1[256] = w == 0 ? b3b : 0.f;
  }
}

// ============================================================================ actor phase, team form
template <class C>
__global__ __launch_bounds__(256, 1) void k_sac_actor_team(SacArgs p, AcmScratch) {
  static_assert(!C::ACMC && !C::BF && C::NB_PAIR == 1 && C::NB_CA == 1, "team actor phase: vanilla fp32 shapes");
  __shared__ float img[kLdsPerWave];
  __shared__ __attribute__((aligned(16))) float tbl[kTabMax];
  __shared__ float red[kWavesPerWG][64];
  load_table(p, tbl);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int ob0 = 2 * w;
  const int ntiles = p.Bp / 32;
  const int ld = p.Bp;
  const float alpha = *p.alpha;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const Lane L = make_lane(img, img + kSmallRow * 32, tbl, ld, tile * 32 + (lane & 31));
    const int b = L.b;
    const bool valid = b < p.B;
    const float g_lp = valid ? alpha * p.inv_B : 0.f;  // d loss / d logpi_b
    // ---- a, logpi = actor(s)  (sac.py:262-266)
    uint64_t a1lo = 0, a1hi = 0, a2lo = 0, a2hi = 0;
    actor_trunk_team<C, true>(p.actor, p.S, C::OB * L.ld4, L, w, p.AH1, p.AH2, a1lo, a1hi, a2lo, a2hi);
    f32x16 hd[C::NB_PAIR];
    load_pair<C>(hd, img);
    team_sync();
    const float lp = squash_write<C>(p, hd, p.EPS2, L);  // a_d -> image rows [0, AOUT), every wave the same
    team_sync();
    f32x16 cin[C::NB_CIN];
    load_cat_gl<C::NB_OB, C::NB_CA>(cin, p.S, C::OB * L.ld4, C::OB, L.ld4, L.vo, img, C::AOUT);
    team_sync();
    // ---- q = min(Q1, Q2)(s, a)  (sac.py:267-270), own-block masks kept for the backward
    uint64_t ma0 = 0, ma1 = 0, ma2 = 0, ma3 = 0, mb0 = 0, mb1 = 0, mb2 = 0, mb3 = 0;
    const float q1 = critic_forward_team<C, false, false>(p.critic[0], cin, L, w, nullptr, nullptr, red, ma0, ma1, ma2, ma3);
    const float q2 = critic_forward_team<C, false, false>(p.critic[1], cin, L, w, nullptr, nullptr, red, mb0, mb1, mb2, mb3);
    const float qmin = fminf(q1, q2);
    const float gq = valid ? -p.inv_B : 0.f;
    const float dqa = q1 < q2 ? gq : (q1 == q2 ? 0.5f * gq : 0.f);
    const float dqb = q2 < q1 ? gq : (q1 == q2 ? 0.5f * gq : 0.f);
    // ---- back through both critics to their action input
    f32x16 dca = zero16();
#pragma unroll 1
    for (int i = 0; i < 2; ++i) {
      const CriticDev& Q = p.critic[i];
      const uint64_t k0 = i ? mb0 : ma0, k1 = i ? mb1 : ma1, k2 = i ? mb2 : ma2, k3 = i ? mb3 : ma3;
      const float dqi = i ? dqb : dqa;
      const float* w3 = tbl + Q.tw3;
#pragma unroll 1
      for (int k = 0; k < 2; ++k) {
        const int ob = ob0 + k;
        float tv[16];
        tvals(w3, ob, L.h4, tv);
#pragma unroll
        for (int q = 0; q < 16; ++q) L.bl[(32 * ob + ru(q)) * 32] = getbit(k2, k3, ob, q) ? dqi * tv[q] : 0.f;
      }
      team_sync();
      dense_lds_team<2, 8, false>(Q.W2T, ob0, img, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
        for (int q = 0; q < 16; ++q) L.bl[(32 * ob + ru(q)) * 32] = getbit(k0, k1, ob, q) ? acc[q] : 0.f;
      });
      team_sync();
      dense_lds_team<1, 1, false>(Q.W1Ta, 0, img, nullptr, [&](int, const f32x16& acc) { dca += acc; });
    }
    // d loss / d a_d into image rows [0, AOUT) (the heads backward reads it in the pairing layout)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ur = ru(q);
      if (ur + L.h4 < C::AOUT) L.bl[ur * 32] = dca[q];
    }
    team_sync();
    // ---- heads backward in the pairing layout (squash, denorm, custom loss, logpi): sac.hip's actor phase
    float sac_part = (valid && L.h == 0) ? fsub_rn(alpha * lp, qmin) : 0.f;
    float dist_part = 0.f;
    const float cl_scale = valid ? p.custom_loss * 2.f * p.inv_B / (float)C::AOUT : 0.f;
    const int h8 = 8 * L.h;
    {
      const rsrc_t epsr = rsrc_n(p.EPS2, C::AOUT * L.ld4);
      const rsrc_t s2r = rsrc_n(p.S2, C::OB * L.ld4);
      const bool closs = p.custom_loss != 0.f;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int j0 = r;
        const int j = j0 + h8;
        const bool ok = j < C::AOUT;
        const int jj = ok ? j : 0;
        const float mu = hd[0][r];
        const float lsr = hd[0][r + 8];
        const float e = fm_ldb(epsr, j0, L.ld4, L.vp);
        const float s2 = closs ? fm_ldb(s2r, j0, L.ld4, L.vp) : 0.f;
        const float ls = fminf(fmaxf(lsr, -20.f), 2.f);
        const float sc = expf(ls);
        const float u = fadd_rn(mu, fmul_rn(e, sc));
        const float d = fsub_rn(u, mu);
        const float t = tanhf(u);
        const float lim = actor_lim<true>(p, L.tbl, jj);
        const float a = fmul_rn(t, lim);
        float g_ad = L.pl[j0 * 32];
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
        hd[0][r] = ok ? gmu : 0.f;
        hd[0][r + 8] = ok ? gls : 0.f;
      }
      if (w == 0) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          if (r + h8 < C::AOUT) {
            fm_st(rsrc(p.ADH), r, L.ld4, L.vp, hd[0][r]);
            fm_st(rsrc(p.ADH), C::AOUT + r, L.ld4, L.vp, hd[0][r + 8]);
          }
        }
      }
    }
    team_sync();  // the image rows read by the heads backward (L.pl) are rewritten below
    // ---- dh2 = Wh^T dheads * relu'(h2) (own blocks); dh1 = W2^T dh2 * relu'(h1)
    dense_team<C::NB_PAIR, C::RV_PAIR>(p.actor.WhT, ob0, hd, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ur = 32 * ob + ru(q);
        const float v = getbit(a2lo, a2hi, ob, q) ? acc[q] : 0.f;
        L.bl[ur * 32] = v;
        fm_st_op(rsrc(p.AD2), ur, L.ld4, L.vo, v);
      }
    });
    team_sync();
    dense_lds_team<2, 8, false>(p.actor.W2T, ob0, img, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q = 0; q < 16; ++q)
        fm_st_op(rsrc(p.AD1), 32 * ob + ru(q), L.ld4, L.vo, getbit(a1lo, a1hi, ob, q) ? acc[q] : 0.f);
    });
    const float ps = wave_sum(sac_part);
    const float pd = wave_sum(dist_part);
    const float pl = wave_sum((valid && L.h == 0) ? lp : 0.f);
    if (w == 0 && lane == 0) {
      p.part[tile * kParts + 2] = ps;
      p.part[tile * kParts + 3] = pd;
      p.part[tile * kParts + 4] = pl;
    }
  }
}

}  // namespace spp
