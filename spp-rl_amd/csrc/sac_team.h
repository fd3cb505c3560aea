// Small-batch ("team") forms of the SAC phase kernels (gfx950), for batches of at most one 32-sample tile
// per CU (BASELINE.json configs[0]: vanilla SAC, B = 100, rltoolkit/algorithms/sac/sac.py:218-280).
//
// k_sac_critic_phase / k_sac_actor_phase give each 32-sample tile to ONE wave, which runs every layer of the
// phase as a serial chain of 32x32x2 f32 MFMAs; at B = 100 that is 4 waves on 4 SIMDs of one CU, and the
// phase is that chain's length (MFMA-bound: ~8 layer-equivalents x 1,024 MFMAs x 64 cycles).  Here a tile
// gets a workgroup of TW waves sharing the tile's LDS image: 8 for the critic phase (two per SIMD: one's
// MFMA chain covers the other's LDS / weight-load latency), 4 for the actor phase (more live state).  Each
// 256-wide layer is split by output blocks -- wave w computes the 8/TW blocks from (8/TW)*w -- and each
// 1-block layer (the heads, the critics' action-input gradient) by input blocks, its TW partial tiles summed
// through LDS in wave order.  A workgroup barrier separates a
// layer's last image read from its first image write, another the write from the next layer's reads.  The
// per-sample work (squash, log-prob, targets, losses) is computed by every wave on the same values in the
// same order, so every wave holds the same scalars and the barrier sequence is uniform; HBM writes of
// replicated values are made by wave 0 only.  Each tile runs on its own CU, one tile
// per workgroup (grid = min(tiles, CUs), api.hip's sac_grid).
//
// Same math as the one-wave kernels (sac.hip); the summation order of the q reduction and of the fused fc3
// weight gradient differs (wave-partials in fixed order), so results agree within fp32 rounding, not bit
// for bit.  Vanilla-SAC shapes only (no ACM in the critic input, fp32, heads <= 2 pairing blocks).
#pragma once
#include "sac.hip"

namespace spp {

// waves per tile: the critic phase runs 8 (two per SIMD); the actor phase 4 (its live state does not fit 8
// waves' 256-register budget without spilling)
constexpr int kTeamCritic = 8, kTeamActor = 4;

__device__ __forceinline__ void team_sync() { __syncthreads(); }

// ReLU masks of the wave's own output blocks only (k = ob - ob0 < 8/TW <= 2): 16 bits per block in one register
__device__ __forceinline__ void setown(uint32_t& m, int k, uint32_t bits) {
  m |= bits << (16 * k);
  asm volatile("" : "+v"(m));
}
__device__ __forceinline__ bool getown(uint32_t m, int k, int q) { return (m >> (16 * k + q)) & 1u; }

// A 1-output-block layer over the 256-unit image (ib-major image with one output block), split by input
// blocks: wave w's 16 MFMAs over block w, the 8 partial tiles summed through LDS (part) in wave order, the
// bias first.  Every wave returns the same tile.  Reads the image and part; team-synchronised on return (the
// image may be written, part reused).
template <bool BIAS, int TW>
__device__ __forceinline__ f32x16 dense1_ksplit(const float4* __restrict__ Wf, const float* img, const float* biasL,
                                                float (*part)[16][64], int w) {
  constexpr int NIB = 8 / TW;  // input blocks per wave
  const int lane = lane_id();
  const int h = lane >> 5;
  const float* l = img + 4 * h * 32 + (lane & 31);
  const rsrc_t wr = rsrc(Wf);
  const uint32_t l16 = 16u * lane;
  float4 c[NIB][4];
  f32x16 x[NIB];
#pragma unroll
  for (int k = 0; k < NIB; ++k) {
#pragma unroll
    for (int q = 0; q < 4; ++q) c[k][q] = wfrag(wr, l16, ((NIB * w + k) * 4 + q) * 1024);
#pragma unroll
    for (int r = 0; r < 16; ++r) x[k][r] = l[(32 * (NIB * w + k) + ru(r)) * 32];
  }
  f32x16 acc = zero16();
#pragma unroll
  for (int k = 0; k < NIB; ++k)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      acc = mfma(c[k][q].x, x[k][4 * q + 0], acc);
      acc = mfma(c[k][q].y, x[k][4 * q + 1], acc);
      acc = mfma(c[k][q].z, x[k][4 * q + 2], acc);
      acc = mfma(c[k][q].w, x[k][4 * q + 3], acc);
    }
#pragma unroll
  for (int r = 0; r < 16; ++r) part[w][r][lane] = acc[r];
  team_sync();
  f32x16 t;
  if constexpr (BIAS) t = bias_tile(biasL, 0, h);
  else t = zero16();
#pragma unroll
  for (int v = 0; v < TW; ++v)
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] += part[v][r][lane];
  team_sync();
  return t;
}

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

// This wave's NOW output blocks ob0 .. of a register-input layer with 8 output blocks (ob-major image,
// sac.hip's dense); the epilogue may write the image: the caller has synchronised after the team's last image
// read.
template <int NBI, uint64_t RV, int NOW, typename Epi>
__device__ __forceinline__ void dense_team(const float4* __restrict__ Wf, int ob0, const f32x16 (&in)[NBI],
                                           const float* biasL, Epi&& epi) {
  dense<NBI, RV>(Wf + (size_t)ob0 * NBI * 4 * 64, NOW, in, biasL + 32 * ob0,
                 [&](int j, const f32x16& acc) { epi(ob0 + j, acc); });
}
template <int NBI, uint64_t RV, int NOW, typename Epi>
__device__ __forceinline__ void dense_team(const float4* __restrict__ Wf, int ob0, const f32x16 (&in)[NBI],
                                           decltype(nullptr), Epi&& epi) {
  dense<NBI, RV>(Wf + (size_t)ob0 * NBI * 4 * 64, NOW, in, nullptr,
                 [&](int j, const f32x16& acc) { epi(ob0 + j, acc); });
}

// Actor trunk (sac.hip actor_trunk), team form: h1 / h2 split by blocks (masks of the wave's own blocks only),
// heads (one block, split by input blocks) written to rows [0, 2*AOUT) by wave 0.
// Returns with the heads in the image, team-synchronised.
template <class C, bool ST, int TW>
__device__ __forceinline__ void actor_trunk_team(const ActorDev& A, const float* X, int xbytes, const Lane& L,
                                                 int w, float* H1g, float* H2g, float (*part)[16][64],
                                                 uint32_t& m1, uint32_t& m2) {
  static_assert(C::NB_H2 == 1, "team heads: one output block");
  constexpr int NOW = 8 / TW;
  const int ob0 = NOW * w;
  {
    f32x16 x[C::NB_OB];
    gm_load<C::NB_OB>(x, X, xbytes, C::OB, L.ld4, L.vo);
    const rsrc_t hr = rsrc(H1g);
    dense_team<C::NB_OB, C::RV_X, NOW>(A.W1, ob0, x, L.tbl + A.tb1, [&](int ob, const f32x16& acc) {
      uint32_t bits = 0;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ur = 32 * ob + ru(q);
        const float v = fmaxf(acc[q], 0.f);
        L.bl[ur * 32] = v;
        if constexpr (ST) fm_st_op(hr, ur, L.ld4, L.vo, v);
        bits |= (uint32_t)(v > 0.f) << q;
      }
      setown(m1, ob - ob0, bits);
    });
  }
  team_sync();
  {
    const rsrc_t hr = rsrc(H2g);
    dense_lds_team<NOW, 8, true>(A.W2, ob0, L.img, L.tbl + A.tb2, [&](int ob, const f32x16& acc) {
      uint32_t bits = 0;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ur = 32 * ob + ru(q);
        const float v = fmaxf(acc[q], 0.f);
        L.bl[ur * 32] = v;
        if constexpr (ST) fm_st_op(hr, ur, L.ld4, L.vo, v);
        bits |= (uint32_t)(v > 0.f) << q;
      }
      setown(m2, ob - ob0, bits);
    });
  }
  team_sync();
  const f32x16 hd = dense1_ksplit<true, TW>(A.Wh, L.img, L.tbl + A.tbh, part, w);
  if (w == 0) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ur = ru(q);
      if (ur + L.h4 < 2 * C::AOUT) L.bl[ur * 32] = hd[q];
    }
  }
  team_sync();
}

// Critic forward through L2 (sac.hip critic_forward), team form: returns q (every wave the same value; the
// per-wave partials of w3 . relu(h2) summed in wave order through red).  H2L: h2 of the wave's own blocks
// goes to the image (the fused fc3 weight gradient reads it there).  Caller: the image is free to write.
template <class C, bool ST, bool H2L, int TW>
__device__ __forceinline__ float critic_forward_team(const CriticDev& Q, const f32x16 (&xin)[C::NB_CIN],
                                                     const Lane& L, int w, float* H1g, float* H2g,
                                                     float (*red)[64], uint32_t& m1, uint32_t& m2) {
  constexpr int NOW = 8 / TW;
  const int ob0 = NOW * w;
  const rsrc_t h1r = rsrc(H1g), h2r = rsrc(H2g);
  dense_team<C::NB_CIN, C::RV_CIN, NOW>(Q.W1, ob0, xin, L.tbl + Q.tb1, [&](int ob, const f32x16& acc) {
    uint32_t bits = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ur = 32 * ob + ru(q);
      const float v = fmaxf(acc[q], 0.f);
      L.bl[ur * 32] = v;
      if constexpr (ST) fm_st_op(h1r, ur, L.ld4, L.vo, v);
      bits |= (uint32_t)(v > 0.f) << q;
    }
    setown(m1, ob - ob0, bits);
  });
  team_sync();
  float qp = 0.f;
  const float* w3 = L.tbl + Q.tw3;
  dense_lds_team<NOW, 8, true>(Q.W2, ob0, L.img, L.tbl + Q.tb2, [&](int ob, const f32x16& acc) {
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
    setown(m2, ob - ob0, bits);
  });
  const int lane = lane_id();
  red[w][lane] = qp;
  team_sync();
  float s = red[0][lane];
#pragma unroll
  for (int v = 1; v < TW; ++v) s += red[v][lane];
  return s + __shfl_xor(s, 32, 64) + *Q.b3;
}

// ============================================================================ critic phase, team form
template <class C, int TW = kTeamCritic>
__global__ __launch_bounds__(TW * 64, 1) void k_sac_critic_team(SacArgs p) {
  static_assert(!C::ACMC && !C::BF && C::F3 && C::NB_PAIR == 1, "team critic phase: vanilla fp32 shapes");
  __shared__ float img[kLdsPerWave];
  __shared__ __attribute__((aligned(16))) float tbl[kTabMax];
  constexpr int NOW = 8 / TW;
  constexpr int UW = 32 * NOW;  // fc3 units per wave
  __shared__ float red[TW][64];
  __shared__ float s_dq[TW][32];
  __shared__ float part[TW][16][64];
  load_table(p, tbl);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int ob0 = NOW * w;
  const int ntiles = p.Bp / 32;
  const int ld = p.Bp;
  const float alpha = *p.alpha;
  float w3a = 0.f, w3b = 0.f, b3a = 0.f, b3b = 0.f;  // fused fc3 grads of unit UW*w + lane % UW (bias: wave 0)
  // critic split (grid = 2 x tiles, api.hip sac_critic_grid): workgroup 2t + c runs tile t's target (both target
  // critics, computed by both workgroups of the tile) and critic c only; else every critic of every tile
  const bool split = (int)gridDim.x == 2 * ntiles;
  const int c0 = split ? (int)(blockIdx.x & 1) : 0, c1 = split ? c0 + 1 : 2;
  const int tstride = split ? ntiles : (int)gridDim.x;
  for (int tile = split ? (int)(blockIdx.x >> 1) : (int)blockIdx.x; tile < ntiles; tile += tstride) {
    const Lane L = make_lane(img, img + kSmallRow * 32, tbl, ld, tile * 32 + (lane & 31));
    const int b = L.b;
    const bool valid = b < p.B;
    uint32_t d0 = 0, d1 = 0;
    // ---- target action a' ~ pi(s'), logpi'   (sac.py:230-236)
    actor_trunk_team<C, false, TW>(p.actor, p.S2, C::OB * L.ld4, L, w, nullptr, nullptr, part, d0, d1);
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
    const float q1t = critic_forward_team<C, false, false, TW>(p.targ[0], tin, L, w, nullptr, nullptr, red, d0, d1);
    const float q2t = critic_forward_team<C, false, false, TW>(p.targ[1], tin, L, w, nullptr, nullptr, red, d0, d1);
    const float notdone = 1.f - p.DN[b];
    const float y = fadd_rn(p.R[b], fmul_rn(p.gamma * notdone, fsub_rn(fminf(q1t, q2t), alpha * lp2)));
    // ---- both critics: forward, MSE grad, backward to the weight-gradient operands (sac.py:243-252)
    float lq0 = 0.f, lq1 = 0.f;
#pragma unroll 1
    for (int i = c0; i < c1; ++i) {
      uint32_t m1 = 0, m2 = 0;
      f32x16 xin[C::NB_CIN];
      load_cat_gg<C::NB_OB, C::NB_CA>(xin, p.S, C::OB, p.ACT, C::CA, L.ld4, L.vo);
      const CriticDev& Q = p.critic[i];
      const float q = critic_forward_team<C, true, true, TW>(Q, xin, L, w, p.H1[i], nullptr, red, m1, m2);
      const float diff = fsub_rn(q, y);
      const float dq = valid ? fmul_rn(2.f * diff, p.inv_B) : 0.f;
      const float lqi = (valid && L.h == 0) ? diff * diff : 0.f;
      if (i == 0) lq0 = lqi; else lq1 = lqi;
      // fc3 weight gradient of this wave's units (dW3 = dq . h2^T, db3 = sum dq): h2 rows UW*w .. are this
      // wave's own image rows; lane l sums unit UW*w + l % UW over its 32*UW/64 samples (a lane half each when
      // UW = 32, combined across the halves)
      if (L.h == 0) s_dq[w][L.s] = dq;
      SPP_XLANE_SYNC();
      {
        constexpr int NS = 32 * UW / 64;
        const int u = UW * w + lane % UW;
        const int s0 = NS * (lane / UW);
        const float* row = img + u * 32;
        float acc = 0.f;
#pragma unroll 8
        for (int j = 0; j < NS; ++j) {
          const int s2 = s0 + ((j + u) & (NS - 1));
          acc = fmaf(row[s2], s_dq[w][s2], acc);
        }
        if constexpr (UW == 32) acc += __shfl_xor(acc, 32, 64);
        if (i == 0) w3a += acc; else w3b += acc;
      }
      const float dsum = wave_sum(L.h == 0 ? dq : 0.f);
      if (i == 0) b3a += dsum; else b3b += dsum;
      SPP_XLANE_SYNC();  // own rows rewritten below
      // delta2 = dq * w3 * relu'(h2), own blocks, staged in the image and stored feature-major
      const rsrc_t d2r = rsrc(p.D2[i]);
      const float* w3 = tbl + Q.tw3;
#pragma unroll 1
      for (int k = 0; k < NOW; ++k) {
        const int ob = ob0 + k;
        float tv[16];
        tvals(w3, ob, L.h4, tv);
#pragma unroll
        for (int q2 = 0; q2 < 16; ++q2) {
          const int ur = 32 * ob + ru(q2);
          const float v = getown(m2, k, q2) ? dq * tv[q2] : 0.f;
          L.bl[ur * 32] = v;
          fm_st_op(d2r, ur, L.ld4, L.vo, v);
        }
      }
      team_sync();
      // delta1 = (W2^T delta2) * relu'(h1), own blocks
      const rsrc_t d1r = rsrc(p.D1[i]);
      dense_lds_team<NOW, 8, false>(Q.W2T, ob0, img, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
        for (int q2 = 0; q2 < 16; ++q2)
          fm_st_op(d1r, 32 * ob + ru(q2), L.ld4, L.vo, getown(m1, ob - ob0, q2) ? acc[q2] : 0.f);
      });
    }
    const float s0 = wave_sum(lq0), s1 = wave_sum(lq1);
    if (w == 0 && lane == 0) {
      if (c0 == 0) p.part[tile * kParts + 0] = s0;
      if (c1 == 2) p.part[tile * kParts + 1] = s1;
    }
  }
  // this wave's fc3 partials [256 weights | bias] per critic: units UW*w .. (from lanes 0 .. UW-1), zeros
  // elsewhere (k_dw_reduce sums the TW slots of each workgroup)
  const int64_t wg = (int64_t)blockIdx.x * TW + w;
  float* o0 = p.W3P[0] + wg * p.w3p_stride;
  float* o1 = p.W3P[1] + wg * p.w3p_stride;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int idx = lane + 64 * k;
    const bool own = idx / UW == w;
    const float va = __shfl(w3a, idx % UW, 64), vb = __shfl(w3b, idx % UW, 64);
    o0[idx] = own ? va : 0.f;
    o1[idx] = own ? vb : 0.f;
  }
  if (lane == 0) {
    o0[256] = w == 0 ? b3a : 0.f;
    o1[256] = w == 0 ? b3b : 0.f;
  }
}

// ============================================================================ actor phase, team form
template <class C, int TW = kTeamActor>
__global__ __launch_bounds__(TW * 64, 1) void k_sac_actor_team(SacArgs p, AcmScratch) {
  static_assert(!C::ACMC && !C::BF && C::NB_PAIR == 1 && C::NB_CA == 1, "team actor phase: vanilla fp32 shapes");
  __shared__ float img[kLdsPerWave];
  __shared__ __attribute__((aligned(16))) float tbl[kTabMax];
  constexpr int NOW = 8 / TW;
  __shared__ float red[TW][64];
  __shared__ float part[TW][16][64];
  __shared__ float hpark[16][64];  // the heads tile (mu | raw log-std), parked by wave 0 through the critics
  __shared__ float apark[8 * 32];  // a_d rows [0, AOUT) of the image: the second critic's action input
  __shared__ float dpark[16][64];  // the first critic's d loss / d a tile
  load_table(p, tbl);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int ob0 = NOW * w;
  const int ntiles = p.Bp / 32;
  const int ld = p.Bp;
  const float alpha = *p.alpha;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const Lane L = make_lane(img, img + kSmallRow * 32, tbl, ld, tile * 32 + (lane & 31));
    const int b = L.b;
    const bool valid = b < p.B;
    const float g_lp = valid ? alpha * p.inv_B : 0.f;  // d loss / d logpi_b
    // ---- a, logpi = actor(s)  (sac.py:262-266)
    uint32_t a1 = 0, a2 = 0;
    actor_trunk_team<C, true, TW>(p.actor, p.S, C::OB * L.ld4, L, w, p.AH1, p.AH2, part, a1, a2);
    f32x16 hd[C::NB_PAIR];
    load_pair<C>(hd, img);
    team_sync();
    const float lp = squash_write<C>(p, hd, p.EPS2, L);  // a_d -> image rows [0, AOUT), every wave the same
    if (w == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) hpark[r][lane] = hd[0][r];
    }
    team_sync();
    if (w == 0) {
      for (int i = lane; i < C::AOUT * 32; i += 64) apark[i] = img[i];
    }
    float q1, q2;
    // ---- q = min(Q1, Q2)(s, a)  (sac.py:267-270), own-block masks kept for the backward
    uint32_t ma1 = 0, ma2 = 0, mb1 = 0, mb2 = 0;
    {
      f32x16 cin[C::NB_CIN];
      load_cat_gl<C::NB_OB, C::NB_CA>(cin, p.S, C::OB * L.ld4, C::OB, L.ld4, L.vo, img, C::AOUT);
      team_sync();
      q1 = critic_forward_team<C, false, false, TW>(p.critic[0], cin, L, w, nullptr, nullptr, red, ma1, ma2);
    }
    {
      f32x16 cin[C::NB_CIN];  // (apark: written by wave 0 before the first critic's barriers)
      load_cat_gl<C::NB_OB, C::NB_CA>(cin, p.S, C::OB * L.ld4, C::OB, L.ld4, L.vo, apark, C::AOUT);
      q2 = critic_forward_team<C, false, false, TW>(p.critic[1], cin, L, w, nullptr, nullptr, red, mb1, mb2);
    }
    const float qmin = fminf(q1, q2);
    const float gq = valid ? -p.inv_B : 0.f;
    const float dqa = q1 < q2 ? gq : (q1 == q2 ? 0.5f * gq : 0.f);
    const float dqb = q2 < q1 ? gq : (q1 == q2 ? 0.5f * gq : 0.f);
    // ---- back through both critics to their action input
    f32x16 dca;  // d loss / d a: critic 0's tile parked in LDS (dpark) through critic 1's backward
#pragma unroll 1
    for (int i = 0; i < 2; ++i) {
      const CriticDev& Q = p.critic[i];
      const uint32_t k1m = i ? mb1 : ma1, k2m = i ? mb2 : ma2;
      const float dqi = i ? dqb : dqa;
      const float* w3 = tbl + Q.tw3;
#pragma unroll 1
      for (int k = 0; k < NOW; ++k) {
        const int ob = ob0 + k;
        float tv[16];
        tvals(w3, ob, L.h4, tv);
#pragma unroll
        for (int q = 0; q < 16; ++q) L.bl[(32 * ob + ru(q)) * 32] = getown(k2m, k, q) ? dqi * tv[q] : 0.f;
      }
      team_sync();
      dense_lds_team<NOW, 8, false>(Q.W2T, ob0, img, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
        for (int q = 0; q < 16; ++q) L.bl[(32 * ob + ru(q)) * 32] = getown(k1m, ob - ob0, q) ? acc[q] : 0.f;
      });
      team_sync();
      const f32x16 t = dense1_ksplit<false, TW>(Q.W1Ta, img, nullptr, part, w);
      if (i == 0) {
        if (w == 0) {
#pragma unroll
          for (int r = 0; r < 16; ++r) dpark[r][lane] = t[r];
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) dca[r] = (0.f + dpark[r][lane]) + t[r];
      }
    }
    // d loss / d a_d into image rows [0, AOUT) (the heads backward reads it in the pairing layout)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ur = ru(q);
      if (ur + L.h4 < C::AOUT) L.bl[ur * 32] = dca[q];
    }
    team_sync();
#pragma unroll
    for (int r = 0; r < 16; ++r) hd[0][r] = hpark[r][lane];
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
    dense_team<C::NB_PAIR, C::RV_PAIR, NOW>(p.actor.WhT, ob0, hd, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int ur = 32 * ob + ru(q);
        const float v = getown(a2, ob - ob0, q) ? acc[q] : 0.f;
        L.bl[ur * 32] = v;
        fm_st_op(rsrc(p.AD2), ur, L.ld4, L.vo, v);
      }
    });
    team_sync();
    dense_lds_team<NOW, 8, false>(p.actor.W2T, ob0, img, nullptr, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q = 0; q < 16; ++q)
        fm_st_op(rsrc(p.AD1), 32 * ob + ru(q), L.ld4, L.vo, getown(a1, ob - ob0, q) ? acc[q] : 0.f);
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

namespace spp {

// ============================================================================ rollout action, team form
// k_policy_act (sac.hip) for the plain (vanilla SAC) handles: the actor trunk of each 32-env tile split over a
// TW-wave workgroup (actor_trunk_team), then the per-env action of DDPG.noise_action / SAC sampling
// (ddpg.py:171-180, sac.py:182-196) computed by every wave and written by wave 0.  Same arithmetic as
// k_policy_act's plain branch.
template <class C, int TW = kTeamCritic>
__global__ __launch_bounds__(TW * 64, 1) void k_policy_act_team(SacArgs p, ActArgs a) {
  static_assert(C::NB_PAIR == 1, "team act: one pairing block");
  __shared__ float img[kLdsPerWave];
  __shared__ __attribute__((aligned(16))) float tbl[kTabMax];
  __shared__ float part[TW][16][64];
  load_table(p, tbl);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int ntiles = (a.E + 31) / 32;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int e = tile * 32 + (lane & 31);
    const bool valid = e < a.E;
    const int er = valid ? e : 0;
    Lane L = make_lane(img, img + kSmallRow * 32, tbl, 1, er * C::OB);  // row-major obs: ld = 1
    const bool use_actor = a.mode == 1 || a.mode == 2;
    f32x16 hd[C::NB_PAIR];
    if (use_actor) {
      uint32_t d0 = 0, d1 = 0;
      actor_trunk_team<C, false, TW>(p.actor, a.obs, a.E * C::OB * 4, L, w, nullptr, nullptr, part, d0, d1);
      load_pair<C>(hd, img);
    }
    const int h8 = 8 * L.h;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int j = r + h8;
      if (j < C::AOUT) {
        const float lim = actor_lim<true>(p, L.tbl, j);
        float act;
        if (a.mode == 0 || a.mode == 3) {
          act = valid ? a.eps[er * C::AOUT + j] : 0.f;  // action_space.sample() drawn by the caller
        } else {  // DDPG.noise_action: a + act_noise * N(0,1), clip to [-lim, lim]
          const float mu = hd[0][r];
          float u = mu;
          if (a.mode == 1 && a.eps) {
            const float ls = fminf(fmaxf(hd[0][r + 8], -20.f), 2.f);
            u = fadd_rn(mu, fmul_rn(valid ? a.eps[er * C::AOUT + j] : 0.f, expf(ls)));
          }
          act = fmul_rn(tanhf(u), lim);
          if (a.mode == 1 && a.noise) act = fadd_rn(act, a.act_noise * (valid ? a.noise[er * C::AOUT + j] : 0.f));
          act = fminf(fmaxf(act, -lim), lim);
        }
        if (valid && w == 0) {
          a.target_out[er * C::AOUT + j] = act;
          a.env_out[er * C::AOUT + j] = act;  // process_action: identity (ddpg.py:371-384)
        }
      }
    }
    team_sync();  // the next tile's trunk rewrites the image the heads were read from
  }
}

}  // namespace spp
