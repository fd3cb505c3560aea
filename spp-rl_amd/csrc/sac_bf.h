// SAC_AcM critic phase of the bf16 kernel sets (BASELINE.json configs[4]: bf16 MFMA MLP + fp32 targets) with
// TWO 32-sample tiles per wave.
//
// Why: in the one-tile bf16 critic phase (sac.hip) every wave streams its own copy of each 256 x 256 layer's
// weight fragments from the XCD's L2 (128 KiB of bf16 per layer and tile).  Four waves per CU then ask the L2
// for 512 KiB per layer while their MFMAs take 4 x 128 v_mfma_f32_32x32x16_bf16 = 4K cycles per SIMD: the
// layers ran at 2-3x their MFMA time on the L2 -> CU stream (profiles/r02/region_prof_ant_bf16.txt,
// profiles/r05/pmc_sq_phase.txt: 39 % of wave cycles waiting on memory).  Here each fragment feeds the same
// k-step of two tiles (two MFMAs per 16-B fragment load), halving the fragment bytes per sample.
//
// LDS: the activation hand-off between layers is per lane (a lane reads back exactly the units it wrote, as in
// sac.hip), now stored as the bf16 MFMA operands themselves: chunk c = 2 ib + s of a lane holds the 8 bf16 of
// k-step s of input block ib (registers 8s .. 8s+7 of its D-layout tile, RNE: the conversion the fp32 image's
// reader applied), at byte 16 (64 c + lane) -- 16 KiB per tile, one ds_write_b128 / ds_read_b128 per k-step,
// conflict-free.  The narrow fp32 hand-offs (the squashed target action a'_d, the ACM's 64 / 32 / ac rows) reuse
// a tile's 16 KiB as an fp32 [row][32] image while its bf16 operands are dead.  Two tiles per wave therefore fit
// the one-tile kernel's 32 KiB per wave.
//
// The actor heads run in the pairing output order (MAP_PAIR image ActorDev::WhP: register r < 8 of lane half h
// in block ib = mu_j, r + 8 = log_sigma_j, j = 16 ib + 8 h + r), so the squash of sac_acm.py:44-45 is the heads
// layer's epilogue, in registers, with no pairing hand-off through LDS.
//
// Per pair of tiles, as k_sac_critic_phase (rltoolkit/acm/off_policy/sac_acm.py:30-58 targets, :114-131 both
// critics forward + backward): target actor trunk + heads + squash, the frozen ACM on [s' | a'_d] (acm_critic),
// both target critics (soft-min, y), then each critic's forward, d mse / dq, delta2 and W2^T delta2 with the
// weight-gradient operands H1 / H2 / D1 / D2 / DQ stored feature-major as bf16 (op_st), as the one-tile kernel.
// Only the acm_critic sets use it (api / kset choose); with an odd tile count the last pair repeats its first
// tile and stores nothing for the copy.
#pragma once
// tiles per fragment in the critics' first layers (1: one tile at a time; A/B)
#ifndef SPP_BF16_L1_TILES
#define SPP_BF16_L1_TILES 1
#endif

namespace spp {


// bf16 operand image of a tile at this lane: chunk c at img[64 c]
struct Img16 {
  bf16x8* p;  // (generic pointer into LDS: the compiler emits ds_read_b128 / ds_write_b128 for the aligned 16 B)
  __device__ __forceinline__ bf16x8 ld(int c) const { return p[64 * c]; }
  __device__ __forceinline__ void st(int c, const bf16x8& v) const { p[64 * c] = v; }
};
// a lane's row stride made opaque at its use: the products row * ld4 of an epilogue's feature-major stores are then
// formed there, not hoisted to the top of the tile loop and kept live in SGPRs (which then spill into VGPR lanes)
__device__ __forceinline__ int ld4_here(int ld4) {
  asm volatile("" : "+s"(ld4));
  return ld4;
}
// the output block ob of a layer (fp32 D-layout values) as the next layer's operand chunks 2 ob, 2 ob + 1
__device__ __forceinline__ void img16_put(const Img16& im, int ob, const float (&v)[16]) {
  bf16x8 lo, hi;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    lo[j] = (__bf16)v[j];
    hi[j] = (__bf16)v[8 + j];
  }
  im.st(2 * ob, lo);
  im.st(2 * ob + 1, hi);
}

// Register-input bf16 layer over NT tiles (dense16_impl with every fragment feeding NT MFMAs): bin[t][q] is
// k-step q of tile t (st_ib / st_s order), epi(ob, t, acc) per output block and tile.
template <int NT, int NBI, uint64_t RV, bool BIAS, typename Epi>
__device__ __forceinline__ void dense16_tiles(const float4* __restrict__ Wf, int NBO,
                                              const bf16x8 (&bin)[NT][st_total(RV, NBI)], const float* biasL,
                                              Epi&& epi) {
  constexpr int NS = st_total(RV, NBI);
  const int lane = lane_id();
  const int h = lane >> 5;
  const rsrc_t wr = rsrc(Wf);
  const uint32_t l16 = 16u * lane;
  constexpr int OBSTRIDE = NBI * 2 * 64 * 16;
  float4 cur[NS];
  static_for<0, NS>([&](auto Q) {
    constexpr int q = Q;
    cur[q] = wfrag(wr, l16, (st_ib(RV, NBI, q) * 2 + st_s(RV, NBI, q)) * 1024);
  });
  auto chain = [&](int ob, f32x16 (&acc)[NT]) {
    f32x16 b0;
    if constexpr (BIAS) b0 = bias_tile(biasL, ob, h);
    else b0 = zero16();
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = b0;
    const int wn = (ob + 1 < NBO ? ob + 1 : ob) * OBSTRIDE;
    float4 nxt[NS];
    static_for<0, NS>([&](auto Q) {
      constexpr int q = Q;
      nxt[q] = wfrag(wr, l16, wn + (st_ib(RV, NBI, q) * 2 + st_s(RV, NBI, q)) * 1024);
    });
    static_for<0, NS>([&](auto Q) {
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma16(frag16(cur[(int)Q]), bin[t][(int)Q], acc[t]);
    });
#pragma unroll
    for (int q = 0; q < NS; ++q) cur[q] = nxt[q];
  };
  f32x16 prev[NT];
  chain(0, prev);
#pragma unroll 1
  for (int ob = 1; ob < NBO; ++ob) {
    f32x16 acc[NT];
    chain(ob, acc);
#pragma unroll
    for (int t = 0; t < NT; ++t) epi(ob - 1, t, prev[t]);
#pragma unroll
    for (int t = 0; t < NT; ++t) prev[t] = acc[t];
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) epi(NBO - 1, t, prev[t]);
}

// Output blocks [O0, O0 + NO) of a 256-input bf16 layer over NT tiles from their operand images.  The fragments of
// those blocks (2 per block and input block, ib-major image) stream through a ring of D input blocks, loaded D - 1
// blocks ahead; each fragment feeds NT MFMAs; input block ib+1's operand chunks are read while block ib's MFMAs
// issue.  All image reads precede the epilogues (epi(IC<ob>, t, acc)), which may overwrite the images only when
// this call covers every output block.
template <int NT, int NBO, int O0, int NO, bool BIAS, typename Epi>
__device__ __forceinline__ void dense16_lds_part(const float4* __restrict__ Wf, const Img16 (&im)[NT],
                                                 const float* biasL, Epi&& epi) {
  constexpr int NF = 2 * NO;            // fragments per input block
  constexpr int D = 2;                 // ring depth in input blocks (registers: D x NF x 4)
  const int lane = lane_id();
  const int h = lane >> 5;
  const rsrc_t wr = rsrc(Wf);
  const uint32_t l16 = 16u * lane;
  f32x16 acc[NT][NO];
  static_for<0, NO>([&](auto O) {
    f32x16 b0;
    if constexpr (BIAS) b0 = bias_tile(biasL, O0 + (int)O, h);
    else b0 = zero16();
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t][O] = b0;
  });
  float4 fr[D][NF];
  auto load = [&](auto IBC, auto SL) {
    constexpr int ib = IBC, sl = SL;
    static_for<0, NF>([&](auto J) {
      constexpr int j = J;
      fr[sl][j] = wfrag(wr, l16, ((ib * NBO + O0 + (j >> 1)) * 2 + (j & 1)) * 1024);
    });
  };
  static_for<0, D - 1>([&](auto I) { load(I, I); });
  bf16x8 bx[2][NT][2];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    bx[0][t][0] = im[t].ld(0);
    bx[0][t][1] = im[t].ld(1);
  }
  static_for<0, 8>([&](auto IB) {
    constexpr int ib = IB;
    if constexpr (ib + D - 1 < 8) load(IC<ib + D - 1>{}, IC<(ib + D - 1) % D>{});
    if constexpr (ib + 1 < 8) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        bx[(ib + 1) & 1][t][0] = im[t].ld(2 * (ib + 1));
        bx[(ib + 1) & 1][t][1] = im[t].ld(2 * (ib + 1) + 1);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    static_for<0, NO>([&](auto O) {
      constexpr int o = O;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t][o] = mfma16(frag16(fr[ib % D][2 * o]), bx[ib & 1][t][0], acc[t][o]);
        acc[t][o] = mfma16(frag16(fr[ib % D][2 * o + 1]), bx[ib & 1][t][1], acc[t][o]);
      }
    });
  });
  static_for<0, NO>([&](auto O) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      __builtin_amdgcn_sched_barrier(0);  // one block's epilogue at a time (its accumulator reads stay with it)
      epi(IC<O0 + (int)O>{}, t, acc[t][O]);
    }
  });
}
// the whole layer in one pass (its epilogues may overwrite the images)
template <int NT, int NBO, bool BIAS, typename Epi>
__device__ __forceinline__ void dense16_lds_tiles(const float4* __restrict__ Wf, const Img16 (&im)[NT],
                                                  const float* biasL, Epi&& epi) {
  dense16_lds_part<NT, NBO, 0, NBO, BIAS>(Wf, im, biasL, static_cast<Epi&&>(epi));
}
// in two passes over the input, output blocks [0, 4) then [4, NBO): half the accumulators (the epilogues must not
// write the images)
template <int NT, int NBO, bool BIAS, typename Epi>
__device__ __forceinline__ void dense16_lds_halves(const float4* __restrict__ Wf, const Img16 (&im)[NT],
                                                   const float* biasL, Epi&& epi) {
  static_assert(NBO > 4, "two halves");
  dense16_lds_part<NT, NBO, 0, 4, BIAS>(Wf, im, biasL, epi);
  dense16_lds_part<NT, NBO, 4, NBO - 4, BIAS>(Wf, im, biasL, epi);
}

// the k-steps of a register tile as bf16 MFMA operands (st_ib / st_s order: dense16_tiles' bin)
template <int NBI, uint64_t RV>
__device__ __forceinline__ void to_steps(const f32x16 (&x)[NBI], bf16x8 (&b)[st_total(RV, NBI)]) {
  static_for<0, st_total(RV, NBI)>([&](auto Q) {
    constexpr int q = Q;
    b[q] = to_bf16x8<st_s(RV, NBI, q)>(x[st_ib(RV, NBI, q)]);
  });
}

// ============================================================================ critic phase, 2 tiles per wave
template <class C>
__global__ __launch_bounds__(256, 1) void k_sac_critic_phase2(SacArgs p) {
  static_assert(C::BF && !C::F3 && C::ACMC, "bf16 acm_critic sets");
  constexpr int NT = 2;
  constexpr int AREA = kLdsPerWave / NT;  // floats per tile: 16 KiB
  static_assert(AREA * 4 >= 16 * 64 * 16 && AREA >= 128 * 32, "a tile's area holds its 16 operand chunks and an "
                                                                "fp32 [128][32] image");
  static_assert(C::AOUT <= 128 && C::AC <= 32, "narrow fp32 rows");
  __shared__ __attribute__((aligned(16))) float smem[kWavesPerWG * kLdsPerWave];
  __shared__ __attribute__((aligned(16))) float tbl[kTabMax];
  SPP_TP_INIT();
  load_table(p, tbl);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5;
  const int ntiles = p.Bp / 32, npairs = (ntiles + 1) / 2;
  const int ld = p.Bp;
  const float alpha = *p.alpha;
  float* area[NT];
  Img16 im[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    area[t] = smem + w * kLdsPerWave + t * AREA;
    im[t].p = reinterpret_cast<bf16x8*>(area[t]) + lane;
  }
  constexpr int kSmall = 64;  // fp32 rows of the ACM's narrow image within a tile's area
  for (int pr = blockIdx.x * kWavesPerWG + w; pr < npairs; pr += gridDim.x * kWavesPerWG) {
    const int tl[NT] = {2 * pr, 2 * pr + 1 < ntiles ? 2 * pr + 1 : 2 * pr};
    const bool st1 = tl[1] != tl[0];  // the second tile stores (a repeated last tile computes, stores nothing)
    Lane L[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) L[t] = make_lane(area[t], area[t] + kSmall * 32, tbl, ld, tl[t] * 32 + (lane & 31));
    auto stores = [&](int t) { return t == 0 || st1; };
    // the operand stores' lane offsets: a repeated tile's point past every buffer (the hardware range check drops
    // them: no branch around the stores, which costs the layer loops their register allocation)
    uint32_t vst[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) vst[t] = stores(t) ? L[t].vo : 0xFFFFFFFEu;
    // a critic's first layer ([obs | action] inputs from HBM, registers): both tiles per fragment
    // (SPP_BF16_L1_TILES = 2) or one tile at a time (1)
    auto l1_layer = [&](const float4* W, const float* bias, auto&& load, auto&& epi) {
      constexpr int NS = st_total(C::RV_CIN, C::NB_CIN);
      if constexpr (SPP_BF16_L1_TILES == NT) {
        bf16x8 bin[NT][NS];
#pragma unroll
        for (int t = 0; t < NT; ++t) load(t, bin[t]);
        dense16_tiles<NT, C::NB_CIN, C::RV_CIN, true>(W, 8, bin, bias, epi);
      } else {
        static_for<0, NT>([&](auto TT) {
          constexpr int T = TT;
          bf16x8 bin[1][NS];
          load(T, bin[0]);
          dense16_tiles<1, C::NB_CIN, C::RV_CIN, true>(W, 8, bin, bias,
                                                       [&](int ob, int, const f32x16& acc) { epi(ob, T, acc); });
        });
      }
    };
    SPP_TP(0);
    // ---- target action a' ~ pi(s'): trunk, heads in pairing order, squash in the heads epilogue (sac_acm.py:44-45),
    // one tile at a time (these layers overwrite their own input image: all 8 output blocks at once)
    float lp2[NT];
    static_for<0, NT>([&](auto TT) {
      constexpr int T = TT;
      const Img16 imt[1] = {im[T]};
      const Lane& Lt = L[T];
      {
        bf16x8 bin[1][st_total(C::RV_X, C::NB_OB)];
        f32x16 x[C::NB_OB];
        gm_load<C::NB_OB>(x, p.S2, C::OB * Lt.ld4, C::OB, Lt.ld4, Lt.vo);
        to_steps<C::NB_OB, C::RV_X>(x, bin[0]);
        dense16_tiles<1, C::NB_OB, C::RV_X, true>(p.actor.W1, 8, bin, tbl + p.actor.tb1,
                                                  [&](int ob, int, const f32x16& acc) {
          float v[16];
#pragma unroll
          for (int q = 0; q < 16; ++q) v[q] = fmaxf(acc[q], 0.f);
          img16_put(imt[0], ob, v);
        });
      }
      SPP_TP(1);
      dense16_lds_tiles<1, 8, true>(p.actor.W2, imt, tbl + p.actor.tb2, [&](auto O, int, const f32x16& acc) {
        float v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = fmaxf(acc[q], 0.f);
        img16_put(imt[0], (int)O, v);
      });
      SPP_TP(2);
      float lp = 0.f, corr = 0.f;
      const float* bh = tbl + p.actor.tbh;  // [mu bias | log_sigma bias], AOUT each
      const rsrc_t er = rsrc_n(p.EPS1, C::AOUT * Lt.ld4);
      dense16_lds_tiles<1, C::NB_PAIR, false>(p.actor.WhP, imt, nullptr, [&](auto O, int, const f32x16& acc) {
        constexpr int ib = O;
        float ev[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) ev[r] = fm_ldb(er, 16 * ib + r, Lt.ld4, Lt.vp);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int j0 = 16 * ib + r, j = j0 + 8 * h;
          const bool ok = j < C::AOUT;
          const int jj = ok ? j : 0;
          const float mu = acc[r] + bh[jj];
          const float ls = fminf(fmaxf(acc[r + 8] + bh[C::AOUT + jj], -20.f), 2.f);
          const float e = ev[r];
          const float sc = t_exp<true>(ls);
          const float u = fadd_rn(mu, fmul_rn(e, sc));
          const float lpj = -0.5f * e * e - ls - kLogSqrt2Pi;  // (the bf16 sets' algebraic log-prob, sac.hip)
          const float cj = 2.f * fsub_rn(fsub_rn(kLog2, u), t_softplus<true>(-2.f * u));
          lp += ok ? lpj : 0.f;
          corr += ok ? cj : 0.f;
          const float a = fmul_rn(t_tanh<true>(u), actor_lim<true>(p, tbl, jj));
          const float ad = denorm<true>(p, tbl, jj, a);
          if (ok) Lt.pl[j0 * 32] = ad;  // a'_d, natural fp32 row j of the tile's image (all chunk reads done)
        }
      });
      SPP_XLANE_SYNC();
      const float tot = lp + __shfl_xor(lp, 32, 64), tc = corr + __shfl_xor(corr, 32, 64);
      lp2[T] = fsub_rn(tot, tc);
      SPP_TP(3);
    });
    // ---- the frozen ACM on [s' | a'_d] -> c (:46-48), per tile; c kept in registers for both target critics
    f32x16 creg[NT][1];
#pragma unroll  // (per tile; unrolled: the Lane array is indexed by compile-time tiles only)
    for (int t = 0; t < NT; ++t) {
      f32x16 xin[C::NB_ACMIN];
      load_cat_gl<C::NB_OB, C::NB_AOUT>(xin, p.S2, C::OB * L[t].ld4, C::OB, L[t].ld4, L[t].vo, area[t], C::AOUT);
      SPP_XLANE_SYNC();  // (the ACM's narrow rows overlap a'_d's: every a'_d read is issued before them)
      acm_forward<C, false>(p, xin, L[t], nullptr, nullptr, nullptr);
      SPP_XLANE_SYNC();
      const float* sl = L[t].sl;  // small rows [0, AC): c, natural layout (lane half h: units ru(r) + 4h)
#pragma unroll
      for (int r = 0; r < 16; ++r) creg[t][0][r] = (ru(r) + 4 * h < C::AC) ? sl[ru(r) * 32] : 0.f;
    }
    SPP_TP(5);
    // ---- soft-min twin target (:50-56)
    float qt[2][NT];
#pragma unroll 1
    for (int k = 0; k < 2; ++k) {
      const CriticDev& Q = p.targ[k];
      auto tin = [&](int t, bf16x8 (&b)[st_total(C::RV_CIN, C::NB_CIN)]) {  // [s' | c] of tile t
        f32x16 xs[C::NB_OB], x[C::NB_CIN];
        gm_load<C::NB_OB>(xs, p.S2, C::OB * L[t].ld4, C::OB, L[t].ld4, L[t].vo);
#pragma unroll
        for (int ib = 0; ib < C::NB_OB; ++ib) x[ib] = xs[ib];
        x[C::NB_OB] = creg[t][0];
        to_steps<C::NB_CIN, C::RV_CIN>(x, b);
      };
      auto tepi = [&](int ob, int t, const f32x16& acc) {
        float v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = fmaxf(acc[q], 0.f);
        img16_put(im[t], ob, v);
      };
      l1_layer(Q.W1, tbl + Q.tb1, tin, tepi);
      SPP_TP(6 + 2 * k);
      float qp[NT] = {0.f, 0.f};
      const float* w3 = tbl + Q.tw3;
      dense16_lds_halves<NT, 8, true>(Q.W2, im, tbl + Q.tb2, [&](auto O, int t, const f32x16& acc) {
        float tv[16];
        tvals(w3, (int)O, 4 * h, tv);
#pragma unroll
        for (int q = 0; q < 16; ++q) qp[t] = fmaf(fmaxf(acc[q], 0.f), tv[q], qp[t]);
      });
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const float qv = qp[t] + __shfl_xor(qp[t], 32, 64) + *Q.b3;
        if (k == 0) qt[0][t] = qv;  // (no runtime index into a register array)
        else qt[1][t] = qv;
      }
      SPP_TP(7 + 2 * k);
    }
    float y[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int b = L[t].b;
      const float notdone = 1.f - p.DN[b];
      y[t] = fadd_rn(p.R[b], fmul_rn(p.gamma * notdone, fsub_rn(fminf(qt[0][t], qt[1][t]), alpha * lp2[t])));
    }
    SPP_TP(10);
    // ---- both critics: forward, MSE gradient, backward to the weight-gradient operands (:117-131)
    float lq[2][NT];
#pragma unroll 1
    for (int i = 0; i < 2; ++i) {
      const CriticDev& Q = p.critic[i];
      uint64_t m1lo[NT] = {0, 0}, m1hi[NT] = {0, 0}, m2lo[NT] = {0, 0}, m2hi[NT] = {0, 0};
      {
        auto cin = [&](int t, bf16x8 (&b)[st_total(C::RV_CIN, C::NB_CIN)]) {  // [s | a_env] of tile t
          f32x16 x[C::NB_CIN];
          load_cat_gg<C::NB_OB, C::NB_CA>(x, p.S, C::OB, p.AENV, C::CA, L[t].ld4, L[t].vo);
          to_steps<C::NB_CIN, C::RV_CIN>(x, b);
        };
        const rsrc_t h1r = rsrc(p.H1[i]);
        auto cepi = [&](int ob, int t, const f32x16& acc) {
          float v[16];
          uint32_t bits = 0;
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            v[q] = fmaxf(acc[q], 0.f);
            bits |= (uint32_t)(v[q] > 0.f) << q;
          }
          img16_put(im[t], ob, v);
          const int l4 = ld4_here(L[t].ld4);
#pragma unroll
          for (int q = 0; q < 16; ++q) op_st<true>(h1r, 32 * ob + ru(q), l4, vst[t], v[q]);
          setbits(m1lo[t], m1hi[t], ob, bits);
        };
        l1_layer(Q.W1, tbl + Q.tb1, cin, cepi);
      }
      SPP_TP(11);
      float qp[NT] = {0.f, 0.f};
      const float* w3 = tbl + Q.tw3;
      {
        const rsrc_t h2r = rsrc(p.H2[i]);
        dense16_lds_halves<NT, 8, true>(Q.W2, im, tbl + Q.tb2, [&](auto O, int t, const f32x16& acc) {
          constexpr int ob = O;
          float tv[16];
          tvals(w3, ob, 4 * h, tv);
          uint32_t bits = 0;
          const int l4 = ld4_here(L[t].ld4);
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const float v = fmaxf(acc[q], 0.f);
            op_st<true>(h2r, 32 * ob + ru(q), l4, vst[t], v);
            qp[t] = fmaf(v, tv[q], qp[t]);
            bits |= (uint32_t)(v > 0.f) << q;
          }
          setbits(m2lo[t], m2hi[t], ob, bits);
        });
      }
      float dq[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int b = L[t].b;
        const bool valid = b < p.B;
        const float q = qp[t] + __shfl_xor(qp[t], 32, 64) + *Q.b3;
        const float diff = fsub_rn(q, y[t]);
        dq[t] = valid ? fmul_rn(2.f * diff, p.inv_B) : 0.f;  // d mse / dq
        const float lqv = (valid && h == 0) ? diff * diff : 0.f;
        if (i == 0) lq[0][t] = lqv;
        else lq[1][t] = lqv;
        if (h == 0 && stores(t)) p.DQ[i][b] = dq[t];  // (k_dw: dW3 = dq . h2^T)
      }
      SPP_TP(12);
      // delta2 = dq * w3 * relu'(h2) -> the operand image and D2
      const rsrc_t d2r = rsrc(p.D2[i]);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
#pragma unroll 1
        for (int ob = 0; ob < 8; ++ob) {
          float tv[16], v[16];
          tvals(w3, ob, 4 * h, tv);
          const int l4 = ld4_here(L[t].ld4);
#pragma unroll
          for (int q2 = 0; q2 < 16; ++q2) {
            v[q2] = getbit(m2lo[t], m2hi[t], ob, q2) ? dq[t] * tv[q2] : 0.f;
            op_st<true>(d2r, 32 * ob + ru(q2), l4, vst[t], v[q2]);
          }
          img16_put(im[t], ob, v);
        }
      }
      SPP_TP(13);
      // delta1 = (W2^T delta2) * relu'(h1) -> D1
      const rsrc_t d1r = rsrc(p.D1[i]);
      dense16_lds_halves<NT, 8, false>(Q.W2T, im, nullptr, [&](auto O, int t, const f32x16& acc) {
        constexpr int ob = O;
        const int l4 = ld4_here(L[t].ld4);
#pragma unroll
        for (int q2 = 0; q2 < 16; ++q2)
          op_st<true>(d1r, 32 * ob + ru(q2), l4, vst[t], getbit(m1lo[t], m1hi[t], ob, q2) ? acc[q2] : 0.f);
      });
      SPP_TP(14);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const float s0 = wave_sum(lq[0][t]), s1 = wave_sum(lq[1][t]);
      if (lane == 0 && stores(t)) {
        p.part[tl[t] * kParts + 0] = s0;
        p.part[tl[t] * kParts + 1] = s1;
      }
    }
    SPP_TP(15);
  }
  SPP_TP_FLUSH();
}

}  // namespace spp
