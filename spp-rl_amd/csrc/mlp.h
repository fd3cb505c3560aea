// Register-tile MLP machinery for the per-sample update kernels.
//
// A wave owns 32 samples.  A "tile" of U units is f32x16 t[ceil(U/32)] in the
// v_mfma_f32_32x32x2_f32 D layout: lane l = (h = l>>5, s = l&31) register r of
// block ib holds unit 32*ib + unit_of(r, h) of sample s.  A layer
//     out^T[N][32] = W[N][K] . in^T[K][32]
// runs as MFMAs whose B operand is the lane's own input register (no data
// movement between layers inside the MFMA chain) and whose A operand is a
// weight fragment read from a pre-packed "fragment image" of W in HBM/L2:
//     Wf[((ob*NBI + ib)*4 + rq)*64 + lane] (float4, element j) =
//        W[out_map(ob, lane&31)][in_map(ib, 4*rq + j, lane>>5)]
// so every wave-instruction is one coalesced 1 KiB dwordx4 load.
// Hidden activations are handed between layers through a per-wave LDS image
// [unit][32 samples] (conflict-free ds_read_b32/ds_write_b32).
#pragma once
#include "common.h"

namespace spp {
// Cross-lane hand-over through the wave's LDS image.  Most layer boundaries are same-lane (a lane
// reads back the units it wrote), but the heads' pairing layout (row j0 + 8h) and the natural
// layout (row u + 4h) map a row to different lane halves.  Per-thread program order says nothing
// about another lane's store, so without a fence the compiler may schedule such a read above the
// writing lane's store whenever it can prove the two per-lane addresses distinct; this compiler
// memory barrier pins every store before it ahead of every load after it (no instruction emitted;
// LDS operations of one wave complete in order).
#define SPP_XLANE_SYNC() asm volatile("" ::: "memory")


// Region timing of the phase kernels (profiling builds only, -DSPP_PROF): each
// wave accumulates s_memtime deltas per region in LDS, flushed to g_tprof.
// sched_barrier keeps the scheduler from moving a region's code across its marker.
#ifdef SPP_PROF
__device__ unsigned long long g_tprof[64];
__shared__ unsigned long long s_tprof[4][32];
__shared__ unsigned long long s_tlast[4];
#ifdef SPP_PROF_DRAIN  // charge each region with the memory traffic it left in flight
#define SPP_TP_DRAIN() asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory")
#else
#define SPP_TP_DRAIN()
#endif
#define SPP_TP_INIT()                                                            \
  {                                                                              \
    const int w_ = threadIdx.x >> 6;                                             \
    if ((threadIdx.x & 63) < 32 && w_ < 4) s_tprof[w_][threadIdx.x & 63] = 0;    \
    if ((threadIdx.x & 63) == 0 && w_ < 4) s_tlast[w_] = clock64();              \
  }
#define SPP_TP(k)                                                                \
  {                                                                              \
    __builtin_amdgcn_sched_barrier(0);                                           \
    SPP_TP_DRAIN();                                                              \
    const unsigned long long t_ = clock64();                                     \
    __builtin_amdgcn_sched_barrier(0);                                           \
    const int w_ = threadIdx.x >> 6;                                             \
    if ((threadIdx.x & 63) == 0 && w_ < 4) {                                     \
      s_tprof[w_][k] += t_ - s_tlast[w_];                                        \
      s_tlast[w_] = t_;                                                          \
    }                                                                            \
  }
#define SPP_TP_FLUSH()                                                           \
  {                                                                              \
    const int w_ = threadIdx.x >> 6, l_ = threadIdx.x & 63;                      \
    if (l_ < 32 && w_ < 4) atomicAdd(&g_tprof[l_], s_tprof[w_][l_]);             \
  }
#else
#define SPP_TP_INIT()
#define SPP_TP(k)
#define SPP_TP_FLUSH()
#endif
// markers inside the dense layers (off with -DSPP_PROF_NODENSE: then a kernel's
// top-level regions include their layers)
#if defined(SPP_PROF) && !defined(SPP_PROF_NODENSE)
#define SPP_TPD(k) SPP_TP(k)
#else
#define SPP_TPD(k)
#endif
// markers between the dense layers of the critics' backward (only with -DSPP_PROF_NODENSE)
#if defined(SPP_PROF) && defined(SPP_PROF_NODENSE)
#define SPP_TPN(k) SPP_TP(k)
#else
#define SPP_TPN(k)
#endif

// ---------------------------------------------------------------- layout maps
// How (block, register, half) positions of a tile map to logical indices of a
// vector.  Used by the pack kernels (device) and by loaders.
enum MapKind : int {
  MAP_NAT = 0,      // logical = 32*blk + unit_of(r,h), valid < n0
  MAP_CAT = 1,      // blocks < nb0: natural (< n0); then natural second segment (< n1) -> off1 + u
  MAP_PAIR = 2,     // actor heads: r<8: mu_j, r>=8: logsig_j, j = 16*blk + 8*h + (r&7), valid j < n0;
                    // logical mu_j = j, logsig_j = n0 + j
  MAP_PAIR_MU = 3,  // MAP_PAIR restricted to the mu slots (r < 8): logical j
  MAP_CAT_PAIRMU = 4  // blocks < nb0 natural (< n0); then MAP_PAIR_MU (< n1) -> off1 + j
};

struct MapDesc {
  int kind, n0, nb0, n1, off1;
};

__host__ __device__ inline int map_index(const MapDesc& m, int blk, int r, int h) {
  int u = (r & 3) + 8 * (r >> 2) + 4 * h;
  switch (m.kind) {
    case MAP_NAT: {
      int x = 32 * blk + u;
      return x < m.n0 ? x : -1;
    }
    case MAP_CAT: {
      if (blk < m.nb0) {
        int x = 32 * blk + u;
        return x < m.n0 ? x : -1;
      }
      int x = 32 * (blk - m.nb0) + u;
      return x < m.n1 ? m.off1 + x : -1;
    }
    case MAP_PAIR: {
      int j = 16 * blk + 8 * h + (r & 7);
      if (j >= m.n0) return -1;
      return r < 8 ? j : m.n0 + j;
    }
    case MAP_PAIR_MU: {
      int j = 16 * blk + 8 * h + (r & 7);
      return (r < 8 && j < m.n0) ? j : -1;
    }
    case MAP_CAT_PAIRMU: {
      if (blk < m.nb0) {
        int x = 32 * blk + u;
        return x < m.n0 ? x : -1;
      }
      int j = 16 * (blk - m.nb0) + 8 * h + (r & 7);
      return (r < 8 && j < m.n1) ? m.off1 + j : -1;
    }
  }
  return -1;
}
// D-layout output row i of a 32-row block corresponds to register q, half h:
__host__ __device__ inline void row_to_pos(int i, int& q, int& h) {
  h = (i >> 2) & 1;
  q = (i & 3) + 4 * (i >> 3);
}

// Per-block count of valid register quads, packed 3 bits per block.
constexpr uint64_t rv_nat(int K, int nb) {
  uint64_t m = 0;
  for (int ib = 0; ib < nb; ++ib) m |= (uint64_t)(regs_valid(K, ib) / 4) << (3 * ib);
  return m;
}
constexpr uint64_t rv_cat(int n0, int nb0, int n1, int nb1) {
  return rv_nat(n0, nb0) | (rv_nat(n1, nb1) << (3 * nb0));
}
constexpr uint64_t rv_pair(int n, int nb) {  // all 4 quads of each pair block
  uint64_t m = 0;
  for (int ib = 0; ib < nb; ++ib) m |= (uint64_t)(16 * ib < n ? 4 : 0) << (3 * ib);
  return m;
}
constexpr uint64_t rv_pairmu(int n, int nb) {  // mu quads only (regs 0..7)
  uint64_t m = 0;
  for (int ib = 0; ib < nb; ++ib) m |= (uint64_t)(16 * ib < n ? 2 : 0) << (3 * ib);
  return m;
}
constexpr uint64_t rv_cat_pairmu(int n0, int nb0, int n1, int nb1) {
  return rv_nat(n0, nb0) | (rv_pairmu(n1, nb1) << (3 * nb0));
}
constexpr int rv_get(uint64_t m, int ib) { return (int)((m >> (3 * ib)) & 7); }
constexpr int rv_total(uint64_t m, int nb) {
  int t = 0;
  for (int ib = 0; ib < nb; ++ib) t += rv_get(m, ib);
  return t;
}
constexpr int chunk_of(int nq) { return nq <= 8 ? nq : (nq % 8 == 0 ? 8 : (nq % 4 == 0 ? 4 : nq)); }

// ---------------------------------------------------------------- dense layer
template <int N>
struct IC {
  static constexpr int value = N;
  __host__ __device__ constexpr operator int() const { return N; }
};
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(IC<B>{});
    static_for<B + 1, E>(f);
  }
}
// flat register-quad index q of a layer -> (input block, quad within block)
constexpr int q_ib(uint64_t RV, int NBI, int q) {
  int base = 0;
  for (int b = 0; b < NBI; ++b) {
    if (q < base + rv_get(RV, b)) return b;
    base += rv_get(RV, b);
  }
  return NBI - 1;
}
constexpr int q_rq(uint64_t RV, int NBI, int q) {
  int base = 0;
  for (int b = 0; b < NBI; ++b) {
    if (q < base + rv_get(RV, b)) return q - base;
    base += rv_get(RV, b);
  }
  return 0;
}

// Unit of register r for lane half 0; unit_of(r, h) = ru(r) + 4h.
__device__ __forceinline__ constexpr int ru(int r) { return (r & 3) + 8 * (r >> 2); }

// Bias of output block ob from a natural-order LDS table biasL[32*NBO]:
// register q of lane half h is unit 32*ob + ru(q) + 4h (4 consecutive units per
// register quad -> one broadcast ds_read_b128 each).
__device__ __forceinline__ f32x16 bias_tile(const float* biasL, int ob, int h) {
  f32x16 acc;
  const float4* b4 = reinterpret_cast<const float4*>(biasL + 32 * ob + 4 * h);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float4 v = b4[2 * k];  // units 8k + 4h .. 8k + 4h + 3
    acc[4 * k + 0] = v.x;
    acc[4 * k + 1] = v.y;
    acc[4 * k + 2] = v.z;
    acc[4 * k + 3] = v.w;
  }
  return acc;
}

// Weight fragments through a buffer resource: wave-uniform byte offset in
// soffset (pinned in an SGPR), the lane's 16 B slot in ONE shared voffset VGPR,
// so no per-layer 64-bit lane addresses exist to be hoisted out of the tile loop.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t rsrc_n(const void* p, int nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, nbytes, 0x00020000);
}
__device__ __forceinline__ rsrc_t rsrc(const void* p) { return rsrc_n(p, 0x7fffffff); }
__device__ __forceinline__ float4 wfrag(rsrc_t w, uint32_t lane16, int off) {
  asm volatile("" : "+s"(off));
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(w, lane16, off, 0));
}

// Register-input layer (small K): out blocks ob = 0..NBO-1 (runtime), acc
// initialised from the LDS bias table (nullptr -> 0), epi(ob, acc) consumes each
// block.  Weight image ob-major: Wf[((ob*NBI + ib)*4 + rq)*64 + lane].
// Weight fragments stream through a 2-deep register ring of CH float4 so the
// next chunk's loads are in flight while the current chunk's MFMAs issue.
// Software-pipelined by one block: block ob's MFMA chain is issued before block
// ob-1's epilogue, so the epilogue's VALU / LDS / store work fills the chain's
// MFMA issue gaps instead of serialising behind it.
template <int NBI, uint64_t RV, bool BIAS, typename Epi>
__device__ __forceinline__ void dense_impl(const float4* __restrict__ Wf, int NBO, const f32x16 (&in)[NBI],
                                           const float* biasL, Epi&& epi) {
  constexpr int NQ = rv_total(RV, NBI);
  static_assert(NQ > 0, "empty layer");
  constexpr int CH = chunk_of(NQ);
  constexpr int NC = NQ / CH;
  static_assert(NQ % CH == 0, "chunking");
  const int lane = lane_id();
  const int h = lane >> 5;
  const rsrc_t wr = rsrc(Wf);
  const uint32_t l16 = 16u * lane;
  constexpr int OBSTRIDE = NBI * 4 * 64 * 16;  // bytes per output block
  float4 cur[CH];
  static_for<0, CH>([&](auto I) {
    constexpr int q = decltype(I)::value;
    cur[q] = wfrag(wr, l16, (q_ib(RV, NBI, q) * 4 + q_rq(RV, NBI, q)) * 1024);
  });
  auto chain = [&](int ob) {
    f32x16 acc;
    if constexpr (BIAS) acc = bias_tile(biasL, ob, h);
    else acc = zero16();
    const int obn = ob + 1 < NBO ? ob + 1 : ob;
    static_for<0, NC>([&](auto C) {
      constexpr int c = decltype(C)::value;
      constexpr int nc = (c + 1 < NC) ? c + 1 : 0;
      const int wn = ((c + 1 < NC) ? ob : obn) * OBSTRIDE;
      float4 nxt[CH];
      static_for<0, CH>([&](auto I) {
        constexpr int q = nc * CH + decltype(I)::value;
        nxt[decltype(I)::value] = wfrag(wr, l16, wn + (q_ib(RV, NBI, q) * 4 + q_rq(RV, NBI, q)) * 1024);
      });
      static_for<0, CH>([&](auto I) {
        constexpr int i = decltype(I)::value;
        constexpr int q = c * CH + i;
        constexpr int ib = q_ib(RV, NBI, q);
        constexpr int rq = q_rq(RV, NBI, q);
        acc = mfma(cur[i].x, in[ib][4 * rq + 0], acc);
        acc = mfma(cur[i].y, in[ib][4 * rq + 1], acc);
        acc = mfma(cur[i].z, in[ib][4 * rq + 2], acc);
        acc = mfma(cur[i].w, in[ib][4 * rq + 3], acc);
      });
#pragma unroll
      for (int i = 0; i < CH; ++i) cur[i] = nxt[i];
    });
    return acc;
  };
  SPP_TPD(23);
  f32x16 prev = chain(0);
#pragma unroll 1
  for (int ob = 1; ob < NBO; ++ob) {
    const f32x16 acc = chain(ob);
    epi(ob - 1, prev);
    prev = acc;
  }
  SPP_TPD(24);
  epi(NBO - 1, prev);
  SPP_TPD(25);
}

constexpr int cgcd(int a, int b) { return b ? cgcd(b, a % b) : a; }

// 256-input layer reading its input straight from the wave's LDS image
// img[unit][32] (all 8 blocks), all NBO output blocks accumulated at once
// (acc[NBO] lives in the accumulation registers), input blocks streamed in the
// outer loop.  Weight image ib-major: Wf[((ib*NBO + ob)*4 + rq)*64 + lane], so
// the whole layer is ONE linear stream of 1 KiB fragments, consumed in chunks
// of CH float4 (= one (input block, output block) pair) through a D-deep
// register ring: chunk g+D-1's loads are issued (pinned by a scheduling
// barrier) before chunk g's MFMAs, i.e. (D-1)*CH*4 MFMAs of latency cover per
// load.  The last input block is peeled: output block ob is final after its
// chunk there, and its epilogue epi(ob, acc) is issued together with block
// ob+1's MFMAs.  All image reads happen before the peeled block, so epi may
// overwrite img.
template <int NBO, bool BIAS, typename Epi>
__device__ __forceinline__ void dense_lds_impl(const float4* __restrict__ Wf, const float* img, const float* biasL,
                                               Epi&& epi) {
  constexpr int NQ = NBO * 4;               // float4 per input block
  constexpr int CH = 4;                     // float4 per chunk
  constexpr int NCI = NQ / CH;              // chunks per input block (= NBO)
  constexpr int D = 4;                      // ring depth (chunks)
  constexpr int U = NCI * D / cgcd(NCI, D);  // chunks per loop iteration
  constexpr int IBU = U / NCI;              // input blocks per iteration
  constexpr int G = 8 * NCI;                // chunks in the layer
  static_assert(8 % IBU == 0, "input blocks per iteration");
  constexpr int NIT = 8 / IBU;
  const int lane = lane_id();
  const int h = lane >> 5;
  const float* l = img + 4 * h * 32 + (lane & 31);
  const rsrc_t wr = rsrc(Wf);
  const uint32_t l16 = 16u * lane;
  f32x16 acc[NBO];
  static_for<0, NBO>([&](auto O) {
    if constexpr (BIAS) acc[O] = bias_tile(biasL, O, h);
    else acc[O] = zero16();
  });
  float4 ring[D][CH];
  static_for<0, D - 1>([&](auto I) {
    static_for<0, CH>([&](auto J) { ring[I][J] = wfrag(wr, l16, ((int)I * CH + (int)J) * 1024); });
  });
  f32x16 xin[IBU];
  static_for<0, IBU>([&](auto K) {
#pragma unroll
    for (int r = 0; r < 16; ++r) xin[K][r] = l[(32 * (int)K + ru(r)) * 32];
  });
  // chunk u of iteration it: refill the ring D-1 chunks ahead, then its MFMAs
  auto step = [&](auto UC, int it) {
    constexpr int u = UC;
    constexpr int sn = (u + D - 1) % D;
    const int gn = it * U + u + D - 1;
    if (gn < G) {
      static_for<0, CH>([&](auto J) { ring[sn][J] = wfrag(wr, l16, (gn * CH + (int)J) * 1024); });
    }
    __builtin_amdgcn_sched_barrier(0);
    constexpr int s = u % D;
    constexpr int kb = u / NCI;
    constexpr int ob = u % NCI;
    static_for<0, CH>([&](auto J) {
      constexpr int rq = J;
      acc[ob] = mfma(ring[s][J].x, xin[kb][4 * rq + 0], acc[ob]);
      acc[ob] = mfma(ring[s][J].y, xin[kb][4 * rq + 1], acc[ob]);
      acc[ob] = mfma(ring[s][J].z, xin[kb][4 * rq + 2], acc[ob]);
      acc[ob] = mfma(ring[s][J].w, xin[kb][4 * rq + 3], acc[ob]);
    });
  };
  SPP_TPD(20);
#pragma unroll 1
  for (int it = 0; it < NIT - 1; ++it) {
    f32x16 xnx[IBU];
    static_for<0, IBU>([&](auto K) {
#pragma unroll
      for (int r = 0; r < 16; ++r) xnx[K][r] = l[(32 * ((it + 1) * IBU + (int)K) + ru(r)) * 32];
    });
    static_for<0, U>([&](auto UC) { step(UC, it); });
    static_for<0, IBU>([&](auto K) { xin[K] = xnx[K]; });
  }
  static_for<0, U>([&](auto UC) {
    step(UC, NIT - 1);
    constexpr int u = UC;
    if constexpr (u / NCI == IBU - 1 && u % NCI >= 1) epi(IC<u % NCI - 1>{}, acc[u % NCI - 1]);
  });
  SPP_TPD(21);
  epi(IC<NBO - 1>{}, acc[NBO - 1]);
  SPP_TPD(22);
}

// ---------------------------------------------------------------- bf16 MFMA layers
// v_mfma_f32_32x32x16_bf16: lane (i = l&31, h = l>>5) holds A[i][k = 8h + j] and
// B[k = 8h + j][i], j = 0..7; D layout as the f32 form.  The input tile's registers
// 8s .. 8s+7 (s = 0, 1) of block ib, converted to bf16 (RNE), are k-step s of that block:
// element j of lane half h is unit unit_of(8s + j, h) (the k order inside a step is the
// D-layout row order).  Weight images hold the matching 8 bf16 per lane:
//   Wf16[((ob*NBI + ib)*2 + s)*64 + lane] (ob-major) / [((ib*NBO + ob)*2 + s)*64 + lane]
//   element j = bf16(W[out_map(ob, lane&31)][in_map(ib, 8s + j, lane>>5)])
// (k_pack_matrix with PackJob::bf16).  Accumulation is fp32.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x16 mfma16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x8 frag16(float4 v) { return __builtin_bit_cast(bf16x8, v); }
template <int S>
__device__ __forceinline__ bf16x8 to_bf16x8(const f32x16& t) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)t[8 * S + j];
  return r;
}
// k-steps of block ib that carry a valid register quad
constexpr int st_get(uint64_t RV, int ib) { return (rv_get(RV, ib) + 1) / 2; }
constexpr int st_total(uint64_t RV, int nb) {
  int t = 0;
  for (int ib = 0; ib < nb; ++ib) t += st_get(RV, ib);
  return t;
}
constexpr int st_ib(uint64_t RV, int NBI, int q) {
  int base = 0;
  for (int b = 0; b < NBI; ++b) {
    if (q < base + st_get(RV, b)) return b;
    base += st_get(RV, b);
  }
  return NBI - 1;
}
constexpr int st_s(uint64_t RV, int NBI, int q) {
  int base = 0;
  for (int b = 0; b < NBI; ++b) {
    if (q < base + st_get(RV, b)) return q - base;
    base += st_get(RV, b);
  }
  return 0;
}

// Register-input layer, bf16 MFMA: the inputs are converted once, every output block's
// fragments (one 16-B buffer load per k-step) are fetched one block ahead, and block ob's
// MFMA chain is issued before block ob-1's epilogue (as dense_impl).
template <int NBI, uint64_t RV, bool BIAS, typename Epi>
__device__ __forceinline__ void dense16_impl(const float4* __restrict__ Wf, int NBO, const f32x16 (&in)[NBI],
                                             const float* biasL, Epi&& epi) {
  constexpr int NS = st_total(RV, NBI);
  static_assert(NS > 0, "empty layer");
  const int lane = lane_id();
  const int h = lane >> 5;
  const rsrc_t wr = rsrc(Wf);
  const uint32_t l16 = 16u * lane;
  constexpr int OBSTRIDE = NBI * 2 * 64 * 16;  // bytes per output block
  bf16x8 bin[NS];
  static_for<0, NS>([&](auto Q) {
    constexpr int q = Q;
    bin[q] = to_bf16x8<st_s(RV, NBI, q)>(in[st_ib(RV, NBI, q)]);
  });
  float4 cur[NS];
  static_for<0, NS>([&](auto Q) {
    constexpr int q = Q;
    cur[q] = wfrag(wr, l16, (st_ib(RV, NBI, q) * 2 + st_s(RV, NBI, q)) * 1024);
  });
  auto chain = [&](int ob) {
    f32x16 acc;
    if constexpr (BIAS) acc = bias_tile(biasL, ob, h);
    else acc = zero16();
    const int wn = (ob + 1 < NBO ? ob + 1 : ob) * OBSTRIDE;
    float4 nxt[NS];
    static_for<0, NS>([&](auto Q) {
      constexpr int q = Q;
      nxt[q] = wfrag(wr, l16, wn + (st_ib(RV, NBI, q) * 2 + st_s(RV, NBI, q)) * 1024);
    });
    static_for<0, NS>([&](auto Q) { acc = mfma16(frag16(cur[(int)Q]), bin[(int)Q], acc); });
#pragma unroll
    for (int q = 0; q < NS; ++q) cur[q] = nxt[q];
    return acc;
  };
  f32x16 prev = chain(0);
#pragma unroll 1
  for (int ob = 1; ob < NBO; ++ob) {
    const f32x16 acc = chain(ob);
    epi(ob - 1, prev);
    prev = acc;
  }
  epi(NBO - 1, prev);
}

// 256-input layer from the LDS image, bf16 MFMA: all NBO output blocks accumulate at once;
// input block ib+1's fragments (2 per output block, 128 VGPRs for both buffers) are loaded
// while block ib's MFMAs issue, and block ib+1's LDS image reads follow block ib's MFMAs.
// A finer ring (4-fragment chunks, 4 / 6 / 8 deep: 12 / 20 / 28 fragments in flight instead
// of 16) measured slower: Ant bf16 critic phase 1.668 ms -> 1.752 / 1.721 / 1.731 ms
// (profiles/r05/ab_bf16_ring.txt); a third whole block spills.
// Output-block chains (all 8 input blocks converted to bf16 registers once, one 16-MFMA chain per
// output block with the previous block's epilogue under it, as dense16_impl) measured slower too:
// 1.686 -> 1.770 ms, bit-identical results.
template <int NBO, bool BIAS, typename Epi>
__device__ __forceinline__ void dense16_lds_impl(const float4* __restrict__ Wf, const float* img, const float* biasL,
                                                 Epi&& epi) {
  const int lane = lane_id();
  const int h = lane >> 5;
  const float* l = img + 4 * h * 32 + (lane & 31);
  const rsrc_t wr = rsrc(Wf);
  const uint32_t l16 = 16u * lane;
  f32x16 acc[NBO];
  static_for<0, NBO>([&](auto O) {
    if constexpr (BIAS) acc[O] = bias_tile(biasL, O, h);
    else acc[O] = zero16();
  });
  float4 fr[2][2 * NBO];
  static_for<0, 2 * NBO>([&](auto J) { fr[0][J] = wfrag(wr, l16, (int)J * 1024); });
  f32x16 x;
#pragma unroll
  for (int r = 0; r < 16; ++r) x[r] = l[ru(r) * 32];
  static_for<0, 8>([&](auto IB) {
    constexpr int ib = IB;
    const bf16x8 b0 = to_bf16x8<0>(x), b1 = to_bf16x8<1>(x);
    if constexpr (ib + 1 < 8) {
      static_for<0, 2 * NBO>([&](auto J) {
        fr[(ib + 1) & 1][J] = wfrag(wr, l16, ((ib + 1) * NBO * 2 + (int)J) * 1024);
      });
    }
    __builtin_amdgcn_sched_barrier(0);
    static_for<0, NBO>([&](auto O) {
      constexpr int ob = O;
      acc[ob] = mfma16(frag16(fr[ib & 1][2 * ob]), b0, acc[ob]);
      acc[ob] = mfma16(frag16(fr[ib & 1][2 * ob + 1]), b1, acc[ob]);
    });
    if constexpr (ib + 1 < 8) {
#pragma unroll
      for (int r = 0; r < 16; ++r) x[r] = l[(32 * (ib + 1) + ru(r)) * 32];
    }
  });
  static_for<0, NBO>([&](auto O) { epi(IC<(int)O>{}, acc[O]); });
}

// Front ends: BF selects the bf16 MFMA form (the weight images must be bf16 images).
template <int NBI, uint64_t RV, bool BF = false, typename Epi>
__device__ __forceinline__ void dense(const float4* __restrict__ Wf, int NBO, const f32x16 (&in)[NBI],
                                      const float* biasL, Epi&& epi) {
  if constexpr (BF) dense16_impl<NBI, RV, true>(Wf, NBO, in, biasL, static_cast<Epi&&>(epi));
  else dense_impl<NBI, RV, true>(Wf, NBO, in, biasL, static_cast<Epi&&>(epi));
}
template <int NBI, uint64_t RV, bool BF = false, typename Epi>
__device__ __forceinline__ void dense(const float4* __restrict__ Wf, int NBO, const f32x16 (&in)[NBI], decltype(nullptr),
                                      Epi&& epi) {
  if constexpr (BF) dense16_impl<NBI, RV, false>(Wf, NBO, in, nullptr, static_cast<Epi&&>(epi));
  else dense_impl<NBI, RV, false>(Wf, NBO, in, nullptr, static_cast<Epi&&>(epi));
}
template <int NBO, bool BF = false, typename Epi>
__device__ __forceinline__ void dense_lds(const float4* __restrict__ Wf, const float* img, const float* biasL,
                                          Epi&& epi) {
  if constexpr (BF) dense16_lds_impl<NBO, true>(Wf, img, biasL, static_cast<Epi&&>(epi));
  else dense_lds_impl<NBO, true>(Wf, img, biasL, static_cast<Epi&&>(epi));
}
template <int NBO, bool BF = false, typename Epi>
__device__ __forceinline__ void dense_lds(const float4* __restrict__ Wf, const float* img, decltype(nullptr),
                                          Epi&& epi) {
  if constexpr (BF) dense16_lds_impl<NBO, false>(Wf, img, nullptr, static_cast<Epi&&>(epi));
  else dense_lds_impl<NBO, false>(Wf, img, nullptr, static_cast<Epi&&>(epi));
}

// ---------------------------------------------------------------- loaders / stores

// Cache policy of the weight-gradient operand stores (activations / deltas that only k_dw reads
// back, in a later launch): SPP_OPST_AUX is the buffer instruction's cache-policy operand.
// 2 = nt: measured (profiles/r02/ab_nt.txt) the default policy's lines of this write stream
// evict weight fragments the other waves of the XCD re-read from L2 (critic phase 1.6-2.8 % faster).
#ifndef SPP_OPST_AUX
#define SPP_OPST_AUX 2
#endif
// cache policy of the feature-major streaming loads (staged minibatch, eps, scratch re-reads)
#ifndef SPP_STREAM_LD_AUX
#define SPP_STREAM_LD_AUX 0
#endif

// Feature-major arrays X[f][ld] are addressed as X[urow*ld + loff] with the
// wave-uniform row urow = 32*ib + ru(r) and ONE 32-bit per-lane offset
// loff = 4*h*ld + b (kept in a single VGPR; Bp*256 < 2^31 is asserted on the host).
__device__ __forceinline__ int lane_off(int ld, int b) { return 4 * (lane_id() >> 5) * ld + b; }

// LDS image [unit][32]: lane (h, s) reads unit 32*ib + unit_of(r, h) of sample s.
template <int NB>
__device__ __forceinline__ void lds_load(f32x16 (&t)[NB], const float* lds) {
  const int lane = lane_id();
  const float* l = lds + 4 * (lane >> 5) * 32 + (lane & 31);
#pragma unroll
  for (int ib = 0; ib < NB; ++ib)
#pragma unroll
    for (int r = 0; r < 16; ++r) t[ib][r] = l[(32 * ib + ru(r)) * 32];
}
// 2-D fp32 arrays in HBM through buffer resources: element (row, column) at
// byte offset row*ld4 + the lane's column offset vo.  row*ld4 is wave-uniform
// and pinned in an SGPR at each access (no CSE'd / hoisted per-row offsets).
// Unbounded accesses put it in soffset (no VALU); bounded ones (rsrc_n with the
// array's byte size) put it in voffset so the hardware range check returns 0 /
// drops the access for rows past the array (raw-buffer checks exclude soffset).
// Byte offsets stay below 2^31 (asserted on the host).
__device__ __forceinline__ int soff(int row, int ld4) {
  int so = row * ld4;
  asm volatile("" : "+s"(so));
  return so;
}
__device__ __forceinline__ float fm_ld(rsrc_t r, int row, int ld4, uint32_t vo) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, soff(row, ld4), SPP_STREAM_LD_AUX));
}
__device__ __forceinline__ void fm_st(rsrc_t r, int row, int ld4, uint32_t vo, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, vo, soff(row, ld4), 0);
}
__device__ __forceinline__ void fm_st_op(rsrc_t r, int row, int ld4, uint32_t vo, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, vo, soff(row, ld4), SPP_OPST_AUX);
}
// bf16 2-D array [rows][ld] addressed with the fp32 array's (row, ld4, vo): byte offsets halved.
// RNE conversion, the same one the bf16 MFMA operand packs use.
__device__ __forceinline__ void fm_st16(rsrc_t r, int row, int ld4, uint32_t vo, float v) {
  const __bf16 b = (__bf16)v;
  __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, b), r, vo >> 1, soff(row, ld4 >> 1),
                                        SPP_OPST_AUX);
}
// weight-gradient operand store: bf16 kernel sets write the activations / deltas k_dw reads as bf16
template <bool BF>
__device__ __forceinline__ void op_st(rsrc_t r, int row, int ld4, uint32_t vo, float v) {
  if constexpr (BF) fm_st16(r, row, ld4, vo, v);
  else fm_st_op(r, row, ld4, vo, v);
}
__device__ __forceinline__ float fm_ldb(rsrc_t r, int row, int ld4, uint32_t vo) {
  return __builtin_bit_cast(float,
                            __builtin_amdgcn_raw_buffer_load_b32(r, vo + (uint32_t)soff(row, ld4), 0, SPP_STREAM_LD_AUX));
}
__device__ __forceinline__ void fm_stb(rsrc_t r, int row, int ld4, uint32_t vo, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, vo + (uint32_t)soff(row, ld4), 0, 0);
}
// Global array X (nbytes long) with F logical rows at this lane's column;
// units >= F read 0 (feature-major X[f][ld]: nbytes = F*ld4; row-major [E][F]
// with ld4 = 4: nbytes = E*F*4, the select masks the neighbouring env's values).
template <int NB>
__device__ __forceinline__ void gm_load(f32x16 (&t)[NB], const float* X, int nbytes, int F, int ld4, uint32_t vo) {
  const rsrc_t xr = rsrc_n(X, nbytes);
  const int h4 = 4 * (lane_id() >> 5);
#pragma unroll
  for (int ib = 0; ib < NB; ++ib)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int u0 = 32 * ib + ru(r);
      if (u0 < F) {
        const float v = fm_ldb(xr, u0, ld4, vo);
        t[ib][r] = (u0 + h4 < F) ? v : 0.f;
      } else {
        t[ib][r] = 0.f;
      }
    }
}

// Hide a wave-uniform pointer from loop-invariant code motion (stops the
// compiler from hoisting hundreds of per-tile-invariant loads into registers).
template <class T>
__device__ __forceinline__ T* opaque(T* p) {
  asm volatile("" : "+s"(p));
  return p;
}

}  // namespace spp
