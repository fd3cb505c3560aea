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
struct IC { static constexpr int value = N; };
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

// out blocks ob = 0..NBO-1 (runtime), acc initialised from the packed bias
// image biasP[(ob*16 + q)*2 + h] (NULL -> 0), epi(ob, acc) consumes each block.
// Weight fragments stream through a 2-deep register ring of CH float4 so the
// next chunk's loads are in flight while the current chunk's MFMAs issue.
template <int NBI, uint64_t RV, typename Epi>
__device__ __forceinline__ void dense(const float4* __restrict__ Wf, int NBO, const f32x16 (&in)[NBI],
                                      const float* __restrict__ biasP, Epi&& epi) {
  constexpr int NQ = rv_total(RV, NBI);
  static_assert(NQ > 0, "empty layer");
  constexpr int CH = chunk_of(NQ);
  constexpr int NC = NQ / CH;
  static_assert(NQ % CH == 0, "chunking");
  const int lane = lane_id();
  const int h = lane >> 5;
  const float4* wl = Wf + lane;
  constexpr int OBSTRIDE = NBI * 4 * 64;
  float4 cur[CH];
  static_for<0, CH>([&](auto I) {
    constexpr int q = decltype(I)::value;
    cur[q] = wl[(q_ib(RV, NBI, q) * 4 + q_rq(RV, NBI, q)) * 64];
  });
#pragma unroll 1
  for (int ob = 0; ob < NBO; ++ob) {
    f32x16 acc;
    if (biasP) {
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[q] = biasP[(ob * 16 + q) * 2 + h];
    } else {
      acc = zero16();
    }
    const int obn = ob + 1 < NBO ? ob + 1 : ob;
    static_for<0, NC>([&](auto C) {
      constexpr int c = decltype(C)::value;
      constexpr int nc = (c + 1 < NC) ? c + 1 : 0;
      const float4* wn = wl + (size_t)((c + 1 < NC) ? ob : obn) * OBSTRIDE;
      float4 nxt[CH];
      static_for<0, CH>([&](auto I) {
        constexpr int q = nc * CH + decltype(I)::value;
        nxt[decltype(I)::value] = wn[(q_ib(RV, NBI, q) * 4 + q_rq(RV, NBI, q)) * 64];
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
    epi(ob, acc);
  }
}

// ---------------------------------------------------------------- loaders / stores
// Unit of register r for lane half 0; unit_of(r, h) = ru(r) + 4h.
__device__ __forceinline__ constexpr int ru(int r) { return (r & 3) + 8 * (r >> 2); }

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
// Feature-major global array X[f][ld] at this lane's column, units < F.
template <int NB>
__device__ __forceinline__ void gm_load(f32x16 (&t)[NB], const float* __restrict__ X, int F, int ld, int loff) {
  const int h4 = 4 * (lane_id() >> 5);
#pragma unroll
  for (int ib = 0; ib < NB; ++ib)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int u0 = 32 * ib + ru(r);
      t[ib][r] = (u0 + h4 < F) ? X[u0 * ld + loff] : 0.f;
    }
}

// Hide a wave-uniform pointer from loop-invariant code motion (stops the
// compiler from hoisting hundreds of per-tile-invariant loads into registers).
template <class T>
__device__ __forceinline__ T* opaque(T* p) {
  asm volatile("" : "+s"(p));
  return p;
}

// Packed-vector image vP[(ob*16 + q)*2 + h] (bias / last-layer weight vectors).
__device__ __forceinline__ float vec_at(const float* __restrict__ vP, int ob, int q) {
  return vP[(ob * 16 + q) * 2 + (lane_id() >> 5)];
}

}  // namespace spp
