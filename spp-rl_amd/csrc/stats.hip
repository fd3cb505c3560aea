// update_obs_mean_std (rltoolkit/buffer/replay_buffer.py:83-96) over the live replay rows
// X = obs[obs_idx[0:len)], by sample-bracketed exact selection: ONE read of X.
//
//   k_st_sample   S = min(len, 16384 | 65536) stride-sampled rows gathered by a grid (one row per
//                 thread), stored column-major as keys
//   k_st_bracket  one workgroup per column: the column's S keys in registers (16 | 64 per
//                 thread); the 4 bracket ranks (lo / hi around the 99th and the 1st percentile,
//                 sample ranks +-(4 sigma + 4)) by an 8-bit radix select whose histograms live in
//                 LDS (one histogram per distinct prefix, the bin search a wave-wide prefix scan)
//   k_st_pass     one read of every live row.  Lanes take (row, column) pairs of G = 64 / ob
//                 consecutive rows (one row, two column halves for ob > 64), so a wave's loads
//                 cover contiguous row runs.  Per lane: fp64 moments about a pivot; per target
//                 the count of keys outside the bracket on the far side and of keys equal to
//                 either bound.  Keys strictly inside a bracket are appended (LDS atomic cursor)
//                 to the workgroup's LDS list for (column, target), then copied to global
//                 lists; a full LDS list spills to a global overflow list.  Per-workgroup
//                 partials (moments, counts) go to a slab.  The grid is sized so every
//                 workgroup is resident at once (36 KiB of LDS: 4 per CU).
//   k_st_select   one workgroup per (column, target): reduces the slabs, places the 2 ranks numpy's
//                 'linear' percentile needs (floor((len-1) q) and the next) in
//                 [outside | = lo | candidates | = hi | outside], gathers the candidates into LDS
//                 (block prefix sum over the list lengths) and radix-selects them there from
//                 their common key prefix on.  mean / std and the running max (target 0) or
//                 min (target 1) are written here, and the overflow counter is re-zeroed for the
//                 next call.  A rank outside the bracket (a sample miss) falls back to a radix
//                 select over the column's raw data; more candidates than the LDS holds are
//                 visited in the global lists: the result is exact in every case.
// Keys: fkey() is the order-preserving uint32 image of a float (replay.hip).
#pragma once
#include "replay.h"

namespace spp {

constexpr int kStSampSmall = 16384;  // len <= kStBigLen: 16 keys x 1024 threads
constexpr int kStSampBig = 65536;    // beyond: 64 keys x 1024 threads
constexpr int64_t kStBigLen = 4000000;
constexpr int kStLdsKeys = 6144;     // per-workgroup LDS list space (keys), split over 2 ob lists
constexpr int kStOvfCap = 1 << 18;   // overflow keys per (column, target)
constexpr int kStPassThreads = 256;
constexpr int kStUnroll = 8;         // row groups per lane and iteration (halved for ob > 64); 2 iterations in flight
constexpr int kStNblkMax = 1024;     // pass workgroups (<= select threads)
constexpr int kStSelThreads = 1024;
constexpr int kStSelKeys = 32768;    // candidates gathered into the select workgroup's LDS

__host__ __device__ inline int st_list_cap(int ob) {
  const int c = kStLdsKeys / (2 * ob);
  return c < 256 ? c : 256;
}

// ---------------------------------------------------------------- LDS radix select
// Up to NQ ranks over a key set the workgroup visits with visit(fn): every thread calls fn(key)
// for the keys it owns.  Query q starts from the known bits qpre[q] / qmask[q] (the masks are
// whole-bit prefixes; queries may share a prefix, and then share a histogram).  On return
// qpre[q] is the key of rank qrank[q] (in the set restricted to the starting prefix).
// Needs blockDim.x >= 64 * NQ; qpre / qmask / qrank / hist in LDS.  At most MAXP digit passes are
// made; returns true if a query still has unknown digits then (the state is resumable: a later call
// over the keys that match the queries' prefixes continues it).
// Histograms hold kStCopies copies of every bin (lane & 7 picks the copy): the keys of a digit
// pass usually fall into a handful of bins, and same-address LDS atomics of one instruction
// serialise, so the copies cut that serialisation 8-fold.  hist: [NQ][256][kStCopies].
constexpr int kStCopies = 8;
template <int NQ, int MAXP = 4, class Visit>
__device__ bool st_radix_select(uint32_t* qpre, uint32_t* qmask, uint32_t* qrank, Visit visit, uint32_t* hist) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  [[maybe_unused]] int passes = 0;
  for (int shift = 24; shift >= 0; shift -= 8) {
    const uint32_t dm = 0xffu << shift;
    uint32_t pre[NQ], msk[NQ];
    int rep[NQ];
    bool act[NQ], any = false;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      pre[q] = qpre[q];
      msk[q] = qmask[q];
      act[q] = (msk[q] & dm) != dm;
      any |= act[q];
      rep[q] = q;
#pragma unroll
      for (int p = 0; p < q; ++p)
        if (rep[q] == q && pre[p] == pre[q] && msk[p] == msk[q]) rep[q] = rep[p];
    }
    if (!any) continue;  // uniform: every thread read the same state
    if constexpr (MAXP < 4) {
      if (passes == MAXP) return true;
      ++passes;
    }
    for (int i = tid; i < NQ * 256 * kStCopies; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    uint32_t* hl = hist + (lane & (kStCopies - 1));
    visit([&](uint32_t k) {
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        if (act[q] && rep[q] == q && (k & msk[q]) == pre[q])
          atomicAdd(&hl[(q * 256 + ((k >> shift) & 255)) * kStCopies], 1u);
    });
    __syncthreads();
    if (w < NQ && act[w]) {
      const uint4* hh = reinterpret_cast<const uint4*>(hist + (rep[w] * 256 + 4 * lane) * kStCopies);
      uint32_t c4[4], sum = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint4 a = hh[2 * j], b = hh[2 * j + 1];
        c4[j] = a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w;
        sum += c4[j];
      }
      uint32_t incl = sum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
      }
      const uint32_t excl = incl - sum, r = qrank[w];
      const bool mine = r >= excl && r < incl;
      const bool none = __ballot(mine) == 0ull;  // rank past the set (inconsistent input): last bin
      if (mine || (none && lane == 63)) {
        uint32_t acc = excl;
        int d = 4 * lane + 3;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (acc + c4[j] > r) {
            d = 4 * lane + j;
            break;
          }
          acc += c4[j];
        }
        qpre[w] = (pre[w] & ~dm) | ((uint32_t)d << shift);
        qmask[w] = msk[w] | dm;
        qrank[w] = r - acc;
      }
    }
    __syncthreads();
  }
  return false;
}

// ---------------------------------------------------------------- sample bracket
// k_st_sample: the S-row stride sample rows ((2s + 1) len) / (2S) (all rows when S == len), one
// sample row per thread over a grid of workgroups (a random-row gather needs many CUs' worth of
// outstanding misses), written column-major as keys: samp[c][s].
__global__ __launch_bounds__(256) void k_st_sample(ReplayDev r, int64_t len, int S, uint32_t* __restrict__ samp) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  const int ob = r.ob;
  const double step = (double)len / (2.0 * (double)S);  // exact enough for a sample; row s when S == len
  const int64_t row = min((int64_t)((double)(2 * s + 1) * step), len - 1);
  const float* x = r.obs + r.obs_idx[row] * ob;
  for (int c0 = 0; c0 < ob; c0 += 16) {
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = c0 + i < ob ? x[c0 + i] : 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (c0 + i < ob) samp[(int64_t)(c0 + i) * S + s] = fkey(v[i]);
  }
}

// bounds[(c*2 + t)*2 + {0,1}] = {lo, hi} keys of target t (0: 99th, 1: 1st percentile) from the
// column's S sample keys (KPT per thread, coalesced reads of samp[c][:]).
// The S keys of column c may come in segments (the data-parallel union sample, [world][ob][Sl] rank-major):
// key j at samp[(j / Sl) * seg + c * Sl + j % Sl]; one segment (Sl = S) is the local [ob][S] sample.
template <int KPT>
__global__ __launch_bounds__(1024) void k_st_bracket(const uint32_t* __restrict__ samp, int S,
                                                      uint32_t* __restrict__ bounds, int Sl, int64_t seg,
                                                      int mstd) {
  __shared__ __attribute__((aligned(16))) uint32_t hist[4 * 256 * kStCopies];
  __shared__ uint32_t qpre[4], qmask[4], qrank[4];
  __shared__ int qn;
  __shared__ int qt[4];
  const int c = blockIdx.x, tid = threadIdx.x;
  uint32_t v[KPT];
#pragma unroll
  for (int i = 0; i < KPT; ++i) {
    int j = i * 1024 + tid;
    j = j < S ? j : S - 1;
    v[i] = samp[(int64_t)(j / Sl) * seg + (int64_t)c * Sl + j % Sl];
  }
  if (tid == 0) {
    int n = 0;
    for (int t = 0; t < 2; ++t) {
      const double p = t == 0 ? 0.99 : 0.01;
      const int64_t f = (int64_t)floor(p * (double)(S - 1));
      const int m = (int)ceil(mstd * sqrt((double)S * p * (1.0 - p))) + 4;
      const int64_t lo_i = f - m, hi_i = f + 1 + m;
      // a bracket touching the sample's end extends to the key range's end (nothing outside)
      if (lo_i <= 0) {
        bounds[(c * 2 + t) * 2 + 0] = 0u;
      } else {
        qt[n] = (c * 2 + t) * 2 + 0;
        qrank[n] = (uint32_t)lo_i;
        ++n;
      }
      if (hi_i >= S - 1) {
        bounds[(c * 2 + t) * 2 + 1] = 0xffffffffu;
      } else {
        qt[n] = (c * 2 + t) * 2 + 1;
        qrank[n] = (uint32_t)hi_i;
        ++n;
      }
    }
    for (int q = 0; q < 4; ++q) {
      qpre[q] = 0;
      qmask[q] = q < n ? 0u : 0xffffffffu;  // unused slots: fully known (inactive)
    }
    qn = n;
  }
  __syncthreads();
  if (qn == 0) return;
  st_radix_select<4>(
      qpre, qmask, qrank,
      [&](auto&& fn) {
#pragma unroll
        for (int i = 0; i < KPT; ++i)
          if (i * 1024 + tid < S) fn(v[i]);
      },
      hist);
  if (tid < qn) bounds[qt[tid]] = qpre[tid];
}

// ---------------------------------------------------------------- the data pass
// Lane geometry: G rows per wave step, column half j of lane l is column colj(l, j) or -1.
__host__ __device__ inline int st_groups(int ob) { return ob <= 64 ? 64 / ob : 1; }
__device__ __forceinline__ int st_col(int ob, int lane, int j) {
  if (ob <= 64) return (j == 0 && lane < st_groups(ob) * ob) ? lane % ob : -1;
  const int c = lane + 64 * j;
  return c < ob ? c : -1;
}

struct StPassArgs {
  ReplayDev r;
  int64_t len;
  const uint32_t* bounds;  // [ob][2][2]
  const float* pivot;      // [ob] or null (first live row)
  double* part;            // [nblk][ob][2]       moment partials
  uint32_t* cpart;         // [nblk][ob][6]       count partials: per target outside, == lo, == hi
  uint32_t* wgl;           // [nblk][ob][2][cap]  per-workgroup candidate lists
  uint32_t* wgn;           // [nblk][ob][2]       keys in each list (<= cap)
  uint32_t* ovf;           // [ob][2][kStOvfCap]  keys past a list's capacity (row stride kStOvfCap)
  uint32_t* ovf_n;         // [ob][2]             (zero on entry; k_st_select re-zeroes)
  int cap;                 // st_list_cap(ob), or less (sppReplaySetObsStatsCaps)
  int ovf_cap;             // keys kept per overflow list: kStOvfCap, or less (sppReplaySetObsStatsCaps)
};

// WIDE: ob > 64 (two column halves per lane).  OFF32: the obs ring is < 4 GiB, so every load is a
// uniform 64-bit base plus ONE 32-bit per-lane byte offset (saddr form: 1 VGPR per address).
template <bool WIDE, bool OFF32>
__global__ __launch_bounds__(kStPassThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_st_pass(StPassArgs a) {
  constexpr int W = kStPassThreads / 64;
  constexpr int U = WIDE ? kStUnroll / 2 : kStUnroll;  // row groups per iteration (2 loads each if WIDE)
  __shared__ uint32_t lst[kStLdsKeys];   // [ob][2][cap]
  __shared__ uint32_t lcnt[256];         // [ob][2] list cursors
  __shared__ uint32_t ccnt[128 * 6];     // [ob][6] counts
  __shared__ double rs[W * 64][2][2];    // per lane: [j][s1, s2]
  const int ob = a.r.ob, G = st_groups(ob), cap = a.cap;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  for (int i = tid; i < 2 * ob; i += kStPassThreads) lcnt[i] = 0;
  for (int i = tid; i < 6 * ob; i += kStPassThreads) ccnt[i] = 0;
  const int64_t wv = (int64_t)blockIdx.x * W + w, nw = (int64_t)gridDim.x * W;
  const int g = ob <= 64 ? lane / ob : 0;
  const int col[2] = {st_col(ob, lane, 0), WIDE ? st_col(ob, lane, 1) : -1};
  const float* p0 = a.pivot ? a.pivot : a.r.obs + a.r.obs_idx[0] * ob;
  double piv[2];
  uint32_t lo[2][2], hi[2][2];
  double s1[2] = {0.0, 0.0}, s2[2] = {0.0, 0.0};
  uint32_t cout[2][2] = {{0, 0}, {0, 0}}, ceq[2][2] = {{0, 0}, {0, 0}};  // ceq: == lo | == hi << 16
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = col[j] < 0 ? 0 : col[j];
    piv[j] = (double)p0[c];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      lo[j][t] = a.bounds[(c * 2 + t) * 2 + 0];
      hi[j][t] = a.bounds[(c * 2 + t) * 2 + 1];
    }
  }
  __syncthreads();
  const int64_t ngroups = (a.len + G - 1) / G;
  // Software pipeline over iterations of U row groups: iteration i+1's rows are
  // requested (their obs_idx came one iteration earlier) and iteration i+2's obs_idx issued
  // before iteration i's keys are classified, so the data pass overlaps its own compute.
  // Every load is unconditional (clamped row / column), so none sits in a branch with its wait.
  const int64_t last = a.len - 1;
  const int c0 = col[0] < 0 ? 0 : col[0], c1 = col[1] < 0 ? 0 : col[1];
  const int64_t it_rows = nw * U;  // row groups per iteration (all waves)
  const char* obs_b = reinterpret_cast<const char*>(a.r.obs);
  const char* idx_b = reinterpret_cast<const char*>(a.r.obs_idx);
  auto ld_idx = [&](int64_t row) -> int {  // ring slots < capacity < 2^31
    if constexpr (OFF32) return *reinterpret_cast<const int*>(idx_b + (uint32_t)row * 8u);  // low word
    else return (int)a.r.obs_idx[row];
  };
  auto ld_x = [&](int slot, int c) -> float {
    if constexpr (OFF32) return *reinterpret_cast<const float*>(obs_b + ((uint32_t)slot * (uint32_t)ob + (uint32_t)c) * 4u);
    else return a.r.obs[(int64_t)slot * ob + c];
  };
  // validity is kept apart from the loaded slot (a select on the loaded value lets the compiler
  // sink the load into a branch with its own wait)
  auto idx_load = [&](int64_t rg0, int (&n)[U], uint32_t& vm) {
    vm = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = (rg0 + u * nw) * G + g;
      n[u] = ld_idx(min(row, last));
      vm |= (uint32_t)(row < a.len && col[0] >= 0) << u;
    }
  };
  auto x_load = [&](const int (&n)[U], float (&x)[2][U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) x[0][u] = ld_x(n[u], c0);
    if constexpr (WIDE) {
#pragma unroll
      for (int u = 0; u < U; ++u) x[1][u] = ld_x(n[u], c1);
    }
  };
  // bracket widths: key in [lo, hi]  <=>  key - lo <= hi - lo  (unsigned; lo <= hi by construction)
  uint32_t wd[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int t = 0; t < 2; ++t) wd[j][t] = hi[j][t] - lo[j][t];
  // one key: moments, far-side counts; the rare keys inside a bracket take the slow path.
  // V: the iteration has rows past len (per-row validity); full iterations skip it.
  auto proc = [&](auto VC, int j, float xv, bool v) {
    constexpr bool V = decltype(VC)::value;
    double d = (double)xv - piv[j];
    if constexpr (V) d = v ? d : 0.0;
    s1[j] += d;
    s2[j] = fma(d, d, s2[j]);
    const uint32_t key = fkey(xv);
    bool o0 = key > hi[j][0], o1 = key < lo[j][1];
    bool in0 = key - lo[j][0] <= wd[j][0], in1 = key - lo[j][1] <= wd[j][1];
    if constexpr (V) {
      o0 = o0 && v; o1 = o1 && v; in0 = in0 && v; in1 = in1 && v;
    }
    cout[j][0] += (uint32_t)o0;
    cout[j][1] += (uint32_t)o1;
    if (in0 || in1) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (!(t ? in1 : in0)) continue;
        const uint32_t l = lo[j][t], h = hi[j][t];
        if (key == l) {
          ceq[j][t] += 1u;
        } else if (key == h) {
          ceq[j][t] += 1u << 16;
        } else {
          const int ct = col[j] * 2 + t;
          const uint32_t f = atomicAdd(&lcnt[ct], 1u);
          if (f < (uint32_t)cap) {
            lst[ct * cap + f] = key;
          } else {
            const uint32_t o = atomicAdd(&a.ovf_n[ct], 1u);
            if (o < (uint32_t)a.ovf_cap) a.ovf[(int64_t)ct * kStOvfCap + o] = key;
          }
        }
      }
    }
  };
  // Two-deep pipeline: iteration i+1's rows are requested (their obs_idx arrived one iteration
  // earlier) and iteration i+2's obs_idx issued before iteration i's keys are classified.
  int nA[U];
  uint32_t vA, vX;
  float xA[2][U];
  idx_load(wv, nA, vA);
  x_load(nA, xA);
  vX = vA;
  idx_load(wv + it_rows, nA, vA);
  for (int64_t rg0 = wv; rg0 < ngroups; rg0 += it_rows) {
    float xB[2][U];
    x_load(nA, xB);
    const uint32_t v = vX;
    vX = vA;
    idx_load(rg0 + 2 * it_rows, nA, vA);
    // every row of the iteration is live: lanes without a column are masked once, no per-key validity
    const bool full = (rg0 + (int64_t)(U - 1) * nw) * G + G - 1 < a.len;
    if (full) {
      if (col[0] >= 0) {
#pragma unroll
        for (int u = 0; u < U; ++u) proc(IC<0>{}, 0, xA[0][u], true);
      }
      if constexpr (WIDE) {
        if (col[1] >= 0) {
#pragma unroll
          for (int u = 0; u < U; ++u) proc(IC<0>{}, 1, xA[1][u], true);
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) proc(IC<1>{}, 0, xA[0][u], (v >> u) & 1u);
      if constexpr (WIDE) {
#pragma unroll
        for (int u = 0; u < U; ++u) proc(IC<1>{}, 1, xA[1][u], ((v >> u) & 1u) && col[1] >= 0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xA[0][u] = xB[0][u];
      if constexpr (WIDE) xA[1][u] = xB[1][u];
    }
  }
  // lane partials -> LDS -> one partial per (workgroup, column)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    rs[tid][j][0] = s1[j];
    rs[tid][j][1] = s2[j];
    if (col[j] >= 0) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (cout[j][t]) atomicAdd(&ccnt[col[j] * 6 + 3 * t + 0], cout[j][t]);
        if (ceq[j][t] & 0xffffu) atomicAdd(&ccnt[col[j] * 6 + 3 * t + 1], ceq[j][t] & 0xffffu);
        if (ceq[j][t] >> 16) atomicAdd(&ccnt[col[j] * 6 + 3 * t + 2], ceq[j][t] >> 16);
      }
    }
  }
  __syncthreads();
  for (int c = tid; c < ob; c += kStPassThreads) {
    double m1 = 0.0, m2 = 0.0;
    const int j = ob <= 64 ? 0 : c / 64;
    for (int q = 0; q < W; ++q)
      for (int gg = 0; gg < G; ++gg) {
        const int l = 64 * q + (ob <= 64 ? gg * ob + c : c - 64 * j);
        m1 += rs[l][j][0];
        m2 += rs[l][j][1];
      }
    a.part[((int64_t)blockIdx.x * ob + c) * 2 + 0] = m1;
    a.part[((int64_t)blockIdx.x * ob + c) * 2 + 1] = m2;
  }
  for (int i = tid; i < 6 * ob; i += kStPassThreads) a.cpart[(int64_t)blockIdx.x * ob * 6 + i] = ccnt[i];
  for (int i = tid; i < 2 * ob; i += kStPassThreads)
    a.wgn[(int64_t)blockIdx.x * ob * 2 + i] = min(lcnt[i], (uint32_t)cap);
  uint32_t* dst = a.wgl + (int64_t)blockIdx.x * ob * 2 * cap;
  for (int i = tid; i < 2 * ob * cap; i += kStPassThreads)
    if ((uint32_t)(i % cap) < lcnt[i / cap]) dst[i] = lst[i];
}

inline void st_launch_pass(const StPassArgs& pa, int nblk, hipStream_t st) {
  const bool wide = pa.r.ob > 64;
  const bool off32 = (uint64_t)pa.r.cap * (uint64_t)pa.r.ob * 4u < (1ull << 32) && pa.len < ((int64_t)1 << 29);
  if (wide && off32) hipLaunchKernelGGL((k_st_pass<true, true>), dim3(nblk), dim3(kStPassThreads), 0, st, pa);
  else if (wide) hipLaunchKernelGGL((k_st_pass<true, false>), dim3(nblk), dim3(kStPassThreads), 0, st, pa);
  else if (off32) hipLaunchKernelGGL((k_st_pass<false, true>), dim3(nblk), dim3(kStPassThreads), 0, st, pa);
  else hipLaunchKernelGGL((k_st_pass<false, false>), dim3(nblk), dim3(kStPassThreads), 0, st, pa);
}

// ---------------------------------------------------------------- select
struct StSelArgs {
  ReplayDev r;
  int64_t len;
  int nblk, cap;
  const double* part;
  const uint32_t* cpart;
  const uint32_t* bounds;
  const uint32_t* wgl;
  const uint32_t* wgn;
  const uint32_t* ovf;
  uint32_t* ovf_n;
  const float* pivot;
  float *mean, *std, *max_out, *min_out;
  int first_update;
  int ovf_cap;
};

__global__ __launch_bounds__(kStSelThreads) void k_st_select(StSelArgs a) {
  constexpr int T = kStSelThreads;
  constexpr int NW = T / 64;
  __shared__ uint32_t cand[kStSelKeys];
  __shared__ double rd[2][NW];
  __shared__ uint32_t rc[4][NW];
  __shared__ __attribute__((aligned(16))) uint32_t hist[2 * 256 * kStCopies];
  __shared__ uint32_t vals[2], qpre[2], qmask[2], qrank[2];
  __shared__ int qslot[2], nq, mode;  // mode: 0 candidates in LDS, 1 raw column, 2 global lists
  const int c = blockIdx.x, t = blockIdx.y, tid = threadIdx.x, ob = a.r.ob;
  const int lane = tid & 63, wv = tid >> 6;
  const int ct = c * 2 + t;
  const int cap = a.cap;
  // ---- moments (target 0), this target's counts, list lengths: thread b owns workgroup b
  const int b = tid;
  double m1 = 0.0, m2 = 0.0;
  uint32_t cc[3] = {0, 0, 0}, nb = 0;
  if (b < a.nblk) {
    if (t == 0) {
      m1 = a.part[((int64_t)b * ob + c) * 2 + 0];
      m2 = a.part[((int64_t)b * ob + c) * 2 + 1];
    }
#pragma unroll
    for (int f = 0; f < 3; ++f) cc[f] = a.cpart[((int64_t)b * ob + c) * 6 + 3 * t + f];
    nb = a.wgn[(int64_t)b * ob * 2 + ct];
  }
  // inclusive wave scan of the list lengths (candidate offsets)
  uint32_t incl = nb;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  m1 = wave_sum_d(m1);
  m2 = wave_sum_d(m2);
#pragma unroll
  for (int f = 0; f < 3; ++f)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cc[f] += __shfl_xor(cc[f], o, 64);
  if (lane == 63) rc[3][wv] = incl;
  if (lane == 0) {
    rd[0][wv] = m1;
    rd[1][wv] = m2;
#pragma unroll
    for (int f = 0; f < 3; ++f) rc[f][wv] = cc[f];
  }
  __syncthreads();
  uint32_t woff = 0;
  for (int q = 0; q < wv; ++q) woff += rc[3][q];
  const uint32_t off = woff + incl - nb;  // this workgroup list's first slot
  const int64_t n = a.len;
  const uint32_t novf_raw = a.ovf_n[ct];
  const uint32_t novf = min(novf_raw, (uint32_t)a.ovf_cap);
  if (tid == 0) {
    double s1 = 0.0, s2 = 0.0;
    int64_t out = 0, eql = 0, eqh = 0, nl = 0;
    // rolled: unrolled, the 6 x 16 partials were all loaded up front and spilled to scratch
#pragma unroll 1
    for (int q = 0; q < NW; ++q) {
      s1 += rd[0][q];
      s2 += rd[1][q];
      out += rc[0][q];
      eql += rc[1][q];
      eqh += rc[2][q];
      nl += rc[3][q];
    }
    const int64_t ncd = nl + novf_raw;
    const bool cand_ok = novf_raw <= (uint32_t)a.ovf_cap;
    if (t == 0) {
      const double mu = s1 / (double)n;
      const double var = fmax(s2 / (double)n - mu * mu, 0.0);
      const double piv = (double)(a.pivot ? a.pivot[c] : a.r.obs[a.r.obs_idx[0] * ob + c]);
      a.mean[c] = (float)(piv + mu);
      a.std[c] = (float)sqrt(var);
    }
    const uint32_t lo = a.bounds[ct * 2], hi = a.bounds[ct * 2 + 1];
    const int64_t k0 = (int64_t)floor((double)(n - 1) * (t ? 0.01 : 0.99));
    // position of the bracket's first element in the column's order
    const int64_t start = t ? out : n - out - eqh - ncd - eql;
    const int cp = __clz(lo ^ hi);
    const uint32_t mk = cp >= 32 ? 0xffffffffu : (cp == 0 ? 0u : ~(0xffffffffu >> cp));
    int nqq = 0;
    bool raw = false;
    for (int u = 0; u < 2; ++u) {
      const int64_t rk = u ? (k0 + 1 < n ? k0 + 1 : n - 1) : k0;
      const int64_t jj = rk - start;
      if (jj >= 0 && jj < eql) {
        vals[u] = lo;
      } else if (jj >= eql && jj < eql + ncd && cand_ok) {
        qslot[nqq] = u;
        qpre[nqq] = lo & mk;
        qmask[nqq] = mk;
        qrank[nqq] = (uint32_t)(jj - eql);
        ++nqq;
      } else if (jj >= eql + ncd && jj < eql + ncd + eqh) {
        vals[u] = hi;
      } else {  // outside the bracket or an overflowed list: select over the raw column
        qslot[nqq] = u;
        qpre[nqq] = 0;
        qmask[nqq] = 0;
        qrank[nqq] = (uint32_t)rk;
        ++nqq;
        raw = true;
      }
    }
    if (raw) {  // one key set per select: re-express candidate queries as raw-column ranks
      for (int q = 0; q < nqq; ++q)
        if (qmask[q] != 0) {
          qpre[q] = 0;
          qmask[q] = 0;
          qrank[q] = (uint32_t)(start + eql + qrank[q]);
        }
    }
    for (int q = nqq; q < 2; ++q) qmask[q] = 0xffffffffu;  // inactive
    nq = nqq;
    mode = raw ? 1 : (ncd <= kStSelKeys ? 0 : 2);
  }
  __syncthreads();
  const int md = mode;
  if (nq > 0 && md == 0) {  // gather the candidates into LDS: thread b copies list b
    const uint32_t* L = a.wgl + ((int64_t)b * ob * 2 + ct) * cap;
    for (uint32_t i = 0; i < nb; i += 8) {
      uint32_t k8[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) k8[u] = i + u < nb ? L[i + u] : 0u;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (i + u < nb) cand[off + i + u] = k8[u];
    }
    uint32_t tot = 0;
    for (int q = 0; q < NW; ++q) tot += rc[3][q];
    const uint32_t* ovf = a.ovf + (int64_t)ct * kStOvfCap;
    for (uint32_t i = tid; i < novf; i += T) cand[tot + i] = ovf[i];
    __syncthreads();
    const uint32_t ncd = tot + novf;
    st_radix_select<2>(qpre, qmask, qrank,
                       [&](auto&& fn) {
                         for (uint32_t i = tid; i < ncd; i += T) fn(cand[i]);
                       },
                       hist);
  } else if (nq > 0 && md == 2) {
    // too many candidates for LDS: digit passes over the global lists until the keys that still match a
    // query's prefix fit in LDS (usually one pass), then those are gathered and the select ends in LDS
    const uint32_t* wgl = a.wgl;
    const uint32_t* ovf = a.ovf + (int64_t)ct * kStOvfCap;
    auto visit_global = [&](auto&& fn) {
      const uint32_t* L = wgl + ((int64_t)b * ob * 2 + ct) * cap;
      for (uint32_t i = 0; i < nb; i += 4) {
        uint32_t k4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) k4[u] = i + u < nb ? L[i + u] : 0u;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (i + u < nb) fn(k4[u]);
      }
      for (uint32_t i = tid; i < novf; i += T) fn(ovf[i]);
    };
    __shared__ uint32_t s_nc;
    while (st_radix_select<2, 1>(qpre, qmask, qrank, visit_global, hist)) {
      if (tid == 0) s_nc = 0;
      __syncthreads();
      const int nqa = nq;
      const uint32_t p0 = qpre[0], k0m = qmask[0], p1 = qpre[1], k1m = qmask[1];
      visit_global([&](uint32_t k) {
        if ((k & k0m) == p0 || (nqa > 1 && (k & k1m) == p1)) {
          const uint32_t slot = atomicAdd(&s_nc, 1u);
          if (slot < (uint32_t)kStSelKeys) cand[slot] = k;
        }
      });
      __syncthreads();
      const uint32_t nc = s_nc;
      if (nc <= (uint32_t)kStSelKeys) {
        st_radix_select<2>(qpre, qmask, qrank,
                           [&](auto&& fn) {
                             for (uint32_t i = tid; i < nc; i += T) fn(cand[i]);
                           },
                           hist);
        break;
      }
      __syncthreads();  // every thread has read s_nc before the next round resets it
    }
  } else if (nq > 0) {
    const ReplayDev r = a.r;
    st_radix_select<2>(qpre, qmask, qrank,
                       [&](auto&& fn) {
                         for (int64_t i0 = tid; i0 < n; i0 += 4 * (int64_t)T) {
                           uint32_t k4[4];
#pragma unroll
                           for (int u = 0; u < 4; ++u) {
                             const int64_t i = i0 + u * (int64_t)T;
                             k4[u] = i < n ? fkey(r.obs[r.obs_idx[i] * ob + c]) : 0u;
                           }
#pragma unroll
                           for (int u = 0; u < 4; ++u)
                             if (i0 + u * (int64_t)T < n) fn(k4[u]);
                         }
                       },
                       hist);
  }
  if (nq > 0 && tid < nq) vals[qslot[tid]] = qpre[tid];
  __syncthreads();
  if (tid == 0) {
    const double g = np_frac(n, t ? 0.01 : 0.99);
    const double x0 = (double)funkey(vals[0]);
    const double x1 = (double)funkey(vals[1]);
    const float res = (float)np_lerp(x0, x1, g);  // numpy _lerp
    if (t == 0) a.max_out[c] = a.first_update ? res : fmaxf(res, a.max_out[c]);
    else a.min_out[c] = a.first_update ? res : fminf(res, a.min_out[c]);
    a.ovf_n[ct] = 0;  // every reader of this counter is past the barrier above
  }
}

// ================================================================ data-parallel: one data pass
// update_obs_mean_std over the union of the ranks' shards (replay_buffer.py:83-96) with ONE
// read of the local rows per call (the host runs the collectives between the phases):
//   phase 0  k_st_sample of Sl local rows into this rank's slot of samp [world][ob][Sl]   -> all-gather samp
//   phase 1  k_st_bracket over the union sample (identical bounds on every rank), k_st_pass over the local
//            rows (moments about the replicated pivot, far-side / bound counts, candidate lists), k_dp_reduce
//            -> exch [ob][2] moments | [ob][2][kDpCnt] counts (fp64, exact)                -> all-reduce exch
//   phases 2..5  k_dp_round r = 0..3: radix-select the two 'linear' ranks of each (column, target) in the
//            union of the ranks' candidate lists, 8 bits per round (a rank outside the bracket -- a sample
//            miss -- or an overflowed list selects over the raw column instead; 32 bits = 4 rounds either
//            way); each round's [ob][2][2][256] histogram                                    -> all-reduce hist
//   phase 6  k_dp_final: percentiles (numpy 'linear'), running max / min, mean / std.
// Every rank runs the same kernels on the same reduced data, so every rank holds the same statistics.
constexpr int kDpCnt = 5;  // per (column, target): outside, == lo, == hi, candidates, overflowed lists (flag)

constexpr int kDpCandCap = 32768;  // compacted local candidates per (column, target); more: the rounds walk the lists

// Grid (ob, 2), kStSelThreads threads: the pass's slabs -> exch (this rank's moments and counts), and this
// rank's candidate keys of (column, target) compacted to cand[ct][0 .. ncand) (block prefix sum over the
// workgroup lists, then the overflow list) so every round reads them with the whole workgroup.
__global__ __launch_bounds__(kStSelThreads) void k_dp_reduce(int ob, int nblk, int cap, int ovf_cap,
                                                            const double* __restrict__ part,
                                                            const uint32_t* __restrict__ cpart,
                                                            const uint32_t* __restrict__ wgl,
                                                            const uint32_t* __restrict__ wgn,
                                                            const uint32_t* __restrict__ ovf,
                                                            const uint32_t* __restrict__ ovf_n, double* __restrict__ exch,
                                                            uint32_t* __restrict__ cand, uint32_t* __restrict__ ncand) {
  constexpr int T = kStSelThreads, NW = T / 64;
  const int c = blockIdx.x, t = blockIdx.y, ct = c * 2 + t, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int b = tid;  // thread b owns pass workgroup b (nblk <= kStNblkMax = T)
  double m1 = 0.0, m2 = 0.0;
  uint32_t cc[3] = {0, 0, 0}, nb = 0;
  if (b < nblk) {
    if (t == 0) {
      m1 = part[((int64_t)b * ob + c) * 2 + 0];
      m2 = part[((int64_t)b * ob + c) * 2 + 1];
    }
#pragma unroll
    for (int f = 0; f < 3; ++f) cc[f] = cpart[((int64_t)b * ob + c) * 6 + 3 * t + f];
    nb = wgn[(int64_t)b * ob * 2 + ct];
  }
  uint32_t incl = nb;  // inclusive wave scan of the list lengths
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  m1 = wave_sum_d(m1);
  m2 = wave_sum_d(m2);
#pragma unroll
  for (int f = 0; f < 3; ++f)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cc[f] += __shfl_xor(cc[f], o, 64);
  __shared__ double rd[2][NW];
  __shared__ uint32_t rc[4][NW];
  if (lane == 63) rc[3][wv] = incl;
  if (lane == 0) {
    rd[0][wv] = m1;
    rd[1][wv] = m2;
#pragma unroll
    for (int f = 0; f < 3; ++f) rc[f][wv] = cc[f];
  }
  __syncthreads();
  uint32_t woff = 0, tot = 0;
  for (int q = 0; q < NW; ++q) {
    if (q < wv) woff += rc[3][q];
    tot += rc[3][q];
  }
  const uint32_t no_raw = ovf_n[ct], no = min(no_raw, (uint32_t)ovf_cap);
  const uint32_t n_all = tot + no;
  uint32_t* dst = cand + (int64_t)ct * kDpCandCap;
  __shared__ uint32_t offs[T + 1];  // exclusive list offsets; offs[nblk] = tot
  offs[b] = woff + incl - nb;
  if (b == T - 1) offs[T] = tot;
  __syncthreads();
  if (n_all <= (uint32_t)kDpCandCap) {  // key i: binary search of its list in offs, then an independent load
    constexpr int B = 8;  // keys in flight per thread: the loads of a batch are independent
    for (uint32_t i0 = tid; i0 < tot; i0 += B * T) {
      uint32_t v[B];
#pragma unroll
      for (int k = 0; k < B; ++k) {
        const uint32_t i = i0 + k * T;
        if (i < tot) {
          int lo = 0, hi = nblk - 1;  // the last list with offs <= i (empty lists share offsets: the last)
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (offs[mid] <= i) lo = mid;
            else hi = mid - 1;
          }
          v[k] = wgl[((int64_t)lo * ob * 2 + ct) * cap + (i - offs[lo])];
        }
      }
#pragma unroll
      for (int k = 0; k < B; ++k)
        if (i0 + k * T < tot) dst[i0 + k * T] = v[k];
    }
    const uint32_t* O = ovf + (int64_t)ct * kStOvfCap;
    for (uint32_t i = tid; i < no; i += T) dst[tot + i] = O[i];
  }
  if (tid == 0) {
    double s1 = 0.0, s2 = 0.0, out = 0.0, eql = 0.0, eqh = 0.0;
    for (int q = 0; q < NW; ++q) {
      s1 += rd[0][q];
      s2 += rd[1][q];
      out += rc[0][q];
      eql += rc[1][q];
      eqh += rc[2][q];
    }
    if (t == 0) {
      exch[c * 2 + 0] = s1;
      exch[c * 2 + 1] = s2;
    }
    double* e = exch + 2 * ob + (int64_t)ct * kDpCnt;
    e[0] = out;
    e[1] = eql;
    e[2] = eqh;
    e[3] = (double)tot + (double)no_raw;  // the true candidate count (a capped overflow list still counts all)
    e[4] = no_raw > (uint32_t)ovf_cap ? 1.0 : 0.0;
    ncand[ct] = n_all <= (uint32_t)kDpCandCap ? n_all : 0xffffffffu;  // all-ones: walk the lists
  }
}

struct DpQuery {
  uint32_t pre, mask, rank;
  int src;  // 0: resolved (pre is the key), 1: candidate lists, 2: raw column
};

struct StDpArgs {
  ReplayDev r;
  int64_t len;         // local live rows
  int64_t n_global;
  int nblk, cap, ovf_cap;
  const uint32_t* bounds;
  const uint32_t* wgl;
  const uint32_t* wgn;
  const uint32_t* ovf;
  uint32_t* ovf_n;
  const uint32_t* cand;   // [ob][2][kDpCandCap] compacted local candidates (k_dp_reduce)
  const uint32_t* ncand;  // [ob][2] their count (all-ones: walk the pass's lists)
  const double* exch;  // all-reduced
  uint32_t* hist;      // [ob][2][2][256], all-reduced between rounds
  DpQuery* q;          // [ob][2][2] device state (replicated: every rank derives the same)
  const float* pivot;
  float *mean, *std, *max_out, *min_out;
  int first_update;
};

// digit geometry of a query whose mask holds kb known top bits
__device__ __forceinline__ void dp_digit(uint32_t mask, int& shift, int& dbits) {
  const int kb = __popc(mask);
  shift = kb >= 24 ? 0 : 24 - kb;
  dbits = 32 - kb - shift;
}

// Advance query u of (c, t) with its reduced histogram of the last round (thread 0 of the workgroup).
__device__ void dp_consume(DpQuery& Q, const uint32_t* h) {
  if (Q.src == 0) return;
  int shift, dbits;
  dp_digit(Q.mask, shift, dbits);
  const int nb = 1 << dbits;
  uint32_t acc = 0;
  int d = -1, last = 0;
  for (int b = 0; b < nb; ++b) {
    if (h[b]) last = b;
    if (d < 0 && acc + h[b] > Q.rank) d = b;
    else if (d < 0) acc += h[b];
  }
  if (d < 0) {  // rank past the set (inconsistent counts): the last non-empty bin
    d = last;
    acc = 0;
    for (int b = 0; b < d; ++b) acc += h[b];
  }
  const uint32_t dm = (uint32_t)(nb - 1) << shift;
  Q.pre = (Q.pre & ~dm) | ((uint32_t)d << shift);
  Q.mask |= dm;
  Q.rank -= acc;
  if (Q.mask == 0xffffffffu) Q.src = 0;
}

// dp_consume by one whole wave over an LDS copy of the histogram: lane l holds bins 4l..4l+3, a wave scan of
// their sums finds the digit's lane (every lane returns the same query).
__device__ DpQuery dp_consume_wave(DpQuery Q, const uint32_t* h, int lane) {
  if (Q.src == 0) return Q;
  int shift, dbits;
  dp_digit(Q.mask, shift, dbits);
  const int nb = 1 << dbits;
  uint32_t v[4], s = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = 4 * lane + k < nb ? h[4 * lane + k] : 0u;
    s += v[k];
  }
  uint32_t incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t x = __shfl_up(incl, o, 64);
    if (lane >= o) incl += x;
  }
  const uint32_t excl = incl - s;
  const uint64_t hitm = __ballot(excl <= Q.rank && Q.rank < incl);
  int L, d = 0;
  uint32_t acc = 0;
  if (hitm) {
    L = __ffsll((unsigned long long)hitm) - 1;
    int dd = 4 * lane + 3;
    uint32_t a = excl, run = excl;
    bool f = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // first bin whose running sum passes the rank
      if (!f && run + v[k] > Q.rank) {
        dd = 4 * lane + k;
        a = run;
        f = true;
      }
      run += v[k];
    }
    d = __shfl(dd, L, 64);
    acc = __shfl(a, L, 64);
  } else {  // rank past the set (inconsistent counts): the last non-empty bin
    const uint64_t nz = __ballot(s != 0);
    L = nz ? 63 - __clzll((long long)nz) : 0;
    int dd = 4 * lane;
    uint32_t a = excl, run = excl;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (v[k]) {
        dd = 4 * lane + k;
        a = run;
      }
      run += v[k];
    }
    d = __shfl(dd, L, 64);
    acc = __shfl(a, L, 64);
  }
  const uint32_t dm = (uint32_t)(nb - 1) << shift;
  Q.pre = (Q.pre & ~dm) | ((uint32_t)d << shift);
  Q.mask |= dm;
  Q.rank -= acc;
  if (Q.mask == 0xffffffffu) Q.src = 0;
  return Q;
}

// One round (r = 0..3): derive (r = 0) or advance (r > 0) the queries, then this rank's histogram of their
// next digit.  Grid (ob, 2), kStSelThreads threads.
__global__ __launch_bounds__(kStSelThreads) void k_dp_round(StDpArgs a, int r) {
  constexpr int T = kStSelThreads;
  __shared__ uint32_t hl[2][256 * kStCopies];
  __shared__ DpQuery qs[2];
  const int c = blockIdx.x, t = blockIdx.y, tid = threadIdx.x, ob = a.r.ob, ct = c * 2 + t;
  DpQuery* qg = a.q + ct * 2;
  uint32_t* hg = a.hist + (int64_t)ct * 2 * 256;
  if (r == 0) {
    if (tid == 0) {
      const double* e = a.exch + 2 * ob + (int64_t)ct * kDpCnt;
      const int64_t n = a.n_global, out = (int64_t)e[0], eql = (int64_t)e[1], eqh = (int64_t)e[2],
                    ncd = (int64_t)e[3];
      const bool cand_ok = e[4] == 0.0;
      const uint32_t lo = a.bounds[ct * 2], hi = a.bounds[ct * 2 + 1];
      const int64_t k0 = (int64_t)floor((double)(n - 1) * (t ? 0.01 : 0.99));
      const int64_t start = t ? out : n - out - eqh - ncd - eql;
      const int cp = __clz(lo ^ hi);
      const uint32_t mk = cp >= 32 ? 0xffffffffu : (cp == 0 ? 0u : ~(0xffffffffu >> cp));
      for (int u = 0; u < 2; ++u) {
        const int64_t rk = u ? (k0 + 1 < n ? k0 + 1 : n - 1) : k0;
        const int64_t jj = rk - start;
        DpQuery Q;
        if (jj >= 0 && jj < eql) {
          Q = {lo, 0xffffffffu, 0, 0};
        } else if (jj >= eql && jj < eql + ncd && cand_ok) {
          Q = {lo & mk, mk, (uint32_t)(jj - eql), 1};
          if (mk == 0xffffffffu) Q.src = 0;
        } else if (jj >= eql + ncd && jj < eql + ncd + eqh) {
          Q = {hi, 0xffffffffu, 0, 0};
        } else {  // outside the bracket (a sample miss) or an overflowed list: the raw column
          Q = {0u, 0u, (uint32_t)rk, 2};
        }
        qs[u] = Q;
        qg[u] = Q;
      }
    }
  } else {
    uint32_t* hs = &hl[0][0];  // the reduced histograms of the last round, staged before the zeroing below
    if (tid < 512) hs[tid] = hg[tid];
    __syncthreads();
    const int wv = tid >> 6;
    if (wv < 2) {
      const DpQuery Q = dp_consume_wave(qg[wv], hs + wv * 256, tid & 63);
      if ((tid & 63) == 0) {
        qs[wv] = Q;
        qg[wv] = Q;
      }
    }
    __syncthreads();
  }
  for (int i = tid; i < 2 * 256 * kStCopies; i += T) (&hl[0][0])[i] = 0;
  __syncthreads();
  const DpQuery q0 = qs[0], q1 = qs[1];
  int sh[2], db[2];
  dp_digit(q0.mask, sh[0], db[0]);
  dp_digit(q1.mask, sh[1], db[1]);
  const int cp = tid & (kStCopies - 1);
  auto hit = [&](uint32_t k, int src) {
    if (q0.src == src && (k & q0.mask) == q0.pre)
      atomicAdd(&hl[0][(((k >> sh[0]) & ((1u << db[0]) - 1)) * kStCopies) + cp], 1u);
    if (q1.src == src && (k & q1.mask) == q1.pre)
      atomicAdd(&hl[1][(((k >> sh[1]) & ((1u << db[1]) - 1)) * kStCopies) + cp], 1u);
  };
  const uint32_t ncl = a.ncand[ct];
  if ((q0.src == 1 || q1.src == 1) && ncl != 0xffffffffu) {  // this rank's compacted candidate keys of (c, t)
    const uint32_t* C = a.cand + (int64_t)ct * kDpCandCap;
    constexpr int B = 8;
    for (uint32_t i0 = tid; i0 < ncl; i0 += B * T) {
      uint32_t v[B];
#pragma unroll
      for (int k = 0; k < B; ++k) v[k] = i0 + k * T < ncl ? C[i0 + k * T] : 0u;
#pragma unroll
      for (int k = 0; k < B; ++k)
        if (i0 + k * T < ncl) hit(v[k], 1);
    }
  } else if (q0.src == 1 || q1.src == 1) {  // too many to compact: the pass's lists + overflow
    if (tid < a.nblk) {
      const uint32_t nb = a.wgn[(int64_t)tid * ob * 2 + ct];
      const uint32_t* L = a.wgl + ((int64_t)tid * ob * 2 + ct) * a.cap;
      for (uint32_t i = 0; i < nb; ++i) hit(L[i], 1);
    }
    const uint32_t no = min(a.ovf_n[ct], (uint32_t)a.ovf_cap);
    const uint32_t* O = a.ovf + (int64_t)ct * kStOvfCap;
    for (uint32_t i = tid; i < no; i += T) hit(O[i], 1);
  }
  if (q0.src == 2 || q1.src == 2) {  // the raw local column
    const ReplayDev rr = a.r;
    for (int64_t i = tid; i < a.len; i += T) hit(fkey(rr.obs[rr.obs_idx[i] * ob + c]), 2);
  }
  __syncthreads();
  for (int i = tid; i < 2 * 256; i += T) {
    const uint32_t* p = &hl[i >> 8][(i & 255) * kStCopies];
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < kStCopies; ++k) sum += p[k];
    hg[i] = sum;
  }
}

// Phase 6: the last round's histograms resolve every query; numpy 'linear' percentile, running max / min;
// target 0 also writes mean / std from the all-reduced moments.  Grid (ob, 2), two waves (one per query).
__global__ __launch_bounds__(128) void k_dp_final(StDpArgs a) {
  const int c = blockIdx.x, t = blockIdx.y, ob = a.r.ob, ct = c * 2 + t, wv = threadIdx.x >> 6;
  __shared__ uint32_t hs[2][256];
  __shared__ DpQuery qs[2];
  for (int i = threadIdx.x; i < 512; i += 128) (&hs[0][0])[i] = a.hist[(int64_t)ct * 512 + i];
  __syncthreads();
  const DpQuery Qw = dp_consume_wave(a.q[ct * 2 + wv], hs[wv], threadIdx.x & 63);
  if ((threadIdx.x & 63) == 0) qs[wv] = Qw;
  __syncthreads();
  if (threadIdx.x) return;
  const DpQuery Q[2] = {qs[0], qs[1]};
  const int64_t n = a.n_global;
  if (t == 0) {
    const double mu = a.exch[c * 2 + 0] / (double)n;
    const double var = fmax(a.exch[c * 2 + 1] / (double)n - mu * mu, 0.0);
    a.mean[c] = (float)((double)a.pivot[c] + mu);
    a.std[c] = (float)sqrt(var);
  }
  const double g = np_frac(n, t ? 0.01 : 0.99);
  const double x0 = (double)funkey(Q[0].pre), x1 = (double)funkey(Q[1].pre);
  const float res = (float)np_lerp(x0, x1, g);  // numpy _lerp
  if (t == 0) a.max_out[c] = a.first_update ? res : fmaxf(res, a.max_out[c]);
  else a.min_out[c] = a.first_update ? res : fminf(res, a.min_out[c]);
  a.ovf_n[ct] = 0;  // the local overflow lists were last read by round 3
}

}  // namespace spp
