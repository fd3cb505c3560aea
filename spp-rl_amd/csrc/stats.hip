// update_obs_mean_std (rltoolkit/buffer/replay_buffer.py:83-96) over the live replay rows
// X = obs[obs_idx[0:len)], by sample-bracketed exact selection: ONE read of X.
//
//   k_st_bracket  one workgroup per column: S = min(len, 4096 | 16384) stride-sampled rows -> sort
//                 keys, a 256 | 1024-thread bitonic sort (16 keys per thread: in-register,
//                 cross-lane shuffle, only the cross-wave stages through LDS); each target percentile
//                 (99th, 1st) is bracketed by the sample ranks +-(4 sigma + 4) around it
//   k_st_pass     one read of every live row.  Lanes take (row, column) pairs of G = 64 / ob
//                 consecutive rows (one row, two column halves for ob > 64), so a wave's loads
//                 cover contiguous row runs.  Per lane: fp64 moments about a pivot; per target
//                 the count of keys outside the bracket on the far side and of keys equal to
//                 either bound; the keys strictly inside go to the lane's LDS slots, then to one
//                 list per (workgroup, column, target) (a global overflow list, one atomic per
//                 key, only past the slots / the list capacity); per-workgroup partials of
//                 moments and counts to a slab.  No atomics on the fast path.
//   k_st_select   one workgroup per (column, target): reduces the slabs, places the 2 ranks numpy's
//                 'linear' percentile needs (floor((len-1) q) and the next) in
//                 [outside | = lo | candidates | = hi | outside] and radix-selects them inside
//                 the candidates (thread i reads workgroup list i) from their common key prefix
//                 on (8-bit digits).  mean / std and the running max (target 0) or min
//                 (target 1) are written here.  A rank outside the bracket (a sample miss) or an
//                 overflowed list falls back to a radix select over the column's raw data: the
//                 result is exact in every case.
// Keys: fkey() is the order-preserving uint32 image of a float (replay.hip).
#pragma once
#include "replay.h"

namespace spp {

constexpr int kStSampMax = 16384;   // bracketing sample per column (16 keys x 1024 threads)
constexpr int kStSampSmall = 4096;  // len <= kStBigLen: 16 keys x 256 threads
constexpr int64_t kStBigLen = 2000000;
constexpr int kStLaneK = 8;          // LDS candidate slots per (lane, column half, target)
constexpr int kStWgCap = 128;        // candidate keys per (workgroup, column, target) list
constexpr int kStOvfCap = 1 << 18;   // overflow keys per (column, target)
constexpr int kStPassThreads = 256;
constexpr int kStUnroll = 8;         // row groups per lane in flight

// ---------------------------------------------------------------- sample bracket
// Bitonic network position e = 16 * tid + i; partner e ^ j; ascending where (e & k) == 0.
template <int J>
__device__ __forceinline__ void bitonic_in_thread(uint32_t (&v)[16], int tid, int k) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    constexpr int jj = J;
    const int p = i ^ jj;
    if (p > i) {
      const bool up = ((16 * tid + i) & k) == 0;
      const uint32_t a = v[i], b = v[p];
      const bool sw = (a > b) == up;
      v[i] = sw ? b : a;
      v[p] = sw ? a : b;
    }
  }
}

// 16 * NT keys in NT threads (v: this thread's 16), ascending.  lds: 16 * NT words, element e
// at (e % 16) * NT + e / 16 (conflict-free for a fixed i across lanes).
template <int NT>
__device__ void block_sort16(uint32_t (&v)[16], uint32_t* lds) {
  const int tid = threadIdx.x;
  constexpr int P = 16 * NT;
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= 1024) {  // partner in another wave
#pragma unroll
        for (int i = 0; i < 16; ++i) lds[i * NT + tid] = v[i];
        __syncthreads();
        const int pt = tid ^ (j >> 4);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int e = 16 * tid + i;
          const uint32_t o = lds[i * NT + pt];
          const bool keep_min = (e < (e ^ j)) == ((e & k) == 0);
          v[i] = keep_min ? min(v[i], o) : max(v[i], o);
        }
        __syncthreads();
      } else if (j >= 16) {  // partner lane of the same wave
        const int lm = j >> 4;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int e = 16 * tid + i;
          const uint32_t o = __shfl_xor(v[i], lm, 64);
          const bool keep_min = (e < (e ^ j)) == ((e & k) == 0);
          v[i] = keep_min ? min(v[i], o) : max(v[i], o);
        }
      } else if (j == 8) {
        bitonic_in_thread<8>(v, tid, k);
      } else if (j == 4) {
        bitonic_in_thread<4>(v, tid, k);
      } else if (j == 2) {
        bitonic_in_thread<2>(v, tid, k);
      } else {
        bitonic_in_thread<1>(v, tid, k);
      }
    }
  }
}

// bounds[(c*2 + t)*2 + {0,1}] = {lo, hi} keys of target t (0: 99th, 1: 1st percentile), from
// the S-row stride sample rows ((2s + 1) len) / (2S) (all rows when S == len).
// NT threads sort S <= 16 NT keys: 256 (S = 4096) up to 2M live rows, 1024 (S = 16384) beyond, so
// the bracket (~0.8 / sqrt(S) of the rows) keeps the candidate lists within their capacity.
template <int NT>
__global__ __launch_bounds__(NT) void k_st_bracket(ReplayDev r, int64_t len, int S, uint32_t* __restrict__ bounds) {
  __shared__ uint32_t sk[16 * NT];
  const int c = blockIdx.x, tid = threadIdx.x, ob = r.ob;
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int j = 16 * tid + i;
    uint32_t k = 0xffffffffu;  // padding sorts last
    if (j < S) {
      const int64_t row = ((2 * (int64_t)j + 1) * len) / (2 * (int64_t)S);
      k = fkey(r.obs[r.obs_idx[row] * ob + c]);
    }
    v[i] = k;
  }
  block_sort16<NT>(v, sk);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) sk[16 * tid + i] = v[i];
  __syncthreads();
  if (tid < 2) {
    const double p = tid == 0 ? 0.99 : 0.01;
    const int64_t f = (int64_t)floor(p * (double)(S - 1));
    const int m = (int)ceil(4.0 * sqrt((double)S * p * (1.0 - p))) + 4;
    const int64_t lo_i = f - m, hi_i = f + 1 + m;
    // a bracket touching the sample's end extends to the key range's end (nothing outside)
    bounds[(c * 2 + tid) * 2 + 0] = lo_i <= 0 ? 0u : sk[lo_i];
    bounds[(c * 2 + tid) * 2 + 1] = hi_i >= S - 1 ? 0xffffffffu : sk[hi_i];
  }
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
  uint32_t* cpart;         // [nblk][ob][2][3]    count partials: outside, == lo, == hi
  uint32_t* wgl;           // [nblk][ob][2][kStWgCap]  per-workgroup candidate lists
  uint32_t* wgn;           // [nblk][ob][2]            keys in each list (<= kStWgCap)
  uint32_t* ovf;           // [ob][2][kStOvfCap]  keys past a lane's slots or a list's capacity
  uint32_t* ovf_n;         // [ob][2]             (zeroed before the pass)
};

__global__ __launch_bounds__(kStPassThreads) void k_st_pass(StPassArgs a) {
  constexpr int W = kStPassThreads / 64;
  __shared__ double rs[W][64][2][2];   // per lane: [j][s1, s2]
  __shared__ uint32_t rcn[W][64][2][6];  // per lane: [j][t * 3 + (outside, == lo, == hi)]
  __shared__ uint32_t lst[W][64][2][2][kStLaneK];  // per lane candidate slots
  __shared__ uint8_t lfill[W][64][2][2];
  const int ob = a.r.ob, G = st_groups(ob);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int64_t wv = (int64_t)blockIdx.x * W + w, nw = (int64_t)gridDim.x * W;
  const int g = ob <= 64 ? lane / ob : 0;
  const int col[2] = {st_col(ob, lane, 0), st_col(ob, lane, 1)};
  const float* p0 = a.pivot ? a.pivot : a.r.obs + a.r.obs_idx[0] * ob;
  float piv[2];
  uint32_t lo[2][2], hi[2][2];
  double s1[2] = {0.0, 0.0}, s2[2] = {0.0, 0.0};
  uint32_t cout[2][2] = {{0, 0}, {0, 0}}, ceq[2][2] = {{0, 0}, {0, 0}};  // ceq: == lo | == hi << 16
  uint32_t fill[2][2] = {{0, 0}, {0, 0}};
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = col[j] < 0 ? 0 : col[j];
    piv[j] = p0[c];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      lo[j][t] = a.bounds[(c * 2 + t) * 2 + 0];
      hi[j][t] = a.bounds[(c * 2 + t) * 2 + 1];
    }
  }
  const int64_t ngroups = (a.len + G - 1) / G;
  // the obs_idx of the next iteration's rows are requested before this iteration's data is
  // used: the dependent index -> row load pair overlaps across iterations
  int nidx[kStUnroll];  // ring slots < capacity < 2^31
#pragma unroll
  for (int u = 0; u < kStUnroll; ++u) {
    const int64_t row = (wv + u * nw) * G + g;
    nidx[u] = (row < a.len && col[0] >= 0) ? (int)a.r.obs_idx[row] : -1;
  }
  for (int64_t rg0 = wv; rg0 < ngroups; rg0 += nw * kStUnroll) {
    int64_t base[kStUnroll];
    bool ok[kStUnroll];
#pragma unroll
    for (int u = 0; u < kStUnroll; ++u) {
      ok[u] = nidx[u] >= 0;
      base[u] = ok[u] ? (int64_t)nidx[u] * ob : 0;
    }
#pragma unroll
    for (int u = 0; u < kStUnroll; ++u) {
      const int64_t row = (rg0 + (kStUnroll + u) * nw) * G + g;
      nidx[u] = (row < a.len && col[0] >= 0) ? (int)a.r.obs_idx[row] : -1;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j == 1 && ob <= 64) break;
      float x[kStUnroll];
#pragma unroll
      for (int u = 0; u < kStUnroll; ++u) x[u] = (ok[u] && col[j] >= 0) ? a.r.obs[base[u] + col[j]] : 0.f;
#pragma unroll
      for (int u = 0; u < kStUnroll; ++u) {
        if (!(ok[u] && col[j] >= 0)) continue;
        const double d = (double)x[u] - (double)piv[j];
        s1[j] += d;
        s2[j] += d * d;
        const uint32_t key = fkey(x[u]);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const uint32_t l = lo[j][t], h = hi[j][t];
          cout[j][t] += (uint32_t)(t ? key < l : key > h);
          ceq[j][t] += (uint32_t)(key == l) | ((uint32_t)(key == h && h != l) << 16);
          if (key > l && key < h) {
            const uint32_t f = fill[j][t]++;
            if (f < (uint32_t)kStLaneK) {
              lst[w][lane][j][t][f] = key;
            } else {
              const int ct = col[j] * 2 + t;
              const uint32_t o = atomicAdd(&a.ovf_n[ct], 1u);
              if (o < (uint32_t)kStOvfCap) a.ovf[(int64_t)ct * kStOvfCap + o] = key;
            }
          }
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int t = 0; t < 2; ++t) lfill[w][lane][j][t] = (uint8_t)(fill[j][t] < (uint32_t)kStLaneK ? fill[j][t] : kStLaneK);
  // lane partials -> LDS -> one partial per (workgroup, column)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    rs[w][lane][j][0] = s1[j];
    rs[w][lane][j][1] = s2[j];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      rcn[w][lane][j][3 * t + 0] = cout[j][t];
      rcn[w][lane][j][3 * t + 1] = ceq[j][t] & 0xffffu;
      rcn[w][lane][j][3 * t + 2] = ceq[j][t] >> 16;
    }
  }
  __syncthreads();
  for (int c = tid; c < ob; c += blockDim.x) {
    double m1 = 0.0, m2 = 0.0;
    uint32_t cn[6] = {0, 0, 0, 0, 0, 0};
    const int j = ob <= 64 ? 0 : c / 64;
    for (int q = 0; q < W; ++q)
      for (int gg = 0; gg < G; ++gg) {
        const int l = ob <= 64 ? gg * ob + c : c - 64 * j;
        m1 += rs[q][l][j][0];
        m2 += rs[q][l][j][1];
#pragma unroll
        for (int f = 0; f < 6; ++f) cn[f] += rcn[q][l][j][f];
      }
    a.part[((int64_t)blockIdx.x * ob + c) * 2 + 0] = m1;
    a.part[((int64_t)blockIdx.x * ob + c) * 2 + 1] = m2;
#pragma unroll
    for (int f = 0; f < 6; ++f) a.cpart[((int64_t)blockIdx.x * ob + c) * 6 + f] = cn[f];
  }
  // the lanes' candidate slots -> this workgroup's list per (column, target)
  for (int ct = tid; ct < 2 * ob; ct += blockDim.x) {
    const int c = ct >> 1, t = ct & 1;
    const int j = ob <= 64 ? 0 : c / 64;
    uint32_t* dst = a.wgl + ((int64_t)blockIdx.x * ob * 2 + ct) * kStWgCap;
    uint32_t n = 0;
    for (int q = 0; q < W; ++q)
      for (int gg = 0; gg < G; ++gg) {
        const int l = ob <= 64 ? gg * ob + c : c - 64 * j;
        const int m = lfill[q][l][j][t];
        for (int i = 0; i < m; ++i) {
          const uint32_t key = lst[q][l][j][t][i];
          if (n < (uint32_t)kStWgCap) {
            dst[n++] = key;
          } else {
            const uint32_t o = atomicAdd(&a.ovf_n[ct], 1u);
            if (o < (uint32_t)kStOvfCap) a.ovf[(int64_t)ct * kStOvfCap + o] = key;
          }
        }
      }
    a.wgn[(int64_t)blockIdx.x * ob * 2 + ct] = n;
  }
}

// ---------------------------------------------------------------- select
// Radix select (8-bit digits) of up to 2 ranks over a key set that the workgroup visits with
// visit(fn): every thread calls fn(key) for the keys it owns.  Each query starts from
// qpre / qmask: the bits known in advance (the candidates' common prefix: counting those
// digits would put every key into one bin).
template <class Visit>
__device__ void st_radix_select(int nq, uint32_t* qpre, uint32_t* qmask, uint32_t* qrank, Visit visit,
                                uint32_t (*hist)[256]) {
  const int tid = threadIdx.x;
  for (int shift = 24; shift >= 0; shift -= 8) {
    const uint32_t dm = 0xffu << shift;
    bool any = false;
    for (int q = 0; q < nq; ++q) any |= (qmask[q] & dm) != dm;
    if (!any) continue;
    for (int i = tid; i < 2 * 256; i += blockDim.x) hist[i >> 8][i & 255] = 0;
    __syncthreads();
    const uint32_t m0 = qmask[0], p0 = qpre[0], m1 = nq > 1 ? qmask[1] : 0u, p1 = nq > 1 ? qpre[1] : 1u;
    const bool a0 = (m0 & dm) != dm, a1 = nq > 1 && (m1 & dm) != dm;
    visit([&](uint32_t k) {
      if (a0 && (k & m0) == p0) atomicAdd(&hist[0][(k >> shift) & 255], 1u);
      if (a1 && (k & m1) == p1) atomicAdd(&hist[1][(k >> shift) & 255], 1u);
    });
    __syncthreads();
    if (tid < nq && (qmask[tid] & dm) != dm) {
      const uint32_t fixed = qpre[tid] & dm;
      uint32_t acc = 0, r = qrank[tid];
      int bin = 255;
      for (int d = 0; d < 256; ++d) {
        if ((((uint32_t)d << shift) & qmask[tid] & dm) != fixed) continue;  // outside the known bits
        if (acc + hist[tid][d] > r) {
          bin = d;
          break;
        }
        acc += hist[tid][d];
      }
      qpre[tid] = (qpre[tid] & ~dm) | ((uint32_t)bin << shift);
      qmask[tid] |= dm;
      qrank[tid] = r - acc;
    }
    __syncthreads();
  }
}

struct StSelArgs {
  ReplayDev r;
  int64_t len;
  int nblk;
  const double* part;
  const uint32_t* cpart;
  const uint32_t* bounds;
  const uint32_t* wgl;
  const uint32_t* wgn;
  const uint32_t* ovf;
  const uint32_t* ovf_n;
  const float* pivot;
  float *mean, *std, *max_out, *min_out;
  int first_update;
};

constexpr int kStSelThreads = 1024;

__global__ __launch_bounds__(kStSelThreads) void k_st_select(StSelArgs a) {
  constexpr int T = kStSelThreads;
  __shared__ double rd[2][T / 64];
  __shared__ uint32_t rc[4][T / 64];
  __shared__ uint32_t hist[2][256];
  __shared__ uint32_t vals[2], qpre[2], qmask[2], qrank[2];
  __shared__ int qslot[2], nq, mode;  // mode: 0 candidates, 1 raw column
  const int c = blockIdx.x, t = blockIdx.y, tid = threadIdx.x, ob = a.r.ob;
  const int lane = tid & 63, wv = tid >> 6;
  const int ct = c * 2 + t;
  // ---- moments (target 0), this target's counts, candidate count, over the workgroup partials
  double m1 = 0.0, m2 = 0.0;
  uint32_t cc[4] = {0, 0, 0, 0};
  for (int k = tid; k < a.nblk; k += T) {
    if (t == 0) {
      m1 += a.part[((int64_t)k * ob + c) * 2 + 0];
      m2 += a.part[((int64_t)k * ob + c) * 2 + 1];
    }
#pragma unroll
    for (int f = 0; f < 3; ++f) cc[f] += a.cpart[((int64_t)k * ob + c) * 6 + 3 * t + f];
    cc[3] += a.wgn[(int64_t)k * ob * 2 + ct];
  }
  m1 = wave_sum_d(m1);
  m2 = wave_sum_d(m2);
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cc[f] += __shfl_xor(cc[f], o, 64);
  if (lane == 0) {
    rd[0][wv] = m1;
    rd[1][wv] = m2;
#pragma unroll
    for (int f = 0; f < 4; ++f) rc[f][wv] = cc[f];
  }
  __syncthreads();
  const int64_t n = a.len;
  const uint32_t novf_raw = a.ovf_n[ct];
  const uint32_t novf = min(novf_raw, (uint32_t)kStOvfCap);
  if (tid == 0) {
    double s1 = 0.0, s2 = 0.0;
    int64_t out = 0, eql = 0, eqh = 0, nl = 0;
    for (int q = 0; q < T / 64; ++q) {
      s1 += rd[0][q];
      s2 += rd[1][q];
      out += rc[0][q];
      eql += rc[1][q];
      eqh += rc[2][q];
      nl += rc[3][q];
    }
    const int64_t ncd = nl + novf_raw;
    const bool cand_ok = novf_raw <= (uint32_t)kStOvfCap;
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
    nq = nqq;
    mode = raw ? 1 : 0;
  }
  __syncthreads();
  if (nq > 0) {
    if (mode == 0) {  // thread i visits workgroup list i, then a stride of the overflow keys
      const uint32_t* wgl = a.wgl;
      const uint32_t* wgn = a.wgn;
      const uint32_t* ovf = a.ovf + (int64_t)ct * kStOvfCap;
      const int nblk = a.nblk;
      st_radix_select(nq, qpre, qmask, qrank,
                      [&](auto&& fn) {
                        for (int b = tid; b < nblk; b += T) {
                          const uint32_t* L = wgl + ((int64_t)b * ob * 2 + ct) * kStWgCap;
                          const uint32_t m = wgn[(int64_t)b * ob * 2 + ct];
                          for (uint32_t i = 0; i < m; i += 4) {
                            uint32_t k4[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) k4[u] = i + u < m ? L[i + u] : 0u;
#pragma unroll
                            for (int u = 0; u < 4; ++u)
                              if (i + u < m) fn(k4[u]);
                          }
                        }
                        for (uint32_t i = tid; i < novf; i += T) fn(ovf[i]);
                      },
                      hist);
    } else {
      const ReplayDev r = a.r;
      st_radix_select(nq, qpre, qmask, qrank,
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
    if (tid < nq) vals[qslot[tid]] = qpre[tid];
  }
  __syncthreads();
  if (tid == 0) {
    const double vi = (double)(n - 1) * (t ? 0.01 : 0.99);
    const double g = vi - floor(vi);
    const double x0 = (double)funkey(vals[0]);
    const double x1 = (double)funkey(vals[1]);
    const double diff = x1 - x0;
    const float res = (float)(g >= 0.5 ? x1 - diff * (1.0 - g) : x0 + diff * g);  // numpy _lerp
    if (t == 0) a.max_out[c] = a.first_update ? res : fmaxf(res, a.max_out[c]);
    else a.min_out[c] = a.first_update ? res : fminf(res, a.min_out[c]);
  }
}

}  // namespace spp
