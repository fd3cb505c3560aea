// Replay ring (rltoolkit/buffer/replay_buffer.py) device kernels, exact obs
// statistics, counter-based RNG and the synthetic env.
#include "replay.h"

namespace spp {

// ---------------------------------------------------------------- ring writes
// MetaReplayBuffer.add_obs (:56-60): rows e -> slot (base + e) % cap
__global__ void k_replay_add_obs(float* obs, int64_t cap, int ob, const float* src, int E, int64_t base) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)E * ob) return;
  const int64_t e = i / ob, f = i % ob;
  obs[((base + e) % cap) * ob + f] = src[i];
}

// add_acm_action (:332-333) + add_timestep (:65-75) + ReplayBuffer.addition (:133-137) into the timestep
// records (replay.h).  One thread per element: [E][aout] action values, then [E][ac] ACM actions, then the E
// record heads (one 16-B store each, plus the obs_idx array), so consecutive lanes write consecutive words of
// consecutive records (the rows of one vector step are consecutive slots except at the Q6 wrap).
__global__ void k_replay_add_step(ReplayDev r, const int64_t* __restrict__ meta /*[3][E]: prev, next, ts*/, int E,
                                  const float* act, const float* acm, const float* rew, const uint8_t* done,
                                  const uint8_t* end) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t na = (int64_t)E * r.aout, nm = (int64_t)E * r.ac;
  if (i < na) {
    const int64_t e = i / r.aout, f = i - e * r.aout;
    r.rec[meta[2 * E + e] * r.rw + rec_act(r) + f] = __float_as_uint(act ? act[i] : 0.f);
  } else if (i < na + nm) {
    const int64_t j = i - na, e = j / r.ac, f = j - e * r.ac;
    r.rec[meta[2 * E + e] * r.rw + kRecAcm + f] = __float_as_uint(acm ? acm[j] : 0.f);
  } else if (i < na + nm + E) {
    const int e = (int)(i - na - nm);
    const int64_t t = meta[2 * E + e];
    r.obs_idx[t] = meta[e];
    *reinterpret_cast<uint4*>(r.rec + t * r.rw) =
        make_uint4((uint32_t)meta[e], (uint32_t)meta[E + e], __float_as_uint(rew[e]),
                   (uint32_t)(done[e] != 0) | ((uint32_t)(end[e] != 0) << 8));
  }
}

// ---------------------------------------------------------------- gathers
// _sample_batch (:233-261) + sample_batch (:385-398), reference row-major layout
__global__ void k_replay_gather_rm(ReplayDev r, const int64_t* __restrict__ idx, int B, float* obs, float* nobs,
                                   float* act, float* rew, int8_t* done, float* acm) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int64_t t = idx[b];
  const uint32_t* rc = r.rec + t * r.rw;
  const uint4 hd = *reinterpret_cast<const uint4*>(rc);
  const int64_t o = hd.x, n = hd.y;
  for (int f = 0; f < r.ob; ++f) {
    if (obs) obs[(int64_t)b * r.ob + f] = r.obs[o * r.ob + f];
    if (nobs) nobs[(int64_t)b * r.ob + f] = r.obs[n * r.ob + f];
  }
  if (act)
    for (int f = 0; f < r.aout; ++f) act[(int64_t)b * r.aout + f] = __uint_as_float(rc[rec_act(r) + f]);
  if (acm)
    for (int f = 0; f < r.ac; ++f) acm[(int64_t)b * r.ac + f] = __uint_as_float(rc[kRecAcm + f]);
  if (rew) rew[b] = __uint_as_float(hd.z);
  if (done) done[b] = (int8_t)(hd.w & 1u);
}

// Fused sample -> feature-major staging of the update batch (zero padded to Bp).
// One thread per (sample, feature-row) so each feature row is written coalesced.
// Tile of kStageTile samples per 256-thread workgroup: each replay row is read
// contiguously (consecutive lanes = consecutive floats of one row), staged in LDS
// [tile][w], then written feature-major (consecutive lanes = consecutive samples),
// so both the random-row gather and the transposed store are coalesced.
constexpr int kStageTile = 64;

// element (row, f) of the source at src[row * stride + f] (obs rows: stride = w; record fields: stride = rw,
// src = the field's first word)
__device__ __forceinline__ void stage_rows(const float* __restrict__ src, int64_t stride, const int64_t* rows, int w,
                                           int valid, float* lds, float* dst, int64_t Bp, int64_t b0) {
  // rows [b0, b0 + kStageTile) of the padded batch; only b < Bp exist in dst
  const int n = kStageTile * w;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int s = i / w, f = i - s * w;
    lds[s * w + f] = s < valid ? src[rows[s] * stride + f] : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int f = i / kStageTile, s = i - f * kStageTile;
    if (b0 + s < Bp) dst[f * Bp + b0 + s] = lds[s * w + f];
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_replay_stage_fm(ReplayDev r, const int64_t* __restrict__ idx, int B, int Bp,
                                                         float* S, float* S2, float* ACT, float* AENV, float* R,
                                                         float* DN) {
  extern __shared__ float stg[];  // [kStageTile][max(ob, aout)]
  __shared__ int64_t rt[kStageTile], ro[kStageTile], rn[kStageTile];
  const int64_t b0 = (int64_t)blockIdx.x * kStageTile;
  const int valid = (int)min((int64_t)kStageTile, (int64_t)B - b0 > 0 ? (int64_t)B - b0 : 0);
  if (threadIdx.x < kStageTile) {
    const int s = threadIdx.x;
    const int64_t t = s < valid ? idx[b0 + s] : 0;
    const uint4 hd = s < valid ? *reinterpret_cast<const uint4*>(r.rec + t * r.rw) : make_uint4(0, 0, 0, 0);
    rt[s] = t;
    ro[s] = hd.x;
    rn[s] = hd.y;
    if (b0 + s < Bp) {
      R[b0 + s] = __uint_as_float(hd.z);
      DN[b0 + s] = (float)(hd.w & 1u);
    }
  }
  __syncthreads();
  const float* recf = reinterpret_cast<const float*>(r.rec);
  stage_rows(r.obs, r.ob, ro, r.ob, valid, stg, S, Bp, b0);
  stage_rows(r.obs, r.ob, rn, r.ob, valid, stg, S2, Bp, b0);
  if (ACT) stage_rows(recf + rec_act(r), r.rw, rt, r.aout, valid, stg, ACT, Bp, b0);
  stage_rows(recf + kRecAcm, r.rw, rt, r.ac, valid, stg, AENV, Bp, b0);
}

// Second form (the default): kStage2Tile = 32 samples per workgroup, the four row gathers (obs,
// next obs, action, ACM action) issued together before one barrier, then the four transposed
// stores.  Lane geometry per array of width w is fixed per thread (no per-element division):
// narrow rows (w <= 64) put G = 64 / w rows side by side in a wave (lane -> row g = lane / w,
// column lane % w), wide rows take one row per wave step with columns lane, lane + 64.  The
// 4 waves deal the row steps round-robin and keep up to kStage2Ld loads per lane in flight.
// The store side writes each feature row's 32 samples as one 128-B run; LDS rows have an odd
// stride (w | 1) so the transposed reads are conflict-free.
constexpr int kStage2Tile = 32;
constexpr int kStage2Ld = 16;

__host__ __device__ inline int stage2_stride(int w) { return w | 1; }
__host__ __device__ inline size_t stage2_lds_bytes(int ob, int aout, int ac, bool act) {
  return sizeof(float) * kStage2Tile * (2 * stage2_stride(ob) + (act ? stage2_stride(aout) : 0) + stage2_stride(ac));
}

struct Stage2Geo {
  int w, G, g, f0, nsteps, nc;
  bool on;
  __device__ Stage2Geo(int w_, int lane) : w(w_) {
    const bool narrow = w <= 64;
    G = narrow ? 64 / w : 1;
    g = narrow ? lane / w : 0;
    f0 = narrow ? lane - g * w : lane;
    on = narrow ? lane < G * w : true;
    nsteps = (kStage2Tile + G - 1) / G;
    nc = (w + 63) / 64;  // column chunks (1 or 2 for w <= 128)
  }
};

// Items of this wave for one array: (step st = wv + 4 k, chunk j) flattened as i = k * nc + j.
__device__ __forceinline__ int stage2_items(const Stage2Geo& G, int wv) {
  const int ks = G.nsteps > wv ? (G.nsteps - wv + 3) / 4 : 0;
  return ks * G.nc;
}

__device__ __forceinline__ void stage2_gather(const float* __restrict__ src, int64_t stride, const int64_t* rows,
                                              int valid, const Stage2Geo& G, int wv, float* l) {
  const int n = stage2_items(G, wv), ls = stage2_stride(G.w);
  for (int i0 = 0; i0 < n; i0 += kStage2Ld) {
    float v[kStage2Ld];
    int at[kStage2Ld];
#pragma unroll
    for (int u = 0; u < kStage2Ld; ++u) {
      const int i = i0 + u;
      const int k = i / G.nc, j = i - k * G.nc;  // nc is 1 or 2: a shift / compare, not a division loop
      const int s = (wv + 4 * k) * G.G + G.g, f = G.f0 + 64 * j;
      const bool ok = i < n && G.on && s < kStage2Tile && f < G.w;
      at[u] = ok ? s * ls + f : -1;
      v[u] = (ok && s < valid) ? src[rows[s] * stride + f] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kStage2Ld; ++u)
      if (at[u] >= 0) l[at[u]] = v[u];
  }
}

__device__ __forceinline__ void stage2_store(const float* l, int w, float* dst, int64_t Bp, int64_t b0) {
  const int s = threadIdx.x & (kStage2Tile - 1), ls = stage2_stride(w);
  if (b0 + s >= Bp) return;
  for (int f = threadIdx.x / kStage2Tile; f < w; f += 256 / kStage2Tile) dst[f * Bp + b0 + s] = l[s * ls + f];
}

__global__ __launch_bounds__(256) void k_replay_stage_fm2(ReplayDev r, const int64_t* __restrict__ idx, int B, int Bp,
                                                          float* S, float* S2, float* ACT, float* AENV, float* R,
                                                          float* DN) {
  extern __shared__ float stg[];
  __shared__ int64_t rt[kStage2Tile], ro[kStage2Tile], rn[kStage2Tile];
  const int64_t b0 = (int64_t)blockIdx.x * kStage2Tile;
  const int valid = (int)min((int64_t)kStage2Tile, (int64_t)B - b0 > 0 ? (int64_t)B - b0 : 0);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid < kStage2Tile) {
    const int s = tid;
    const int64_t t = s < valid ? idx[b0 + s] : 0;
    const uint4 hd = s < valid ? *reinterpret_cast<const uint4*>(r.rec + t * r.rw) : make_uint4(0, 0, 0, 0);
    rt[s] = t;
    ro[s] = hd.x;
    rn[s] = hd.y;
    if (b0 + s < Bp) {
      R[b0 + s] = __uint_as_float(hd.z);
      DN[b0 + s] = (float)(hd.w & 1u);
    }
  }
  __syncthreads();
  float* lo = stg;
  float* ln = lo + kStage2Tile * stage2_stride(r.ob);
  float* la = ln + kStage2Tile * stage2_stride(r.ob);
  float* lm = la + (ACT ? kStage2Tile * stage2_stride(r.aout) : 0);
  const Stage2Geo go(r.ob, lane), gm(r.ac, lane);
  const float* recf = reinterpret_cast<const float*>(r.rec);
  stage2_gather(r.obs, r.ob, ro, valid, go, wv, lo);
  stage2_gather(r.obs, r.ob, rn, valid, go, wv, ln);
  if (ACT) stage2_gather(recf + rec_act(r), r.rw, rt, valid, Stage2Geo(r.aout, lane), wv, la);
  stage2_gather(recf + kRecAcm, r.rw, rt, valid, gm, wv, lm);
  __syncthreads();
  stage2_store(lo, r.ob, S, Bp, b0);
  stage2_store(ln, r.ob, S2, Bp, b0);
  if (ACT) stage2_store(la, r.aout, ACT, Bp, b0);
  stage2_store(lm, r.ac, AENV, Bp, b0);
}

// last_end (replay_buffer.py:170-177) and the walk of last_rollout (:335-383): out[0] = the first
// index at distance 0, 1, ... back from p (cyclic over [0, len)) with end set; out[1] = the first
// one at distance 1 .. len back from out[0] (itself when it is the only end).  -1: none.
__global__ __launch_bounds__(1024) void k_replay_last_rollout(const uint32_t* __restrict__ rec, int rw, int64_t len,
                                                              int64_t p, int64_t* out) {
  __shared__ int best;
  __shared__ int64_t at;
  const int tid = threadIdx.x;
  for (int pass = 0; pass < 2; ++pass) {
    const int64_t from = pass == 0 ? p : at;
    const int64_t k0 = pass, k1 = pass == 0 ? len : len + 1;  // distance range [k0, k1)
    if (tid == 0) best = 0x7fffffff;
    __syncthreads();
    for (int64_t base = k0; base < k1; base += 1024) {
      const int64_t k = base + tid;
      if (k < k1) {
        int64_t i = (from - k) % len;
        if (i < 0) i += len;
        if ((rec[i * rw + 3] >> 8) & 1u) atomicMin(&best, (int)(k - base));  // the record's end flag
      }
      __syncthreads();
      const int b = best;
      __syncthreads();
      if (b != 0x7fffffff) {
        if (tid == 0) {
          int64_t i = (from - (base + b)) % len;
          at = i < 0 ? i + len : i;
        }
        break;
      }
      if (base + 1024 >= k1 && tid == 0) at = -1;
    }
    __syncthreads();
    if (tid == 0) out[pass] = at;
    if (at < 0) return;  // uniform (read after the barrier)
    __syncthreads();
  }
}

// rbuffer_sample_acm (:404-430) + AcMTrainer.acm_cat (acm.py:260-264): row-major
// x[b] = [obs[:, acm_ob_idx] | next_obs[:, acm_ob_idx]] (the identity when r.acm_cols is null),
// y[b] = acm action; kStageTile samples per workgroup, consecutive lanes read and write
// consecutive floats of one row.
__global__ __launch_bounds__(256) void k_replay_gather_acm(ReplayDev r, const int64_t* __restrict__ idx, int B,
                                                           float* x, float* y) {
  __shared__ int64_t rt[kStageTile], ro[kStageTile], rn[kStageTile];
  const int64_t b0 = (int64_t)blockIdx.x * kStageTile;
  const int valid = (int)min((int64_t)kStageTile, (int64_t)B - b0);
  if (threadIdx.x < valid) {
    const int64_t t = idx[b0 + threadIdx.x];
    const uint2 hd = *reinterpret_cast<const uint2*>(r.rec + t * r.rw);
    rt[threadIdx.x] = t;
    ro[threadIdx.x] = hd.x;
    rn[threadIdx.x] = hd.y;
  }
  __syncthreads();
  const int ob = r.ob, w = 2 * ob;
  for (int i = threadIdx.x; i < valid * w; i += blockDim.x) {
    const int s = i / w, f = i - s * w;
    const int c = f < ob ? f : f - ob;
    const int col = r.acm_cols ? r.acm_cols[c] : c;
    x[(b0 + s) * w + f] = r.obs[(f < ob ? ro[s] : rn[s]) * ob + col];
  }
  for (int i = threadIdx.x; i < valid * r.ac; i += blockDim.x) {
    const int s = i / r.ac, f = i - s * r.ac;
    y[(b0 + s) * r.ac + f] = __uint_as_float(r.rec[rt[s] * r.rw + kRecAcm + f]);
  }
}

// ---------------------------------------------------------------- obs statistics
// update_obs_mean_std (:83-96) over X = obs[obs_idx[0:len)]
__device__ __forceinline__ uint32_t fkey(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float funkey(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// Exact order statistics by 4-pass 8-bit radix select over the fp32 keys, for the
// 4 ranks of each column: lo / hi of the 99th percentile, lo / hi of the 1st.
// state[(c*4 + q)*3 + {0,1,2}] = {prefix, mask, rank remaining}.
//
// Pass 1 (k_stats_p1): one read of every live row: shifted fp64 moments
// (pivot = the first live row; var = E[(x-p)^2] - E[x-p]^2) and the top-byte
// histogram, shared by the 4 ranks (empty prefix).  Threads (ty, tx) of a
// 16x16 block take column tx (+16 j) of rows ty (+16 k): 64 B runs per row.
// Passes 2-4 (k_stats_pk): per-rank histograms of the next byte among the rows
// that match each rank's prefix.  k_stats_sel: one workgroup per column sums
// the per-block slabs, picks each rank's digit and, after the last byte, writes
// numpy's 'linear' percentile, running max / min and mean / std.
constexpr int kStatsBlocks = 1024;      // pass-1 workgroups (moment partials)
constexpr int kStatsColsPerThread = 8;  // columns per tx lane (ob <= 128)
constexpr int kStatsRows = 8;  // rows in flight per thread (index then row loads)

// Non-zero LDS bins -> the global histogram (device atomics; sparse after pass 1).
__device__ __forceinline__ void flush_hist(const uint32_t* sh, int n, uint32_t* g) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t v = sh[i];
    if (v) atomicAdd(&g[i], v);
  }
}

__global__ __launch_bounds__(256) void k_stats_p1(ReplayDev r, int64_t len, uint32_t* __restrict__ ghist,
                                                  double* __restrict__ part, const float* __restrict__ pivot) {
  extern __shared__ uint32_t sh1[];  // [ob][256] + reduction scratch
  const int ob = r.ob;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  for (int i = threadIdx.x; i < ob * 256; i += blockDim.x) sh1[i] = 0;
  __syncthreads();
  const float* p0 = pivot ? pivot : r.obs + r.obs_idx[0] * ob;  // moment shift
  double s1[kStatsColsPerThread], s2[kStatsColsPerThread];
  float piv[kStatsColsPerThread];
#pragma unroll
  for (int j = 0; j < kStatsColsPerThread; ++j) {
    s1[j] = s2[j] = 0.0;
    const int c = tx + 16 * j;
    piv[j] = c < ob ? p0[c] : 0.f;
  }
  const int64_t stride = (int64_t)gridDim.x * 16;
  for (int64_t i0 = (int64_t)blockIdx.x * 16 + ty; i0 < len; i0 += stride * kStatsRows) {
    int64_t base[kStatsRows];
#pragma unroll
    for (int k = 0; k < kStatsRows; ++k) {
      const int64_t i = i0 + k * stride;
      base[k] = i < len ? r.obs_idx[i] * ob : -1;
    }
#pragma unroll
    for (int j = 0; j < kStatsColsPerThread; ++j) {
      const int c = tx + 16 * j;
      if (c >= ob) break;
      float x[kStatsRows];
#pragma unroll
      for (int k = 0; k < kStatsRows; ++k) x[k] = base[k] >= 0 ? r.obs[base[k] + c] : 0.f;
#pragma unroll
      for (int k = 0; k < kStatsRows; ++k)
        if (base[k] >= 0) {
          const double d = (double)x[k] - (double)piv[j];
          s1[j] += d;
          s2[j] += d * d;
          atomicAdd(&sh1[c * 256 + (fkey(x[k]) >> 24)], 1u);
        }
    }
  }
  __syncthreads();
  flush_hist(sh1, ob * 256, ghist);
  // moments: reduce over ty (16 rows of threads) through LDS, per column
  double* red = reinterpret_cast<double*>(sh1 + ((ob * 256 + 1) & ~1));
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kStatsColsPerThread; ++j) {
    const int c = tx + 16 * j;
    if (16 * j >= ob) break;
    red[(ty * 16 + tx) * 2 + 0] = s1[j];
    red[(ty * 16 + tx) * 2 + 1] = s2[j];
    __syncthreads();
    if (ty == 0 && c < ob) {
      double a = 0.0, b = 0.0;
      for (int y = 0; y < 16; ++y) {
        a += red[(y * 16 + tx) * 2 + 0];
        b += red[(y * 16 + tx) * 2 + 1];
      }
      part[((int64_t)blockIdx.x * ob + c) * 2 + 0] = a;
      part[((int64_t)blockIdx.x * ob + c) * 2 + 1] = b;
    }
    __syncthreads();
  }
}

// Passes 2.. (k_stats_pk): per-rank histograms of the next dbits-bit digit (bits
// [shift, shift+dbits)) among the rows matching each rank's prefix, all columns in one read of
// the data: LDS [ob][4][1 << dbits].  dbits = 8 (shifts 16, 8, 0: 3 passes) while that fits
// 128 KiB (ob <= 32), else 6 (shifts 18, 12, 6, 0: 4 passes, <= 128 KiB for ob <= 128).
// 1024 threads (64 row lanes x 16 column lanes) keep enough loads in flight per CU.
constexpr int kStatsPkThreads = 1024;
__global__ __launch_bounds__(kStatsPkThreads) void k_stats_pk(ReplayDev r, int64_t len, int shift, int dbits,
                                                              const uint32_t* __restrict__ state,
                                                              uint32_t* __restrict__ ghist) {
  extern __shared__ uint32_t shk[];  // [ob][4][1 << dbits]
  // the ranks' (prefix, mask) per (column, rank) in LDS: 64 registers per thread held them before, which
  // spilled at 1024 threads (128 VGPRs); one broadcast LDS read per (column, rank) and row batch now
  __shared__ uint2 qpm[16 * kStatsColsPerThread * 4];
  const int ob = r.ob;
  const int bins = 1 << dbits;
  const int nb = ob * 4 * bins;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) shk[i] = 0;
  for (int i = threadIdx.x; i < ob * 4; i += blockDim.x) qpm[i] = make_uint2(state[i * 3 + 0], state[i * 3 + 1]);
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4, nty = blockDim.x >> 4;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * nty;
  for (int64_t i0 = (int64_t)blockIdx.x * nty + ty; i0 < len; i0 += stride * kStatsRows) {
    int64_t base[kStatsRows];
#pragma unroll
    for (int k = 0; k < kStatsRows; ++k) {
      const int64_t i = i0 + k * stride;
      base[k] = i < len ? r.obs_idx[i] * ob : -1;
    }
#pragma unroll
    for (int j = 0; j < kStatsColsPerThread; ++j) {
      const int c = tx + 16 * j;
      if (c >= ob) break;
      uint32_t kk[kStatsRows];
#pragma unroll
      for (int k = 0; k < kStatsRows; ++k) kk[k] = base[k] >= 0 ? fkey(r.obs[base[k] + c]) : 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint2 pm = qpm[c * 4 + q];
#pragma unroll
        for (int k = 0; k < kStatsRows; ++k)
          if (base[k] >= 0 && (kk[k] & pm.y) == pm.x)
            atomicAdd(&shk[(c * 4 + q) * bins + ((kk[k] >> shift) & (bins - 1))], 1u);
      }
    }
  }
  __syncthreads();
  flush_hist(shk, nb, ghist);
}

// One workgroup (256 threads = bins) per column of the group; consumes (and
// re-zeroes) the global histogram.  first: one shared [ob][256] histogram
// (pass 1) and the moment partials are reduced too.
__global__ __launch_bounds__(256) void k_stats_sel(uint32_t* __restrict__ ghist, int nblk, int ob, int col0,
                                                   int ncols, int shift, int dbits, int first,
                                                   const double* __restrict__ part,
                                                   int64_t len, uint32_t* __restrict__ state, double* __restrict__ mom,
                                                   float* max_out, float* min_out, int first_update) {
  __shared__ uint32_t cnt[4][256];
  __shared__ double rd[2][256];
  const int c = col0 + blockIdx.x, t = threadIdx.x;
  const int nbins = first ? 256 : 1 << dbits;  // pass 1: top byte; later passes: dbits-bit digits
  for (int q = 0; q < (first ? 1 : 4); ++q) {
    if (t >= nbins) break;
    const int64_t off = first ? (int64_t)c * 256 + t : ((int64_t)blockIdx.x * 4 + q) * nbins + t;
    cnt[q][t] = ghist[off];
    ghist[off] = 0;
  }
  if (first) {
    // fp64 moments of column c (shifted by the pivot)
    double a = 0.0, b = 0.0;
    for (int k = t; k < nblk; k += 256) {
      a += part[((int64_t)k * ob + c) * 2 + 0];
      b += part[((int64_t)k * ob + c) * 2 + 1];
    }
    rd[0][t] = a;
    rd[1][t] = b;
  }
  __syncthreads();
  if (first) {
    for (int o = 128; o > 0; o >>= 1) {
      if (t < o) {
        rd[0][t] += rd[0][t + o];
        rd[1][t] += rd[1][t + o];
      }
      __syncthreads();
    }
  }
  // Each rank's digit: the bin d with (counts below d) <= rank < (counts through d), found by an
  // inclusive block scan of the histogram (one per rank after pass 1) instead of a serial walk.
  __shared__ uint32_t pfx[4][256];
  __shared__ uint32_t srank[4], sacc[4];
  __shared__ int sbin[4];
  const int nh = first ? 1 : 4;
  if (t < 4) {
    const int q = t;
    uint32_t* st = state + (c * 4 + q) * 3;
    uint32_t rank;
    if (first) {  // ranks of np.percentile's lerp neighbours: floor((len-1) q) and the next
      const double qq = q < 2 ? 0.99 : 0.01;
      const int64_t lo = (int64_t)floor((double)(len - 1) * qq);
      const int64_t v = (q & 1) ? (lo + 1 < len ? lo + 1 : len - 1) : lo;
      rank = (uint32_t)v;
      st[0] = st[1] = 0;
    } else {
      rank = st[2];
    }
    srank[q] = rank;
    sbin[q] = nbins - 1;  // rank past the total: last bin, everything below it counted
  }
  for (int q = 0; q < nh; ++q)
    if (t < nbins) pfx[q][t] = cnt[q][t];
  __syncthreads();
  for (int o = 1; o < nbins; o <<= 1) {
    uint32_t v[4];
    for (int q = 0; q < nh; ++q) v[q] = (t < nbins && t >= o) ? pfx[q][t - o] : 0u;
    __syncthreads();
    for (int q = 0; q < nh; ++q)
      if (t < nbins) pfx[q][t] += v[q];
    __syncthreads();
  }
  if (t < 4) sacc[t] = pfx[first ? 0 : t][nbins - 1];
  __syncthreads();
  if (t < nbins) {
    for (int q = 0; q < 4; ++q) {
      const int hq = first ? 0 : q;
      const uint32_t inc = pfx[hq][t], exc = inc - cnt[hq][t];
      if (exc <= srank[q] && srank[q] < inc) {  // at most one bin per rank
        sbin[q] = t;
        sacc[q] = exc;
      }
    }
  }
  __syncthreads();
  if (t < 4) {
    uint32_t* st = state + (c * 4 + t) * 3;
    st[0] |= (uint32_t)sbin[t] << shift;
    st[1] |= (uint32_t)(nbins - 1) << shift;
    st[2] = srank[t] - sacc[t];
  }
  if (first && t == 0) {
    const double n = (double)len;
    const double m1 = rd[0][0] / n;
    const double var = fmax(rd[1][0] / n - m1 * m1, 0.0);
    mom[c * 2 + 0] = m1;  // mean - pivot (the pivot is added by k_stats_moments_out)
    mom[c * 2 + 1] = sqrt(var);
  }
  if (shift == 0) {
    __syncthreads();
    if (t == 0) {
      double res[2];
      const double qs[2] = {0.99, 0.01};
      for (int k = 0; k < 2; ++k) {
        const double g = np_frac(len, qs[k]);
        const double a = (double)funkey(state[(c * 4 + 2 * k) * 3 + 0]);
        const double b = (double)funkey(state[(c * 4 + 2 * k + 1) * 3 + 0]);
        res[k] = np_lerp(a, b, g);  // numpy _lerp
      }
      const float cmax = (float)res[0], cmin = (float)res[1];
      max_out[c] = first_update ? cmax : fmaxf(cmax, max_out[c]);
      min_out[c] = first_update ? cmin : fminf(cmin, min_out[c]);
    }
  }
}

// Sum of the pass-1 block partials per column -> out[ob][2] (the data-parallel
// exchange operand: ranks all-reduce these sums and their histograms).
__global__ void k_stats_reduce_part(const double* __restrict__ part, int nblk, int ob, double* __restrict__ out) {
  __shared__ double rd[2][256];
  const int c = blockIdx.x, t = threadIdx.x;
  double a = 0.0, b = 0.0;
  for (int k = t; k < nblk; k += 256) {
    a += part[((int64_t)k * ob + c) * 2 + 0];
    b += part[((int64_t)k * ob + c) * 2 + 1];
  }
  rd[0][t] = a;
  rd[1][t] = b;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) {
      rd[0][t] += rd[0][t + o];
      rd[1][t] += rd[1][t + o];
    }
    __syncthreads();
  }
  if (t == 0) {
    out[c * 2 + 0] = rd[0][0];
    out[c * 2 + 1] = rd[1][0];
  }
}

// mean = pivot + E[x - pivot]; std from the shifted moments (fp32 casts, replay_buffer.py:87-90)
__global__ void k_stats_moments_out(ReplayDev r, const double* mom, float* mean_out, float* std_out,
                                    const float* pivot) {
  const int c = threadIdx.x;
  if (c >= r.ob) return;
  const double piv = (double)(pivot ? pivot[c] : r.obs[r.obs_idx[0] * r.ob + c]);
  mean_out[c] = (float)(piv + mom[c * 2 + 0]);
  std_out[c] = (float)mom[c * 2 + 1];
}

// ---------------------------------------------------------------- RNG
__global__ void k_rand_normal(float* out, int64_t n, uint64_t seed, uint64_t offset) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (4 * i >= n) return;
  const u32x4 r = philox(seed, offset, (uint64_t)i);
  float a, b, c, d;
  box_muller(r.x, r.y, a, b);
  box_muller(r.z, r.w, c, d);
  const float v[4] = {a, b, c, d};
  for (int k = 0; k < 4; ++k)
    if (4 * i + k < n) out[4 * i + k] = v[k];
}
// uniform ints in [0, high) by masked rejection on 32-bit philox words
__global__ void k_rand_index(int64_t* out, int64_t n, int64_t high, uint64_t seed, uint64_t offset) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (high <= 1) {
    out[i] = 0;
    return;
  }
  const uint64_t rng = (uint64_t)(high - 1);
  uint64_t mask = rng;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
  for (uint64_t round = 0;; ++round) {
    const u32x4 r = philox(seed, offset + (round << 40), (uint64_t)i);
    const uint64_t w = ((uint64_t)r.x << 32) | r.y;
    const uint64_t v = w & mask;
    if (v <= rng || round == 63) {
      out[i] = (int64_t)(v <= rng ? v : v % (rng + 1));
      return;
    }
  }
}

// ---------------------------------------------------------------- synthetic env
// SURVEY.md Appendix A SynthEnv: s' = tanh(A s) + 0.1 * resize(a, ob); r = -|a|^2 + s'[0]
__global__ void k_synth_env(const float* A, const float* obs, const float* act, int E, int ob, int ac, float* nobs,
                            float* rew) {
  // one thread per (env, state unit): s'_i = tanh(A_i . s) + 0.1 a[i % ac]; unit 0 also writes r
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)E * ob) return;
  const int64_t e = t / ob;
  const int i = (int)(t - e * ob);
  const float* s = obs + e * ob;
  const float* a = act + e * ac;
  const float* Ai = A + (int64_t)i * ob;
  float acc = 0.f;
  for (int j = 0; j < ob; ++j) acc = fmaf(Ai[j], s[j], acc);
  const float v = tanhf(acc) + 0.1f * a[i % ac];
  nobs[t] = v;
  if (i == 0) {
    float n2 = 0.f;
    for (int j = 0; j < ac; ++j) n2 = fmaf(a[j], a[j], n2);
    rew[e] = -n2 + v;
  }
}


// uniform floats in [lo, hi) per element (gym Box.sample for the pre-train collector)
__global__ void k_rand_uniform(float* out, int64_t n, const float* lo, const float* hi, int period, uint64_t seed,
                               uint64_t offset) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (4 * i >= n) return;
  const u32x4 r = philox(seed, offset, (uint64_t)i);
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
  for (int k = 0; k < 4; ++k) {
    const int64_t j = 4 * i + k;
    if (j >= n) break;
    const int c = (int)(j % period);
    const float u = (float)(w[k] >> 8) * (1.0f / 16777216.0f);  // [0, 1), 24 bits
    out[j] = lo[c] + u * (hi[c] - lo[c]);
  }
}

// Per-env episode bookkeeping of the vectorized collector (StatsLogger /
// Memory.average_returns_per_rollout, rltoolkit/stats_logger.py:19-26):
// ep_ret += r; at an episode end the return is folded into sums = {sum, count}
// (fp64) and ep_ret restarts at 0.  end may be NULL (no env ended this step).
__global__ void k_episode_accum(const float* rew, const uint8_t* end, int E, float* ep_ret, double* sums) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  double s = 0.0, c = 0.0;
  if (e < E) {
    const float r = ep_ret[e] + rew[e];
    if (end && end[e]) {
      s = (double)r;
      c = 1.0;
      ep_ret[e] = 0.f;
    } else {
      ep_ret[e] = r;
    }
  }
  if (!end) return;
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_down(s, o);
    c += __shfl_down(c, o);
  }
  if ((threadIdx.x & 63) == 0 && c > 0.0) {
    atomicAdd(&sums[0], s);
    atomicAdd(&sums[1], c);
  }
}

// Rows of obs for which mask[e] != 0 are replaced by fresh N(0,1) states
// (SynthEnv.reset), the rest are kept.
__global__ void k_synth_reset(float* obs, const uint8_t* mask, int E, int ob, uint64_t seed, uint64_t offset) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)E * ob) return;
  if (mask && !mask[i / ob]) return;
  const u32x4 r = philox(seed, offset, (uint64_t)i);
  float a, b;
  box_muller(r.x, r.y, a, b);
  obs[i] = a;
}


// MemoryMeta.normalize / denormalize (rltoolkit/buffer/memory.py:76-127) elementwise
// over [rows][ob], the same fp32 operation order as the fused device helpers:
//   min-max : (x - mid) / (hi - mid + 1e-8)     |  mid + x * (hi - lo) / 2
//   z-score : clamp((x - mean) / (std + 1e-8), -10, 10)  |  (std + 1e-8) * x + mean
__device__ __forceinline__ float obs_norm1(float v, int j, const float* lo, const float* hi, const float* mean,
                                           const float* std, int min_max, int inverse) {
  if (min_max) {
    const float l = lo[j], h = hi[j];
    const float mid = fadd_rn(h, l) * 0.5f;
    return inverse ? fadd_rn(mid, fmul_rn(v, fsub_rn(h, l) * 0.5f))
                   : fdiv_rn(fsub_rn(v, mid), fadd_rn(fsub_rn(h, mid), 1e-8f));
  }
  return inverse ? fadd_rn(fmul_rn(fadd_rn(std[j], 1e-8f), v), mean[j])
                 : fminf(fmaxf(fdiv_rn(fsub_rn(v, mean[j]), fadd_rn(std[j], 1e-8f)), -10.f), 10.f);
}

__global__ void k_obs_normalize(const float* __restrict__ x, int64_t n, int ob, const float* lo, const float* hi,
                                const float* mean, const float* std, int min_max, int inverse, float* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = obs_norm1(x[i], (int)(i % ob), lo, hi, mean, std, min_max, inverse);
}

// The staged batch's sample_batch tail (replay_buffer.py:247-249) and DDPG_AcM.make_unbiased_update
// (acm/off_policy/ddpg_acm.py:59-73) on the feature-major staging arrays [ob][Bp]: with `norm`, the staged
// obs and next obs are normalised in place (the buffer's obs_norm); with `act_next`, the critic's action
// operand becomes the (normalised) next obs.  Columns b >= B (padding) stay zero.
__global__ void k_stage_post(float* S, float* S2, float* ACT, int ob, int B, int Bp, const float* lo, const float* hi,
                             const float* mean, const float* std, int min_max, int norm, int act_next) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)ob * B) return;
  const int f = (int)(i / B), b = (int)(i - (int64_t)f * B);
  const int64_t o = (int64_t)f * Bp + b;
  float s2 = S2[o];
  if (norm) {
    S[o] = obs_norm1(S[o], f, lo, hi, mean, std, min_max, 0);
    s2 = obs_norm1(s2, f, lo, hi, mean, std, min_max, 0);
    S2[o] = s2;
  }
  if (act_next) ACT[o] = s2;
}

}  // namespace spp
