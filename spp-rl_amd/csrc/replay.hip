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

// add_acm_action (:332-333) + add_timestep (:65-75) + ReplayBuffer.addition (:133-137)
__global__ void k_replay_add_step(ReplayDev r, const int64_t* __restrict__ meta /*[3][E]: prev, next, ts*/, int E,
                                  const float* act, const float* acm, const float* rew, const uint8_t* done,
                                  const uint8_t* end) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int64_t t = meta[2 * E + e];
  r.obs_idx[t] = meta[e];
  r.next_idx[t] = meta[E + e];
  for (int f = 0; f < r.aout; ++f) r.act[t * r.aout + f] = act ? act[(int64_t)e * r.aout + f] : 0.f;
  for (int f = 0; f < r.ac; ++f) r.acm[t * r.ac + f] = acm ? acm[(int64_t)e * r.ac + f] : 0.f;
  r.rew[t] = rew[e];
  r.done[t] = done[e];
  r.end[t] = end[e];
}

// ---------------------------------------------------------------- gathers
// _sample_batch (:233-261) + sample_batch (:385-398), reference row-major layout
__global__ void k_replay_gather_rm(ReplayDev r, const int64_t* __restrict__ idx, int B, float* obs, float* nobs,
                                   float* act, float* rew, int8_t* done, float* acm) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int64_t t = idx[b];
  const int64_t o = r.obs_idx[t], n = r.next_idx[t];
  for (int f = 0; f < r.ob; ++f) {
    if (obs) obs[(int64_t)b * r.ob + f] = r.obs[o * r.ob + f];
    if (nobs) nobs[(int64_t)b * r.ob + f] = r.obs[n * r.ob + f];
  }
  if (act)
    for (int f = 0; f < r.aout; ++f) act[(int64_t)b * r.aout + f] = r.act[t * r.aout + f];
  if (acm)
    for (int f = 0; f < r.ac; ++f) acm[(int64_t)b * r.ac + f] = r.acm[t * r.ac + f];
  if (rew) rew[b] = r.rew[t];
  if (done) done[b] = (int8_t)r.done[t];
}

// Fused sample -> feature-major staging of the update batch (zero padded to Bp).
// One thread per (sample, feature-row) so each feature row is written coalesced.
__global__ void k_replay_stage_fm(ReplayDev r, const int64_t* __restrict__ idx, int B, int Bp, float* S, float* S2,
                                  float* ACT, float* AENV, float* R, float* DN) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= Bp) return;
  const bool v = b < B;
  const int64_t t = v ? idx[b] : 0;
  const int64_t o = v ? r.obs_idx[t] : 0, n = v ? r.next_idx[t] : 0;
  for (int f = 0; f < r.ob; ++f) {
    S[f * (int64_t)Bp + b] = v ? r.obs[o * r.ob + f] : 0.f;
    S2[f * (int64_t)Bp + b] = v ? r.obs[n * r.ob + f] : 0.f;
  }
  if (ACT)
    for (int f = 0; f < r.aout; ++f) ACT[f * (int64_t)Bp + b] = v ? r.act[t * r.aout + f] : 0.f;
  for (int f = 0; f < r.ac; ++f) AENV[f * (int64_t)Bp + b] = v ? r.acm[t * r.ac + f] : 0.f;
  R[b] = v ? r.rew[t] : 0.f;
  DN[b] = v ? (float)r.done[t] : 0.f;
}

// rbuffer_sample_acm (:404-430) + AcMTrainer.acm_cat (acm.py:260-264)
__global__ void k_replay_gather_acm(ReplayDev r, const int64_t* __restrict__ idx, int B, float* x, float* y) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int64_t t = idx[b];
  const int64_t o = r.obs_idx[t], n = r.next_idx[t];
  const int ob = r.ob;
  for (int f = 0; f < ob; ++f) {
    x[(int64_t)b * 2 * ob + f] = r.obs[o * ob + f];
    x[(int64_t)b * 2 * ob + ob + f] = r.obs[n * ob + f];
  }
  for (int f = 0; f < r.ac; ++f) y[(int64_t)b * r.ac + f] = r.acm[t * r.ac + f];
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

// column sums (pass 0) / centred square sums (pass 1) in fp64, per-block partials
__global__ void k_stats_moments(ReplayDev r, int64_t len, const double* mean, double* part, int pass) {
  extern __shared__ double sred[];  // [blockDim.x]
  const int ob = r.ob;
  for (int c = 0; c < ob; ++c) {
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len; i += (int64_t)gridDim.x * blockDim.x) {
      const double x = (double)r.obs[r.obs_idx[i] * ob + c];
      if (pass == 0) s += x;
      else {
        const double d = x - mean[c];
        s += d * d;
      }
    }
    sred[threadIdx.x] = s;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
      if ((int)threadIdx.x < o) sred[threadIdx.x] += sred[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) part[(int64_t)blockIdx.x * ob + c] = sred[0];
    __syncthreads();
  }
}
__global__ void k_stats_reduce(const double* part, int nblk, int ob, int64_t len, double* out, int sqrt_out) {
  const int c = threadIdx.x;
  if (c >= ob) return;
  double s = 0.0;
  for (int k = 0; k < nblk; ++k) s += part[(int64_t)k * ob + c];
  s /= (double)len;
  out[c] = sqrt_out ? sqrt(s) : s;
}

// Radix select, 8 bits per pass, for 4 ranks per column:
// state[c*4 + q] = {prefix, mask, rank_remaining} (uint32 x3, rank fits 32 bits)
__global__ void k_stats_hist(ReplayDev r, int64_t len, int col0, int ncols, int shift, const uint32_t* state,
                             uint32_t* hist /*[nblk][ncols][4][256]*/) {
  extern __shared__ uint32_t sh[];  // [ncols][4][256]
  const int nb = ncols * 4 * 256;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) sh[i] = 0;
  __syncthreads();
  const int ob = r.ob;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len; i += (int64_t)gridDim.x * blockDim.x) {
    const float* row = r.obs + r.obs_idx[i] * ob + col0;
    for (int c = 0; c < ncols; ++c) {
      const uint32_t k = fkey(row[c]);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t* st = state + ((col0 + c) * 4 + q) * 3;
        if ((k & st[1]) == st[0]) atomicAdd(&sh[(c * 4 + q) * 256 + ((k >> shift) & 255)], 1u);
      }
    }
  }
  __syncthreads();
  uint32_t* out = hist + (int64_t)blockIdx.x * nb;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) out[i] = sh[i];
}
// one workgroup (256 threads) per (column, rank)
__global__ void k_stats_select(const uint32_t* hist, int nblk, int col0, int ncols, int shift, uint32_t* state) {
  __shared__ uint32_t cnt[256];
  const int cq = blockIdx.x;  // local (c, q)
  const int nb = ncols * 4 * 256;
  uint32_t s = 0;
  for (int k = 0; k < nblk; ++k) s += hist[(int64_t)k * nb + cq * 256 + threadIdx.x];
  cnt[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t* st = state + (col0 * 4 + cq) * 3;
    uint32_t rank = st[2], acc = 0;
    int bin = 255;
    for (int d = 0; d < 256; ++d) {
      if (acc + cnt[d] > rank) { bin = d; break; }
      acc += cnt[d];
    }
    st[0] |= (uint32_t)bin << shift;
    st[1] |= 255u << shift;
    st[2] = rank - acc;
  }
}
// final: numpy 'linear' percentile lerp, fp32 cast, running max/min, mean/std cast
__global__ void k_stats_finish(const uint32_t* state, const double* mean, const double* std, int ob, int64_t len,
                               float* mean_out, float* std_out, float* max_out, float* min_out, int first) {
  const int c = threadIdx.x;
  if (c >= ob) return;
  double res[2];
  const double qs[2] = {0.99, 0.01};
  for (int k = 0; k < 2; ++k) {
    const double vi = (double)(len - 1) * qs[k];
    const double lo = floor(vi);
    const double g = vi - lo;
    const double a = (double)funkey(state[(c * 4 + 2 * k) * 3 + 0]);
    const double b = (double)funkey(state[(c * 4 + 2 * k + 1) * 3 + 0]);
    const double diff = b - a;
    res[k] = g >= 0.5 ? b - diff * (1.0 - g) : a + diff * g;
  }
  const float cmax = (float)res[0], cmin = (float)res[1];
  mean_out[c] = (float)mean[c];
  std_out[c] = (float)std[c];
  max_out[c] = first ? cmax : fmaxf(cmax, max_out[c]);
  min_out[c] = first ? cmin : fminf(cmin, min_out[c]);
}
__global__ void k_stats_init(uint32_t* state, int ob, int64_t len) {
  const int c = threadIdx.x;
  if (c >= ob) return;
  const double qs[2] = {0.99, 0.01};
  for (int k = 0; k < 2; ++k) {
    const int64_t lo = (int64_t)floor((double)(len - 1) * qs[k]);
    const int64_t hi = lo + 1 < len ? lo + 1 : len - 1;
    uint32_t* a = state + (c * 4 + 2 * k) * 3;
    uint32_t* b = state + (c * 4 + 2 * k + 1) * 3;
    a[0] = a[1] = 0;
    a[2] = (uint32_t)lo;
    b[0] = b[1] = 0;
    b[2] = (uint32_t)hi;
  }
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
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const float* s = obs + (int64_t)e * ob;
  const float* a = act + (int64_t)e * ac;
  float s0 = 0.f;
  for (int i = 0; i < ob; ++i) {
    float acc = 0.f;
    for (int j = 0; j < ob; ++j) acc = fmaf(A[i * ob + j], s[j], acc);
    const float v = tanhf(acc) + 0.1f * a[i % ac];
    nobs[(int64_t)e * ob + i] = v;
    if (i == 0) s0 = v;
  }
  float n2 = 0.f;
  for (int j = 0; j < ac; ++j) n2 = fmaf(a[j], a[j], n2);
  rew[e] = -n2 + s0;
}

}  // namespace spp
