// PPO advantage and loss kernels (gfx950).
//
//  k_gae_seq    PPO.calculate_q_val + calculate_gae (rltoolkit/algorithms/a2c/a2c.py:247-265,
//               algorithms/ppo/ppo.py:117-150) over E independent streams, time-major [T][E]:
//               one lane per stream walks its T steps backwards with the reference's exact
//               float32 operation order (bit-exact).  HBM-bound: 4 B read x 3 + 2 x 1 B + 8 B
//               written per transition.
//  k_gae_scan   the same recurrence as a reverse affine scan a_t = b_t + c_t * a_{t+1}
//               (b_t = delta_t + [end & !done] gl V(s'_t), c_t = [!done & !end] gl) for few,
//               long streams: one workgroup per stream, 1024-step chunks scanned with wavefront
//               shuffles + an LDS pass over the 16 wave totals, carried chunk to chunk.  The
//               reassociation changes rounding (fp32 tolerance, not bit-exact).
//  k_ppo_clip   PPO._clip_loss (ppo.py:194-204) forward + d loss / d new_logprob, with
//               utils.kl_divergence (utils.py:48-59) partial sums.
//  k_adv_norm   AdvantageDataset normalisation (algorithms/ppo/advantage_dataset.py:8-12):
//               (A - mean) / (std_unbiased + 1.2e-7).
#include "common.h"

namespace spp {

// q = r + gamma*(1-d)*V(s') in torch's evaluation order (a2c.py:264)
__device__ __forceinline__ float ppo_q(float r, float d, float vn, float gamma) {
  return fadd_rn(r, fmul_rn(fmul_rn(gamma, fsub_rn(1.f, d)), vn));
}

__global__ void k_gae_seq(const float* __restrict__ rew, const float* __restrict__ v, const float* __restrict__ vn,
                          const uint8_t* __restrict__ done, const uint8_t* __restrict__ end, int64_t T, int64_t E,
                          float gamma, double disc, float* __restrict__ q_out, float* __restrict__ adv) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const float discf = (float)disc;
  float gae = 0.f;
  for (int64_t t = T - 1; t >= 0; --t) {
    const int64_t i = t * E + e;
    const float q = ppo_q(rew[i], done[i] ? 1.f : 0.f, vn[i], gamma);
    const float delta = fsub_rn(q, v[i]);
    if (q_out) q_out[i] = q;
    if (done[i]) {
      gae = delta;  // gae = 0 (python int): 0 * discount + delta
    } else if (end[i]) {
      // gae = critic(next_obs).item() (python float): the product runs in double,
      // then torch casts it to float32 before adding the float32 delta
      gae = fadd_rn((float)((double)vn[i] * disc), delta);
    } else {
      gae = fadd_rn(fmul_rn(gae, discf), delta);
    }
    adv[i] = gae;
  }
}

constexpr int kScanThreads = 1024;

// reverse-scan combine: (b, c) o (b2, c2) = (b + c*b2, c*c2)
__global__ __launch_bounds__(kScanThreads) void k_gae_scan(const float* __restrict__ rew, const float* __restrict__ v,
                                                           const float* __restrict__ vn,
                                                           const uint8_t* __restrict__ done,
                                                           const uint8_t* __restrict__ end, int64_t T, int64_t E,
                                                           float gamma, float gl, float* __restrict__ q_out,
                                                           float* __restrict__ adv) {
  __shared__ float wb[kScanThreads / 64], wc[kScanThreads / 64], enter[kScanThreads / 64];
  __shared__ float carry_s;
  const int64_t e = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int NW = kScanThreads / 64;
  float carry = 0.f;
  const int64_t nchunk = (T + kScanThreads - 1) / kScanThreads;
  for (int64_t ch = nchunk - 1; ch >= 0; --ch) {
    const int64_t t = ch * kScanThreads + tid;
    float b = 0.f, c = 1.f;  // identity beyond T
    if (t < T) {
      const int64_t i = t * E + e;
      const bool dn = done[i] != 0, en = end[i] != 0;
      const float q = ppo_q(rew[i], dn ? 1.f : 0.f, vn[i], gamma);
      const float delta = fsub_rn(q, v[i]);
      if (q_out) q_out[i] = q;
      b = (en && !dn) ? fadd_rn(fmul_rn(gl, vn[i]), delta) : delta;
      c = (!dn && !en) ? gl : 0.f;
    }
    // inclusive suffix scan inside the wave (lane i combines with lanes > i)
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const float b2 = __shfl_down(b, off, 64), c2 = __shfl_down(c, off, 64);
      if (lane + off < 64) {
        b = fadd_rn(b, fmul_rn(c, b2));
        c = fmul_rn(c, c2);
      }
    }
    if (lane == 0) {
      wb[w] = b;
      wc[w] = c;
    }
    __syncthreads();
    // value entering each wave from its right (later waves, then the next chunk)
    if (tid == 0) {
      float x = carry;
      for (int w2 = NW - 1; w2 >= 0; --w2) {
        enter[w2] = x;
        x = fadd_rn(wb[w2], fmul_rn(wc[w2], x));
      }
      carry_s = x;
    }
    __syncthreads();
    if (t < T) adv[t * E + e] = fadd_rn(b, fmul_rn(c, enter[w]));
    carry = carry_s;
    __syncthreads();
  }
}

// Clip loss partials: per block sums of min(r*A, clip(r)*A) and (lp_old - lp_new);
// grad[i] = d(-mean(min(.)))/d lp_new[i] with torch's tie / clamp rules
// (minimum: ties split the gradient; clamp: passes on [1-eps, 1+eps]).
__global__ void k_ppo_clip(const float* __restrict__ lp_old, const float* __restrict__ lp_new,
                           const float* __restrict__ adv, int B, float eps, float* __restrict__ grad,
                           double* __restrict__ part) {
  __shared__ double s0[256], s1[256];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  double m = 0.0, kl = 0.0;
  if (i < B) {
    const float r = expf(fsub_rn(lp_new[i], lp_old[i]));
    const float lo = 1.f - eps, hi = 1.f + eps;
    const float rc = fminf(fmaxf(r, lo), hi);
    const float A = adv[i];
    const float u = fmul_rn(r, A), uc = fmul_rn(rc, A);
    m = (double)fminf(u, uc);
    kl = (double)fsub_rn(lp_old[i], lp_new[i]);
    if (grad) {
      const float wu = u < uc ? 1.f : (u == uc ? 0.5f : 0.f);
      const float wc = 1.f - wu;
      const float pass = (r >= lo && r <= hi) ? 1.f : 0.f;
      // d/d lp_new of -(1/B) * min(r A, clip(r) A); dr/dlp_new = r
      grad[i] = -(wu * A * r + wc * A * pass * r) / (float)B;
    }
  }
  s0[threadIdx.x] = m;
  s1[threadIdx.x] = kl;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      s0[threadIdx.x] += s0[threadIdx.x + o];
      s1[threadIdx.x] += s1[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s0[0];
    part[2 * blockIdx.x + 1] = s1[0];
  }
}

// out[0] = -mean(min(.)) (actor clip loss), out[1] = mean(lp_old - lp_new) (KL)
__global__ void k_ppo_clip_finish(const double* __restrict__ part, int nblk, int B, float* __restrict__ out) {
  __shared__ double s0[256], s1[256];
  double a = 0.0, b = 0.0;
  for (int i = threadIdx.x; i < nblk; i += blockDim.x) {
    a += part[2 * i];
    b += part[2 * i + 1];
  }
  s0[threadIdx.x] = a;
  s1[threadIdx.x] = b;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      s0[threadIdx.x] += s0[threadIdx.x + o];
      s1[threadIdx.x] += s1[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = (float)(-s0[0] / B);
    out[1] = (float)(s1[0] / B);
  }
}

// Advantage normalisation, single pass of fp64 moments then an elementwise pass.
__global__ void k_adv_moments(const float* __restrict__ a, int64_t n, double* __restrict__ part) {
  __shared__ double s0[256], s1[256];
  double x = 0.0, x2 = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = a[i];
    x += v;
    x2 += v * v;
  }
  s0[threadIdx.x] = x;
  s1[threadIdx.x] = x2;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      s0[threadIdx.x] += s0[threadIdx.x + o];
      s1[threadIdx.x] += s1[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s0[0];
    part[2 * blockIdx.x + 1] = s1[0];
  }
}

__global__ void k_adv_norm(const float* __restrict__ a, int64_t n, const double* __restrict__ part, int nblk,
                           float* __restrict__ out) {
  __shared__ float ms[2];
  if (threadIdx.x == 0) {
    double s = 0.0, s2 = 0.0;
    for (int i = 0; i < nblk; ++i) {
      s += part[2 * i];
      s2 += part[2 * i + 1];
    }
    const double mean = s / (double)n;
    const double var = n > 1 ? fmax(0.0, (s2 - s * mean) / (double)(n - 1)) : 0.0;
    ms[0] = (float)mean;
    ms[1] = fadd_rn((float)sqrt(var), 1.2e-7f);
  }
  __syncthreads();
  const float mean = ms[0], den = ms[1];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = fdiv_rn(fsub_rn(a[i], mean), den);
}


// Data-parallel AdvantageDataset normalisation: ranks all-reduce the
// fp64 (sum, sum of squares) of k_adv_sum2 and normalise with the global n.
__global__ void k_adv_sum2(const double* __restrict__ part, int nblk, double* __restrict__ sums) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double s = 0.0, s2 = 0.0;
  for (int i = 0; i < nblk; ++i) {
    s += part[2 * i];
    s2 += part[2 * i + 1];
  }
  sums[0] = s;
  sums[1] = s2;
}
__global__ void k_adv_norm_g(const float* __restrict__ a, int64_t n_local, const double* __restrict__ sums,
                             int64_t n, float* __restrict__ out) {
  const double mean = sums[0] / (double)n;
  const double var = n > 1 ? fmax(0.0, (sums[1] - sums[0] * mean) / (double)(n - 1)) : 0.0;
  const float m = (float)mean, den = fadd_rn((float)sqrt(var), 1.2e-7f);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_local; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = fdiv_rn(fsub_rn(a[i], m), den);
}

}  // namespace spp
