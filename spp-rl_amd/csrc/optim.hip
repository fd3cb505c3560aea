// Fragment-image packing, fused Adam(+polyak), temperature step and loss
// finalisation.
//   Adam      torch.optim.Adam single-tensor step (rltoolkit/rl.py:62)
//   polyak    rltoolkit/algorithms/sac/sac.py:186-199 (mul_ then add_, two roundings)
//   alpha     sac.py:201-216 + sac_acm.py:153-159 (log_alpha is float64)
#include "internal.h"

namespace spp {

__device__ __forceinline__ float pack_src(const PackJob& J, int n, int k) {
  if (n < 0 || k < 0) return 0.f;
  const int row = J.trans ? k : n;
  const int col = J.coff + (J.trans ? n : k);
  const float* base = row < J.split ? J.W + (int64_t)row * J.ld : J.W2 + (int64_t)(row - J.split) * J.ld;
  return base[col];
}

// bf16 image: element (ob, ib, s, lane) = 8 bf16 W[out(ob, lane&31)][in(ib, 8s + j, lane>>5)], RNE
__device__ void pack_bf16(const PackJob& J) {
  const int64_t total = (int64_t)J.NBO * J.NBI * 2 * 64;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int lane = (int)(i & 63);
    int64_t rest = i >> 6;
    const int s = (int)(rest & 1);
    rest >>= 1;
    const int ib = J.ibmajor ? (int)(rest / J.NBO) : (int)(rest % J.NBI);
    const int ob = J.ibmajor ? (int)(rest % J.NBO) : (int)(rest / J.NBI);
    int q, hh;
    row_to_pos(lane & 31, q, hh);
    const int n = map_index(J.out, ob, q, hh);
    typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
    bf16x8_t v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (__bf16)pack_src(J, n, map_index(J.in, ib, 8 * s + j, lane >> 5));
    J.dst[i] = __builtin_bit_cast(float4, v);
  }
}

__global__ void k_pack_matrix(const PackJob* __restrict__ jobs) {
  const PackJob J = jobs[blockIdx.y];
  if (J.bf16) {
    pack_bf16(J);
    return;
  }
  const int64_t total = (int64_t)J.NBO * J.NBI * 4 * 64;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int lane = (int)(i & 63);
    int64_t rest = i >> 6;
    const int rq = (int)(rest & 3);
    rest >>= 2;
    const int ib = J.ibmajor ? (int)(rest / J.NBO) : (int)(rest % J.NBI);
    const int ob = J.ibmajor ? (int)(rest % J.NBO) : (int)(rest / J.NBI);
    int q, hh;
    row_to_pos(lane & 31, q, hh);
    const int n = map_index(J.out, ob, q, hh);
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = map_index(J.in, ib, 4 * rq + j, lane >> 5);
      float x = 0.f;
      if (n >= 0 && k >= 0) {
        const int row = J.trans ? k : n;
        const int col = J.coff + (J.trans ? n : k);
        const float* base = row < J.split ? J.W + (int64_t)row * J.ld : J.W2 + (int64_t)(row - J.split) * J.ld;
        x = base[col];
      }
      v[j] = x;
    }
    J.dst[i] = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// Inverse of k_pack_matrix for tests: every image element that carries a weight is written back
// (as fp32) to its position in the flat parameter buffer starting at `base` (out[(src - base)]),
// so the caller can compare an image with the fp32 parameters (bf16 images: with their RNE values).
__global__ void k_unpack_matrix(PackJob J, const float* base, float* out) {
  const int per = J.bf16 ? 2 : 4;  // k-steps (bf16, 8 values) / register quads (fp32, 4) per block pair
  const int64_t total = (int64_t)J.NBO * J.NBI * per * 64;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int lane = (int)(i & 63);
    int64_t rest = i >> 6;
    const int sq = (int)(rest % per);
    rest /= per;
    const int ib = J.ibmajor ? (int)(rest / J.NBO) : (int)(rest % J.NBI);
    const int ob = J.ibmajor ? (int)(rest % J.NBO) : (int)(rest / J.NBI);
    int q, hh;
    row_to_pos(lane & 31, q, hh);
    const int n = map_index(J.out, ob, q, hh);
    if (n < 0) continue;
    const float4 raw = J.dst[i];
    const int nv = J.bf16 ? 8 : 4;
    for (int j = 0; j < nv; ++j) {
      const int k = map_index(J.in, ib, nv * sq + j, lane >> 5);
      if (k < 0) continue;
      float x;
      if (J.bf16) {
        typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
        x = (float)__builtin_bit_cast(bf16x8_t, raw)[j];
      } else {
        x = j == 0 ? raw.x : (j == 1 ? raw.y : (j == 2 ? raw.z : raw.w));
      }
      const int row = J.trans ? k : n;
      const int col = J.coff + (J.trans ? n : k);
      const float* src = row < J.split ? J.W + (int64_t)row * J.ld : J.W2 + (int64_t)(row - J.split) * J.ld;
      out[(src + col) - base] = x;
    }
  }
}

// One Adam step per element (+ optional polyak of the matching target element).
__global__ void k_adam(const AdamJob* __restrict__ jobs, float neg_step, float bc2s, float tau) {
  const AdamJob J = jobs[blockIdx.y];
  const float omb1 = 0.1f, b2 = 0.999f, omb2 = 0.001f, eps = 1e-8f;
  const float omtau = (float)(1.0 - (double)tau);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < J.n; i += (int64_t)gridDim.x * blockDim.x) {
    const float g = J.g[i];
    float m = J.m[i], v = J.v[i];
    m = fadd_rn(m, fmul_rn(omb1, fsub_rn(g, m)));                  // exp_avg.lerp_(g, 1-b1)
    v = fadd_rn(fmul_rn(v, b2), fmul_rn(fmul_rn(omb2, g), g));     // mul_(b2).addcmul_(g, g, 1-b2)
    const float denom = fadd_rn(fdiv_rn(sqrtf(v), bc2s), eps);   // (sqrt(v)/bc2s).add_(eps)
    const float p = fadd_rn(J.p[i], fmul_rn(neg_step, fdiv_rn(m, denom)));  // addcdiv_
    J.m[i] = m;
    J.v[i] = v;
    J.p[i] = p;
    if (J.targ) {
      const float t = fmul_rn(J.targ[i], omtau);
      J.targ[i] = fadd_rn(t, fmul_rn(tau, p));
    }
  }
}

// Deterministic block reduction of per-tile partial sums (double accumulate).
__device__ double block_sum(const float* part, int ntiles, int stride, int slot) {
  __shared__ double red[256];
  double s = 0.0;
  for (int t = threadIdx.x; t < ntiles; t += blockDim.x) s += (double)part[(int64_t)t * stride + slot];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

// NS consecutive partial slots [slot0, slot0 + NS) of every tile summed in ONE pass by kFinThreads
// threads (several tiles' loads in flight per thread), then one fixed-order LDS tree per slot:
// deterministic, and one memory latency chain instead of one per slot.
constexpr int kFinThreads = 1024;
template <int NS>
__device__ void block_sums(const float* part, int ntiles, int stride, int slot0, double (&out)[NS]) {
  __shared__ double red[NS][kFinThreads];
  double s[NS];
#pragma unroll
  for (int j = 0; j < NS; ++j) s[j] = 0.0;
#pragma unroll 4
  for (int t = threadIdx.x; t < ntiles; t += kFinThreads) {
    const float* p = part + (int64_t)t * stride + slot0;
#pragma unroll
    for (int j = 0; j < NS; ++j) s[j] += (double)p[j];
  }
#pragma unroll
  for (int j = 0; j < NS; ++j) red[j][threadIdx.x] = s[j];
  __syncthreads();
  for (int o = kFinThreads / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
#pragma unroll
      for (int j = 0; j < NS; ++j) red[j][threadIdx.x] += red[j][threadIdx.x + o];
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < NS; ++j) out[j] = red[j][0];
}

// losses[0..1] = critic MSEs (sac_acm.py:117-123); launched with kFinThreads threads
__global__ __launch_bounds__(kFinThreads) void k_finalize_critic(const float* part, int ntiles, int B, float* losses) {
  double l[2];
  block_sums<2>(part, ntiles, 8, 0, l);
  const double l0 = l[0], l1 = l[1];
  if (threadIdx.x == 0 && losses) {
    losses[0] = (float)(l0 / B);
    losses[1] = (float)(l1 / B);
  }
}

// Actor losses (sac_acm.py:77-86) and the temperature-gradient operand
// c = mean(-logpi - H) (sac.py:214-216), written for an optional all-reduce.
__global__ __launch_bounds__(kFinThreads) void k_actor_partials(const float* part, int ntiles, int B, int aout,
                                                               float custom_loss, double target_entropy,
                                                               float* alpha_grad, float* losses) {
  double v[3];
  block_sums<3>(part, ntiles, 8, 2, v);
  const double ssac = v[0], sdist = v[1], slp = v[2];
  if (threadIdx.x != 0) return;
  const double sac = ssac / B;
  const double dist = sdist / ((double)B * aout);
  *alpha_grad = (float)(-(slp / B) - target_entropy);
  if (losses) {
    losses[2] = (float)(custom_loss != 0.f ? sac + (double)custom_loss * dist : sac);
    losses[3] = custom_loss != 0.f ? (float)sac : 0.f;
    losses[4] = custom_loss != 0.f ? (float)dist : 0.f;
  }
}

// Temperature Adam step on float64 log_alpha (sac.py:107-110, sac_acm.py:153-159).
// alpha_state = {log_alpha, m, v, alpha}; g = exp(log_alpha) * c.
__global__ void k_alpha_step(const float* alpha_grad, double lr, int64_t step, double* alpha_state, float* alpha_f32,
                             float* losses) {
  if (threadIdx.x != 0) return;
  const double la = alpha_state[0];
  const double c = (double)*alpha_grad;
  const double g = exp(la) * c;
  double m = alpha_state[1], v = alpha_state[2];
  m = m + (1.0 - 0.9) * (g - m);
  v = v * 0.999 + (1.0 - 0.999) * g * g;
  const double bc1 = 1.0 - pow(0.9, (double)step), bc2s = sqrt(1.0 - pow(0.999, (double)step));
  const double nla = la - (lr / bc1) * (m / (sqrt(v) / bc2s + 1e-8));
  alpha_state[0] = nla;
  alpha_state[1] = m;
  alpha_state[2] = v;
  alpha_state[3] = exp(nla);
  *alpha_f32 = (float)exp(nla);
  if (losses) {
    losses[5] = (float)g;
    losses[6] = (float)exp(nla);
  }
}

// ACM regression loss (acm.py:253): mean over B*ac
__global__ void k_finalize_acm(const float* part, int ntiles, int B, int ac, float* loss) {
  const double s = block_sum(part, ntiles, 1, 0);
  if (threadIdx.x == 0 && loss) *loss = (float)(s / ((double)B * ac));
}

// DDPG_AcM losses {critic, actor, ddpg, dist} (ddpg_acm.py:133-143, :181)
__global__ __launch_bounds__(kFinThreads) void k_finalize_ddpg_critic(const float* part, int ntiles, int B,
                                                                     float* losses) {
  double v[1];
  block_sums<1>(part, ntiles, 8, 0, v);
  const double l0 = v[0];
  if (threadIdx.x == 0 && losses) losses[0] = (float)(l0 / B);
}
__global__ __launch_bounds__(kFinThreads) void k_finalize_ddpg_actor(const float* part, int ntiles, int B, int aout,
                                                                    float custom_loss, float* losses) {
  double v[2];
  block_sums<2>(part, ntiles, 8, 2, v);
  const double sq = v[0], sd = v[1];
  if (threadIdx.x != 0 || !losses) return;
  const double ddpg = sq / B, dist = sd / ((double)B * aout);
  losses[1] = (float)(custom_loss != 0.f ? ddpg + (double)custom_loss * dist : ddpg);
  losses[2] = custom_loss != 0.f ? (float)ddpg : 0.f;
  losses[3] = custom_loss != 0.f ? (float)dist : 0.f;
}

// BasicAcM regression: loss, and the gradients of its scale parameters t, t1
// (grad buffer slots 0 and 1..ac, state_dict order) from the per-tile partials.
__global__ void k_finalize_bacm(const float* part, int ntiles, int stride, int B, int ac, float* grad, float* loss) {
  const double s = block_sum(part, ntiles, stride, 0);
  const double dt = block_sum(part, ntiles, stride, 1);
  if (threadIdx.x == 0) {
    if (loss) *loss = (float)(s / ((double)B * ac));
    grad[0] = (float)dt;
  }
  for (int k = 0; k < ac; ++k) {
    const double v = block_sum(part, ntiles, stride, 2 + k);
    if (threadIdx.x == 0) grad[1 + k] = (float)v;
  }
}

}  // namespace spp
