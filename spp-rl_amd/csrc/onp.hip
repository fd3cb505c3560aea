// On-policy (A2C / PPO) per-sample kernels for the 64-wide tanh MLPs of
// rltoolkit/basic_model.py:7-76 (same "samples on lanes" MFMA tiles as sac.hip):
//   Actor  : log_scale [aout]; fc1 ob->64, fc2 64->64, fc3 64->aout; mu = tanh(fc3) * lim,
//            Normal(mu, exp(log_scale)) (Independent over aout)
//   Critic : fc1 ob->64, fc2 64->64, fc3 64->1 (tanh hidden)
//
//  k_onp_value        V(x)                                   (a2c.py:257-265, ppo.py:131)
//  k_onp_critic_grad  0.5*mean((q - V(x))^2) backward        (a2c.py:209-219)
//  k_onp_actor_grad   PPO clip loss - ent*H backward through the Gaussian actor
//                     (ppo.py:174-190, 194-204; on_policy.py:189-205)
//  k_onp_act          a ~ Normal(mu, sigma) (or mu), log_prob (basic_model.py:32-51)
// Per-wave LDS image rows: hidden tiles at rows [0, 64).
#include "sac_kernels.h"

namespace spp {

template <int OB_, int AOUT_>
struct OCfg {
  static constexpr int OB = OB_, AOUT = AOUT_;
  static constexpr int NB_OB = blocks_of(OB), NB_AOUT = blocks_of(AOUT);
  static constexpr uint64_t RV_X = rv_nat(OB, NB_OB);
  static constexpr uint64_t RV_H = rv_nat(64, 2);
  static constexpr uint64_t RV_AOUT = rv_nat(AOUT, NB_AOUT);
};
constexpr float kLogSqrt2PiO = 0.91893853320467274178f;

struct OnpNet {
  const float4 *W1, *W2, *W3, *W3T, *W2T;  // W3T / W2T: backward images
  int tb1, tb2, tb3;                       // LDS table offsets (critic: tb3 = fc3 weight row)
  const float* b3;                         // critic fc3 bias (canonical scalar)
};
struct OnpArgs {
  int N, Np;
  const float* X;     // row-major [N][ob] inputs (normalised obs)
  OnpNet actor, critic;
  const float* log_scale;  // [aout] canonical actor parameter
  const float* lim;        // [aout]
  // critic regression / value
  const float* Q;          // [N] targets
  float* V;                // [N] values out
  // actor update
  const float *ACT, *LP_OLD, *ADV, *NXT;  // [N][aout], [N], [N], [N][aout] (next obs, dist loss) or null
  float eps_clip;
  // acting
  const float* EPS;   // [N][aout] standard normal or null (deterministic)
  float *ACT_OUT, *LP_OUT;
  // dW operands (feature-major [rows][Np]) and per-tile partials
  float *XT, *H1, *H2, *D1, *D2, *D3;
  float* part;        // [ntiles][stride]
  int pstride;
  TabSeg seg[8];
  int nseg;
};

__device__ __forceinline__ void onp_table(const OnpArgs& p, float* tbl) {
  for (int s = 0; s < p.nseg; ++s) {
    const TabSeg g = p.seg[s];
    for (int i = threadIdx.x; i < g.npad; i += blockDim.x) tbl[g.off + i] = i < g.n ? g.src[i] : 0.f;
  }
  __syncthreads();
}

// x tile (row-major input, units < OB) for sample b of this lane
template <class C>
__device__ __forceinline__ void onp_load_x(f32x16 (&x)[C::NB_OB], const OnpArgs& p, int br, bool valid, int h4) {
#pragma unroll
  for (int ib = 0; ib < C::NB_OB; ++ib)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int u = 32 * ib + ru(r) + h4;
      x[ib][r] = (u < C::OB && valid) ? p.X[(int64_t)br * C::OB + u] : 0.f;
    }
}

// h1 = tanh(fc1 x), h2 = tanh(fc2 h1); both tiles returned (and left in LDS rows [0,64) = h2)
template <class C>
__device__ __forceinline__ void onp_trunk(const OnpNet& n, const f32x16 (&x)[C::NB_OB], const float* tbl, float* img,
                                          float* bl, f32x16 (&h1)[2], f32x16 (&h2)[2]) {
  dense<C::NB_OB, C::RV_X>(n.W1, 2, x, tbl + n.tb1, [&](int ob, const f32x16& acc) {
#pragma unroll
    for (int q = 0; q < 16; ++q) bl[(32 * ob + ru(q)) * 32] = tanhf(acc[q]);
  });
  lds_load<2>(h1, img);
  dense<2, C::RV_H>(n.W2, 2, h1, tbl + n.tb2, [&](int ob, const f32x16& acc) {
#pragma unroll
    for (int q = 0; q < 16; ++q) bl[(32 * ob + ru(q)) * 32] = tanhf(acc[q]);
  });
  lds_load<2>(h2, img);
}

template <class C>
__device__ __forceinline__ float onp_value(const OnpNet& n, const f32x16 (&h2)[2], const float* tbl, int h4) {
  float v = 0.f;
#pragma unroll
  for (int ib = 0; ib < 2; ++ib)
#pragma unroll
    for (int q = 0; q < 16; ++q) v = fmaf(h2[ib][q], tbl[n.tb3 + 32 * ib + ru(q) + h4], v);
  return v + __shfl_xor(v, 32, 64) + *n.b3;
}

#define SPP_ONP_PROLOGUE                                                     \
  __shared__ float smem[4 * 64 * 32];                                        \
  __shared__ __attribute__((aligned(16))) float tbl[1024];                   \
  onp_table(p, tbl);                                                         \
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5;    \
  const int h4 = 4 * h, s = lane & 31;                                       \
  float* img = smem + w * 64 * 32;                                           \
  float* bl = img + h4 * 32 + s;                                             \
  const int ntiles = p.Np / 32;

template <class C>
__global__ __launch_bounds__(256) void k_onp_value(OnpArgs p) {
  SPP_ONP_PROLOGUE
  for (int tile = blockIdx.x * 4 + w; tile < ntiles; tile += gridDim.x * 4) {
    const int b = tile * 32 + s;
    const bool valid = b < p.N;
    f32x16 x[C::NB_OB], h1[2], h2[2];
    onp_load_x<C>(x, p, valid ? b : 0, valid, h4);
    onp_trunk<C>(p.critic, x, tbl, img, bl, h1, h2);
    const float v = onp_value<C>(p.critic, h2, tbl, h4);
    if (valid && h == 0) p.V[b] = v;
  }
}

// critic_loss = 0.5 * (q - V)^2 .mean(); dV = -(q - V) / N
template <class C>
__global__ __launch_bounds__(256) void k_onp_critic_grad(OnpArgs p) {
  SPP_ONP_PROLOGUE
  const float invN = 1.f / (float)p.N;
  for (int tile = blockIdx.x * 4 + w; tile < ntiles; tile += gridDim.x * 4) {
    const int b = tile * 32 + s;
    const bool valid = b < p.N;
    const int br = valid ? b : 0;
    f32x16 x[C::NB_OB], h1[2], h2[2];
    onp_load_x<C>(x, p, br, valid, h4);
#pragma unroll
    for (int ib = 0; ib < C::NB_OB; ++ib)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (32 * ib + ru(r) + h4 < C::OB) p.XT[(int64_t)(32 * ib + ru(r) + h4) * p.Np + b] = x[ib][r];
    onp_trunk<C>(p.critic, x, tbl, img, bl, h1, h2);
    const float v = onp_value<C>(p.critic, h2, tbl, h4);
    const float adv = valid ? fsub_rn(p.Q[br], v) : 0.f;
    const float dv = -adv * invN;
    if (h == 0) p.D3[b] = dv;
    f32x16 d2[2];
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int u = 32 * ib + ru(q) + h4;
        p.H1[(int64_t)u * p.Np + b] = h1[ib][q];
        p.H2[(int64_t)u * p.Np + b] = h2[ib][q];
        d2[ib][q] = dv * tbl[p.critic.tb3 + u] * (1.f - h2[ib][q] * h2[ib][q]);
        p.D2[(int64_t)u * p.Np + b] = d2[ib][q];
      }
    dense<2, C::RV_H>(p.critic.W2T, 2, d2, nullptr, [&](int ob, const f32x16& acc) {
      const f32x16 hh = ob == 0 ? h1[0] : h1[1];
#pragma unroll
      for (int q = 0; q < 16; ++q)
        p.D1[(int64_t)(32 * ob + ru(q) + h4) * p.Np + b] = acc[q] * (1.f - hh[q] * hh[q]);
    });
    const float l = wave_sum((valid && h == 0) ? 0.5f * adv * adv : 0.f);
    if (lane == 0) p.part[tile * p.pstride] = l;
  }
}

// PPO actor step on a minibatch: logp of the stored actions under the current
// policy, clip-objective gradient (torch minimum / clamp rules), backward.
// partials: [0] sum min(r A, clip(r) A), [1] sum (lp_old - lp_new), [2] sum dist^2,
// [3 + j] sum d logp / d log_scale_j weighted by d loss / d logp.
template <class C>
__global__ __launch_bounds__(256) void k_onp_actor_grad(OnpArgs p) {
  SPP_ONP_PROLOGUE
  const float invN = 1.f / (float)p.N;
  const float lo = 1.f - p.eps_clip, hi = 1.f + p.eps_clip;
  for (int tile = blockIdx.x * 4 + w; tile < ntiles; tile += gridDim.x * 4) {
    const int b = tile * 32 + s;
    const bool valid = b < p.N;
    const int br = valid ? b : 0;
    f32x16 x[C::NB_OB], h1[2], h2[2];
    onp_load_x<C>(x, p, br, valid, h4);
#pragma unroll
    for (int ib = 0; ib < C::NB_OB; ++ib)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (32 * ib + ru(r) + h4 < C::OB) p.XT[(int64_t)(32 * ib + ru(r) + h4) * p.Np + b] = x[ib][r];
    onp_trunk<C>(p.actor, x, tbl, img, bl, h1, h2);
    // mu tile
    f32x16 t3[C::NB_AOUT];
    dense<2, C::RV_H>(p.actor.W3, C::NB_AOUT, h2, tbl + p.actor.tb3, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int ib = 0; ib < C::NB_AOUT; ++ib)
        if (ib == ob)
#pragma unroll
          for (int q = 0; q < 16; ++q) t3[ib][q] = tanhf(acc[q]);
    });
    // log_prob (torch Normal: -(a-mu)^2/(2 var) - log(scale) - log(sqrt(2 pi)), summed)
    float lp = 0.f, dist = 0.f;
#pragma unroll
    for (int ib = 0; ib < C::NB_AOUT; ++ib)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int j = 32 * ib + ru(q) + h4;
        if (j < C::AOUT) {
          const float sc = expf(p.log_scale[j]);
          const float mu = fmul_rn(t3[ib][q], p.lim[j]);
          const float a = valid ? p.ACT[(int64_t)br * C::AOUT + j] : 0.f;
          const float d = fsub_rn(a, mu);
          lp += fsub_rn(fsub_rn(fdiv_rn(-fmul_rn(d, d), 2.f * fmul_rn(sc, sc)), logf(sc)), kLogSqrt2PiO);
          if (p.NXT && valid) {
            const float e = fsub_rn(a, p.NXT[(int64_t)br * C::AOUT + j]);
            dist += e * e;
          }
        }
      }
    lp += __shfl_xor(lp, 32, 64);
    // clip objective (ppo.py:199-203) and its gradient wrt lp_new
    float m = 0.f, kl = 0.f, glp = 0.f;
    if (valid) {
      const float lpo = p.LP_OLD[br], A = p.ADV[br];
      const float r = expf(fsub_rn(lp, lpo));
      const float rc = fminf(fmaxf(r, lo), hi);
      const float u1 = fmul_rn(r, A), u2 = fmul_rn(rc, A);
      m = fminf(u1, u2);
      kl = fsub_rn(lpo, lp);
      const float wu = u1 < u2 ? 1.f : (u1 == u2 ? 0.5f : 0.f);
      const float pass = (r >= lo && r <= hi) ? 1.f : 0.f;
      glp = -(wu * A * r + (1.f - wu) * A * pass * r) * invN;
    }
    // back to mu, log_scale and the fc3 pre-activation
    f32x16 du3[C::NB_AOUT];
    float gls[C::NB_AOUT * 16];
#pragma unroll
    for (int ib = 0; ib < C::NB_AOUT; ++ib)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int j = 32 * ib + ru(q) + h4;
        float g = 0.f, gl = 0.f;
        if (j < C::AOUT && valid) {
          const float sc = expf(p.log_scale[j]);
          const float var = fmul_rn(sc, sc);
          const float mu = fmul_rn(t3[ib][q], p.lim[j]);
          const float d = fsub_rn(p.ACT[(int64_t)br * C::AOUT + j], mu);
          const float gmu = glp * d / var;
          gl = glp * (d * d / var - 1.f);
          g = gmu * p.lim[j] * (1.f - t3[ib][q] * t3[ib][q]);
        }
        du3[ib][q] = g;
        gls[ib * 16 + q] = gl;
        if (j < C::AOUT) p.D3[(int64_t)j * p.Np + b] = g;
      }
    f32x16 d2[2];
    dense<C::NB_AOUT, C::RV_AOUT>(p.actor.W3T, 2, du3, nullptr, [&](int ob, const f32x16& acc) {
      const f32x16 hh = ob == 0 ? h2[0] : h2[1];
      f32x16 v;
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = acc[q] * (1.f - hh[q] * hh[q]);
      if (ob == 0) d2[0] = v;
      else d2[1] = v;
    });
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int u = 32 * ib + ru(q) + h4;
        p.H1[(int64_t)u * p.Np + b] = h1[ib][q];
        p.H2[(int64_t)u * p.Np + b] = h2[ib][q];
        p.D2[(int64_t)u * p.Np + b] = d2[ib][q];
      }
    dense<2, C::RV_H>(p.actor.W2T, 2, d2, nullptr, [&](int ob, const f32x16& acc) {
      const f32x16 hh = ob == 0 ? h1[0] : h1[1];
#pragma unroll
      for (int q = 0; q < 16; ++q)
        p.D1[(int64_t)(32 * ob + ru(q) + h4) * p.Np + b] = acc[q] * (1.f - hh[q] * hh[q]);
    });
    const float sm = wave_sum(h == 0 ? m : 0.f), sk = wave_sum(h == 0 ? kl : 0.f), sd = wave_sum(dist);
    if (lane == 0) {
      p.part[tile * p.pstride + 0] = sm;
      p.part[tile * p.pstride + 1] = sk;
      p.part[tile * p.pstride + 2] = sd;
    }
    // log_scale partials: unit j lives in (block ib, reg q, half h) with j = 32 ib + ru(q) + 4h
#pragma unroll
    for (int ib = 0; ib < C::NB_AOUT; ++ib)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        float v = gls[ib * 16 + q];
        // sum over the 32 samples of this half
#pragma unroll
        for (int off = 16; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        const int j = 32 * ib + ru(q) + h4;
        if (s == 0 && j < C::AOUT) p.part[tile * p.pstride + 3 + j] = v;
      }
  }
}

// Basic Actor.act (basic_model.py:32-51) continuous: mu = tanh(fc3)*lim;
// a = mu + sigma * eps (eps NULL -> deterministic mu); logp = Normal(mu, sigma).log_prob(a).sum()
template <class C>
__global__ __launch_bounds__(256) void k_onp_act(OnpArgs p) {
  SPP_ONP_PROLOGUE
  for (int tile = blockIdx.x * 4 + w; tile < ntiles; tile += gridDim.x * 4) {
    const int b = tile * 32 + s;
    const bool valid = b < p.N;
    const int br = valid ? b : 0;
    f32x16 x[C::NB_OB], h1[2], h2[2];
    onp_load_x<C>(x, p, br, valid, h4);
    onp_trunk<C>(p.actor, x, tbl, img, bl, h1, h2);
    float lp = 0.f;
    dense<2, C::RV_H>(p.actor.W3, C::NB_AOUT, h2, tbl + p.actor.tb3, [&](int ob, const f32x16& acc) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int j = 32 * ob + ru(q) + h4;
        if (j < C::AOUT) {
          const float sc = expf(p.log_scale[j]);
          const float mu = fmul_rn(tanhf(acc[q]), p.lim[j]);
          const float a = (p.EPS && valid) ? fadd_rn(mu, fmul_rn(sc, p.EPS[(int64_t)br * C::AOUT + j])) : mu;
          const float d = fsub_rn(a, mu);
          lp += fsub_rn(fsub_rn(fdiv_rn(-fmul_rn(d, d), 2.f * fmul_rn(sc, sc)), logf(sc)), kLogSqrt2PiO);
          if (valid) p.ACT_OUT[(int64_t)br * C::AOUT + j] = a;
        }
      }
    });
    lp += __shfl_xor(lp, 32, 64);
    if (valid && h == 0 && p.LP_OUT) p.LP_OUT[b] = lp;
  }
}
#undef SPP_ONP_PROLOGUE

// losses: out[0] critic loss (mean) | actor: out[0] -mean(min), out[1] KL, out[2] dist MSE;
// log_scale grad (state_dict slot 0..aout-1 of the actor grad buffer) += partials - ent_coef
__global__ void k_onp_finish_critic(const float* part, int ntiles, int stride, int N, float* out) {
  const double l = block_sum(part, ntiles, stride, 0);
  if (threadIdx.x == 0 && out) out[0] = (float)(l / N);
}
// out[3] = entropy of Independent(Normal(mu, exp(log_scale))) = sum_j 0.5 + 0.5 log(2 pi) + log_scale_j.
// All 3 + aout partial slots are reduced in one pass (one sync): thread t sums slot t % ns over the
// tiles t / ns, t / ns + nsub, ...; the nsub sub-sums of a slot are then added in order.
__global__ void k_onp_finish_actor(const float* part, int ntiles, int stride, int N, int aout, float ent_coef,
                                   const float* log_scale, float* gls, float* out) {
  __shared__ double red[256];
  const int ns = 3 + aout, nsub = (int)blockDim.x / ns, t = threadIdx.x;
  const int slot = t % ns, sub = t / ns;
  double s = 0.0;
  if (sub < nsub)
    for (int i = sub; i < ntiles; i += nsub) s += (double)part[(int64_t)i * stride + slot];
  red[t] = s;
  __syncthreads();
  if (t < ns) {
    double tot = 0.0;
    for (int k = 0; k < nsub; ++k) tot += red[k * ns + t];
    if (t == 0 && out) out[0] = (float)(-tot / N);
    if (t == 1 && out) out[1] = (float)(tot / N);
    if (t == 2 && out) out[2] = (float)(tot / ((double)N * aout));
    if (t >= 3) gls[t - 3] = (float)(tot - (double)ent_coef);
  }
  if (t == 0 && out) {
    double ent = 0.0;
    for (int j = 0; j < aout; ++j) ent += 0.5 + 0.91893853320467274178 + (double)log_scale[j];
    out[3] = (float)ent;
  }
}

}  // namespace spp
