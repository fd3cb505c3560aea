// Persistent minibatch SGD of the AcM (rltoolkit/basic_model.py:108-132, 64-32 tanh,
// out = tanh(fc3) * ac_lim) on one workgroup: AcMTrainer.update_acm's inner loop
// (acm/acm.py:266-303: shuffled minibatches, MSE, Adam) or update_acm_batches
// (:356-372), many sequential steps in ONE launch.
//
// The reference's ACM regression is a long chain of tiny dependent steps (64..128
// samples, ~4.5K parameters): issued as separate kernels it is launch-latency bound
// (tens of microseconds per step).  Here the parameters live in LDS for the whole
// launch, every step's batch is gathered from the HBM replay ring straight into LDS,
// forward / backward run from LDS, and each thread keeps the gradient and Adam
// moments of the parameters it owns in registers.
//
// LDS layout (augmented, bias as an extra input column equal to 1):
//   W1a [64][I1P]  (I1P = round_up(IN + 1, 4); column IN = fc1.bias)
//   W2a [32][68]   (column 64 = fc2.bias)
//   W3a [AC][36]   (column 32 = fc3.bias)
//   X  [BS][I1P]  (X[b][IN] = 1), H1 [BS][68] (H1[b][64] = 1), H2 [BS][36] (H2[b][32] = 1)
// Gradient "quads" = 4 consecutive augmented columns of one row; thread t owns quads
// t, t + 256, ...; padding columns have zero inputs, so their gradient, moments and
// parameters stay exactly 0.
#include "replay.h"

namespace spp {

constexpr int kSgdThreads = 256;
constexpr int kSgdMaxBatch = 128;

struct AcmSgdArgs {
  ReplayDev r;
  const int64_t* idx;  // [nsteps * bs] ring timestep rows, consumed in order
  int nsteps, bs;
  float* params;       // canonical AcM flat buffer (state_dict order)
  float* m;            // Adam exp_avg
  float* v;            // Adam exp_avg_sq
  float lr;
  int64_t step0;       // Adam steps already taken
  const float* lim;    // [ac]
  float* loss_sum;     // += sum of the steps' batch losses (fp32 scalar)
};

template <int IN, int AC>
struct SgdCfg {
  static constexpr int I1P = (IN + 1 + 3) / 4 * 4;
  static constexpr int H1P = 68, H2P = 36;
  static constexpr int NQ1 = 64 * I1P / 4, NQ2 = 32 * H1P / 4, NQ3 = AC * H2P / 4;
  static constexpr int NQ = NQ1 + NQ2 + NQ3;
  static constexpr int RQ = (NQ + kSgdThreads - 1) / kSgdThreads;  // quads per thread
  static constexpr int NP = 64 * IN + 64 + 32 * 64 + 32 + AC * 32 + AC;  // canonical parameter count
};

// canonical flat index of augmented (layer, row, col); -1 for padding
template <class C, int IN, int AC>
__device__ __forceinline__ int sgd_canon(int layer, int row, int col) {
  if (layer == 0) {
    if (col < IN) return row * IN + col;
    return col == IN ? 64 * IN + row : -1;
  }
  if (layer == 1) {
    const int o = 64 * IN + 64;
    if (col < 64) return o + row * 64 + col;
    return col == 64 ? o + 32 * 64 + row : -1;
  }
  const int o = 64 * IN + 64 + 32 * 64 + 32;
  if (col < 32) return o + row * 32 + col;
  return col == 32 ? o + AC * 32 + row : -1;
}

// quad q -> (layer, row, first column)
template <class C>
__device__ __forceinline__ void sgd_quad(int q, int& layer, int& row, int& c0) {
  if (q < C::NQ1) {
    layer = 0; row = q / (C::I1P / 4); c0 = 4 * (q % (C::I1P / 4));
  } else if (q < C::NQ1 + C::NQ2) {
    q -= C::NQ1;
    layer = 1; row = q / (C::H1P / 4); c0 = 4 * (q % (C::H1P / 4));
  } else {
    q -= C::NQ1 + C::NQ2;
    layer = 2; row = q / (C::H2P / 4); c0 = 4 * (q % (C::H2P / 4));
  }
}

template <int IN, int AC>
__global__ __launch_bounds__(kSgdThreads, 1) void k_acm_sgd(AcmSgdArgs a) {
  using C = SgdCfg<IN, AC>;
  constexpr int I1P = C::I1P, H1P = C::H1P, H2P = C::H2P;
  __shared__ __attribute__((aligned(16))) float W1[64 * I1P];
  __shared__ __attribute__((aligned(16))) float W2[32 * H1P];
  __shared__ __attribute__((aligned(16))) float W3[AC * H2P];
  __shared__ __attribute__((aligned(16))) float X[kSgdMaxBatch * I1P];
  __shared__ __attribute__((aligned(16))) float H1[kSgdMaxBatch * H1P];  // h1, later dz1
  __shared__ __attribute__((aligned(16))) float H2[kSgdMaxBatch * H2P];
  __shared__ __attribute__((aligned(16))) float D2[kSgdMaxBatch * 32];
  __shared__ float D3[kSgdMaxBatch * AC];
  __shared__ float Y[kSgdMaxBatch * AC];
  __shared__ float lsum[kSgdThreads / 64];
  __shared__ int64_t rows[kSgdMaxBatch][3];
  const int t = threadIdx.x;
  const int bs = a.bs;
  const int ob = IN / 2;
  auto wrow = [&](int layer, int row) -> float* {  // augmented row of a layer's image
    return layer == 0 ? W1 + row * I1P : (layer == 1 ? W2 + row * H1P : W3 + row * H2P);
  };
  // parameters -> augmented LDS images (zero padding)
  for (int i = t; i < 64 * I1P; i += kSgdThreads) {
    const int c = sgd_canon<C, IN, AC>(0, i / I1P, i % I1P);
    W1[i] = c >= 0 ? a.params[c] : 0.f;
  }
  for (int i = t; i < 32 * H1P; i += kSgdThreads) {
    const int c = sgd_canon<C, IN, AC>(1, i / H1P, i % H1P);
    W2[i] = c >= 0 ? a.params[c] : 0.f;
  }
  for (int i = t; i < AC * H2P; i += kSgdThreads) {
    const int c = sgd_canon<C, IN, AC>(2, i / H2P, i % H2P);
    W3[i] = c >= 0 ? a.params[c] : 0.f;
  }
  // owned quads: Adam moments in registers
  float4 m4[C::RQ], v4[C::RQ];
#pragma unroll
  for (int k = 0; k < C::RQ; ++k) {
    const int q = t + kSgdThreads * k;
    float mm[4] = {0.f, 0.f, 0.f, 0.f}, vv[4] = {0.f, 0.f, 0.f, 0.f};
    if (q < C::NQ) {
      int layer, row, c0;
      sgd_quad<C>(q, layer, row, c0);
      for (int j = 0; j < 4; ++j) {
        const int c = sgd_canon<C, IN, AC>(layer, row, c0 + j);
        if (c >= 0) {
          mm[j] = a.m[c];
          vv[j] = a.v[c];
        }
      }
    }
    m4[k] = make_float4(mm[0], mm[1], mm[2], mm[3]);
    v4[k] = make_float4(vv[0], vv[1], vv[2], vv[3]);
  }
  float loss_acc = 0.f;
  const float inv_n = 1.f / (float)(bs * AC);
  __syncthreads();
  for (int st = 0; st < a.nsteps; ++st) {
    // ---- gather the batch: X[b] = [obs | next_obs | 1 | 0..], Y[b] = acm action (acm.py:260-264)
    if (t < bs) {
      const int64_t row = a.idx[(int64_t)st * bs + t];
      rows[t][0] = row;
      rows[t][1] = a.r.obs_idx[row];
      rows[t][2] = a.r.next_idx[row];
    }
    __syncthreads();
    for (int i = t; i < bs * I1P; i += kSgdThreads) {
      const int b = i / I1P, k = i % I1P;
      float x = 0.f;
      if (k < ob) x = a.r.obs[rows[b][1] * ob + k];
      else if (k < IN) x = a.r.obs[rows[b][2] * ob + (k - ob)];
      else if (k == IN) x = 1.f;
      X[i] = x;
    }
    for (int i = t; i < bs * AC; i += kSgdThreads) Y[i] = a.r.acm[rows[i / AC][0] * AC + (i % AC)];
    __syncthreads();
    // ---- forward: h1 = tanh(fc1 x), h2 = tanh(fc2 h1), out = tanh(fc3 h2) * lim
    for (int i = t; i < bs * H1P; i += kSgdThreads) {
      const int b = i / H1P, j = i % H1P;
      float z = 0.f;
      if (j < 64) {
        const float4* w = reinterpret_cast<const float4*>(W1 + j * I1P);
        const float4* x = reinterpret_cast<const float4*>(X + b * I1P);
#pragma unroll
        for (int k = 0; k < I1P / 4; ++k) {
          const float4 ww = w[k], xx = x[k];
          z = fmaf(ww.x, xx.x, z); z = fmaf(ww.y, xx.y, z); z = fmaf(ww.z, xx.z, z); z = fmaf(ww.w, xx.w, z);
        }
        z = tanhf(z);
      } else {
        z = j == 64 ? 1.f : 0.f;
      }
      H1[i] = z;
    }
    __syncthreads();
    for (int i = t; i < bs * H2P; i += kSgdThreads) {
      const int b = i / H2P, j = i % H2P;
      float z = 0.f;
      if (j < 32) {
        const float4* w = reinterpret_cast<const float4*>(W2 + j * H1P);
        const float4* x = reinterpret_cast<const float4*>(H1 + b * H1P);
#pragma unroll
        for (int k = 0; k < H1P / 4; ++k) {
          const float4 ww = w[k], xx = x[k];
          z = fmaf(ww.x, xx.x, z); z = fmaf(ww.y, xx.y, z); z = fmaf(ww.z, xx.z, z); z = fmaf(ww.w, xx.w, z);
        }
        z = tanhf(z);
      } else {
        z = j == 32 ? 1.f : 0.f;
      }
      H2[i] = z;
    }
    __syncthreads();
    // out, MSE loss, dz3 = dL/d fc3 = 2 (out - y) / n * lim * (1 - tanh^2)
    float lpart = 0.f;
    for (int i = t; i < bs * AC; i += kSgdThreads) {
      const int b = i / AC, c = i % AC;
      const float4* w = reinterpret_cast<const float4*>(W3 + c * H2P);
      const float4* x = reinterpret_cast<const float4*>(H2 + b * H2P);
      float z = 0.f;
#pragma unroll
      for (int k = 0; k < H2P / 4; ++k) {
        const float4 ww = w[k], xx = x[k];
        z = fmaf(ww.x, xx.x, z); z = fmaf(ww.y, xx.y, z); z = fmaf(ww.z, xx.z, z); z = fmaf(ww.w, xx.w, z);
      }
      const float th = tanhf(z), lim = a.lim[c];
      const float e = th * lim - Y[i];
      lpart = fmaf(e, e, lpart);
      D3[i] = 2.f * e * inv_n * lim * (1.f - th * th);
    }
    for (int o = 32; o > 0; o >>= 1) lpart += __shfl_xor(lpart, o, 64);
    if ((t & 63) == 0) lsum[t >> 6] = lpart;
    __syncthreads();
    if (t == 0) loss_acc += (lsum[0] + lsum[1] + lsum[2] + lsum[3]) * inv_n;
    // dz2 = (W3^T dz3) * (1 - h2^2)
    for (int i = t; i < bs * 32; i += kSgdThreads) {
      const int b = i / 32, j = i % 32;
      float g = 0.f;
#pragma unroll
      for (int c = 0; c < AC; ++c) g = fmaf(W3[c * H2P + j], D3[b * AC + c], g);
      const float h = H2[b * H2P + j];
      D2[i] = g * (1.f - h * h);
    }
    __syncthreads();
    // ---- gradients of the owned quads, part 1: layers 2 (dz2 x h1) and 3 (dz3 x h2)
    float4 g4[C::RQ];
#pragma unroll
    for (int k = 0; k < C::RQ; ++k) {
      g4[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      const int q = t + kSgdThreads * k;
      if (q >= C::NQ1 && q < C::NQ) {
        int layer, row, c0;
        sgd_quad<C>(q, layer, row, c0);
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        if (layer == 1) {
          for (int b = 0; b < bs; ++b) {
            const float d = D2[b * 32 + row];
            const float4 x = *reinterpret_cast<const float4*>(H1 + b * H1P + c0);
            acc.x = fmaf(d, x.x, acc.x); acc.y = fmaf(d, x.y, acc.y); acc.z = fmaf(d, x.z, acc.z); acc.w = fmaf(d, x.w, acc.w);
          }
        } else {
          for (int b = 0; b < bs; ++b) {
            const float d = D3[b * AC + row];
            const float4 x = *reinterpret_cast<const float4*>(H2 + b * H2P + c0);
            acc.x = fmaf(d, x.x, acc.x); acc.y = fmaf(d, x.y, acc.y); acc.z = fmaf(d, x.z, acc.z); acc.w = fmaf(d, x.w, acc.w);
          }
        }
        g4[k] = acc;
      }
    }
    __syncthreads();  // H1 (h1) is read above; it becomes dz1 below
    // dz1 = (W2^T dz2) * (1 - h1^2), in place of h1
    for (int i = t; i < bs * 64; i += kSgdThreads) {
      const int b = i / 64, j = i % 64;
      float g = 0.f;
#pragma unroll 8
      for (int r = 0; r < 32; ++r) g = fmaf(W2[r * H1P + j], D2[b * 32 + r], g);
      const float h = H1[b * H1P + j];
      H1[b * H1P + j] = g * (1.f - h * h);
    }
    __syncthreads();
    // part 2: layer 1 (dz1 x x)
#pragma unroll
    for (int k = 0; k < C::RQ; ++k) {
      const int q = t + kSgdThreads * k;
      if (q < C::NQ1) {
        int layer, row, c0;
        sgd_quad<C>(q, layer, row, c0);
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int b = 0; b < bs; ++b) {
          const float d = H1[b * H1P + row];
          const float4 x = *reinterpret_cast<const float4*>(X + b * I1P + c0);
          acc.x = fmaf(d, x.x, acc.x); acc.y = fmaf(d, x.y, acc.y); acc.z = fmaf(d, x.z, acc.z); acc.w = fmaf(d, x.w, acc.w);
        }
        g4[k] = acc;
      }
    }
    // ---- Adam (torch.optim.Adam, same operation order as k_adam) on the owned quads
    const double tstep = (double)(a.step0 + st + 1);
    const float neg_step = (float)(-((double)a.lr / (1.0 - pow(0.9, tstep))));
    const float bc2s = (float)sqrt(1.0 - pow(0.999, tstep));
    const float omb1 = 0.1f, b2 = 0.999f, omb2 = 0.001f, eps = 1e-8f;
    __syncthreads();  // every thread has read the parameters it needs (dz1 used W2)
#pragma unroll
    for (int k = 0; k < C::RQ; ++k) {
      const int q = t + kSgdThreads * k;
      if (q < C::NQ) {
        int layer, row, c0;
        sgd_quad<C>(q, layer, row, c0);
        float* p = wrow(layer, row) + c0;
        float gg[4] = {g4[k].x, g4[k].y, g4[k].z, g4[k].w};
        float mm[4] = {m4[k].x, m4[k].y, m4[k].z, m4[k].w};
        float vv[4] = {v4[k].x, v4[k].y, v4[k].z, v4[k].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float g = gg[j];
          mm[j] = fadd_rn(mm[j], fmul_rn(omb1, fsub_rn(g, mm[j])));
          vv[j] = fadd_rn(fmul_rn(vv[j], b2), fmul_rn(fmul_rn(omb2, g), g));
          const float denom = fadd_rn(fdiv_rn(sqrtf(vv[j]), bc2s), eps);
          p[j] = fadd_rn(p[j], fmul_rn(neg_step, fdiv_rn(mm[j], denom)));
        }
        m4[k] = make_float4(mm[0], mm[1], mm[2], mm[3]);
        v4[k] = make_float4(vv[0], vv[1], vv[2], vv[3]);
      }
    }
    __syncthreads();
  }
  // ---- write back parameters and moments (canonical layout)
#pragma unroll
  for (int k = 0; k < C::RQ; ++k) {
    const int q = t + kSgdThreads * k;
    if (q < C::NQ) {
      int layer, row, c0;
      sgd_quad<C>(q, layer, row, c0);
      const float* p = wrow(layer, row) + c0;
      const float mm[4] = {m4[k].x, m4[k].y, m4[k].z, m4[k].w}, vv[4] = {v4[k].x, v4[k].y, v4[k].z, v4[k].w};
      for (int j = 0; j < 4; ++j) {
        const int c = sgd_canon<C, IN, AC>(layer, row, c0 + j);
        if (c >= 0) {
          a.params[c] = p[j];
          a.m[c] = mm[j];
          a.v[c] = vv[j];
        }
      }
    }
  }
  if (t == 0) *a.loss_sum += loss_acc;
}

}  // namespace spp
