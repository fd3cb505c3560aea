// Weight gradients as split-K MFMA GEMMs over the batch:
//   dW[n][k] = sum_b A[n][b] * X[k][b],   db[n] = sum_b A[n][b]
// A = per-sample layer-output gradients (delta) and X = layer inputs, both
// feature-major [rows][Bp] as written by the per-sample kernels.  One
// workgroup (8 waves) owns the whole <=256x256 output of one job for one
// sample range; partial slabs are summed in a fixed order (deterministic).
#include "common.h"
#include "internal.h"

namespace spp {

constexpr int kDwThreads = 512;
constexpr int kDwChunk = 32;       // samples per LDS stage
constexpr int kDwPad = kDwChunk + 1;

__global__ __launch_bounds__(kDwThreads, 1) void k_dw(const DwJob* __restrict__ jobs, const int* __restrict__ item_job,
                                                      const int* __restrict__ item_split) {
  __shared__ float sA[256 * kDwPad];
  __shared__ float sX[256 * kDwPad];
  const int item = blockIdx.x;
  const DwJob J = jobs[item_job[item]];
  const int split = item_split[item];
  const int t = threadIdx.x, w = t >> 6, lane = t & 63, h = lane >> 5;
  const int64_t ld = J.Bp;
  const int64_t b_begin = (int64_t)split * J.split_len;
  const int64_t b_end = min<int64_t>(b_begin + J.split_len, (int64_t)J.Bp);
  const int N = J.N, K = J.K0 + J.K1;
  const int Nr = (N + 31) & ~31, Kr = (K + 31) & ~31;
  // wave tile: n blocks [4*(w>>2), +4), k blocks [2*(w&3), +2)
  const int nb0 = 4 * (w >> 2), kb0 = 2 * (w & 3);
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero16();
  float dbsum = 0.f;
  // staging: each thread moves 4 float4 of A and 4 of X per stage
  float4 ra[4], rx[4];
  auto gload = [&](int64_t b0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (t >> 3) + 64 * i, c4 = t & 7;
      const int64_t off = b0 + 4 * c4;
      ra[i] = row < N ? *reinterpret_cast<const float4*>(J.A + (int64_t)row * ld + off) : make_float4(0, 0, 0, 0);
      const float* xr = row < J.K0 ? J.X0 + (int64_t)row * ld : (row < K ? J.X1 + (int64_t)(row - J.K0) * ld : nullptr);
      rx[i] = xr ? *reinterpret_cast<const float4*>(xr + off) : make_float4(0, 0, 0, 0);
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (t >> 3) + 64 * i, c = 4 * (t & 7);
      if (row < Nr) {
        float* d = sA + row * kDwPad + c;
        d[0] = ra[i].x; d[1] = ra[i].y; d[2] = ra[i].z; d[3] = ra[i].w;
      }
      if (row < Kr) {
        float* d = sX + row * kDwPad + c;
        d[0] = rx[i].x; d[1] = rx[i].y; d[2] = rx[i].z; d[3] = rx[i].w;
      }
    }
  };
  const bool nact[4] = {32 * (nb0 + 0) < N, 32 * (nb0 + 1) < N, 32 * (nb0 + 2) < N, 32 * (nb0 + 3) < N};
  const bool kact[2] = {32 * (kb0 + 0) < K, 32 * (kb0 + 1) < K};
  if (b_begin < b_end) gload(b_begin);
  for (int64_t b0 = b_begin; b0 < b_end; b0 += kDwChunk) {
    __syncthreads();
    lstore();
    __syncthreads();
    if (b0 + kDwChunk < b_end) gload(b0 + kDwChunk);
    if (J.db && t < 2 * Nr && (t >> 1) < N) {
      const float* rowp = sA + (t >> 1) * kDwPad + 16 * (t & 1);
#pragma unroll
      for (int c = 0; c < 16; ++c) dbsum += rowp[c];
    }
#pragma unroll
    for (int kk = 0; kk < kDwChunk / 2; ++kk) {
      const int col = 2 * kk + h;
      float bf[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = kact[j] ? sX[(32 * (kb0 + j) + (lane & 31)) * kDwPad + col] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (!nact[i]) continue;
        const float af = sA[(32 * (nb0 + i) + (lane & 31)) * kDwPad + col];
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (kact[j]) acc[i][j] = mfma(af, bf[j], acc[i][j]);
      }
    }
  }
  // write the partial (or final) result
  float* out = J.nsplit == 1 ? nullptr : J.slab + (int64_t)split * J.slab_stride;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (!nact[i] || !kact[j]) continue;
      const int k = 32 * (kb0 + j) + (lane & 31);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int n = 32 * (nb0 + i) + unit_of(q, h);
        if (n < N && k < K) {
          if (out) out[(int64_t)n * K + k] = acc[i][j][q];
          else J.dW[(int64_t)n * K + k] = acc[i][j][q];
        }
      }
    }
  if (J.db) {
    const float tot = dbsum + __shfl_xor(dbsum, 1, 64);
    if ((t & 1) == 0 && (t >> 1) < N) {
      if (out) out[(int64_t)N * K + (t >> 1)] = tot;
      else J.db[t >> 1] = tot;
    }
  }
}

// Fixed-order reduction of the split slabs.
__global__ void k_dw_reduce(const DwJob* __restrict__ jobs) {
  const DwJob J = jobs[blockIdx.y];
  if (J.nsplit == 1) return;
  const int N = J.N, K = J.K0 + J.K1;
  const int64_t total = (int64_t)N * K + (J.db ? N : 0);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int sp = 0; sp < J.nsplit; ++sp) s += J.slab[(int64_t)sp * J.slab_stride + e];
    if (e < (int64_t)N * K) J.dW[e] = s;
    else J.db[e - (int64_t)N * K] = s;
  }
}

}  // namespace spp
