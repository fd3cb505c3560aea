// Shared device/host helpers for libspprl (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

// bf16 SAC kernel sets: fuse the critics' fc3 weight gradient into the critic phase (1) or hand h2 / dq to a
// k_dw job (0).  Compile-time A/B (tools/build_variant.py -DSPP_BF16_FUSE3=...); fp32 sets always fuse.
// Measured round 5 (Ant bf16, 100 steps, profiles/r05/ab_fuse3_*.json): fused critic phase 1.8145 ms,
// unfused 1.6787 ms (+0.027 ms of k_dw), step 6.79 -> 6.71 ms: the bf16 default is the k_dw job.
// The bf16 acm_critic sets' critic phase with two 32-sample tiles per wave (k_sac_critic_phase2, sac_bf.h; A/B) or
// the one-tile kernel (0, the default).  Measured round 6 (Ant bf16, profiles/r06/bf16_two_tile/): the two-tile
// kernel's 256-wide LDS-input layers run 1.3-1.7x faster per tile, but its critic phase took 1.93 ms against
// 1.66 ms: the first layers and their HBM input loads slowed down more than the shared fragments saved, and the
// 6.25 pairs per wave leave a 7-pair tail.
#ifndef SPP_BF16_TWO_TILES
#define SPP_BF16_TWO_TILES 0
#endif
#ifndef SPP_BF16_FUSE3
#define SPP_BF16_FUSE3 0
#endif

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace spp {

constexpr int kWave = 64;
constexpr int kTile = 32;    // samples per wave tile (MFMA N dimension)
constexpr int kHidden = 256; // actor / critic hidden width (sac/models.py:17-20)

// ---------------------------------------------------------------- host error state
void set_error(const char* fmt, ...);
const char* get_error();

#define SPP_CHECK_HIP(expr)                                                        \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) {                                                        \
      ::spp::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr, hipGetErrorString(e_)); \
      return SPP_E_HIP;                                                            \
    }                                                                              \
  } while (0)

#define SPP_REQUIRE(cond, code, ...)        \
  do {                                      \
    if (!(cond)) {                          \
      ::spp::set_error(__VA_ARGS__);        \
      return code;                          \
    }                                       \
  } while (0)

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }
inline int cdiv(int64_t x, int64_t m) { return (int)((x + m - 1) / m); }

// ---------------------------------------------------------------- device helpers
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// 32x32x2 f32 MFMA D-layout: lane l, register r holds row (r&3)+8(r>>2)+4(l>>5),
// column l&31.  Rows are hidden units, columns are the wave's 32 samples.
__device__ __forceinline__ int unit_of(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// Registers of an input block that carry at least one unit < K (units of
// register group g = r>>2 are [8g, 8g+8)).
constexpr int regs_valid(int K, int ib) {
  return (K - 32 * ib) <= 0 ? 0 : ((K - 32 * ib) >= 32 ? 16 : 4 * ((K - 32 * ib + 7) / 8));
}
constexpr int blocks_of(int n) { return (n + 31) / 32; }

// float-exact (no contraction) helpers where the reference rounds twice
// Separately rounded fp32 ops: hipcc contracts a*b+c into an FMA by default
// (-ffp-contract=fast, and __fmul_rn/__fadd_rn are plain operators), which
// changes rounding against the reference's torch/numpy evaluation order.
__device__ __forceinline__ float fmul_rn(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ float fadd_rn(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}
__device__ __forceinline__ float fsub_rn(float a, float b) {
#pragma clang fp contract(off)
  return a - b;
}
__device__ __forceinline__ float fdiv_rn(float a, float b) { return __fdiv_rn(a, b); }

// numpy's _lerp of np.percentile(..., 'linear') between the order statistics a <= b at fraction g, with
// its two separate fp64 roundings (a contracted fma can land on the other side of an fp32 rounding
// midpoint of the final cast)
__device__ __forceinline__ double np_lerp(double a, double b, double g) {
#pragma clang fp contract(off)
  const double diff = b - a;
  return g >= 0.5 ? b - diff * (1.0 - g) : a + diff * g;
}
// its interpolation fraction: virtual index (n - 1) q rounded BEFORE the floor is taken off (a contracted
// fma(q, n - 1, -floor) keeps the product's low bits and moves g by ~1e-12)
__device__ __forceinline__ double np_frac(int64_t n, double q) {
#pragma clang fp contract(off)
  const double vi = (double)(n - 1) * q;
  return vi - floor(vi);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------- Philox4x32-10
struct u32x4 { uint32_t x, y, z, w; };
__host__ __device__ __forceinline__ u32x4 philox(uint64_t key64, uint64_t ctr_hi, uint64_t ctr_lo) {
  uint32_t k0 = (uint32_t)key64, k1 = (uint32_t)(key64 >> 32);
  uint32_t c0 = (uint32_t)ctr_lo, c1 = (uint32_t)(ctr_lo >> 32), c2 = (uint32_t)ctr_hi, c3 = (uint32_t)(ctr_hi >> 32);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1; c3 = (uint32_t)p0; c0 = n0; c2 = n2;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}
__device__ __forceinline__ float u01(uint32_t x) { return ((x >> 8) + 0.5f) * (1.0f / 16777216.0f); }
// two standard normals from one philox word pair (Box-Muller)
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float& n0, float& n1) {
  float u = u01(a), v = u01(b);
  float r = sqrtf(-2.f * logf(u));
  float s, c;
  sincosf(6.283185307179586f * v, &s, &c);
  n0 = r * c;
  n1 = r * s;
}

}  // namespace spp
