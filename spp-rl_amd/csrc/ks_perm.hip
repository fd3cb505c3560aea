// Device random permutation of [0, n): the shuffle of a DataLoader(shuffle=True) epoch
// (rltoolkit/acm/acm.py:275 for update_acm, acm/on_policy.py:176-190 / algorithms/ppo/ppo.py:174-188 for the
// PPO minibatch epochs) drawn on the device: one 64-bit Philox4x32-10 key per index (counter = offset + i under
// the caller's seed), then a stable LSD radix sort of (key, index) pairs; the permutation is the sorted index
// column.  torch.randperm on the device stalls the stream for 0.3-0.7 ms of host-side work per call (merge /
// duplicate-key passes between launches, measured in the PPO kernel trace); this is two launches and a sort
// with no host round trip.  Deterministic for a (seed, offset); not the reference's CPU generator stream
// (its permutation values are never reproduced: DESIGN.md §2).
#include <rocprim/device/device_radix_sort.hpp>

#include "common.h"
#include "spprl.h"

namespace spp {

__global__ void k_perm_keys(uint64_t* keys, int64_t* idx, int64_t n, uint64_t seed, uint64_t offset) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const u32x4 r = philox(seed, 0x5045524dULL, offset + (uint64_t)i);  // "PERM" stream of the seed
    keys[i] = ((uint64_t)r.x << 32) | r.y;
    idx[i] = i;
  }
}

// Large n (>= kPermFeistelMin): a keyed Feistel bijection of [0, 2^b) (b = the even bit count covering n - 1, 6
// rounds, round keys from the seed's Philox "FEIS" stream at the offset, round function the murmur3 32-bit
// finaliser of (half ^ key)) restricted to [0, n) by cycle walking (re-apply while the image is >= n: a
// permutation of [0, n), about 1-4 applications per index).  One O(n) launch with no scratch instead of the
// 64-bit (key, index) radix sort (8 passes over 16 B per index: ~1.4 ms at the world-8 ACM ring's 14.4M rows).
// A pseudo-random permutation (Luby-Rackoff), not a uniform draw over all n! orders; the DataLoader's shuffle
// only asks for an unbiased order, and the small-n path that the order-frequency test covers stays the sort.
constexpr int64_t kPermFeistelMin = (int64_t)1 << 20;

__device__ __forceinline__ uint32_t perm_fmix(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

__global__ void k_perm_feistel(int64_t* out, int64_t n, int half, uint64_t seed, uint64_t offset) {
  const u32x4 ka = philox(seed, 0x46454953ULL, offset), kb = philox(seed, 0x46454953ULL, offset + 1);  // "FEIS"
  const uint32_t key[6] = {ka.x, ka.y, ka.z, ka.w, kb.x, kb.y};
  const uint32_t mask = (half >= 32) ? 0xffffffffu : ((1u << half) - 1u);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t x = (uint64_t)i;
    do {
      uint32_t L = (uint32_t)(x >> half) & mask, R = (uint32_t)x & mask;
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        const uint32_t t = L ^ (perm_fmix(R ^ key[r]) & mask);
        L = R;
        R = t;
      }
      x = ((uint64_t)L << half) | R;
    } while (x >= (uint64_t)n);
    out[i] = (int64_t)x;
  }
}

static size_t perm_sort_bytes(int64_t n) {
  size_t bytes = 0;
  rocprim::radix_sort_pairs(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr, (const int64_t*)nullptr,
                            (int64_t*)nullptr, (size_t)n, 0, 64, (hipStream_t)0, false);
  return bytes;
}

}  // namespace spp

using namespace spp;

extern "C" {

// scratch layout: keys_in [n] u64 | keys_out [n] u64 | idx_in [n] i64 | pad to 256 B | the sort's temporary
// storage (256-byte aligned like a hipMalloc block, whatever n: 24 n is only 8-byte aligned for odd n)
static size_t perm_tmp_offset(int64_t n) { return ((3 * (size_t)n * 8 + 255) / 256) * 256; }

int64_t sppRandPermScratchBytes(int64_t n) {
  if (n <= 0) return 0;
  if (n >= kPermFeistelMin) return 256;  // (the Feistel path needs none; a non-null buffer keeps one contract)
  return (int64_t)(perm_tmp_offset(n) + ((perm_sort_bytes(n) + 255) / 256) * 256);
}

sppStatus sppRandPerm(int64_t* out, int64_t n, uint64_t seed, uint64_t offset, void* scratch, int64_t scratch_bytes,
                      void* stream) {
  if (n == 0) return SPP_OK;
  if (!out || n < 0 || !scratch || scratch_bytes < sppRandPermScratchBytes(n)) return SPP_E_INVALID_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (n >= kPermFeistelMin) {
    int b = 0;
    while (b < 62 && ((uint64_t)(n - 1) >> b) != 0) ++b;
    b += b & 1;  // even: two equal halves
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(k_perm_feistel, dim3((unsigned)blocks), dim3(256), 0, st, out, n, b / 2, seed, offset);
    return hipGetLastError() == hipSuccess ? SPP_OK : SPP_E_HIP;
  }
  char* base = static_cast<char*>(scratch);
  uint64_t* keys_in = reinterpret_cast<uint64_t*>(base);
  uint64_t* keys_out = keys_in + n;
  int64_t* idx_in = reinterpret_cast<int64_t*>(keys_out + n);
  void* tmp = base + perm_tmp_offset(n);
  size_t tmp_bytes = (size_t)scratch_bytes - perm_tmp_offset(n);
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_perm_keys, dim3((unsigned)blocks), dim3(256), 0, st, keys_in, idx_in, n, seed, offset);
  if (hipGetLastError() != hipSuccess) return SPP_E_HIP;
  if (rocprim::radix_sort_pairs(tmp, tmp_bytes, keys_in, keys_out, idx_in, out, (size_t)n, 0, 64, st, false) !=
      hipSuccess)
    return SPP_E_HIP;
  return hipGetLastError() == hipSuccess ? SPP_OK : SPP_E_HIP;
}

}  // extern "C"
