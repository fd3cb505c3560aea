// Shared pieces of the persistent AcM regression SGD (rltoolkit/basic_model.py:108-132, 64-32 tanh,
// out = tanh(fc3) * ac_lim): AcMTrainer.update_acm's inner loop (acm/acm.py:266-303: shuffled
// minibatches, MSE, Adam) or update_acm_batches (:356-372), many sequential steps in ONE launch.
// The kernel itself is k_mlp_sgd (sgd_mlp.hip: every layer on the fp32 matrix cores); this file holds the
// write-through slab accessors and the bounded arrival barrier of its multi-workgroup form.
#include "common.h"

namespace spp {

// Arrival barrier of the multi-workgroup SGD.  The counter address is kept in a VGPR so the add and the
// polls are vector-memory operations.  Bounded: after `spin` polls (0: kSgdSpins, ~0.2 s; < 0: none, the test
// hook's forced timeout) a wait times out, sets *err and every later wait of the launch returns at once.
// The per-step gradient hand-over between the workgroups is write-through: every slab word is stored
// sc1 (aux 16) and every load of slab words is an sc1 load, so the arrival needs no agent-scope release
// (its L2 write-back cost ~6.5 us per step with a freshly written 18 KB slab) and no acquire
// (cdna_hip_programming.md Guideline 16, R1 with sc1 loads; MI355X_MICROARCH.md visibility table row 1):
// stores -> every wave's vmcnt(0) -> workgroup barrier -> lane 0 relaxed agent add -> relaxed poll -> barrier.
constexpr int kSc1 = 16;  // buffer cache-policy operand: sc1
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sgd_rsrc(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void slab_st4(__amdgpu_buffer_rsrc_t r, int idx, float4 v) {
  typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r, 4u * (uint32_t)idx, 0, kSc1);
}
__device__ __forceinline__ void slab_st1(__amdgpu_buffer_rsrc_t r, int idx, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, 4u * (uint32_t)idx, 0, kSc1);
}
__device__ __forceinline__ float4 slab_ld4(__amdgpu_buffer_rsrc_t r, int idx) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, 4u * (uint32_t)idx, 0, kSc1));
}
__device__ __forceinline__ float slab_ld1(__amdgpu_buffer_rsrc_t r, int idx) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, 4u * (uint32_t)idx, 0, kSc1));
}
// idle(): work of the workgroup's threads while lane 0 waits for the other workgroups (thread 0 runs it after
// its poll); it must not touch the handed-over data
constexpr int kSgdSpins = 1 << 23;
// The arrival counter is sharded over kSgdShards ints, each on its own 128-B line (ctr[kSgdShardStride k]): a
// workgroup adds to shard blockIdx % kSgdShards (the XCD it is dealt to under round-robin placement -- speed only,
// the sum is what is waited for), so the G arrivals of a step meet on 8 lines instead of serialising on one (one
// device-scope atomic costs ~12 ns at the memory side: MI355X_MICROARCH.md fan-in row), and the poll reads the 8
// shards at once and waits for their sum.
#ifndef SPP_SGD_SHARDS
#define SPP_SGD_SHARDS 8
#endif
#ifndef SPP_SGD_SHARD_STRIDE
#define SPP_SGD_SHARD_STRIDE 32
#endif
#ifndef SPP_SGD_POLL_SLEEP
#define SPP_SGD_POLL_SLEEP 1
#endif
constexpr int kSgdShards = SPP_SGD_SHARDS, kSgdShardStride = SPP_SGD_SHARD_STRIDE;
// Published parameters (the second hand-off of a step) in kSgdPubReps replicas, kMlSlabMax floats apart: every
// workgroup reloads ALL parameters after the publish, so with one copy the G workgroups' reloads of the same few KB
// meet on the few memory channels that hold them; workgroup g reads replica g % kSgdPubReps (its XCD's under
// round-robin placement -- speed only, every replica holds the same values).
#ifndef SPP_SGD_PUB_REPS
#define SPP_SGD_PUB_REPS 1
#endif
constexpr int kSgdPubReps = SPP_SGD_PUB_REPS;
// The shard reduce after the first hand-off: 1 = each thread sums a strided group of the G slabs' chunks as it
// loads them and Adam adds the groups' sums; 0 = the chunks are staged in LDS and summed by one thread per slot.
#ifndef SPP_SGD_PRED
#define SPP_SGD_PRED 1
#endif
template <class Idle>
__device__ __forceinline__ void sgd_arrive_wait_wt(int* ctr, int target, int* err, int* s_dead, int spin, Idle&& idle) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 slab stores are written through
  __syncthreads();                                   // ... and every other wave's
  if (threadIdx.x == 0 && !*s_dead) {
    int off = 0;
    asm volatile("" : "+v"(off));
    int* c = ctr + off;
    __hip_atomic_fetch_add(c + kSgdShardStride * (blockIdx.x % kSgdShards), 1, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (spin < 0) {  // test hook: every wait gives up at once (a co-residency miss, deterministically)
      *s_dead = 1;
      err[off] = 1;
    } else {
      const int limit = spin > 0 ? spin : kSgdSpins;
      int spins = 0;
      while (true) {
        int v[kSgdShards];
#pragma unroll
        for (int k = 0; k < kSgdShards; ++k)
          v[k] = __hip_atomic_load(c + kSgdShardStride * k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int sum = 0;
#pragma unroll
        for (int k = 0; k < kSgdShards; ++k) sum += v[k];
        if (sum >= target) break;
        if (SPP_SGD_POLL_SLEEP > 0) __builtin_amdgcn_s_sleep(SPP_SGD_POLL_SLEEP);
        if (++spins > limit) {
          *s_dead = 1;
          err[off] = 1;
          break;
        }
      }
    }
  }
  idle();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the slab loads below the poll
  __syncthreads();
}
__device__ __forceinline__ void sgd_arrive_wait_wt(int* ctr, int target, int* err, int* s_dead, int spin) {
  sgd_arrive_wait_wt(ctr, target, err, s_dead, spin, [] {});
}

}  // namespace spp
