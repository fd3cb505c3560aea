// Weight gradients as split-K MFMA GEMMs over the batch:
//   dW[n][k] = sum_b A[n][b] * X[k][b],   db[n] = sum_b A[n][b]
// A = per-sample layer-output gradients (delta) and X = layer inputs, both
// feature-major [rows][Bp] as written by the per-sample kernels.
//
// One work item = (job, sample range).  A workgroup of 4 waves owns the whole
// <=256x256 output of its item: wave w holds the 128x128 quadrant
// (n blocks 4*(w>>1).., k blocks 4*(w&1)..) as 16 accumulator tiles.  The
// operands need no LDS: the sum over samples is order-free, so lane half h
// takes samples [b+8h, b+8h+8) of its row as two float4 and feeds them to 8
// consecutive MFMA k-steps for both A and X (same sample<->k map on both
// sides).  Each lane streams its 4 A rows and 4 X rows straight from HBM
// through an R-deep register ring (loads for step t+R-1 issued before step
// t's MFMAs; R from dw_ring, deeper for thin tile sets).  Partial slabs are
// summed in a fixed order by k_dw_reduce (deterministic, no atomics).
//
// Operand element types are per job (DwJob::a_bf / x_bf): the bf16 kernel sets store the
// activations and deltas they hand to this kernel as bf16 [rows][Bp] (half the bytes written
// and read back; the bf16 MFMA rounds fp32 operands to bf16 with the same conversion), while
// staged inputs (s, a), the per-sample dq and the head deltas stay fp32.  A bf16 operand
// row-step is one 16-B load of the lane half's 8 samples, fed to the MFMA as is.
#include "common.h"
#include "internal.h"

namespace spp {

constexpr int kDwThreads = 256;

// Steps (16 samples each) in flight for an NI x NJ tile set: the R-1 steps ahead should carry
// >= ~8K cycles of MFMA work (HBM latency under load), within ~168 VGPRs of operand ring.
// fp32: 8 x 64-cycle 32x32x2 MFMAs per block pair and step (4x4: R = 2); bf16: one 32-cycle
// 32x32x16 per block pair and step, so the ring runs as deep as the registers allow (bf16
// operand rows take one float4 per step, fp32 rows two).
template <int NI, int NJ, bool BF = false, bool ABF = false, bool XBF = false>
constexpr int dw_ring() {
  constexpr int cyc = NI * NJ * (BF ? 32 : 512);
  constexpr int want = 1 + (8192 + cyc - 1) / cyc;
  constexpr int cap = 168 / (4 * (NI * (ABF ? 1 : 2) + NJ * (XBF ? 1 : 2)));
  constexpr int r = want < cap ? want : cap;
  return r < 2 ? 2 : (r > 8 ? 8 : r);
}

// One step = 16 samples: lane half h takes samples [16t + 8h, +8) of each of
// its rows as two adjacent float4 (a full 64 B run per row and half), i.e. 8
// MFMA k-steps per row pair.
__device__ __forceinline__ bf16x8 pack8(const float4& a, const float4& b) {
  bf16x8 r;
  r[0] = (__bf16)a.x; r[1] = (__bf16)a.y; r[2] = (__bf16)a.z; r[3] = (__bf16)a.w;
  r[4] = (__bf16)b.x; r[5] = (__bf16)b.y; r[6] = (__bf16)b.z; r[7] = (__bf16)b.w;
  return r;
}

// BF: one v_mfma_f32_32x32x16_bf16 per (row block, column block) per 16-sample step: lane half
// h's 8 samples are exactly the MFMA's k = 8h + j slots on both operands (bf16 agents, mlp_bf16).
__device__ __forceinline__ bf16x8 as_bf8(const float4& a) { return __builtin_bit_cast(bf16x8, a); }
// sum of the 8 bf16 of a 16-B operand word (the bias gradient of a bf16 delta row)
__device__ __forceinline__ float sum_bf8(const float4& a) {
  const uint32_t w[4] = {__builtin_bit_cast(uint32_t, a.x), __builtin_bit_cast(uint32_t, a.y),
                         __builtin_bit_cast(uint32_t, a.z), __builtin_bit_cast(uint32_t, a.w)};
  float s[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    s[i] = __builtin_bit_cast(float, w[i] << 16) + __builtin_bit_cast(float, w[i] & 0xffff0000u);
  return (s[0] + s[1]) + (s[2] + s[3]);
}

// ABF / XBF: the A / X operand rows are bf16 (BF only); row pointers are then __bf16* cast to float*.
// Operand loads use the default cache policy: nt loads were measured slower (both lane
// halves of a wave reuse each L1 line).
__device__ __forceinline__ float4 dw_ld(const float* p) { return *reinterpret_cast<const float4*>(p); }

template <int NI, int NJ, bool DB, bool BF = false, bool ABF = false, bool XBF = false>
__device__ __forceinline__ void dw_tile(const float* const (&ap)[4], const float* const (&xp)[4], int nsteps,
                                        f32x16 (&acc)[4][4], float (&bs)[4]) {
  constexpr int R = dw_ring<NI, NJ, BF, ABF, XBF>();
  float4 ra[R][NI][2], rx[R][NJ][2];
  const float* a0[NI];
  const float* x0[NJ];
  static_for<0, NI>([&](auto I) { a0[I] = ap[I]; });
  static_for<0, NJ>([&](auto J) { x0[J] = xp[J]; });
  auto load = [&](auto SL, int t) {
    constexpr int sl = decltype(SL)::value;
    static_for<0, NI>([&](auto I) {
      if constexpr (ABF) {
        ra[sl][I][0] = dw_ld(reinterpret_cast<const float*>(reinterpret_cast<const __bf16*>(a0[I]) + 16 * t));
      } else {
        ra[sl][I][0] = dw_ld(a0[I] + 16 * t);
        ra[sl][I][1] = dw_ld(a0[I] + 16 * t + 4);
      }
    });
    static_for<0, NJ>([&](auto J) {
      if constexpr (XBF) {
        rx[sl][J][0] = dw_ld(reinterpret_cast<const float*>(reinterpret_cast<const __bf16*>(x0[J]) + 16 * t));
      } else {
        rx[sl][J][0] = dw_ld(x0[J] + 16 * t);
        rx[sl][J][1] = dw_ld(x0[J] + 16 * t + 4);
      }
    });
  };
  static_for<0, R - 1>([&](auto S) {
    if ((int)S < nsteps) load(S, (int)S);
  });
#pragma unroll 1
  for (int t0 = 0; t0 < nsteps; t0 += R) {
    static_for<0, R>([&](auto U) {
      constexpr int u = U;
      constexpr int sn = (u + R - 1) % R;
      if (t0 + u >= nsteps) return;
      const int tn = t0 + u + R - 1;
      if (tn < nsteps) load(IC<sn>{}, tn);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (BF) {
        static_for<0, NI>([&](auto I) {
          if constexpr (DB && ABF) {
            bs[I] += sum_bf8(ra[u][I][0]);
          } else if constexpr (DB) {
            const float4 a0 = ra[u][I][0], a1 = ra[u][I][1];
            bs[I] += ((a0.x + a0.y) + (a0.z + a0.w)) + ((a1.x + a1.y) + (a1.z + a1.w));
          }
          const bf16x8 av = ABF ? as_bf8(ra[u][I][0]) : pack8(ra[u][I][0], ra[u][I][1]);
          static_for<0, NJ>([&](auto J) {
            const bf16x8 xv = XBF ? as_bf8(rx[u][J][0]) : pack8(rx[u][J][0], rx[u][J][1]);
            acc[I][J] = mfma16(av, xv, acc[I][J]);
          });
        });
      } else {
        static_for<0, NI>([&](auto I) {
          static_for<0, 2>([&](auto P) {
            const float4 av = ra[u][I][P];
            if constexpr (DB) bs[I] += (av.x + av.y) + (av.z + av.w);
            static_for<0, NJ>([&](auto J) {
              const float4 xv = rx[u][J][P];
              acc[I][J] = mfma(av.x, xv.x, acc[I][J]);
              acc[I][J] = mfma(av.y, xv.y, acc[I][J]);
              acc[I][J] = mfma(av.z, xv.z, acc[I][J]);
              acc[I][J] = mfma(av.w, xv.w, acc[I][J]);
            });
          });
        });
      }
    });
  }
}

// 256 x 256 fp32 jobs (the hidden-layer weight gradients of the critics and the actor): the
// workgroup's operand rows are staged through LDS so every A / X byte leaves HBM once per item.
// (In dw_tile each A row is streamed by the two waves that share its row blocks and each X row by
// the two that share its column blocks: twice the bytes, ~4.9 TB/s at the MFMA rate.)
// Step = 32 samples = one 128-B line per row; the step's 512 rows ([A (256) | X (256)] x 128 B = 64 KiB)
// arrive by LDS-DMA (global_load_lds_dwordx4: 8 rows per wave-instruction, 16 per wave, no VGPR
// destination), one step ahead, into the other of two LDS buffers.  The LDS image is lane-linear
// (row r at 128 r bytes); the 16-B slot q of row r holds piece q ^ ((r >> 1) & 7) of the row (the
// swizzle is applied on the global SOURCE address and undone on the read), which makes the MFMA
// operand reads (lane c reads row c of its block, ds_read_b128) bank-conflict free.
typedef __attribute__((address_space(1))) void glob_void;
typedef __attribute__((address_space(3))) void lds_void;
__device__ __forceinline__ void dw_big_lds(const DwJob& J, int b_begin, int nsteps, int nb0, int kb0, bool db,
                                           f32x16 (&acc)[4][4], float (&bs)[4]) {
  __shared__ __attribute__((aligned(16))) float lds[2][512 * 32];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, h = lane >> 5, c = lane & 31;
  const int64_t ld = J.Bp;
  // instruction k of wave w: rows 128 w + 8 k + (lane >> 3), slot lane & 7 <- piece (lane & 7) ^ ((row >> 1) & 7)
  //   = (lane & 7) ^ ((lane >> 4) & 3) ^ (4 (k & 1))
  const int pe = (lane & 7) ^ ((lane >> 4) & 3);
  // wave-uniform row base (SGPRs) + one 32-bit per-lane offset per instruction parity
  // wave-uniform values forced into SGPRs (the job fields may arrive in VGPRs)
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const float* wsel = wu < 2 ? J.A : J.X0;
  const uint64_t wbits = (uint64_t)(size_t)wsel;
  const uint64_t wbu = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)wbits) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(wbits >> 32)) << 32);
  const int64_t ldu = (int64_t)__builtin_amdgcn_readfirstlane((int)ld);  // Bp < 2^31
  const int bbu = __builtin_amdgcn_readfirstlane(b_begin);
  const float* wb = opaque(reinterpret_cast<const float*>((size_t)wbu) + (int64_t)(128 * (wu & 1)) * ldu + bbu);
  const uint32_t off0 = (uint32_t)((lane >> 3) * ld + 4 * pe), off1 = off0 ^ 16u;  // pe ^ 4: 16 floats
  // The DMA is issued by inline asm: for the builtin the compiler cannot tell the LDS-DMA's
  // destination from the buffer being read and waits vmcnt(0) before every ds_read, which serialises
  // the next step's loads with this step's MFMAs.  Here the only wait is the explicit one before the
  // step's closing barrier (the loop holds no other vector-memory loads whose counts it could skew).
  auto issue = [&](int t, int buf) {
    const uint32_t dst = (uint32_t)(size_t)(lds_void*)&lds[buf][(128 * wu) * 32];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float* src = opaque(wb + ((int64_t)(8 * k) * ldu + 32 * t)) + ((k & 1) ? off1 : off0);
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(src), "s"(dst + 1024u * k)
                   : "memory");
    }
  };
  // Operand registers are double-buffered across the step's two sub-steps (16 samples each): the
  // reads of the next sub-step are in flight while the current one's 128 MFMAs issue, so no LDS
  // latency is exposed.  A step's sub-step 1 reads are complete (lgkmcnt) before the step's closing
  // barrier, after which buffer t & 1 may be refilled by DMA for step t + 2.
  const int sw = (c >> 1) & 7;  // the read-side swizzle of rows 32 b + c
  auto rd = [&](const float* L, int s, float4 (&ra)[4][2], float4 (&rx)[4][2]) {
    const int q0 = (4 * s + 2 * h) ^ sw, q1 = (4 * s + 2 * h + 1) ^ sw;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float* pa = L + (32 * (nb0 + i) + c) * 32;
      const float* px = L + (256 + 32 * (kb0 + i) + c) * 32;
      ra[i][0] = *reinterpret_cast<const float4*>(pa + 4 * q0);
      ra[i][1] = *reinterpret_cast<const float4*>(pa + 4 * q1);
      rx[i][0] = *reinterpret_cast<const float4*>(px + 4 * q0);
      rx[i][1] = *reinterpret_cast<const float4*>(px + 4 * q1);
    }
  };
  auto mm = [&](const float4 (&ra)[4][2], const float4 (&rx)[4][2]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const float4 av = ra[i][p];
        if (db) bs[i] += (av.x + av.y) + (av.z + av.w);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 xv = rx[j][p];
          acc[i][j] = mfma(av.x, xv.x, acc[i][j]);
          acc[i][j] = mfma(av.y, xv.y, acc[i][j]);
          acc[i][j] = mfma(av.z, xv.z, acc[i][j]);
          acc[i][j] = mfma(av.w, xv.w, acc[i][j]);
        }
      }
  };
  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (nsteps > 1) issue(1, 1);
  float4 ra0[4][2], rx0[4][2], ra1[4][2], rx1[4][2];
  rd(lds[0], 0, ra0, rx0);
#pragma unroll 1
  for (int t = 0; t < nsteps; ++t) {
    rd(lds[t & 1], 1, ra1, rx1);
    mm(ra0, rx0);
    if (t + 1 < nsteps) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // my DMA for t + 1 landed, my reads of t done
      __syncthreads();  // every wave's DMA landed and every wave is done reading buffer t & 1
      if (t + 2 < nsteps) issue(t + 2, t & 1);
      rd(lds[(t + 1) & 1], 0, ra0, rx0);
    }
    mm(ra1, rx1);
  }
}

// 256 x 256 jobs with bf16 A and X rows (the bf16 sets' hidden-layer weight gradients): the same LDS-DMA staging
// with a 64-sample step, which is again one 128-B line per row (8 slots of 8 bf16, the same swizzle): the rows are
// addressed as 4-byte words (ld = Bp / 2, the step 32 words), so the DMA issue is dw_big_lds's.  A step holds 4
// k-steps of v_mfma_f32_32x32x16_bf16; k-step s reads one 16-B slot per row, slot 2s + h (lane half h takes
// samples 8h..8h+7 of the k-step on both operands, as dw_tile's bf16 form), double-buffered across the k-steps.
// Per item the k-steps run in sample order, as in k_dw<true>.  Needs b_begin and the item's range multiples of 64.
__device__ __forceinline__ void dw_big_lds16(const DwJob& J, int b_begin, int nsteps, int nb0, int kb0, bool db,
                                             f32x16 (&acc)[4][4], float (&bs)[4]) {
  __shared__ __attribute__((aligned(16))) float lds[2][512 * 32];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, h = lane >> 5, c = lane & 31;
  const int64_t ld = J.Bp / 2;  // words per bf16 row
  const int pe = (lane & 7) ^ ((lane >> 4) & 3);
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const float* wsel = wu < 2 ? J.A : J.X0;
  const uint64_t wbits = (uint64_t)(size_t)wsel;
  const uint64_t wbu = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)wbits) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(wbits >> 32)) << 32);
  const int64_t ldu = (int64_t)__builtin_amdgcn_readfirstlane((int)ld);
  const int bbu = __builtin_amdgcn_readfirstlane(b_begin / 2);  // first sample's word
  const float* wb = opaque(reinterpret_cast<const float*>((size_t)wbu) + (int64_t)(128 * (wu & 1)) * ldu + bbu);
  const uint32_t off0 = (uint32_t)((lane >> 3) * ld + 4 * pe), off1 = off0 ^ 16u;
  auto issue = [&](int t, int buf) {
    const uint32_t dst = (uint32_t)(size_t)(lds_void*)&lds[buf][(128 * wu) * 32];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float* src = opaque(wb + ((int64_t)(8 * k) * ldu + 32 * t)) + ((k & 1) ? off1 : off0);
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(src), "s"(dst + 1024u * k)
                   : "memory");
    }
  };
  const int sw = (c >> 1) & 7;
  auto rd = [&](const float* L, int s, float4 (&ra)[4], float4 (&rx)[4]) {
    const int q = (2 * s + h) ^ sw;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ra[i] = *reinterpret_cast<const float4*>(L + (32 * (nb0 + i) + c) * 32 + 4 * q);
      rx[i] = *reinterpret_cast<const float4*>(L + (256 + 32 * (kb0 + i) + c) * 32 + 4 * q);
    }
  };
  auto mm = [&](const float4 (&ra)[4], const float4 (&rx)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (db) bs[i] += sum_bf8(ra[i]);
      const bf16x8 av = as_bf8(ra[i]);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(av, as_bf8(rx[j]), acc[i][j]);
    }
  };
  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (nsteps > 1) issue(1, 1);
  float4 ra0[4], rx0[4], ra1[4], rx1[4];
  rd(lds[0], 0, ra0, rx0);
#pragma unroll 1
  for (int t = 0; t < nsteps; ++t) {
    const float* L = lds[t & 1];
    rd(L, 1, ra1, rx1);
    mm(ra0, rx0);
    rd(L, 2, ra0, rx0);
    mm(ra1, rx1);
    rd(L, 3, ra1, rx1);
    mm(ra0, rx0);
    if (t + 1 < nsteps) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // my DMA for t + 1 landed, my reads of t done
      __syncthreads();  // every wave's DMA landed and every wave is done reading buffer t & 1
      if (t + 2 < nsteps) issue(t + 2, t & 1);
      rd(lds[(t + 1) & 1], 0, ra0, rx0);
    }
    mm(ra1, rx1);
  }
}

// Partial (or final) result of an item's (nb0, kb0) quadrant; rows >= nrow2 go to the second output
// (dW2 / db2).
__device__ __forceinline__ void dw_store(const DwJob& J, int split, int part, int nb0, int kb0, int ni, int nj,
                                         bool db, const f32x16 (&acc)[4][4], const float (&bs)[4]) {
  // recomputed here, not carried over the tile loop: the prologue's per-row indices, kept live across the
  // MFMA loop for these stores, were what spilled to scratch
  int tid = threadIdx.x;
  asm volatile("" : "+v"(nb0), "+v"(kb0), "+v"(ni), "+v"(nj), "+v"(split), "+v"(part), "+v"(tid));
  const int lane = tid & 63, h = lane >> 5, c = lane & 31;
  const int N = J.N, K = J.K0 + J.K1;
  const bool direct = J.nsplit * J.wsplit == 1;
  float* slab = direct ? nullptr : J.slab + (int64_t)(split * J.wsplit + part) * J.slab_stride;
  // row n's destination: one 64-bit row pointer live at a time (rows outer, the row's column blocks inner:
  // precomputing every (row, column) address is what spilled this kernel's VGPRs)
  auto row_w = [&](int n) -> float* {
    if (!direct) return slab + (int64_t)n * K;
    return n < J.nrow2 ? J.dW + (int64_t)n * K : J.dW2 + (int64_t)(n - J.nrow2) * K;
  };
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i >= ni) break;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int n = 32 * (nb0 + i) + unit_of(q, h);
      if (n >= N) continue;
      float* rowp = row_w(n);
      asm volatile("" : "+v"(rowp));  // keep the row pointer from being hoisted across the unrolled rows
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j >= nj) break;
        const int k = 32 * (kb0 + j) + c;
        if (k < K) rowp[k] = acc[i][j][q];
      }
    }
    if (db) {
      const float tot = bs[i] + __shfl_xor(bs[i], 32, 64);
      const int n = 32 * (nb0 + i) + c;
      if (h == 0 && n < N) {
        if (!direct) slab[(int64_t)N * K + n] = tot;
        else if (n < J.nrow2) J.db[n] = tot;
        else J.db2[n - J.nrow2] = tot;
      }
    }
  }
}

// BFK: the bf16 job sets (every job of a launch has the agent's bf16 flag); one kernel per
// precision so each gets its own register allocation.
template <bool BFK>
__global__ __launch_bounds__(kDwThreads, 1) void k_dw(const DwJob* __restrict__ jobs, const int* __restrict__ item_job,
                                                      const int* __restrict__ item_split) {
  const int item = blockIdx.x;
  const DwJob J = jobs[item_job[item]];
  const int split = item_split[item];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, c = lane & 31;
  const int64_t ld = J.Bp;
  // Waves whose output quadrant would be empty take part of the samples instead:
  //   wsplit 4 (N, K <= 128): all 4 waves on quadrant (0, 0), a quarter of the samples each;
  //   wsplit 2 (one side <= 128): 2 quadrants along the wide side, 2 sample halves each.
  const int N = J.N, K = J.K0 + J.K1;
  const bool wsp = J.wsplit > 1;
  int nb0 = 4 * (w >> 1), kb0 = 4 * (w & 1), part = 0;
  if (J.wsplit == 4) {
    nb0 = kb0 = 0;
    part = w;
  } else if (J.wsplit == 2) {
    if (N <= 128) {
      nb0 = 0;
      part = w >> 1;
    } else {
      kb0 = 0;
      part = w & 1;
    }
  }
  int b_begin = split * J.split_len;
  int b_end = min(b_begin + J.split_len, J.Bp);
  if (wsp) {  // parts of whole 32-sample units
    const int q = (((b_end - b_begin + J.wsplit - 1) / J.wsplit) + 31) & ~31;
    b_begin = min(b_begin + part * q, b_end);
    b_end = min(b_begin + q, b_end);
  }
  const int nsteps = (b_end - b_begin) / 16;  // ranges are multiples of 32 samples
  const int ni = min(4, max(0, (N + 31) / 32 - nb0));
  const int nj = min(4, max(0, (K + 31) / 32 - kb0));
  if (ni == 0 || nj == 0) return;
  const bool db = J.db != nullptr && kb0 == 0;
  // per-lane row pointers at this item's first sample; rows past N / K are
  // clamped to row 0 (their outputs are never stored)
  const float* ap[4];
  const float* xp[4];
  const int esa = J.a_bf ? 2 : 4, esx = J.x_bf ? 2 : 4;  // operand element sizes
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int n = 32 * (nb0 + i) + c;
    n = n < N ? n : 0;
    ap[i] = reinterpret_cast<const float*>(reinterpret_cast<const char*>(J.A) +
                                           esa * ((int64_t)n * ld + b_begin + 8 * h));
    int k = 32 * (kb0 + i) + c;
    k = k < K ? k : 0;
    const float* xr = k < J.K0 ? J.X0 : J.X1;
    const int64_t kr = k < J.K0 ? k : k - J.K0;
    xp[i] = reinterpret_cast<const float*>(reinterpret_cast<const char*>(xr) + esx * (kr * ld + b_begin + 8 * h));
  }
  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = zero16();
  float bs[4] = {0.f, 0.f, 0.f, 0.f};
  // operand types: 0 fp32 MFMA; bf16 MFMA with (A, X) element types fp32/fp32, bf16/fp32,
  // bf16/bf16, fp32/bf16.  The bf16 forms instantiate 1, 2 and 4 blocks per side only (a 3-block
  // side runs as 4 with its last row block clamped to row 0 and never stored): 4 x 9 shapes.
  const int mode = BFK ? 1 + J.a_bf + 2 * J.x_bf : 0;
#define SPP_DW_T(I, J_, ...)                                                    \
  if (db) dw_tile<I, J_, true, ##__VA_ARGS__>(ap, xp, nsteps, acc, bs);         \
  else dw_tile<I, J_, false, ##__VA_ARGS__>(ap, xp, nsteps, acc, bs);
#define SPP_DW_CASE(I, J_)                                                      \
  case (I) * 8 + (J_): SPP_DW_T(I, J_) break;
#define SPP_DW_CASE16(I, J_)                                                    \
  case (I) * 8 + (J_):                                                          \
    switch (mode) {                                                             \
      case 1: SPP_DW_T(I, J_, true) break;                                      \
      case 2: SPP_DW_T(I, J_, true, true) break;                                \
      case 4: SPP_DW_T(I, J_, true, true, true) break;                          \
      default: SPP_DW_T(I, J_, true, false, true) break;                        \
    }                                                                           \
    break;
  if constexpr (!BFK) {
    switch (ni * 8 + nj) {
      SPP_DW_CASE(1, 1) SPP_DW_CASE(1, 2) SPP_DW_CASE(1, 3) SPP_DW_CASE(1, 4)
      SPP_DW_CASE(2, 1) SPP_DW_CASE(2, 2) SPP_DW_CASE(2, 3) SPP_DW_CASE(2, 4)
      SPP_DW_CASE(3, 1) SPP_DW_CASE(3, 2) SPP_DW_CASE(3, 3) SPP_DW_CASE(3, 4)
      SPP_DW_CASE(4, 1) SPP_DW_CASE(4, 2) SPP_DW_CASE(4, 3) SPP_DW_CASE(4, 4)
    }
  } else {
    const int ni4 = ni == 3 ? 4 : ni, nj4 = nj == 3 ? 4 : nj;
    switch (ni4 * 8 + nj4) {
      SPP_DW_CASE16(1, 1) SPP_DW_CASE16(1, 2) SPP_DW_CASE16(1, 4)
      SPP_DW_CASE16(2, 1) SPP_DW_CASE16(2, 2) SPP_DW_CASE16(2, 4)
      SPP_DW_CASE16(4, 1) SPP_DW_CASE16(4, 2) SPP_DW_CASE16(4, 4)
    }
  }
#undef SPP_DW_CASE
#undef SPP_DW_CASE16
#undef SPP_DW_T
  dw_store(J, split, part, nb0, kb0, ni, nj, db, acc, bs);
}

// 256 x 256 fp32 items (host: DwJob N = K0 = 256, K1 = 0, wsplit = 1, not bf16), listed first in a
// phase's item table: their own kernel, so the LDS-DMA path gets the kernel's whole register budget
// (double-buffered operands) and k_dw's thin / mid items carry no 128 KiB static LDS.
__global__ __launch_bounds__(kDwThreads, 1) void k_dw_big(const DwJob* __restrict__ jobs,
                                                          const int* __restrict__ item_job,
                                                          const int* __restrict__ item_split) {
  const int item = blockIdx.x;
  const DwJob J = jobs[item_job[item]];
  const int split = item_split[item];
  const int w = threadIdx.x >> 6;
  const int nb0 = 4 * (w >> 1), kb0 = 4 * (w & 1);
  const int b_begin = split * J.split_len;
  const int b_end = min(b_begin + J.split_len, J.Bp);
  const int nsteps = (b_end - b_begin) / 32;  // ranges are multiples of 32 samples
  const bool db = J.db != nullptr && kb0 == 0;
  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = zero16();
  float bs[4] = {0.f, 0.f, 0.f, 0.f};
  if (nsteps > 0) dw_big_lds(J, b_begin, nsteps, nb0, kb0, db, acc, bs);
  dw_store(J, split, 0, nb0, kb0, 4, 4, db, acc, bs);
}

// 256 x 256 bf16-operand items (host: as k_dw_big's, both operands bf16, item ranges multiples of 64 samples).
__global__ __launch_bounds__(kDwThreads, 1) void k_dw_big16(const DwJob* __restrict__ jobs,
                                                            const int* __restrict__ item_job,
                                                            const int* __restrict__ item_split) {
  const int item = blockIdx.x;
  const DwJob J = jobs[item_job[item]];
  const int split = item_split[item];
  const int w = threadIdx.x >> 6;
  const int nb0 = 4 * (w >> 1), kb0 = 4 * (w & 1);
  const int b_begin = split * J.split_len;
  const int b_end = min(b_begin + J.split_len, J.Bp);
  const int nsteps = (b_end - b_begin) / 64;  // ranges are multiples of 64 samples (host: lds_big)
  const bool db = J.db != nullptr && kb0 == 0;
  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = zero16();
  float bs[4] = {0.f, 0.f, 0.f, 0.f};
  if (nsteps > 0) dw_big_lds16(J, b_begin, nsteps, nb0, kb0, db, acc, bs);
  dw_store(J, split, 0, nb0, kb0, 4, 4, db, acc, bs);
}

// Fixed-order reduction of the split slabs: one thread per element of a job's [N*K | N] image,
// slabs summed in split order.  A job has few elements (<= 64K) against 128-256 slabs, so the
// walk is latency-bound: one element per thread (4x the threads of a float4 walk) and 16
// slabs' loads in flight.
__global__ void k_dw_reduce(const DwJob* __restrict__ jobs) {
  const DwJob J = jobs[blockIdx.y];
  const int nslab = J.nsplit * J.wsplit;
  if (nslab == 1) return;
  const int N = J.N, K = J.K0 + J.K1;
  const int64_t nw = (int64_t)N * K;
  const int64_t total = nw + (J.db ? N : 0);
  const int G = dw_red_group(nslab, nw + N);  // lanes per element (as the host sized the grid; a power of 2 dividing 64)
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t e = gid / G;
  const int g = (int)(gid % G);
  if (e >= total) return;  // whole groups: e is the same for the G lanes of a group
  const float* p = J.slab + e;
  float s = 0.f;
  if (G == 1) {
    int sp = 0;
    for (; sp + 16 <= nslab; sp += 16) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = p[(int64_t)(sp + u) * J.slab_stride];
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
    for (; sp < nslab; ++sp) s += p[(int64_t)sp * J.slab_stride];
  } else {
    // lane g sums slabs g, g + G, ... (16 loads per round trip), then a fixed butterfly over the group; lane 0's
    // operand order is the same on every run, and only lane 0 writes
    for (int sp = g; sp < nslab; sp += 16 * G) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = sp + u * G < nslab ? p[(int64_t)(sp + u * G) * J.slab_stride] : 0.f;
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
    for (int o = G / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (g != 0) return;
  }
  if (e < nw) {
    const int n = (int)(e / K), k = (int)(e % K);
    if (n < J.nrow2) J.dW[(int64_t)n * K + k] = s;
    else J.dW2[(int64_t)(n - J.nrow2) * K + k] = s;
  } else {
    const int n = (int)(e - nw);
    if (n < J.nrow2) J.db[n] = s;
    else J.db2[n - J.nrow2] = s;
  }
}

}  // namespace spp
