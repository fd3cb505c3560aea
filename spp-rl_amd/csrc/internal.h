// Internal job descriptors shared between kernels and the host API.
#pragma once
#include "common.h"
#include "mlp.h"

namespace spp {

// weight-gradient GEMM job (dw.hip)
struct DwJob {
  const float* A;   // delta [N][Bp]
  const float* X0;  // input segment 0 [K0][Bp]
  const float* X1;  // input segment 1 [K1][Bp] (may be null)
  float* dW;        // rows [0, nrow2) of [N][K0+K1], canonical
  float* db;        // [nrow2] or null
  float* dW2;       // rows [nrow2, N) (second output, e.g. the log-std head), or null
  float* db2;
  float* slab;      // split partials [nsplit * wsplit][slab_stride]
  int64_t slab_stride;
  int N, K0, K1, Bp;
  int split_len, nsplit, nrow2;
  int wsplit;       // 4: output <= 128x128, the 4 waves of an item split its samples (one slab each); else 1
  int bf16;         // 1: bf16 MFMA (operands rounded to bf16 in registers, fp32 accumulation)
  int a_bf, x_bf;   // (bf16 only) A / X rows hold bf16 elements ([rows][Bp] __bf16), else fp32
  int fused;        // 1: no work items -- a phase kernel writes the nsplit slabs (per wave); only reduced
};

// dw.hip (own translation unit, ks_dw.hip): the split-K weight-gradient launch + fixed-order reduce
// over nitems work items of jobs[0, njobs); item_job / item_split index the job table; the first
// nlds items are 256 x 256 jobs staged through LDS (k_dw_big; bf16 sets: k_dw_big16, bf16 A and X rows), the
// rest run in k_dw; bf16: the set's jobs are bf16 MFMA jobs (DwJob::bf16).
void launch_dw_kernels(const DwJob* jobs, const int* item_job, const int* item_split, int nitems, int nlds,
                       int njobs, int64_t max_elems, bool bf16, hipStream_t st);
// k_dw_reduce: lanes that sum one output element of a job with nslab partial slabs of `elems` elements
// (fixed-order reduce).  One lane per element (consecutive lanes read consecutive elements of a slab:
// coalesced) for the split-K GEMM jobs; a group of 16 lanes per element for the few-element, many-slab jobs
// (the fused fc3 jobs' 257 x one-partial-per-wave), whose one-lane serial sums were the launch's critical
// path; max_elems counts lanes
inline __host__ __device__ int dw_red_group(int nslab, int64_t elems) { return nslab >= 64 && elems <= 4096 ? 16 : 1; }

// fragment-image pack job: logical L[n][k] of a source matrix S (row stride ld)
//   L[n][k] = trans ? S[k][coff + n] : S[n][coff + k]; source rows >= split come from W2
// image order: ob-major ((ob*NBI + ib)*4 + rq)*64 + lane (dense), or
//              ib-major ((ib*NBO + ob)*4 + rq)*64 + lane (dense_lds)
struct PackJob {
  const float* W;
  const float* W2;
  int split, ld, trans, coff;
  MapDesc out, in;
  int NBO, NBI, ibmajor;
  float4* dst;
  int bf16;  // 1: bf16 image for v_mfma_f32_32x32x16_bf16 (2 fragments of 8 bf16 per block pair, mlp.h)
};

struct AdamJob {
  float* p;
  const float* g;
  float* m;
  float* v;
  float* targ;  // polyak target or null
  int64_t n;
};

}  // namespace spp
