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
  float* dW;        // [N][K0+K1] canonical
  float* db;        // [N] or null
  float* slab;      // split partials
  int64_t slab_stride;
  int N, K0, K1, Bp;
  int split_len, nsplit;
};

// fragment-image pack job: logical L[n][k] of a source matrix S (row stride ld)
//   L[n][k] = trans ? S[k][coff + n] : S[n][coff + k]; source rows >= split come from W2
struct PackJob {
  const float* W;
  const float* W2;
  int split, ld, trans, coff;
  MapDesc out, in;
  int NBO, NBI;
  float4* dst;
};
// vector image: dst[(ob*16 + q)*2 + h] = v[map(ob, q, h)] (idx >= split -> v2[idx - split])
struct VecJob {
  const float* v;
  const float* v2;
  int split;
  MapDesc map;
  int NB;
  float* dst;
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
