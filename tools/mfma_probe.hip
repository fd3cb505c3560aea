// Empirical lane maps of v_mfma_f32_32x32x2_f32 (layout probe, not product code).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ void probe(int mode, int L0, float* out) {
  int l = threadIdx.x;
  float a = 0.f, b = 0.f;
  if (mode == 0) { a = (l == L0) ? 1.f : 0.f; b = 1.f; }
  else { a = 1.f; b = (l == L0) ? 1.f : 0.f; }
  f32x16 c;
  for (int i = 0; i < 16; ++i) c[i] = 0.f;
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  for (int i = 0; i < 16; ++i) out[l * 16 + i] = c[i];
}
int main() {
  float* d; hipMalloc(&d, 64 * 16 * 4);
  float h[64 * 16];
  int lanes[] = {0, 1, 5, 31, 32, 33, 63};
  for (int mode = 0; mode < 2; ++mode)
    for (int li = 0; li < 7; ++li) {
      int L0 = lanes[li];
      hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, mode, L0, d);
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      printf("mode %s L0=%d nonzero (lane,reg):", mode ? "B" : "A", L0);
      int cnt = 0;
      for (int l = 0; l < 64; ++l) for (int r = 0; r < 16; ++r) if (h[l * 16 + r] != 0.f) { if (cnt < 12) printf(" (%d,%d)=%g", l, r, h[l*16+r]); cnt++; }
      printf("  [count %d]\n", cnt);
    }
  return 0;
}
