// Semantics of v_cvt_scalef32_pk_fp4_f32 on gfx950 (f32 pair -> two e2m1 nibbles in byte `index` of
// the old dword): scale convention, rounding of ties, the sign of values that round to zero, and the
// nibble order -- for the residual plane's digits d/2, d in [-4, 4] (bnn_fp6.h).  One line per case.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/probe_cvt_fp4 tools/probes/probe_cvt_fp4.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void cvt_k(const float* x, int n, float scale, unsigned* out) {
  const int i = threadIdx.x;
  if (2 * i + 1 >= n) return;
  unsigned w = 0xFFFFFFFFu;   // old bytes: the other three must stay
  w = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(w, x[2 * i], x[2 * i + 1], scale, 1);
  out[i] = w;
}

int main() {
  const float vals[] = {0.f, 0.5f, 1.f, 1.5f, 2.f, -0.5f, -1.f, -1.5f, -2.f, 0.25f, 0.75f, 1.25f, 1.75f, -0.25f,
                        -0.75f, -1.25f, -1.75f, -0.1f, -0.f, 0.1f, 0.2499f, 0.2501f, -0.2501f, 2.2f, 3.f, 0.f};
  const int n = sizeof(vals) / sizeof(vals[0]);
  float* dx;
  unsigned* dout;
  unsigned ho[64];
  (void)hipMalloc(&dx, sizeof(vals));
  (void)hipMalloc(&dout, sizeof(ho));
  (void)hipMemcpy(dx, vals, sizeof(vals), hipMemcpyHostToDevice);
  const float scales[2] = {1.f, 0.5f};
  for (float sc : scales) {
    hipLaunchKernelGGL(cvt_k, dim3(1), dim3(32), 0, 0, dx, n, sc, dout);
    (void)hipMemcpy(ho, dout, sizeof(unsigned) * (n / 2), hipMemcpyDeviceToHost);
    for (int i = 0; i < n / 2; ++i) {
      const unsigned b = (ho[i] >> 8) & 0xFFu;
      printf("scale %.2f  x = (%8.4f, %8.4f) -> byte 1 = 0x%02x (lo nibble 0x%x, hi 0x%x), other bytes 0x%08x\n", sc,
             vals[2 * i], vals[2 * i + 1], b, b & 15u, b >> 4, ho[i] | 0x0000FF00u);
    }
  }
  return 0;
}
