// Semantics of v_cvt_scalef32_2xpk16_fp6_f32 on gfx950 (the FP6 pack conversion): which scale
// convention (x / scale or x * scale), the output bit layout (element i at bits 6i of 6 dwords?),
// and exactness for the digit values d/8, d in [-16, 16].  Prints one line per test.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v16f __attribute__((ext_vector_type(16)));
typedef int v6i __attribute__((ext_vector_type(6)));
typedef _Float16 v32h __attribute__((ext_vector_type(32)));

__global__ void cvt16_k(const float* x, unsigned* out, float scale) {
  v32h a;
  for (int i = 0; i < 32; ++i) a[i] = (_Float16)x[i];
  v6i r = __builtin_amdgcn_cvt_scalef32_pk32_fp6_f16(a, scale);
  if (threadIdx.x == 0)
    for (int i = 0; i < 6; ++i) out[i] = (unsigned)r[i];
}

__global__ void cvt_k(const float* x, unsigned* out, float scale) {
  v16f a, b;
  for (int i = 0; i < 16; ++i) { a[i] = x[i]; b[i] = x[16 + i]; }
  v6i r = __builtin_amdgcn_cvt_scalef32_2xpk16_fp6_f32(a, b, scale);
  if (threadIdx.x == 0)
    for (int i = 0; i < 6; ++i) out[i] = (unsigned)r[i];
}

static unsigned code_of(int d) { return d < 0 ? (0x20u | (unsigned)(-d)) : (unsigned)d; }

int main() {
  float hx[32];
  float* dx;
  unsigned* dout;
  unsigned ho[6];
  (void)hipMalloc(&dx, sizeof(hx));
  (void)hipMalloc(&dout, sizeof(ho));
  const float scales[3] = {1.0f, 8.0f, 0.125f};
  for (int mode = 0; mode < 3; ++mode) {   // 0: x = d/8, 1: x = d (f32 2xpk16); 2: x = d (f16 pk32)
    for (int si = 0; si < 3; ++si) {
      for (int i = 0; i < 32; ++i) {
        const int d = (i % 33) - 16;
        hx[i] = mode == 0 ? d / 8.0f : (float)d;   // modes 1, 2: integers
      }
      (void)hipMemcpy(dx, hx, sizeof(hx), hipMemcpyHostToDevice);
      if (mode < 2) hipLaunchKernelGGL(cvt_k, dim3(1), dim3(64), 0, 0, dx, dout, scales[si]);
      else hipLaunchKernelGGL(cvt16_k, dim3(1), dim3(64), 0, 0, dx, dout, scales[si]);
      (void)hipMemcpy(ho, dout, sizeof(ho), hipMemcpyDeviceToHost);
      int match = 0;
      for (int i = 0; i < 32; ++i) {
        const int bit = 6 * i;
        unsigned long long w = ho[bit / 32];
        if (bit / 32 + 1 < 6) w |= (unsigned long long)ho[bit / 32 + 1] << 32;
        const unsigned c = (unsigned)((w >> (bit % 32)) & 63u);
        match += c == code_of((i % 33) - 16);
      }
      printf("x=%s scale=%g: %d/32 codes match e2m3(d/8) at bits 6i; dwords %08x %08x %08x %08x %08x %08x\n",
             mode == 0 ? "d/8" : (mode == 1 ? "d" : "d f16 pk32"), scales[si], match, ho[0], ho[1], ho[2], ho[3], ho[4], ho[5]);
    }
  }
  return 0;
}
