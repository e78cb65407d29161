// Probe (MI355X): sustained issue rate of the block-scaled MFMA by operand format, and of the
// int8 MFMA, with 8 independent accumulators per wave, 4 waves per CU, every CU busy.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int FA, int FB>
__global__ __launch_bounds__(256) void kscale(float* out, int iters, int seed) {
  const int tx = (int)threadIdx.x;
  v8i a = {seed, tx, 3, 5, 7, 9, 0, 0}, b = {tx, seed, 1, 2, 3, 4, 0, 0};
  v16f acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = v16f{0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      acc[i] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc[i], FA, FB, 0, 127, 0, 127);
  }
  float s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i][threadIdx.x & 15];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void ki8(float* out, int iters, int seed) {
  v4i a = {seed, (int)threadIdx.x, 3, 5}, b = {(int)threadIdx.x, seed, 1, 2};
  v16i acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = v16i{0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[i], 0, 0, 0);
  }
  int s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i][threadIdx.x & 15];
  out[blockIdx.x * 256 + threadIdx.x] = (float)s;
}

template <typename F>
float timeit(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  f();
  hipEventRecord(a);
  f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  float* out; hipMalloc(&out, 256 * 1024 * 4 * 8);
  const int blocks = 256 * 4, iters = 2000;
  const double macs = (double)blocks * 4 /*waves*/ * iters * 8 * 32 * 32 * 64;
  auto rep = [&](const char* n, float ms, double k) {
    printf("%-22s %8.3f ms  %8.1f TOPS  (%.1f cycles/MFMA/SIMD at 2.4 GHz)\n", n, ms, 2 * macs * k / ms / 1e9,
           ms * 1e-3 * 2.4e9 / (iters * 8.0 * 1 /*wave per SIMD*/ ));
  };
  rep("fp4 x fp4", timeit([&] { hipLaunchKernelGGL((kscale<4, 4>), dim3(blocks), dim3(256), 0, 0, out, iters, 1); }), 1);
  rep("fp6(e2m3) x fp4", timeit([&] { hipLaunchKernelGGL((kscale<2, 4>), dim3(blocks), dim3(256), 0, 0, out, iters, 1); }), 1);
  rep("fp6 x fp6", timeit([&] { hipLaunchKernelGGL((kscale<2, 2>), dim3(blocks), dim3(256), 0, 0, out, iters, 1); }), 1);
  rep("fp8 x fp4", timeit([&] { hipLaunchKernelGGL((kscale<0, 4>), dim3(blocks), dim3(256), 0, 0, out, iters, 1); }), 1);
  rep("fp8 x fp8", timeit([&] { hipLaunchKernelGGL((kscale<0, 0>), dim3(blocks), dim3(256), 0, 0, out, iters, 1); }), 1);
  rep("i8 32x32x32", timeit([&] { hipLaunchKernelGGL(ki8, dim3(blocks), dim3(256), 0, 0, out, iters, 1); }), 0.5);
  return 0;
}
