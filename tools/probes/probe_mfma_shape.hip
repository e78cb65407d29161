// Probe (MI355X): FP6(e2m3) x FP4 block-scaled MFMA throughput by shape on RANDOM operands
// (32x32x64 vs 16x16x128), every CU busy, one or two waves per SIMD, after ~2 s of back-to-back
// launches so the clock has settled under load (MI355X_MICROARCH.md, 'DVFS give-back').  Each
// wave alternates two random operand sets so the multiplier inputs toggle every MFMA.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void k32(const int* __restrict__ rnd, float* out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  v8i a0, a1, b0, b1;
  for (int i = 0; i < 8; ++i) {
    a0[i] = i < 6 ? rnd[(t * 32 + i) & 0xFFFFF] & 0x37373737 : 0;   // e2m3 codes, |d| <= 15
    a1[i] = i < 6 ? rnd[(t * 32 + 8 + i) & 0xFFFFF] & 0x37373737 : 0;
    b0[i] = i < 4 ? rnd[(t * 32 + 16 + i) & 0xFFFFF] & 0xABABABAB : 0;   // fp4 codes 0, 2, 8, 10
    b1[i] = i < 4 ? rnd[(t * 32 + 24 + i) & 0xFFFFF] & 0xABABABAB : 0;
  }
  v16f acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = v16f{0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i)
      acc[i] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4((i & 1) ? a1 : a0, (i & 2) ? b1 : b0, acc[i], 2, 4,
                                                               0, 100, 0, 127);
  }
  float s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][threadIdx.x & 15];
  out[t] = s;
}

template <int NACC>
__global__ __launch_bounds__(256) void k16(const int* __restrict__ rnd, float* out, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  v8i a0, a1, b0, b1;
  for (int i = 0; i < 8; ++i) {
    a0[i] = i < 6 ? rnd[(t * 32 + i) & 0xFFFFF] & 0x37373737 : 0;
    a1[i] = i < 6 ? rnd[(t * 32 + 8 + i) & 0xFFFFF] & 0x37373737 : 0;
    b0[i] = i < 4 ? rnd[(t * 32 + 16 + i) & 0xFFFFF] & 0xABABABAB : 0;
    b1[i] = i < 4 ? rnd[(t * 32 + 24 + i) & 0xFFFFF] & 0xABABABAB : 0;
  }
  v4f acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = v4f{0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i)
      acc[i] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4((i & 1) ? a1 : a0, (i & 2) ? b1 : b0, acc[i], 2, 4,
                                                                0, 100, 0, 127);
  }
  float s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][threadIdx.x & 3];
  out[t] = s;
}

template <typename F>
double run(F launch, double macs_per_launch, const char* name) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  // settle: ~2 s of back-to-back launches
  hipEventRecord(a);
  launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms1;
  hipEventElapsedTime(&ms1, a, b);
  const int n = (int)(2000.0 / (ms1 > 0.01 ? ms1 : 0.01)) + 1;
  for (int i = 0; i < n; ++i) launch();
  hipEventRecord(a);
  for (int i = 0; i < 10; ++i) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  ms /= 10;
  const double tops = 2 * macs_per_launch / (ms * 1e-3) / 1e12;
  printf("%-34s %8.3f ms  %7.3f POPS  (%.1f%% of 10.07)\n", name, ms, tops / 1e3, tops / 100.66);
  return tops;
}

int main() {
  const int nr = 1 << 20;
  std::vector<int> h(nr);
  uint32_t s = 12345;
  for (int i = 0; i < nr; ++i) {
    s ^= s << 13; s ^= s >> 17; s ^= s << 5;
    h[i] = (int)s;
  }
  int* rnd;
  float* out;
  hipMalloc(&rnd, nr * 4);
  hipMalloc(&out, 256 * 2048 * 4);
  hipMemcpy(rnd, h.data(), nr * 4, hipMemcpyHostToDevice);
  const int iters = 4000;
  for (int wps = 1; wps <= 2; ++wps) {
    const int blocks = 256 * wps;   // 4 waves per block: wps waves per SIMD
    char nm[64];
    snprintf(nm, sizeof nm, "32x32x64  8 acc, %d wave/SIMD", wps);
    run([&] { hipLaunchKernelGGL(k32<8>, dim3(blocks), dim3(256), 0, 0, rnd, out, iters); },
        (double)blocks * 4 * iters * 8 * 32 * 32 * 64, nm);
    snprintf(nm, sizeof nm, "16x16x128 16 acc, %d wave/SIMD", wps);
    run([&] { hipLaunchKernelGGL(k16<16>, dim3(blocks), dim3(256), 0, 0, rnd, out, iters); },
        (double)blocks * 4 * iters * 16 * 16 * 16 * 128, nm);
  }
  hipFree(rnd);
  hipFree(out);
  return 0;
}
