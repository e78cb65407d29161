// Probe (MI355X): write bandwidth of a GEMM output stream by store pattern.  C = M x N fp32, written
// once per launch by 128 x 512 tiles (8 waves of 64 x 128, the FP6 GEMM's epilogue map):
//   A  "patch":  each instruction 8 rows x 128 B (8 lanes per row segment), as the GEMM epilogue now
//   B  "rows":   each instruction 1 KB of one row (64 lanes x 16 B), a wave owning 16 whole tile rows
//   C  "linear": the matrix as one flat array, thread-contiguous float4 (the plain-fill reference)
// each with plain and non-temporal stores, every workgroup's tile written at once (as in the GEMM,
// where all CUs reach the epilogue in the same round) -- GB/s over the best of 10 launches.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/probe_store tools/probes/probe_store_pattern.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef float v4f __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void st(float* p, v4f v) {
  if (NT) __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(p));
  else *reinterpret_cast<v4f*>(p) = v;
}

template <bool NT>
__global__ __launch_bounds__(512) void k_patch(float* C, int M, int N, int gn) {
  const int tm = blockIdx.x / gn, tn = blockIdx.x % gn;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, wm = wave / 4, wn = wave % 4;
  const v4f v = {1.f, 2.f, 3.f, (float)lane};
  for (int u = 0; u < 4; ++u)
    for (int t = 0; t < 2; ++t)
      for (int ps = 0; ps < 4; ++ps) {
        const int row = tm * 128 + wm * 64 + t * 32 + (lane >> 3) + 8 * ps;
        const int col = tn * 512 + wn * 128 + u * 32 + 4 * (lane & 7);
        st<NT>(C + (int64_t)row * N + col, v);
      }
}

template <bool NT>
__global__ __launch_bounds__(512) void k_rows(float* C, int M, int N, int gn) {
  const int tm = blockIdx.x / gn, tn = blockIdx.x % gn;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const v4f v = {1.f, 2.f, 3.f, (float)lane};
  for (int r = 0; r < 16; ++r)
    for (int half = 0; half < 2; ++half) {
      const int row = tm * 128 + wave * 16 + r;
      const int col = tn * 512 + half * 256 + 4 * lane;
      st<NT>(C + (int64_t)row * N + col, v);
    }
}

template <bool NT>
__global__ __launch_bounds__(512) void k_linear(float* C, int64_t n4) {
  const v4f v = {1.f, 2.f, 3.f, 4.f};
  for (int64_t i = (int64_t)blockIdx.x * 512 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 512)
    st<NT>(C + 4 * i, v);
}

template <typename F>
static float best_ms(F launch) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e30f;
  for (int it = 0; it < 12; ++it) {
    hipEventRecord(a);
    launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    if (it >= 2 && ms < best) best = ms;
  }
  return best;
}

int main() {
  const int shapes[2][2] = {{65536, 8192}, {8192, 8192}};
  float* C = nullptr;
  if (hipMalloc(&C, (size_t)65536 * 8192 * 4) != hipSuccess) return 1;
  for (auto& s : shapes) {
    const int M = s[0], N = s[1], gm = M / 128, gn = N / 512;
    const double gb = (double)M * N * 4 / 1e9;
    const float p0 = best_ms([&] { hipLaunchKernelGGL(k_patch<false>, dim3(gm * gn), dim3(512), 0, 0, C, M, N, gn); });
    const float p1 = best_ms([&] { hipLaunchKernelGGL(k_patch<true>, dim3(gm * gn), dim3(512), 0, 0, C, M, N, gn); });
    const float r0 = best_ms([&] { hipLaunchKernelGGL(k_rows<false>, dim3(gm * gn), dim3(512), 0, 0, C, M, N, gn); });
    const float r1 = best_ms([&] { hipLaunchKernelGGL(k_rows<true>, dim3(gm * gn), dim3(512), 0, 0, C, M, N, gn); });
    const int64_t n4 = (int64_t)M * N / 4;
    const float l0 = best_ms([&] { hipLaunchKernelGGL(k_linear<false>, dim3(4096), dim3(512), 0, 0, C, n4); });
    const float l1 = best_ms([&] { hipLaunchKernelGGL(k_linear<true>, dim3(4096), dim3(512), 0, 0, C, n4); });
    printf("C %d x %d fp32 (%.2f GB): patch %.3f ms %.0f GB/s | nt %.3f ms %.0f GB/s ; rows %.3f ms %.0f GB/s | nt %.3f "
           "ms %.0f GB/s ; linear %.3f ms %.0f GB/s | nt %.3f ms %.0f GB/s\n",
           M, N, gb, p0, gb / p0 * 1e3, p1, gb / p1 * 1e3, r0, gb / r0 * 1e3, r1, gb / r1 * 1e3, l0, gb / l0 * 1e3, l1,
           gb / l1 * 1e3);
  }
  hipFree(C);
  return 0;
}
