// Where do the first two rounds of a 2-workgroups-per-CU grid land?  256-thread workgroups holding
// 62 KB of LDS each (as the 64 x 512 FP6 GEMM tile, gemm_fp6_k<1, 4, 2, 4, 2, ..., RES = 1>): each
// records blockIdx, HW_ID (CU / SH / SE / TG slot), XCC_ID and its start time (s_memrealtime,
// 100 MHz), then spins ~40 us.  Prints, per CU, the blocks it ran in launch order, and whether the
// second resident of every CU in the first round is a block of [256, 512) -- the rule the FP6
// GEMM's first-round stagger relies on.
//   hipcc --offload-arch=gfx950 -O2 tools/probes/probe_wg_placement.hip -o /tmp/probe_wg && /tmp/probe_wg
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <tuple>
#include <vector>

__global__ __launch_bounds__(256, 2) void place_k(unsigned* o, long spin) {
  extern __shared__ char lds[];
  unsigned hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const unsigned long t0 = __builtin_amdgcn_s_memrealtime();
  lds[threadIdx.x] = (char)threadIdx.x;
  while ((long)(__builtin_amdgcn_s_memrealtime() - t0) < spin) __builtin_amdgcn_s_sleep(8);
  __syncthreads();
  if (threadIdx.x == 0) {
    o[blockIdx.x * 4 + 0] = hw;
    o[blockIdx.x * 4 + 1] = xcc;
    o[blockIdx.x * 4 + 2] = (unsigned)t0;
    o[blockIdx.x * 4 + 3] = (unsigned)lds[5];
  }
}

int main() {
  const int G = 2048;
  unsigned* d = nullptr;
  if (hipMalloc(&d, G * 16) != hipSuccess) return 1;
  hipLaunchKernelGGL(place_k, dim3(G), dim3(256), 62 * 1024, 0, d, 4000L);   // warm-up
  hipLaunchKernelGGL(place_k, dim3(G), dim3(256), 62 * 1024, 0, d, 4000L);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::vector<unsigned> h(G * 4);
  hipMemcpy(h.data(), d, G * 16, hipMemcpyDeviceToHost);
  unsigned tmin = 0xffffffffu;
  for (int b = 0; b < G; ++b) tmin = std::min(tmin, h[b * 4 + 2]);
  // CU key: (xcc, se, sh, cu)
  std::map<std::tuple<int, int, int, int>, std::vector<int>> cu;
  for (int b = 0; b < G; ++b) {
    const unsigned hw = h[b * 4];
    const int cuid = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7, xcc = (int)h[b * 4 + 1] & 15;
    cu[{xcc, se, sh, cuid}].push_back(b);
  }
  printf("distinct CUs used: %zu\n", cu.size());
  int ok = 0, bad = 0, shown = 0;
  for (auto& kv : cu) {
    auto& v = kv.second;   // blocks in index order; the first two started in round 1
    std::vector<std::pair<unsigned, int>> byt;
    for (int b : v) byt.push_back({h[b * 4 + 2] - tmin, b});
    std::sort(byt.begin(), byt.end());
    if (byt.size() >= 2) {
      const int a = byt[0].second, b = byt[1].second;
      const bool rule = (a < 256) != (b < 256) && a < 512 && b < 512;
      rule ? ++ok : ++bad;
    }
    if (shown < 12) {
      ++shown;
      printf("xcc %d se %d sh %d cu %2d:", std::get<0>(kv.first), std::get<1>(kv.first), std::get<2>(kv.first),
             std::get<3>(kv.first));
      for (size_t i = 0; i < byt.size() && i < 10; ++i)
        printf(" b%d(t%u tg%u)", byt[i].second, byt[i].first / 100, (h[byt[i].second * 4] >> 16) & 15);
      printf("\n");
    }
  }
  printf("CUs whose first two residents are one block of [0, 256) and one of [256, 512): %d of %d\n", ok, ok + bad);
  return 0;
}
