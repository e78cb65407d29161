// Probe (run once on MI355X): operand layout of v_mfma_scale_f32_32x32x64_f8f6f4 with an FP6 e2m3
// A operand (cbsz = 2) and an FP4 e2m1 B operand (blgp = 4), and the per-lane E8M0 scales.
// Hypotheses: lane l holds A[row l%32][k = 32*(l/32) + j], j = 0..31, element j at bits 6j..6j+5
// of the 6-dword operand; scale byte of lane l scales that lane's 32 elements (block l/32 of row
// l%32) -- B likewise with columns.  Prints mismatch counts against an exact host product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cmath>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ void k(const uint32_t* a6, const uint32_t* b4, const int* sa, const int* sb, float* d) {
  const int l = threadIdx.x;
  v8i A = {0, 0, 0, 0, 0, 0, 0, 0}, B = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 6; ++i) A[i] = a6[l * 6 + i];
  for (int i = 0; i < 4; ++i) B[i] = b4[l * 4 + i];
  v16f acc = {0};
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, acc, 2, 4, 0, sa[l], 0, sb[l]);
  for (int i = 0; i < 16; ++i) d[l * 16 + i] = acc[i];
}

static uint32_t e2m3(int d) {   // integer digit d in [-16,16] as e2m3 code of d/8
  uint32_t s = d < 0 ? 0x20 : 0, m = (uint32_t)std::abs(d);
  if (m < 8) return s | m;                    // subnormal: m/8
  if (m < 16) return s | (1u << 3) | (m - 8); // 1.f * 2^0
  return s | (2u << 3);                       // 16/8 = 2.0
}
static uint32_t e2m1(int t) { return t > 0 ? 0x2 : (t < 0 ? 0xA : 0); }

int main() {
  int A[32][64], B[32][64], ea[32][2], eb[32][2];
  srand(7);
  for (int r = 0; r < 32; ++r)
    for (int k = 0; k < 64; ++k) { A[r][k] = rand() % 33 - 16; B[r][k] = rand() % 3 - 1; }
  for (int r = 0; r < 32; ++r)
    for (int b = 0; b < 2; ++b) { ea[r][b] = rand() % 9 - 4; eb[r][b] = rand() % 5 - 2; }
  uint32_t ha[64 * 6] = {0}, hb[64 * 4] = {0};
  int hsa[64], hsb[64];
  for (int l = 0; l < 64; ++l) {
    const int r = l % 32, blk = l / 32;
    for (int j = 0; j < 32; ++j) {
      const uint64_t code = e2m3(A[r][32 * blk + j]);
      const int bit = 6 * j;
      ha[l * 6 + bit / 32] |= (uint32_t)(code << (bit % 32));
      if (bit % 32 > 26) ha[l * 6 + bit / 32 + 1] |= (uint32_t)(code >> (32 - bit % 32));
      hb[l * 4 + j / 8] |= e2m1(B[r][32 * blk + j]) << (4 * (j % 8));
    }
    hsa[l] = 127 + 3 + ea[r][blk];   // digit/8 * 2^(3+e) = digit * 2^e
    hsb[l] = 127 + eb[r][blk];
  }
  uint32_t *da, *db; int *dsa, *dsb; float* dd;
  hipMalloc(&da, sizeof ha); hipMalloc(&db, sizeof hb); hipMalloc(&dsa, sizeof hsa); hipMalloc(&dsb, sizeof hsb);
  hipMalloc(&dd, 64 * 16 * 4);
  hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice); hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
  hipMemcpy(dsa, hsa, sizeof hsa, hipMemcpyHostToDevice); hipMemcpy(dsb, hsb, sizeof hsb, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
  float hd[64 * 16];
  hipMemcpy(hd, dd, sizeof hd, hipMemcpyDeviceToHost);
  int bad = 0, checked = 0;
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 16; ++i) {
      const int row = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5), col = l & 31;
      double ref = 0;
      for (int k = 0; k < 64; ++k)
        ref += (double)A[row][k] * std::ldexp(1.0, ea[row][k / 32]) * B[col][k] * std::ldexp(1.0, eb[col][k / 32]);
      ++checked;
      if (hd[l * 16 + i] != (float)ref) { if (bad < 5) printf("row %d col %d got %g want %g\n", row, col, hd[l * 16 + i], ref); ++bad; }
    }
  printf("fp6 x fp4 scaled MFMA: %d of %d outputs wrong\n", bad, checked);
  return bad != 0;
}
