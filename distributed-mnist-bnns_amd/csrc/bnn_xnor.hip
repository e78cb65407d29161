// Subsystem (2), second implementation: XNOR/AND-popcount binary GEMM on the VALU.
//
// The reference's "binary" values are ternary (sign(0) = 0, models/binarized_modules.py:13), so
// each operand carries two bit-planes: s (1 where x<0) and nz (1 where x!=0).  For 32 k at once:
//     dot = popc(nzA & nzB) - 2*popc(nzA & nzB & (sA ^ sB))
// = 5 VALU ops per 32 MACs (v_and, v_xor, v_and, 2x v_bcnt_u32_b32 with accumulate).
// Same contract as the (1,1) form of bnn_gemm_i8: C = dot + bias, bit-exact.
#include <algorithm>

#include "bnn_common.h"

namespace bnn {
namespace {

constexpr int XT = 64;   // output tile (rows and cols)
constexpr int KWC = 32;  // words per LDS stage (1024 k)

__global__ __launch_bounds__(256) void gemm_xnor_k(const uint32_t* __restrict__ As,
                                                   const uint32_t* __restrict__ Anz, int64_t lda,
                                                   const uint32_t* __restrict__ Bs,
                                                   const uint32_t* __restrict__ Bnz, int64_t ldb,
                                                   const float* __restrict__ bias, float* __restrict__ C,
                                                   int64_t ldc, int M, int N, int kw, int gn) {
  __shared__ uint32_t sAs[XT][KWC + 1], sAn[XT][KWC + 1], sBs[XT][KWC + 1], sBn[XT][KWC + 1];
  const int t = threadIdx.x;
  const int tm = blockIdx.x / gn, tn = blockIdx.x % gn;
  const int m0 = tm * XT, n0 = tn * XT;
  const int ty = t >> 4, tx = t & 15;
  // loader: thread -> row t/4, words (t%4)*8 .. +7
  const int lr = t >> 2, lw = (t & 3) * 8;
  const int64_t arow = min(m0 + lr, M - 1), brow = min(n0 + lr, N - 1);
  int acc_nz[4][4] = {}, acc_x[4][4] = {};
  for (int w0 = 0; w0 < kw; w0 += KWC) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sAs[lr][lw + j] = As[arow * lda + w0 + lw + j];
      sAn[lr][lw + j] = Anz[arow * lda + w0 + lw + j];
      sBs[lr][lw + j] = Bs[brow * ldb + w0 + lw + j];
      sBn[lr][lw + j] = Bnz[brow * ldb + w0 + lw + j];
    }
    __syncthreads();
#pragma unroll 4
    for (int w = 0; w < KWC; ++w) {
      uint32_t as[4], an[4], bs[4], bn[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        as[i] = sAs[ty * 4 + i][w];
        an[i] = sAn[ty * 4 + i][w];
        bs[i] = sBs[tx + 16 * i][w];
        bn[i] = sBn[tx + 16 * i][w];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t mk = an[i] & bn[j];
          acc_nz[i][j] += __builtin_popcount(mk);
          acc_x[i][j] += __builtin_popcount((as[i] ^ bs[j]) & mk);
        }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = m0 + ty * 4 + i;
    if (row >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + tx + 16 * j;
      if (col >= N) continue;
      float f = (float)(acc_nz[i][j] - 2 * acc_x[i][j]);
      if (bias) f += bias[col];
      C[(int64_t)row * ldc + col] = f;
    }
  }
}

}  // namespace
}  // namespace bnn

using namespace bnn;

BNN_API int bnn_gemm_xnor(const uint32_t* As, const uint32_t* Anz, int64_t lda, const uint32_t* Bs,
                          const uint32_t* Bnz, int64_t ldb, const float* bias, float* C, int64_t ldc,
                          int64_t M, int64_t N, int64_t kw, void* stream) {
  if (!As || !Anz || !Bs || !Bnz || !C || M < 0 || N < 0 || kw < 0 || kw % KWC != 0 || lda < kw ||
      ldb < kw || ldc < N || M > 0x7fffffff || N > 0x7fffffff) {
    set_error("bnn_gemm_xnor: bad arguments (M=%lld N=%lld kw=%lld; kw must be a multiple of 32)",
              (long long)M, (long long)N, (long long)kw);
    return kErrInval;
  }
  if (M == 0 || N == 0) return 0;
  if (kw == 0) {
    set_error("bnn_gemm_xnor: kw == 0 is not supported");
    return kErrInval;
  }
  const int gm = (int)((M + XT - 1) / XT), gn = (int)((N + XT - 1) / XT);
  hipLaunchKernelGGL(gemm_xnor_k, dim3((unsigned)((int64_t)gm * gn)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), As, Anz, lda, Bs, Bnz, ldb, bias, C, ldc,
                     (int)M, (int)N, (int)kw, gn);
  return check_launch("bnn_gemm_xnor");
}
