// u8 pixel operands of the first BinarizeLinear (f3: the input pipeline).
//
// The reference feeds x = ToTensor(u8) = u / 255 (optionally Normalize((m,), (s,)),
// mnist-distributed-BNNS2.py:82) into fc1 (mnist-dist2.py:60, models/binarized_modules.py:80,
// input not binarised because size(1) == 784).  Every such x is an affine image of the byte:
//   x = a * v + c,   v = u - 128 in [-128, 127],  a = 1 / (255 s),  c = (128 / 255 - m) / s,
// so with v kept as an int8 plane the first layer's products are exact integer sums on the int8
// MFMA (one pass instead of the three digit planes an fp32 x needs).  With s0 = c / a
// (= 128 for ToTensor) the offset is folded back into the integer sum before any rounding:
//   fc1:  y[b][n]  = a * (sum_k v[b][k] W_b[n][k] + s0 * R[n]) + bias[n],  R[n] = sum_k W_b[n][k]
//   dW1:  dW[n][k] = a * g[n] * (sum_b D[b][n] v[b][k] + s0 * T[n]),  T[n] = sum_b D[b][n]
// (D = the digits of dY, g = their column scale, bnn_quant_cols_t_dsum), so for ToTensor both are
// the exact integer sums over u itself: a pixel column that is zero across the batch gets an
// exactly zero weight gradient, as the reference's fp32 GEMM gives it (Adam then leaves that
// weight untouched).  bnn_pixels_pack writes the int8 rows v (the fc1 A operand) and their
// transpose (the dW1 B operand) in one pass over the bytes; bnn_row_sums gives R.
#include <algorithm>
#include <cstdint>

#include "bnn.h"
#include "bnn_common.h"

namespace bnn {
namespace {

constexpr int PT = 64;   // pixel tile edge (rows x bytes)

// grid (k tiles, m tiles), 256 threads: thread t owns row t/4 and the 16-byte chunk t%4 of a
// 64 x 64 byte tile; rows are stored straight from registers, the transpose goes through LDS.
__global__ __launch_bounds__(256) void pixels_pack_k(const uint8_t* __restrict__ x, int64_t M, int64_t K,
                                                     int64_t ldx, int8_t* __restrict__ q, int64_t ldq,
                                                     int8_t* __restrict__ qt, int64_t ldqt) {
  __shared__ uint32_t tile[PT][PT / 4 + 1];   // +1 dword: transposed reads spread over banks
  const int t = threadIdx.x, r = t >> 2, c = t & 3;
  const int64_t m = (int64_t)blockIdx.y * PT + r;
  const int64_t k = (int64_t)blockIdx.x * PT + 16 * c;
  uint32_t w[4] = {0u, 0u, 0u, 0u};
  if (m < M) {
    const uint8_t* src = x + m * ldx + k;
    if (k + 16 <= K && ((reinterpret_cast<uintptr_t>(src) & 15u) == 0)) {
      const uint4 u = *reinterpret_cast<const uint4*>(src);
      w[0] = u.x ^ 0x80808080u;
      w[1] = u.y ^ 0x80808080u;
      w[2] = u.z ^ 0x80808080u;
      w[3] = u.w ^ 0x80808080u;
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (k + j < K) w[j >> 2] |= (uint32_t)(src[j] ^ 0x80u) << (8 * (j & 3));
    }
  }
  if (q && m < M && k < ldq) *reinterpret_cast<uint4*>(q + m * ldq + k) = make_uint4(w[0], w[1], w[2], w[3]);
  if (!qt) return;
#pragma unroll
  for (int j = 0; j < 4; ++j) tile[r][4 * c + j] = w[j];
  __syncthreads();
  // transposed: thread t writes qt row kk = k0 + t/4, bytes m0 + 16(t%4) .. +15
  const int kr = t >> 2;
  const int64_t kk = (int64_t)blockIdx.x * PT + kr;
  const int64_t mm = (int64_t)blockIdx.y * PT + 16 * c;
  if (kk >= K || mm >= ldqt) return;
  uint32_t o[4] = {0u, 0u, 0u, 0u};
  const uint8_t* tb = reinterpret_cast<const uint8_t*>(&tile[0][0]);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int row = 16 * c + j;
    o[j >> 2] |= (uint32_t)tb[row * (PT + 4) + kr] << (8 * (j & 3));
  }
  *reinterpret_cast<uint4*>(qt + kk * ldqt + mm) = make_uint4(o[0], o[1], o[2], o[3]);
}

// out[n] = sum_k q[n][k] (exact): one wave per row, 4 rows per block.
__global__ __launch_bounds__(256) void row_sums_k(const int8_t* __restrict__ q, int64_t N, int64_t K,
                                                  int64_t ldq, int64_t* __restrict__ out) {
  const int64_t n = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (n >= N) return;
  const int8_t* row = q + n * ldq;
  int s = 0;
  for (int64_t k = lane; k < K; k += 64) s += row[k];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) out[n] = s;
}

// ToTensor's image of a byte back to the byte: u = rint(255 x) when 0 <= u <= 255 and x is, bit for
// bit, fl(u / 255) (torchvision's img.float().div(255) on the host: a correctly rounded division) or
// fl(u * fl(1 / 255)) (the same division by a scalar on the GPU, which torch runs as a multiply by
// the reciprocal); else bad |= 1 (one vector atomic per wave that saw a mismatch).  4 elements per
// thread (16-B loads), grid-stride.
__global__ __launch_bounds__(256) void unit_to_pixels_k(const float* __restrict__ x, int64_t n, uint8_t* __restrict__ u,
                                                        int* __restrict__ bad) {
  bool miss = false;
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    const float e[4] = {v.x, v.y, v.z, v.w};
    uint32_t w = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float r = rintf(e[j] * 255.f);
      const bool ok = r >= 0.f && r <= 255.f && ((r / 255.f) == e[j] || r * (1.f / 255.f) == e[j]);
      miss |= !ok;
      w |= (uint32_t)(ok ? (int)r : 0) << (8 * j);
    }
    reinterpret_cast<uint32_t*>(u)[i] = w;
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float r = rintf(x[i] * 255.f);
    const bool ok = r >= 0.f && r <= 255.f && ((r / 255.f) == x[i] || r * (1.f / 255.f) == x[i]);
    miss |= !ok;
    u[i] = (uint8_t)(ok ? (int)r : 0);
  }
  if (__any(miss) && (threadIdx.x & 63) == 0) atomicOr(bad, 1);
}

}  // namespace
}  // namespace bnn

using namespace bnn;

BNN_API int bnn_unit_to_pixels(const float* x, int64_t n, uint8_t* u, int32_t* bad, void* stream) {
  if (!x || !u || !bad || n < 0 || !aligned16(x) || (reinterpret_cast<uintptr_t>(u) & 3) != 0) {
    set_error("bnn_unit_to_pixels: bad arguments (n=%lld; x 16-B, u 4-B aligned)", (long long)n);
    return kErrInval;
  }
  if (n == 0) return 0;
  const int64_t blocks = std::min<int64_t>((n / 4 + 255) / 256 + 1, 8192);
  hipLaunchKernelGGL(unit_to_pixels_k, dim3((unsigned)blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     x, n, u, reinterpret_cast<int*>(bad));
  return check_launch("bnn_unit_to_pixels");
}

BNN_API int bnn_pixels_pack(const uint8_t* x, int64_t M, int64_t K, int64_t ldx, int8_t* q, int64_t ldq,
                            int8_t* qt, int64_t ldqt, void* stream) {
  if (!x || M < 0 || K <= 0 || ldx < K || (!q && !qt) ||
      (q && (ldq < round_up(K, 64) || ldq % 16 != 0 || !aligned16(q))) ||
      (qt && (ldqt < round_up(M, 64) || ldqt % 16 != 0 || !aligned16(qt))) ||
      M > 0x7fffffffLL * PT || K > 0x7fffffffLL) {
    set_error("bnn_pixels_pack: bad arguments (M=%lld K=%lld ldx=%lld ldq=%lld ldqt=%lld; ldq >= round_up(K,64), "
              "ldqt >= round_up(M,64), both multiples of 16)",
              (long long)M, (long long)K, (long long)ldx, (long long)ldq, (long long)ldqt);
    return kErrInval;
  }
  const int64_t kcols = std::max(q ? ldq : 0, K);
  const int64_t mrows = std::max(M, qt ? ldqt : 0);
  if (mrows == 0) return 0;
  const dim3 grid((unsigned)((kcols + PT - 1) / PT), (unsigned)((mrows + PT - 1) / PT));
  if (grid.y > 65535u) {
    set_error("bnn_pixels_pack: M too large (%lld rows)", (long long)M);
    return kErrInval;
  }
  hipLaunchKernelGGL(pixels_pack_k, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), x, M, K, ldx, q,
                     ldq, qt, ldqt);
  return check_launch("bnn_pixels_pack");
}

BNN_API int bnn_row_sums(const int8_t* q, int64_t N, int64_t K, int64_t ldq, int64_t* out, void* stream) {
  if (!q || !out || N < 0 || K < 0 || ldq < K || K > (1LL << 40)) {
    set_error("bnn_row_sums: bad arguments (N=%lld K=%lld ldq=%lld)", (long long)N, (long long)K,
              (long long)ldq);
    return kErrInval;
  }
  if (N == 0) return 0;
  hipLaunchKernelGGL(row_sums_k, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     q, N, K, ldq, out);
  return check_launch("bnn_row_sums");
}
