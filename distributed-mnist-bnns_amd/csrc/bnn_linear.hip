// fp32 Linear with a narrow output (N <= 16): the BinCNN's classifier, nn.Linear(7*7*32, 10)
// (the reference's binarized CNN, BASELINE config 4), forward and backward.  A library GEMM spends
// ~16 us per product on this 4096 x 1568 x 10 shape (three products per step); each pass here reads
// its fp32 operand once at HBM rate.
//
//   fwd: y[m][n] = sum_k x[m][k] w[n][k] + b[n]
//   bwd: dx[m][k] = sum_n dy[m][n] w[n][k];  dw[n][k] = sum_m dy[m][n] x[m][k];  db[n] = sum_m dy[m][n]
//
// fp32 products and fp32 sums in a fixed order (deterministic; the numerics class of torch's fp32
// F.linear, in another summation order).  The weight gradient is summed per block of rows into a
// workspace and folded over the blocks in block order.
#include "bnn_common.h"

namespace bnn {
namespace {

constexpr int LS_NMAX = 16;
constexpr int LS_T = 256;

__device__ __forceinline__ float4 ldf4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// 16 rows per workgroup, 16 lanes per row: lane j takes the float4 columns 4j, 4j + 64, ...; all of
// w (N x K floats, dynamic LDS) is staged once per workgroup -- every row group would read it from
// L2 otherwise -- so the K loop has no barrier and its x loads run ahead; the 16 partial dot
// products of a row fold with a fixed xor tree inside the 16-lane group
template <int N>
__global__ __launch_bounds__(LS_T) void linear_nsmall_fwd_k(const float* __restrict__ x, int64_t M, int64_t K,
                                                            const float* __restrict__ w,
                                                            const float* __restrict__ b, float* __restrict__ y) {
  extern __shared__ float4 ws4[];
  const int t = threadIdx.x, j = t & 15;
  const int K4 = (int)(K / 4);
  for (int i = t; i < N * K4; i += LS_T) ws4[i] = reinterpret_cast<const float4*>(w)[i];
  __syncthreads();
  const int64_t row = (int64_t)blockIdx.x * (LS_T / 16) + (t >> 4);
  if (row >= M) return;
  const float4* xr = reinterpret_cast<const float4*>(x + row * K);
  float acc[N];
#pragma unroll
  for (int n = 0; n < N; ++n) acc[n] = 0.f;
#pragma unroll 8
  for (int k4 = j; k4 < K4; k4 += 16) {
    const float4 xv = xr[k4];
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const float4 wv = ws4[n * K4 + k4];
      acc[n] = fmaf(xv.x, wv.x, acc[n]);
      acc[n] = fmaf(xv.y, wv.y, acc[n]);
      acc[n] = fmaf(xv.z, wv.z, acc[n]);
      acc[n] = fmaf(xv.w, wv.w, acc[n]);
    }
  }
#pragma unroll
  for (int o = 1; o < 16; o <<= 1)
#pragma unroll
    for (int n = 0; n < N; ++n) acc[n] += __shfl_xor(acc[n], o, 16);
  if (j == 0) {
#pragma unroll
    for (int n = 0; n < N; ++n) y[row * N + n] = acc[n] + (b ? b[n] : 0.f);
  }
}

// rows [blk * rpb, ..) of the batch: thread t owns the float4 columns 4t, 4t + 1024, ...; for each
// column it holds w's N x 4 values and the block's dW partial, walking the block's rows (dy rows
// staged in LDS): dx is written, the partial goes to part[blk][N][K]
template <int N>
__global__ __launch_bounds__(LS_T) void linear_nsmall_bwd_k(const float* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ dy, int64_t M, int64_t K,
                                                            int64_t rpb, float* __restrict__ dx,
                                                            float* __restrict__ part, float* __restrict__ dbp) {
  __shared__ float dys[64][N];
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = (r0 + rpb < M) ? r0 + rpb : M;
  float dbs = 0.f;                     // thread t < N, first column pass: this block's sum of dy[:, t]
  // every thread runs the same number of column passes (the row loop has barriers); a thread past
  // K in the last pass stages dy and computes nothing
  for (int64_t kb = 0; kb < K; kb += 4 * LS_T) {
    const int64_t k = kb + 4 * (int64_t)t;
    const bool live = k < K;
    float4 wc[N], dw[N];
#pragma unroll
    for (int n = 0; n < N; ++n) {
      wc[n] = live ? ldf4(w + n * K + k) : make_float4(0.f, 0.f, 0.f, 0.f);
      dw[n] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int64_t rb = r0; rb < r1; rb += 64) {
      const int64_t re = (rb + 64 < r1) ? rb + 64 : r1;
      __syncthreads();
      for (int i = t; i < (int)(re - rb) * N; i += LS_T) dys[i / N][i % N] = dy[rb * N + i];
      __syncthreads();
      if (kb == 0 && t < N)
        for (int r = 0; r < (int)(re - rb); ++r) dbs += dys[r][t];
      if (!live) continue;
      for (int64_t r = rb; r < re; ++r) {
        const float4 xv = ldf4(x + r * K + k);
        float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int n = 0; n < N; ++n) {
          const float g = dys[r - rb][n];
          o.x = fmaf(g, wc[n].x, o.x);
          o.y = fmaf(g, wc[n].y, o.y);
          o.z = fmaf(g, wc[n].z, o.z);
          o.w = fmaf(g, wc[n].w, o.w);
          dw[n].x = fmaf(g, xv.x, dw[n].x);
          dw[n].y = fmaf(g, xv.y, dw[n].y);
          dw[n].z = fmaf(g, xv.z, dw[n].z);
          dw[n].w = fmaf(g, xv.w, dw[n].w);
        }
        if (dx) *reinterpret_cast<float4*>(dx + r * K + k) = o;
      }
    }
    if (live && part != nullptr) {
      float* pb = part + (int64_t)blockIdx.x * N * K;
#pragma unroll
      for (int n = 0; n < N; ++n) *reinterpret_cast<float4*>(pb + n * K + k) = dw[n];
    }
  }
  if (t < N && dbp != nullptr) dbp[(int64_t)blockIdx.x * N + t] = dbs;
}

// dw[i] = sum over blocks of part[blk][i]: a workgroup takes 32 outputs x 8 segments of the blocks
// (coalesced 128-B rows per load, 8 loads in flight per thread), the segments folded in order;
// db[n] (one extra workgroup) = the blocks' dy column sums (dbp[blk][n]) in block order
__global__ __launch_bounds__(LS_T) void linear_nsmall_fold_k(const float* __restrict__ part, int64_t G, int64_t NK,
                                                             float* __restrict__ dw, const float* __restrict__ dbp,
                                                             int N, float* __restrict__ db) {
  __shared__ float rf[8 * 32];         // [8 segments][32 outputs]
  const int t = threadIdx.x;
  const int64_t nfold = (NK + 31) / 32;
  if ((int64_t)blockIdx.x < nfold) {
    if (dw == nullptr) return;
    const int o = t & 31, seg = t >> 5;
    const int64_t i = (int64_t)blockIdx.x * 32 + o;
    const int64_t g0 = seg * ((G + 7) / 8), g1 = (g0 + (G + 7) / 8 < G) ? g0 + (G + 7) / 8 : G;
    float s = 0.f;
    if (i < NK) {
      int64_t g = g0;
      for (; g + 8 <= g1; g += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = part[(g + u) * NK + i];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
      }
      for (; g < g1; ++g) s += part[g * NK + i];
    }
    rf[seg * 32 + o] = s;
    __syncthreads();
    if (t < 32 && i < NK) {
      float a = 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u) a += rf[u * 32 + o];
      dw[i] = a;
    }
    return;
  }
  if (db == nullptr) return;
  // db[n] = the blocks' partial sums: thread (n = t % 16, segment t / 16 of the blocks), the 16
  // segments folded in order
  const int n = t & 15, seg = t >> 4;
  const int64_t gs = (G + 15) / 16, g0 = seg * gs, g1 = (g0 + gs < G) ? g0 + gs : G;
  float a = 0.f;
  if (n < N)
    for (int64_t g = g0; g < g1; ++g) a += dbp[g * N + n];
  rf[seg * 16 + n] = a;
  __syncthreads();
  if (t < N) {
    float d = 0.f;
#pragma unroll
    for (int u = 0; u < 16; ++u) d += rf[u * 16 + t];
    db[t] = d;
  }
}

int64_t ls_rows_per_block(int64_t M) {
  // at most 512 blocks (the dW partials stay <= 512 x N x K floats), at least 16 rows each
  const int64_t r = (M + 511) / 512;
  return r < 16 ? 16 : r;
}

#define BNN_LS_SWITCH(N_, CALL)                                                       \
  switch (N_) {                                                                       \
    case 10: { constexpr int NV = 10; CALL; } break;                                  \
    case 1: { constexpr int NV = 1; CALL; } break;                                    \
    case 2: { constexpr int NV = 2; CALL; } break;                                    \
    case 4: { constexpr int NV = 4; CALL; } break;                                    \
    case 8: { constexpr int NV = 8; CALL; } break;                                    \
    case 16: { constexpr int NV = 16; CALL; } break;                                  \
    default: set_error("bnn_linear_nsmall: N = %lld not built (1, 2, 4, 8, 10, 16)", (long long)(N_)); \
      return kErrInval;                                                               \
  }

// out[n] = sum_m y[m][n] for a narrow matrix (N <= 16; the head's bias gradient db4 = dY4.sum(0)):
// ONE workgroup, 64 row lanes x 16 column lanes, each lane summing its rows in order (double), the
// 64 row lanes folded in order -- fixed order (deterministic), one launch for batches up to
// CS_MAX_M rows (a torch reduction took ~10 us at 4096 rows in the HIP-graph MLP step)
constexpr int CS_T = 1024;
constexpr int64_t CS_MAX_M = 32768;
__global__ __launch_bounds__(CS_T) void col_sums_narrow_k(const float* __restrict__ y, int64_t M, int N, int64_t ld,
                                                          float* __restrict__ out) {
  __shared__ double red[CS_T / 16][16];
  const int t = threadIdx.x, n = t & 15, rl = t >> 4;
  double s = 0.0;
  if (n < N) {
    int64_t r = rl;
    for (; r + 3 * (CS_T / 16) < M; r += 4 * (CS_T / 16)) {   // 4 loads in flight
      const float a = y[r * ld + n], b = y[(r + CS_T / 16) * ld + n];
      const float c = y[(r + 2 * (CS_T / 16)) * ld + n], d = y[(r + 3 * (CS_T / 16)) * ld + n];
      s += (double)a;
      s += (double)b;
      s += (double)c;
      s += (double)d;
    }
    for (; r < M; r += CS_T / 16) s += (double)y[r * ld + n];
  }
  red[rl][n] = s;
  __syncthreads();
  if (rl == 0 && n < N) {
    double a = 0.0;
    for (int i = 0; i < CS_T / 16; ++i) a += red[i][n];
    out[n] = (float)a;
  }
}

}  // namespace
}  // namespace bnn

using namespace bnn;

BNN_API int64_t bnn_linear_nsmall_workspace(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  // per block: its dW partial (N x K) and its dy column sums (N)
  return ((M + ls_rows_per_block(M) - 1) / ls_rows_per_block(M)) * N * (K + 1) * (int64_t)sizeof(float);
}

BNN_API int bnn_linear_nsmall_fwd(const float* x, int64_t M, int64_t K, const float* w, const float* b, int64_t N,
                                  float* y, void* stream) {
  if (!w || (M > 0 && (!x || !y || !aligned16(x))) || M < 0 || K <= 0 || K % 4 != 0 || N <= 0 || N > LS_NMAX ||
      !aligned16(w) || N * K > 16384) {
    set_error("bnn_linear_nsmall_fwd: bad arguments (M=%lld K=%lld N=%lld; K %% 4 == 0, N <= 16, N*K <= 16384 "
              "(w in 64 KiB of LDS), 16-B aligned)",
              (long long)M, (long long)K, (long long)N);
    return kErrInval;
  }
  if (M == 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)((M + LS_T / 16 - 1) / (LS_T / 16)));
  BNN_LS_SWITCH(N, hipLaunchKernelGGL((linear_nsmall_fwd_k<NV>), grid, dim3(LS_T), (size_t)N * K * sizeof(float), s,
                                      x, M, K, w, b, y));
  return check_launch("bnn_linear_nsmall_fwd");
}

BNN_API int bnn_linear_nsmall_bwd(const float* x, const float* w, const float* dy, int64_t M, int64_t K, int64_t N,
                                  float* dx, float* dw, float* db, void* work, int64_t work_bytes, void* stream) {
  if (!w || (M > 0 && (!x || !dy || !aligned16(x) || (dx && !aligned16(dx)))) || M < 0 || K <= 0 || K % 4 != 0 ||
      N <= 0 || N > LS_NMAX || !aligned16(w) || ((dw || db) && M > 0 && (!work || !aligned16(work) ||
      work_bytes < bnn_linear_nsmall_workspace(M, N, K)))) {
    set_error("bnn_linear_nsmall_bwd: bad arguments (M=%lld K=%lld N=%lld work=%lld; K %% 4 == 0, N <= 16, "
              "16-B aligned, workspace bnn_linear_nsmall_workspace)", (long long)M, (long long)K, (long long)N,
              (long long)work_bytes);
    return kErrInval;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (M == 0) {
    if (dw) (void)hipMemsetAsync(dw, 0, N * K * sizeof(float), s);
    if (db) (void)hipMemsetAsync(db, 0, N * sizeof(float), s);
    return check_launch("bnn_linear_nsmall_bwd");
  }
  const int64_t rpb = ls_rows_per_block(M), G = (M + rpb - 1) / rpb;
  float* part = reinterpret_cast<float*>(work);
  const int64_t NK = N * K, nb = (NK + 31) / 32;
  float* dbp = part ? part + G * NK : nullptr;
  if (dx || dw || db)
    BNN_LS_SWITCH(N, hipLaunchKernelGGL((linear_nsmall_bwd_k<NV>), dim3((unsigned)G), dim3(LS_T), 0, s, x, w, dy, M,
                                        K, rpb, dx, dw ? part : nullptr, db ? dbp : nullptr));
  if (dw || db)
    hipLaunchKernelGGL(linear_nsmall_fold_k, dim3((unsigned)(nb + 1)), dim3(LS_T), 0, s, part, G, NK, dw, dbp,
                       (int)N, db);
  return check_launch("bnn_linear_nsmall_bwd");
}

BNN_API int bnn_col_sums_narrow(const float* y, int64_t M, int64_t N, int64_t ld, float* out, void* stream) {
  if (!y || !out || M <= 0 || M > CS_MAX_M || N <= 0 || N > 16 || ld < N) {
    set_error("bnn_col_sums_narrow: bad arguments (M=%lld N=%lld ld=%lld; 0 < M <= %lld, 0 < N <= 16)",
              (long long)M, (long long)N, (long long)ld, (long long)CS_MAX_M);
    return kErrInval;
  }
  hipLaunchKernelGGL(col_sums_narrow_k, dim3(1), dim3(CS_T), 0, reinterpret_cast<hipStream_t>(stream), y, M, (int)N,
                     ld, out);
  return check_launch("bnn_col_sums_narrow");
}
