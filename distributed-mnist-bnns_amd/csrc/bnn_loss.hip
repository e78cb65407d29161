// The training step's loss: torch.nn.CrossEntropyLoss (reduction 'mean') on the nets' LogSoftmax
// output (mnist-dist2.py:71-76 returns F.log_softmax / nn.LogSoftmax; the training loop applies
// criterion = nn.CrossEntropyLoss(), mnist-dist2.py:118-137), forward and backward, for the narrow
// class dimension of the MNIST heads (C <= 64, here 10).
//
//   fwd: lse_i = max_i + log(sum_j exp(p_ij - max_i)),  l_i = lse_i - p[i][y_i],  loss = sum_i l_i / n
//   bwd: dp[i][j] = go / n * (exp(p_ij - lse_i) - [j == y_i])
//
// with torch's ignore_index: a row whose target equals it contributes neither a loss term nor a
// gradient (dp row = 0), and n = the number of the other rows (all rows ignored: loss NaN, as
// torch's 0 / 0).  n is formed on the device and kept in the workspace for the backward.
//
// torch runs this as log_softmax + nll_loss (+ their two backward kernels and a zero fill); the
// nll_loss forward reduction is a single workgroup (63 us at M = 65536).  Here: one thread per row,
// fp32 row arithmetic as torch's log_softmax (max subtraction, expf / logf), the row losses summed
// in double per 256-row block in row order and the blocks folded in block order by a one-workgroup
// kernel (up to 16384 rows: one 1024-thread workgroup does both); every order is fixed
// (deterministic); lse is kept per row for the backward, whose loss gradient go is read on the
// device (no host synchronisation: the step stays capturable in a HIP graph).
#include "bnn_common.h"

namespace bnn {
namespace {

constexpr int CE_T = 256;

template <int C>
__device__ __forceinline__ float row_lse(const float* __restrict__ pr, float (&v)[C]) {
#pragma unroll
  for (int j = 0; j < C; ++j) v[j] = pr[j];
  float mx = v[0];
#pragma unroll
  for (int j = 1; j < C; ++j) mx = fmaxf(mx, v[j]);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < C; ++j) s += expf(v[j] - mx);
  return mx + logf(s);
}

// one row's loss term and count (0, 0 for an ignored row)
template <int C>
__device__ __forceinline__ void row_loss(const float* __restrict__ p, const int64_t* __restrict__ y, int64_t i,
                                         int64_t ignore, float* __restrict__ lse, double& l, int& n) {
  float v[C];
  const float ls = row_lse<C>(p + i * C, v);
  lse[i] = ls;
  const int64_t yi = y[i];
  if (yi == ignore) return;
  float py = __builtin_nanf("");   // a target outside [0, C) makes the loss NaN
#pragma unroll
  for (int j = 0; j < C; ++j) py = (j == yi) ? v[j] : py;
  l += (double)(ls - py);
  n += 1;
}

template <int C>
__global__ __launch_bounds__(CE_T) void ce_fwd_k(const float* __restrict__ p, const int64_t* __restrict__ y,
                                                int64_t M, int64_t ignore, float* __restrict__ lse,
                                                double* __restrict__ part) {
  const int t = threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * CE_T + t;
  double l = 0.0;
  int n = 0;
  if (i < M) row_loss<C>(p, y, i, ignore, lse, l, n);
  // block sum in row order: a fixed shuffle tree per wave, then the 4 waves in order
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    l += __shfl_xor(l, o, 64);
    n += __shfl_xor(n, o, 64);
  }
  __shared__ double ws[CE_T / 64];
  __shared__ int wn[CE_T / 64];
  if ((t & 63) == 0) {
    ws[t >> 6] = l;
    wn[t >> 6] = n;
  }
  __syncthreads();
  if (t == 0) {
    double s = 0.0;
    int c = 0;
#pragma unroll
    for (int w = 0; w < CE_T / 64; ++w) {
      s += ws[w];
      c += wn[w];
    }
    part[2 * blockIdx.x] = s;
    part[2 * blockIdx.x + 1] = (double)c;
  }
}

__global__ __launch_bounds__(CE_T) void ce_fold_k(const double* __restrict__ part, int64_t nb, float* __restrict__ loss,
                                                 float* __restrict__ cnt) {
  // one workgroup: thread t sums blocks t, t + 256, ... in order, then a fixed tree over threads
  const int t = threadIdx.x;
  double s = 0.0, c = 0.0;
  for (int64_t b = t; b < nb; b += CE_T) {
    s += part[2 * b];
    c += part[2 * b + 1];
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    s += __shfl_xor(s, o, 64);
    c += __shfl_xor(c, o, 64);
  }
  __shared__ double ws[CE_T / 64], wc[CE_T / 64];
  if ((t & 63) == 0) {
    ws[t >> 6] = s;
    wc[t >> 6] = c;
  }
  __syncthreads();
  if (t == 0) {
    double a = 0.0, n = 0.0;
#pragma unroll
    for (int w = 0; w < CE_T / 64; ++w) {
      a += ws[w];
      n += wc[w];
    }
    loss[0] = (float)(a / n);
    cnt[0] = (float)n;
  }
}

// small batches (M <= CE_ONE_MAX): the whole forward in ONE workgroup of 1024 threads, thread t
// taking rows t, t + 1024, ... in order, then a fixed tree -- no second (fold) launch
constexpr int CE_T1 = 1024;
constexpr int64_t CE_ONE_MAX = 16384;

template <int C>
__global__ __launch_bounds__(CE_T1) void ce_fwd1_k(const float* __restrict__ p, const int64_t* __restrict__ y,
                                                  int64_t M, int64_t ignore, float* __restrict__ lse,
                                                  float* __restrict__ loss, float* __restrict__ cnt) {
  const int t = threadIdx.x;
  double l = 0.0;
  int n = 0;
  // U rows per trip, all their loads issued before any is used (the same row order as one at a time)
  constexpr int U = C <= 16 ? 4 : 1;
  for (int64_t i0 = t; i0 < M; i0 += U * CE_T1) {
    float v[U][C];
    int64_t yv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = min(i0 + (int64_t)u * CE_T1, M - 1);   // clamped: unconditional loads
#pragma unroll
      for (int j = 0; j < C; ++j) v[u][j] = p[i * C + j];
      yv[u] = y[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * CE_T1;
      if (i >= M) break;
      float mx = v[u][0];
#pragma unroll
      for (int j = 1; j < C; ++j) mx = fmaxf(mx, v[u][j]);
      float sm = 0.f;
#pragma unroll
      for (int j = 0; j < C; ++j) sm += expf(v[u][j] - mx);
      const float ls = mx + logf(sm);
      lse[i] = ls;
      if (yv[u] == ignore) continue;
      float py = __builtin_nanf("");
#pragma unroll
      for (int j = 0; j < C; ++j) py = (j == yv[u]) ? v[u][j] : py;
      l += (double)(ls - py);
      n += 1;
    }
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    l += __shfl_xor(l, o, 64);
    n += __shfl_xor(n, o, 64);
  }
  __shared__ double ws[CE_T1 / 64];
  __shared__ int wn[CE_T1 / 64];
  if ((t & 63) == 0) {
    ws[t >> 6] = l;
    wn[t >> 6] = n;
  }
  __syncthreads();
  if (t == 0) {
    double a = 0.0;
    int c = 0;
#pragma unroll
    for (int w = 0; w < CE_T1 / 64; ++w) {
      a += ws[w];
      c += wn[w];
    }
    loss[0] = (float)(a / (double)c);
    cnt[0] = (float)c;
  }
}

// one thread per element (row-major, coalesced loads and stores; a row's 10 elements over 10 lanes)
template <int C>
__global__ __launch_bounds__(CE_T) void ce_bwd_k(const float* __restrict__ p, const int64_t* __restrict__ y,
                                                const float* __restrict__ lse, const float* __restrict__ cnt,
                                                const float* __restrict__ go, int64_t M, int64_t ignore,
                                                float* __restrict__ dp) {
  const int64_t e = (int64_t)blockIdx.x * CE_T + threadIdx.x;
  if (e >= M * C) return;
  const int64_t i = e / C;
  const int j = (int)(e - i * C);
  const float g = go[0] / cnt[0];
  const int64_t yi = y[i];
  dp[e] = yi == ignore ? 0.f : g * (expf(p[e] - lse[i]) - (j == yi ? 1.f : 0.f));
}

}  // namespace
}  // namespace bnn

using namespace bnn;

#define BNN_CE_SWITCH(C, ...)                        \
  switch (C) {                                       \
    case 10: { constexpr int CV = 10; __VA_ARGS__; } break; \
    case 2: { constexpr int CV = 2; __VA_ARGS__; } break;   \
    case 16: { constexpr int CV = 16; __VA_ARGS__; } break; \
    case 32: { constexpr int CV = 32; __VA_ARGS__; } break; \
    case 64: { constexpr int CV = 64; __VA_ARGS__; } break; \
    default: break;                                  \
  }

BNN_API int bnn_cross_entropy_ok(int64_t C) { return C == 2 || C == 10 || C == 16 || C == 32 || C == 64; }

// workspace: lse per row (fp32), the kept-row count (fp32, 16 B), two doubles per 256-row block
static int64_t ce_lse_bytes(int64_t M) { return (M * (int64_t)sizeof(float) + 15) / 16 * 16; }

BNN_API int64_t bnn_cross_entropy_workspace(int64_t M) {
  if (M <= 0) return 0;
  return ce_lse_bytes(M) + 16 + ((M + CE_T - 1) / CE_T) * 2 * (int64_t)sizeof(double);
}

BNN_API int bnn_cross_entropy_fwd(const float* p, const int64_t* y, int64_t M, int64_t C, int64_t ignore_index,
                                  float* loss, void* work, int64_t work_bytes, void* stream) {
  if (M <= 0 || !p || !y || !loss || !work || !bnn_cross_entropy_ok(C) ||
      work_bytes < bnn_cross_entropy_workspace(M)) {
    set_error("bnn_cross_entropy_fwd: bad arguments (M=%lld C=%lld work=%lld; M > 0, C in {2,10,16,32,64}, "
              "workspace bnn_cross_entropy_workspace(M))", (long long)M, (long long)C, (long long)work_bytes);
    return kErrInval;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* lse = reinterpret_cast<float*>(work);
  float* cnt = reinterpret_cast<float*>(reinterpret_cast<char*>(work) + ce_lse_bytes(M));
  double* part = reinterpret_cast<double*>(reinterpret_cast<char*>(work) + ce_lse_bytes(M) + 16);
  const int64_t nb = (M + CE_T - 1) / CE_T;
  if (M <= CE_ONE_MAX) {
    BNN_CE_SWITCH((int)C, hipLaunchKernelGGL((ce_fwd1_k<CV>), dim3(1), dim3(CE_T1), 0, s, p, y, M, ignore_index, lse,
                                              loss, cnt));
    return check_launch("bnn_cross_entropy_fwd");
  }
  BNN_CE_SWITCH((int)C, hipLaunchKernelGGL((ce_fwd_k<CV>), dim3((unsigned)nb), dim3(CE_T), 0, s, p, y, M, ignore_index,
                                            lse, part));
  hipLaunchKernelGGL(ce_fold_k, dim3(1), dim3(CE_T), 0, s, part, nb, loss, cnt);
  return check_launch("bnn_cross_entropy_fwd");
}

BNN_API int bnn_cross_entropy_bwd(const float* p, const int64_t* y, int64_t M, int64_t C, int64_t ignore_index,
                                  const float* go, const void* work, float* dp, void* stream) {
  if (M <= 0 || !p || !y || !go || !work || !dp || !bnn_cross_entropy_ok(C)) {
    set_error("bnn_cross_entropy_bwd: bad arguments (M=%lld C=%lld)", (long long)M, (long long)C);
    return kErrInval;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const float* lse = reinterpret_cast<const float*>(work);
  const float* cnt = reinterpret_cast<const float*>(reinterpret_cast<const char*>(work) + ce_lse_bytes(M));
  BNN_CE_SWITCH((int)C, hipLaunchKernelGGL((ce_bwd_k<CV>), dim3((unsigned)((M * CV + CE_T - 1) / CE_T)), dim3(CE_T), 0, s,
                                            p, y, lse, cnt, go, M, ignore_index, dp));
  return check_launch("bnn_cross_entropy_bwd");
}
