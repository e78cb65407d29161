// The training step's loss: torch.nn.CrossEntropyLoss (reduction 'mean') on the nets' LogSoftmax
// output (mnist-dist2.py:71-76 returns F.log_softmax / nn.LogSoftmax; the training loop applies
// criterion = nn.CrossEntropyLoss(), mnist-dist2.py:118-137), forward and backward, for the narrow
// class dimension of the MNIST heads (C <= 64, here 10).
//
//   fwd: lse_i = max_i + log(sum_j exp(p_ij - max_i)),  l_i = lse_i - p[i][y_i],  loss = sum_i l_i / M
//   bwd: dp[i][j] = go / M * (exp(p_ij - lse_i) - [j == y_i])
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

template <int C>
__global__ __launch_bounds__(CE_T) void ce_fwd_k(const float* __restrict__ p, const int64_t* __restrict__ y,
                                                int64_t M, float* __restrict__ lse, double* __restrict__ part) {
  const int t = threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * CE_T + t;
  double l = 0.0;
  if (i < M) {
    float v[C];
    const float ls = row_lse<C>(p + i * C, v);
    lse[i] = ls;
    const int64_t yi = y[i];
    float py = __builtin_nanf("");   // a target outside [0, C) makes the loss NaN
#pragma unroll
    for (int j = 0; j < C; ++j) py = (j == yi) ? v[j] : py;
    l = (double)(ls - py);
  }
  // block sum in row order: a fixed shuffle tree per wave, then the 4 waves in order
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) l += __shfl_xor(l, o, 64);
  __shared__ double ws[CE_T / 64];
  if ((t & 63) == 0) ws[t >> 6] = l;
  __syncthreads();
  if (t == 0) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < CE_T / 64; ++w) s += ws[w];
    part[blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(CE_T) void ce_fold_k(const double* __restrict__ part, int64_t nb, int64_t M,
                                                 float* __restrict__ loss) {
  // one workgroup: thread t sums blocks t, t + 256, ... in order, then a fixed tree over threads
  const int t = threadIdx.x;
  double s = 0.0;
  for (int64_t b = t; b < nb; b += CE_T) s += part[b];
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) s += __shfl_xor(s, o, 64);
  __shared__ double ws[CE_T / 64];
  if ((t & 63) == 0) ws[t >> 6] = s;
  __syncthreads();
  if (t == 0) {
    double a = 0.0;
#pragma unroll
    for (int w = 0; w < CE_T / 64; ++w) a += ws[w];
    loss[0] = (float)(a / (double)M);
  }
}

// small batches (M <= CE_ONE_MAX): the whole forward in ONE workgroup of 1024 threads, thread t
// taking rows t, t + 1024, ... in order, then a fixed tree -- no second (fold) launch
constexpr int CE_T1 = 1024;
constexpr int64_t CE_ONE_MAX = 16384;

template <int C>
__global__ __launch_bounds__(CE_T1) void ce_fwd1_k(const float* __restrict__ p, const int64_t* __restrict__ y,
                                                  int64_t M, float* __restrict__ lse, float* __restrict__ loss) {
  const int t = threadIdx.x;
  double l = 0.0;
  for (int64_t i = t; i < M; i += CE_T1) {
    float v[C];
    const float ls = row_lse<C>(p + i * C, v);
    lse[i] = ls;
    const int64_t yi = y[i];
    float py = __builtin_nanf("");
#pragma unroll
    for (int j = 0; j < C; ++j) py = (j == yi) ? v[j] : py;
    l += (double)(ls - py);
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) l += __shfl_xor(l, o, 64);
  __shared__ double ws[CE_T1 / 64];
  if ((t & 63) == 0) ws[t >> 6] = l;
  __syncthreads();
  if (t == 0) {
    double a = 0.0;
#pragma unroll
    for (int w = 0; w < CE_T1 / 64; ++w) a += ws[w];
    loss[0] = (float)(a / (double)M);
  }
}

template <int C>
__global__ __launch_bounds__(CE_T) void ce_bwd_k(const float* __restrict__ p, const int64_t* __restrict__ y,
                                                const float* __restrict__ lse, const float* __restrict__ go,
                                                int64_t M, float* __restrict__ dp) {
  const int64_t i = (int64_t)blockIdx.x * CE_T + threadIdx.x;
  if (i >= M) return;
  const float g = go[0] / (float)M;
  const float ls = lse[i];
  const int64_t yi = y[i];
  const float* pr = p + i * C;
  float* dr = dp + i * C;
#pragma unroll
  for (int j = 0; j < C; ++j) dr[j] = g * (expf(pr[j] - ls) - (j == yi ? 1.f : 0.f));
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

BNN_API int64_t bnn_cross_entropy_workspace(int64_t M) {
  // lse per row (fp32) + one double per 256-row block
  if (M <= 0) return 0;
  return (M * (int64_t)sizeof(float) + 15) / 16 * 16 + ((M + CE_T - 1) / CE_T) * (int64_t)sizeof(double);
}

BNN_API int bnn_cross_entropy_fwd(const float* p, const int64_t* y, int64_t M, int64_t C, float* loss, void* work,
                                  int64_t work_bytes, void* stream) {
  if (M <= 0 || !p || !y || !loss || !work || !bnn_cross_entropy_ok(C) ||
      work_bytes < bnn_cross_entropy_workspace(M)) {
    set_error("bnn_cross_entropy_fwd: bad arguments (M=%lld C=%lld work=%lld; M > 0, C in {2,10,16,32,64}, "
              "workspace bnn_cross_entropy_workspace(M))", (long long)M, (long long)C, (long long)work_bytes);
    return kErrInval;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* lse = reinterpret_cast<float*>(work);
  double* part = reinterpret_cast<double*>(reinterpret_cast<char*>(work) + (M * (int64_t)sizeof(float) + 15) / 16 * 16);
  const int64_t nb = (M + CE_T - 1) / CE_T;
  if (M <= CE_ONE_MAX) {
    BNN_CE_SWITCH((int)C, hipLaunchKernelGGL((ce_fwd1_k<CV>), dim3(1), dim3(CE_T1), 0, s, p, y, M, lse, loss));
    return check_launch("bnn_cross_entropy_fwd");
  }
  BNN_CE_SWITCH((int)C, hipLaunchKernelGGL((ce_fwd_k<CV>), dim3((unsigned)nb), dim3(CE_T), 0, s, p, y, M, lse, part));
  hipLaunchKernelGGL(ce_fold_k, dim3(1), dim3(CE_T), 0, s, part, nb, M, loss);
  return check_launch("bnn_cross_entropy_fwd");
}

BNN_API int bnn_cross_entropy_bwd(const float* p, const int64_t* y, int64_t M, int64_t C, const float* go,
                                  const void* work, float* dp, void* stream) {
  if (M <= 0 || !p || !y || !go || !work || !dp || !bnn_cross_entropy_ok(C)) {
    set_error("bnn_cross_entropy_bwd: bad arguments (M=%lld C=%lld)", (long long)M, (long long)C);
    return kErrInval;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const float* lse = reinterpret_cast<const float*>(work);
  BNN_CE_SWITCH((int)C, hipLaunchKernelGGL((ce_bwd_k<CV>), dim3((unsigned)((M + CE_T - 1) / CE_T)), dim3(CE_T), 0, s,
                                            p, y, lse, go, M, dp));
  return check_launch("bnn_cross_entropy_bwd");
}
