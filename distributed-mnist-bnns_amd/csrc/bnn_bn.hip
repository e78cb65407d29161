// BatchNorm1d (train/eval) with an optional fused Hardtanh, for the [B, C] activations between
// the binarized layers (mnist-dist2.py:52-74: fc -> BatchNorm1d -> Hardtanh).
//
// torch's channels-last BN kernels take ~17-21 ms per call on a [65536, 8192] fp32 tensor on
// MI355X (profiles/r01_wide_b65536_kernel_stats.csv): this file replaces them with HBM-streaming
// passes -- a column reduction (per 256-row chunk, merged in a fixed order: deterministic) and a
// float4 elementwise pass.
//
// Forward (train): mean, biased var over the batch; y = (x-mean)*invstd*gamma + beta;
// running_mean/var updated with the unbiased var (torch semantics); hardtanh -> clamp(y,-1,1).
// Backward: with g = dy * (hardtanh ? (-1 < y < 1) : 1) (y recomputed from x, not stored),
// dbeta = sum g, dgamma = sum g*xhat, dx = gamma*invstd*(g - dbeta/n - xhat*dgamma/n).
#include <algorithm>
#include <cmath>

#include "bnn_common.h"

namespace bnn {
namespace {

constexpr int BN_ROWS = 256;  // rows per partial-statistics chunk

inline int64_t bn_chunks(int64_t M) { return std::max<int64_t>(1, (M + BN_ROWS - 1) / BN_ROWS); }

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// MODE 0: per-chunk (mean, M2), accumulated as deviations from the chunk's first row so the
//         float partials see deviations rather than raw magnitudes; merged with Chan's formula.
// MODE 1: per-chunk (sum g, sum g*xhat) with g = dy*mask(y).
// One thread = 4 adjacent columns (float4), rows walked in 16-row float partials folded to double.
template <int MODE>
__global__ __launch_bounds__(256) void bn_reduce_k(const float* __restrict__ x, const float* __restrict__ dy,
                                                   int64_t M, int64_t C, const float* __restrict__ mean,
                                                   const float* __restrict__ invstd,
                                                   const float* __restrict__ gamma,
                                                   const float* __restrict__ beta, int hardtanh,
                                                   double* __restrict__ p0, double* __restrict__ p1) {
  const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (c >= C) return;
  const int64_t r0 = (int64_t)blockIdx.y * BN_ROWS;
  const int64_t r1 = (M < r0 + BN_ROWS) ? M : r0 + BN_ROWS;
  double a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
  float mu[4], is[4] = {1, 1, 1, 1}, ga[4] = {1, 1, 1, 1}, be[4] = {0, 0, 0, 0};
  if (MODE == 0) {
    const float4 sv = ld4(x + r0 * C + c);
    mu[0] = sv.x;
    mu[1] = sv.y;
    mu[2] = sv.z;
    mu[3] = sv.w;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mu[j] = mean[c + j];
      is[j] = invstd[c + j];
      ga[j] = gamma ? gamma[c + j] : 1.f;
      be[j] = beta ? beta[c + j] : 0.f;
    }
  }
  for (int64_t r = r0; r < r1; r += 16) {
    float fa[4] = {0, 0, 0, 0}, fb[4] = {0, 0, 0, 0};
    const int64_t re = (r + 16 < r1) ? r + 16 : r1;
    for (int64_t rr = r; rr < re; ++rr) {
      const float4 xv = ld4(x + rr * C + c);
      const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
      if (MODE == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = xs[j] - mu[j];
          fa[j] += d;
          fb[j] = fmaf(d, d, fb[j]);
        }
      } else {
        const float4 gv = ld4(dy + rr * C + c);
        const float gs[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float xh = (xs[j] - mu[j]) * is[j];
          const float y = fmaf(xh, ga[j], be[j]);
          const float g = (!hardtanh || (y > -1.f && y < 1.f)) ? gs[j] : 0.f;
          fa[j] += g;
          fb[j] = fmaf(g, xh, fb[j]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] += (double)fa[j];
      b[j] += (double)fb[j];
    }
  }
  const int64_t o = blockIdx.y * C + c;
  if (MODE == 0) {
    const double n = (double)(r1 - r0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double dm = a[j] / n;
      p0[o + j] = (double)mu[j] + dm;  // chunk mean
      p1[o + j] = b[j] - a[j] * dm;    // chunk M2 = sum d^2 - (sum d)^2 / n
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p0[o + j] = a[j];
      p1[o + j] = b[j];
    }
  }
}

__global__ __launch_bounds__(256) void bn_fwd_final_k(const double* __restrict__ p0, const double* __restrict__ p1,
                                                      int64_t M, int64_t C, int64_t R, float momentum, float eps,
                                                      float* __restrict__ rmean, float* __restrict__ rvar,
                                                      float* __restrict__ save_mean,
                                                      float* __restrict__ save_invstd) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  double n = 0.0, mean = 0.0, m2 = 0.0;
  for (int64_t r = 0; r < R; ++r) {  // Chan et al. merge in a fixed order
    const int64_t hi = ((r + 1) * BN_ROWS < M) ? (r + 1) * BN_ROWS : M;
    const double nb = (double)(hi - r * BN_ROWS);
    const double mb = p0[r * C + c], m2b = p1[r * C + c];
    const double nt = n + nb, delta = mb - mean;
    mean += delta * nb / nt;
    m2 += m2b + delta * delta * n * nb / nt;
    n = nt;
  }
  double var = m2 / n;
  if (var < 0.0) var = 0.0;
  save_mean[c] = (float)mean;
  save_invstd[c] = (float)(1.0 / std::sqrt(var + (double)eps));
  if (rmean != nullptr && momentum >= 0.f) {
    const double unb = M > 1 ? m2 / (n - 1.0) : var;
    rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
    rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unb);
  }
}

__global__ __launch_bounds__(256) void bn_invstd_k(const float* __restrict__ rv, float* __restrict__ out,
                                                   int64_t C, float eps) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c < C) out[c] = (float)(1.0 / std::sqrt((double)rv[c] + (double)eps));
}

// y = (x-mean)*invstd*gamma + beta  [then clamp]; train (batch stats) and eval (running stats).
// Per-column vectors are read as float4 (C % 4 == 0, 16-B aligned).
__device__ __forceinline__ float4 ld4_or(const float* p, int64_t c, float dflt) {
  return p ? ld4(p + c) : make_float4(dflt, dflt, dflt, dflt);
}

__global__ __launch_bounds__(256) void bn_apply_k(const float* __restrict__ x, int64_t M, int64_t C,
                                                  const float* __restrict__ mean,
                                                  const float* __restrict__ invstd,
                                                  const float* __restrict__ gamma,
                                                  const float* __restrict__ beta, int hardtanh,
                                                  float* __restrict__ y) {
  const int64_t n4 = M * C / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const int64_t c = (i * 4) % C;
    const float4 xv = ld4(x + i * 4), mv = ld4(mean + c), iv = ld4(invstd + c);
    const float4 gv = ld4_or(gamma, c, 1.f), bv = ld4_or(beta, c, 0.f);
    float v[4] = {fmaf((xv.x - mv.x) * iv.x, gv.x, bv.x), fmaf((xv.y - mv.y) * iv.y, gv.y, bv.y),
                  fmaf((xv.z - mv.z) * iv.z, gv.z, bv.z), fmaf((xv.w - mv.w) * iv.w, gv.w, bv.w)};
    if (hardtanh) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = fminf(fmaxf(v[j], -1.f), 1.f);
    }
    *reinterpret_cast<float4*>(y + i * 4) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

__global__ __launch_bounds__(256) void bn_bwd_final_k(const double* __restrict__ p0,
                                                      const double* __restrict__ p1, int64_t C, int64_t R,
                                                      float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                      float* __restrict__ k0, float* __restrict__ k1) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  double s = 0.0, s2 = 0.0;
  for (int64_t r = 0; r < R; ++r) {
    s += p0[r * C + c];
    s2 += p1[r * C + c];
  }
  if (dbeta) dbeta[c] = (float)s;
  if (dgamma) dgamma[c] = (float)s2;
  k0[c] = (float)s;
  k1[c] = (float)s2;
}

__global__ __launch_bounds__(256) void bn_bwd_apply_k(const float* __restrict__ x, const float* __restrict__ dy,
                                                      int64_t M, int64_t C, const float* __restrict__ mean,
                                                      const float* __restrict__ invstd,
                                                      const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, int hardtanh,
                                                      const float* __restrict__ sg,
                                                      const float* __restrict__ sgx,
                                                      float* __restrict__ dx) {
  const int64_t n4 = M * C / 4;
  const float inv_n = 1.f / (float)M;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const int64_t c = (i * 4) % C;
    const float4 xv = ld4(x + i * 4), gv = ld4(dy + i * 4);
    const float4 mv = ld4(mean + c), iv = ld4(invstd + c), s0 = ld4(sg + c), s1 = ld4(sgx + c);
    const float4 gav = ld4_or(gamma, c, 1.f), bev = ld4_or(beta, c, 0.f);
    const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, gs[4] = {gv.x, gv.y, gv.z, gv.w};
    const float ms[4] = {mv.x, mv.y, mv.z, mv.w}, is[4] = {iv.x, iv.y, iv.z, iv.w};
    const float ga[4] = {gav.x, gav.y, gav.z, gav.w}, be[4] = {bev.x, bev.y, bev.z, bev.w};
    const float a0[4] = {s0.x, s0.y, s0.z, s0.w}, a1[4] = {s1.x, s1.y, s1.z, s1.w};
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float xh = (xs[j] - ms[j]) * is[j];
      const float y = fmaf(xh, ga[j], be[j]);
      const float g = (!hardtanh || (y > -1.f && y < 1.f)) ? gs[j] : 0.f;
      o[j] = ga[j] * is[j] * (g - a0[j] * inv_n - xh * (a1[j] * inv_n));
    }
    *reinterpret_cast<float4*>(dx + i * 4) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

inline int grid_for(int64_t n) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 16384));
}

bool bn_args_ok(const float* x, int64_t M, int64_t C) {
  return x && M > 0 && C > 0 && C % 4 == 0 && aligned16(x) && bn_chunks(M) <= 65535;
}

bool vec_ok(const float* p) { return p == nullptr || aligned16(p); }

}  // namespace
}  // namespace bnn

using namespace bnn;

BNN_API int64_t bnn_bn_workspace(int64_t M, int64_t C) {
  // two double partial arrays [R][C] + two float vectors [C]
  return 2 * bn_chunks(M) * C * (int64_t)sizeof(double) + 2 * round_up(C * 4, 256);
}

BNN_API int bnn_bn_fwd_train(const float* x, int64_t M, int64_t C, const float* gamma, const float* beta,
                             float* running_mean, float* running_var, float momentum, float eps,
                             float* save_mean, float* save_invstd, float* y, int32_t hardtanh, void* work,
                             void* stream) {
  if (!bn_args_ok(x, M, C) || !save_mean || !save_invstd || !work || !vec_ok(y) ||
      (running_mean == nullptr) != (running_var == nullptr) || !vec_ok(gamma) || !vec_ok(beta) ||
      !aligned16(save_mean) || !aligned16(save_invstd)) {
    set_error("bnn_bn_fwd_train: bad arguments (M=%lld C=%lld; C must be a multiple of 4, M > 0)",
              (long long)M, (long long)C);
    return kErrInval;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t R = bn_chunks(M);
  double* p0 = reinterpret_cast<double*>(work);
  double* p1 = p0 + R * C;
  hipLaunchKernelGGL(bn_reduce_k<0>, dim3((unsigned)((C / 4 + 255) / 256), (unsigned)R), dim3(256), 0, s, x,
                     nullptr, M, C, nullptr, nullptr, nullptr, nullptr, 0, p0, p1);
  hipLaunchKernelGGL(bn_fwd_final_k, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, p0, p1, M, C, R,
                     momentum, eps, running_mean, running_var, save_mean, save_invstd);
  if (y != nullptr)   // y == NULL: statistics only (the fused apply+pack path writes no fp32 y)
    hipLaunchKernelGGL(bn_apply_k, dim3(grid_for(M * C / 4)), dim3(256), 0, s, x, M, C, save_mean, save_invstd,
                       gamma, beta, hardtanh, y);
  return check_launch("bnn_bn_fwd_train");
}

BNN_API int bnn_bn_fwd_eval(const float* x, int64_t M, int64_t C, const float* gamma, const float* beta,
                            const float* running_mean, const float* running_var, float eps, float* y,
                            int32_t hardtanh, void* work, void* stream) {
  if (!bn_args_ok(x, M, C) || !running_mean || !running_var || !y || !work || !aligned16(y) ||
      !aligned16(running_mean) || !vec_ok(gamma) || !vec_ok(beta)) {
    set_error("bnn_bn_fwd_eval: bad arguments");
    return kErrInval;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* istd = reinterpret_cast<float*>(work);
  hipLaunchKernelGGL(bn_invstd_k, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, running_var, istd, C, eps);
  hipLaunchKernelGGL(bn_apply_k, dim3(grid_for(M * C / 4)), dim3(256), 0, s, x, M, C, running_mean, istd, gamma,
                     beta, hardtanh, y);
  return check_launch("bnn_bn_fwd_eval");
}

BNN_API int bnn_bn_bwd(const float* x, const float* dy, int64_t M, int64_t C, const float* gamma,
                       const float* beta, const float* save_mean, const float* save_invstd, int32_t hardtanh,
                       float* dx, float* dgamma, float* dbeta, void* work, void* stream) {
  if (!bn_args_ok(x, M, C) || !dy || !aligned16(dy) || !save_mean || !save_invstd || !work ||
      (dx && !aligned16(dx)) || !vec_ok(gamma) || !vec_ok(beta) || !aligned16(save_mean) ||
      !aligned16(save_invstd)) {
    set_error("bnn_bn_bwd: bad arguments");
    return kErrInval;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t R = bn_chunks(M);
  double* p0 = reinterpret_cast<double*>(work);
  double* p1 = p0 + R * C;
  float* k0 = reinterpret_cast<float*>(p1 + R * C);
  float* k1 = reinterpret_cast<float*>(reinterpret_cast<char*>(k0) + round_up(C * 4, 256));
  hipLaunchKernelGGL(bn_reduce_k<1>, dim3((unsigned)((C / 4 + 255) / 256), (unsigned)R), dim3(256), 0, s, x, dy,
                     M, C, save_mean, save_invstd, gamma, beta, hardtanh, p0, p1);
  hipLaunchKernelGGL(bn_bwd_final_k, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, p0, p1, C, R, dgamma,
                     dbeta, k0, k1);
  if (dx) {
    hipLaunchKernelGGL(bn_bwd_apply_k, dim3(grid_for(M * C / 4)), dim3(256), 0, s, x, dy, M, C, save_mean,
                       save_invstd, gamma, beta, hardtanh, k0, k1, dx);
  }
  return check_launch("bnn_bn_bwd");
}
