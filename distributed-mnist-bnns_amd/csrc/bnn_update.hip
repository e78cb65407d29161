// Subsystem (3) helpers: Hardtanh STE mask and the fused latent-weight update.
//
// The reference's caller protocol (mnist-dist2.py:131-137) is
//     p.data.copy_(p.org); optimizer.step(); p.org.copy_(p.data.clamp_(-1,1))
// around torch.optim.Adam (mnist-dist2.py:91).  bnn_adam_clamp applies Adam to the latent
// weight and clamps it in one HBM pass (7 fp32 streams: p, g, m, v read; p, m, v written).
#include <algorithm>
#include <cmath>

#include "bnn_common.h"

namespace bnn {
namespace {

__global__ __launch_bounds__(256) void hardtanh_bwd_k(const float* __restrict__ x,
                                                      const float* __restrict__ g,
                                                      float* __restrict__ out, int64_t n, int vec) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  auto f = [](float xv, float gv) { return (xv > -1.f && xv < 1.f) ? gv : 0.f; };
  int64_t tail = 0;
  if (vec) {
    const int64_t n4 = n / 4;
    for (int64_t i = i0; i < n4; i += stride) {
      const float4 xv = reinterpret_cast<const float4*>(x)[i];
      const float4 gv = reinterpret_cast<const float4*>(g)[i];
      reinterpret_cast<float4*>(out)[i] =
          make_float4(f(xv.x, gv.x), f(xv.y, gv.y), f(xv.z, gv.z), f(xv.w, gv.w));
    }
    tail = n4 * 4;
  }
  for (int64_t i = tail + i0; i < n; i += stride) out[i] = f(x[i], g[i]);
}

// Adam + clamp over a flat tensor (math: adam_elem in bnn_common.h).
__global__ __launch_bounds__(256) void adam_clamp_k(float* __restrict__ p, int64_t n, AdamArgs a0) {
  const AdamArgs a = adam_resolve(a0);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float mi = a.m[i], vi = a.v[i];
    p[i] = adam_elem(p[i], a.g[i], mi, vi, a);
    a.m[i] = mi;
    a.v[i] = vi;
  }
}

}  // namespace

// torch computes the bias corrections as Python floats (double) from the step count.
void adam_bias_correction(float lr, float beta1, float beta2, int64_t step, float* step_size, float* bc2_sqrt) {
  const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
  const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
  *step_size = (float)((double)lr / bc1);
  *bc2_sqrt = (float)std::sqrt(bc2);
}

namespace {

inline int grid_for(int64_t n) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
}

}  // namespace
}  // namespace bnn

using namespace bnn;

BNN_API int bnn_hardtanh_bwd(const float* x, const float* g, float* out, int64_t n, void* stream) {
  if (!x || !g || !out || n < 0) {
    set_error("bnn_hardtanh_bwd: bad arguments");
    return kErrInval;
  }
  if (n == 0) return 0;
  const int vec = aligned16(x) && aligned16(g) && aligned16(out);
  hipLaunchKernelGGL(hardtanh_bwd_k, dim3(grid_for(n / 4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), x, g, out, n, vec);
  return check_launch("bnn_hardtanh_bwd");
}

BNN_API int bnn_adam_clamp(float* p, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                           float lr, float beta1, float beta2, float eps, int64_t step,
                           float grad_scale, int32_t clamp, void* stream) {
  if (n < 0 || (n > 0 && (!p || !grad || !exp_avg || !exp_avg_sq)) || step < 1) {   // n == 0: nothing to do
    set_error("bnn_adam_clamp: bad arguments");
    return kErrInval;
  }
  if (n == 0) return 0;
  float step_size, bc2_sqrt;
  adam_bias_correction(lr, beta1, beta2, step, &step_size, &bc2_sqrt);
  const AdamArgs a{grad, exp_avg, exp_avg_sq, beta1, beta2, eps, step_size, bc2_sqrt, grad_scale, clamp};
  hipLaunchKernelGGL(adam_clamp_k, dim3(grid_for(n)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), p, n, a);
  return check_launch("bnn_adam_clamp");
}

BNN_API int bnn_adam_clamp_sched(float* p, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                                 float beta1, float beta2, float eps, const float* sched, const int64_t* ctr,
                                 float grad_scale, int32_t clamp, void* stream) {
  if (n < 0 || (n > 0 && (!p || !grad || !exp_avg || !exp_avg_sq)) || !sched || !ctr) {
    set_error("bnn_adam_clamp_sched: bad arguments");
    return kErrInval;
  }
  if (n == 0) return 0;
  AdamArgs a{grad, exp_avg, exp_avg_sq, beta1, beta2, eps, 0.f, 1.f, grad_scale, clamp};
  a.sched = sched;
  a.ctr = ctr;
  hipLaunchKernelGGL(adam_clamp_k, dim3(grid_for(n)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), p, n, a);
  return check_launch("bnn_adam_clamp_sched");
}

// Multi-tensor form: up to ADAM_MT tensors (the small parameters -- biases, BatchNorm affine
// parameters, the head -- each of which would otherwise be its own launch of a few microseconds)
// in ONE launch, blockIdx.y = tensor; per-tensor bias corrections (or the device-step table).
namespace bnn {
namespace {
constexpr int ADAM_MT = 16;
struct AdamMulti {
  float* p[ADAM_MT];
  const float* g[ADAM_MT];
  float* m[ADAM_MT];
  float* v[ADAM_MT];
  int64_t n[ADAM_MT];
  float step_size[ADAM_MT], bc2_sqrt[ADAM_MT];
  int clamp[ADAM_MT];
  float b1, b2, eps, gscale;
  const float* sched;
  const int64_t* ctr;
};

__global__ __launch_bounds__(256) void adam_clamp_multi_k(AdamMulti am) {
  const int j = blockIdx.y;
  AdamArgs a{am.g[j], am.m[j], am.v[j], am.b1, am.b2, am.eps, am.step_size[j], am.bc2_sqrt[j], am.gscale,
             am.clamp[j]};
  a.sched = am.sched;
  a.ctr = am.ctr;
  a = adam_resolve(a);
  float* __restrict__ p = am.p[j];
  const int64_t n = am.n[j], stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float mi = a.m[i], vi = a.v[i];
    p[i] = adam_elem(p[i], a.g[i], mi, vi, a);
    a.m[i] = mi;
    a.v[i] = vi;
  }
}
}  // namespace
}  // namespace bnn

BNN_API int bnn_adam_clamp_multi(int32_t count, float* const* p, const float* const* grad, float* const* exp_avg,
                                 float* const* exp_avg_sq, const int64_t* n, const int64_t* step,
                                 const int32_t* clamp, float lr, float beta1, float beta2, float eps,
                                 const float* sched, const int64_t* ctr, float grad_scale, void* stream) {
  if (count < 0 || count > ADAM_MT || (count > 0 && (!p || !grad || !exp_avg || !exp_avg_sq || !n || !step || !clamp)) ||
      ((sched == nullptr) != (ctr == nullptr))) {
    set_error("bnn_adam_clamp_multi: bad arguments (count %d, at most %d tensors per launch)", count, ADAM_MT);
    return kErrInval;
  }
  AdamMulti am{};
  int64_t nmax = 0;
  int k = 0;
  for (int j = 0; j < count; ++j) {
    if (n[j] < 0 || (n[j] > 0 && (!p[j] || !grad[j] || !exp_avg[j] || !exp_avg_sq[j])) || (!sched && step[j] < 1)) {
      set_error("bnn_adam_clamp_multi: bad tensor %d", j);
      return kErrInval;
    }
    if (n[j] == 0) continue;
    am.p[k] = p[j], am.g[k] = grad[j], am.m[k] = exp_avg[j], am.v[k] = exp_avg_sq[j], am.n[k] = n[j];
    am.clamp[k] = clamp[j];
    if (sched) {
      am.step_size[k] = 0.f, am.bc2_sqrt[k] = 1.f;     // from the device-step table
    } else {
      adam_bias_correction(lr, beta1, beta2, step[j], &am.step_size[k], &am.bc2_sqrt[k]);
    }
    nmax = std::max(nmax, n[j]);
    ++k;
  }
  if (k == 0) return 0;
  am.b1 = beta1, am.b2 = beta2, am.eps = eps, am.gscale = grad_scale, am.sched = sched, am.ctr = ctr;
  const unsigned gx = (unsigned)std::min<int64_t>((nmax + 255) / 256, 1024);
  hipLaunchKernelGGL(adam_clamp_multi_k, dim3(gx, (unsigned)k), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), am);
  return check_launch("bnn_adam_clamp_multi");
}

BNN_API int bnn_adam_schedule(float lr, float beta1, float beta2, int64_t step0, int64_t n, float* out) {
  if (!out || n < 0 || step0 < 1) {
    set_error("bnn_adam_schedule: bad arguments");
    return kErrInval;
  }
  for (int64_t i = 0; i < n; ++i) adam_bias_correction(lr, beta1, beta2, step0 + i, &out[2 * i], &out[2 * i + 1]);
  return 0;
}

namespace bnn {
namespace {
__global__ void counter_add_k(int64_t* ctr, int64_t v) {
  if (threadIdx.x == 0) ctr[0] += v;
}
}  // namespace
}  // namespace bnn

BNN_API int bnn_counter_add(int64_t* ctr, int64_t v, void* stream) {
  if (!ctr) {
    set_error("bnn_counter_add: null counter");
    return kErrInval;
  }
  hipLaunchKernelGGL(counter_add_k, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), ctr, v);
  return check_launch("bnn_counter_add");
}
