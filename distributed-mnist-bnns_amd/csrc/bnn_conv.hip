// Binary conv2d (NCHW fp32 in/out), im2col-free: BinarizeConv2d.forward
// (models/binarized_modules.py:93-107) and its autograd.
//
// Forward: every output element gathers its receptive field directly from the NCHW input (zero
// padding contributes 0), binarising input (when the :94 rule applies) and the latent weight on
// the fly.  Ternary x ternary sums are exact int32, so the output is bit-exact against
// F.conv2d(sign(x), sign(w)) + bias.  The MNIST-scale channel counts (Ci <= 16, Co <= 32) make
// this a latency/L2-bound kernel; the int8-MFMA implicit-GEMM form is the next step.
#include <algorithm>

#include "bnn_common.h"

namespace bnn {
namespace {

struct ConvShape {
  int64_t N, C, H, W, Co, KH, KW, OH, OW;
  int stride, pad, dil, groups;
};

inline int grid_for(int64_t n) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 65536));
}

__global__ __launch_bounds__(256) void conv_fwd_k(const float* __restrict__ x, int binarize,
                                                  const float* __restrict__ w,
                                                  const float* __restrict__ bias,
                                                  float* __restrict__ y, ConvShape s) {
  const int64_t total = s.N * s.Co * s.OH * s.OW;
  const int64_t cig = s.C / s.groups, cog = s.Co / s.groups;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    const int64_t ow = e % s.OW, oh = (e / s.OW) % s.OH, co = (e / (s.OW * s.OH)) % s.Co,
                  n = e / (s.OW * s.OH * s.Co);
    const int64_t g = co / cog;
    int iacc = 0;
    float facc = 0.f;
    for (int64_t ci = 0; ci < cig; ++ci) {
      const float* xp = x + ((n * s.C + g * cig + ci) * s.H) * s.W;
      const float* wp = w + (co * cig + ci) * s.KH * s.KW;
      for (int64_t kh = 0; kh < s.KH; ++kh) {
        const int64_t ih = oh * s.stride - s.pad + kh * s.dil;
        if (ih < 0 || ih >= s.H) continue;
        for (int64_t kw = 0; kw < s.KW; ++kw) {
          const int64_t iw = ow * s.stride - s.pad + kw * s.dil;
          if (iw < 0 || iw >= s.W) continue;
          const int wb = tsign(wp[kh * s.KW + kw]);
          const float xv = xp[ih * s.W + iw];
          if (binarize)
            iacc += tsign(xv) * wb;
          else
            facc = fmaf(xv, (float)wb, facc);
        }
      }
    }
    float out = binarize ? (float)iacc : facc;
    if (bias) out += bias[co];
    y[e] = out;
  }
}

__global__ __launch_bounds__(256) void conv_bwd_data_k(const float* __restrict__ dy,
                                                       const float* __restrict__ w,
                                                       float* __restrict__ dx, ConvShape s) {
  const int64_t total = s.N * s.C * s.H * s.W;
  const int64_t cig = s.C / s.groups, cog = s.Co / s.groups;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    const int64_t iw = e % s.W, ih = (e / s.W) % s.H, c = (e / (s.W * s.H)) % s.C, n = e / (s.W * s.H * s.C);
    const int64_t g = c / cig, ci = c % cig;
    float acc = 0.f;
    for (int64_t co = g * cog; co < (g + 1) * cog; ++co) {
      const float* dyp = dy + ((n * s.Co + co) * s.OH) * s.OW;
      const float* wp = w + (co * cig + ci) * s.KH * s.KW;
      for (int64_t kh = 0; kh < s.KH; ++kh) {
        const int64_t th = ih + s.pad - kh * s.dil;
        if (th < 0 || th % s.stride != 0) continue;
        const int64_t oh = th / s.stride;
        if (oh >= s.OH) continue;
        for (int64_t kw = 0; kw < s.KW; ++kw) {
          const int64_t tw = iw + s.pad - kw * s.dil;
          if (tw < 0 || tw % s.stride != 0) continue;
          const int64_t ow = tw / s.stride;
          if (ow >= s.OW) continue;
          acc = fmaf(dyp[oh * s.OW + ow], (float)tsign(wp[kh * s.KW + kw]), acc);
        }
      }
    }
    dx[e] = acc;
  }
}

// dW (and dB) partial sums: element e < nw is a weight (co, ci, kh, kw), e >= nw a bias co.
// blockIdx.y = chunk of the batch; partials in double, reduced in a fixed order afterwards.
__global__ __launch_bounds__(256) void conv_bwd_filter_k(const float* __restrict__ dy,
                                                         const float* __restrict__ x, int binarize,
                                                         double* __restrict__ part, int64_t nelem,
                                                         int64_t nchunks, ConvShape s, int with_bias) {
  const int64_t nw = s.Co * (s.C / s.groups) * s.KH * s.KW;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nelem) return;
  const int64_t chunk = blockIdx.y;
  const int64_t n0 = chunk * s.N / nchunks, n1 = (chunk + 1) * s.N / nchunks;
  const int64_t cig = s.C / s.groups, cog = s.Co / s.groups;
  double acc = 0.0;
  if (e < nw) {
    const int64_t kw = e % s.KW, kh = (e / s.KW) % s.KH, ci = (e / (s.KW * s.KH)) % cig,
                  co = e / (s.KW * s.KH * cig);
    const int64_t c = (co / cog) * cig + ci;
    for (int64_t n = n0; n < n1; ++n) {
      const float* dyp = dy + ((n * s.Co + co) * s.OH) * s.OW;
      const float* xp = x + ((n * s.C + c) * s.H) * s.W;
      float part_acc = 0.f;
      for (int64_t oh = 0; oh < s.OH; ++oh) {
        const int64_t ih = oh * s.stride - s.pad + kh * s.dil;
        if (ih < 0 || ih >= s.H) continue;
        for (int64_t ow = 0; ow < s.OW; ++ow) {
          const int64_t iw = ow * s.stride - s.pad + kw * s.dil;
          if (iw < 0 || iw >= s.W) continue;
          const float xv = xp[ih * s.W + iw];
          part_acc = fmaf(dyp[oh * s.OW + ow], binarize ? (float)tsign(xv) : xv, part_acc);
        }
      }
      acc += (double)part_acc;
    }
  } else if (with_bias) {
    const int64_t co = e - nw;
    for (int64_t n = n0; n < n1; ++n) {
      const float* dyp = dy + ((n * s.Co + co) * s.OH) * s.OW;
      float part_acc = 0.f;
      for (int64_t p = 0; p < s.OH * s.OW; ++p) part_acc += dyp[p];
      acc += (double)part_acc;
    }
  }
  part[chunk * nelem + e] = acc;
}

__global__ __launch_bounds__(256) void conv_bwd_filter_reduce_k(const double* __restrict__ part,
                                                                int64_t nelem, int64_t nchunks,
                                                                int64_t nw, float* __restrict__ dw,
                                                                float* __restrict__ db) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nelem) return;
  double acc = 0.0;
  for (int64_t c = 0; c < nchunks; ++c) acc += part[c * nelem + e];
  if (e < nw)
    dw[e] = (float)acc;
  else if (db)
    db[e - nw] = (float)acc;
}

bool make_shape(int64_t N, int64_t C, int64_t H, int64_t W, int64_t Co, int64_t KH, int64_t KW,
                int32_t stride, int32_t pad, int32_t dil, int32_t groups, ConvShape* s) {
  if (N < 0 || C <= 0 || H <= 0 || W <= 0 || Co <= 0 || KH <= 0 || KW <= 0 || stride <= 0 || pad < 0 ||
      dil <= 0 || groups <= 0 || C % groups != 0 || Co % groups != 0)
    return false;
  const int64_t oh = (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1;
  const int64_t ow = (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1;
  if (oh <= 0 || ow <= 0) return false;
  *s = ConvShape{N, C, H, W, Co, KH, KW, oh, ow, stride, pad, dil, groups};
  return true;
}

int64_t filter_chunks(int64_t N, int64_t nelem) {
  const int64_t blocks_e = (nelem + 255) / 256;
  const int64_t want = (2048 + blocks_e - 1) / blocks_e;
  return std::max<int64_t>(1, std::min<int64_t>({want, N, (int64_t)65535}));
}

}  // namespace
}  // namespace bnn

using namespace bnn;

BNN_API int bnn_conv2d_fwd(const float* x, int32_t binarize_input, const float* w_latent,
                           const float* bias, float* y, int64_t N, int64_t C, int64_t H, int64_t W,
                           int64_t Co, int64_t KH, int64_t KW, int32_t stride, int32_t pad,
                           int32_t dil, int32_t groups, void* stream) {
  ConvShape s;
  if (!x || !w_latent || !y || !make_shape(N, C, H, W, Co, KH, KW, stride, pad, dil, groups, &s)) {
    set_error("bnn_conv2d_fwd: bad arguments");
    return kErrInval;
  }
  const int64_t total = N * Co * s.OH * s.OW;
  if (total == 0) return 0;
  hipLaunchKernelGGL(conv_fwd_k, dim3(grid_for(total)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), x, binarize_input, w_latent, bias, y, s);
  return check_launch("bnn_conv2d_fwd");
}

BNN_API int bnn_conv2d_bwd_data(const float* dy, const float* w_latent, float* dx, int64_t N,
                                int64_t C, int64_t H, int64_t W, int64_t Co, int64_t KH, int64_t KW,
                                int32_t stride, int32_t pad, int32_t dil, int32_t groups, void* stream) {
  ConvShape s;
  if (!dy || !w_latent || !dx || !make_shape(N, C, H, W, Co, KH, KW, stride, pad, dil, groups, &s)) {
    set_error("bnn_conv2d_bwd_data: bad arguments");
    return kErrInval;
  }
  const int64_t total = N * C * H * W;
  if (total == 0) return 0;
  hipLaunchKernelGGL(conv_bwd_data_k, dim3(grid_for(total)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), dy, w_latent, dx, s);
  return check_launch("bnn_conv2d_bwd_data");
}

BNN_API int64_t bnn_conv2d_bwd_filter_workspace(int64_t N, int64_t C, int64_t Co, int64_t KH,
                                                int64_t KW, int32_t groups) {
  if (groups <= 0 || C % groups != 0) return 0;
  const int64_t nelem = Co * (C / groups) * KH * KW + Co;
  return filter_chunks(std::max<int64_t>(N, 1), nelem) * nelem * (int64_t)sizeof(double);
}

BNN_API int bnn_conv2d_bwd_filter(const float* dy, const float* x, int32_t binarize_input, float* dw,
                                  float* db, void* work, int64_t N, int64_t C, int64_t H, int64_t W,
                                  int64_t Co, int64_t KH, int64_t KW, int32_t stride, int32_t pad,
                                  int32_t dil, int32_t groups, void* stream) {
  ConvShape s;
  if (!dy || !x || !dw || !work || !make_shape(N, C, H, W, Co, KH, KW, stride, pad, dil, groups, &s)) {
    set_error("bnn_conv2d_bwd_filter: bad arguments");
    return kErrInval;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t nw = Co * (C / groups) * KH * KW;
  const int64_t nelem = nw + Co;
  const int64_t nchunks = filter_chunks(std::max<int64_t>(N, 1), nelem);
  double* part = reinterpret_cast<double*>(work);
  if (N == 0) {
    (void)hipMemsetAsync(part, 0, nchunks * nelem * sizeof(double), st);
  } else {
    hipLaunchKernelGGL(conv_bwd_filter_k, dim3((unsigned)((nelem + 255) / 256), (unsigned)nchunks),
                       dim3(256), 0, st, dy, x, binarize_input, part, nelem, nchunks, s, db != nullptr);
  }
  hipLaunchKernelGGL(conv_bwd_filter_reduce_k, dim3((unsigned)((nelem + 255) / 256)), dim3(256), 0, st,
                     part, nelem, nchunks, nw, dw, db);
  return check_launch("bnn_conv2d_bwd_filter");
}
