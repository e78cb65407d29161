// Binary conv2d (NCHW fp32 in/out), im2col-free: BinarizeConv2d.forward
// (models/binarized_modules.py:93-107) and its autograd.
//
// Forward: every output element gathers its receptive field directly from the NCHW input (zero
// padding contributes 0), binarising input (when the :94 rule applies) and the latent weight on
// the fly.  Ternary x ternary sums are exact int32, so the output is bit-exact against
// F.conv2d(sign(x), sign(w)) + bias.  The MNIST-scale channel counts (Ci <= 16, Co <= 32) make
// this a latency/L2-bound kernel; the int8-MFMA implicit-GEMM form is the next step.
#include <algorithm>

#include <type_traits>

#include "bnn_common.h"

#include <map>
#include <mutex>
#include <vector>
#include "bnn_bn2d.h"

#include <cstring>
#include <vector>

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


// ------------------------------------------------------------------------------------------------
// LDS-tiled fast path (groups == 1, stride == 1, dilation == 1, pad <= K-1, one sample's planes
// fit in LDS -- the MNIST-scale convolutions of the build CNN).  One workgroup per sample (fwd,
// bwd_data) or per chunk of samples (bwd_filter); weights and the zero-padded sample staged in LDS
// once; each thread keeps all output channels of its pixel in registers.
//  * forward, binarised input: ternary activations and weights packed 4 channels per int32 word,
//    v_dot4c_i32_i8 -> exact integer sums (bit-exact like the generic kernel);
//  * forward, fp32 input (the C == 3 rule): fp32 FMAs;
//  * backward data: fp32 dY x sign(W) FMAs; backward filter: fp32 dY x x_used FMAs, per-workgroup
//    partial sums reduced in double in a fixed order.
constexpr int TILE_T = 256;

struct TileGeo {
  int C, H, W, Co, KH, KW, OH, OW, pad, Hp, Wp, C4;
};

constexpr int64_t kMaxTileLds = 160 * 1024;   // a single workgroup may own the CU's whole LDS

inline bool tile_geom_ok(const ConvShape& s) {
  return s.groups == 1 && s.stride == 1 && s.dil == 1 && s.pad <= s.KH - 1 && s.pad <= s.KW - 1 &&
         s.Co <= 64 && s.C <= 64;
}

inline int pick_co(int64_t co) { return co <= 8 ? 8 : co <= 16 ? 16 : co <= 32 ? 32 : 64; }

// Dynamic LDS bytes of each tiled kernel (must match the carve-up inside the kernels).
inline int64_t fwd_tile_lds(const ConvShape& s, bool bin) {
  const int64_t Hp = s.H + 2 * s.pad, Wp = s.W + 2 * s.pad, C4 = (s.C + 3) / 4, CO = pick_co(s.Co);
  return bin ? (s.KH * s.KW * C4 * CO + Hp * Wp * C4) * 4 : (s.KH * s.KW * s.C * CO + s.C * Hp * Wp) * 4;
}
inline int64_t bwd_data_tile_lds(const ConvShape& s) {
  const int64_t CI = pick_co(s.C);
  return (s.KH * s.KW * s.Co * CI + s.Co * (s.OH + 2 * (s.KH - 1)) * (s.OW + 2 * (s.KW - 1))) * 4;
}
inline int64_t filter_tile_lds(const ConvShape& s) {
  return ((s.H + 2 * s.pad) * (s.W + 2 * s.pad) * s.C + s.OH * s.OW * pick_co(s.Co)) * 4;
}

template <typename K>
inline void allow_lds(K kernel, int64_t bytes) {
  if (bytes > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)bytes);
}

inline TileGeo geo(const ConvShape& s) {
  return TileGeo{(int)s.C, (int)s.H, (int)s.W, (int)s.Co, (int)s.KH, (int)s.KW, (int)s.OH, (int)s.OW, s.pad,
                 (int)(s.H + 2 * s.pad), (int)(s.W + 2 * s.pad), (int)((s.C + 3) / 4)};
}

template <int CO>
__global__ __launch_bounds__(TILE_T) void conv_fwd_bin_tile_k(const float* __restrict__ x,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ bias,
                                                              float* __restrict__ y, TileGeo g) {
  extern __shared__ __attribute__((aligned(16))) int lds[];
  int* ws = lds;                                   // [KH][KW][C4][CO] packed signs
  int* xs = lds + g.KH * g.KW * g.C4 * CO;         // [Hp][Wp][C4] packed signs
  const int n = blockIdx.x, t = threadIdx.x;
  const int nw = g.KH * g.KW * g.C4 * CO, nx = g.Hp * g.Wp * g.C4;
  for (int i = t; i < nw; i += TILE_T) {
    const int co = i % CO, cg = (i / CO) % g.C4, kk = i / (CO * g.C4);
    const int kh = kk / g.KW, kw = kk % g.KW;
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // clamped, unconditional loads: the four batch
      const int ci = min(4 * cg + j, g.C - 1);
      v[j] = w[((min(co, g.Co - 1) * g.C + ci) * g.KH + kh) * g.KW + kw];
    }
    int word = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (co < g.Co && 4 * cg + j < g.C) word |= (tsign(v[j]) & 255) << (8 * j);
    ws[i] = word;
  }
  for (int i = t; i < nx; i += TILE_T) xs[i] = 0;
  __syncthreads();
  int8_t* xs8 = reinterpret_cast<int8_t*>(xs);
  const float* xn = x + (int64_t)n * g.C * g.H * g.W;
  const int nin = g.C * g.H * g.W;
  for (int i0 = t; i0 < nin; i0 += 4 * TILE_T) {   // coalesced over the NCHW plane, 4 loads in flight
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = xn[min(i0 + j * TILE_T, nin - 1)];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = i0 + j * TILE_T;
      const int iw = i % g.W, ih = (i / g.W) % g.H, c = i / (g.W * g.H);
      if (i < nin) xs8[((ih + g.pad) * g.Wp + (iw + g.pad)) * g.C4 * 4 + c] = (int8_t)tsign(v[j]);
    }
  }
  __syncthreads();
  for (int p = t; p < g.OH * g.OW; p += TILE_T) {
    const int oh = p / g.OW, ow = p % g.OW;
    int acc[CO];
#pragma unroll
    for (int co = 0; co < CO; ++co) acc[co] = 0;
    for (int kh = 0; kh < g.KH; ++kh)
      for (int kw = 0; kw < g.KW; ++kw) {
        const int* xp = xs + ((oh + kh) * g.Wp + (ow + kw)) * g.C4;
        const int* wp = ws + (kh * g.KW + kw) * g.C4 * CO;
        for (int cg = 0; cg < g.C4; ++cg) {
          const int xv = xp[cg];
#pragma unroll
          for (int co = 0; co < CO; ++co) acc[co] = __builtin_amdgcn_sdot4(xv, wp[cg * CO + co], acc[co], false);
        }
      }
    float* yp = y + (int64_t)n * g.Co * g.OH * g.OW + p;
#pragma unroll
    for (int co = 0; co < CO; ++co)
      if (co < g.Co) yp[(int64_t)co * g.OH * g.OW] = (float)acc[co] + (bias ? bias[co] : 0.f);
  }
}

// Single-channel binary input (the BinCNN's first layer): 4 kw taps per dot4 instead of one useful
// byte in four.  Input signs as bytes [Hp][Wq] (Wq = round_up(Wp, 4), zero halo, 16 slack bytes),
// weights [KH][KWG][CO] words holding taps 4g..4g+3 of one row (zero beyond KW).  A pixel's
// window of row kh starts at byte b = (oh+kh)*Wq + ow: the KWG+1 dwords from b/4 and
// v_alignbyte give its taps in order; bytes past KW meet zero weight bytes.  Integer sums, so
// bit-identical to conv_fwd_bin_tile_k.
// OT = float: y = sum + bias; int8_t / int16_t (bnn_conv2d_fwd_q): the exact sum alone, the bias
// added by the consumer (fl(I + bias) = the fp32 value).
template <typename OT>
__device__ __forceinline__ OT conv_out(int acc, const float* bias, int co) {
  if constexpr (std::is_same<OT, float>::value) return (float)acc + (bias ? bias[co] : 0.f);
  else return (OT)acc;
}

template <int CO, int KWG, typename OT = float>
__global__ __launch_bounds__(TILE_T) void conv_fwd_bin_c1_k(const float* __restrict__ x,
                                                            const float* __restrict__ w,
                                                            const float* __restrict__ bias,
                                                            OT* __restrict__ y, TileGeo g, int Wq) {
  extern __shared__ __attribute__((aligned(16))) int lds[];
  int* ws = lds;                                   // [KH][KWG][CO]
  int* xw = lds + g.KH * KWG * CO;                 // [Hp][Wq / 4] words of sign bytes
  const int n = blockIdx.x, t = threadIdx.x;
  const int nw = g.KH * KWG * CO, nxw = (g.Hp * Wq + 16) / 4;
  for (int i = t; i < nw; i += TILE_T) {
    const int co = i % CO, r = i / CO, kg = r % KWG, kh = r / KWG;
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)   // clamped, unconditional: the loads batch
      v[j] = w[(min(co, g.Co - 1) * g.KH + kh) * g.KW + min(4 * kg + j, g.KW - 1)];
    int word = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (co < g.Co && 4 * kg + j < g.KW) word |= (tsign(v[j]) & 255) << (8 * j);
    ws[i] = word;
  }
  for (int i = t; i < nxw; i += TILE_T) xw[i] = 0;
  __syncthreads();
  int8_t* xb = reinterpret_cast<int8_t*>(xw);
  const float* xn = x + (int64_t)n * g.H * g.W;
  const int nin = g.H * g.W;
  for (int i0 = t; i0 < nin; i0 += 4 * TILE_T) {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = xn[min(i0 + j * TILE_T, nin - 1)];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = i0 + j * TILE_T, ih = i / g.W, iw = i - ih * g.W;
      if (i < nin) xb[(ih + g.pad) * Wq + iw + g.pad] = (int8_t)tsign(v[j]);
    }
  }
  __syncthreads();
  for (int p = t; p < g.OH * g.OW; p += TILE_T) {
    const int oh = p / g.OW, ow = p - oh * g.OW;
    int acc[CO];
#pragma unroll
    for (int co = 0; co < CO; ++co) acc[co] = 0;
    for (int kh = 0; kh < g.KH; ++kh) {
      const int b = (oh + kh) * Wq + ow, sh = b & 3;
      const int* src = xw + (b >> 2);
      int d[KWG + 1];
#pragma unroll
      for (int k = 0; k <= KWG; ++k) d[k] = src[k];
      const int* wr = ws + kh * KWG * CO;
#pragma unroll
      for (int kg = 0; kg < KWG; ++kg) {
        const int xv = (int)__builtin_amdgcn_alignbyte((unsigned)d[kg + 1], (unsigned)d[kg], (unsigned)sh);
#pragma unroll
        for (int co = 0; co < CO; ++co) acc[co] = __builtin_amdgcn_sdot4(xv, wr[kg * CO + co], acc[co], false);
      }
    }
    OT* yp = y + (int64_t)n * g.Co * g.OH * g.OW + p;
#pragma unroll
    for (int co = 0; co < CO; ++co)
      if (co < g.Co) yp[(int64_t)co * g.OH * g.OW] = conv_out<OT>(acc[co], bias, co);
  }
}

template <int CO>
__global__ __launch_bounds__(TILE_T) void conv_fwd_f32_tile_k(const float* __restrict__ x,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ bias,
                                                              float* __restrict__ y, TileGeo g) {
  extern __shared__ __attribute__((aligned(16))) float ldsf[];
  float* ws = ldsf;                                // [KH][KW][C][CO] signs
  float* xs = ldsf + g.KH * g.KW * g.C * CO;       // [C][Hp][Wp]
  const int n = blockIdx.x, t = threadIdx.x;
  const int nw = g.KH * g.KW * g.C * CO, nx = g.C * g.Hp * g.Wp;
  for (int i = t; i < nw; i += TILE_T) {
    const int co = i % CO, ci = (i / CO) % g.C, kk = i / (CO * g.C);
    ws[i] = co < g.Co ? (float)tsign(w[((co * g.C + ci) * g.KH + kk / g.KW) * g.KW + kk % g.KW]) : 0.f;
  }
  for (int i = t; i < nx; i += TILE_T) xs[i] = 0.f;
  __syncthreads();
  const float* xn = x + (int64_t)n * g.C * g.H * g.W;
  for (int i = t; i < g.C * g.H * g.W; i += TILE_T) {
    const int iw = i % g.W, ih = (i / g.W) % g.H, c = i / (g.W * g.H);
    xs[(c * g.Hp + ih + g.pad) * g.Wp + iw + g.pad] = xn[i];
  }
  __syncthreads();
  for (int p = t; p < g.OH * g.OW; p += TILE_T) {
    const int oh = p / g.OW, ow = p % g.OW;
    float acc[CO];
#pragma unroll
    for (int co = 0; co < CO; ++co) acc[co] = 0.f;
    for (int ci = 0; ci < g.C; ++ci)
      for (int kh = 0; kh < g.KH; ++kh)
        for (int kw = 0; kw < g.KW; ++kw) {
          const float xv = xs[(ci * g.Hp + oh + kh) * g.Wp + ow + kw];
          const float* wp = ws + ((kh * g.KW + kw) * g.C + ci) * CO;
#pragma unroll
          for (int co = 0; co < CO; ++co) acc[co] = fmaf(xv, wp[co], acc[co]);
        }
    float* yp = y + (int64_t)n * g.Co * g.OH * g.OW + p;
#pragma unroll
    for (int co = 0; co < CO; ++co)
      if (co < g.Co) yp[(int64_t)co * g.OH * g.OW] = acc[co] + (bias ? bias[co] : 0.f);
  }
}

// dX[ci][ih][iw] = sum_{co,kh,kw} dY[co][ih+pad-kh][iw+pad-kw] * sign(W[co][ci][kh][kw]).
template <int CI>
__global__ __launch_bounds__(TILE_T) void conv_bwd_data_tile_k(const float* __restrict__ dy,
                                                               const float* __restrict__ w,
                                                               float* __restrict__ dx, TileGeo g) {
  extern __shared__ __attribute__((aligned(16))) float ldsf[];
  const int PH = g.KH - 1, PW = g.KW - 1;
  const int OHp = g.OH + 2 * PH, OWp = g.OW + 2 * PW;
  float* ws = ldsf;                                // [KH][KW][Co][CI] signs
  float* ds = ldsf + g.KH * g.KW * g.Co * CI;      // [Co][OHp][OWp], zero border
  const int n = blockIdx.x, t = threadIdx.x;
  const int nw = g.KH * g.KW * g.Co * CI, nd = g.Co * OHp * OWp;
  for (int i = t; i < nw; i += TILE_T) {
    const int ci = i % CI, co = (i / CI) % g.Co, kk = i / (CI * g.Co);
    ws[i] = ci < g.C ? (float)tsign(w[((co * g.C + ci) * g.KH + kk / g.KW) * g.KW + kk % g.KW]) : 0.f;
  }
  for (int i = t; i < nd; i += TILE_T) ds[i] = 0.f;
  __syncthreads();
  const float* dn = dy + (int64_t)n * g.Co * g.OH * g.OW;
  for (int i = t; i < g.Co * g.OH * g.OW; i += TILE_T) {
    const int ow = i % g.OW, oh = (i / g.OW) % g.OH, co = i / (g.OW * g.OH);
    ds[(co * OHp + oh + PH) * OWp + ow + PW] = dn[i];
  }
  __syncthreads();
  for (int p = t; p < g.H * g.W; p += TILE_T) {
    const int ih = p / g.W, iw = p % g.W;
    float acc[CI];
#pragma unroll
    for (int ci = 0; ci < CI; ++ci) acc[ci] = 0.f;
    for (int co = 0; co < g.Co; ++co)
      for (int kh = 0; kh < g.KH; ++kh)
        for (int kw = 0; kw < g.KW; ++kw) {
          // oh = ih + pad - kh  ->  padded row oh + PH
          const float dv = ds[(co * OHp + ih + g.pad - kh + PH) * OWp + iw + g.pad - kw + PW];
          const float* wp = ws + ((kh * g.KW + kw) * g.Co + co) * CI;
#pragma unroll
          for (int ci = 0; ci < CI; ++ci) acc[ci] = fmaf(dv, wp[ci], acc[ci]);
        }
    float* xp = dx + (int64_t)n * g.C * g.H * g.W + p;
#pragma unroll
    for (int ci = 0; ci < CI; ++ci)
      if (ci < g.C) xp[(int64_t)ci * g.H * g.W] = acc[ci];
  }
}

// Partial dW over a chunk of samples: thread -> (combo = (ci,kh,kw), pixel phase), CO accumulators.
// part[(blockIdx.x * nphase + phase)][co * ncombo + combo]; bias partials in part[...][CO*ncombo + co].
template <int CO>
__global__ __launch_bounds__(TILE_T) void conv_bwd_filter_tile_k(const float* __restrict__ dy,
                                                                 const float* __restrict__ x, int binarize,
                                                                 float* __restrict__ part, int64_t N,
                                                                 int spb, TileGeo g, int with_bias) {
  extern __shared__ __attribute__((aligned(16))) float ldsf[];
  float* xs = ldsf;                                // [C][Hp][Wp]
  float* ds = ldsf + g.C * g.Hp * g.Wp;            // [OH*OW][CO]
  const int ncombo = g.C * g.KH * g.KW;
  const int nphase = TILE_T / ncombo > 0 ? TILE_T / ncombo : 1;
  const int t = threadIdx.x;
  const int phase = t / ncombo, combo0 = t % ncombo;
  const int nelem = CO * ncombo + CO;
  float acc[2][CO];  // a thread may own two combos when ncombo > 256
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int co = 0; co < CO; ++co) acc[a][co] = 0.f;
  float bacc = 0.f;
  const int64_t n0 = (int64_t)blockIdx.x * spb, n1 = (n0 + spb < N) ? n0 + spb : N;
  for (int64_t n = n0; n < n1; ++n) {
    __syncthreads();
    for (int i = t; i < g.C * g.Hp * g.Wp; i += TILE_T) xs[i] = 0.f;
    __syncthreads();
    const float* xn = x + n * g.C * g.H * g.W;
    for (int i = t; i < g.C * g.H * g.W; i += TILE_T) {
      const int iw = i % g.W, ih = (i / g.W) % g.H, c = i / (g.W * g.H);
      const float v = xn[i];
      xs[(c * g.Hp + ih + g.pad) * g.Wp + iw + g.pad] = binarize ? (float)tsign(v) : v;
    }
    const float* dn = dy + n * g.Co * g.OH * g.OW;
    for (int i = t; i < CO * g.OH * g.OW; i += TILE_T) {
      const int co = i % CO, pp = i / CO;
      ds[i] = co < g.Co ? dn[(int64_t)co * g.OH * g.OW + pp] : 0.f;
    }
    __syncthreads();
    if (phase < nphase) {
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int combo = combo0 + a * TILE_T;
        if (combo >= ncombo || (a == 1 && nphase > 1)) continue;
        const int ci = combo / (g.KH * g.KW), kk = combo % (g.KH * g.KW), kh = kk / g.KW, kw = kk % g.KW;
        for (int pp = phase; pp < g.OH * g.OW; pp += nphase) {
          const int oh = pp / g.OW, ow = pp % g.OW;
          const float xv = xs[(ci * g.Hp + oh + kh) * g.Wp + ow + kw];
          const float* dp = ds + pp * CO;
#pragma unroll
          for (int co = 0; co < CO; ++co) acc[a][co] = fmaf(dp[co], xv, acc[a][co]);
        }
      }
    }
    if (with_bias && t < g.Co) {
      float s = 0.f;
      for (int pp = 0; pp < g.OH * g.OW; ++pp) s += ds[pp * CO + t];
      bacc += s;
    }
  }
  float* blk = part + (int64_t)blockIdx.x * nphase * nelem;
  if (phase < nphase) {
    float* pb = blk + (int64_t)phase * nelem;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int combo = combo0 + a * TILE_T;
      if (combo >= ncombo || (a == 1 && nphase > 1)) continue;
#pragma unroll
      for (int co = 0; co < CO; ++co) pb[co * ncombo + combo] = acc[a][co];
    }
  }
  if (t < CO) {  // the block's bias sums live in its phase-0 row; other rows' bias slots are zero
    blk[CO * ncombo + t] = (with_bias && t < g.Co) ? bacc : 0.f;
    for (int ph = 1; ph < nphase; ++ph) blk[(int64_t)ph * nelem + CO * ncombo + t] = 0.f;
  }
}

// Partials -> dW / dB in two fixed-order stages (deterministic): stage 1 sums a contiguous slice of
// the parts for 256 elements per workgroup (grid.y = slices, so the reduction is spread over the
// chip instead of one serial walk per element); stage 2 folds the <= FILTER_SLICES slice sums.
constexpr int FILTER_SLICES = 64;

inline int64_t filter_slices(int64_t nparts) { return std::min<int64_t>(std::max<int64_t>(nparts, 1), FILTER_SLICES); }

__global__ __launch_bounds__(256) void conv_filter_tile_reduce1_k(const float* __restrict__ part, int64_t nparts,
                                                                  int64_t nelem, int64_t nslices,
                                                                  double* __restrict__ slice) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nelem) return;
  const int64_t q0 = blockIdx.y * nparts / nslices, q1 = (blockIdx.y + 1) * nparts / nslices;
  double acc = 0.0;
  int64_t q = q0;
  for (; q + 4 <= q1; q += 4) {   // 4 independent loads in flight per thread
    const float v0 = part[q * nelem + e], v1 = part[(q + 1) * nelem + e];
    const float v2 = part[(q + 2) * nelem + e], v3 = part[(q + 3) * nelem + e];
    acc += (double)v0;
    acc += (double)v1;
    acc += (double)v2;
    acc += (double)v3;
  }
  for (; q < q1; ++q) acc += (double)part[q * nelem + e];
  slice[blockIdx.y * nelem + e] = acc;
}

__global__ __launch_bounds__(256) void conv_filter_tile_reduce2_k(const double* __restrict__ slice, int64_t nslices,
                                                                  int CO, int ncombo, int Co,
                                                                  float* __restrict__ dw, float* __restrict__ db) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nelem = (int64_t)CO * ncombo + CO;
  if (e >= nelem) return;
  double acc = 0.0;
  int64_t q = 0;
  for (; q + 8 <= nslices; q += 8) {   // 8 independent loads in flight; the adds stay in order
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = slice[(q + j) * nelem + e];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j];
  }
  for (; q < nslices; ++q) acc += slice[q * nelem + e];
  if (e < (int64_t)CO * ncombo) {
    const int64_t co = e / ncombo, combo = e % ncombo;
    if (co < Co) dw[co * ncombo + combo] = (float)acc;
  } else if (db) {
    const int64_t co = e - (int64_t)CO * ncombo;
    if (co < Co) db[co] = (float)acc;
  }
}

// ------------------------------------------------------------------ one-input-channel filter gradient (VALU)
// dW[co][kh][kw] = sum_{n,oh,ow} dY[n][co][oh][ow] * Xb[n][oh + kh - pad][ow + kw - pad] (+ dB = sum dY)
// for a layer with ONE input channel (the BinCNN's conv1, 16 x 1 x 5 x 5 over 28 x 28; binarized_
// modules.py:100-101 binarises its input): KH*KW MACs per dY element, 1.3 G MACs at B = 4096 -- ~20 us
// of VALU, so the pass is bound by reading dY once (205 MB), which it does with coalesced 16-B loads
// (a channel plane's 4-pixel units walked by consecutive lanes).  The bf16x3 MFMA form spent its
// time staging dY into LDS three planes at a time (106 us).  Per sample the (binarised) input plane
// sits in LDS with a zero halo, double-buffered (the next sample's plane is loaded into registers
// while this one is used); thread = (channel co = t / TPC, the units r, r + TPC, ... of its plane),
// keeping its channel's KH*KW sums and the bias sum in fp32 registers over the workgroup's samples;
// the TPC threads of a channel are folded in a fixed order into the workgroup's partial row
// (conv_filter_tile_reduce{1,2}_k, double).  Deterministic.
constexpr int C1F_T = 256, C1F_SPB = 4, C1F_PX = 4, C1F_UB = 8;

struct C1Filt {
  int H, W, OH, OW, Co, pad, XR, XW, TPC;   // XR x XW: the haloed input plane in LDS
};

template <int KH, int KW>
__global__ __launch_bounds__(C1F_T) void conv_bwd_filter_c1_k(const float* __restrict__ dy,
                                                              const float* __restrict__ x, int binarize,
                                                              float* __restrict__ part, int64_t N, C1Filt g,
                                                              int with_bias) {
  constexpr int NX = (KW + 6) / 4;   // float4 pieces of an input row a 4-pixel unit reads
  constexpr int KK = KH * KW;
  extern __shared__ __attribute__((aligned(16))) float c1s[];
  const int plane = g.XR * g.XW;
  float* red = c1s;                  // [C1F_T][KK + 1] fold buffer, aliasing the planes at the end
  const int t = threadIdx.x;
  const int co = t / g.TPC, r = t - co * g.TPC;
  const int hw = g.H * g.W, ohw = g.OH * g.OW, nu = ohw / 4, uq = g.OW / 4;
  for (int i = t; i < 2 * plane; i += C1F_T) c1s[i] = 0.f;   // zero halos (interiors rewritten per sample)
  float acc[KK], bacc = 0.f;
#pragma unroll
  for (int k = 0; k < KK; ++k) acc[k] = 0.f;
  const int64_t n0 = (int64_t)blockIdx.x * C1F_SPB, n1 = n0 + C1F_SPB < N ? n0 + C1F_SPB : N;
  float px[C1F_PX];
  auto fetch = [&](int64_t n) {   // clamped, unconditional: the loads batch
#pragma unroll
    for (int s = 0; s < C1F_PX; ++s) px[s] = x[n * hw + min(t + s * C1F_T, hw - 1)];
  };
  auto put = [&](int b) {
    for (int s = 0; s < C1F_PX; ++s) {
      const int i = t + s * C1F_T;
      if (i < hw) {
        const int ih = i / g.W, iw = i - ih * g.W;
        c1s[b * plane + (ih + g.pad) * g.XW + iw + g.pad] = binarize ? (float)tsign(px[s]) : px[s];
      }
    }
  };
  __syncthreads();
  if (n0 < n1) {
    fetch(n0);
    put(0);
  }
  for (int64_t n = n0; n < n1; ++n) {
    const int b = (int)((n - n0) & 1);
    __syncthreads();   // plane b complete; plane b ^ 1's last reader (sample n - 1) is done
    if (n + 1 < n1) fetch(n + 1);
    if (co < g.Co) {
      const float* xb = c1s + b * plane;
      const float* dn = dy + (n * g.Co + co) * (int64_t)ohw;
      // C1F_UB units' dY loads issued together (one HBM latency per batch, not per unit)
      for (int u0 = r; u0 < nu; u0 += C1F_UB * g.TPC) {
        float4 dv[C1F_UB];
#pragma unroll
        for (int i = 0; i < C1F_UB; ++i) {
          const int u = min(u0 + i * g.TPC, nu - 1);   // clamped, unconditional: the loads batch
          dv[i] = *reinterpret_cast<const float4*>(dn + 4 * u);
        }
#pragma unroll
        for (int i = 0; i < C1F_UB; ++i) {
          const int u = u0 + i * g.TPC;
          if (u >= nu) break;
          const float4 d = dv[i];
          const int oh = u / uq, ow0 = 4 * (u - oh * uq);
          bacc += (d.x + d.y) + (d.z + d.w);
#pragma unroll
          for (int kh = 0; kh < KH; ++kh) {
            float xr[4 * NX];
#pragma unroll
            for (int j = 0; j < NX; ++j) {
              const float4 v = *reinterpret_cast<const float4*>(xb + (oh + kh) * g.XW + ow0 + 4 * j);
              xr[4 * j] = v.x, xr[4 * j + 1] = v.y, xr[4 * j + 2] = v.z, xr[4 * j + 3] = v.w;
            }
#pragma unroll
            for (int kw = 0; kw < KW; ++kw) {
              float a = acc[kh * KW + kw];
              a = fmaf(d.x, xr[kw], a);
              a = fmaf(d.y, xr[kw + 1], a);
              a = fmaf(d.z, xr[kw + 2], a);
              a = fmaf(d.w, xr[kw + 3], a);
              acc[kh * KW + kw] = a;
            }
          }
        }
      }
    }
    if (n + 1 < n1) put(b ^ 1);
  }
  // fixed-order fold of a channel's TPC threads
  __syncthreads();                   // every plane read is done before red overwrites them
#pragma unroll
  for (int k = 0; k < KK; ++k) red[t * (KK + 1) + k] = acc[k];
  red[t * (KK + 1) + KK] = bacc;
  __syncthreads();
  const int64_t nelem = (int64_t)g.Co * KK + g.Co;
  float* row = part + (int64_t)blockIdx.x * nelem;
  for (int e = t; e < g.Co * (KK + 1); e += C1F_T) {
    const int c = e / (KK + 1), k = e - c * (KK + 1);
    float s = 0.f;
    for (int q = 0; q < g.TPC; ++q) s += red[(c * g.TPC + q) * (KK + 1) + k];
    if (k < KK) row[c * KK + k] = s;
    else row[(int64_t)g.Co * KK + c] = with_bias ? s : 0.f;
  }
}

// conv1's filter gradient straight from its BatchNorm2d + Hardtanh + MaxPool2d(2) backward (the
// BinCNN's first layer, mnist-dist.py:31-51 template): dY is formed per 2x2 window from the conv's
// compact output z (its exact int8 / int16 sums + bias), the pooled gradient and the batch
// statistics -- bn2_window + bn2_window_dz, the arithmetic of bn2d_bwd_apply_k -- and multiplied
// straight into the filter sums, so the fp32 dY (205 MB at B = 4096) is neither written by a
// BatchNorm pass nor re-read here.  Unit = (pooled row, 4 output columns): two output rows, two
// windows; its KH + 1 input rows are read once for both.  Otherwise as conv_bwd_filter_c1_k.
constexpr int C1BN_UB = 4;   // units per load batch (8 would leave 2 waves per SIMD: 178 VGPRs)

struct C1Bn {
  X2 z;
  const float* dyp;                                  // pooled gradient [N][Co][OH/2][OW/2]
  const float *mean, *invstd, *gamma, *beta, *sg, *sgx;
  float inv_n;
  int hardtanh;
};

template <int KH, int KW, int XF>
__global__ __launch_bounds__(C1F_T) void conv_bwd_filter_c1bn_k(C1Bn bn, const float* __restrict__ x, int binarize,
                                                                float* __restrict__ part, int64_t N, C1Filt g,
                                                                int with_bias) {
  constexpr int NX = (KW + 6) / 4;
  constexpr int KK = KH * KW;
  extern __shared__ __attribute__((aligned(16))) float c1s[];
  const int plane = g.XR * g.XW;
  float* red = c1s;
  const int t = threadIdx.x;
  const int co = t / g.TPC, r = t - co * g.TPC;
  const int hw = g.H * g.W, ohw = g.OH * g.OW, uq = g.OW / 4, nu = (g.OH / 2) * uq, pw = g.OW / 2;
  for (int i = t; i < 2 * plane; i += C1F_T) c1s[i] = 0.f;
  float acc[KK], bacc = 0.f;
#pragma unroll
  for (int k = 0; k < KK; ++k) acc[k] = 0.f;
  // this thread's channel: the normalisation and the statistics terms of its backward
  const int cc = co < g.Co ? co : 0;
  const Bn2Chan k = bn2_chan(cc, bn.mean, bn.invstd, bn.gamma, bn.beta);
  const float m0 = bn.sg[cc] * bn.inv_n, m1 = bn.sgx[cc] * bn.inv_n, sc = k.ga * k.is;
  const float zb = x2_bias<XF>(bn.z, cc);
  const int64_t n0 = (int64_t)blockIdx.x * C1F_SPB, n1 = n0 + C1F_SPB < N ? n0 + C1F_SPB : N;
  float px[C1F_PX];
  auto fetch = [&](int64_t n) {
#pragma unroll
    for (int s = 0; s < C1F_PX; ++s) px[s] = x[n * hw + min(t + s * C1F_T, hw - 1)];
  };
  auto put = [&](int b) {
    for (int s = 0; s < C1F_PX; ++s) {
      const int i = t + s * C1F_T;
      if (i < hw) {
        const int ih = i / g.W, iw = i - ih * g.W;
        c1s[b * plane + (ih + g.pad) * g.XW + iw + g.pad] = binarize ? (float)tsign(px[s]) : px[s];
      }
    }
  };
  __syncthreads();
  if (n0 < n1) {
    fetch(n0);
    put(0);
  }
  for (int64_t n = n0; n < n1; ++n) {
    const int b = (int)((n - n0) & 1);
    __syncthreads();
    if (n + 1 < n1) fetch(n + 1);
    if (co < g.Co) {
      const float* xb = c1s + b * plane;
      const int64_t zo = (n * g.Co + co) * (int64_t)ohw, po = (n * g.Co + co) * (int64_t)(ohw / 4);
      for (int u0 = r; u0 < nu; u0 += C1BN_UB * g.TPC) {
        float4 zt[C1BN_UB], zbt[C1BN_UB];
        float2 gp[C1BN_UB];
#pragma unroll
        for (int i = 0; i < C1BN_UB; ++i) {   // clamped, unconditional: the loads batch
          const int u = min(u0 + i * g.TPC, nu - 1);
          const int pr = u / uq, ow0 = 4 * (u - pr * uq);
          zt[i] = x2_ld4<XF>(bn.z, zo + (int64_t)(2 * pr) * g.OW + ow0, zb);
          zbt[i] = x2_ld4<XF>(bn.z, zo + (int64_t)(2 * pr + 1) * g.OW + ow0, zb);
          gp[i] = *reinterpret_cast<const float2*>(bn.dyp + po + (int64_t)pr * pw + ow0 / 2);
        }
#pragma unroll
        for (int i = 0; i < C1BN_UB; ++i) {
          const int u = u0 + i * g.TPC;
          if (u >= nu) break;
          const int pr = u / uq, ow0 = 4 * (u - pr * uq);
          float o0[4], o1[4];
          bn2_window_dz(bn2_window(make_float2(zt[i].x, zt[i].y), make_float2(zbt[i].x, zbt[i].y), k, bn.hardtanh),
                        gp[i].x, m0, m1, sc, bn.hardtanh, o0);
          bn2_window_dz(bn2_window(make_float2(zt[i].z, zt[i].w), make_float2(zbt[i].z, zbt[i].w), k, bn.hardtanh),
                        gp[i].y, m0, m1, sc, bn.hardtanh, o1);
          const float dt[4] = {o0[0], o0[1], o1[0], o1[1]}, db[4] = {o0[2], o0[3], o1[2], o1[3]};
          bacc += ((dt[0] + dt[1]) + (dt[2] + dt[3])) + ((db[0] + db[1]) + (db[2] + db[3]));
          float xr[KH + 1][4 * NX];
#pragma unroll
          for (int rr = 0; rr <= KH; ++rr)
#pragma unroll
            for (int j = 0; j < NX; ++j) {
              const float4 v = *reinterpret_cast<const float4*>(xb + (2 * pr + rr) * g.XW + ow0 + 4 * j);
              xr[rr][4 * j] = v.x, xr[rr][4 * j + 1] = v.y, xr[rr][4 * j + 2] = v.z, xr[rr][4 * j + 3] = v.w;
            }
#pragma unroll
          for (int kh = 0; kh < KH; ++kh)
#pragma unroll
            for (int kw = 0; kw < KW; ++kw) {
              float a = acc[kh * KW + kw];
#pragma unroll
              for (int j = 0; j < 4; ++j) a = fmaf(dt[j], xr[kh][kw + j], a);
#pragma unroll
              for (int j = 0; j < 4; ++j) a = fmaf(db[j], xr[kh + 1][kw + j], a);
              acc[kh * KW + kw] = a;
            }
        }
      }
    }
    if (n + 1 < n1) put(b ^ 1);
  }
  __syncthreads();
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) red[t * (KK + 1) + kk] = acc[kk];
  red[t * (KK + 1) + KK] = bacc;
  __syncthreads();
  const int64_t nelem = (int64_t)g.Co * KK + g.Co;
  float* row = part + (int64_t)blockIdx.x * nelem;
  for (int e = t; e < g.Co * (KK + 1); e += C1F_T) {
    const int c = e / (KK + 1), kk = e - c * (KK + 1);
    float s = 0.f;
    for (int q = 0; q < g.TPC; ++q) s += red[(c * g.TPC + q) * (KK + 1) + kk];
    if (kk < KK) row[c * KK + kk] = s;
    else row[(int64_t)g.Co * KK + c] = with_bias ? s : 0.f;
  }
}

// ------------------------------------------------------------------ f32-MFMA implicit-GEMM backward
// Both backward convolutions as implicit GEMMs on v_mfma_f32_16x16x4_f32 (exact f32 products,
// f32 accumulation: the same numerics class as the fp32 reference's sgemm, at the f32 matrix
// rate).  Operands are gathered from LDS images of one sample at a time (no im2col in HBM);
// each workgroup walks IPB samples so the staged weights / accumulators amortise.
//   16x16x4 lane map: A[i = l&15][k = l>>4], B[k = l>>4][j = l&15]; D col = l&15, row = 4*(l>>4)+r.
// floor(i / d) for the staging loops through a float reciprocal: exact while i < 2^20 (the
// fractional part of (i + 0.5) / d is >= 0.5 / d, far above the float rounding of the product).
__device__ __forceinline__ int fdivi(int i, float inv_d) { return (int)(((float)i + 0.5f) * inv_d); }

constexpr int MF_T = 256;        // 4 waves
constexpr int MF_IPB = 8;        // samples per workgroup

typedef float mf4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ mf4 mfma16x4(float a, float b, mf4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Backward data: dX[ci][pix] = sum_k Wb[k][ci] * dYhalo[pix_base(pix) + koff(k)], k = (co, kh, kw).
// GEMM per sample: M = ci (NT tiles of 16), N = pixels (tiles of 16, split over the 4 waves), K = Co*KH*KW.
struct MfData {
  int C, H, W, Co, KH, KW, OH, OW, pad, OHp, OWp, K, Kp, CIp, ntile_pix;
};

template <int NT, int MT>
__global__ __launch_bounds__(MF_T) void conv_bwd_data_mfma_k(const float* __restrict__ dy,
                                                             const float* __restrict__ w,
                                                             float* __restrict__ dx, int64_t N, MfData g) {
  extern __shared__ __attribute__((aligned(16))) float ldsf[];
  unsigned short* wsb = reinterpret_cast<unsigned short*>(ldsf);            // bf16 signs [Kp][CIp]
  float* ds = reinterpret_cast<float*>(wsb + g.Kp * g.CIp);                   // [Co][OHp][OWp]
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int hT = g.KH - 1 - g.pad, wT = g.KW - 1 - g.pad, KK = g.KH * g.KW;
  for (int i = t; i < g.Kp * g.CIp; i += MF_T) {
    const int k = i / g.CIp, ci = i - k * g.CIp;
    int v = 0;
    if (k < g.K && ci < g.C) {
      const int co = k / KK, kk = k - co * KK;
      v = tsign(w[(co * g.C + ci) * KK + kk]);
    }
    wsb[i] = v > 0 ? 0x3F80 : (v < 0 ? 0xBF80 : 0);   // +-1 / 0 as bf16 (exact)
  }
  const int nds = g.Co * g.OHp * g.OWp;
  for (int i = t; i < nds; i += MF_T) ds[i] = 0.f;
  // this wave's pixel tiles: wv, wv+4, ...; per lane the B column (pixel) base offset
  const int HW = g.H * g.W;
  int pbase[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    int pix = (wv + 4 * m) * 16 + (lane & 15);
    if (pix >= HW) pix = 0;   // padded column: computed, never stored
    const int ih = pix / g.W, iw = pix - ih * g.W;
    pbase[m] = (ih + g.KH - 1) * g.OWp + iw + g.KW - 1;
  }
  const int my_tiles = (g.ntile_pix - wv + 3) / 4;
  const int64_t n0 = (int64_t)blockIdx.x * MF_IPB, n1 = (n0 + MF_IPB < N) ? n0 + MF_IPB : N;
  const int ohw = g.OH * g.OW;
  const float inv_ow = 1.f / (float)g.OW, inv_oh = 1.f / (float)g.OH;
  const float inv_kk = 1.f / (float)KK, inv_kw = 1.f / (float)g.KW;
  const int ohwp = g.OHp * g.OWp;
  for (int64_t n = n0; n < n1; ++n) {
    __syncthreads();   // previous sample's reads of ds are done (and the set-up above on entry)
    const float* dn = dy + n * g.Co * ohw;
    for (int i = t; i < g.Co * ohw; i += MF_T) {
      const int row = fdivi(i, inv_ow), ow = i - row * g.OW;   // row = co * OH + oh
      const int co = fdivi(row, inv_oh), oh = row - co * g.OH;
      ds[(co * g.OHp + oh + hT) * g.OWp + ow + wT] = dn[i];
    }
    __syncthreads();
    mf4 acc[NT][MT];
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[a][m] = mf4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < g.Kp; k0 += 4) {
      const int k = k0 + (lane >> 4);
      // koff(k) computed, not read: keeps the ds gather off a dependent LDS round trip.  k >= K
      // (zero weights) is clamped to a valid address; no branch in the loop body.  (A register
      // double-buffer of the operands made hipcc rotate the accumulators through AGPR copies
      // every step -- slower; the plain loop is kept.)
      const int kc = min(k, g.K - 1);
      const int co = fdivi(kc, inv_kk), kk = kc - co * KK, kh = fdivi(kk, inv_kw), kw = kk - kh * g.KW;
      const int ko = co * ohwp - kh * g.OWp - kw;
      float av[NT], bv[MT];
#pragma unroll
      for (int a = 0; a < NT; ++a)
        av[a] = __uint_as_float((unsigned)wsb[k * g.CIp + a * 16 + (lane & 15)] << 16);
#pragma unroll
      for (int m = 0; m < MT; ++m) bv[m] = ds[pbase[m] + ko];   // all MT tiles: branch-free body
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int a = 0; a < NT; ++a) acc[a][m] = mfma16x4(av[a], bv[m], acc[a][m]);
    }
    float* xn = dx + n * g.C * HW;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if (m >= my_tiles) continue;
      const int pix = (wv + 4 * m) * 16 + (lane & 15);
      if (pix >= HW) continue;
#pragma unroll
      for (int a = 0; a < NT; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ci = a * 16 + 4 * (lane >> 4) + r;
          if (ci < g.C) xn[(int64_t)ci * HW + pix] = acc[a][m][r];
        }
    }
  }
}

// ------------------------------------------------------------------ backward data on the bf16 MFMA (x3)
// dX[ci][pix] = sum_k Wb[ci][k] * dY[k](pix) with k = (tap, co), co innermost: every fp32 dY value is
// split EXACTLY into three bf16 terms (d1 = trunc_bf16(y), d2 = trunc_bf16(y - d1), d3 = y - d1 - d2,
// 24 mantissa bits = 3 x 8), the ternary weights are exact in bf16, so the three
// v_mfma_f32_16x16x32_bf16 passes multiply exactly and accumulate in fp32 (the fp32 reference's
// numerics class) at 3 bf16 passes = 1.6x the fp32-MFMA rate per pass... and 8x the K per
// instruction: K = 32 (8 channels of one tap per lane: one ds_read_b128 from a channels-innermost
// halo image [OHp][OWp][Cop] per plane), where the f32 MFMA takes 4.
//   16x16x32 bf16 lane map: A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15], D[4(l>>4)+r][l&15].
typedef short bf8 __attribute__((ext_vector_type(8)));

// Workgroup barrier that orders LDS only: waits for this wave's LDS operations (lgkmcnt(0)), not
// for its global loads -- a __syncthreads() (workgroup release fence) would also drain vmcnt and
// with it the loads in flight.  s_waitcnt simm16: vmcnt 63 | expcnt 7 | lgkmcnt 0.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xF | (7 << 4) | (0 << 8) | (3 << 14));
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

constexpr int B3_W = 8, B3_T = 64 * B3_W;   // 8 waves: two per SIMD, so LDS / MFMA latency overlaps
// samples per bf16x3 workgroup: 16 once that still gives >= 256 workgroups (one round over the CUs
// at N = 4096; the per-workgroup set-up amortises), else MF_IPB (the filter workspace's bound)
inline int b3_ipb(int64_t N) { return N >= 16 * 256 ? 16 : MF_IPB; }

struct B3Data {
  int C, H, W, Co, Cop, KH, KW, OH, OW, pad, OHp, OWp, taps, Kp, ntile_pix;
  int ps;    // halo pixel stride in bf16 elements, = 16 (mod 32): a 16-lane ds_read_b128 group holds
             // pixels p = 0..15 with chunk c or c + 1 ({0-3, 12-15} vs {4-11}), and 16-B quad
             // 6p + [4 <= p <= 11] (mod 16) is one-to-one -- conflict-free when a tile is one image row
  int ws;    // weight row stride: Kp + 16 (the same rule for the A reads)
  int rowt;  // 1: pixel tiles are image rows (W <= 16, lanes >= W idle); 0: 16 consecutive pixels
};

__device__ __forceinline__ void bf16x3_split(float y, unsigned short& d1, unsigned short& d2, unsigned short& d3) {
  const uint32_t u = __float_as_uint(y);
  const uint32_t h1 = u & 0xFFFF0000u;                 // truncation: y - d1 is exact in fp32
  const float r1 = y - __uint_as_float(h1);
  const uint32_t h2 = __float_as_uint(r1) & 0xFFFF0000u;
  const float r2 = r1 - __uint_as_float(h2);           // <= 8 significant bits left: exact in bf16
  d1 = (unsigned short)(h1 >> 16);
  d2 = (unsigned short)(h2 >> 16);
  d3 = (unsigned short)(__float_as_uint(r2) >> 16);
}

constexpr int B3_DU = 2;   // register-prefetched dY units per thread (backward data)

template <int NT, int MT>
__global__ __launch_bounds__(B3_T) void conv_bwd_data_bf3_k(const float* __restrict__ dy, const float* __restrict__ w,
                                                            float* __restrict__ dx, int64_t N, B3Data g,
                                                            int ipb) {
  extern __shared__ __attribute__((aligned(16))) float ldsf[];
  unsigned short* wsb = reinterpret_cast<unsigned short*>(ldsf);          // [16 NT][ws] ternary bf16
  unsigned short* img = wsb + 16 * NT * g.ws;                              // 3 x [OHp * OWp][ps]
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int KK = g.KH * g.KW;
  const int plane = g.OHp * g.OWp * g.ps;
  const float inv_ws = 1.f / (float)g.ws, inv_cop = 1.f / (float)g.Cop, inv_kw = 1.f / (float)g.KW;
  for (int i0 = t; i0 < 16 * NT * g.ws; i0 += 8 * B3_T) {   // 8 loads per thread in flight
    float v[8];
    bool ok[8];
#pragma unroll
    for (int k8 = 0; k8 < 8; ++k8) {
      const int i = i0 + k8 * B3_T;
      const int ci = fdivi(i, inv_ws), k = i - ci * g.ws;
      const int tap = fdivi(k, inv_cop), co = k - tap * g.Cop;
      ok[k8] = i < 16 * NT * g.ws && ci < g.C && k < g.Kp && tap < g.taps && co < g.Co;
      v[k8] = w[ok[k8] ? (co * g.C + ci) * KK + tap : 0];   // clamped, unconditional: loads batch
    }
#pragma unroll
    for (int k8 = 0; k8 < 8; ++k8) {
      const int i = i0 + k8 * B3_T;
      const int sv = ok[k8] ? tsign(v[k8]) : 0;
      if (i < 16 * NT * g.ws) wsb[i] = sv > 0 ? 0x3F80 : (sv < 0 ? 0xBF80 : 0);
    }
  }
  for (int i = t; i < 3 * plane; i += B3_T) img[i] = 0;   // zero halo (interior rewritten per sample)
  const int hT = g.KH - 1 - g.pad, wT = g.KW - 1 - g.pad;
  const int HW = g.H * g.W, ohw = g.OH * g.OW;
  // pixel of lane l in tile tt: image row tt, column l & 15 (rowt), or the 16 consecutive pixels
  // 16 tt + (l & 15); -1 = a padded column (computed at a clamped address, never stored)
  auto tile_pix = [&](int tt, int col) -> int {
    if (g.rowt) return (col < g.W && tt < g.H) ? tt * g.W + col : -1;
    const int p = tt * 16 + col;
    return p < HW ? p : -1;
  };
  int hb[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int tt = wv + B3_W * m, col = lane & 15;
    int ih, iw;
    if (g.rowt) {
      ih = min(tt, g.H - 1);
      iw = min(col, g.W - 1);
    } else {
      const int pix = max(tile_pix(tt, col), 0);
      ih = pix / g.W;
      iw = pix - ih * g.W;
    }
    hb[m] = ih * g.OWp + iw;
  }
  const int my_tiles = (g.ntile_pix - wv + B3_W - 1) / B3_W;
  const int chunk = lane >> 4;
  const int64_t n0 = (int64_t)blockIdx.x * ipb, n1 = (n0 + ipb < N) ? n0 + ipb : N;
  const float inv_ohw = 1.f / (float)ohw, inv_ow = 1.f / (float)g.OW;
  const int nunit = (g.Cop / 8) * ohw;    // staging unit = 8 channels of one pixel
  // lanes walk consecutive pixels of one 8-channel group: each of the 8 loads is coalesced, each
  // plane's 16-B chunk one ds_write_b128.  The thread's first B3_DU units of the next sample are
  // loaded into registers (clamped, unconditional: they batch) while this one is multiplied.
  auto put = [&](int u, const float* v) {
    const int c8 = fdivi(u, inv_ohw), r = u - c8 * ohw;
    const int oh = fdivi(r, inv_ow), ow = r - oh * g.OW;
    bf8 v1, v2, v3;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float y = 8 * c8 + j < g.Co ? v[j] : 0.f;
      unsigned short d1, d2, d3;
      bf16x3_split(y, d1, d2, d3);
      v1[j] = (short)d1;
      v2[j] = (short)d2;
      v3[j] = (short)d3;
    }
    const int o = ((oh + hT) * g.OWp + ow + wT) * g.ps + 8 * c8;
    *reinterpret_cast<bf8*>(img + o) = v1;
    *reinterpret_cast<bf8*>(img + plane + o) = v2;
    *reinterpret_cast<bf8*>(img + 2 * plane + o) = v3;
  };
  auto load_unit = [&](int64_t n, int u, float* v) {
    const int uc = min(u, nunit - 1);
    const int c8 = fdivi(uc, inv_ohw), r = uc - c8 * ohw;
    const float* dn = dy + n * (int64_t)g.Co * ohw + r;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = dn[min(8 * c8 + j, g.Co - 1) * ohw];
  };
  float ud[B3_DU][8];
  auto fetch = [&](int64_t n) {
#pragma unroll
    for (int s = 0; s < B3_DU; ++s) load_unit(n, t + s * B3_T, ud[s]);
  };
  if (n0 < n1) fetch(n0);
  for (int64_t n = n0; n < n1; ++n) {
    lds_barrier();   // previous sample's fragment reads are done (and the set-up above on entry)
#pragma unroll
    for (int s = 0; s < B3_DU; ++s)
      if (t + s * B3_T < nunit) put(t + s * B3_T, ud[s]);
    for (int u = t + B3_DU * B3_T; u < nunit; u += B3_T) {
      float v[8];
      load_unit(n, u, v);
      put(u, v);
    }
    if (n + 1 < n1) fetch(n + 1);
    lds_barrier();
    mf4 acc[NT][MT];
#pragma unroll
    for (int a = 0; a < NT; ++a)
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[a][m] = mf4{0.f, 0.f, 0.f, 0.f};
    if (g.Cop == 32 && g.Kp == 32 * g.taps) {
      // one k-step = one tap (32 channels): the tap, its (kh, kw) and the halo offset are uniform
      // (scalar registers), each lane's fragment addresses a fixed base plus that offset -- the
      // general loop below spends ~20 VALU per k-step on per-lane index arithmetic.  Same MFMAs in
      // the same order (bit-identical).
      const int abase = (lane & 15) * g.ws + 8 * chunk;
      int bbase[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) bbase[m] = hb[m] * g.ps + 8 * chunk;
      int kh = 0, kw = 0;
      for (int tap = 0; tap < g.taps; ++tap) {
        const int hoff = ((g.KH - 1 - kh) * g.OWp + (g.KW - 1 - kw)) * g.ps;
        bf8 av[NT];
#pragma unroll
        for (int a = 0; a < NT; ++a)
          av[a] = *reinterpret_cast<const bf8*>(wsb + a * 16 * g.ws + abase + 32 * tap);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          bf8 bv[MT];
#pragma unroll
          for (int m = 0; m < MT; ++m)
            bv[m] = *reinterpret_cast<const bf8*>(img + j * plane + bbase[m] + hoff);
#pragma unroll
          for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int a = 0; a < NT; ++a)
              acc[a][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[a], bv[m], acc[a][m], 0, 0, 0);
        }
        if (++kw == g.KW) {
          kw = 0;
          ++kh;
        }
      }
    } else {
      for (int k0 = 0; k0 < g.Kp; k0 += 32) {
        const int k = k0 + 8 * chunk;
        const int tq = fdivi(k, inv_cop), co0 = k - tq * g.Cop;
        const int tap = min(tq, g.taps - 1);                 // padded k: zero weights
        const int kh = fdivi(tap, inv_kw), kw = tap - kh * g.KW;
        const int hoff = (g.KH - 1 - kh) * g.OWp + (g.KW - 1 - kw);
        bf8 av[NT];
#pragma unroll
        for (int a = 0; a < NT; ++a)
          av[a] = *reinterpret_cast<const bf8*>(wsb + (a * 16 + (lane & 15)) * g.ws + k);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          bf8 bv[MT];
#pragma unroll
          for (int m = 0; m < MT; ++m)
            bv[m] = *reinterpret_cast<const bf8*>(img + j * plane + (hb[m] + hoff) * g.ps + co0);
#pragma unroll
          for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int a = 0; a < NT; ++a)
              acc[a][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[a], bv[m], acc[a][m], 0, 0, 0);
        }
      }
    }
    float* xn = dx + n * (int64_t)g.C * HW;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      if (m >= my_tiles) continue;
      const int pix = tile_pix(wv + B3_W * m, lane & 15);
      if (pix < 0) continue;
#pragma unroll
      for (int a = 0; a < NT; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ci = a * 16 + 4 * chunk + r;
          if (ci < g.C) xn[(int64_t)ci * HW + pix] = acc[a][m][r];
        }
    }
  }
}

// Backward filter on the bf16 MFMA (x3): dW[co][combo] = sum_{n,p} dY[n][co][p] * Xb[n][combo](p),
// combo = (ci, kh, kw).  A = dY (the three exact bf16 terms, rows co, K = pixels), B = the ternary
// input (exact in bf16; binarised, or any input that is exact in bf16 -- see b3_filt_geom).  K runs
// over output pixels in rows padded to OWq = round_up(OW, 8), so a lane's 8 consecutive k are 8
// pixels of one row: one ds_read_b128 from dY's plane, and one from the kw-shifted copy of the
// input row (KW copies, so every tap's 8-pixel window starts 16-B aligned).  Each wave owns a set
// of combo tiles for all co tiles (the A fragments are loaded once per k-step and reused).
//   Staging, per sample: the thread's dY units (8 pixels of a row; B3_UD of them) and its slice of
// the flat input (B3_PX elements, coalesced; fewer for the widest tilings) are loaded into
// registers with clamped, unconditional loads (a guarded load is a branch, and the loads would not
// batch), issued right after the previous sample's registers were written out, so they fly under
// its image build and MFMA phase (barriers wait on LDS only).  The input lands once as ternary bf16 in a zero-haloed image xh;
// the KW shifted copies are built from xh in LDS.  dB: each unit's owner thread accumulates the
// unit's sum over the workgroup's samples in LDS; channels are folded once at the end.
constexpr int B3_UD = 4, B3_PX = 8;

struct B3Filt {
  int C, H, W, Co, KH, KW, OH, OW, pad, Hp, OWq, Kp, Kd, xrow, Co16, NA, ncombo, ntn, WT, KS, Wh;
  int CS, XL;   // shifted copies: channel stride and copy stride (bf16), padded for conflict-free B reads
};

template <int NA, int MT>
__global__ __launch_bounds__(B3_T) void conv_bwd_filter_bf3_k(const float* __restrict__ dy,
                                                              const float* __restrict__ x, int binarize,
                                                              float* __restrict__ part, int64_t N, B3Filt g,
                                                              int with_bias, int ipb) {
  extern __shared__ __attribute__((aligned(16))) float ldsf[];
  unsigned short* dyp = reinterpret_cast<unsigned short*>(ldsf);       // 3 x [Co16][Kd]
  const int PL = g.Co16 * g.Kd;
  unsigned short* xs = dyp + 3 * PL;                                    // KW x [C][Hp][xrow]
  const int XL = g.XL;
  unsigned short* xh = xs + g.KW * XL;                                  // [C][Hp][Wh], zero halo
  const int XH = g.C * g.Hp * g.Wh;
  float* bpart = reinterpret_cast<float*>(xh + ((XH + 7) & ~7));      // [Co16][Kp / 8]
  __shared__ float sbias[64];
  const float inv_kk = 1.f / (float)(g.KH * g.KW), inv_kw = 1.f / (float)g.KW, inv_owq = 1.f / (float)g.OWq;
  const float inv_dq = 1.f / (float)(g.OH * (g.OWq / 8)), inv_nq = 1.f / (float)(g.OWq / 8);
  const float inv_xq = 1.f / (float)(g.C * g.Hp * (g.OWq / 8)), inv_hq = 1.f / (float)(g.Hp * (g.OWq / 8));
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int grp = wv % g.WT, ks = wv / g.WT;
  const int KK = g.KH * g.KW;
  const int nq = g.OWq / 8, kq = g.Kp / 8;
  const int ohw = g.OH * g.OW, hw = g.H * g.W;
  const float inv_hw = 1.f / (float)hw, inv_w = 1.f / (float)g.W;
  if (t < 64) sbias[t] = 0.f;
  for (int i = t; i < 3 * PL; i += B3_T) dyp[i] = 0;     // zero tails: co >= Co, k >= OH*OWq
  for (int i = t; i < XH; i += B3_T) xh[i] = 0;
  for (int i = t; i < g.Co16 * kq; i += B3_T) bpart[i] = 0.f;
  int boff[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int nt = min(grp + g.WT * m, g.ntn - 1);
    int combo = nt * 16 + (lane & 15);
    if (combo >= g.ncombo) combo = 0;   // padded column: computed, never stored
    const int ci = fdivi(combo, inv_kk), kk = combo - ci * KK, kh = fdivi(kk, inv_kw), kw = kk - kh * g.KW;
    boff[m] = kw * g.XL + ci * g.CS + kh * g.xrow;
  }
  const int my_tiles = (g.ntn - grp + g.WT - 1) / g.WT;
  mf4 acc[NA][MT];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[a][m] = mf4{0.f, 0.f, 0.f, 0.f};
  const int kslice = g.Kp / g.KS, k_lo = ks * kslice, k_hi = k_lo + kslice;
  const int chunk = lane >> 4;
  const int ndu = g.Co16 * g.OH * nq;                    // dY units (8 pixels of a row)
  const int nxu = g.KW * g.C * g.Hp * nq;                 // shifted-copy units (8 of a row)
  // this thread's dY units u = t + 512 s: source offset of pixel 0 and the valid-pixel count
  constexpr int W_ = NA * MT, UD = W_ >= 24 ? 1 : (W_ >= 12 ? B3_UD / 2 : B3_UD), PX = W_ >= 12 ? B3_PX / 2 : B3_PX;
  int usrc[UD], uvalid[UD];
#pragma unroll
  for (int s = 0; s < UD; ++s) {
    const int u = min(t + s * B3_T, ndu - 1);
    const int co = fdivi(u, inv_dq), r = u - co * (g.OH * nq), oh = fdivi(r, inv_nq), q = r - oh * nq;
    const int ow0 = 8 * q;
    uvalid[s] = (t + s * B3_T < ndu && co < g.Co) ? min(8, g.OW - ow0) : 0;
    usrc[s] = min(co, g.Co - 1) * ohw + oh * g.OW + min(ow0, g.OW - 1);
  }
  const int tot_x = g.C * hw;
  float ud[UD][8], px[PX];
  auto fetch = [&](int64_t n) {   // clamped, unconditional: the loads batch
    const float* dn = dy + n * (int64_t)g.Co * ohw;
    const float* xn = x + n * (int64_t)tot_x;
#pragma unroll
    for (int s = 0; s < UD; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) ud[s][j] = dn[usrc[s] + min(j, max(uvalid[s] - 1, 0))];
#pragma unroll
    for (int s = 0; s < PX; ++s) px[s] = xn[min(t + s * B3_T, tot_x - 1)];
  };
  auto put_unit = [&](int u, const float* v, int valid) {   // 3 bf16 planes + the unit's dB partial
    const int co = fdivi(u, inv_dq), r = u - co * (g.OH * nq), oh = fdivi(r, inv_nq), q = r - oh * nq;
    bf8 v1, v2, v3;
    float bsum = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float y = j < valid ? v[j] : 0.f;
      bsum += y;
      unsigned short d1, d2, d3;
      bf16x3_split(y, d1, d2, d3);
      v1[j] = (short)d1;
      v2[j] = (short)d2;
      v3[j] = (short)d3;
    }
    const int o = co * g.Kd + oh * g.OWq + 8 * q;
    *reinterpret_cast<bf8*>(dyp + o) = v1;
    *reinterpret_cast<bf8*>(dyp + PL + o) = v2;
    *reinterpret_cast<bf8*>(dyp + 2 * PL + o) = v3;
    bpart[co * kq + oh * nq + q] += bsum;   // this thread owns the unit for every sample
  };
  auto put_x = [&](int i, float v) {
    const int c = fdivi(i, inv_hw), r = i - c * hw, ih = fdivi(r, inv_w), iw = r - ih * g.W;
    const float xv = binarize ? (float)tsign(v) : v;
    xh[(c * g.Hp + ih + g.pad) * g.Wh + iw + g.pad] = (unsigned short)(__float_as_uint(xv) >> 16);
  };
  const int64_t n0 = (int64_t)blockIdx.x * ipb, n1 = (n0 + ipb < N) ? n0 + ipb : N;
  if (n0 < n1) fetch(n0);
  for (int64_t n = n0; n < n1; ++n) {
    lds_barrier();   // previous sample's fragment and xh reads are done
#pragma unroll
    for (int s = 0; s < UD; ++s)
      if (t + s * B3_T < ndu) put_unit(t + s * B3_T, ud[s], uvalid[s]);
#pragma unroll
    for (int s = 0; s < PX; ++s)
      if (t + s * B3_T < tot_x) put_x(t + s * B3_T, px[s]);
    for (int u = t + UD * B3_T; u < ndu; u += B3_T) {   // beyond the register slots: direct
      const int co = fdivi(u, inv_dq), r = u - co * (g.OH * nq), oh = fdivi(r, inv_nq), q = r - oh * nq;
      const int valid = co < g.Co ? min(8, g.OW - 8 * q) : 0;
      const float* src = dy + n * (int64_t)g.Co * ohw + min(co, g.Co - 1) * ohw + oh * g.OW;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = src[min(8 * q + j, g.OW - 1)];
      put_unit(u, v, valid);
    }
    for (int i = t + PX * B3_T; i < tot_x; i += B3_T) put_x(i, x[n * (int64_t)tot_x + i]);
    if (n + 1 < n1) fetch(n + 1);   // in flight across the copy build and the MFMA phase
    lds_barrier();
    for (int u = t; u < nxu; u += B3_T) {   // shifted copies from xh: copy kw, column p = x col p + kw - pad
      const int kw = fdivi(u, inv_xq), r0 = u - kw * (g.C * g.Hp * nq);
      const int c = fdivi(r0, inv_hq), r1 = r0 - c * (g.Hp * nq), ihh = fdivi(r1, inv_nq), q = r1 - ihh * nq;
      const unsigned short* src = xh + (c * g.Hp + ihh) * g.Wh + 8 * q + kw;
      bf8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (short)src[j];
      *reinterpret_cast<bf8*>(xs + kw * XL + c * g.CS + ihh * g.xrow + 8 * q) = v;
    }
    lds_barrier();
    for (int k0 = k_lo; k0 < k_hi; k0 += 32) {
      const int kk = k0 + 8 * chunk;
      const int ohq = fdivi(kk, inv_owq), ow0 = kk - ohq * g.OWq;
      const int oh = min(ohq, g.OH - 1);                   // k tail: zero dY, any valid input row
      bf8 av[NA][3];
#pragma unroll
      for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          av[a][j] = *reinterpret_cast<const bf8*>(dyp + j * PL + (16 * a + (lane & 15)) * g.Kd + kk);
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const bf8 bv = *reinterpret_cast<const bf8*>(xs + boff[m] + oh * g.xrow + ow0);
#pragma unroll
        for (int a = 0; a < NA; ++a)
#pragma unroll
          for (int j = 0; j < 3; ++j)
            acc[a][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[a][j], bv, acc[a][m], 0, 0, 0);
      }
    }
  }
  __syncthreads();
  if (with_bias) {   // dB: wave w folds channels w, w+8, ... (fixed order: deterministic)
    for (int co = wv; co < g.Co; co += B3_W) {
      float sb = 0.f;
      for (int i = lane; i < kq; i += 64) sb += bpart[co * kq + i];
      const double tb = wave_sum((double)sb);
      if (lane == 0) sbias[co] = (float)tb;
    }
  }
  __syncthreads();
  const int64_t nelem = (int64_t)g.Co * g.ncombo + g.Co;
  float* row = part + ((int64_t)blockIdx.x * g.KS + ks) * nelem;
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    if (m >= my_tiles) continue;
    const int combo = (grp + g.WT * m) * 16 + (lane & 15);
    if (combo >= g.ncombo) continue;
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = 16 * a + 4 * chunk + r;
        if (co < g.Co) row[(int64_t)co * g.ncombo + combo] = acc[a][m][r];
      }
  }
  if (t < g.Co) {   // bias partial in k-slice 0's row, zero in the others
    part[((int64_t)blockIdx.x * g.KS) * nelem + (int64_t)g.Co * g.ncombo + t] = with_bias ? sbias[t] : 0.f;
    for (int q2 = 1; q2 < g.KS; ++q2)
      part[((int64_t)blockIdx.x * g.KS + q2) * nelem + (int64_t)g.Co * g.ncombo + t] = 0.f;
  }
}

// Backward filter: dW[co][combo] = sum_{n,p} dY[n][co][p] * Xs[n][combo][p], combo = (ci, kh, kw).
// Tiles (co16, combo16) are dealt to WT wave groups; the remaining 4/WT factor splits the pixel
// range (K), each (block, k-slice) writing one partial row for conv_filter_tile_reduce{1,2}_k.
struct MfFilt {
  int C, H, W, Co, KH, KW, OH, OW, pad, Hp, Wp, P, Pp, Co16, ncombo, ntn, ntiles, WT, KS;
};

template <int MT>
__global__ __launch_bounds__(MF_T) void conv_bwd_filter_mfma_k(const float* __restrict__ dy,
                                                               const float* __restrict__ x, int binarize,
                                                               float* __restrict__ part, int64_t N,
                                                               MfFilt g, int with_bias) {
  extern __shared__ __attribute__((aligned(16))) float ldsf[];
  float* xs = ldsf;                               // [C][Hp][Wp], zero border
  float* dys = xs + ((g.C * g.Hp * g.Wp + 3) & ~3);   // [Co16][Pp], zero padded, 16-B aligned
  int* poff = reinterpret_cast<int*>(dys + g.Co16 * g.Pp);   // [Pp]
  __shared__ float sbias[64];                     // per-channel dB of this workgroup's samples
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int grp = wv % g.WT, ks = wv / g.WT;
  const int KK = g.KH * g.KW;
  if (t < 64) sbias[t] = 0.f;
  for (int i = t; i < g.C * g.Hp * g.Wp; i += MF_T) xs[i] = 0.f;
  for (int i = t; i < g.Co16 * g.Pp; i += MF_T) dys[i] = 0.f;
  for (int p = t; p < g.Pp; p += MF_T) {
    const int oh = p / g.OW, ow = p - oh * g.OW;
    poff[p] = p < g.P ? oh * g.Wp + ow : 0;
  }
  // this wave's tiles t = grp + WT*m; per lane the B column (combo) offset and the A row (co)
  int boff[MT], arow[MT];
  const int my_tiles = (g.ntiles - grp + g.WT - 1) / g.WT;
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int tt = min(grp + g.WT * m, g.ntiles - 1);   // past this wave's tiles: valid, unused
    const int mt = tt / g.ntn, nt = tt - mt * g.ntn;
    int combo = nt * 16 + (lane & 15);
    if (combo >= g.ncombo) combo = 0;   // padded column: computed, never stored
    const int ci = combo / KK, kk = combo - ci * KK, kh = kk / g.KW, kw = kk - kh * g.KW;
    boff[m] = (ci * g.Hp + kh) * g.Wp + kw;
    arow[m] = (mt * 16 + (lane & 15)) * g.Pp;   // A[i = co][k = p]
  }
  mf4 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = mf4{0.f, 0.f, 0.f, 0.f};
  float bacc = 0.f;
  const int pslice = g.Pp / g.KS, p_lo = ks * pslice, p_hi = p_lo + pslice;
  const float inv_w = 1.f / (float)g.W, inv_h = 1.f / (float)g.H, inv_p = 1.f / (float)g.P;
  const float inv_ow = 1.f / (float)g.OW;
  const int64_t n0 = (int64_t)blockIdx.x * MF_IPB, n1 = (n0 + MF_IPB < N) ? n0 + MF_IPB : N;
  for (int64_t n = n0; n < n1; ++n) {
    __syncthreads();
    const float* xn = x + n * g.C * g.H * g.W;
    for (int i = t; i < g.C * g.H * g.W; i += MF_T) {
      const int row = fdivi(i, inv_w), iw = i - row * g.W;   // row = c * H + ih
      const int c = fdivi(row, inv_h), ih = row - c * g.H;
      const float v = xn[i];
      xs[(c * g.Hp + ih + g.pad) * g.Wp + iw + g.pad] = binarize ? (float)tsign(v) : v;
    }
    const float* dn = dy + n * g.Co * g.P;
    if (g.Pp == g.P && ((g.Co * g.P) & 3) == 0) {   // dense rows: straight 16-B copy
      for (int i = 4 * t; i < g.Co * g.P; i += 4 * MF_T)
        *reinterpret_cast<float4*>(dys + i) = *reinterpret_cast<const float4*>(dn + i);
    } else {
      for (int i = t; i < g.Co * g.P; i += MF_T) {
        const int co = fdivi(i, inv_p), p = i - co * g.P;
        dys[co * g.Pp + p] = dn[i];
      }
    }
    __syncthreads();
    auto gather = [&](int p0, float* av, float* bv) {
      const int p = p0 + (lane >> 4);
      const int pc = min(p, g.P - 1);   // p >= P: zero dY column, any valid x address
      const int oh = fdivi(pc, inv_ow), ow = pc - oh * g.OW;
      const int po = oh * g.Wp + ow;
#pragma unroll
      for (int m = 0; m < MT; ++m) {   // all MT tiles: branch-free body
        av[m] = dys[arow[m] + p];
        bv[m] = xs[boff[m] + po];
      }
    };
    float av[MT], bv[MT], an[MT], bn[MT];
    gather(p_lo, an, bn);
    for (int p0 = p_lo; p0 < p_hi; p0 += 4) {   // software-pipelined as in the data kernel
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        av[m] = an[m];
        bv[m] = bn[m];
      }
      gather(min(p0 + 4, p_hi - 4), an, bn);
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[m] = mfma16x4(av[m], bv[m], acc[m]);
    }
    if (with_bias) {   // dB: wave w sums channels w, w+4, ... across its 64 lanes (not one serial lane)
      for (int co = wv; co < g.Co; co += 4) {
        float sb = 0.f;
        for (int p = lane; p < g.P; p += 64) sb += dys[co * g.Pp + p];
        const double tot = wave_sum((double)sb);
        if (lane == 0) sbias[co] += (float)tot;
      }
    }
  }
  __syncthreads();
  if (t < g.Co) bacc = sbias[t];
  const int64_t nelem = (int64_t)g.Co * g.ncombo + g.Co;
  float* row = part + ((int64_t)blockIdx.x * g.KS + ks) * nelem;
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    if (m >= my_tiles) continue;
    const int tt = grp + g.WT * m;
    const int mt = tt / g.ntn, nt = tt - mt * g.ntn;
    const int combo = nt * 16 + (lane & 15);
    if (combo >= g.ncombo) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = mt * 16 + 4 * (lane >> 4) + r;
      if (co < g.Co) row[(int64_t)co * g.ncombo + combo] = acc[m][r];
    }
  }
  if (t < g.Co) {   // bias partial in k-slice 0's row, zero in the others
    part[((int64_t)blockIdx.x * g.KS) * nelem + (int64_t)g.Co * g.ncombo + t] = with_bias ? bacc : 0.f;
    for (int q = 1; q < g.KS; ++q) part[((int64_t)blockIdx.x * g.KS + q) * nelem + (int64_t)g.Co * g.ncombo + t] = 0.f;
  }
}

// Forward binary conv as an implicit GEMM on v_mfma_i32_16x16x64_i8 (exact integer sums, so the
// output equals the reference's F.conv2d on sign()ed operands bit for bit, + one fp32 bias add).
// K order = (tap, 16-channel chunk): one lane's 16-byte fragment is 16 channels of one tap of one
// pixel, a single ds_read_b128 from the channels-innermost int8 image xs[Hp][Wp][C].
//   A[i = co][k]  = sign(W[co][ci][kh][kw])   (ws[co][KCp*16], zero for padded chunks)
//   B[k][j = pix] = sign(x[ci][oh+kh-pad][ow+kw-pad])
//   16x16x64 lane map: row/col = l&15, 16-byte chunk (l>>4) of the 64-byte k-step; D row 4(l>>4)+r.
struct MfFwd {
  int C, H, W, Co, KH, KW, OH, OW, pad, Hp, Wp, CB, KC, KCp, ntile_pix;
};

constexpr int FW_IPB = 8;    // samples per forward workgroup (the weight staging amortises)
constexpr int FW_PX = 16;    // per-thread register slots of the next sample's input

template <int COT, typename OT = float>
__global__ __launch_bounds__(MF_T) void conv_fwd_i8mfma_k(const float* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ bias, OT* __restrict__ y,
                                                          int64_t N, MfFwd g) {
  extern __shared__ __attribute__((aligned(16))) float ldsf[];
  int8_t* ws = reinterpret_cast<int8_t*>(ldsf);                 // [COT*16][KCp*16]
  int8_t* xs = ws + COT * 16 * g.KCp * 16;                      // [Hp][Wp][C]
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int KK = g.KH * g.KW, rowb = g.KCp * 16;
  {   // ternary weights, 8 loads per thread in flight (clamped, unconditional: they batch)
    const int nws = COT * 16 * rowb;
    const float inv_rowb = 1.f / (float)rowb, inv_cb = 1.f / (float)g.CB;
    for (int i0 = t; i0 < nws; i0 += 8 * MF_T) {
      float v[8];
      bool ok[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int i = i0 + k * MF_T;
        const int co = fdivi(i, inv_rowb), kb = i - co * rowb, ch = kb >> 4, ci16 = kb & 15;
        const int tap = fdivi(ch, inv_cb), ci = (ch - tap * g.CB) * 16 + ci16;
        ok[k] = i < nws && co < g.Co && ch < g.KC;
        v[k] = w[ok[k] ? (co * g.C + ci) * KK + tap : 0];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (i0 + k * MF_T < nws) ws[i0 + k * MF_T] = (int8_t)(ok[k] ? tsign(v[k]) : 0);
    }
  }
  const int nxs = g.Hp * g.Wp * g.C;
  for (int i = t; i < nxs; i += MF_T) xs[i] = 0;
  // this wave's pixel tiles wv, wv+4, wv+8, wv+12 (clamped: computed, never stored)
  const int HW = g.H * g.W, OHW = g.OH * g.OW;
  int pbase[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    int pix = (wv + 4 * m) * 16 + (lane & 15);
    if (pix >= OHW) pix = 0;
    const int oh = pix / g.OW, ow = pix - oh * g.OW;
    pbase[m] = (oh * g.Wp + ow) * g.C;
  }
  const int my_tiles = (g.ntile_pix - wv + 3) / 4;
  const int h = lane >> 4;
  const float inv_w = 1.f / (float)g.W, inv_hw = 1.f / (float)HW;
  const int64_t n0 = (int64_t)blockIdx.x * FW_IPB, n1 = (n0 + FW_IPB < N) ? n0 + FW_IPB : N;
  const int tot = g.C * HW;
  auto put = [&](int i, float v) {
    const int c = fdivi(i, inv_hw), r = i - c * HW, ih = fdivi(r, inv_w), iw = r - ih * g.W;
    xs[((ih + g.pad) * g.Wp + iw + g.pad) * g.C + c] = (int8_t)tsign(v);
  };
  // the next sample's input: flat, clamped, unconditional loads (they batch), in flight across
  // the MFMA phase and the output stores (the barriers wait on LDS only)
  float px[FW_PX];
  auto fetch = [&](int64_t n) {
    const float* xn = x + n * (int64_t)tot;
#pragma unroll
    for (int s = 0; s < FW_PX; ++s) px[s] = xn[min(t + s * MF_T, tot - 1)];
  };
  if (n0 < n1) fetch(n0);
  for (int64_t n = n0; n < n1; ++n) {
    lds_barrier();   // previous sample's fragment reads are done (and the set-up above on entry)
#pragma unroll
    for (int s = 0; s < FW_PX; ++s)
      if (t + s * MF_T < tot) put(t + s * MF_T, px[s]);
    for (int i = t + FW_PX * MF_T; i < tot; i += MF_T) put(i, x[n * (int64_t)tot + i]);
    if (n + 1 < n1) fetch(n + 1);
    lds_barrier();
    v4i acc[COT][4];
#pragma unroll
    for (int a = 0; a < COT; ++a)
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[a][m] = v4i{0, 0, 0, 0};
    for (int ks = 0; ks < g.KCp / 4; ++ks) {
      const int ch = min(4 * ks + h, g.KC - 1);   // padded chunks: zero weights, valid address
      const int tap = ch / g.CB, cb = ch - tap * g.CB;
      const int kh = tap / g.KW, kw = tap - kh * g.KW;
      const int xo = (kh * g.Wp + kw) * g.C + cb * 16;
      v4i av[COT], bv[4];
#pragma unroll
      for (int a = 0; a < COT; ++a)
        av[a] = *reinterpret_cast<const v4i*>(ws + (a * 16 + (lane & 15)) * rowb + (4 * ks + h) * 16);
#pragma unroll
      for (int m = 0; m < 4; ++m) bv[m] = *reinterpret_cast<const v4i*>(xs + pbase[m] + xo);
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int a = 0; a < COT; ++a)
          acc[a][m] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av[a], bv[m], acc[a][m], 0, 0, 0);
    }
    OT* yn = y + n * g.Co * OHW;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      if (m >= my_tiles) continue;
      const int pix = (wv + 4 * m) * 16 + (lane & 15);
      if (pix >= OHW) continue;
#pragma unroll
      for (int a = 0; a < COT; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = a * 16 + 4 * h + r;
          if (co < g.Co) yn[(int64_t)co * OHW + pix] = conv_out<OT>(acc[a][m][r], bias, co);
        }
    }
  }
}

inline bool mf_fwd_geom(const ConvShape& s, MfFwd* g, int64_t* lds) {
  if (!(s.groups == 1 && s.stride == 1 && s.dil == 1 && s.C % 16 == 0 && s.C <= 64 && s.Co <= 64 &&
        s.pad <= s.KH - 1 && s.pad <= s.KW - 1))
    return false;
  MfFwd d;
  d.C = (int)s.C; d.H = (int)s.H; d.W = (int)s.W; d.Co = (int)s.Co; d.KH = (int)s.KH; d.KW = (int)s.KW;
  d.OH = (int)s.OH; d.OW = (int)s.OW; d.pad = s.pad;
  d.Hp = d.H + 2 * d.pad; d.Wp = d.W + 2 * d.pad;
  d.CB = d.C / 16;
  d.KC = d.KH * d.KW * d.CB;
  d.KCp = (int)round_up(d.KC, 4);
  d.ntile_pix = (d.OH * d.OW + 15) / 16;
  if (d.ntile_pix > 16 || (int64_t)d.C * d.H * d.W >= (1 << 20)) return false;
  // gathered pixel (oh + kh, ow + kw) stays inside the padded image
  if (d.OH - 1 + d.KH - 1 >= d.Hp || d.OW - 1 + d.KW - 1 >= d.Wp) return false;
  const int cot = (d.Co + 15) / 16;
  *lds = (int64_t)(cot == 3 ? 4 : cot) * 16 * d.KCp * 16 + round_up((int64_t)d.Hp * d.Wp * d.C, 16);
  *g = d;
  return *lds <= kMaxTileLds;
}

inline bool mf_data_geom(const ConvShape& s, MfData* g, int64_t* lds) {
  if (!(s.groups == 1 && s.stride == 1 && s.dil == 1 && s.pad <= s.KH - 1 && s.pad <= s.KW - 1 && s.C <= 32))
    return false;
  MfData d;
  d.C = (int)s.C; d.H = (int)s.H; d.W = (int)s.W; d.Co = (int)s.Co; d.KH = (int)s.KH; d.KW = (int)s.KW;
  d.OH = (int)s.OH; d.OW = (int)s.OW; d.pad = s.pad;
  d.OHp = d.OH + 2 * (d.KH - 1 - d.pad);
  d.OWp = d.OW + 2 * (d.KW - 1 - d.pad);
  d.K = d.Co * d.KH * d.KW;
  d.Kp = (int)round_up(d.K, 4);
  d.CIp = d.C <= 16 ? 16 : 32;
  d.ntile_pix = (d.H * d.W + 15) / 16;
  if ((d.ntile_pix + 3) / 4 > 16 || (int64_t)d.Co * d.OH * d.OW >= (1 << 20)) return false;
  *lds = (int64_t)d.Kp * d.CIp * 2 + (int64_t)d.Co * d.OHp * d.OWp * 4;
  *g = d;
  return *lds <= kMaxTileLds;
}

inline bool b3_data_geom(const ConvShape& s, B3Data* g, int64_t* lds) {
  if (!(s.groups == 1 && s.stride == 1 && s.dil == 1 && s.pad <= s.KH - 1 && s.pad <= s.KW - 1 && s.C <= 32))
    return false;
  B3Data d;
  d.C = (int)s.C; d.H = (int)s.H; d.W = (int)s.W; d.Co = (int)s.Co; d.KH = (int)s.KH; d.KW = (int)s.KW;
  d.OH = (int)s.OH; d.OW = (int)s.OW; d.pad = s.pad;
  d.Cop = (int)round_up(d.Co, 8);
  d.OHp = d.OH + 2 * (d.KH - 1 - d.pad);
  d.OWp = d.OW + 2 * (d.KW - 1 - d.pad);
  d.taps = d.KH * d.KW;
  d.Kp = (int)round_up((int64_t)d.taps * d.Cop, 32);
  d.rowt = d.W <= 16 ? 1 : 0;
  d.ntile_pix = d.rowt ? d.H : (d.H * d.W + 15) / 16;
  d.ps = (int)round_up(d.Cop, 32) + 16;
  d.ws = d.Kp + 16;
  if ((d.ntile_pix + B3_W - 1) / B3_W > 16 || (int64_t)d.Co * d.OH * d.OW >= (1 << 20)) return false;
  const int nt = d.C <= 16 ? 1 : 2;
  *lds = (int64_t)16 * nt * d.ws * 2 + (int64_t)3 * d.OHp * d.OWp * d.ps * 2;
  *g = d;
  return *lds <= kMaxTileLds;
}

// LDS cycles of one wave's ds_read_b128 on gfx950 (MI355X_MICROARCH.md §LDS): four 16-lane groups
// {0-3,12-15,20-27}, {4-11,16-19,28-31} and the same + 32, bank (a/4) mod 64; a group costs the
// largest number of distinct dword addresses on one bank.
static int lds_b128_cycles(const int (&addr)[64]) {
  static const int grp[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                 {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                 {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                 {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
  int tot = 0;
  for (int gi = 0; gi < 4; ++gi) {
    int dw[64];
    for (int i = 0; i < 16; ++i)
      for (int w = 0; w < 4; ++w) dw[4 * i + w] = addr[grp[gi][i]] / 4 + w;
    std::sort(dw, dw + 64);
    const int n = (int)(std::unique(dw, dw + 64) - dw);
    int cnt[64] = {0}, worst = 1;
    for (int i = 0; i < n; ++i) worst = std::max(worst, ++cnt[((dw[i] % 64) + 64) % 64]);
    tot += worst;
  }
  return tot;
}

// The filter kernel's B reads (one 16-combo tile per lane group row, 4 k-chunks) under a copy
// layout: total LDS cycles over the first k-steps and every combo tile.
static int b3_filt_b_cycles(const B3Filt& d, int CS, int XL) {
  int tot = 0;
  const int ksteps = std::min(d.Kp / 32, 4);
  for (int ks = 0; ks < ksteps; ++ks)
    for (int nt = 0; nt < d.ntn; ++nt) {
      int addr[64];
      for (int l = 0; l < 64; ++l) {
        int combo = nt * 16 + (l & 15);
        if (combo >= d.ncombo) combo = 0;
        const int ci = combo / (d.KH * d.KW), kk = combo - ci * d.KH * d.KW, kh = kk / d.KW, kw = kk - kh * d.KW;
        const int kq = 32 * ks + 8 * (l >> 4), ohq = kq / d.OWq, ow0 = kq - ohq * d.OWq;
        addr[l] = 2 * (kw * XL + ci * CS + kh * d.xrow + std::min(ohq, d.OH - 1) * d.xrow + ow0);
      }
      tot += lds_b128_cycles(addr);
    }
  return tot;
}

// Pads of the shifted copies' channel stride (CS = Hp * xrow + cpad) and copy stride
// (XL = C * CS + xpad), both multiples of 8 bf16 (16-B aligned pieces), chosen by the bank model
// above: the plain layout put all KW copies of a combo row on the same banks (5-way conflicts on
// the BinCNN's conv2).  Memoised per shape.
static void b3_filt_copy_layout(B3Filt* d) {
  struct Key { int C, Hp, xrow, KH, KW, OH, OWq, Kp; };
  static std::vector<std::pair<Key, std::pair<int, int>>> memo;
  const Key key{d->C, d->Hp, d->xrow, d->KH, d->KW, d->OH, d->OWq, d->Kp};
  for (const auto& e : memo)
    if (std::memcmp(&e.first, &key, sizeof(Key)) == 0) {
      d->CS = e.second.first;
      d->XL = e.second.second;
      return;
    }
  const int ideal = 4 * std::min(d->Kp / 32, 4) * d->ntn;   // every read conflict-free
  int best = -1, bcs = d->Hp * d->xrow, bxl = d->C * d->Hp * d->xrow;
  for (int cpad = 0; cpad < 64 && best != ideal; cpad += 8)
    for (int xpad = 0; xpad < 256 && best != ideal; xpad += 8) {
      const int CS = d->Hp * d->xrow + cpad, XL = d->C * CS + xpad;
      const int c = b3_filt_b_cycles(*d, CS, XL);
      if (best < 0 || c < best) {
        best = c;
        bcs = CS;
        bxl = XL;
      }
    }
  d->CS = bcs;
  d->XL = bxl;
  memo.push_back({key, {bcs, bxl}});
}

// bf16x3 filter kernel: the input must be exact in bf16 -- binarised (the BinCNN's layers both are)
inline bool b3_filt_geom(const ConvShape& s, int binarize, B3Filt* g, int64_t* lds) {
  if (!(binarize && s.groups == 1 && s.stride == 1 && s.dil == 1 && s.Co <= 64 && s.pad <= s.KH - 1 &&
        s.pad <= s.KW - 1))
    return false;
  B3Filt d;
  d.C = (int)s.C; d.H = (int)s.H; d.W = (int)s.W; d.Co = (int)s.Co; d.KH = (int)s.KH; d.KW = (int)s.KW;
  d.OH = (int)s.OH; d.OW = (int)s.OW; d.pad = s.pad;
  d.Hp = d.H + 2 * d.pad;
  d.OWq = (int)round_up(d.OW, 8);
  d.Co16 = (int)round_up(d.Co, 16);
  d.NA = d.Co16 / 16;
  d.ncombo = d.C * d.KH * d.KW;
  d.ntn = (d.ncombo + 15) / 16;
  d.WT = d.ntn >= 8 ? 8 : (d.ntn >= 4 ? 4 : (d.ntn >= 2 ? 2 : 1));
  d.KS = B3_W / d.WT;
  d.Kp = (int)round_up((int64_t)d.OH * d.OWq, 32 * d.KS);
  d.Kd = d.Kp + 16;   // = 16 (mod 32): conflict-free A reads (as B3Data::ws)
  d.xrow = d.OWq;
  d.Wh = (int)round_up((int64_t)d.OWq + d.KW - 1, 8);   // xh columns read: 8q + kw + j < OWq + KW - 1
  if ((d.ntn + d.WT - 1) / d.WT > 8) return false;
  if ((int64_t)d.C * d.H * d.W >= (1 << 20) || (int64_t)d.Co * d.OH * d.OW >= (1 << 20)) return false;
  b3_filt_copy_layout(&d);
  // rows read: oh + kh < OH + KH - 1 <= Hp (stride 1, pad <= K-1)
  *lds = (int64_t)3 * d.Co16 * d.Kd * 2 + (int64_t)d.KW * d.XL * 2 +
         round_up((int64_t)d.C * d.Hp * d.Wh, 8) * 2 + (int64_t)d.Co16 * (d.Kp / 8) * 4;
  *g = d;
  return *lds <= kMaxTileLds;
}

inline bool mf_filt_geom(const ConvShape& s, MfFilt* g, int64_t* lds) {
  if (!(s.groups == 1 && s.stride == 1 && s.dil == 1 && s.Co <= 64)) return false;
  MfFilt d;
  d.C = (int)s.C; d.H = (int)s.H; d.W = (int)s.W; d.Co = (int)s.Co; d.KH = (int)s.KH; d.KW = (int)s.KW;
  d.OH = (int)s.OH; d.OW = (int)s.OW; d.pad = s.pad;
  d.Hp = d.H + 2 * d.pad; d.Wp = d.W + 2 * d.pad;
  d.P = d.OH * d.OW;
  d.Co16 = (int)round_up(d.Co, 16);
  d.ncombo = d.C * d.KH * d.KW;
  d.ntn = (d.ncombo + 15) / 16;
  d.ntiles = (d.Co16 / 16) * d.ntn;
  d.WT = d.ntiles >= 4 ? 4 : (d.ntiles >= 2 ? 2 : 1);
  d.KS = 4 / d.WT;
  d.Pp = (int)round_up(d.P, 4 * d.KS);
  if ((d.ntiles + d.WT - 1) / d.WT > 16) return false;
  if ((int64_t)d.C * d.H * d.W >= (1 << 20) || (int64_t)d.Co * d.P >= (1 << 20)) return false;
  // every gathered x index stays inside the padded image: oh + kh < Hp, ow + kw < Wp
  if (d.OH - 1 + d.KH - 1 >= d.Hp || d.OW - 1 + d.KW - 1 >= d.Wp) return false;
  *lds = (round_up((int64_t)d.C * d.Hp * d.Wp, 4) + (int64_t)d.Co16 * d.Pp + d.Pp) * 4;
  *g = d;
  return *lds <= kMaxTileLds;
}

// Launch a tiled kernel with `lds` dynamic bytes (lifting the 64 KiB default cap when needed).
#define BNN_TILE_LAUNCH(KER, ...) \
  do { allow_lds(KER, (int64_t)lds); hipLaunchKernelGGL(KER, __VA_ARGS__); } while (0)

constexpr int FILTER_SPB = 8;  // samples per bwd_filter workgroup

int64_t tile_filter_parts(const ConvShape& s) {
  const int ncombo = (int)(s.C * s.KH * s.KW);
  const int nphase = TILE_T / ncombo > 0 ? TILE_T / ncombo : 1;
  return ((s.N + FILTER_SPB - 1) / FILTER_SPB) * nphase;
}
}  // namespace
}  // namespace bnn

using namespace bnn;

#ifndef BNN_CONV_POPC_DEFAULT
#define BNN_CONV_POPC_DEFAULT 0
#endif

// 1 (default): backward data on the bf16x3 MFMA kernel, backward filter / forward on the f32-MFMA
// and int8-MFMA implicit-GEMM kernels, where the shape allows; 2: the f32-MFMA backward data
// kernel instead of bf16x3; 0: the VALU LDS-tiled / generic kernels (the parity tests' cross-checks).
static int g_conv_mfma = 1;

// 1 (default): a one-input-channel layer's filter gradient on the VALU kernel (conv_bwd_filter_c1_k);
// 0: the MFMA / tiled kernels as for any other layer
static int g_conv_c1f = 1;

// The binarised-input forward's engine (bnn_conv_popc.hip): 1 = the VALU popcount kernels where their
// geometry allows (C == 16 or C == 1), 0 = the int8-MFMA / dot4 kernels.  Default: set from the
// measured times of both on the BinCNN's layers (DESIGN.md §6 "Conv engines").
static int g_conv_popc = BNN_CONV_POPC_DEFAULT;

namespace bnn {
bool popc_fwd_ok(int64_t N, int64_t C, int64_t H, int64_t W, int64_t Co, int64_t KH, int64_t KW, int stride, int pad,
                 int dil, int groups);
int64_t popc_wpack_words(int64_t Co, int64_t C, int64_t K);
int popc_fwd_launch(const float* x, const float* w_latent, const float* bias, void* y, int yfmt, int64_t N, int64_t C,
                    int64_t H, int64_t W, int64_t Co, int64_t K, int pad, uint32_t* wpk, hipStream_t st);
}  // namespace bnn

BNN_API int bnn_conv_set_popc(int32_t on) {
  if (on < 0) return g_conv_popc;      // query
  g_conv_popc = on != 0;
  return 0;
}

// The popcount engine's packed weight words: one device buffer per (device, stream), so launches on
// different streams never share one.  A buffer only grows outside graph capture (the eager warm-up
// step before a capture sizes it), and a buffer that was outgrown is retired, never freed: a HIP
// graph captured earlier may still hold its pointer and write it on replay.
static uint32_t* popc_wpack_buffer(int64_t words, hipStream_t st) {
  struct Buf {
    uint32_t* p;
    int64_t cap;
  };
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, Buf> bufs;
  static std::vector<uint32_t*> retired;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  Buf& b = bufs[{dev, st}];
  if (b.cap >= words) return b.p;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) return nullptr;
  const int64_t n = std::max<int64_t>(words, 8192);
  uint32_t* p = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&p), (size_t)n * sizeof(uint32_t)) != hipSuccess) return nullptr;
  if (b.p != nullptr) retired.push_back(b.p);
  b = Buf{p, n};
  return p;
}

static bool popc_pick(const ConvShape& s, int binarize) {
  return binarize && g_conv_popc &&
         popc_fwd_ok(s.N, s.C, s.H, s.W, s.Co, s.KH, s.KW, s.stride, s.pad, s.dil, s.groups);
}

static int popc_run(const ConvShape& s, const float* x, const float* w, const float* bias, void* y, int yfmt,
                    hipStream_t st, const char* who) {
  uint32_t* wpk = popc_wpack_buffer(popc_wpack_words(s.Co, s.C, s.KH), st);
  if (wpk == nullptr) {
    set_error("%s: no popcount weight buffer (first use inside a graph capture, or out of memory)", who);
    return kErrInval;
  }
  return popc_fwd_launch(x, w, bias, y, yfmt, s.N, s.C, s.H, s.W, s.Co, s.KH, s.pad, wpk, st);
}

BNN_API int bnn_conv_set_c1_filter(int32_t on) {
  g_conv_c1f = on != 0;
  return 0;
}

inline bool c1_filt_geom(const ConvShape& s, C1Filt* g, int64_t* lds) {
  if (s.C != 1 || s.groups != 1 || s.stride != 1 || s.dil != 1 || !((s.KH == 5 && s.KW == 5) || (s.KH == 3 && s.KW == 3)) ||
      s.OW % 4 != 0 || s.Co > 64 || C1F_T % s.Co != 0 || s.pad > s.KH - 1 || s.H * s.W > C1F_PX * C1F_T)
    return false;
  const int NX = ((int)s.KW + 6) / 4;
  // row pitch: XW / 4 = OW / 4 (mod 16), so the 16 consecutive units a ds_read_b128 lane group reads
  // (~2.3 rows of OW / 4 units) land on 16 distinct 4-bank quads -- conflict-free (a 32-float pitch
  // put rows 0 and 2 on the same banks)
  const int base4 = (int)(round_up(std::max<int64_t>(s.W + 2 * s.pad, s.OW - 4 + 4 * NX), 4) / 4);
  const int uq = (int)(s.OW / 4) % 16;
  const int XW = 4 * (uq + 16 * ((base4 - uq + 15) / 16));
  const int XR = (int)std::max<int64_t>(s.H + 2 * s.pad, s.OH + s.KH - 1);
  const int64_t bytes = std::max<int64_t>(2 * (int64_t)XR * XW, (int64_t)C1F_T * (s.KH * s.KW + 1)) *
                        (int64_t)sizeof(float);
  if (bytes > kMaxTileLds) return false;
  *g = C1Filt{(int)s.H, (int)s.W, (int)s.OH, (int)s.OW, (int)s.Co, s.pad, XR, XW, (int)(C1F_T / s.Co)};
  *lds = bytes;
  return true;
}

BNN_API int bnn_conv_set_mfma(int32_t mode) {
  g_conv_mfma = mode < 0 ? 1 : (mode > 2 ? 1 : mode);
  return 0;
}

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
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (popc_pick(s, binarize_input)) return popc_run(s, x, w_latent, bias, y, 0, st, "bnn_conv2d_fwd");
  MfFwd mf;
  int64_t mlds = 0;
  if (binarize_input && g_conv_mfma && mf_fwd_geom(s, &mf, &mlds)) {
    const size_t lds = (size_t)mlds;
    const dim3 grid((unsigned)((N + FW_IPB - 1) / FW_IPB));
    const int cot = (mf.Co + 15) / 16;
    if (cot == 1) BNN_TILE_LAUNCH(conv_fwd_i8mfma_k<1>, grid, dim3(MF_T), lds, st, x, w_latent, bias, y, N, mf);
    else if (cot == 2) BNN_TILE_LAUNCH(conv_fwd_i8mfma_k<2>, grid, dim3(MF_T), lds, st, x, w_latent, bias, y, N, mf);
    else BNN_TILE_LAUNCH(conv_fwd_i8mfma_k<4>, grid, dim3(MF_T), lds, st, x, w_latent, bias, y, N, mf);
    return check_launch("bnn_conv2d_fwd");
  }
  if (binarize_input && g_conv_mfma && s.C == 1 && s.KW <= 8 && tile_geom_ok(s)) {
    const TileGeo g = geo(s);
    const int Wq = (int)round_up(g.Wp, 4), kwg = s.KW <= 4 ? 1 : 2;
    const size_t lds = (size_t)(s.KH * kwg * pick_co(Co) * 4 + g.Hp * Wq + 16);
#define BNN_C1(CO_, KG_) BNN_TILE_LAUNCH((conv_fwd_bin_c1_k<CO_, KG_>), dim3(N), dim3(TILE_T), lds, st, x, w_latent, bias, y, g, Wq)
    switch (pick_co(Co) * 4 + kwg) {
      case 8 * 4 + 1: BNN_C1(8, 1); break;
      case 8 * 4 + 2: BNN_C1(8, 2); break;
      case 16 * 4 + 1: BNN_C1(16, 1); break;
      case 16 * 4 + 2: BNN_C1(16, 2); break;
      case 32 * 4 + 1: BNN_C1(32, 1); break;
      case 32 * 4 + 2: BNN_C1(32, 2); break;
      case 64 * 4 + 1: BNN_C1(64, 1); break;
      default: BNN_C1(64, 2); break;
    }
#undef BNN_C1
    return check_launch("bnn_conv2d_fwd");
  }
  if (tile_geom_ok(s) && fwd_tile_lds(s, binarize_input != 0) <= kMaxTileLds) {
    const TileGeo g = geo(s);
    const int CO = pick_co(Co);
    const size_t lds = (size_t)fwd_tile_lds(s, binarize_input != 0);
    if (binarize_input) {
      switch (CO) {
        case 8: BNN_TILE_LAUNCH(conv_fwd_bin_tile_k<8>, dim3(N), dim3(TILE_T), lds, st, x, w_latent, bias, y, g); break;
        case 16: BNN_TILE_LAUNCH(conv_fwd_bin_tile_k<16>, dim3(N), dim3(TILE_T), lds, st, x, w_latent, bias, y, g); break;
        case 32: BNN_TILE_LAUNCH(conv_fwd_bin_tile_k<32>, dim3(N), dim3(TILE_T), lds, st, x, w_latent, bias, y, g); break;
        default: BNN_TILE_LAUNCH(conv_fwd_bin_tile_k<64>, dim3(N), dim3(TILE_T), lds, st, x, w_latent, bias, y, g); break;
      }
    } else {
      switch (CO) {
        case 8: BNN_TILE_LAUNCH(conv_fwd_f32_tile_k<8>, dim3(N), dim3(TILE_T), lds, st, x, w_latent, bias, y, g); break;
        case 16: BNN_TILE_LAUNCH(conv_fwd_f32_tile_k<16>, dim3(N), dim3(TILE_T), lds, st, x, w_latent, bias, y, g); break;
        case 32: BNN_TILE_LAUNCH(conv_fwd_f32_tile_k<32>, dim3(N), dim3(TILE_T), lds, st, x, w_latent, bias, y, g); break;
        default: BNN_TILE_LAUNCH(conv_fwd_f32_tile_k<64>, dim3(N), dim3(TILE_T), lds, st, x, w_latent, bias, y, g); break;
      }
    }
    return check_launch("bnn_conv2d_fwd");
  }
  hipLaunchKernelGGL(conv_fwd_k, dim3(grid_for(total)), dim3(256), 0, st, x, binarize_input, w_latent, bias, y, s);
  return check_launch("bnn_conv2d_fwd");
}

template <typename OT>
static void launch_c1_q(const ConvShape& s, const float* x, const float* w_latent, OT* y, hipStream_t st) {
  const TileGeo g = geo(s);
  const int Wq = (int)round_up(g.Wp, 4), kwg = s.KW <= 4 ? 1 : 2;
  const size_t lds = (size_t)(s.KH * kwg * pick_co(s.Co) * 4 + g.Hp * Wq + 16);
  const dim3 grid((unsigned)s.N);
#define BNN_C1Q(CO_, KG_) \
  BNN_TILE_LAUNCH((conv_fwd_bin_c1_k<CO_, KG_, OT>), grid, dim3(TILE_T), lds, st, x, w_latent, nullptr, y, g, Wq)
  switch (pick_co(s.Co) * 4 + kwg) {
    case 8 * 4 + 1: BNN_C1Q(8, 1); break;
    case 8 * 4 + 2: BNN_C1Q(8, 2); break;
    case 16 * 4 + 1: BNN_C1Q(16, 1); break;
    case 16 * 4 + 2: BNN_C1Q(16, 2); break;
    case 32 * 4 + 1: BNN_C1Q(32, 1); break;
    case 32 * 4 + 2: BNN_C1Q(32, 2); break;
    case 64 * 4 + 1: BNN_C1Q(64, 1); break;
    default: BNN_C1Q(64, 2); break;
  }
#undef BNN_C1Q
}

// Which compact-output kernel bnn_conv2d_fwd_q runs for a shape: 1 = int8 MFMA, 2 = single-channel
// dot4, 3 = popcount, 0 = none (the shape is refused).  Shared by the entry and its query so they cannot disagree.
static int fwd_q_path(const ConvShape& s, MfFwd* mf, int64_t* mlds) {
  if (popc_pick(s, 1)) return 3;
  if (g_conv_mfma && mf_fwd_geom(s, mf, mlds)) return 1;
  if (g_conv_mfma && s.C == 1 && s.KW <= 8 && tile_geom_ok(s)) return 2;
  return 0;
}

static bool fwd_q_args_ok(int32_t yfmt, int64_t N, int64_t C, int64_t H, int64_t W, int64_t Co, int64_t KH,
                          int64_t KW, int32_t stride, int32_t pad, int32_t dil, int32_t groups, ConvShape* s) {
  return (yfmt == 1 || yfmt == 2) && make_shape(N, C, H, W, Co, KH, KW, stride, pad, dil, groups, s) &&
         C * KH * KW <= (yfmt == 1 ? 127 : 32767);
}

// 1 when bnn_conv2d_fwd_q accepts the shape (same geometry checks, nothing launched), else 0: the
// host asks before it emits a compact conv output, so an unsupported shape takes the fp32 output
// instead of failing.
BNN_API int bnn_conv2d_fwd_q_ok(int32_t yfmt, int64_t N, int64_t C, int64_t H, int64_t W, int64_t Co, int64_t KH,
                                int64_t KW, int32_t stride, int32_t pad, int32_t dil, int32_t groups) {
  ConvShape s;
  if (!fwd_q_args_ok(yfmt, N, C, H, W, Co, KH, KW, stride, pad, dil, groups, &s)) return 0;
  MfFwd mf;
  int64_t mlds = 0;
  return fwd_q_path(s, &mf, &mlds) != 0 ? 1 : 0;
}

// The binary-input forward writing the exact integer sums (no bias) as int8 (yfmt 1: C*KH*KW <= 127)
// or int16 (yfmt 2: <= 32767) for a BatchNorm2d that reads fl(I + bias) (bnn_bn2d_*_q): the
// int8-MFMA kernel (C % 16 == 0) or the single-channel dot4 kernel; other shapes are refused
// (bnn_conv2d_fwd_q_ok tells which).
BNN_API int bnn_conv2d_fwd_q(const float* x, const float* w_latent, void* y, int32_t yfmt, int64_t N, int64_t C,
                             int64_t H, int64_t W, int64_t Co, int64_t KH, int64_t KW, int32_t stride, int32_t pad,
                             int32_t dil, int32_t groups, void* stream) {
  ConvShape s;
  if (!x || !w_latent || !y || !fwd_q_args_ok(yfmt, N, C, H, W, Co, KH, KW, stride, pad, dil, groups, &s)) {
    set_error("bnn_conv2d_fwd_q: bad arguments (yfmt 1 needs C*KH*KW <= 127, 2 <= 32767)");
    return kErrInval;
  }
  if (N * Co * s.OH * s.OW == 0) return 0;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  MfFwd mf;
  int64_t mlds = 0;
  const int path = fwd_q_path(s, &mf, &mlds);
#define BNN_QOUT(OT_, ...) do { if (yfmt == 1) { using OT_ = int8_t; __VA_ARGS__; } else { using OT_ = int16_t; __VA_ARGS__; } } while (0)
  if (path == 1) {
    const size_t lds = (size_t)mlds;
    const dim3 grid((unsigned)((N + FW_IPB - 1) / FW_IPB));
    const int cot = (mf.Co + 15) / 16;
    BNN_QOUT(OT, {
      OT* yo = reinterpret_cast<OT*>(y);
      if (cot == 1) BNN_TILE_LAUNCH((conv_fwd_i8mfma_k<1, OT>), grid, dim3(MF_T), lds, st, x, w_latent, nullptr, yo, N, mf);
      else if (cot == 2) BNN_TILE_LAUNCH((conv_fwd_i8mfma_k<2, OT>), grid, dim3(MF_T), lds, st, x, w_latent, nullptr, yo, N, mf);
      else BNN_TILE_LAUNCH((conv_fwd_i8mfma_k<4, OT>), grid, dim3(MF_T), lds, st, x, w_latent, nullptr, yo, N, mf);
    });
    return check_launch("bnn_conv2d_fwd_q");
  }
  if (path == 3) return popc_run(s, x, w_latent, nullptr, y, yfmt, st, "bnn_conv2d_fwd_q");
  if (path == 2) {
    if (yfmt == 1) launch_c1_q<int8_t>(s, x, w_latent, reinterpret_cast<int8_t*>(y), st);
    else launch_c1_q<int16_t>(s, x, w_latent, reinterpret_cast<int16_t*>(y), st);
    return check_launch("bnn_conv2d_fwd_q");
  }
#undef BNN_QOUT
  set_error("bnn_conv2d_fwd_q: no compact-output kernel for this shape (C %% 16 == 0 up to 64, or C == 1)");
  return kErrInval;
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
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  B3Data bd;
  int64_t blds = 0;
  if (g_conv_mfma == 1 && b3_data_geom(s, &bd, &blds)) {
    const size_t lds = (size_t)blds;
    const int ipb = b3_ipb(N);
    const dim3 grid((unsigned)((N + ipb - 1) / ipb));
    const int per_wave = (bd.ntile_pix + B3_W - 1) / B3_W;
#define BNN_B3D(NT_, MT_) BNN_TILE_LAUNCH((conv_bwd_data_bf3_k<NT_, MT_>), grid, dim3(B3_T), lds, st, dy, w_latent, dx, N, bd, ipb)
    if (bd.C <= 16) {
      if (per_wave <= 1) BNN_B3D(1, 1); else if (per_wave <= 2) BNN_B3D(1, 2); else if (per_wave <= 4) BNN_B3D(1, 4);
      else if (per_wave <= 8) BNN_B3D(1, 8); else BNN_B3D(1, 16);
    } else {
      if (per_wave <= 1) BNN_B3D(2, 1); else if (per_wave <= 2) BNN_B3D(2, 2); else if (per_wave <= 4) BNN_B3D(2, 4);
      else if (per_wave <= 8) BNN_B3D(2, 8); else BNN_B3D(2, 16);
    }
#undef BNN_B3D
    return check_launch("bnn_conv2d_bwd_data");
  }
  MfData md;
  int64_t mlds = 0;
  if (g_conv_mfma && mf_data_geom(s, &md, &mlds)) {
    const size_t lds = (size_t)mlds;
    const dim3 grid((unsigned)((N + MF_IPB - 1) / MF_IPB));
    const int per_wave = (md.ntile_pix + 3) / 4;
#define BNN_MFD(NT_, MT_) BNN_TILE_LAUNCH((conv_bwd_data_mfma_k<NT_, MT_>), grid, dim3(MF_T), lds, st, dy, w_latent, dx, N, md)
    if (md.CIp == 16) {
      if (per_wave <= 1) BNN_MFD(1, 1); else if (per_wave <= 2) BNN_MFD(1, 2); else if (per_wave <= 4) BNN_MFD(1, 4);
      else if (per_wave <= 8) BNN_MFD(1, 8); else if (per_wave <= 13) BNN_MFD(1, 13); else BNN_MFD(1, 16);
    } else {
      if (per_wave <= 1) BNN_MFD(2, 1); else if (per_wave <= 2) BNN_MFD(2, 2); else if (per_wave <= 4) BNN_MFD(2, 4);
      else if (per_wave <= 8) BNN_MFD(2, 8); else BNN_MFD(2, 16);
    }
#undef BNN_MFD
    return check_launch("bnn_conv2d_bwd_data");
  }
  if (tile_geom_ok(s) && bwd_data_tile_lds(s) <= kMaxTileLds) {
    const TileGeo g = geo(s);
    const int CI = pick_co(C);
    const size_t lds = (size_t)bwd_data_tile_lds(s);
    switch (CI) {
      case 8: BNN_TILE_LAUNCH(conv_bwd_data_tile_k<8>, dim3(N), dim3(TILE_T), lds, st, dy, w_latent, dx, g); break;
      case 16: BNN_TILE_LAUNCH(conv_bwd_data_tile_k<16>, dim3(N), dim3(TILE_T), lds, st, dy, w_latent, dx, g); break;
      case 32: BNN_TILE_LAUNCH(conv_bwd_data_tile_k<32>, dim3(N), dim3(TILE_T), lds, st, dy, w_latent, dx, g); break;
      default: BNN_TILE_LAUNCH(conv_bwd_data_tile_k<64>, dim3(N), dim3(TILE_T), lds, st, dy, w_latent, dx, g); break;
    }
    return check_launch("bnn_conv2d_bwd_data");
  }
  hipLaunchKernelGGL(conv_bwd_data_k, dim3(grid_for(total)), dim3(256), 0, st, dy, w_latent, dx, s);
  return check_launch("bnn_conv2d_bwd_data");
}

// Host-only plan query (no GPU): the bf16x3 backward kernels' LDS layouts for a shape --
// out[0..3] = data kernel (ps, ws, rowt, lds bytes) or -1s, out[4..8] = filter kernel (Kd, CS, XL,
// lds bytes, modelled LDS cycles of its B reads per ds_read_b128 x 100; 400 = conflict-free) or -1s.
BNN_API int bnn_conv_bf3_plan(int64_t N, int64_t C, int64_t H, int64_t W, int64_t Co, int64_t KH, int64_t KW,
                              int32_t stride, int32_t pad, int32_t dil, int32_t groups, int64_t* out) {
  ConvShape s;
  if (!out || !make_shape(std::max<int64_t>(N, 1), C, H, W, Co, KH, KW, stride, pad, dil, groups, &s)) {
    set_error("bnn_conv_bf3_plan: bad arguments");
    return kErrInval;
  }
  for (int i = 0; i < 9; ++i) out[i] = -1;
  B3Data bd;
  int64_t lds = 0;
  if (b3_data_geom(s, &bd, &lds)) {
    out[0] = bd.ps;
    out[1] = bd.ws;
    out[2] = bd.rowt;
    out[3] = lds;
  }
  B3Filt bf;
  if (b3_filt_geom(s, 1, &bf, &lds)) {
    out[4] = bf.Kd;
    out[5] = bf.CS;
    out[6] = bf.XL;
    out[7] = lds;
    const int reads = std::min(bf.Kp / 32, 4) * bf.ntn;
    out[8] = 100 * (int64_t)b3_filt_b_cycles(bf, bf.CS, bf.XL) / reads;
  }
  return 0;
}

BNN_API int64_t bnn_conv2d_bwd_filter_workspace(int64_t N, int64_t C, int64_t Co, int64_t KH,
                                                int64_t KW, int32_t groups) {
  if (groups <= 0 || C % groups != 0) return 0;
  const int64_t nelem = Co * (C / groups) * KH * KW + Co;
  const int64_t generic = filter_chunks(std::max<int64_t>(N, 1), nelem) * nelem * (int64_t)sizeof(double);
  // tiled path: float partials [parts][CO*ncombo + CO]
  const int CO = pick_co(Co);
  const int ncombo = (int)(C * KH * KW);
  const int nphase = TILE_T / ncombo > 0 ? TILE_T / ncombo : 1;
  const int64_t parts = ((std::max<int64_t>(N, 1) + FILTER_SPB - 1) / FILTER_SPB) * nphase;
  const int64_t tnel = (int64_t)CO * ncombo + CO;
  const int64_t tiled = round_up(parts * tnel * (int64_t)sizeof(float), 256) +
                        filter_slices(parts) * tnel * (int64_t)sizeof(double);
  const int64_t mparts = ((std::max<int64_t>(N, 1) + MF_IPB - 1) / MF_IPB) * B3_W;   // k-slices <= 8
  const int64_t mnel = Co * ncombo + Co;
  const int64_t mfma = round_up(mparts * mnel * (int64_t)sizeof(float), 256) +
                       filter_slices(mparts) * mnel * (int64_t)sizeof(double);
  const int64_t cparts = (std::max<int64_t>(N, 1) + C1F_SPB - 1) / C1F_SPB;   // conv_bwd_filter_c1_k
  const int64_t c1 = round_up(cparts * mnel * (int64_t)sizeof(float), 256) +
                     filter_slices(cparts) * mnel * (int64_t)sizeof(double);
  return std::max(std::max(generic, tiled), std::max(mfma, c1));
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
  C1Filt cf;
  int64_t clds = 0;
  if (N > 0 && g_conv_c1f && g_conv_mfma != 0 && c1_filt_geom(s, &cf, &clds)) {
    const int64_t nblk = (N + C1F_SPB - 1) / C1F_SPB;
    const int64_t nel = nw + Co;
    float* part = reinterpret_cast<float*>(work);
    const size_t lds = (size_t)clds;
    if (KH == 5) BNN_TILE_LAUNCH((conv_bwd_filter_c1_k<5, 5>), dim3((unsigned)nblk), dim3(C1F_T), lds, st, dy, x,
                                 binarize_input, part, N, cf, db != nullptr);
    else BNN_TILE_LAUNCH((conv_bwd_filter_c1_k<3, 3>), dim3((unsigned)nblk), dim3(C1F_T), lds, st, dy, x,
                         binarize_input, part, N, cf, db != nullptr);
    const int64_t nsl = filter_slices(nblk);
    double* slice = reinterpret_cast<double*>(reinterpret_cast<char*>(work) +
                                              round_up(nblk * nel * (int64_t)sizeof(float), 256));
    hipLaunchKernelGGL(conv_filter_tile_reduce1_k, dim3((unsigned)((nel + 255) / 256), (unsigned)nsl), dim3(256), 0,
                       st, part, nblk, nel, nsl, slice);
    hipLaunchKernelGGL(conv_filter_tile_reduce2_k, dim3((unsigned)((nel + 255) / 256)), dim3(256), 0, st, slice,
                       nsl, (int)Co, (int)(KH * KW), (int)Co, dw, db);
    return check_launch("bnn_conv2d_bwd_filter");
  }
  B3Filt bf;
  int64_t blds = 0;
  if (N > 0 && g_conv_mfma == 1 && b3_filt_geom(s, binarize_input, &bf, &blds)) {
    const int ipb = b3_ipb(N);
    const int64_t nblk = (N + ipb - 1) / ipb;
    const int64_t parts = nblk * bf.KS;
    const int64_t nel = (int64_t)Co * bf.ncombo + Co;
    float* part = reinterpret_cast<float*>(work);
    const size_t lds = (size_t)blds;
    const int per_wave = (bf.ntn + bf.WT - 1) / bf.WT;
#define BNN_B3F(NA_, MT_) BNN_TILE_LAUNCH((conv_bwd_filter_bf3_k<NA_, MT_>), dim3((unsigned)nblk), dim3(B3_T), lds, st, dy, x, binarize_input, part, N, bf, db != nullptr, ipb)
#define BNN_B3F_MT(NA_) \
    if (per_wave <= 1) BNN_B3F(NA_, 1); else if (per_wave <= 2) BNN_B3F(NA_, 2); else if (per_wave <= 4) BNN_B3F(NA_, 4); \
    else BNN_B3F(NA_, 8);
    if (bf.NA == 1) { BNN_B3F_MT(1) } else if (bf.NA == 2) { BNN_B3F_MT(2) } else if (bf.NA == 3) { BNN_B3F_MT(3) } else { BNN_B3F_MT(4) }
#undef BNN_B3F_MT
#undef BNN_B3F
    const int64_t nsl = filter_slices(parts);
    double* slice = reinterpret_cast<double*>(reinterpret_cast<char*>(work) +
                                              round_up(parts * nel * (int64_t)sizeof(float), 256));
    hipLaunchKernelGGL(conv_filter_tile_reduce1_k, dim3((unsigned)((nel + 255) / 256), (unsigned)nsl), dim3(256), 0,
                       st, part, parts, nel, nsl, slice);
    hipLaunchKernelGGL(conv_filter_tile_reduce2_k, dim3((unsigned)((nel + 255) / 256)), dim3(256), 0, st, slice,
                       nsl, (int)Co, bf.ncombo, (int)Co, dw, db);
    return check_launch("bnn_conv2d_bwd_filter");
  }
  MfFilt mf;
  int64_t mlds = 0;
  if (N > 0 && g_conv_mfma && mf_filt_geom(s, &mf, &mlds)) {
    const int64_t nblk = (N + MF_IPB - 1) / MF_IPB;
    const int64_t parts = nblk * mf.KS;
    const int64_t nel = (int64_t)Co * mf.ncombo + Co;
    float* part = reinterpret_cast<float*>(work);
    const size_t lds = (size_t)mlds;
    const int per_wave = (mf.ntiles + mf.WT - 1) / mf.WT;
#define BNN_MFF(MT_) BNN_TILE_LAUNCH(conv_bwd_filter_mfma_k<MT_>, dim3((unsigned)nblk), dim3(MF_T), lds, st, dy, x, binarize_input, part, N, mf, db != nullptr)
    if (per_wave <= 1) BNN_MFF(1); else if (per_wave <= 2) BNN_MFF(2); else if (per_wave <= 4) BNN_MFF(4);
    else if (per_wave <= 8) BNN_MFF(8); else if (per_wave <= 13) BNN_MFF(13); else BNN_MFF(16);
#undef BNN_MFF
    const int64_t nsl = filter_slices(parts);
    double* slice = reinterpret_cast<double*>(reinterpret_cast<char*>(work) +
                                              round_up(parts * nel * (int64_t)sizeof(float), 256));
    hipLaunchKernelGGL(conv_filter_tile_reduce1_k, dim3((unsigned)((nel + 255) / 256), (unsigned)nsl), dim3(256), 0,
                       st, part, parts, nel, nsl, slice);
    hipLaunchKernelGGL(conv_filter_tile_reduce2_k, dim3((unsigned)((nel + 255) / 256)), dim3(256), 0, st, slice,
                       nsl, (int)Co, mf.ncombo, (int)Co, dw, db);
    return check_launch("bnn_conv2d_bwd_filter");
  }
  if (N > 0 && tile_geom_ok(s) && C * KH * KW <= 2 * TILE_T && filter_tile_lds(s) <= kMaxTileLds) {
    const TileGeo g = geo(s);
    const int CO = pick_co(Co);
    const int ncombo = (int)(C * KH * KW);
    const int64_t nblk = (N + FILTER_SPB - 1) / FILTER_SPB;
    const int64_t parts = tile_filter_parts(s);
    float* part = reinterpret_cast<float*>(work);
    const size_t lds = (size_t)filter_tile_lds(s);
    switch (CO) {
      case 8: BNN_TILE_LAUNCH(conv_bwd_filter_tile_k<8>, dim3((unsigned)nblk), dim3(TILE_T), lds, st, dy, x, binarize_input, part, N, FILTER_SPB, g, db != nullptr); break;
      case 16: BNN_TILE_LAUNCH(conv_bwd_filter_tile_k<16>, dim3((unsigned)nblk), dim3(TILE_T), lds, st, dy, x, binarize_input, part, N, FILTER_SPB, g, db != nullptr); break;
      case 32: BNN_TILE_LAUNCH(conv_bwd_filter_tile_k<32>, dim3((unsigned)nblk), dim3(TILE_T), lds, st, dy, x, binarize_input, part, N, FILTER_SPB, g, db != nullptr); break;
      default: BNN_TILE_LAUNCH(conv_bwd_filter_tile_k<64>, dim3((unsigned)nblk), dim3(TILE_T), lds, st, dy, x, binarize_input, part, N, FILTER_SPB, g, db != nullptr); break;
    }
    const int64_t nel = (int64_t)CO * ncombo + CO;
    const int64_t nsl = filter_slices(parts);
    double* slice = reinterpret_cast<double*>(reinterpret_cast<char*>(work) +
                                              round_up(parts * nel * (int64_t)sizeof(float), 256));
    hipLaunchKernelGGL(conv_filter_tile_reduce1_k, dim3((unsigned)((nel + 255) / 256), (unsigned)nsl), dim3(256), 0,
                       st, part, parts, nel, nsl, slice);
    hipLaunchKernelGGL(conv_filter_tile_reduce2_k, dim3((unsigned)((nel + 255) / 256)), dim3(256), 0, st, slice,
                       nsl, CO, ncombo, (int)Co, dw, db);
    return check_launch("bnn_conv2d_bwd_filter");
  }
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

// 1 when bnn_conv2d_bwd_filter_bn takes the shape: the one-input-channel filter kernel's geometry
// (bnn_conv_set_c1_filter on, the MFMA engines on) with an even OH and OW % 4 == 0
BNN_API int bnn_conv2d_bwd_filter_bn_ok(int64_t N, int64_t C, int64_t H, int64_t W, int64_t Co, int64_t KH,
                                        int64_t KW, int32_t stride, int32_t pad, int32_t dil, int32_t groups) {
  ConvShape s;
  C1Filt cf;
  int64_t lds = 0;
  return (N > 0 && g_conv_c1f && g_conv_mfma != 0 && make_shape(N, C, H, W, Co, KH, KW, stride, pad, dil, groups, &s) &&
          c1_filt_geom(s, &cf, &lds) && s.OH % 2 == 0 && s.OW % 4 == 0)
             ? 1
             : 0;
}

// bnn_conv2d_bwd_filter with dY = the BatchNorm2d(+Hardtanh)+MaxPool2d(2) backward of the pooled
// gradient dyp (bnn_bn2d_bwd_q's dx, never written): z = the conv's compact output (zfmt 1 int8 /
// 2 int16 sums, zbias [Co]), mean / invstd / gamma / beta its BatchNorm's, sg / sgx the sums from
// bnn_bn2d_bwd_stats_q, inv_n = 1 / (N OH OW).  Same shapes as bnn_conv2d_bwd_filter_bn_ok.
BNN_API int bnn_conv2d_bwd_filter_bn(const void* zq, const float* zbias, int32_t zfmt, const float* dyp,
                                     const float* mean, const float* invstd, const float* gamma, const float* beta,
                                     const float* sg, const float* sgx, float inv_n, int32_t hardtanh, const float* x,
                                     int32_t binarize_input, float* dw, float* db, void* work, int64_t N, int64_t C,
                                     int64_t H, int64_t W, int64_t Co, int64_t KH, int64_t KW, int32_t stride,
                                     int32_t pad, int32_t dil, int32_t groups, void* stream) {
  ConvShape s;
  C1Filt cf;
  int64_t clds = 0;
  if (!zq || !dyp || !mean || !invstd || !sg || !sgx || !x || !dw || !work || (zfmt != 1 && zfmt != 2) ||
      !bnn_conv2d_bwd_filter_bn_ok(N, C, H, W, Co, KH, KW, stride, pad, dil, groups) ||
      !make_shape(N, C, H, W, Co, KH, KW, stride, pad, dil, groups, &s) || !c1_filt_geom(s, &cf, &clds) ||
      (reinterpret_cast<uintptr_t>(dyp) & 7) != 0 || (reinterpret_cast<uintptr_t>(zq) & 7) != 0 ||
      N * Co * s.OH * s.OW * zfmt >= (1LL << 31)) {   // the compact sums are read by 32-bit buffer offsets
    set_error("bnn_conv2d_bwd_filter_bn: bad arguments");
    return kErrInval;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t nblk = (N + C1F_SPB - 1) / C1F_SPB;
  const int64_t nw = Co * KH * KW, nel = nw + Co;
  float* part = reinterpret_cast<float*>(work);
  const size_t lds = (size_t)clds;
  const C1Bn bn{X2{zq, zbias}, dyp, mean, invstd, gamma, beta, sg, sgx, inv_n, hardtanh};
#define BNN_C1BN(KH_, XF_) BNN_TILE_LAUNCH((conv_bwd_filter_c1bn_k<KH_, KH_, XF_>), dim3((unsigned)nblk), dim3(C1F_T), \
                                           lds, st, bn, x, binarize_input, part, N, cf, db != nullptr)
  if (KH == 5) {
    if (zfmt == 1) BNN_C1BN(5, 1); else BNN_C1BN(5, 2);
  } else {
    if (zfmt == 1) BNN_C1BN(3, 1); else BNN_C1BN(3, 2);
  }
#undef BNN_C1BN
  const int64_t nsl = filter_slices(nblk);
  double* slice = reinterpret_cast<double*>(reinterpret_cast<char*>(work) +
                                            round_up(nblk * nel * (int64_t)sizeof(float), 256));
  hipLaunchKernelGGL(conv_filter_tile_reduce1_k, dim3((unsigned)((nel + 255) / 256), (unsigned)nsl), dim3(256), 0,
                     st, part, nblk, nel, nsl, slice);
  hipLaunchKernelGGL(conv_filter_tile_reduce2_k, dim3((unsigned)((nel + 255) / 256)), dim3(256), 0, st, slice, nsl,
                     (int)Co, (int)(KH * KW), (int)Co, dw, db);
  return check_launch("bnn_conv2d_bwd_filter_bn");
}
