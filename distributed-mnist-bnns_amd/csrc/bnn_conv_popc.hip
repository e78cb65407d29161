// The binary convolution's forward on the VALU popcount unit: the second engine north_star asks the
// BinarizeConv2d forward to be built with (models/binarized_modules.py:93-105: input binarised
// unless C == 3, F.conv2d(sign(x), sign(w)) with zero padding, + bias), picked against the int8-MFMA
// / dot4 kernels of bnn_conv.hip by their measured times (DESIGN.md §6 "Conv engines").
//
// Ternary operands (sign(0) = 0: zero padding, exact-zero activations and pixels) are two bit
// planes -- s (x < 0) and z (x != 0) -- and a dot product over a word of taps is
//     sum = popc(z_x & z_w) - 2 popc(z_x & z_w & (s_x ^ s_w))
// (pairs where both are nonzero count +1, those with different signs -1): and, xor, and and two
// accumulating v_bcnt_u32 = 5 VALU per word, exact integer sums.
//
// Two packings, chosen by the channel count:
//   C == 16 (the BinCNN's conv2): a pixel's 16 channels are 16 bits; the 32-bit words pair two
//     horizontally adjacent taps (pixel (h, w) in the low half, (h, w + 1) in the high half), so a
//     5 x 5 window is 5 rows x 3 words (the last word's high half is a zero weight) = 15 words,
//     400 MACs in 75 VALU;
//   C == 1 (conv1 on binarised pixels): an image row is one bit row (padded width <= 32), and a
//     K x K window (K*K <= 32) is ONE word gathered from K rows (ubfe + lshl_or per row), K*K MACs
//     in 5 VALU per output channel.
// One lane per output pixel; the window words sit in registers and are reused across all output
// channels, whose weight words (packed per forward by conv_popc_wpack_k, wave-uniform) are scalar
// loads.  Output: the int16 / int8 sums of bnn_conv2d_fwd_q (the compact hand-off to the fused
// BatchNorm2d) or fp32 + bias (bnn_conv2d_fwd).
#include <algorithm>
#include <type_traits>

#include "bnn_common.h"

namespace bnn {
namespace {

constexpr int PC_T = 256;
constexpr int PC_IPB = 4;      // images per workgroup (C == 16)
constexpr int PC1_IPB = 8;     // images per workgroup (C == 1)

struct PopcShape {
  int N, C, H, W, Co, K, pad, OH, OW;
  int Hp, Wp;        // padded input extent (+1 column for the tap pairs)
};

// Weight words per output channel.  C == 16: [K rows][NJ pair words][2 planes]; C == 1: [2 planes].
// One thread per word pair (C == 16: per (co, kh, j); C == 1: per co), its taps' loads unrolled so
// they are in flight together (a serial walk per channel took 11 us for conv2's 32 channels).
__global__ __launch_bounds__(256) void conv_popc_wpack_k(const float* __restrict__ w, PopcShape s,
                                                        uint32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int K = s.K;
  if (s.C == 1) {
    if (i >= s.Co) return;
    uint32_t sg = 0, nz = 0;
#pragma unroll
    for (int t = 0; t < 32; ++t) {         // tap (kh, kw) at bit K*kh + kw, as the window words
      if (t < K * K) {
        const float v = w[i * K * K + t];
        sg |= (uint32_t)(v < 0.f) << t;
        nz |= (uint32_t)(tsign(v) != 0) << t;   // sign(NaN) = 0, as every ternary kernel
      }
    }
    out[i * 2] = sg;
    out[i * 2 + 1] = nz;
    return;
  }
  const int NJ = (K + 1) / 2;
  if (i >= s.Co * K * NJ) return;
  const int co = i / (K * NJ), r = i - co * (K * NJ), kh = r / NJ, j = r - kh * NJ;
  uint32_t sg = 0, nz = 0;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int kw = 2 * j + half;
    if (kw < K) {
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const float v = w[((co * 16 + c) * K + kh) * K + kw];
        sg |= (uint32_t)(v < 0.f) << (16 * half + c);
        nz |= (uint32_t)(tsign(v) != 0) << (16 * half + c);
      }
    }
  }
  out[i * 2] = sg;
  out[i * 2 + 1] = nz;
}

template <typename OT>
__device__ __forceinline__ void popc_store(OT* y, int64_t i, int sum, const float* bias, int co) {
  if constexpr (std::is_same<OT, float>::value) {
    y[i] = (float)sum + (bias ? bias[co] : 0.f);      // exact sum, then the bias add (:103-105)
  } else {
    y[i] = (OT)sum;
  }
}

// C == 16, K <= 7: workgroup = PC_IPB images.  LDS: per image the 16-channel sign / nonzero words of
// the zero-padded image (u16), then the tap-pair words (u32) the lanes read their windows from.
template <int K, typename OT>
__global__ __launch_bounds__(PC_T) void conv_fwd_popc16_k(const float* __restrict__ x, const uint32_t* __restrict__ wpk,
                                                          const float* __restrict__ bias, OT* __restrict__ y,
                                                          PopcShape s) {
  constexpr int NJ = (K + 1) / 2;
  extern __shared__ __attribute__((aligned(16))) uint32_t pc_smem[];
  const int t = threadIdx.x;
  const int n0 = blockIdx.x * PC_IPB;
  const int nimg = min(PC_IPB, s.N - n0);
  const int HW = s.H * s.W, PP = s.Hp * s.Wp;
  uint16_t* sp = reinterpret_cast<uint16_t*>(pc_smem);                 // [img][Hp][Wp] sign bits
  uint16_t* zp = sp + PC_IPB * PP;                                      // nonzero bits
  uint32_t* s2 = pc_smem + (2 * PC_IPB * PP + 1) / 2;                   // [img][Hp][Wp] pair words
  uint32_t* z2 = s2 + PC_IPB * PP;
  // zero-padded bit images
  for (int i = t; i < PC_IPB * PP; i += PC_T) {
    const int img = i / PP, r = i - img * PP, hp = r / s.Wp, wp = r - hp * s.Wp;
    const int h = hp - s.pad, w = wp - s.pad;
    uint32_t sg = 0, nz = 0;
    if (img < nimg && h >= 0 && h < s.H && w >= 0 && w < s.W) {
      const float* xp = x + ((int64_t)(n0 + img) * 16) * HW + h * s.W + w;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const float v = xp[c * HW];
        sg |= (uint32_t)(v < 0.f) << c;
        nz |= (uint32_t)(tsign(v) != 0) << c;
      }
    }
    sp[i] = (uint16_t)sg;
    zp[i] = (uint16_t)nz;
  }
  __syncthreads();
  for (int i = t; i < PC_IPB * PP; i += PC_T) {
    const int r = i % PP, wp = r % s.Wp;
    const bool last = wp + 1 >= s.Wp;
    s2[i] = (uint32_t)sp[i] | (last ? 0u : (uint32_t)sp[i + 1] << 16);
    z2[i] = (uint32_t)zp[i] | (last ? 0u : (uint32_t)zp[i + 1] << 16);
  }
  __syncthreads();
  const int OHW = s.OH * s.OW;
  for (int p = t; p < nimg * OHW; p += PC_T) {
    const int img = p / OHW, o = p - img * OHW, oh = o / s.OW, ow = o - oh * s.OW;
    uint32_t xs[K][NJ], xz[K][NJ];
#pragma unroll
    for (int kh = 0; kh < K; ++kh)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int i = img * PP + (oh + kh) * s.Wp + ow + 2 * j;
        xs[kh][j] = s2[i];
        xz[kh][j] = z2[i];
      }
    OT* yo = y + (int64_t)(n0 + img) * s.Co * OHW + o;
    for (int co = 0; co < s.Co; ++co) {
      const uint32_t* wc = wpk + co * K * NJ * 2;      // wave-uniform: scalar loads
      uint32_t a1 = 0, a2 = 0;
#pragma unroll
      for (int kh = 0; kh < K; ++kh)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const uint32_t m = xz[kh][j] & wc[(kh * NJ + j) * 2 + 1];
          const uint32_t d = m & (xs[kh][j] ^ wc[(kh * NJ + j) * 2]);
          a1 = __popc(m) + a1;
          a2 = __popc(d) + a2;
        }
      popc_store<OT>(yo, (int64_t)co * OHW, (int)a1 - 2 * (int)a2, bias, co);
    }
  }
}

// C == 1, K*K <= 32, padded width <= 32: workgroup = PC1_IPB images; LDS: one sign and one nonzero
// bit row per padded image row.
template <int K, typename OT>
__global__ __launch_bounds__(PC_T) void conv_fwd_popc1_k(const float* __restrict__ x, const uint32_t* __restrict__ wpk,
                                                         const float* __restrict__ bias, OT* __restrict__ y,
                                                         PopcShape s) {
  __shared__ uint32_t rs[PC1_IPB][40], rz[PC1_IPB][40];
  const int t = threadIdx.x;
  const int n0 = blockIdx.x * PC1_IPB;
  const int nimg = min(PC1_IPB, s.N - n0);
  // bit rows: thread per (image, padded row)
  for (int i = t; i < PC1_IPB * s.Hp; i += PC_T) {
    const int img = i / s.Hp, hp = i - img * s.Hp, h = hp - s.pad;
    uint32_t sg = 0, nz = 0;
    if (img < nimg && h >= 0 && h < s.H) {
      const float* xr = x + ((int64_t)(n0 + img) * s.H + h) * s.W;
      for (int w = 0; w < s.W; ++w) {
        const float v = xr[w];
        sg |= (uint32_t)(v < 0.f) << (w + s.pad);
        nz |= (uint32_t)(tsign(v) != 0) << (w + s.pad);
      }
    }
    rs[img][hp] = sg;
    rz[img][hp] = nz;
  }
  __syncthreads();
  const int OHW = s.OH * s.OW;
  constexpr uint32_t RM = (1u << K) - 1u;
  for (int p = t; p < nimg * OHW; p += PC_T) {
    const int img = p / OHW, o = p - img * OHW, oh = o / s.OW, ow = o - oh * s.OW;
    uint32_t ws = 0, wz = 0;      // the K x K window as one word (row kh at bits K*kh)
#pragma unroll
    for (int kh = 0; kh < K; ++kh) {
      ws |= ((rs[img][oh + kh] >> ow) & RM) << (K * kh);
      wz |= ((rz[img][oh + kh] >> ow) & RM) << (K * kh);
    }
    OT* yo = y + (int64_t)(n0 + img) * s.Co * OHW + o;
    for (int co = 0; co < s.Co; ++co) {
      const uint32_t m = wz & wpk[2 * co + 1];
      const uint32_t d = m & (ws ^ wpk[2 * co]);
      popc_store<OT>(yo, (int64_t)co * OHW, __popc(m) - 2 * __popc(d),
                     bias, co);
    }
  }
}

}  // namespace

// The geometry the popcount engine takes: binarised input, stride 1, dilation 1, one group, square
// kernel K odd with pad <= K - 1; C == 16 (K <= 7) or C == 1 (K*K <= 32, W + 2 pad <= 32).
bool popc_fwd_ok(int64_t N, int64_t C, int64_t H, int64_t W, int64_t Co, int64_t KH, int64_t KW, int stride, int pad,
                 int dil, int groups) {
  if (N <= 0 || stride != 1 || dil != 1 || groups != 1 || KH != KW || KH % 2 == 0 || pad > KH - 1 || Co > 4096)
    return false;
  if (C == 16) return KH <= 7 && (H + 2 * pad) * (W + 2 * pad + 1) * 12 * PC_IPB <= 60000 && H * W > 0;
  if (C == 1) return KH * KH <= 32 && W + 2 * pad <= 32 && H + 2 * pad <= 40;
  return false;
}

int64_t popc_wpack_words(int64_t Co, int64_t C, int64_t K) { return C == 1 ? 2 * Co : Co * K * ((K + 1) / 2) * 2; }

// x [N][C][H][W] fp32, w_latent [Co][C][K][K] fp32 (binarised here), yfmt 0 = fp32 (+ bias), 1 = int8
// sums, 2 = int16 sums; wpk: popc_wpack_words uint32 scratch.
int popc_fwd_launch(const float* x, const float* w_latent, const float* bias, void* y, int yfmt, int64_t N, int64_t C,
                    int64_t H, int64_t W, int64_t Co, int64_t K, int pad, uint32_t* wpk, hipStream_t st) {
  PopcShape s{(int)N, (int)C, (int)H, (int)W, (int)Co, (int)K, pad, (int)(H + 2 * pad - K + 1),
              (int)(W + 2 * pad - K + 1), (int)(H + 2 * pad), (int)(W + 2 * pad + 1)};
  const int64_t nwords = C == 1 ? Co : Co * K * ((K + 1) / 2);
  hipLaunchKernelGGL(conv_popc_wpack_k, dim3((unsigned)((nwords + 255) / 256)), dim3(256), 0, st, w_latent, s, wpk);
#define BNN_POPC(KER, IPB, LDS)                                                                              \
  do {                                                                                                     \
    const dim3 g((unsigned)((N + (IPB) - 1) / (IPB)));                                                     \
    if (yfmt == 0) hipLaunchKernelGGL((KER<KK, float>), g, dim3(PC_T), (LDS), st, x, wpk, bias, (float*)y, s); \
    else if (yfmt == 1) hipLaunchKernelGGL((KER<KK, int8_t>), g, dim3(PC_T), (LDS), st, x, wpk, nullptr, (int8_t*)y, s); \
    else hipLaunchKernelGGL((KER<KK, int16_t>), g, dim3(PC_T), (LDS), st, x, wpk, nullptr, (int16_t*)y, s); \
  } while (0)
  if (C == 16) {
    const size_t lds = (size_t)PC_IPB * s.Hp * s.Wp * 12 + 16;
    switch (K) {
      case 1: { constexpr int KK = 1; BNN_POPC(conv_fwd_popc16_k, PC_IPB, lds); } break;
      case 3: { constexpr int KK = 3; BNN_POPC(conv_fwd_popc16_k, PC_IPB, lds); } break;
      case 5: { constexpr int KK = 5; BNN_POPC(conv_fwd_popc16_k, PC_IPB, lds); } break;
      default: { constexpr int KK = 7; BNN_POPC(conv_fwd_popc16_k, PC_IPB, lds); } break;
    }
  } else {
    switch (K) {
      case 1: { constexpr int KK = 1; BNN_POPC(conv_fwd_popc1_k, PC1_IPB, 0); } break;
      case 3: { constexpr int KK = 3; BNN_POPC(conv_fwd_popc1_k, PC1_IPB, 0); } break;
      default: { constexpr int KK = 5; BNN_POPC(conv_fwd_popc1_k, PC1_IPB, 0); } break;
    }
  }
#undef BNN_POPC
  return check_launch("bnn_conv2d_fwd (popcount)");
}

}  // namespace bnn
