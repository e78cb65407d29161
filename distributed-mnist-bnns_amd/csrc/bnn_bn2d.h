// BatchNorm2d(+Hardtanh)(+MaxPool2d(2)) element helpers shared by the BatchNorm2d passes
// (bnn_bn.hip) and the conv filter gradient that forms its dY from them (bnn_conv.hip).
#pragma once
#include "bnn_common.h"

#include <type_traits>

namespace bnn {

struct Bn2Chan {   // per-channel affine of the normalisation
  float mu, is, ga, be;
};

__device__ __forceinline__ Bn2Chan bn2_chan(int64_t c, const float* mean, const float* invstd, const float* gamma,
                                            const float* beta) {
  return Bn2Chan{mean[c], invstd[c], gamma ? gamma[c] : 1.f, beta ? beta[c] : 0.f};
}

// One 2x2 pooling window: pre-activation y (before the clamp) of its 4 elements in torch scan
// order (h, w), the max-pool output and the argmax slot.
struct Win {
  float xh[4], y[4];
  float out;
  int arg;
};

__device__ __forceinline__ Win bn2_window(float2 top, float2 bot, const Bn2Chan& k, int hardtanh) {
  Win w;
  const float xs[4] = {top.x, top.y, bot.x, bot.y};
  float best = -__builtin_inff();
  int arg = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    w.xh[j] = (xs[j] - k.mu) * k.is;
    w.y[j] = fmaf(w.xh[j], k.ga, k.be);
    const float v = hardtanh ? fminf(fmaxf(w.y[j], -1.f), 1.f) : w.y[j];
    if (v > best || v != v) {
      best = v;
      arg = j;
    }
  }
  w.out = best;
  w.arg = arg;
  return w;
}

// The NCHW input of a BatchNorm2d pass: fp32 (XF 0), or (XF 1 / 2) the int8 / int16 exact sums I of
// the binary convolution that produced it (bnn_conv2d_fwd_q) plus its per-channel bias, read as
// x = fl(I + bias[c]) -- the value the conv's fp32 epilogue stores, so every result is bit-identical,
// at 1/4 (conv1: |I| <= 25) or 1/2 the bytes of every pass.
struct X2 {
  const void* p;
  const float* bias;
};

template <int XF>
__device__ __forceinline__ float x2_bias(const X2& x, int64_t c) {
  return (XF != 0 && x.bias != nullptr) ? x.bias[c] : 0.f;
}

// Every read of the compact (int8 / int16) conv outputs goes around the reading CU's vector L1
// (BN2_LOADS 1: nt loads, which the compiler still merges into 16-B instructions).  With plain
// loads the BatchNorm2d forward passes returned different statistics from run to run -- never in
// one process alone, in about one step in ten while other processes used the same GPU (the
// two-rank data-parallel tests run that way) -- although the conv sums in memory were identical
// every time; host synchronisations before and between the passes and a 512 MB L2 eviction left it
// so, loads that bypass L1 (agent-scope sc1, round 5) removed it (0 of 156 steps, plain 11 of 156;
// tools/race_trace.py, profiles/r05_race_*.log).  sc1 and nt loads are served by L2 and skip L1
// alone (MI355X_MICROARCH.md, visibility table), so the stale bytes came from the consumer CU's L1:
// the fix belongs to every consumer of freshly written compact data, the forward and backward
// BatchNorm2d passes and conv1's fused filter gradient alike.  BN2_LOADS 0 / 2
// build the plain / sc1-atomic forms (A/B only).
#ifndef BN2_LOADS
#define BN2_LOADS 1
#endif
template <bool COH>
__device__ __forceinline__ uint2 x2_raw8(const void* p) {
  if constexpr (COH && BN2_LOADS == 2) {
    const uint64_t v =
        __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
  } else if constexpr (COH && BN2_LOADS == 1) {
    const v2u v = __builtin_nontemporal_load(reinterpret_cast<const v2u*>(p));
    return make_uint2(v.x, v.y);
  }
  return *reinterpret_cast<const uint2*>(p);
}
template <bool COH>
__device__ __forceinline__ uint32_t x2_raw4(const void* p) {
  if constexpr (COH && BN2_LOADS == 2)
    return __hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else if constexpr (COH && BN2_LOADS == 1)
    return __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(p));
  return *reinterpret_cast<const uint32_t*>(p);
}
template <bool COH, typename T>
__device__ __forceinline__ T x2_raw_small(const T* p) {   // 1 or 2 bytes
  if constexpr (COH && BN2_LOADS == 2)
    return (T)__hip_atomic_load(reinterpret_cast<const typename std::make_unsigned<T>::type*>(p), __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
  else if constexpr (COH && BN2_LOADS == 1)
    return __builtin_nontemporal_load(p);
  return *p;
}

// 4 consecutive elements of one channel plane from flat index idx (a multiple of 4)
template <int XF, bool COH = true>
__device__ __forceinline__ float4 x2_ld4(const X2& x, int64_t idx, float b) {
  if constexpr (XF == 0) {
    return *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(x.p) + idx);
  } else if constexpr (XF == 1) {
    const uint32_t u = x2_raw4<COH>(reinterpret_cast<const int8_t*>(x.p) + idx);
    return make_float4((float)(int8_t)(u & 0xFF) + b, (float)(int8_t)((u >> 8) & 0xFF) + b,
                       (float)(int8_t)((u >> 16) & 0xFF) + b, (float)(int8_t)(u >> 24) + b);
  } else {
    const uint2 u = x2_raw8<COH>(reinterpret_cast<const int16_t*>(x.p) + idx);
    return make_float4((float)(int16_t)(u.x & 0xFFFF) + b, (float)(int16_t)(u.x >> 16) + b,
                       (float)(int16_t)(u.y & 0xFFFF) + b, (float)(int16_t)(u.y >> 16) + b);
  }
}

// 2 consecutive elements (idx even)
template <int XF, bool COH = true>
__device__ __forceinline__ float2 x2_ld2(const X2& x, int64_t idx, float b) {
  if constexpr (XF == 0) {
    return *reinterpret_cast<const float2*>(reinterpret_cast<const float*>(x.p) + idx);
  } else if constexpr (XF == 1) {
    const uint16_t u = (uint16_t)x2_raw_small<COH>(reinterpret_cast<const int16_t*>(reinterpret_cast<const int8_t*>(x.p) + idx));
    return make_float2((float)(int8_t)(u & 0xFF) + b, (float)(int8_t)(u >> 8) + b);
  } else {
    const uint32_t u = x2_raw4<COH>(reinterpret_cast<const int16_t*>(x.p) + idx);
    return make_float2((float)(int16_t)(u & 0xFFFF) + b, (float)(int16_t)(u >> 16) + b);
  }
}

template <int XF, bool COH = true>
__device__ __forceinline__ float x2_ld1(const X2& x, int64_t idx, float b) {
  if constexpr (XF == 0) return reinterpret_cast<const float*>(x.p)[idx];
  else if constexpr (XF == 1) return (float)x2_raw_small<COH>(reinterpret_cast<const int8_t*>(x.p) + idx) + b;
  else return (float)x2_raw_small<COH>(reinterpret_cast<const int16_t*>(x.p) + idx) + b;
}

// The backward of one 2x2 window (bn2d_bwd_apply_k): dz of its 4 elements (torch scan order) from
// the pooled gradient gp routed to the argmax and masked by the Hardtanh, m0 = sum g / n,
// m1 = sum g xhat / n and sc = gamma * invstd.
__device__ __forceinline__ void bn2_window_dz(const Win& w, float gp, float m0, float m1, float sc, int hardtanh,
                                              float (&o)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float g = (j == w.arg && (!hardtanh || (w.y[j] > -1.f && w.y[j] < 1.f))) ? gp : 0.f;
    o[j] = sc * (g - m0 - w.xh[j] * m1);
  }
}

}  // namespace bnn
