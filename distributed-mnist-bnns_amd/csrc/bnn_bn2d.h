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

// Every read of the compact (int8 / int16) conv outputs is an agent-scope relaxed atomic load
// (global_load ... sc1, 2 to 8 B; 16-B reads are two 8-B loads).  With plain loads the BatchNorm2d
// forward statistics differed from run to run -- never in one process alone, in about one step in
// ten while other processes used the same GPU (the two-rank data-parallel tests run that way) --
// although the conv sums in memory were identical every time (tools/race_trace.py: plain 11 of 156
// steps, profiles/r05_race_*.log).  The atomic form: 0 of 156 (round 5) and 0 of 120 steps (round 6,
// profiles/r06_f_race_trace_atomic.log).  Two other forms failed in round 6: nt loads (the two-rank
// BinCNN test, profiles/r06_c_gpu_tests_a.log) and buffer loads carrying the SAME sc1 bit as the
// atomic loads (6 of 120 steps, profiles/r06_e_race_trace_sc1buf.log) -- so the L1 bypass the sc1
// bit encodes is not by itself what removes the difference, and the mechanism is not identified
// (DESIGN.md §8 lists the evidence).  The consumers: the forward and backward BatchNorm2d passes and
// conv1's fused filter gradient; the rows kernels stage their row pairs through LDS (Rows16 below)
// so that these loads stay address-ordered across the lanes.  BN2_LOADS: 2 atomic (default), 0 plain, 1 sc1 buffer loads, 3 nt
// loads -- A/B only.  Compact buffers are < 2 GB (host checks).
#ifndef BN2_LOADS
#define BN2_LOADS 2
#endif
constexpr int BN2_SC1 = 16;   // buffer-instruction aux bits: sc1

__device__ __forceinline__ __amdgpu_buffer_rsrc_t x2_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

// n-byte load (n = 2, 4, 8 or 16) at byte offset off of a compact buffer, through the L1 policy above
template <int NB, bool COH>
__device__ __forceinline__ auto x2_raw(const void* base, int64_t off) {
  using T = typename std::conditional<NB == 16, v4u, typename std::conditional<NB == 8, v2u,
            typename std::conditional<NB == 4, uint32_t, uint16_t>::type>::type>::type;
  const T* p = reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + off);
  if constexpr (COH && BN2_LOADS == 1) {
    const __amdgpu_buffer_rsrc_t r = x2_rsrc(base);
    if constexpr (NB == 16) return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, BN2_SC1);
    else if constexpr (NB == 8) return __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, BN2_SC1);
    else if constexpr (NB == 4) return __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, BN2_SC1);
    else return __builtin_amdgcn_raw_buffer_load_b16(r, (int)off, 0, BN2_SC1);
  } else if constexpr (COH && BN2_LOADS == 2 && NB <= 8) {
    using U = typename std::conditional<NB == 8, uint64_t,
              typename std::conditional<NB == 4, uint32_t, uint16_t>::type>::type;
    const U v = __hip_atomic_load(reinterpret_cast<const U*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (NB == 8) return v2u{(uint32_t)v, (uint32_t)(v >> 32)};
    else return (T)v;
  } else if constexpr (COH && BN2_LOADS == 2) {   // 16 B: two 8-B atomic loads
    const uint64_t* q = reinterpret_cast<const uint64_t*>(p);
    const uint64_t lo = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t hi = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v4u{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
  } else if constexpr (COH && BN2_LOADS == 3) {
    return __builtin_nontemporal_load(p);
  } else {
    return *p;
  }
}

__device__ __forceinline__ float lo16f(uint32_t u) { return (float)(int16_t)(u & 0xFFFFu); }
__device__ __forceinline__ float hi16f(uint32_t u) { return (float)(int16_t)(u >> 16); }

// 4 consecutive elements of one channel plane from flat index idx (a multiple of 4)
template <int XF, bool COH = true>
__device__ __forceinline__ float4 x2_ld4(const X2& x, int64_t idx, float b) {
  if constexpr (XF == 0) {
    return *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(x.p) + idx);
  } else if constexpr (XF == 1) {
    const uint32_t u = x2_raw<4, COH>(x.p, idx);
    return make_float4((float)(int8_t)(u & 0xFF) + b, (float)(int8_t)((u >> 8) & 0xFF) + b,
                       (float)(int8_t)((u >> 16) & 0xFF) + b, (float)(int8_t)(u >> 24) + b);
  } else {
    const v2u u = x2_raw<8, COH>(x.p, 2 * idx);
    return make_float4(lo16f(u.x) + b, hi16f(u.x) + b, lo16f(u.y) + b, hi16f(u.y) + b);
  }
}

// 2 consecutive elements (idx even)
template <int XF, bool COH = true>
__device__ __forceinline__ float2 x2_ld2(const X2& x, int64_t idx, float b) {
  if constexpr (XF == 0) {
    return *reinterpret_cast<const float2*>(reinterpret_cast<const float*>(x.p) + idx);
  } else if constexpr (XF == 1) {
    const uint32_t u = (uint32_t)x2_raw<2, COH>(x.p, idx);
    return make_float2((float)(int8_t)(u & 0xFF) + b, (float)(int8_t)((u >> 8) & 0xFF) + b);
  } else {
    const uint32_t u = x2_raw<4, COH>(x.p, 2 * idx);
    return make_float2(lo16f(u) + b, hi16f(u) + b);
  }
}

template <int XF, bool COH = true>
__device__ __forceinline__ float x2_ld1(const X2& x, int64_t idx, float b) {
  if constexpr (XF == 0) {
    return reinterpret_cast<const float*>(x.p)[idx];
  } else if constexpr (XF == 1) {
    // the byte's 2-byte-aligned pair, then its half
    const uint32_t u = (uint32_t)x2_raw<2, COH>(x.p, idx & ~(int64_t)1);
    return (float)(int8_t)((idx & 1) ? (u >> 8) : (u & 0xFF)) + b;
  } else {
    return (float)(int16_t)x2_raw<2, COH>(x.p, 2 * idx) + b;
  }
}

// The two rows (2 ph, 2 ph + 1) of a 2x2-pooled plane as 2 PW element pairs each, from row offset xo
// (elements).  int16: the rows are one contiguous run of 8 PW bytes -- 16-B aligned for even PW, 8-B
// for odd (H W 2 = 8 PH PW bytes per plane, 8 ph PW per row pair) -- loaded in 16- / 8-B pieces.
template <int XF, int PW>
__device__ __forceinline__ void x2_rows(const X2& x, int64_t xo, float b, float2 (&top)[PW], float2 (&bot)[PW]) {
  if constexpr (XF == 2) {
    uint32_t w[2 * PW];
    if constexpr (PW % 2 == 0) {
#pragma unroll
      for (int i = 0; i < PW / 2; ++i) {
        const v4u v = x2_raw<16, true>(x.p, 2 * xo + 16 * i);
        w[4 * i] = v.x, w[4 * i + 1] = v.y, w[4 * i + 2] = v.z, w[4 * i + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < PW; ++i) {
        const v2u v = x2_raw<8, true>(x.p, 2 * xo + 8 * i);
        w[2 * i] = v.x, w[2 * i + 1] = v.y;
      }
    }
#pragma unroll
    for (int q = 0; q < PW; ++q) {
      top[q] = make_float2(lo16f(w[q]) + b, hi16f(w[q]) + b);
      bot[q] = make_float2(lo16f(w[PW + q]) + b, hi16f(w[PW + q]) + b);
    }
  } else {
    constexpr int W = 2 * PW;
#pragma unroll
    for (int q = 0; q < PW; ++q) {
      top[q] = x2_ld2<XF>(x, xo + 2 * q, b);
      bot[q] = x2_ld2<XF>(x, xo + W + 2 * q, b);
    }
  }
}

// int16 row pairs of a pooled plane staged through LDS for a workgroup of 256 threads (one pair per
// thread): the lanes load the pairs' 8-B words in address order -- a wave instruction reads 512
// contiguous bytes wherever the pairs are contiguous -- instead of each lane loading its own 4 W-byte
// pair (64 lanes x 16 B spread over 7 KB per instruction: the L1-bypassing atomic loads above cannot
// merge those in L1, every instruction became 64 line requests).  Words per pair: 2 rows x 2 PW
// int16 = PW; LDS stride PW words, padded to odd (2-way bank conflicts at most).
template <int PW>
struct Rows16 {
  static constexpr int NW = PW;
  static constexpr int LD = (PW % 2) ? PW : PW + 1;
};

// stage np (<= 256) pairs; base(pr) = byte offset of pair pr from x.p
template <int PW, typename Base>
__device__ __forceinline__ void rows16_stage(const X2& x, int np, Base base, uint2* lds) {
  constexpr int NW = Rows16<PW>::NW, LD = Rows16<PW>::LD;
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const int w = (int)threadIdx.x + 256 * k;
    const int pr = w / NW, kw = w - pr * NW;
    if (pr < np) {
      const v2u v = x2_raw<8, true>(x.p, base(pr) + 8 * kw);
      lds[pr * LD + kw] = make_uint2(v.x, v.y);
    }
  }
}

// pair t's two rows as PW element pairs each (same values as x2_rows<2, PW>)
template <int PW>
__device__ __forceinline__ void rows16_unpack(const uint2* lds, int t, float b, float2 (&top)[PW], float2 (&bot)[PW]) {
  constexpr int LD = Rows16<PW>::LD;
  uint32_t w[2 * PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const uint2 v = lds[t * LD + i];
    w[2 * i] = v.x, w[2 * i + 1] = v.y;
  }
#pragma unroll
  for (int q = 0; q < PW; ++q) {
    top[q] = make_float2(lo16f(w[q]) + b, hi16f(w[q]) + b);
    bot[q] = make_float2(lo16f(w[PW + q]) + b, hi16f(w[PW + q]) + b);
  }
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
