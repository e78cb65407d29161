// Shared helpers for libbnn (gfx950 / MI355X only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#define BNN_API extern "C" __attribute__((visibility("default")))

namespace bnn {

// Error codes returned by every entry point (include/bnn.h):
//   0 = ok, BNN_EINVAL (-1) = bad arguments, >0 = hipError_t of the failed launch.
constexpr int kErrInval = -1;

void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

int check_launch(const char* what);

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

// GEMM epilogue output stores, non-temporal (the nt bit: streamed, not kept in the caches): the big
// GEMMs' outputs (1-2 GB per launch) are far beyond the 256 MB MALL, and the streamed stores drain
// faster -- pixel GEMM 1188 -> 993 us, FP4 2136 -> 2034, FP6 dX 8572 -> 8476, dW 6808 -> 6760 --
// against +111 us in the pass that reads the pixel GEMM's output next: wide step 47.2 -> 46.6 ms
// (profiles/r05_z_wide_{default,nt}.log).  BNN_NT_STORES=0 builds the plain stores (A/B).
#ifndef BNN_NT_STORES
#define BNN_NT_STORES 1
#endif
__device__ __forceinline__ void out_store4f(float* p, float4 v) {
  if (BNN_NT_STORES) __builtin_nontemporal_store(v4f{v.x, v.y, v.z, v.w}, reinterpret_cast<v4f*>(p));
  else *reinterpret_cast<float4*>(p) = v;
}
__device__ __forceinline__ void out_store2u(void* p, uint32_t lo, uint32_t hi) {
  if (BNN_NT_STORES) __builtin_nontemporal_store(v2u{lo, hi}, reinterpret_cast<v2u*>(p));
  else *reinterpret_cast<uint2*>(p) = make_uint2(lo, hi);
}

// Ternary sign as used by the reference (models/binarized_modules.py:13, Tensor.sign()):
// +1 for x>0, -1 for x<0, 0 for x==0 (NaN maps to 0 here; the reference would propagate NaN).
__device__ __forceinline__ int tsign(float x) { return (x > 0.f) - (x < 0.f); }

// The input of a BatchNorm pass, in one of three forms (XF):
//  0  fp32 x [M][C];
//  1  (z16) the int16 exact dot products I of the ternary BinarizeLinear that produced it
//     (bnn_gemm_fp4_i16) plus that layer's fp32 bias, read as x = fl(I + bias) -- bit-identical to
//     the fp32 value the GEMM epilogue would have stored (it computes the same one rounding), at
//     half the bytes;
//  2  (s20) the exact integer sums S = sum_k u_k sign(w_k) of the u8-pixel layer (bnn_gemm_i8_affine
//     _s20), |S| < 2^19, as 20-bit two's complement: the low 16 bits [M][C] int16 at p and the high
//     4 bits as nibbles [M][C/2] at hi (column 2j in the low nibble of byte j), read as
//     x = fl(fl(S * scale) + bias) -- bit-identical to the fp32 z of bnn_gemm_i8_affine (whose
//     double (S * a) rounds once, as the fp32 product of the exact fl(S) does), at 2.5 bytes.
// bias may be null (a bias-free Linear).
struct XIn {
  const void* p;
  const float* bias;
  const uint8_t* hi = nullptr;   // XF 2: the high nibbles
  float scale = 1.f;             // XF 2: the pixel scale a
};

template <int XF>
__device__ __forceinline__ float4 xin_bias4(const XIn& in, int64_t c) {
  if constexpr (XF != 0) {
    if (in.bias != nullptr) return *reinterpret_cast<const float4*>(in.bias + c);
  }
  return make_float4(0.f, 0.f, 0.f, 0.f);
}

struct S20Raw {
  uint2 lo;
  uint32_t hi;   // 4 nibbles in the low 16 bits
};

// 4 consecutive elements from flat index idx (a multiple of 4) in two steps -- the raw load
// (uint2 of 4 int16, float4, or the s20 pieces) and the conversion with b = xin_bias4 of their
// columns -- so a software-pipelined pass can issue the load early and convert at use (converting
// at issue would make the load's first use, and its wait, immediate).
template <int XF>
using XRaw = typename std::conditional<XF == 1, uint2, typename std::conditional<XF == 2, S20Raw, float4>::type>::type;

template <int XF>
__device__ __forceinline__ XRaw<XF> xin_raw4(const XIn& in, int64_t idx) {
  if constexpr (XF == 1) {
    return *reinterpret_cast<const uint2*>(reinterpret_cast<const int16_t*>(in.p) + idx);
  } else if constexpr (XF == 2) {
    S20Raw r;
    r.lo = *reinterpret_cast<const uint2*>(reinterpret_cast<const int16_t*>(in.p) + idx);
    r.hi = *reinterpret_cast<const uint16_t*>(in.hi + (idx >> 1));
    return r;
  } else {
    return *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(in.p) + idx);
  }
}

// S from a 32-bit window whose bits 0-15 are its low 16 bits and bits 16-19 its nibble (one
// v_alignbit_b32 builds it), sign-extended from bit 19 (v_bfe_i32)
__device__ __forceinline__ int s20_sext(uint32_t w) { return ((int)(w << 12)) >> 12; }

template <int XF>
__device__ __forceinline__ float4 xin_cvt4(const XRaw<XF>& u, const float4& b, float scale = 1.f) {
  if constexpr (XF == 1) {
    return make_float4((float)(int16_t)(u.x & 0xFFFFu) + b.x, (float)(int16_t)(u.x >> 16) + b.y,
                       (float)(int16_t)(u.y & 0xFFFFu) + b.z, (float)(int16_t)(u.y >> 16) + b.w);
  } else if constexpr (XF == 2) {
    // no mul+add contraction: fl(fl(S * scale) + bias), the GEMM epilogue's two roundings
#pragma clang fp contract(off)
    // ({hi >> 4k, lo} >> 16)[31:0]: the element's 16 low bits, then its nibble at bit 16
    const int s0 = s20_sext(__builtin_amdgcn_alignbit(u.hi, u.lo.x << 16, 16));
    const int s1 = s20_sext(__builtin_amdgcn_alignbit(u.hi >> 4, u.lo.x, 16));
    const int s2 = s20_sext(__builtin_amdgcn_alignbit(u.hi >> 8, u.lo.y << 16, 16));
    const int s3 = s20_sext(__builtin_amdgcn_alignbit(u.hi >> 12, u.lo.y, 16));
    return make_float4((float)s0 * scale + b.x, (float)s1 * scale + b.y, (float)s2 * scale + b.z,
                       (float)s3 * scale + b.w);
  } else {
    return u;
  }
}

template <int XF>
__device__ __forceinline__ float4 xin_load4(const XIn& in, int64_t idx, const float4& b) {
  return xin_cvt4<XF>(xin_raw4<XF>(in, idx), b, in.scale);
}

// The training-mode BatchNorm(+Hardtanh) backward for one element (mnist-dist2.py:66-74): with
// xh = ((x - mean) - mean_lo) * invstd, y = xh*gamma + beta, g = dy masked by -1 < y < 1,
// dz = gamma*invstd*(g - a0 - xh*a1), a0 = sum(g)/M, a1 = sum(g*xh)/M.  One definition for every
// pass that forms dz (bn_bwd_apply_k, the fused FP6 and int8 quantising passes), so they agree
// bit for bit.
__device__ __forceinline__ float bn_dz1(float x, float g, float m, float lo, float is, float ga, float be, float a0,
                                        float a1, int hardtanh) {
  // no mul+add contraction: the rounding must not depend on the kernel this is inlined into
#pragma clang fp contract(off)
  const float xh = ((x - m) - lo) * is;
  const float yv = fmaf(xh, ga, be);
  const float gg = (!hardtanh || (yv > -1.f && yv < 1.f)) ? g : 0.f;
  return ga * is * (gg - a0 - xh * a1);
}

// Block-uniform wave index (provably uniform for the compiler -> SGPR).
__device__ __forceinline__ int wave_id() {
  return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Digit quantisation shared by quant_rows / quant_cols_t (see DESIGN.md "fp32 operands"):
// a vector with max|x| = f*2^E (f in [0.5,1)) is scaled by 2^(22-E) to integers |v| <= 2^22 and
// split into balanced base-256 digits v = d2*2^16 + d1*2^8 + d0, d0,d1 in [-128,127],
// d2 in [-65,65].  Scale s = 2^(E-22) is a power of two, so x ~= s*v with |err| <= s/2.
struct Digits { int8_t d0, d1, d2; };

__device__ __forceinline__ Digits to_digits(float x, int shift) {
  const int v = __float2int_rn(ldexpf(x, shift));
  const int d0 = ((v + 128) & 255) - 128;
  const int v1 = (v - d0) >> 8;
  const int d1 = ((v1 + 128) & 255) - 128;
  const int d2 = (v1 - d1) >> 8;
  return Digits{(int8_t)d0, (int8_t)d1, (int8_t)d2};
}

// to_digits' three digits packed as bytes d0 | d1 << 8 | d2 << 16 in one add and one xor: every byte
// of u = v + 0x808080 is d_i + 128 (d0 + 128, d1 + 128 in [0, 255]: no carries), and
// d_i & 255 = (d_i + 128) ^ 0x80 -- bit-identical to packing to_digits' bytes for every v (the top
// digit wraps the same way; unsigned arithmetic: no overflow).
__device__ __forceinline__ uint32_t digits24(float x, int shift) {
  const int v = __float2int_rn(ldexpf(x, shift));
  return (((uint32_t)v + 0x808080u) ^ 0x808080u) & 0xFFFFFFu;
}

// d0 + 256 d1 + 65536 d2 of a packed digit word (the signed bytes' combination) in two ops
__device__ __forceinline__ int digits24_value(uint32_t g) { return (int)((g & 0xFFFFFFu) ^ 0x808080u) - 0x808080; }

// byte b of each of 4 words, packed [w0.b, w1.b, w2.b, w3.b] (three v_perm_b32)
__device__ __forceinline__ uint32_t gather_byte4(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, int b) {
  const uint32_t sel = (uint32_t)b | ((uint32_t)(4 + b) << 8) | 0x0C0C0000u;
  const uint32_t lo = __builtin_amdgcn_perm(w1, w0, sel), hi = __builtin_amdgcn_perm(w3, w2, sel);
  return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

// From the absolute maximum of a vector: the shift 22-E and the scale 2^(E-22).
// amax == 0 -> scale 0 (all digits 0); non-finite -> scale NaN (outputs become NaN).
__device__ __forceinline__ void digit_scale(float amax, int* shift, float* scale) {
  if (!(amax == amax) || amax == __builtin_inff()) {
    *shift = 0;
    *scale = __builtin_nanf("");
    return;
  }
  if (amax == 0.f) {
    *shift = 0;
    *scale = 0.f;
    return;
  }
  int e;
  frexpf(amax, &e);
  *shift = 22 - e;
  *scale = ldexpf(1.f, e - 22);
}

// torch.optim.Adam single-tensor math in fp32 (exp_avg.lerp_, exp_avg_sq.mul_.addcmul_,
// denom = sqrt(v)/sqrt(bc2) + eps, p.addcdiv_(m, denom, -lr/bc1)), then the latent clamp of
// mnist-dist2.py:135-137.  Shared by bnn_adam_clamp and the fused bnn_adam_clamp_pack so both
// produce bit-identical latent weights.
struct AdamArgs {
  const float* g;
  float* m;
  float* v;
  float b1, b2, eps, step_size, bc2_sqrt, gscale;
  int clamp;
  // device-step form (graph-captured steps): (step_size, bc2_sqrt) = sched[2 * ctr[0] + {0, 1}],
  // a host-built table of the same bias corrections (bnn_adam_schedule)
  const float* sched = nullptr;
  const int64_t* ctr = nullptr;
};

// step_size / bc2_sqrt of this launch (from the arguments, or the device-step table)
__device__ __forceinline__ AdamArgs adam_resolve(AdamArgs a) {
  if (a.sched != nullptr) {
    const int64_t i = a.ctr[0];
    a.step_size = a.sched[2 * i];
    a.bc2_sqrt = a.sched[2 * i + 1];
  }
  return a;
}

void adam_bias_correction(float lr, float beta1, float beta2, int64_t step, float* step_size, float* bc2_sqrt);

__device__ __forceinline__ float adam_elem(float p, float g, float& m, float& v, const AdamArgs& a) {
  // no mul+add contraction: both kernels that inline this must round every step identically
#pragma clang fp contract(off)
  const float gi = g * a.gscale;
  m = m + (1.f - a.b1) * (gi - m);
  v = fmaf((1.f - a.b2) * gi, gi, v * a.b2);
  const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
  float pi = p - a.step_size * (m / denom);
  if (a.clamp) pi = fminf(fmaxf(pi, -1.f), 1.f);
  return pi;
}

// Fused nn.Dropout(p) in front of a BatchNorm (mnist-dist2.py:69-70: fc3 -> drop -> bn3).  The
// keep mask is a counter-based hash of (seed, element index), so forward statistics, forward
// apply and both backward passes regenerate the same mask without storing it; kept elements are
// scaled by 1/(1-p) exactly as torch's dropout does (x * scale, grad * scale).
struct Drop {
  uint64_t seed;
  uint32_t thresh;  // keep iff hash < thresh
  int on;
  float scale;      // 1 / (1 - p)
  const int64_t* ctr = nullptr;   // device step counter folded into the seed (bnn_set_seed_counter)
  // keep-bit plane (keep_word below): the forward statistics pass writes the mask once (bits_out),
  // the later passes over the same tensor read it (bits) instead of evaluating the hash again
  const uint32_t* bits = nullptr;
  uint32_t* bits_out = nullptr;
};

// Keep-bit plane of a [M][C] tensor (C % 4 == 0): word (r / 8, c / 4) holds the keep bits of rows
// (r & ~7) + i, columns (c & ~3) + j at bit 4 i + j -- one dword per 8 rows of a thread's float4
// column group, one nibble per row.  (M + 7) / 8 * C / 4 words.
__host__ __device__ __forceinline__ int64_t keep_word(int64_t r, int64_t c, int64_t C) {
  return (r >> 3) * (C >> 2) + (c >> 2);
}
__host__ __device__ __forceinline__ int64_t keep_words(int64_t M, int64_t C) { return (M + 7) / 8 * (C / 4); }

// Process-wide device step counter for graph-captured training steps: dropout launches made
// while it is set draw their mask from seed + ctr[0] * golden, so one captured graph replays with
// a fresh mask per step (forward and backward of a step read the same counter value).
extern const int64_t* g_seed_ctr;   // defined in bnn_bn.hip

__device__ __forceinline__ Drop drop_resolve(Drop d) {
  if (d.on && d.ctr != nullptr) d.seed += (uint64_t)d.ctr[0] * 0xD1B54A32D192ED03ull;
  return d;
}

// 32-bit arithmetic only: one murmur3 fmix32 round of (element index * golden) XOR a 32-bit key
// folded from the 64-bit seed (the key is loop-invariant: the compiler hoists it, so an element
// costs one multiply-xor and the round).  The element index is taken mod 2^32; the mask of every
// pass over the same tensor is the same function of it.  XOR keying (not a Weyl offset) so two
// seeds never give shifted copies of one mask.
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  return h ^ (h >> 16);
}

__device__ __forceinline__ uint32_t drop_key(uint64_t seed) {
  return (uint32_t)seed ^ fmix32((uint32_t)(seed >> 32) ^ 0x5BD1E995u);
}

__device__ __forceinline__ uint32_t drop_hash(uint64_t seed, uint64_t i) {
  return fmix32((uint32_t)i * 0x9E3779B1u ^ drop_key(seed));
}

__device__ __forceinline__ bool drop_keep(const Drop& d, uint64_t i) { return drop_hash(d.seed, i) < d.thresh; }

// keep bits of elements i0 .. i0+3 (bit j): the index products (i0 + j) * golden formed by adds
// from one multiply (the same values mod 2^32; the 32-bit multiply is a quarter-rate instruction)
__device__ __forceinline__ uint32_t drop_bits4(const Drop& d, uint64_t i0) {
  const uint32_t key = drop_key(d.seed), h0 = (uint32_t)i0 * 0x9E3779B1u;
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) m |= (uint32_t)(fmix32((h0 + (uint32_t)j * 0x9E3779B1u) ^ key) < d.thresh) << j;
  return m;
}


inline Drop make_drop(float p, uint64_t seed) {
  Drop d{seed, 0u, 0, 1.f, g_seed_ctr};
  if (p > 0.f && p < 1.f) {
    const double t = (1.0 - (double)p) * 4294967296.0;
    d.thresh = t >= 4294967295.0 ? 4294967295u : (uint32_t)t;
    d.on = 1;
    d.scale = 1.f / (1.f - p);
  }
  return d;
}

}  // namespace bnn
