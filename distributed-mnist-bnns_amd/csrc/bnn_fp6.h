// FP6 (e2m3) digit-plane quantisation of fp32 operands, shared by the FP6 GEMM's quantisers
// (bnn_gemm6.hip) and the fused BatchNorm-backward + quantise pass (bnn_bn.hip).  The scheme and
// the operand layouts are described at the top of bnn_gemm6.hip.
#pragma once
#include "bnn_common.h"

namespace bnn {

constexpr int QB = 32;           // elements per scale block
constexpr int SCALE_BIAS = 111;  // E8M0 byte of plane 0 = e + 111 (= e - 19 + 3 + 127)

// e2m3 code of the integer digit d in [-16, 16] read as d/8.  For |d| <= 16 the code of |d|/8 IS
// |d|: 0..7 are the subnormals m/8 (exponent field 0), 8..15 are 1.mmm (exponent 1, mantissa
// |d| - 8), 16 is 2.0 (exponent 2, mantissa 0) = 0b010000; the sign is bit 5.
__device__ __forceinline__ uint32_t e2m3_code(int d) {
  return d < 0 ? (0x20u | (uint32_t)(-d)) : (uint32_t)d;
}

// Block exponent from the block's |max|: e with amax in [2^(e-1), 2^e); returns the plane-0 E8M0
// byte (255 = NaN for a non-finite block: its outputs become NaN, as the fp32 GEMM's would).
__device__ __forceinline__ int block_scale(float amax, int* shift) {
  if (!(amax == amax) || amax == __builtin_inff()) {
    *shift = 0;
    return 255;
  }
  int e = -111;
  if (amax > 0.f) {
    frexpf(amax, &e);
    e = e < -111 ? -111 : e;     // blocks below 2^-112 quantise to ~0 (error < 2^-130)
  }
  *shift = 19 - e;
  return e + SCALE_BIAS;
}

// 4 balanced base-32 digits of rint(x * 2^shift)
__device__ __forceinline__ void digits4(float x, int shift, int (&d)[4]) {
  int v = __float2int_rn(ldexpf(x, shift));
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int dj = ((v + 16) & 31) - 16;
    d[j] = dj;
    v = (v - dj) >> 5;
  }
  d[3] = v;
}

// The four plane codes of rint(x * 2^shift) (|.| <= 2^19) without the digit arithmetic: with
// w = v + 16 * (1 + 32 + 1024 + 32768) >= 0, the balanced digits are d_j = e_j - 16 for the plain
// base-32 digits e_j of w (e_3 = w >> 15 unmasked, <= 32), and the e2m3 code of d = e - 16 is
// e - 16 for e >= 16, else 32 | (16 - e) = 48 - e, i.e. min(e - 16, 48 - e) in unsigned arithmetic.
// Bit-identical to digits4 + e2m3_code.
constexpr int DIGIT_BIAS = 16 * (1 + 32 + 1024 + 32768);

__device__ __forceinline__ void codes4(float x, int shift, uint32_t (&c)[4]) {
  const uint32_t w = (uint32_t)(__float2int_rn(ldexpf(x, shift)) + DIGIT_BIAS);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t e = j < 3 ? __builtin_amdgcn_ubfe(w, 5 * j, 5) : (w >> 15);
    // e >= 16: e - 16 (<= 16) < 48 - e; e < 16: e - 16 wraps above 48 - e -- one unsigned min
    c[j] = min(e - 16u, 48u - e);
  }
}

// The residual plane of a row operand (the dX GEMMs' dY rows; bnn_gemm6.hip header "residual"): three
// more bits of x below the four digit planes, as ONE FP4 (e2m1) plane.  With v = rint(x 2^shift)
// (the digit planes' integer), 4r = x 2^(shift+2) - 4v is exact in fp32 (|4r| <= 2), and the digit
// d = rint(8r) in [-4, 4] is stored as the e2m1 code of d/2: the conversion unit's round-to-nearest-
// even of 4r onto {0, 0.5, 1, 1.5, 2} (v_cvt_scalef32_pk_fp4_f32, scale 1 -- ties go to the even code
// exactly as rint's; a negative 4r that rounds to zero gives -0, code 8, the same value;
// tools/probes/probe_cvt_fp4.hip, profiles/r05_probe_cvt_fp4.log).  The GEMM scales the plane by
// 2^(e - 21) (E8M0 byte = plane 0's byte - 5), so the five planes sum rint(x 2^(22-e)) 2^(e-22):
// |x - q| <= 2^(e-23) <= max|x_block| 2^-22.  A block with a NaN scale or shift > RES_MAX_SHIFT
// (max|x| < 2^-105, where 2^(shift+2) is no fp32 number) gets a zero residual.
constexpr int RES_MAX_SHIFT = 124;

// the pair's two codes into byte `idx` (compile-time after unrolling) of `old`
__device__ __forceinline__ uint32_t res4_pack2(uint32_t old, float r4a, float r4b, int idx) {
  switch (idx & 3) {
    case 0: return __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(old, r4a, r4b, 1.f, 0);
    case 1: return __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(old, r4a, r4b, 1.f, 1);
    case 2: return __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(old, r4a, r4b, 1.f, 2);
    default: return __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(old, r4a, r4b, 1.f, 3);
  }
}

// one element's code from x itself (ldexp: any shift up to RES_MAX_SHIFT; the slow path of blocks
// outside the magic-fma range, and the lane-per-element quantiser)
__device__ __forceinline__ uint32_t res4_code(float x, int shift) {
  const float v = rintf(ldexpf(x, shift));
  const float r4 = ldexpf(x, shift + 2) - 4.f * v;   // exact
  return __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(0u, r4, 0.f, 1.f, 0) & 15u;
}

__device__ __forceinline__ float absmax_nan(float amax, float x) {
  const float a = fabsf(x);
  return (a == a) ? fmaxf(amax, a) : __builtin_inff();
}

// One 32-element block held by 8 consecutive lanes (q = lane & 7 holds elements 4q..4q+3):
// quantise it and store its record -- lanes q < 4 write plane q (16 B at lo_blk + 16q, 8 B at
// hi_blk + 8q), lane 4 the plane-0 scale byte.  Every lane of the wave must call it (shuffles);
// store = false suppresses this group's writes.
__device__ __forceinline__ void q6_block_store(const float (&v)[4], int lane, bool store, uint8_t* lo_blk,
                                               uint8_t* hi_blk, uint8_t* sc_byte, uint8_t* res_blk = nullptr) {
  const int q = lane & 7;
  float amax = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) amax = absmax_nan(amax, v[j]);
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
  int shift;
  const int sbyte = block_scale(amax, &shift);
  // this lane's 4 elements -> a 24-bit chunk per plane (element 4q+i at bits 6i of the chunk)
  uint32_t chunk[4] = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint32_t cd[4];
    codes4(v[i], shift, cd);
#pragma unroll
    for (int j = 0; j < 4; ++j) chunk[j] |= cd[j] << (6 * i);
  }
  // lane j of the group assembles plane j: chunk of lane p sits at bits 24p..24p+23
  const int plane = q & 3;
  uint32_t w[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t cj = __shfl(chunk[j], (lane & ~7) | p, 64);
      c = (plane == j) ? cj : c;
    }
    const int bit = 24 * p;
    w[bit >> 5] |= c << (bit & 31);
    if ((bit & 31) > 8) w[(bit >> 5) + 1] |= c >> (32 - (bit & 31));
  }
  if (!store) return;
  if (res_blk != nullptr) {   // the residual plane: this lane's 4 elements are nibbles 4q..4q+3
    const bool rz = sbyte == 255 || shift > RES_MAX_SHIFT;
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) r |= (rz ? 0u : res4_code(v[i], shift)) << (4 * i);
    *reinterpret_cast<uint16_t*>(res_blk + 2 * q) = (uint16_t)r;
  }
  if (q < 4) {
    *reinterpret_cast<uint4*>(lo_blk + plane * 16) = make_uint4(w[0], w[1], w[2], w[3]);
    *reinterpret_cast<uint2*>(hi_blk + plane * 8) = make_uint2(w[4], w[5]);
  } else if (q == 4) {
    *sc_byte = (uint8_t)sbyte;
  }
}

// One whole 32-element block quantised by ONE lane, element i read from LDS at src[i * STRIDE]
// (read twice: once for the block max, then for the digits): its four plane records -- plane j's
// 6 dwords, element i at bits 6i -- written as lo (16 B per plane, 64 B) and hi (dwords 4-5 of
// planes 0..3, 32 B), and the plane-0 scale byte.  No cross-lane traffic.
//
// Encoding and packing on the conversion unit: w = rint(x 2^shift) + DIGIT_BIAS as in codes4,
// plane j's 32 digits d = e_j - 16 (e_j the plain base-32 digits of w) are exact in f16 -- formed
// two at a time with packed 16-bit/f16 arithmetic -- and ONE v_cvt_scalef32_pk32_fp6_f16 per plane
// (scale 8: the e2m3 code of d/8) encodes and packs them (element i at bits 6i,
// tools/probes/probe_cvt_fp6.hip).  Bit-identical to codes4 + the manual 6-bit packing.
typedef _Float16 q6v32h __attribute__((ext_vector_type(32)));
typedef _Float16 q6h2 __attribute__((ext_vector_type(2)));
typedef uint32_t q6v16u __attribute__((ext_vector_type(16)));
typedef int q6v6i __attribute__((ext_vector_type(6)));

template <int STRIDE>
__device__ __forceinline__ void q6_block_store_lds(const float* src, bool store, uint8_t* lo_blk, uint8_t* hi_blk,
                                                   uint8_t* sc_byte) {
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < QB; ++i) amax = absmax_nan(amax, src[i * STRIDE]);
  int shift;
  const int sbyte = block_scale(amax, &shift);
  // element pairs (2k, 2k+1) packed in 16-bit halves: P = bits 0..15 of both w (digits 0-2 at
  // bits 0, 5, 10 of each half), Q = their top digit (w >> 15, <= 32)
  uint32_t P[QB / 2], Q[QB / 2];
#pragma unroll
  for (int k = 0; k < QB / 2; ++k) {
    const uint32_t wa = (uint32_t)(__float2int_rn(ldexpf(src[(2 * k) * STRIDE], shift)) + DIGIT_BIAS);
    const uint32_t wb = (uint32_t)(__float2int_rn(ldexpf(src[(2 * k + 1) * STRIDE], shift)) + DIGIT_BIAS);
    P[k] = (wa & 0xFFFFu) | (wb << 16);
    Q[k] = (wa >> 15) | ((wb >> 15) << 16);
  }
  // one plane at a time (not unrolled: the 16 pair words, one f16 vector and one record live at
  // once).  A digit pair e (two 5/6-bit fields) becomes its f16 pair d = e - 16 exactly through
  // the exponent trick: the halves of (e | 0x6400) read as f16 are 1024 + e, minus 1040.
#pragma unroll 1
  for (int j = 0; j < 4; ++j) {
    q6v16u hv;
#pragma unroll
    for (int k = 0; k < QB / 2; ++k) {
      const uint32_t e = j < 3 ? ((P[k] >> (5 * j)) & 0x001F001Fu) | 0x64006400u : Q[k] | 0x64006400u;
      const q6h2 d = __builtin_bit_cast(q6h2, e) - q6h2{(_Float16)1040.f, (_Float16)1040.f};
      hv[k] = __builtin_bit_cast(uint32_t, d);
    }
    const q6v6i rec = __builtin_amdgcn_cvt_scalef32_pk32_fp6_f16(__builtin_bit_cast(q6v32h, hv), 8.0f);
    if (store) {
      *reinterpret_cast<uint4*>(lo_blk + 16 * j) =
          make_uint4((uint32_t)rec[0], (uint32_t)rec[1], (uint32_t)rec[2], (uint32_t)rec[3]);
      *reinterpret_cast<uint2*>(hi_blk + 8 * j) = make_uint2((uint32_t)rec[4], (uint32_t)rec[5]);
    }
  }
  if (store) *sc_byte = (uint8_t)sbyte;
}

// q6_block_store_lds with the block's max|x| given (as the bits of |x|: an unsigned max over
// (bits & 0x7FFFFFFF) ranks NaN above +inf above every finite value, so a block holding a NaN or an
// inf gets the same NaN scale byte as absmax_nan gives it) -- computed while the block was formed,
// so the block is read once.  w = rint(x 2^shift) + DIGIT_BIAS comes from ONE fma: with
// MAGIC = 1.5 2^23 + DIGIT_BIAS, fma(x, 2^shift, MAGIC) lies in [2^23, 2^24) (|rint| <= 2^19),
// where the float grid is the integers and round-to-nearest-even equals rint's (MAGIC is even), so
// its bits are 0x4B400000 + w: the low 16 bits of w are the low 16 bits of the float and
// w >> 15 = bits 15..20.  Blocks with a NaN scale or shift > 126 (max|x| < 2^-107: 2^shift is not
// an fp32 number) take the ldexp path.  CSUM adds the block's elements to csum in element order
// (the same double sum as a separate loop over them).  The record goes to sink.plane(j, lo 16 B,
// hi 8 B) for planes j = 0..3 and sink.scale(byte).  Bit-identical to q6_block_store_lds.
//
// RES (row operands of the dX GEMMs): also the block's residual FP4 plane (two fmas and half a
// conversion per element) to sink.residual(16 B: element i at bits 4i).
template <int STRIDE, bool CSUM, typename Sink, bool RES = false>
__device__ __forceinline__ void q6_block_pre(const float* src, uint32_t amax_bits, Sink& sink, double& csum) {
  int shift;
  const int sbyte = block_scale(__uint_as_float(amax_bits), &shift);
  uint32_t P[QB / 2], Q[QB / 2];
  uint32_t R[RES ? 4 : 1] = {0u};
  if (sbyte != 255 && shift <= 126) {
    const float s = __uint_as_float((uint32_t)(shift + 127) << 23);
    constexpr float MAGIC = 12582912.f + (float)DIGIT_BIAS;
    // 2^(shift+2) (shift <= RES_MAX_SHIFT; else the residual stays zero)
    const bool rok = RES && shift <= RES_MAX_SHIFT;
    const float s4 = rok ? __uint_as_float((uint32_t)(shift + 129) << 23) : 0.f;
#pragma unroll
    for (int k = 0; k < QB / 2; ++k) {
      const float xa = src[(2 * k) * STRIDE], xb = src[(2 * k + 1) * STRIDE];
      if constexpr (CSUM) {
        csum += (double)xa;
        csum += (double)xb;
      }
      const uint32_t ba = __float_as_uint(__builtin_fmaf(xa, s, MAGIC));
      const uint32_t bb = __float_as_uint(__builtin_fmaf(xb, s, MAGIC));
      P[k] = __builtin_amdgcn_perm(bb, ba, 0x05040100u);          // low halves of (a, b)
      Q[k] = __builtin_amdgcn_ubfe(ba, 15, 6) | (__builtin_amdgcn_ubfe(bb, 15, 6) << 16);
      if constexpr (RES) {
        if (rok) {
          // -4v = fl(ba) * -4 + 4 MAGIC and 4r = x 2^(shift+2) - 4v, both exact: two fmas and one
          // conversion per pair (the integer route took ~17 VALU per pair on the critical row waves)
          const float ra = __builtin_fmaf(xa, s4, __builtin_fmaf(__uint_as_float(ba), -4.f, 4.f * MAGIC));
          const float rb = __builtin_fmaf(xb, s4, __builtin_fmaf(__uint_as_float(bb), -4.f, 4.f * MAGIC));
          R[k >> 2] = res4_pack2(R[k >> 2], ra, rb, k);
        }
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < QB / 2; ++k) {
      const float xa = src[(2 * k) * STRIDE], xb = src[(2 * k + 1) * STRIDE];
      if constexpr (CSUM) {
        csum += (double)xa;
        csum += (double)xb;
      }
      const uint32_t wa = (uint32_t)(__float2int_rn(ldexpf(xa, shift)) + DIGIT_BIAS);
      const uint32_t wb = (uint32_t)(__float2int_rn(ldexpf(xb, shift)) + DIGIT_BIAS);
      P[k] = (wa & 0xFFFFu) | (wb << 16);
      Q[k] = (wa >> 15) | ((wb >> 15) << 16);
      if constexpr (RES) {
        if (sbyte != 255 && shift <= RES_MAX_SHIFT)
          R[k >> 2] |= (res4_code(xa, shift) | (res4_code(xb, shift) << 4)) << (8 * (k & 3));
      }
    }
  }
  if constexpr (RES) sink.residual(make_uint4(R[0], R[1], R[2], R[3]));
#pragma unroll 1
  for (int j = 0; j < 4; ++j) {
    q6v16u hv;
#pragma unroll
    for (int k = 0; k < QB / 2; ++k) {
      const uint32_t e = j < 3 ? ((P[k] >> (5 * j)) & 0x001F001Fu) | 0x64006400u : Q[k] | 0x64006400u;
      const q6h2 d = __builtin_bit_cast(q6h2, e) - q6h2{(_Float16)1040.f, (_Float16)1040.f};
      hv[k] = __builtin_bit_cast(uint32_t, d);
    }
    const q6v6i rec = __builtin_amdgcn_cvt_scalef32_pk32_fp6_f16(__builtin_bit_cast(q6v32h, hv), 8.0f);
    sink.plane(j, make_uint4((uint32_t)rec[0], (uint32_t)rec[1], (uint32_t)rec[2], (uint32_t)rec[3]),
               make_uint2((uint32_t)rec[4], (uint32_t)rec[5]));
  }
  sink.scale((uint8_t)sbyte);
}

__device__ __forceinline__ uint32_t abs_bits(float x) { return __float_as_uint(x) & 0x7FFFFFFFu; }

// Rows of the E8M0 scale slab [K/64][rows_pad][2] a quantised operand of `rows` rows needs: the
// GEMM's scale piece is one 1-KiB LDS-DMA of 512 rows from the tile's first row.
inline int64_t q6_scale_rows(int64_t rows) { return (rows + 255) / 256 * 256 + 512; }

}  // namespace bnn
