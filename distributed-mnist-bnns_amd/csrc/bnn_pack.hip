// Subsystem (1): sign-and-pack, plus the fp32 -> digit quantisers that feed fp32 operands
// (fc1 input, backward dY) to the same int8 MFMA GEMM.  All kernels are HBM-bound streams:
// coalesced 16-B loads, LDS-tiled transposes, no atomics, deterministic.
//
// Reference behaviour restated: Binarize(t,'det') = t.sign() (models/binarized_modules.py:11-13)
// applied to inputs (:76, :95) and to the latent weight (:79, :98); sign(0) = 0 -> ternary.
#include <algorithm>

#include "bnn_common.h"

namespace bnn {
namespace {

constexpr int TILE = 64;

// max|v| accumulation that turns NaN into +inf (fmaxf alone would drop NaN) so a non-finite
// row/column gets a NaN scale and propagates NaN like the reference's fp32 GEMM would.
__device__ __forceinline__ float absmax_acc(float amax, float v) {
  const float a = fabsf(v);
  return (a == a) ? fmaxf(amax, a) : __builtin_inff();
}

__device__ __forceinline__ void load16(const float* __restrict__ row, int64_t k, int64_t K, bool vec,
                                       float (&v)[16]) {
  if (vec && k + 16 <= K) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 f = *reinterpret_cast<const float4*>(row + k + 4 * i);
      v[4 * i + 0] = f.x;
      v[4 * i + 1] = f.y;
      v[4 * i + 2] = f.z;
      v[4 * i + 3] = f.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = (k + j < K) ? row[k + j] : 0.f;
  }
}

__device__ __forceinline__ int pack4(int a, int b, int c, int d) {
  return (a & 255) | ((b & 255) << 8) | ((c & 255) << 16) | ((d & 255) << 24);
}

// FP4 (e2m1) code of a ternary value: +1 = 0b0010, -1 = 0b1010, 0 = 0b0000.
__device__ __forceinline__ uint32_t fp4_code(int s) { return s > 0 ? 0x2u : (s < 0 ? 0xAu : 0u); }

// Optional per-column affine map applied before the sign: the BatchNorm output
// y = (x - mean) * invstd * gamma + beta, computed exactly as bn_apply_k does (bnn_bn.hip), so the
// fused BN -> Hardtanh -> sign path sees bit-identical y (Hardtanh does not change a sign).
struct ColAffine {
  const float* mean;
  const float* mean_lo;  // nullable: the lo part of the batch mean (bnn_bn.hip), x - mean = (x - hi) - lo
  const float* invstd;
  const float* gamma;  // nullable
  const float* beta;   // nullable
  int vec;             // all four 16-B aligned -> float4 parameter loads
};

// One 4-element run of a latent-weight row updated in place by Adam + clamp (ADAM mode of
// sign_pack_tile_k: the fused latent update of mnist-dist2.py:131-137 that also writes the next
// forward's ternary operands).  p, g, m, v share the row-major [M][K] layout; off = the row's
// offset, columns k..k+3; sg = the new signs (0 beyond K).
__device__ __forceinline__ void adam4(float* __restrict__ prow, int64_t off, int64_t k, int64_t K, bool vec,
                                      const AdamArgs& a, int (&sg)[4]) {
  if (vec && k + 4 <= K) {
    const float4 pv = *reinterpret_cast<const float4*>(prow + k);
    const float4 gv = *reinterpret_cast<const float4*>(a.g + off + k);
    float4 mv = *reinterpret_cast<const float4*>(a.m + off + k);
    float4 vv = *reinterpret_cast<const float4*>(a.v + off + k);
    float4 np;
    np.x = adam_elem(pv.x, gv.x, mv.x, vv.x, a);
    np.y = adam_elem(pv.y, gv.y, mv.y, vv.y, a);
    np.z = adam_elem(pv.z, gv.z, mv.z, vv.z, a);
    np.w = adam_elem(pv.w, gv.w, mv.w, vv.w, a);
    *reinterpret_cast<float4*>(prow + k) = np;
    *reinterpret_cast<float4*>(a.m + off + k) = mv;
    *reinterpret_cast<float4*>(a.v + off + k) = vv;
    sg[0] = tsign(np.x), sg[1] = tsign(np.y), sg[2] = tsign(np.z), sg[3] = tsign(np.w);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sg[j] = 0;
      if (k + j < K) {
        float mm = a.m[off + k + j], vv = a.v[off + k + j];
        const float np = adam_elem(prow[k + j], a.g[off + k + j], mm, vv, a);
        prow[k + j] = np;
        a.m[off + k + j] = mm;
        a.v[off + k + j] = vv;
        sg[j] = tsign(np);
      }
    }
  }
}

// One 64x64 tile of x -> ternary rows (q: FMT 0 = int8 per element, FMT 1 = FP4 e2m1 nibbles,
// element k in byte k/2, low nibble for even k) and/or the transposed int8 tile (qt).
// ADAM = 1: x is a latent weight updated in place first (adam4), and its new sign is packed.
// PK_COAL 1: the non-Adam modes load whole 256-B row runs too (below); 0: 16 columns per lane
#ifndef PK_COAL
#define PK_COAL 1
#endif
template <int FMT, int AFF = 0, int ADAM = 0>
__global__ __launch_bounds__(256) void sign_pack_tile_k(const float* __restrict__ x, int64_t M,
                                                        int64_t K, int64_t ldx, int8_t* __restrict__ q,
                                                        int64_t ldq, int8_t* __restrict__ qt,
                                                        int64_t ldqt, int vec, ColAffine af = {},
                                                        int rtiles = 1, int64_t ntiles_y = 0,
                                                        AdamArgs ad = {}, int qt4 = 0) {
  // qt4 = 1: the transpose is written as FP4 nibbles (qt rows of ldqt BYTES, element m in byte
  // m/2), the B operand of the FP6 digit GEMMs (bnn_gemm6.hip); 2: the same nibbles in that GEMM's
  // panel layout ([K/512][ldqt/32][512][32 B], bnn_fp4_panelize); else int8 (rows of ldqt elements)
  // rtiles > 1: the workgroup walks rtiles vertically adjacent 64x64 tiles of its column block
  // (the per-column BatchNorm parameters are loaded once per workgroup, not once per tile)
  __shared__ int tile[TILE][TILE + 1];
  const int64_t k0 = (int64_t)blockIdx.x * TILE;
  const int t = threadIdx.x, r = t >> 2, c = (t & 3) * 16;
#if PK_COAL
  // the row-run form: lane = 4 consecutive columns of a 256-B row run, parameters for those 4
  float mu[4], lo[4], is[4], ga[4], be[4];
  constexpr int NP = 4;
  const int64_t cb = k0 + (t & 15) * 4;
#else
  float mu[16], lo[16], is[16], ga[16], be[16];
  constexpr int NP = 16;
  const int64_t cb = k0 + c;
#endif
  if (AFF) {
    // per-column parameters for columns cb .. cb + NP - 1: float4 loads when the run is in range
    if (af.vec && cb + NP <= K) {
#pragma unroll
      for (int i = 0; i < NP / 4; ++i) {
        const float4 a = *reinterpret_cast<const float4*>(af.mean + cb + 4 * i);
        const float4 b = *reinterpret_cast<const float4*>(af.invstd + cb + 4 * i);
        const float4 g = af.gamma ? *reinterpret_cast<const float4*>(af.gamma + cb + 4 * i) : make_float4(1, 1, 1, 1);
        const float4 e = af.beta ? *reinterpret_cast<const float4*>(af.beta + cb + 4 * i) : make_float4(0, 0, 0, 0);
        const float4 l = af.mean_lo ? *reinterpret_cast<const float4*>(af.mean_lo + cb + 4 * i) : make_float4(0, 0, 0, 0);
        mu[4 * i] = a.x; mu[4 * i + 1] = a.y; mu[4 * i + 2] = a.z; mu[4 * i + 3] = a.w;
        lo[4 * i] = l.x; lo[4 * i + 1] = l.y; lo[4 * i + 2] = l.z; lo[4 * i + 3] = l.w;
        is[4 * i] = b.x; is[4 * i + 1] = b.y; is[4 * i + 2] = b.z; is[4 * i + 3] = b.w;
        ga[4 * i] = g.x; ga[4 * i + 1] = g.y; ga[4 * i + 2] = g.z; ga[4 * i + 3] = g.w;
        be[4 * i] = e.x; be[4 * i + 1] = e.y; be[4 * i + 2] = e.z; be[4 * i + 3] = e.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const bool in = cb + j < K;
        mu[j] = in ? af.mean[cb + j] : 0.f;
        lo[j] = (in && af.mean_lo) ? af.mean_lo[cb + j] : 0.f;
        is[j] = in ? af.invstd[cb + j] : 0.f;
        ga[j] = (in && af.gamma) ? af.gamma[cb + j] : 1.f;
        be[j] = (in && af.beta) ? af.beta[cb + j] : 0.f;
      }
    }
  }
  for (int it = 0; it < rtiles; ++it) {
  const int64_t ty = (int64_t)blockIdx.y * rtiles + it;
  if (rtiles > 1 && ty >= ntiles_y) break;   // uniform per workgroup
  if (it > 0) __syncthreads();                // the previous tile's transposed reads are done
  const int64_t m0 = ty * TILE;
  const int64_t m = m0 + r;
  int s[16];
  if constexpr (ADAM) {
    // the update as whole 256-B row runs (16 lanes x float4 per row, 16 rows per pass: every wave
    // load instruction covers 4 full rows; lane = 16 consecutive floats moved 64-B pieces), the new
    // signs through the LDS tile into the row-run layout the packing below uses
    const AdamArgs a = adam_resolve(ad);
    const int ar = t >> 4, ac = (t & 15) * 4;
#pragma unroll
    for (int pr = 0; pr < TILE / 16; ++pr) {
      const int rr = ar + 16 * pr;
      const int64_t mr = m0 + rr;
      int sg[4] = {0, 0, 0, 0};
      if (mr < M) adam4(const_cast<float*>(x) + mr * ldx, mr * ldx, k0 + ac, K, vec, a, sg);
#pragma unroll
      for (int j = 0; j < 4; ++j) tile[rr][ac + j] = sg[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 16; ++j) s[j] = tile[r][c + j];
    if (qt != nullptr) __syncthreads();   // read before the transpose below rewrites the tile
  } else {
#if PK_COAL
    // as the ADAM mode: every wave load instruction covers 4 whole 256-B row runs (lane = 4
    // consecutive columns), the signs go through the LDS tile into the 16-column layout below.
    // The same per-element arithmetic as the 16-column form (bit-identical).
    const int ar = t >> 4, ac = (t & 15) * 4;
#pragma unroll
    for (int pr = 0; pr < TILE / 16; ++pr) {
      const int rr = ar + 16 * pr;
      const int64_t mr = m0 + rr;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (mr < M) {
        const float* row = x + mr * ldx;
        if (vec && cb + 4 <= K) {
          const float4 f = *reinterpret_cast<const float4*>(row + cb);
          v[0] = f.x, v[1] = f.y, v[2] = f.z, v[3] = f.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (cb + j < K) ? row[cb + j] : 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float y = v[j];
        if (AFF) y = (mr < M && cb + j < K) ? fmaf(((y - mu[j]) - lo[j]) * is[j], ga[j], be[j]) : 0.f;
        tile[rr][ac + j] = tsign(y);
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 16; ++j) s[j] = tile[r][c + j];
    if (qt != nullptr) __syncthreads();   // read before the transpose below rewrites the tile
#else
    float v[16];
    if (m < M) {
      load16(x + m * ldx, k0 + c, K, vec, v);
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = 0.f;
    }
    if (AFF) {
#pragma unroll
      for (int j = 0; j < 16; ++j)
        v[j] = (m < M && cb + j < K) ? fmaf(((v[j] - mu[j]) - lo[j]) * is[j], ga[j], be[j]) : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) s[j] = tsign(v[j]);
#endif
  }
  if (FMT == 0 && q != nullptr && m < M && k0 + c < ldq) {
    v4i w;
    w.x = pack4(s[0], s[1], s[2], s[3]);
    w.y = pack4(s[4], s[5], s[6], s[7]);
    w.z = pack4(s[8], s[9], s[10], s[11]);
    w.w = pack4(s[12], s[13], s[14], s[15]);
    *reinterpret_cast<v4i*>(q + m * ldq + k0 + c) = w;
  }
  if (FMT == 1 && q != nullptr && m < M && (k0 + c) / 2 < ldq) {
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      lo |= fp4_code(s[j]) << (4 * j);
      hi |= fp4_code(s[8 + j]) << (4 * j);
    }
    *reinterpret_cast<uint2*>(q + m * ldq + (k0 + c) / 2) = make_uint2(lo, hi);
  }
  if (qt != nullptr) {
#pragma unroll
    for (int j = 0; j < 16; ++j) tile[r][c + j] = s[j];
    __syncthreads();
    const int kk = t >> 2, mc = (t & 3) * 16;
    const int64_t k = k0 + kk;
    if (qt4) {
      if (k < K && (m0 + mc) / 2 < ldqt) {
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          lo |= fp4_code(tile[mc + j][kk]) << (4 * j);
          hi |= fp4_code(tile[mc + 8 + j][kk]) << (4 * j);
        }
        const int64_t m = m0 + mc;
        int8_t* dst = qt4 == 2 ? qt + ((k >> 9) * (ldqt / 32) + (m >> 6)) * 16384 + (k & 511) * 32 + (m & 63) / 2
                               : qt + k * ldqt + m / 2;
        *reinterpret_cast<uint2*>(dst) = make_uint2(lo, hi);
      }
    } else if (k < K && m0 + mc < ldqt) {
      int g[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) g[j] = tile[mc + j][kk];
      v4i w;
      w.x = pack4(g[0], g[1], g[2], g[3]);
      w.y = pack4(g[4], g[5], g[6], g[7]);
      w.z = pack4(g[8], g[9], g[10], g[11]);
      w.w = pack4(g[12], g[13], g[14], g[15]);
      *reinterpret_cast<v4i*>(qt + k * ldqt + m0 + mc) = w;
    }
  }
  }
}

// The benched form of bnn_bn_apply_pack (FP4 rows + FP4 transpose, C % 256 == 0) on 256 x 256
// tiles: sign_pack_tile_k's 64 x 64 tiles give each lane 16 consecutive floats (64-B strided
// loads) and write 32-B fragments of 128-B lines; here every load instruction is one 1-KiB run of
// a row, the FP4 rows leave as one 128-B run per wave instruction, and the transpose leaves as
// whole 128-B lines (256 rows = 128 B of a transposed row).
// Phase 1: wave w walks rows w, w+4, ..; lane l owns columns 4l..4l+3: y = BN(x) (bit-identical to
// sign_pack_tile_k<., 1>), its 4 FP4 codes (16 bits) go to q and into an LDS nibble image
// [256 rows][33 dwords] (dword slot XOR-swizzled by row bits 6-7).
// Phase 2: thread = (8-column block kb, 32-row group mg): 4 x (8 dwords = an 8 x 8 nibble block,
// transposed in registers by three block-swap stages) -> 8 transposed rows x 16 B.
// LDS reads are conflict-free: bank = 32 (mg & 1) + 33 b + (kb ^ ((mg >> 1) << 3)) mod 64.
constexpr int AP_T = 256, AP_LD = 33;
// phase-1 row unroll of the 256 x 256-tile passes (rows in flight per wave); A/B hooks
#ifndef APK_UNROLL
#define APK_UNROLL 4
#endif
#ifndef ADAMPK_UNROLL
#define ADAMPK_UNROLL 4
#endif

__device__ __forceinline__ void nib_swap(uint32_t& a, uint32_t& b, int s, uint32_t mask) {
  const uint32_t t = ((a >> s) ^ b) & mask;
  b ^= t;
  a ^= t << s;
}

// 8 x 8 nibble transpose: x[i] = row i (nibble c at bits 4c) -> x[c] = column c (nibble i at 4i)
__device__ __forceinline__ void nib_transpose8(uint32_t (&x)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) nib_swap(x[i], x[i + 4], 16, 0x0000FFFFu);
#pragma unroll
  for (int i = 0; i < 8; i += 4) {
    nib_swap(x[i], x[i + 2], 8, 0x00FF00FFu);
    nib_swap(x[i + 1], x[i + 3], 8, 0x00FF00FFu);
  }
#pragma unroll
  for (int i = 0; i < 8; i += 2) nib_swap(x[i], x[i + 1], 4, 0x0F0F0F0Fu);
}

// IDN = 1: no BatchNorm (y = x: the plain sign-pack of bnn_sign_pack_fp4 on 256 x 256 tiles), and
// sout (nullable) also receives sign(x) as fp32 -- the drop-in's `input.data = sign(input)` write-back
// (binarized_modules.py:76) from the same read of x.
template <int XF, int IDN = 0>
__global__ __launch_bounds__(256) void bn_apply_pack_fp4_k(XIn xin, int64_t M, int64_t C,
                                                           ColAffine af, uint8_t* __restrict__ q, int64_t ldq,
                                                           uint8_t* __restrict__ qt, int64_t ldqt, int64_t pnks,
                                                           float* __restrict__ sout = nullptr) {
  __shared__ uint32_t img[AP_T * AP_LD];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t k0 = (int64_t)blockIdx.x * AP_T, m0 = (int64_t)blockIdx.y * AP_T;
  const int64_t cb = k0 + 4 * lane;
  float mu[4] = {0.f, 0.f, 0.f, 0.f}, is[4] = {1.f, 1.f, 1.f, 1.f}, ga[4] = {1.f, 1.f, 1.f, 1.f};
  float be[4] = {0.f, 0.f, 0.f, 0.f}, lo[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (!IDN) {
    const float4 mv = *reinterpret_cast<const float4*>(af.mean + cb);
    const float4 iv = *reinterpret_cast<const float4*>(af.invstd + cb);
    const float4 gv = af.gamma ? *reinterpret_cast<const float4*>(af.gamma + cb) : make_float4(1, 1, 1, 1);
    const float4 bv = af.beta ? *reinterpret_cast<const float4*>(af.beta + cb) : make_float4(0, 0, 0, 0);
    const float4 lv = af.mean_lo ? *reinterpret_cast<const float4*>(af.mean_lo + cb) : make_float4(0, 0, 0, 0);
    mu[0] = mv.x, mu[1] = mv.y, mu[2] = mv.z, mu[3] = mv.w;
    is[0] = iv.x, is[1] = iv.y, is[2] = iv.z, is[3] = iv.w;
    ga[0] = gv.x, ga[1] = gv.y, ga[2] = gv.z, ga[3] = gv.w;
    be[0] = bv.x, be[1] = bv.y, be[2] = bv.z, be[3] = bv.w;
    lo[0] = lv.x, lo[1] = lv.y, lo[2] = lv.z, lo[3] = lv.w;
  }
  const float4 xb = xin_bias4<XF>(xin, cb);
  uint16_t* img16 = reinterpret_cast<uint16_t*>(img);
#pragma unroll APK_UNROLL
  for (int i = 0; i < AP_T / 4; ++i) {
    const int r = wave + 4 * i;
    const int64_t m = m0 + r;
    uint32_t code = 0;
    if (m < M) {
      const float4 f = xin_load4<XF>(xin, m * C + cb, xb);
      const float v[4] = {f.x, f.y, f.z, f.w};
      int sg[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sg[j] = IDN ? tsign(v[j]) : tsign(fmaf(((v[j] - mu[j]) - lo[j]) * is[j], ga[j], be[j]));
        code |= fp4_code(sg[j]) << (4 * j);
      }
      *reinterpret_cast<uint16_t*>(q + m * ldq + k0 / 2 + 2 * lane) = (uint16_t)code;
      if (IDN && sout != nullptr)
        *reinterpret_cast<float4*>(sout + m * C + cb) = make_float4((float)sg[0], (float)sg[1], (float)sg[2], (float)sg[3]);
    }
    const int slot = (lane >> 1) ^ (((r >> 6) & 3) << 3);
    img16[(r * AP_LD + slot) * 2 + (lane & 1)] = (uint16_t)code;
  }
  __syncthreads();
  const int mg = t & 7, kb = t >> 3;
  uint32_t out[8][4];
#pragma unroll
  for (int qq = 0; qq < 4; ++qq) {
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = 32 * mg + 8 * qq + i;
      w[i] = img[r * AP_LD + (kb ^ ((mg >> 1) << 3))];
    }
    nib_transpose8(w);
#pragma unroll
    for (int c = 0; c < 8; ++c) out[c][qq] = w[c];
  }
  // pnks > 0: the transpose in the FP4 panel layout of the FP6 GEMM's B operand (bnn_fp4_panelize:
  // [C/512][pnks][512][32 B]) -- row n's 16 B at batch m0 + 32 mg are half mg & 1 of k-step
  // (m0 + 32 mg) / 64; a wave's 8 rows per store are 32-B pieces of 8 lines the c loop completes
#if defined(APK_DIAG_NOQT)   // timing-only build: no transpose stores (wrong results)
  if (out[0][0] == 0x12345678u)
#endif
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int64_t n = k0 + 8 * kb + c;
    uint8_t* dst = pnks > 0 ? qt + ((n >> 9) * pnks + (m0 >> 6) + (mg >> 1)) * 16384 + (n & 511) * 32 + (mg & 1) * 16
                            : qt + n * ldqt + m0 / 2 + 16 * mg;
    *reinterpret_cast<uint4*>(dst) = make_uint4(out[c][0], out[c][1], out[c][2], out[c][3]);
  }
}

// bnn_adam_clamp_pack on 256 x 256 tiles (the layout of bn_apply_pack_fp4_k): phase 1 updates
// each 1-KiB row run of p with Adam + clamp (p, g, m, v read and p, m, v written as whole-line
// float4 runs; sign_pack_tile_k's 64 x 64 tiles move 64-B pieces), packs the new signs into the FP4
// rows and the LDS nibble image; phase 2 writes the FP4 transpose (plain or panel layout) exactly
// as bn_apply_pack_fp4_k does.  Same element arithmetic (adam_elem) as sign_pack_tile_k<1, 0, 1>.
__global__ __launch_bounds__(256) void adam_pack_fp4_k(float* __restrict__ p, AdamArgs a0, int64_t N, int64_t K,
                                                       uint8_t* __restrict__ q, int64_t ldq,
                                                       uint8_t* __restrict__ qt, int64_t ldqt, int64_t pnks) {
  __shared__ uint32_t img[AP_T * AP_LD];
  const AdamArgs a = adam_resolve(a0);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t k0 = (int64_t)blockIdx.x * AP_T, m0 = (int64_t)blockIdx.y * AP_T;
  const int64_t cb = k0 + 4 * lane;
  uint16_t* img16 = reinterpret_cast<uint16_t*>(img);
#pragma unroll ADAMPK_UNROLL
  for (int i = 0; i < AP_T / 4; ++i) {
    const int r = wave + 4 * i;
    const int64_t off = (m0 + r) * K + cb;            // N % 256 == 0: every row is in range
    const float4 pv = *reinterpret_cast<const float4*>(p + off);
    const float4 gv = *reinterpret_cast<const float4*>(a.g + off);
    float4 mv = *reinterpret_cast<const float4*>(a.m + off);
    float4 vv = *reinterpret_cast<const float4*>(a.v + off);
    float4 np;
    np.x = adam_elem(pv.x, gv.x, mv.x, vv.x, a);
    np.y = adam_elem(pv.y, gv.y, mv.y, vv.y, a);
    np.z = adam_elem(pv.z, gv.z, mv.z, vv.z, a);
    np.w = adam_elem(pv.w, gv.w, mv.w, vv.w, a);
    *reinterpret_cast<float4*>(p + off) = np;
    *reinterpret_cast<float4*>(a.m + off) = mv;
    *reinterpret_cast<float4*>(a.v + off) = vv;
    const uint32_t code = fp4_code(tsign(np.x)) | (fp4_code(tsign(np.y)) << 4) | (fp4_code(tsign(np.z)) << 8) |
                          (fp4_code(tsign(np.w)) << 12);
    *reinterpret_cast<uint16_t*>(q + (m0 + r) * ldq + k0 / 2 + 2 * lane) = (uint16_t)code;
    const int slot = (lane >> 1) ^ (((r >> 6) & 3) << 3);
    img16[(r * AP_LD + slot) * 2 + (lane & 1)] = (uint16_t)code;
  }
  __syncthreads();
  const int mg = t & 7, kb = t >> 3;
  uint32_t out[8][4];
#pragma unroll
  for (int qq = 0; qq < 4; ++qq) {
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = 32 * mg + 8 * qq + i;
      w[i] = img[r * AP_LD + (kb ^ ((mg >> 1) << 3))];
    }
    nib_transpose8(w);
#pragma unroll
    for (int c = 0; c < 8; ++c) out[c][qq] = w[c];
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int64_t n = k0 + 8 * kb + c;
    uint8_t* dst = pnks > 0 ? qt + ((n >> 9) * pnks + (m0 >> 6) + (mg >> 1)) * 16384 + (n & 511) * 32 + (mg & 1) * 16
                            : qt + n * ldqt + m0 / 2 + 16 * mg;
    *reinterpret_cast<uint4*>(dst) = make_uint4(out[c][0], out[c][1], out[c][2], out[c][3]);
  }
}

__global__ __launch_bounds__(256) void sign_f32_k(const float* __restrict__ x, float* __restrict__ y,
                                                  int64_t n, int vec) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (vec) {
    const int64_t n4 = n / 4;
    for (int64_t j = i; j < n4; j += stride) {
      float4 f = reinterpret_cast<const float4*>(x)[j];
      f.x = (float)tsign(f.x);
      f.y = (float)tsign(f.y);
      f.z = (float)tsign(f.z);
      f.w = (float)tsign(f.w);
      reinterpret_cast<float4*>(y)[j] = f;
    }
    for (int64_t j = n4 * 4 + i; j < n; j += stride) y[j] = (float)tsign(x[j]);
  } else {
    for (int64_t j = i; j < n; j += stride) y[j] = (float)tsign(x[j]);
  }
}

// One wave per (row, 64-wide k chunk): ballots give the sign and nonzero bit-planes.
__global__ __launch_bounds__(256) void sign_pack_bits_k(const float* __restrict__ x, int64_t M,
                                                        int64_t K, int64_t ldx,
                                                        uint32_t* __restrict__ sb,
                                                        uint32_t* __restrict__ nb, int64_t ldw) {
  const int lane = threadIdx.x & 63;
  const int64_t chunks = (ldw + 1) / 2;
  const int64_t total = M * chunks;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t wv = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); wv < total; wv += nwaves) {
    const int64_t m = wv / chunks, ch = wv % chunks;
    const int64_t k = ch * 64 + lane;
    const float v = (k < K) ? x[m * ldx + k] : 0.f;
    const unsigned long long s = __ballot(v < 0.f);
    // nonzero and not NaN (sign 0, as tsign()), as an integer test: the backend lowers a ballot of
    // the ordered fcmp one (and of fabs(v) > 0) to v_cmp_neq_f32, which is true for NaN
    const unsigned long long z = __ballot((__float_as_uint(v) & 0x7fffffffu) - 1u < 0x7f800000u);
    const int64_t w = ch * 2 + (lane & 1);
    if (lane < 2 && w < ldw) {
      sb[m * ldw + w] = (uint32_t)(lane ? (s >> 32) : s);
      nb[m * ldw + w] = (uint32_t)(lane ? (z >> 32) : z);
    }
  }
}

// Row-scaled digits: one block per row (grid-stride over rows).
__global__ __launch_bounds__(256) void quant_rows_k(const float* __restrict__ x, int64_t M, int64_t K,
                                                    int64_t ldx, int8_t* __restrict__ dg,
                                                    int64_t ldq, int64_t plane,
                                                    float* __restrict__ scale, int vec) {
  __shared__ float red[4];
  const int t = threadIdx.x;
  for (int64_t m = blockIdx.x; m < M; m += gridDim.x) {
    const float* __restrict__ xr = x + m * ldx;
    float amax = 0.f;
    for (int64_t k = 4 * t; k < K; k += 1024) {
      if (vec && k + 4 <= K) {
        const float4 f = *reinterpret_cast<const float4*>(xr + k);
        amax = absmax_acc(absmax_acc(absmax_acc(absmax_acc(amax, f.x), f.y), f.z), f.w);
      } else {
        for (int j = 0; j < 4; ++j)
          if (k + j < K) amax = absmax_acc(amax, xr[k + j]);
      }
    }
    amax = wave_max(amax);
    if ((t & 63) == 0) red[t >> 6] = amax;
    __syncthreads();
    amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    __syncthreads();
    int shift;
    float s;
    digit_scale(amax, &shift, &s);
    if (t == 0) scale[m] = s;
    for (int64_t k = 4 * t; k < ldq; k += 1024) {
      float v[4];
      if (vec && k + 4 <= K) {
        const float4 f = *reinterpret_cast<const float4*>(xr + k);
        v[0] = f.x;
        v[1] = f.y;
        v[2] = f.z;
        v[3] = f.w;
      } else {
        for (int j = 0; j < 4; ++j) v[j] = (k + j < K) ? xr[k + j] : 0.f;
      }
      uint32_t d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = digits24(v[j], shift);
      int8_t* o = dg + m * ldq + k;
      *reinterpret_cast<uint32_t*>(o) = gather_byte4(d[0], d[1], d[2], d[3], 0);
      *reinterpret_cast<uint32_t*>(o + plane) = gather_byte4(d[0], d[1], d[2], d[3], 1);
      *reinterpret_cast<uint32_t*>(o + 2 * plane) = gather_byte4(d[0], d[1], d[2], d[3], 2);
    }
  }
}

constexpr int COL_ROWS = 256;  // most rows per column-statistics chunk

// 256 rows per chunk, halved while the statistics pass would have fewer than 2^17 threads (as
// bnn_bn.hip's reductions): small batches get enough workgroups to fill the chip.
inline int64_t col_chunk_rows(int64_t M, int64_t N) {
  int64_t rows = COL_ROWS;
  while (rows > 1 && ((N + 3) / 4) * ((M + rows - 1) / rows) < (1 << 17) && (M + rows / 2 - 1) / (rows / 2) <= 65535)
    rows >>= 1;
  return rows;
}
inline int64_t col_chunks(int64_t M, int64_t N) {
  const int64_t rows = col_chunk_rows(M, N);
  return std::max<int64_t>(1, (M + rows - 1) / rows);
}

// Pass 1: per (row chunk, column) absolute max and double sum.
__global__ __launch_bounds__(256) void colstats_k(const float* __restrict__ x, int64_t M, int64_t N,
                                                  int64_t ldx, float* __restrict__ pmax,
                                                  double* __restrict__ psum, int64_t crows) {
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.y * crows;
  if (n >= N) return;
  const int64_t r1 = (M < r0 + crows) ? M : r0 + crows;
  float amax = 0.f;
  double sum = 0.0;
  for (int64_t r = r0; r < r1; ++r) {
    const float v = x[r * ldx + n];
    amax = absmax_acc(amax, v);
    sum += (double)v;
  }
  pmax[blockIdx.y * N + n] = amax;
  psum[blockIdx.y * N + n] = sum;
}

// Pass 2: reduce the chunks in a fixed order -> scale[n], colsum[n].
// colstats_k with one float4 (4 adjacent columns) per thread: same per-column row order and
// double accumulation (bit-identical results), a quarter of the load instructions.
__global__ __launch_bounds__(256) void colstats4_k(const float* __restrict__ x, int64_t M, int64_t N,
                                                   int64_t ldx, float* __restrict__ pmax,
                                                   double* __restrict__ psum, int64_t crows) {
  const int64_t n = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const int64_t r0 = (int64_t)blockIdx.y * crows;
  if (n >= N) return;
  const int64_t r1 = (M < r0 + crows) ? M : r0 + crows;
  float amax[4] = {0.f, 0.f, 0.f, 0.f};
  double sum[4] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t r = r0; r < r1; ++r) {
    const float4 v = *reinterpret_cast<const float4*>(x + r * ldx + n);
    const float vs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      amax[j] = absmax_acc(amax[j], vs[j]);
      sum[j] += (double)vs[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    pmax[blockIdx.y * N + n + j] = amax[j];
    psum[blockIdx.y * N + n + j] = sum[j];
  }
}

// 64 columns x 4 chunk groups per workgroup (fixed-order fold of the groups): deterministic, 4x the
// parallelism of one thread per column walking all R chunks.
__global__ __launch_bounds__(256) void colfinal_k(const float* __restrict__ pmax,
                                                  const double* __restrict__ psum, int64_t N,
                                                  int64_t R, float* __restrict__ scale,
                                                  float* __restrict__ colsum, int64_t* __restrict__ dsum) {
  __shared__ float smx[4][64];
  __shared__ double ssm[4][64];
  const int lc = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int64_t n = (int64_t)blockIdx.x * 64 + lc;
  float amax = 0.f;
  double sum = 0.0;
  if (n < N)
    for (int64_t r = grp; r < R; r += 4) {
      amax = fmaxf(amax, pmax[r * N + n]);
      sum += psum[r * N + n];
    }
  smx[grp][lc] = amax;
  ssm[grp][lc] = sum;
  __syncthreads();
  if (grp != 0 || n >= N) return;
  amax = fmaxf(fmaxf(smx[0][lc], smx[1][lc]), fmaxf(smx[2][lc], smx[3][lc]));
  sum = ssm[0][lc] + ssm[1][lc] + ssm[2][lc] + ssm[3][lc];
  int shift;
  float s;
  digit_scale(amax, &shift, &s);
  scale[n] = s;
  if (colsum != nullptr) colsum[n] = (float)sum;
  if (dsum != nullptr) dsum[n] = 0;   // quant_cols_t_k accumulates the digit sums into it
}

// quant_cols_t_k's second half, shared with bn_dz_quant_cols_t_k: the 64 x 64 tile of packed
// digits (row m, column n) written transposed as 3 int8 planes dt[d][n][m], plus the exact digit
// column sums.  Call after the tile is complete (__syncthreads).
// With acc != null the 4-lane part of column n0 + t/4 is added to *acc (every lane of the 4)
// instead of atomically to dsum[n]: a caller walking several tiles of the same columns issues one
// atomic per column at the end.
// Tile element (row, col) at tile[row * LD + col], or with SWZ (LD = 64) at the 16-B chunk
// (col / 4) ^ (4 * ((row / RPL) % 4)): conflict-free both for 16-B row writes and for the
// column reads of qct_store_t (the 4 lanes of a column read rows RPL apart).
template <int LD, bool SWZ, int RPL>
__device__ __forceinline__ int qct_at(const int* tile, int row, int col) {
  if constexpr (SWZ) {
    constexpr int SH = RPL == 32 ? 5 : 4;
    return tile[row * LD + ((((col >> 2) ^ (((row >> SH) & 3) << 2))) << 2) + (col & 3)];
  } else {
    return tile[row * LD + col];
  }
}

// RPL = rows per lane: a tile of 4 * RPL rows, each column written as 4 * RPL contiguous bytes
// per plane (RPL = 32: whole 128-B lines).
template <int LD, bool SWZ, int RPL = 16>
__device__ __forceinline__ void qct_store_t(const int* tile, int t, int64_t n0, int64_t m0, int64_t N,
                                            int64_t ldqt, int64_t plane, int8_t* __restrict__ dt,
                                            int64_t* __restrict__ dsum, long long* acc = nullptr) {
  const int nn = t >> 2, mc = (t & 3) * RPL;
  const int64_t n = n0 + nn;
  // exact integer sum of the combined digits d2*2^16 + d1*2^8 + d0 of column n (|.| <= 2^22 each,
  // so 4 * RPL of them fit an int): sum (g ^ 0x808080) - count * 0x808080 (digits24_value); the 4
  // lanes sharing n are adjacent.  Rows beyond ldqt hold zeros.
  int part = 0;
  if (n < N && m0 + mc < ldqt) {
    uint32_t g[RPL];
#pragma unroll
    for (int j = 0; j < RPL; ++j) g[j] = (uint32_t)qct_at<LD, SWZ, RPL>(tile, mc + j, nn);
#pragma unroll
    for (int d = 0; d < 3; ++d) {
#pragma unroll
      for (int q = 0; q < RPL / 16; ++q) {
        if (m0 + mc + 16 * q >= ldqt) break;
        const uint32_t* gq = g + 16 * q;
        v4i w;
        w.x = (int)gather_byte4(gq[0], gq[1], gq[2], gq[3], d);
        w.y = (int)gather_byte4(gq[4], gq[5], gq[6], gq[7], d);
        w.z = (int)gather_byte4(gq[8], gq[9], gq[10], gq[11], d);
        w.w = (int)gather_byte4(gq[12], gq[13], gq[14], gq[15], d);
        *reinterpret_cast<v4i*>(dt + d * plane + n * ldqt + m0 + mc + 16 * q) = w;
      }
    }
    if (dsum != nullptr) {
#pragma unroll
      for (int j = 0; j < RPL; ++j) part += (int)(g[j] ^ 0x808080u);
      part -= RPL * 0x808080;
    }
  }
  if (dsum != nullptr) {
    part += __shfl_xor(part, 1, 64);
    part += __shfl_xor(part, 2, 64);
    if (acc != nullptr)
      *acc += part;
    else if ((t & 3) == 0 && n < N && part != 0)
      atomicAdd(reinterpret_cast<unsigned long long*>(dsum + n), (unsigned long long)(long long)part);
  }
}

__device__ __forceinline__ void qct_store(const int (&tile)[TILE][TILE + 1], int t, int64_t n0, int64_t m0, int64_t N,
                                          int64_t ldqt, int64_t plane, int8_t* __restrict__ dt,
                                          int64_t* __restrict__ dsum) {
  qct_store_t<TILE + 1, false>(&tile[0][0], t, n0, m0, N, ldqt, plane, dt, dsum);
}

__global__ __launch_bounds__(256) void quant_cols_t_k(const float* __restrict__ x, int64_t M,
                                                      int64_t N, int64_t ldx,
                                                      const float* __restrict__ scale,
                                                      int8_t* __restrict__ dt, int64_t ldqt,
                                                      int64_t plane, int vec, int64_t* __restrict__ dsum) {
  __shared__ int tile[TILE][TILE + 1];
  __shared__ int sh[TILE];
  const int64_t n0 = (int64_t)blockIdx.x * TILE, m0 = (int64_t)blockIdx.y * TILE;
  const int t = threadIdx.x, r = t >> 2, c = (t & 3) * 16;
  if (t < TILE) {
    const int64_t n = n0 + t;
    const float s = (n < N) ? scale[n] : 0.f;
    sh[t] = (s > 0.f && s == s) ? -ilogbf(s) : INT32_MIN;  // INT32_MIN -> digits 0
  }
  __syncthreads();
  const int64_t m = m0 + r;
  float v[16];
  if (m < M) {
    load16(x + m * ldx, n0 + c, N, vec, v);
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int sft = sh[c + j];
    tile[r][c + j] = sft != INT32_MIN ? (int)digits24(v[j], sft) : 0;
  }
  __syncthreads();
  qct_store(tile, t, n0, m0, N, ldqt, plane, dt, dsum);
}

// ------------------------------------------------------------------ BatchNorm backward -> dz^T int8 digits
// The input layer's weight gradient dW1 = dz^T . x (the first BinarizeLinear, fed by u8 pixels:
// bnn_gemm_i8_affine) needs dz only as the int8 digit planes of its columns.  dz is formed from
// (x, dy) with bn_dz1 -- the exact value bnn_bn_bwd writes -- in ONE pass after the statistics
// pass, and never stored.  The column scale comes from an a-priori bound instead of a column-max
// pass over dz: the statistics pass (bn_reduce_k MODE 2) also records max|g| and max|xhat| per
// column, and |dz| = |gamma*invstd| |g - a0 - xhat*a1| <= |gamma*invstd| (max|g| + |a0| + max|xhat| |a1|)
// =: B (times 1 + 2^-16 for bn_dz1's few fp32 roundings).  Digits keep 23 bits below B, i.e.
// |dz - scale*v| <= scale/2 = 2^-23 * 2^ceil(log2 B): log2(B / max|dz|) bits fewer than scaling by
// the true column max (B <= (2 + max|xhat|) |gamma*invstd| max|g| since |a0| <= max|g| and
// |a1| <= max|g| mean|xhat| <= max|g|).  The bias gradient (column sums of dz, double) is
// accumulated by the same pass.
struct BnCols {
  const float *mean, *mean_lo, *invstd, *gamma, *beta, *k0, *k1;
  float inv_n;
  int hardtanh;
};

struct Bn4 {
  float m[4], lo[4], is[4], ga[4], be[4], a0[4], a1[4];
};

__device__ __forceinline__ void ld4a(const float* p, int64_t c, float dflt, float (&o)[4]) {
  const float4 v = p ? *reinterpret_cast<const float4*>(p + c) : make_float4(dflt, dflt, dflt, dflt);
  o[0] = v.x, o[1] = v.y, o[2] = v.z, o[3] = v.w;
}

// the 4 columns' parameters with 16-B loads (C % 4 == 0, vectors 16-B aligned: host check)
__device__ __forceinline__ void bn4_load(const BnCols& b, int64_t c, Bn4& o) {
  ld4a(b.mean, c, 0.f, o.m);
  ld4a(b.mean_lo, c, 0.f, o.lo);
  ld4a(b.invstd, c, 0.f, o.is);
  ld4a(b.gamma, c, 1.f, o.ga);
  ld4a(b.beta, c, 0.f, o.be);
  ld4a(b.k0, c, 0.f, o.a0);
  ld4a(b.k1, c, 0.f, o.a1);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o.a0[j] *= b.inv_n;
    o.a1[j] *= b.inv_n;
  }
}

// colsum[n] = the fixed-order double sum of the quantiser's per-workgroup-row partials
__global__ __launch_bounds__(256) void bn_dz_colsum_k(const double* __restrict__ part, int64_t R, int64_t N,
                                                      float* __restrict__ colsum) {
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  double s = 0.0;
#pragma unroll 8
  for (int64_t r = 0; r < R; ++r) s += part[r * N + n];
  colsum[n] = (float)s;
}

// 64-column strip x QC_RT 64-row tiles per workgroup (the column parameters are loaded once per
// strip); per 64-row tile, stage 1: thread = 4 columns (t % 16) x 4 rows (t / 16), so each thread
// needs the BatchNorm parameters of 4 columns only, into a swizzled 128-row LDS tile; every second
// tile, stage 2 (qct_store_t, 32 rows per lane) writes the 128 rows: 128-B lines per column and
// plane.  Software-pipelined: tile it+1's x / dy rows are loaded before tile it is stored.  With
// part != null the strip's column sums of dz (double; rows in a fixed order) go to
// part[blockIdx.y][N].
constexpr int QC_RT = 8;
#ifndef DZQ_OCC
#define DZQ_OCC 3   // waves per SIMD (<= 168 VGPRs): the pass waits on memory, so occupancy is its lever
#endif

__host__ __device__ inline int64_t qc_strips(int64_t M, int rt = QC_RT) { return (M + TILE * rt - 1) / (TILE * rt); }
// Row tiles per workgroup by shape: QC_RT_SMALL on grids of under 1,024 workgroups at QC_RT (config 3's
// 4096 x 3072 dz: 384 workgroups of 8 sequential tiles), where the chip would sit mostly idle.
#ifndef QC_RT_SMALL
#define QC_RT_SMALL 2
#endif
inline int qc_rt(int64_t M, int64_t C) {
  return ((C + TILE - 1) / TILE) * qc_strips(M, QC_RT) < 1024 ? QC_RT_SMALL : QC_RT;
}

template <int XF>
__global__ __launch_bounds__(256, DZQ_OCC) void bn_dz_quant_cols_t_k(XIn xin, const float* __restrict__ dy,
                                                            int64_t M, int64_t N, BnCols bc,
                                                            const float* __restrict__ scale, int8_t* __restrict__ dt,
                                                            int64_t ldqt, int64_t plane, int64_t* __restrict__ dsum,
                                                            double* __restrict__ part = nullptr, int rt = QC_RT) {
  constexpr int TM = 2 * TILE;                                       // rows per store tile
  __shared__ __attribute__((aligned(16))) int tile[TM * TILE];       // swizzled (qct_at<TILE, true, 32>)
  double csum[4] = {0.0, 0.0, 0.0, 0.0};
  // bijective XCD remap (workgroups b and b+8 share an XCD under round-robin dispatch): an XCD takes
  // a contiguous run of (strip, row-block) tiles, so the four strips whose s20 nibbles share one
  // 128-B line (64 columns = 32 B of nibbles per row) read it through one L2 -- spread over four
  // XCDs each L2 fetched the whole line (PMC: 8.5 B fetched per element against 6.5 algorithmic)
  const int nwg = gridDim.x * gridDim.y, bid = blockIdx.y * gridDim.x + blockIdx.x;
  const int xcd = bid & 7, xq = nwg >> 3, xr = nwg & 7;
  const int L = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (bid >> 3);
  const int bx = L % (int)gridDim.x, by = L / (int)gridDim.x;
  const int64_t n0 = (int64_t)bx * TILE;
  const int t = threadIdx.x, cg = t & 15, rg = t >> 4;
  const int64_t c = n0 + 4 * cg;
  Bn4 b;
  int sft[4];
  if (c < N) {
    bn4_load(bc, c, b);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float s = scale[c + j];
      sft[j] = (s > 0.f && s == s) ? -ilogbf(s) : INT32_MIN;   // INT32_MIN -> digits 0
    }
  }
  XRaw<XF> xv[4];
  float4 gv[4];
  const float4 xb = c < N ? xin_bias4<XF>(xin, c) : make_float4(0.f, 0.f, 0.f, 0.f);
  auto load = [&](int64_t m0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t m = m0 + 4 * rg + i;
      if (c < N && m < M) {
        xv[i] = xin_raw4<XF>(xin, m * N + c);
        gv[i] = *reinterpret_cast<const float4*>(dy + m * N + c);
      }
    }
  };
  const int64_t mb = (int64_t)by * rt * TILE;
  long long dacc = 0;   // this thread's column (n0 + t/4) digit sum over the strip
  load(mb);
  for (int it = 0; it < rt; ++it) {
    const int64_t m0 = mb + (int64_t)it * TILE;
    if (m0 >= ldqt) break;                      // uniform per workgroup
    if (it > 0 && (it & 1) == 0) __syncthreads();   // the previous store tile's reads are done
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t m = m0 + 4 * rg + i;
      const float4 xf = xin_cvt4<XF>(xv[i], xb, xin.scale);
      const float xs[4] = {xf.x, xf.y, xf.z, xf.w}, gs[4] = {gv[i].x, gv[i].y, gv[i].z, gv[i].w};
      int packed[4] = {0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (c < N && m < M) {
          const float v = bn_dz1(xs[j], gs[j], b.m[j], b.lo[j], b.is[j], b.ga[j], b.be[j], b.a0[j], b.a1[j], bc.hardtanh);
          csum[j] += (double)v;
          if (sft[j] != INT32_MIN) packed[j] = (int)digits24(v, sft[j]);
        }
      }
      const int row = (it & 1) * TILE + 4 * rg + i;
      *reinterpret_cast<int4*>(tile + row * TILE + ((cg ^ (((row >> 5) & 3) << 2)) << 2)) =
          make_int4(packed[0], packed[1], packed[2], packed[3]);
    }
    const bool last = it + 1 == rt || m0 + TILE >= ldqt;
    if (!last) load(m0 + TILE);
    if ((it & 1) == 1 || last) {
      if ((it & 1) == 0) {   // an odd tile count: the second half of the store tile is zeros
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = TILE + 4 * rg + i;
          *reinterpret_cast<int4*>(tile + row * TILE + ((cg ^ (((row >> 5) & 3) << 2)) << 2)) = make_int4(0, 0, 0, 0);
        }
      }
      __syncthreads();
      qct_store_t<TILE, true, 32>(tile, t, n0, m0 - (it & 1) * TILE, N, ldqt, plane, dt, dsum, &dacc);
    }
  }
  if (dsum != nullptr && (t & 3) == 0 && n0 + (t >> 2) < N && dacc != 0)
    atomicAdd(reinterpret_cast<unsigned long long*>(dsum + n0 + (t >> 2)), (unsigned long long)dacc);
  if (part != nullptr && by < qc_strips(M, rt)) {
    // fixed-order fold of the 16 row groups' sums (the tile is free: every qct_store read is done)
    __syncthreads();
    double* ps = reinterpret_cast<double*>(tile);   // [16][64] doubles = 8 KiB <= 32 KiB
#pragma unroll
    for (int j = 0; j < 4; ++j) ps[rg * TILE + 4 * cg + j] = csum[j];
    __syncthreads();
    if (t < TILE && n0 + t < N) {
      double s = 0.0;
#pragma unroll
      for (int r = 0; r < 16; ++r) s += ps[r * TILE + t];
      part[(int64_t)by * N + n0 + t] = s;
    }
  }
}

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Transposed operand checks: int8 rows of ldqt elements (multiple of 64, >= round_up(M,64)) or
// FP4 rows of ldqt bytes (multiple of 128, 2*ldqt >= round_up(M,256)); returns the number of
// 64-row tiles the grid must cover so every padding element is written.
bool qt_ok(const int8_t* qt, int64_t M, int64_t ldqt, int qt_fmt) {
  if (!qt) return true;
  if (!aligned16(qt) || qt_fmt < 0 || qt_fmt > 2) return false;
  return qt_fmt >= 1 ? (ldqt % 128 == 0 && 2 * ldqt >= round_up(M, 256))
                     : (ldqt % TILE == 0 && ldqt >= round_up(M, TILE));
}

int64_t qt_tiles(int64_t ldqt, int qt_fmt) { return (qt_fmt >= 1 ? 2 * ldqt : ldqt) / TILE; }

inline int grid_cap(int64_t want) { return (int)std::max<int64_t>(1, std::min<int64_t>(want, 8192)); }

}  // namespace
}  // namespace bnn

using namespace bnn;

BNN_API int bnn_sign_pack_i8(const float* x, int64_t M, int64_t K, int64_t ldx, int8_t* q,
                             int64_t ldq, int8_t* qt, int64_t ldqt, void* stream) {
  if (!x || M < 0 || K < 0 || ldx < K || (!q && !qt)) {
    set_error("bnn_sign_pack_i8: bad arguments (M=%lld K=%lld ldx=%lld)", (long long)M,
              (long long)K, (long long)ldx);
    return kErrInval;
  }
  if (q && (ldq % TILE != 0 || ldq < round_up(K, TILE) || !aligned16(q))) {
    set_error("bnn_sign_pack_i8: ldq=%lld must be a multiple of 64 >= round_up(K,64), q 16-B aligned",
              (long long)ldq);
    return kErrInval;
  }
  if (qt && (ldqt % TILE != 0 || ldqt < round_up(M, TILE) || !aligned16(qt))) {
    set_error("bnn_sign_pack_i8: ldqt=%lld must be a multiple of 64 >= round_up(M,64)", (long long)ldqt);
    return kErrInval;
  }
  if (M == 0 && !qt) return 0;
  const int vec = aligned16(x) && (ldx % 4 == 0);
  const int64_t gx = q ? ldq / TILE : (K + TILE - 1) / TILE;
  const int64_t gy = qt ? ldqt / TILE : (M + TILE - 1) / TILE;
  if (gx == 0 || gy == 0) return 0;
  if (gy > 65535) {
    set_error("bnn_sign_pack_i8: M too large for one launch (%lld)", (long long)M);
    return kErrInval;
  }
  hipLaunchKernelGGL(sign_pack_tile_k<0>, dim3((unsigned)gx, (unsigned)gy), dim3(256), 0, S(stream), x,
                     M, K, ldx, q, ldq, qt, ldqt, vec);
  return check_launch("bnn_sign_pack_i8");
}

BNN_API int bnn_sign_f32(const float* x, float* y, int64_t n, void* stream);

// Whether bnn_sign_pack_fp4 takes the 256 x 256-tile kernel (bn_apply_pack_fp4_k<0, 1>): both outputs
// as FP4 (rows + transpose or panel transpose), whole 256-column tiles, dense 16-B aligned rows, and a
// grid of >= 1024 tiles (below that the 64 x 64 tiles fill the chip better).
static bool sp_wide_ok(const float* x, int64_t M, int64_t K, int64_t ldx, const uint8_t* q4, int64_t ldq4,
                       const int8_t* qt, int64_t ldqt, int32_t qt_fmt) {
  return q4 && qt && (qt_fmt == 1 || qt_fmt == 2) && K % AP_T == 0 && ldx == K && 2 * ldq4 == K && aligned16(x) &&
         (K / AP_T) * ((M + AP_T - 1) / AP_T) >= 1024 && (M + AP_T - 1) / AP_T <= 65535 &&
         2 * ldqt >= (M + AP_T - 1) / AP_T * AP_T;
}

BNN_API int bnn_sign_pack_fp4(const float* x, int64_t M, int64_t K, int64_t ldx, uint8_t* q4, int64_t ldq4,
                              int8_t* qt, int64_t ldqt, int32_t qt_fmt, void* stream) {
  if (!x || M < 0 || K < 0 || ldx < K || (!q4 && !qt)) {
    set_error("bnn_sign_pack_fp4: bad arguments (M=%lld K=%lld ldx=%lld)", (long long)M, (long long)K,
              (long long)ldx);
    return kErrInval;
  }
  if (q4 && (ldq4 % 128 != 0 || 2 * ldq4 < round_up(K, 256) || !aligned16(q4))) {
    set_error("bnn_sign_pack_fp4: ldq4=%lld bytes must be a multiple of 128 covering round_up(K,256)",
              (long long)ldq4);
    return kErrInval;
  }
  if (!qt_ok(qt, M, ldqt, qt_fmt)) {
    set_error("bnn_sign_pack_fp4: ldqt=%lld does not cover M=%lld in qt_fmt %d", (long long)ldqt, (long long)M,
              qt_fmt);
    return kErrInval;
  }
  if (M == 0 && !qt) return 0;
  const int vec = aligned16(x) && (ldx % 4 == 0);
  if (sp_wide_ok(x, M, K, ldx, q4, ldq4, qt, ldqt, qt_fmt)) {   // the 256 x 256-tile form, same codes
    hipLaunchKernelGGL((bn_apply_pack_fp4_k<0, 1>), dim3((unsigned)(K / AP_T), (unsigned)((M + AP_T - 1) / AP_T)),
                       dim3(256), 0, S(stream), XIn{x, nullptr}, M, K, ColAffine{}, q4, ldq4,
                       reinterpret_cast<uint8_t*>(qt), ldqt, qt_fmt == 2 ? ldqt / 32 : (int64_t)0, nullptr);
    return check_launch("bnn_sign_pack_fp4");
  }
  const int64_t gx = q4 ? (2 * ldq4) / TILE : (K + TILE - 1) / TILE;
  const int64_t gy = qt ? qt_tiles(ldqt, qt_fmt) : (M + TILE - 1) / TILE;
  if (gx == 0 || gy == 0) return 0;
  if (gy > 65535) {
    set_error("bnn_sign_pack_fp4: M too large for one launch (%lld)", (long long)M);
    return kErrInval;
  }
  hipLaunchKernelGGL(sign_pack_tile_k<1>, dim3((unsigned)gx, (unsigned)gy), dim3(256), 0, S(stream), x, M, K,
                     ldx, reinterpret_cast<int8_t*>(q4), ldq4, qt, ldqt, vec, ColAffine{}, 1, (int64_t)0, AdamArgs{},
                     qt_fmt);
  return check_launch("bnn_sign_pack_fp4");
}

// bnn_sign_pack_fp4 + the fp32 sign write-back sout[m][k] = sign(x[m][k]) (row pitch K; may be x) from
// one read of x when the 256 x 256-tile form applies; otherwise the two passes.
BNN_API int bnn_sign_pack_fp4_out(const float* x, int64_t M, int64_t K, uint8_t* q4, int64_t ldq4, int8_t* qt,
                                  int64_t ldqt, int32_t qt_fmt, float* sout, void* stream) {
  if (!sout) {
    set_error("bnn_sign_pack_fp4_out: sout required");
    return kErrInval;
  }
  if (sp_wide_ok(x, M, K, K, q4, ldq4, qt, ldqt, qt_fmt) && aligned16(sout)) {
    hipLaunchKernelGGL((bn_apply_pack_fp4_k<0, 1>), dim3((unsigned)(K / AP_T), (unsigned)((M + AP_T - 1) / AP_T)),
                       dim3(256), 0, S(stream), XIn{x, nullptr}, M, K, ColAffine{}, q4, ldq4,
                       reinterpret_cast<uint8_t*>(qt), ldqt, qt_fmt == 2 ? ldqt / 32 : (int64_t)0, sout);
    return check_launch("bnn_sign_pack_fp4_out");
  }
  const int rc = bnn_sign_pack_fp4(x, M, K, K, q4, ldq4, qt, ldqt, qt_fmt, stream);
  if (rc != 0) return rc;
  return bnn_sign_f32(x, sout, M * K, stream);
}

// tuning hook (bnn_adam_pack_set_tile256): 1 (default) = the 256 x 256-tile kernel for grids of at
// least ADAM_T256_MIN_TILES whole tiles (the wide step's 8192 x 8192 weights: 1024), the 64 x 64
// kernel below, whose 16x finer grid keeps every CU busy on small weights (a 2048 x 2048 weight is
// 64 big tiles for 256 CUs); 2 = the big tile whenever the shape allows it (tests); 0 = never
static int ADAM_TILE256 = 1;
constexpr int64_t ADAM_T256_MIN_TILES = 512;

BNN_API int bnn_adam_pack_set_tile256(int32_t on) {
  ADAM_TILE256 = on < 0 ? 0 : (on > 2 ? 2 : on);
  return 0;
}

static int adam_clamp_pack_impl(float* p, const AdamArgs& a, int64_t N, int64_t K, int32_t fmt, void* q,
                                int64_t ldq, int8_t* qt, int64_t ldqt, int32_t qt_fmt, void* stream) {
  const float* grad = a.g;
  const float* exp_avg = a.m;
  const float* exp_avg_sq = a.v;
  if (!p || !grad || !exp_avg || !exp_avg_sq || N <= 0 || K <= 0 || (fmt != 0 && fmt != 1) || (!q && !qt)) {
    set_error("bnn_adam_clamp_pack: bad arguments (N=%lld K=%lld fmt=%d)", (long long)N, (long long)K, fmt);
    return kErrInval;
  }
  if (q && (fmt == 0 ? (ldq % TILE != 0 || ldq < round_up(K, TILE))
                     : (ldq % 128 != 0 || 2 * ldq < round_up(K, 256))) ) {
    set_error("bnn_adam_clamp_pack: ldq=%lld does not cover K=%lld in fmt %d", (long long)ldq, (long long)K, fmt);
    return kErrInval;
  }
  if ((q && !aligned16(q)) || !qt_ok(qt, N, ldqt, qt_fmt)) {
    set_error("bnn_adam_clamp_pack: ldqt=%lld does not cover N=%lld in qt_fmt %d", (long long)ldqt, (long long)N,
              qt_fmt);
    return kErrInval;
  }
  // every element of p is visited exactly once: the grid spans K (and the q padding) x N (and
  // the qt padding); tiles beyond K or N update nothing and only write zero padding
  const int64_t gx = q ? (fmt == 0 ? ldq : 2 * ldq) / TILE : (K + TILE - 1) / TILE;
  const int64_t gy = qt ? qt_tiles(ldqt, qt_fmt) : (N + TILE - 1) / TILE;
  if (gy > 65535 || gx > 0x7fffffff) {
    set_error("bnn_adam_clamp_pack: N too large for one launch (%lld)", (long long)N);
    return kErrInval;
  }
  const int vec = aligned16(p) && aligned16(grad) && aligned16(exp_avg) && aligned16(exp_avg_sq) && (K % 4 == 0);
  if (fmt == 1 && q && qt && (qt_fmt == 1 || qt_fmt == 2) && vec && N % AP_T == 0 && K % AP_T == 0 &&
      2 * ldq == K && 2 * ldqt == N &&
      (ADAM_TILE256 == 2 || (ADAM_TILE256 == 1 && (K / AP_T) * (N / AP_T) >= ADAM_T256_MIN_TILES))) {
    // whole 256 x 256 tiles, no padding: the 1-KiB-run form
    hipLaunchKernelGGL(adam_pack_fp4_k, dim3((unsigned)(K / AP_T), (unsigned)(N / AP_T)), dim3(256), 0, S(stream), p,
                       a, N, K, reinterpret_cast<uint8_t*>(q), ldq, reinterpret_cast<uint8_t*>(qt), ldqt,
                       qt_fmt == 2 ? ldqt / 32 : (int64_t)0);
    return check_launch("bnn_adam_clamp_pack");
  }
  if (fmt == 0)
    hipLaunchKernelGGL((sign_pack_tile_k<0, 0, 1>), dim3((unsigned)gx, (unsigned)gy), dim3(256), 0, S(stream), p, N,
                       K, K, reinterpret_cast<int8_t*>(q), ldq, qt, ldqt, vec, ColAffine{}, 1, (int64_t)0, a, qt_fmt);
  else
    hipLaunchKernelGGL((sign_pack_tile_k<1, 0, 1>), dim3((unsigned)gx, (unsigned)gy), dim3(256), 0, S(stream), p, N,
                       K, K, reinterpret_cast<int8_t*>(q), ldq, qt, ldqt, vec, ColAffine{}, 1, (int64_t)0, a, qt_fmt);
  return check_launch("bnn_adam_clamp_pack");
}

BNN_API int bnn_adam_clamp_pack(float* p, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t N,
                                int64_t K, float lr, float beta1, float beta2, float eps, int64_t step,
                                float grad_scale, int32_t clamp, int32_t fmt, void* q, int64_t ldq, int8_t* qt,
                                int64_t ldqt, int32_t qt_fmt, void* stream) {
  if (step < 1) {
    set_error("bnn_adam_clamp_pack: step must be >= 1");
    return kErrInval;
  }
  float step_size, bc2_sqrt;
  adam_bias_correction(lr, beta1, beta2, step, &step_size, &bc2_sqrt);
  const AdamArgs a{grad, exp_avg, exp_avg_sq, beta1, beta2, eps, step_size, bc2_sqrt, grad_scale, clamp};
  return adam_clamp_pack_impl(p, a, N, K, fmt, q, ldq, qt, ldqt, qt_fmt, stream);
}

BNN_API int bnn_adam_clamp_pack_sched(float* p, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t N,
                                      int64_t K, float beta1, float beta2, float eps, const float* sched,
                                      const int64_t* ctr, float grad_scale, int32_t clamp, int32_t fmt, void* q,
                                      int64_t ldq, int8_t* qt, int64_t ldqt, int32_t qt_fmt, void* stream) {
  if (!sched || !ctr) {
    set_error("bnn_adam_clamp_pack_sched: null schedule / counter");
    return kErrInval;
  }
  AdamArgs a{grad, exp_avg, exp_avg_sq, beta1, beta2, eps, 0.f, 1.f, grad_scale, clamp};
  a.sched = sched;
  a.ctr = ctr;
  return adam_clamp_pack_impl(p, a, N, K, fmt, q, ldq, qt, ldqt, qt_fmt, stream);
}

BNN_API int bnn_sign_f32(const float* x, float* y, int64_t n, void* stream) {
  if (!x || !y || n < 0) {
    set_error("bnn_sign_f32: bad arguments");
    return kErrInval;
  }
  if (n == 0) return 0;
  const int vec = aligned16(x) && aligned16(y);
  hipLaunchKernelGGL(sign_f32_k, dim3(grid_cap((n / 4 + 255) / 256)), dim3(256), 0, S(stream), x, y,
                     n, vec);
  return check_launch("bnn_sign_f32");
}

BNN_API int bnn_sign_pack_bits(const float* x, int64_t M, int64_t K, int64_t ldx, uint32_t* sbits,
                               uint32_t* nzbits, int64_t ldw, void* stream) {
  if (!x || !sbits || !nzbits || M < 0 || K < 0 || ldx < K || ldw < (K + 31) / 32) {
    set_error("bnn_sign_pack_bits: bad arguments");
    return kErrInval;
  }
  if (M == 0 || ldw == 0) return 0;
  const int64_t waves = M * ((ldw + 1) / 2);
  hipLaunchKernelGGL(sign_pack_bits_k, dim3(grid_cap((waves + 3) / 4)), dim3(256), 0, S(stream), x,
                     M, K, ldx, sbits, nzbits, ldw);
  return check_launch("bnn_sign_pack_bits");
}

BNN_API int bnn_quant_rows(const float* x, int64_t M, int64_t K, int64_t ldx, int8_t* digits,
                           int64_t ldq, int64_t plane, float* scale, void* stream) {
  if (!x || !digits || !scale || M < 0 || K < 0 || ldx < K || ldq % TILE != 0 ||
      ldq < round_up(K, TILE) || plane < M * ldq || (plane % 16) != 0 || !aligned16(digits)) {
    set_error("bnn_quant_rows: bad arguments (M=%lld K=%lld ldq=%lld plane=%lld)", (long long)M,
              (long long)K, (long long)ldq, (long long)plane);
    return kErrInval;
  }
  if (M == 0) return 0;
  const int vec = aligned16(x) && (ldx % 4 == 0);
  hipLaunchKernelGGL(quant_rows_k, dim3((unsigned)std::min<int64_t>(M, 65536)), dim3(256), 0,
                     S(stream), x, M, K, ldx, digits, ldq, plane, scale, vec);
  return check_launch("bnn_quant_rows");
}

BNN_API int64_t bnn_quant_cols_workspace(int64_t M, int64_t N) {
  const int64_t R = col_chunks(M, N);
  return round_up(R * N * (int64_t)sizeof(float), 256) + R * N * (int64_t)sizeof(double);
}

BNN_API int bnn_quant_cols_t_dsum(const float* x, int64_t M, int64_t N, int64_t ldx, int8_t* digits_t,
                                  int64_t ldqt, int64_t plane, float* scale, float* colsum, int64_t* dsum,
                                  void* work, void* stream) {
  if (!x || !digits_t || !scale || !work || M < 0 || N < 0 || ldx < N || ldqt % TILE != 0 ||
      ldqt < round_up(M, TILE) || plane < N * ldqt || (plane % 16) != 0 || !aligned16(digits_t)) {
    set_error("bnn_quant_cols_t: bad arguments (M=%lld N=%lld ldqt=%lld plane=%lld)", (long long)M,
              (long long)N, (long long)ldqt, (long long)plane);
    return kErrInval;
  }
  if (N == 0) return 0;
  const int64_t R = col_chunks(M, N);
  if (R > 65535 || ldqt / TILE > 65535) {
    set_error("bnn_quant_cols_t: M too large for one launch (%lld)", (long long)M);
    return kErrInval;
  }
  float* pmax = reinterpret_cast<float*>(work);
  double* psum = reinterpret_cast<double*>(reinterpret_cast<char*>(work) +
                                           round_up(R * N * (int64_t)sizeof(float), 256));
  const unsigned gn = (unsigned)((N + 255) / 256);
  if (M > 0 && aligned16(x) && ldx % 4 == 0 && N % 4 == 0) {
    hipLaunchKernelGGL(colstats4_k, dim3((unsigned)((N / 4 + 255) / 256), (unsigned)R), dim3(256), 0, S(stream), x,
                       M, N, ldx, pmax, psum, col_chunk_rows(M, N));
  } else if (M > 0) {
    hipLaunchKernelGGL(colstats_k, dim3(gn, (unsigned)R), dim3(256), 0, S(stream), x, M, N, ldx, pmax,
                       psum, col_chunk_rows(M, N));
  } else {
    (void)hipMemsetAsync(pmax, 0, R * N * sizeof(float), S(stream));
    (void)hipMemsetAsync(psum, 0, R * N * sizeof(double), S(stream));
  }
  hipLaunchKernelGGL(colfinal_k, dim3((unsigned)((N + 63) / 64)), dim3(256), 0, S(stream), pmax, psum, N, R, scale,
                     colsum, dsum);
  const int vec = aligned16(x) && (ldx % 4 == 0);
  hipLaunchKernelGGL(quant_cols_t_k, dim3((unsigned)((N + TILE - 1) / TILE), (unsigned)(ldqt / TILE)),
                     dim3(256), 0, S(stream), x, M, N, ldx, scale, digits_t, ldqt, plane, vec, dsum);
  return check_launch("bnn_quant_cols_t");
}

BNN_API int bnn_quant_cols_t(const float* x, int64_t M, int64_t N, int64_t ldx, int8_t* digits_t,
                             int64_t ldqt, int64_t plane, float* scale, float* colsum, void* work,
                             void* stream) {
  return bnn_quant_cols_t_dsum(x, M, N, ldx, digits_t, ldqt, plane, scale, colsum, nullptr, work, stream);
}

// the 256 x 256 form from this many tiles up (below it, the 64 x 64 tiles fill the chip better)
#ifndef AP_FAST_MIN_TILES
#define AP_FAST_MIN_TILES 1024
#endif
BNN_API int bnn_bn_apply_pack(const float* x, int64_t M, int64_t C, const float* mean, const float* invstd,
                              const float* mean_lo, const float* gamma, const float* beta, int32_t fmt, void* q,
                              int64_t ldq, int8_t* qt, int64_t ldqt, int32_t qt_fmt, void* stream) {
  const int64_t need = fmt == 1 ? round_up(C, 256) / 2 : round_up(C, TILE);
  const int qf = qt_fmt == 2 ? 1 : qt_fmt;   // 2 = FP4 transpose in the panel layout
  if (!x || !mean || !invstd || M < 0 || C < 0 || (fmt != 0 && fmt != 1) || (!q && !qt) ||
      (q && (ldq < need || ldq % (fmt == 1 ? 128 : TILE) != 0 || !aligned16(q))) || !qt_ok(qt, M, ldqt, qf)) {
    set_error("bnn_bn_apply_pack: bad arguments (M=%lld C=%lld fmt=%d ldq=%lld ldqt=%lld)", (long long)M,
              (long long)C, fmt, (long long)ldq, (long long)ldqt);
    return kErrInval;
  }
  if (M == 0 && !qt) return 0;
  const int vec = aligned16(x) && (C % 4 == 0);
  const int64_t gx = q ? (fmt == 1 ? 2 * ldq : ldq) / TILE : (C + TILE - 1) / TILE;
  const int64_t gy = qt ? qt_tiles(ldqt, qf) : (M + TILE - 1) / TILE;
  if (gx == 0 || gy == 0) return 0;
  if (gy > 65535) {
    set_error("bnn_bn_apply_pack: M too large for one launch (%lld)", (long long)M);
    return kErrInval;
  }
  const ColAffine af{mean, mean_lo, invstd, gamma, beta,
                     aligned16(mean) && aligned16(invstd) && (!gamma || aligned16(gamma)) &&
                         (!beta || aligned16(beta)) && (!mean_lo || aligned16(mean_lo))};
  const bool fast = fmt == 1 && q && qt && (qt_fmt == 1 || qt_fmt == 2) && C % AP_T == 0 && af.vec && vec &&
                    (C / AP_T) * ((M + AP_T - 1) / AP_T) >= AP_FAST_MIN_TILES;
  if (fast) {
    hipLaunchKernelGGL((bn_apply_pack_fp4_k<0>), dim3((unsigned)(C / AP_T), (unsigned)((M + AP_T - 1) / AP_T)),
                       dim3(256), 0, S(stream), XIn{x, nullptr}, M, C, af, reinterpret_cast<uint8_t*>(q), ldq,
                       reinterpret_cast<uint8_t*>(qt), ldqt, qt_fmt == 2 ? ldqt / 32 : (int64_t)0);
    return check_launch("bnn_bn_apply_pack");
  }
  // 4 row tiles per workgroup when that still leaves >= 8K workgroups (amortised parameter loads)
  const int rt = (gx * ((gy + 3) / 4) >= 8192) ? 4 : 1;
  const unsigned gyr = (unsigned)((gy + rt - 1) / rt);
  if (fmt == 1)
    hipLaunchKernelGGL((sign_pack_tile_k<1, 1>), dim3((unsigned)gx, gyr), dim3(256), 0, S(stream), x, M,
                       C, C, reinterpret_cast<int8_t*>(q), ldq, qt, ldqt, vec, af, rt, gy, AdamArgs{}, qt_fmt);
  else
    hipLaunchKernelGGL((sign_pack_tile_k<0, 1>), dim3((unsigned)gx, gyr), dim3(256), 0, S(stream), x, M,
                       C, C, reinterpret_cast<int8_t*>(q), ldq, qt, ldqt, vec, af, rt, gy, AdamArgs{}, qt_fmt);
  return check_launch("bnn_bn_apply_pack");
}

// bnn_bn_apply_pack for the int16 form of the BatchNorm input (XIn z16: x = fl(I + xbias), the
// output of bnn_gemm_fp4_i16): FP4 rows + FP4 transpose only, C % 256 == 0, any M.
BNN_API int bnn_bn_apply_pack_i16(const int16_t* x16, const float* xbias, int64_t M, int64_t C, const float* mean,
                                  const float* invstd, const float* mean_lo, const float* gamma, const float* beta,
                                  uint8_t* q, int64_t ldq, uint8_t* qt, int64_t ldqt, int32_t qt_panel,
                                  void* stream) {
  const ColAffine af{mean, mean_lo, invstd, gamma, beta,
                     aligned16(mean) && aligned16(invstd) && (!gamma || aligned16(gamma)) &&
                         (!beta || aligned16(beta)) && (!mean_lo || aligned16(mean_lo))};
  if (!x16 || (reinterpret_cast<uintptr_t>(x16) & 7) != 0 || (xbias && !aligned16(xbias)) || !mean || !invstd ||
      !af.vec || M <= 0 || C <= 0 || C % AP_T != 0 || !q || !qt || ldq < C / 2 || !aligned16(q) ||
      !qt_ok(reinterpret_cast<const int8_t*>(qt), M, ldqt, 1) || (M + AP_T - 1) / AP_T > 65535) {
    set_error("bnn_bn_apply_pack_i16: bad arguments (M=%lld C=%lld ldq=%lld ldqt=%lld; C %% 256 == 0)", (long long)M,
              (long long)C, (long long)ldq, (long long)ldqt);
    return kErrInval;
  }
  hipLaunchKernelGGL((bn_apply_pack_fp4_k<1>), dim3((unsigned)(C / AP_T), (unsigned)((M + AP_T - 1) / AP_T)),
                     dim3(256), 0, S(stream), XIn{x16, xbias}, M, C, af, q, ldq, qt, ldqt, qt_panel ? ldqt / 32 : (int64_t)0);
  return check_launch("bnn_bn_apply_pack_i16");
}

// bnn_bn_apply_pack for the s20 form of the BatchNorm input (XIn XF 2: x = fl(fl(S * xscale) +
// xbias) from the u8-pixel layer's 20-bit sums, bnn_gemm_i8_affine_bnstats_s20): FP4 rows + FP4
// transpose only, C % 256 == 0, any M.
BNN_API int bnn_bn_apply_pack_s20(const int16_t* xlo, const uint8_t* xhi, const float* xbias, float xscale, int64_t M,
                                  int64_t C, const float* mean, const float* invstd, const float* mean_lo,
                                  const float* gamma, const float* beta, uint8_t* q, int64_t ldq, uint8_t* qt,
                                  int64_t ldqt, int32_t qt_panel, void* stream) {
  const ColAffine af{mean, mean_lo, invstd, gamma, beta,
                     aligned16(mean) && aligned16(invstd) && (!gamma || aligned16(gamma)) &&
                         (!beta || aligned16(beta)) && (!mean_lo || aligned16(mean_lo))};
  if (!xlo || (reinterpret_cast<uintptr_t>(xlo) & 7) != 0 || !xhi || (reinterpret_cast<uintptr_t>(xhi) & 1) != 0 ||
      (xbias && !aligned16(xbias)) || !mean || !invstd || !af.vec || M <= 0 || C <= 0 || C % AP_T != 0 || !q || !qt ||
      ldq < C / 2 || !aligned16(q) || !qt_ok(reinterpret_cast<const int8_t*>(qt), M, ldqt, 1) ||
      (M + AP_T - 1) / AP_T > 65535) {
    set_error("bnn_bn_apply_pack_s20: bad arguments (M=%lld C=%lld ldq=%lld ldqt=%lld; C %% 256 == 0)", (long long)M,
              (long long)C, (long long)ldq, (long long)ldqt);
    return kErrInval;
  }
  hipLaunchKernelGGL((bn_apply_pack_fp4_k<2>), dim3((unsigned)(C / AP_T), (unsigned)((M + AP_T - 1) / AP_T)),
                     dim3(256), 0, S(stream), XIn{xlo, xbias, xhi, xscale}, M, C, af, q, ldq, qt, ldqt,
                     qt_panel ? ldqt / 32 : (int64_t)0);
  return check_launch("bnn_bn_apply_pack_s20");
}

namespace bnn {
int bn_bwd_sums(XIn xin, int xf, const float* dy, int64_t M, int64_t C, const float* gamma, const float* beta,
                const float* save_mean, const float* save_invstd, const float* save_mean_lo, int32_t hardtanh,
                float* dgamma, float* dbeta, void* work, hipStream_t s, const float** k0_out, const float** k1_out,
                float* pmx = nullptr, float* scale = nullptr, int64_t* dsum = nullptr);
int64_t bn_workspace_bytes(int64_t M, int64_t C);
void bn_stat_slots(void* work, int64_t M, int64_t C, const float** k0, const float** k1);
int64_t bn_reduce_chunks(int64_t M, int64_t C);
}  // namespace bnn

// workspace: the statistics pass's | its per-chunk maxima (2 x chunks x C floats) | the
// quantiser's per-strip column sums (strips x C doubles)
static int64_t i8c_pmx_bytes(int64_t M, int64_t C) {
  return round_up(2 * bn_reduce_chunks(M, C) * C * (int64_t)sizeof(float), 256);
}

BNN_API int64_t bnn_bn_bwd_i8cols_workspace(int64_t M, int64_t C) {
  return round_up(bn_workspace_bytes(M, C), 256) + i8c_pmx_bytes(M, C) + qc_strips(M, qc_rt(M, C)) * C * (int64_t)sizeof(double);
}

static int bn_bwd_i8cols_impl(XIn xin, int xf, const float* dy, int64_t M, int64_t C, const float* gamma,
                              const float* beta, const float* save_mean, const float* save_invstd,
                              const float* save_mean_lo, int32_t hardtanh, float* dgamma, float* dbeta,
                              int8_t* digits_t, int64_t ldqt, int64_t plane, float* scale, float* colsum,
                              int64_t* dsum, void* work, void* stream, bool pre) {
  const bool x_ok = xf == 2 ? (xin.p && (reinterpret_cast<uintptr_t>(xin.p) & 7) == 0 && xin.hi &&
                               (reinterpret_cast<uintptr_t>(xin.hi) & 1) == 0 && (!xin.bias || aligned16(xin.bias)))
                            : (xf == 0 && xin.p && aligned16(xin.p));
  if (!x_ok || !dy || !digits_t || !scale || !work || M <= 0 || C <= 0 || C % 4 != 0 ||
      !aligned16(dy) || ldqt % TILE != 0 || ldqt < round_up(M, TILE) || plane < C * ldqt || plane % 16 != 0 ||
      !aligned16(digits_t) || col_chunks(M, C) > 65535 || ldqt / TILE > 65535 || !aligned16(save_mean) ||
      !aligned16(save_invstd) || (save_mean_lo && !aligned16(save_mean_lo)) || (gamma && !aligned16(gamma)) ||
      (beta && !aligned16(beta))) {
    set_error("bnn_bn_bwd_i8cols: bad arguments (M=%lld C=%lld ldqt=%lld plane=%lld)", (long long)M, (long long)C,
              (long long)ldqt, (long long)plane);
    return kErrInval;
  }
  hipStream_t s = S(stream);
  const float *k0, *k1;
  char* qw = reinterpret_cast<char*>(work) + round_up(bn_workspace_bytes(M, C), 256);
  float* pmx = reinterpret_cast<float*>(qw);
  double* part = reinterpret_cast<double*>(qw + i8c_pmx_bytes(M, C));
  // statistics pass + its final merge, which also writes scale (from the bound) and zeroes dsum;
  // pre: bnn_bn_bwd_stats_pre (mode 2) already did, from the dX GEMM's epilogue partials
  if (pre) {
    bn_stat_slots(work, M, C, &k0, &k1);
  } else {
    const int rc = bn_bwd_sums(xin, xf, dy, M, C, gamma, beta, save_mean, save_invstd, save_mean_lo, hardtanh, dgamma, dbeta,
                               work, s, &k0, &k1, pmx, scale, dsum);
    if (rc) return rc;
  }
  const BnCols bc{save_mean, save_mean_lo, save_invstd, gamma, beta, k0, k1, 1.f / (float)M, hardtanh};
  const int rt = qc_rt(M, C);
  const dim3 qg((unsigned)((C + TILE - 1) / TILE), (unsigned)((ldqt / TILE + rt - 1) / rt));
  if (xf == 2)
    hipLaunchKernelGGL(bn_dz_quant_cols_t_k<2>, qg, dim3(256), 0, s, xin, dy, M, C, bc, scale, digits_t, ldqt, plane,
                       dsum, colsum ? part : nullptr, rt);
  else
    hipLaunchKernelGGL(bn_dz_quant_cols_t_k<0>, qg, dim3(256), 0, s, xin, dy, M, C, bc, scale, digits_t, ldqt, plane,
                       dsum, colsum ? part : nullptr, rt);
  if (colsum)
    hipLaunchKernelGGL(bn_dz_colsum_k, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, part, qc_strips(M, rt), C, colsum);
  return check_launch("bnn_bn_bwd_i8cols");
}

BNN_API int bnn_bn_bwd_i8cols(const float* x, const float* dy, int64_t M, int64_t C, const float* gamma,
                              const float* beta, const float* save_mean, const float* save_invstd,
                              const float* save_mean_lo, int32_t hardtanh, float* dgamma, float* dbeta,
                              int8_t* digits_t, int64_t ldqt, int64_t plane, float* scale, float* colsum,
                              int64_t* dsum, void* work, void* stream) {
  return bn_bwd_i8cols_impl(XIn{x, nullptr}, 0, dy, M, C, gamma, beta, save_mean, save_invstd, save_mean_lo, hardtanh,
                            dgamma, dbeta, digits_t, ldqt, plane, scale, colsum, dsum, work, stream, false);
}

// bnn_bn_bwd_i8cols after bnn_bn_bwd_stats_pre (mode 2): the statistics, the digit scale and the
// zeroed digit sums are already in place; only the quantising pass runs
BNN_API int bnn_bn_bwd_i8cols_pre(const float* x, const float* dy, int64_t M, int64_t C, const float* gamma,
                                  const float* beta, const float* save_mean, const float* save_invstd,
                                  const float* save_mean_lo, int32_t hardtanh, float* dgamma, float* dbeta,
                                  int8_t* digits_t, int64_t ldqt, int64_t plane, float* scale, float* colsum,
                                  int64_t* dsum, void* work, void* stream) {
  return bn_bwd_i8cols_impl(XIn{x, nullptr}, 0, dy, M, C, gamma, beta, save_mean, save_invstd, save_mean_lo, hardtanh,
                            dgamma, dbeta, digits_t, ldqt, plane, scale, colsum, dsum, work, stream, true);
}

// bnn_bn_bwd_i8cols[_pre] for the s20 form of the BatchNorm input (the u8-pixel layer's 20-bit sums
// from bnn_gemm_i8_affine_bnstats_s20: x = fl(fl(S * scale) + xbias)); same outputs, bit for bit
BNN_API int bnn_bn_bwd_i8cols_s20(const int16_t* xlo, const uint8_t* xhi, const float* xbias, float xscale,
                                  const float* dy, int64_t M, int64_t C, const float* gamma, const float* beta,
                                  const float* save_mean, const float* save_invstd, const float* save_mean_lo,
                                  int32_t hardtanh, float* dgamma, float* dbeta, int8_t* digits_t, int64_t ldqt,
                                  int64_t plane, float* scale, float* colsum, int64_t* dsum, void* work, void* stream) {
  return bn_bwd_i8cols_impl(XIn{xlo, xbias, xhi, xscale}, 2, dy, M, C, gamma, beta, save_mean, save_invstd,
                            save_mean_lo, hardtanh, dgamma, dbeta, digits_t, ldqt, plane, scale, colsum, dsum, work,
                            stream, false);
}

BNN_API int bnn_bn_bwd_i8cols_s20_pre(const int16_t* xlo, const uint8_t* xhi, const float* xbias, float xscale,
                                      const float* dy, int64_t M, int64_t C, const float* gamma, const float* beta,
                                      const float* save_mean, const float* save_invstd, const float* save_mean_lo,
                                      int32_t hardtanh, float* dgamma, float* dbeta, int8_t* digits_t, int64_t ldqt,
                                      int64_t plane, float* scale, float* colsum, int64_t* dsum, void* work,
                                      void* stream) {
  return bn_bwd_i8cols_impl(XIn{xlo, xbias, xhi, xscale}, 2, dy, M, C, gamma, beta, save_mean, save_invstd,
                            save_mean_lo, hardtanh, dgamma, dbeta, digits_t, ldqt, plane, scale, colsum, dsum, work,
                            stream, true);
}
