// BatchNorm1d (train/eval) with an optional fused Hardtanh, for the [B, C] activations between
// the binarized layers (mnist-dist2.py:52-74: fc -> BatchNorm1d -> Hardtanh).
//
// torch's channels-last BN kernels take ~17-21 ms per call on a [65536, 8192] fp32 tensor on
// MI355X (profiles/r01_wide_b65536_kernel_stats.csv): this file replaces them with HBM-streaming
// passes -- a column reduction (per 256-row chunk, merged in a fixed order: deterministic) and a
// float4 elementwise pass.
//
// Forward (train): mean, biased var over the batch; y = (x-mean)*invstd*gamma + beta;
// the mean is kept as an fp32 pair hi + lo of the batch sum taken in double (exact for the
// integer-plus-bias pre-activations of the binarized layers), and x - mean is evaluated as
// (x - hi) - lo, so the sign of a normalised value that sits within an ulp of the mean (a
// BatchNorm near-tie: z_i ~ mean is common when z is integer-valued) is the sign of the exact
// difference -- the next BinarizeLinear's sign() then agrees with exact arithmetic;
// running_mean/var updated with the unbiased var (torch semantics); hardtanh -> clamp(y,-1,1).
// Backward: with g = dy * (hardtanh ? (-1 < y < 1) : 1) (y recomputed from x, not stored),
// dbeta = sum g, dgamma = sum g*xhat, dx = gamma*invstd*(g - dbeta/n - xhat*dgamma/n).
#include <algorithm>
#include <cmath>

#include "bnn_common.h"
#include "bnn_fp6.h"
#include "bnn_bn2d.h"

namespace bnn {
const int64_t* g_seed_ctr = nullptr;   // bnn_set_seed_counter (declared in bnn_common.h)
namespace {

constexpr int BN_ROWS = 256;  // most rows per partial-statistics chunk

// Rows per chunk of the column reductions: 256, halved while the reduction (one thread per 4
// columns and chunk) would have fewer than 2^17 threads -- a [4096, 3072] batch gets 16-row
// chunks (196 K threads) instead of 48 workgroups, a [65536, 8192] one keeps 256.
#ifndef BN_FILL_LOG2
#define BN_FILL_LOG2 16
#endif
inline int64_t bn_chunk_rows(int64_t M, int64_t C) {
  int64_t rows = BN_ROWS;
  while (rows > 1 && (C / 4) * ((M + rows - 1) / rows) < (1 << BN_FILL_LOG2)) rows >>= 1;
  return rows;
}
inline int64_t bn_chunks(int64_t M, int64_t C) {
  const int64_t rows = bn_chunk_rows(M, C);
  return std::max<int64_t>(1, (M + rows - 1) / rows);
}
inline dim3 reduce_grid(int64_t M, int64_t C) {
  return dim3((unsigned)(((C / 4) * bn_chunks(M, C) + 255) / 256));
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// Drop, drop_hash, drop_resolve, g_seed_ctr: bnn_common.h (the FP4 statistics epilogue evaluates
// the same mask)

// drop_bits4 (bnn_common.h): keep bits of elements i0 .. i0+3, evaluated once and applied to both
// the input and the gradient where a pass needs both

__device__ __forceinline__ void drop4m(const Drop& d, uint32_t m, float (&v)[4]) {
  if (!d.on) return;
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = ((m >> j) & 1u) ? v[j] * d.scale : 0.f;
}

__device__ __forceinline__ void drop4(const Drop& d, uint64_t i0, float (&v)[4]) {
  if (!d.on) return;
  drop4m(d, drop_bits4(d, i0), v);
}


// Waves per SIMD the reduction passes are compiled for (they wait on memory: occupancy is their
// lever; RED_OCC / HRED_OCC = 1 leaves the compiler's choice)
#ifndef RED_OCC
#define RED_OCC 1
#endif
#ifndef HRED_OCC
#define HRED_OCC 1
#endif
#ifndef RED_RB
#define RED_RB 8   // rows per load batch of bn_reduce_k (divides 16)
#endif

// MODE 0: per-chunk (mean, M2), accumulated as deviations from the chunk's first row so the
//         float partials see deviations rather than raw magnitudes; merged with Chan's formula.
// MODE 1: per-chunk (sum g, sum g*xhat) with g = dy*mask(y).
// MODE 2: MODE 1 (the same sums, bit for bit) + per-chunk max|g| and max|xhat| into pmx
//         ([chunks][C] each, max|xhat| R*C floats after max|g|): the a-priori bound on |dz| that
//         bnn_bn_bwd_i8cols scales its int8 column digits by (no column-max pass over dz).
// One thread = 4 adjacent columns (float4), rows walked in 16-row float partials folded to double.
template <int MODE, int XF = 0>
__global__ __launch_bounds__(256, RED_OCC) void bn_reduce_k(XIn xin, const float* __restrict__ dy,
                                                   int64_t M, int64_t C, const float* __restrict__ mean,
                                                   const float* __restrict__ mean_lo,
                                                   const float* __restrict__ invstd,
                                                   const float* __restrict__ gamma,
                                                   const float* __restrict__ beta, int hardtanh,
                                                   double* __restrict__ p0, double* __restrict__ p1,
                                                   int64_t chunk_rows, Drop dp0 = Drop{0, 0, 0, 1.f},
                                                   float* __restrict__ pmx = nullptr) {
  constexpr bool BWD = MODE >= 1;
  const Drop dp = drop_resolve(dp0);
  // thread -> (4-column group, chunk): consecutive threads read consecutive columns of a row
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t C4 = C / 4;
  const int64_t chunk = id / C4;
  const int64_t c = (id - chunk * C4) * 4;
  const int64_t r0 = chunk * chunk_rows;
  if (r0 >= M) return;
  const int64_t r1 = (M < r0 + chunk_rows) ? M : r0 + chunk_rows;
  double a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0}, sx[4] = {0, 0, 0, 0};
  float mu[4], lo[4] = {0, 0, 0, 0}, is[4] = {1, 1, 1, 1}, ga[4] = {1, 1, 1, 1}, be[4] = {0, 0, 0, 0};
  float gmx[4] = {0, 0, 0, 0}, xmx[4] = {0, 0, 0, 0};   // MODE 2
  const float4 xb = xin_bias4<XF>(xin, c);
  if (MODE == 0) {
    const float4 sv = xin_load4<XF>(xin, r0 * C + c, xb);
    mu[0] = sv.x;
    mu[1] = sv.y;
    mu[2] = sv.z;
    mu[3] = sv.w;
    drop4(dp, (uint64_t)(r0 * C + c), mu);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mu[j] = mean[c + j];
      lo[j] = mean_lo ? mean_lo[c + j] : 0.f;
      is[j] = invstd[c + j];
      ga[j] = gamma ? gamma[c + j] : 1.f;
      be[j] = beta ? beta[c + j] : 0.f;
    }
  }
  // rows in batches of RB whose loads are all issued before any is used (several KiB in flight
  // per wave: the pass is latency-bound otherwise); the arithmetic order is unchanged
  constexpr int RB = RED_RB;
  for (int64_t r = r0; r < r1; r += 16) {
    float fa[4] = {0, 0, 0, 0}, fb[4] = {0, 0, 0, 0};
    const int64_t re = (r + 16 < r1) ? r + 16 : r1;
    for (int64_t rb = r; rb < re; rb += RB) {
    float4 xv8[RB], gb[BWD ? RB : 1];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int64_t rr = rb + u < re ? rb + u : re - 1;
      xv8[u] = xin_load4<XF>(xin, rr * C + c, xb);
      if constexpr (BWD) gb[u] = ld4(dy + rr * C + c);
    }
    uint32_t kw = 0;   // MODE 0: the batch's keep bits (rows past the end stay 0)
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int64_t rr = rb + u;
      if (rr >= re) break;
      const float4 xv = xv8[u];
      float xs[4] = {xv.x, xv.y, xv.z, xv.w};
      const uint32_t km = dp.on ? drop_bits4(dp, (uint64_t)(rr * C + c)) : 0u;
      drop4m(dp, km, xs);
      kw |= km << (4 * u);
      if (MODE == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = xs[j] - mu[j];
          fa[j] += d;
          fb[j] = fmaf(d, d, fb[j]);
          sx[j] += (double)xs[j];      // exact batch sum (see file header)
        }
      } else {
        const float4 gv = gb[BWD ? u : 0];
        const float gs[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float xh = ((xs[j] - mu[j]) - lo[j]) * is[j];
          const float y = fmaf(xh, ga[j], be[j]);
          const float g = (!hardtanh || (y > -1.f && y < 1.f)) ? gs[j] : 0.f;
          fa[j] += g;
          fb[j] = fmaf(g, xh, fb[j]);
          if constexpr (MODE == 2) {   // NaN -> inf: the bound (and the scale) become non-finite
            const float ag = fabsf(g), ax = fabsf(xh);
            gmx[j] = (ag == ag) ? fmaxf(gmx[j], ag) : __builtin_inff();
            xmx[j] = (ax == ax) ? fmaxf(xmx[j], ax) : __builtin_inff();
          }
        }
      }
    }
    // the keep-bit plane (host: only with 8-row batches starting at multiples of 8)
    if constexpr (MODE == 0 && RB == 8)
      if (dp.bits_out != nullptr) dp.bits_out[keep_word(rb, c, C)] = kw;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] += (double)fa[j];
      b[j] += (double)fb[j];
    }
  }
  const int64_t o = chunk * C + c;
  if (MODE == 0) {
    const double n = (double)(r1 - r0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double dm = a[j] / n;
      p0[o + j] = sx[j];               // chunk sum
      p1[o + j] = b[j] - a[j] * dm;    // chunk M2 = sum d^2 - (sum d)^2 / n (about the chunk mean)
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p0[o + j] = a[j];
      p1[o + j] = b[j];
    }
    if constexpr (MODE == 2) {
      const int64_t RC = ((M + chunk_rows - 1) / chunk_rows) * C;
      *reinterpret_cast<float4*>(pmx + o) = make_float4(gmx[0], gmx[1], gmx[2], gmx[3]);
      *reinterpret_cast<float4*>(pmx + RC + o) = make_float4(xmx[0], xmx[1], xmx[2], xmx[3]);
    }
  }
}

// Final merges of the per-chunk partials: 16 chunk groups x 16 columns per workgroup (128-B row
// segments per load; 4 columns x 64 groups coalesced worse and ran 1-3x slower), a fixed group
// split and fold order (deterministic).  The forward merge takes two independent passes instead of
// a serial Chan chain (two dependent double divisions per chunk): the batch sum first (its
// fixed-order double sum gives the mean), then M2 = sum_r [M2_r + n_r (S_r / n_r - mean)^2].
#ifndef BN_FF_B
#define BN_FF_B 8   // partials per batched load round (A/B hook; any value keeps the summation order)
#endif
constexpr int FF_COLS = 16, FF_GROUPS = 16, FF_B = BN_FF_B;

inline dim3 ffin_grid(int64_t C) { return dim3((unsigned)((C + FF_COLS - 1) / FF_COLS)); }

__global__ __launch_bounds__(256) void bn_fwd_final_k(const double* __restrict__ p0, const double* __restrict__ p1,
                                                      int64_t M, int64_t C, int64_t R, float momentum, float eps,
                                                      float* __restrict__ rmean, float* __restrict__ rvar,
                                                      float* __restrict__ save_mean,
                                                      float* __restrict__ save_invstd,
                                                      float* __restrict__ save_mean_lo, int64_t chunk_rows,
                                                      int64_t hw) {
  // chunk r covers rows [r*chunk_rows, min((r+1)*chunk_rows, M)) of hw elements each (hw = 1 for
  // BatchNorm1d; H*W for the NCHW BatchNorm2d); p0 = chunk sum, p1 = chunk M2 about its mean
  __shared__ double red[FF_GROUPS][FF_COLS];
  __shared__ double smean[FF_COLS];
  const int lc = threadIdx.x & (FF_COLS - 1), grp = threadIdx.x / FF_COLS;
  const int64_t c = (int64_t)blockIdx.x * FF_COLS + lc;
  const bool live = c < C;
  const int64_t cc = live ? c : C - 1;
  // pass 1: the batch sum
  double s = 0.0;
  for (int64_t rb = grp; rb < R; rb += FF_B * FF_GROUPS) {
    double q[FF_B];
#pragma unroll
    for (int u = 0; u < FF_B; ++u) q[u] = p0[min(rb + u * FF_GROUPS, R - 1) * C + cc];   // loads batch
#pragma unroll
    for (int u = 0; u < FF_B; ++u)
      if (rb + u * FF_GROUPS < R) s += q[u];
  }
  red[grp][lc] = s;
  __syncthreads();
  const double n = (double)(M * hw);
  if (grp == 0) {
    double t = 0.0;
    for (int g = 0; g < FF_GROUPS; ++g) t += red[g][lc];   // fixed order
    smean[lc] = t;
  }
  __syncthreads();
  const double sum = smean[lc], mean = sum / n;
  // pass 2: M2 about the batch mean
  const double nb_full = (double)(chunk_rows * hw), inv_full = 1.0 / nb_full;
  double m2 = 0.0;
  for (int64_t rb = grp; rb < R; rb += FF_B * FF_GROUPS) {
    double q0[FF_B], q1[FF_B];
#pragma unroll
    for (int u = 0; u < FF_B; ++u) {
      const int64_t r = min(rb + u * FF_GROUPS, R - 1);
      q0[u] = p0[r * C + cc];
      q1[u] = p1[r * C + cc];
    }
#pragma unroll
    for (int u = 0; u < FF_B; ++u) {
      const int64_t r = rb + u * FF_GROUPS;
      if (r >= R) break;
      const int64_t hi = ((r + 1) * chunk_rows < M) ? (r + 1) * chunk_rows : M;
      const bool full = hi - r * chunk_rows == chunk_rows;
      const double nb = full ? nb_full : (double)((hi - r * chunk_rows) * hw);
      const double d = (full ? q0[u] * inv_full : q0[u] / nb) - mean;
      m2 += q1[u] + nb * d * d;
    }
  }
  __syncthreads();
  red[grp][lc] = m2;
  __syncthreads();
  if (grp != 0 || !live) return;
  m2 = 0.0;
  for (int g = 0; g < FF_GROUPS; ++g) m2 += red[g][lc];   // fixed order
  double var = m2 / n;
  if (var < 0.0) var = 0.0;
  const float mh = (float)mean;
  save_mean[c] = mh;
  if (save_mean_lo) save_mean_lo[c] = (float)(mean - (double)mh);
  save_invstd[c] = (float)(1.0 / std::sqrt(var + (double)eps));
  if (rmean != nullptr && momentum >= 0.f) {
    const double unb = n > 1.0 ? m2 / (n - 1.0) : var;
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

// Elementwise passes on a 2-D grid: blockIdx.x = 1024-column block (one float4 per thread),
// blockIdx.y = APPLY_ROWS-row chunk.  Each thread keeps its 4 columns' parameters in registers and
// walks the rows (per row the workgroup touches one contiguous 4 KiB segment): no per-element
// index modulo and no per-element reloads of the column vectors.
// Rows per workgroup: 64, halved (down to 4) while the grid has fewer than 2048 workgroups.
constexpr int APPLY_ROWS = 64;

__host__ __device__ inline int64_t apply_rows(int64_t M, int64_t C) {
  int64_t rows = APPLY_ROWS;
  while (rows > 4 && ((C / 4 + 255) / 256) * ((M + rows - 1) / rows) < 2048) rows >>= 1;
  return rows;
}

inline dim3 apply_grid(int64_t M, int64_t C) {
  const int64_t rows = apply_rows(M, C);
  return dim3((unsigned)((C / 4 + 255) / 256), (unsigned)((M + rows - 1) / rows));
}

__global__ __launch_bounds__(256) void bn_apply_k(const float* __restrict__ x, int64_t M, int64_t C,
                                                  const float* __restrict__ mean,
                                                  const float* __restrict__ mean_lo,
                                                  const float* __restrict__ invstd,
                                                  const float* __restrict__ gamma,
                                                  const float* __restrict__ beta, int hardtanh,
                                                  float* __restrict__ y, Drop dp0 = Drop{0, 0, 0, 1.f}) {
  const Drop dp = drop_resolve(dp0);
  const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (c >= C) return;
  const int64_t ar = apply_rows(M, C);
  const int64_t r0 = (int64_t)blockIdx.y * ar, r1 = (r0 + ar < M) ? r0 + ar : M;
  const float4 mv = ld4(mean + c), iv = ld4(invstd + c), lv = ld4_or(mean_lo, c, 0.f);
  const float4 gv = ld4_or(gamma, c, 1.f), bv = ld4_or(beta, c, 0.f);
  const float mu[4] = {mv.x, mv.y, mv.z, mv.w}, is[4] = {iv.x, iv.y, iv.z, iv.w};
  const float lo[4] = {lv.x, lv.y, lv.z, lv.w};
  const float ga[4] = {gv.x, gv.y, gv.z, gv.w}, be[4] = {bv.x, bv.y, bv.z, bv.w};
  for (int64_t r = r0; r < r1; ++r) {
    const float4 xv = ld4(x + r * C + c);
    float xs[4] = {xv.x, xv.y, xv.z, xv.w};
    drop4(dp, (uint64_t)(r * C + c), xs);
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = fmaf(((xs[j] - mu[j]) - lo[j]) * is[j], ga[j], be[j]);
      if (hardtanh) v[j] = fminf(fmaxf(v[j], -1.f), 1.f);
    }
    *reinterpret_cast<float4*>(y + r * C + c) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// I8C (optional, bnn_bn_bwd_i8cols): also folds bn_reduce_k MODE 2's per-chunk max|g| / max|xhat|
// (pmx) and writes the int8 column-digit scale from the bound on |dz| (see bnn_pack.hip,
// bn_dz_quant_cols_t_k) plus zeroed digit sums.
struct I8cBound {
  const float* pmx;       // [R][C] max|g|, then [R][C] max|xhat|; null = off
  const float* invstd;
  const float* gamma;
  float inv_n;
  float* scale;
  int64_t* dsum;
};

// PT = double: bn_reduce_k's per-chunk partials; float: the FP6 dX GEMM's per-tile-row epilogue
// statistics (bnn_gemm_fp6_bnstats -> bnn_bn_bwd_stats_pre)
template <typename PT>
__device__ __forceinline__ void bn_bwd_final_body(const PT* __restrict__ p0,
                                                      const PT* __restrict__ p1, int64_t C, int64_t R,
                                                      float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                      float* __restrict__ k0, float* __restrict__ k1,
                                                      I8cBound ib) {
  __shared__ double sa[FF_GROUPS][FF_COLS], sb[FF_GROUPS][FF_COLS];
  __shared__ float sg[FF_GROUPS][FF_COLS], sx[FF_GROUPS][FF_COLS];
  const int lc = threadIdx.x & (FF_COLS - 1), grp = threadIdx.x / FF_COLS;
  const int64_t c = (int64_t)blockIdx.x * FF_COLS + lc;
  double s = 0.0, s2 = 0.0;
  float gm = 0.f, xm = 0.f;
  if (c < C)
    for (int64_t rb = grp; rb < R; rb += FF_B * FF_GROUPS) {   // batched loads, fixed order
      PT q0[FF_B], q1[FF_B];
      float qg[FF_B], qx[FF_B];
#pragma unroll
      for (int u = 0; u < FF_B; ++u) {
        const int64_t r = rb + u * FF_GROUPS;
        q0[u] = p0[min(r, R - 1) * C + c];   // clamped, unconditional: the loads batch
        q1[u] = p1[min(r, R - 1) * C + c];
        qg[u] = (r < R && ib.pmx != nullptr) ? ib.pmx[r * C + c] : 0.f;
        qx[u] = (r < R && ib.pmx != nullptr) ? ib.pmx[(R + r) * C + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < FF_B; ++u) {
        if (rb + u * FF_GROUPS >= R) break;
        s += q0[u];
        s2 += q1[u];
        gm = fmaxf(gm, qg[u]);
        xm = fmaxf(xm, qx[u]);
      }
    }
  sa[grp][lc] = s;
  sb[grp][lc] = s2;
  sg[grp][lc] = gm;
  sx[grp][lc] = xm;
  __syncthreads();
  if (grp != 0 || c >= C) return;
  s = 0.0, s2 = 0.0;
  for (int gI = 0; gI < FF_GROUPS; ++gI) {   // fixed order
    s += sa[gI][lc];
    s2 += sb[gI][lc];
    gm = fmaxf(gm, sg[gI][lc]);
    xm = fmaxf(xm, sx[gI][lc]);
  }
  if (dbeta) dbeta[c] = (float)s;
  if (dgamma) dgamma[c] = (float)s2;
  k0[c] = (float)s;
  k1[c] = (float)s2;
  if (ib.pmx != nullptr) {
    // |dz| = |gamma*invstd| |g - a0 - xhat*a1| <= |gamma*invstd| (max|g| + |a0| + max|xhat| |a1|), with
    // a0, a1 formed as the passes that compute dz form them; 1 + 2^-16 covers bn_dz1's roundings
    const float is = ib.invstd[c], ga = ib.gamma ? ib.gamma[c] : 1.f;
    const float a0 = (float)s * ib.inv_n, a1 = (float)s2 * ib.inv_n;
    const float bound = fabsf(ga * is) * ((gm + fabsf(a0)) + xm * fabsf(a1)) * (1.f + 0x1p-16f);
    int shift;
    float sc;
    digit_scale(bound, &shift, &sc);
    ib.scale[c] = sc;
    if (ib.dsum != nullptr) ib.dsum[c] = 0;
  }
}

__global__ __launch_bounds__(256) void bn_bwd_final_k(const double* __restrict__ p0, const double* __restrict__ p1,
                                                      int64_t C, int64_t R, float* __restrict__ dgamma,
                                                      float* __restrict__ dbeta, float* __restrict__ k0,
                                                      float* __restrict__ k1,
                                                      I8cBound ib = I8cBound{nullptr, nullptr, nullptr, 0.f, nullptr, nullptr}) {
  bn_bwd_final_body<double>(p0, p1, C, R, dgamma, dbeta, k0, k1, ib);
}

__global__ __launch_bounds__(256) void bn_bwd_final_pre_k(const float* __restrict__ p0, const float* __restrict__ p1,
                                                          int64_t C, int64_t R, float* __restrict__ dgamma,
                                                          float* __restrict__ dbeta, float* __restrict__ k0,
                                                          float* __restrict__ k1, I8cBound ib) {
  bn_bwd_final_body<float>(p0, p1, C, R, dgamma, dbeta, k0, k1, ib);
}

__global__ __launch_bounds__(256) void bn_bwd_apply_k(const float* __restrict__ x, const float* __restrict__ dy,
                                                      int64_t M, int64_t C, const float* __restrict__ mean,
                                                      const float* __restrict__ mean_lo,
                                                      const float* __restrict__ invstd,
                                                      const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, int hardtanh,
                                                      const float* __restrict__ sg,
                                                      const float* __restrict__ sgx, float inv_n,
                                                      float* __restrict__ dx, Drop dp0 = Drop{0, 0, 0, 1.f}) {
  const Drop dp = drop_resolve(dp0);
  // inv_n = 1/M with batch statistics (train); 0 in eval mode, where mean/invstd are the running
  // statistics (constants): dx = gamma*invstd*g
  const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (c >= C) return;
  const int64_t ar = apply_rows(M, C);
  const int64_t r0 = (int64_t)blockIdx.y * ar, r1 = (r0 + ar < M) ? r0 + ar : M;
  const float4 mv = ld4(mean + c), iv = ld4(invstd + c), s0 = ld4(sg + c), s1 = ld4(sgx + c);
  const float4 gav = ld4_or(gamma, c, 1.f), bev = ld4_or(beta, c, 0.f), lv = ld4_or(mean_lo, c, 0.f);
  const float ms[4] = {mv.x, mv.y, mv.z, mv.w}, is[4] = {iv.x, iv.y, iv.z, iv.w};
  const float lo[4] = {lv.x, lv.y, lv.z, lv.w};
  const float ga[4] = {gav.x, gav.y, gav.z, gav.w}, be[4] = {bev.x, bev.y, bev.z, bev.w};
  const float a0[4] = {s0.x * inv_n, s0.y * inv_n, s0.z * inv_n, s0.w * inv_n};
  const float a1[4] = {s1.x * inv_n, s1.y * inv_n, s1.z * inv_n, s1.w * inv_n};
  for (int64_t r = r0; r < r1; ++r) {
    const float4 xv = ld4(x + r * C + c), gv = ld4(dy + r * C + c);
    float xs[4] = {xv.x, xv.y, xv.z, xv.w};
    const float gs[4] = {gv.x, gv.y, gv.z, gv.w};
    const uint32_t km = dp.on ? drop_bits4(dp, (uint64_t)(r * C + c)) : 0u;
    drop4m(dp, km, xs);
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = bn_dz1(xs[j], gs[j], ms[j], lo[j], is[j], ga[j], be[j], a0[j], a1[j], hardtanh);
    drop4m(dp, km, o);   // dropout backward: grad * mask * scale
    *reinterpret_cast<float4*>(dx + r * C + c) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

// ------------------------------------------------------------------ fused backward apply + FP6 quantise
// The apply pass of the BatchNorm backward whose output dz is the upstream gradient dY of the
// BinarizeLinear that produced z (mnist-dist2.py:66-71: fc -> bn -> htanh -> fc).  That layer's
// backward multiplies dY twice on the FP6 MFMA (dX = dY.W_b, dW = dY^T.X_b, bnn_gemm6.hip), so
// this pass writes, besides dz itself (optional), both FP6 digit forms of dz from an LDS tile --
// the rows (blocks of 32 columns) and the transpose (blocks of 32 rows) -- and the per-workgroup
// partial column sums of dz (the bias gradient): dz is never re-read.  Bit-identical digits to
// bnn_quant6_rows / bnn_quant6_cols_t of the same dz.
// Workgroup: Q6T_ROWS (512, or 64 on small batches: q6_rows) rows x 64 columns, walked as sub-tiles
// of 64 rows; C % 64 == 0.  Per sub-tile all 256 threads compute dz (float4 per thread and row)
// into the LDS tile, then waves 0-1 quantise the 128 row blocks (one 32-element block per lane)
// and waves 2-3 the 128 column blocks, their digit records staged in LDS for whole-line stores.
constexpr int Q6T_ROWS = 512, Q6T_SUB = 64, Q6T_COLS = 64, Q6T_LD = Q6T_COLS + 4;
#ifndef Q6_HEAD_OCC
#define Q6_HEAD_OCC 3          // waves per SIMD of the fused head's quantising backward (z16 input)
#endif
// Q6_DIAG_STAMPS (diagnostic build): wave 0 of each workgroup of the q6 passes records s_memtime
// at its phase boundaries (per sub-tile: start, after the dz phase's barrier, after the record
// stores + barrier, after the quantisation + barrier) into g_q6_stamps, a device buffer no output
// reads; bnn_q6_stamps_copy hands them to the host (tools/q6_stamps.py).
#if defined(Q6_DIAG_STAMPS)
constexpr int Q6_ST_WG = 4096, Q6_ST_PH = 4, Q6_ST_SUB = 8;
__device__ unsigned long long g_q6_stamps[2][Q6_ST_WG][Q6_ST_SUB][Q6_ST_PH];
#define Q6_STAMP(sub, ph)                                                                                   \
  do {                                                                                                     \
    const unsigned wgid = blockIdx.y * gridDim.x + blockIdx.x;                                             \
    if (threadIdx.x == 0 && wgid < Q6_ST_WG && (sub) < Q6_ST_SUB)                                          \
      g_q6_stamps[NOUT > 0 ? 1 : 0][wgid][sub][ph] = __builtin_amdgcn_s_memtime();                         \
  } while (0)
#else
#define Q6_STAMP(sub, ph) do { } while (0)
#endif
#if defined(Q6_DIAG_NOQUANT)
constexpr bool Q6_DIAG_NOQUANT_ON = true;
#else
constexpr bool Q6_DIAG_NOQUANT_ON = false;
#endif

// Rows per workgroup of the fused apply: 512 (the parameter table is filled once per workgroup),
// or 64 when that leaves fewer than 1024 workgroups
// (small batches); never fewer rows than a statistics chunk (the column-sum partials reuse the
// statistics workspace, one row per workgroup row).
inline int64_t q6_rows(int64_t M, int64_t C) {
  if ((C / Q6T_COLS) * ((M + Q6T_ROWS - 1) / Q6T_ROWS) >= 1024) return Q6T_ROWS;
  return bn_chunk_rows(M, C) <= Q6T_SUB ? Q6T_SUB : Q6T_ROWS;
}

// The fused head's upstream gradient for 4 columns: g[j] = sum_q dY4[q] * W4[q][c + j] (fp32, q in
// order -- the same rounding in the statistics pass and the apply pass).
// Column pairs on the packed FMA (v_pk_fma_f32: two lanes' fmaf per instruction, the same
// per-element rounding and order as the scalar chain).
typedef float pf2 __attribute__((ext_vector_type(2)));

template <int NOUT>
__device__ __forceinline__ void head_grad4(const float* __restrict__ d4, const float (&wc)[NOUT > 0 ? NOUT : 1][4],
                                           float (&g)[4]) {
  float dq[NOUT];
#pragma unroll
  for (int q = 0; q < NOUT; ++q) dq[q] = d4[q];
#pragma unroll
  for (int jp = 0; jp < 2; ++jp) {
    pf2 s = {0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NOUT; ++q)
      s = __builtin_elementwise_fma(pf2{dq[q], dq[q]}, pf2{wc[q][2 * jp], wc[q][2 * jp + 1]}, s);
    g[2 * jp] = s.x;
    g[2 * jp + 1] = s.y;
  }
}

struct Q6Out {
  float* dx;                       // [M][C] or null
  uint8_t *rlo, *rhi, *rsc;        // rows of dz: [M][C/32][64], [M][C/32][32], [C/64][rsc_rows][2]
  int64_t rsc_rows;
  uint8_t *clo, *chi, *csc;        // dz^T: [C][Mp/32][64], [C][Mp/32][32], [Mp/64][csc_rows][2]
  int64_t csc_rows, nblk_m;        // nblk_m = Mp / 32
  double* part;                    // [workgroup rows of the grid][C] partial column sums, or null
  uint8_t* rres = nullptr;         // the rows' residual FP4 plane [M][C/32][16] (bnn_fp6.h), or null
};

// One sub-tile's digit records staged in LDS: rows (64 rows x 2 blocks of 32 columns) and columns
// (64 columns x 2 blocks of 32 rows), each as its global layout slice -- 128 B lo / 64 B hi per row
// or column (the 16-B chunk q of row i at chunk q ^ (i & 7) (lo) or q ^ (i & 3) (hi): the quantising
// lanes' 16-B writes, 128 B apart, spread over the banks) -- and the scale bytes.
struct Q6Stage {
  uint8_t rlo[64][128], clo[64][128];
  uint8_t rhi[64][64], chi[64][64];
  uint8_t rres[64][32];            // the rows' residual planes: block b of row i at chunk b ^ ((i >> 3) & 1)
  uint8_t rsc[64][2], csc[64][2];
};

// q6_block_pre's sink for block b of row (column) i: plane j's lo 16 B -> chunk 4b + j, hi 8 B ->
// half of chunk 2b + j / 2
struct Q6StageSink {
  uint8_t* lo;
  uint8_t* hi;
  uint8_t* sc;
  int i, b;
  __device__ __forceinline__ void plane(int j, uint4 l, uint2 h) {
    *reinterpret_cast<uint4*>(lo + 16 * ((4 * b + j) ^ (i & 7))) = l;
    *reinterpret_cast<uint2*>(hi + 16 * ((2 * b + (j >> 1)) ^ (i & 3)) + 8 * (j & 1)) = h;
  }
  __device__ __forceinline__ void scale(uint8_t v) { *sc = v; }
  __device__ __forceinline__ void residual(uint4 r) {   // rows only: res = st.rres[i]
    *reinterpret_cast<uint4*>(res + 16 * (b ^ ((i >> 3) & 1))) = r;
  }
  uint8_t* res = nullptr;
};

// The staged records of the sub-tile at rows m0.., columns c0.. to HBM, 16 B per thread and store:
// row lo 64 x 128 B, row hi 64 x 64 B, column lo / hi likewise, the two 128-B scale runs.  Rows at
// or beyond M are not stored (their scale bytes are: 0, inside the slab's padding, as it was
// initialised).
__device__ __forceinline__ void q6_stage_store(const Q6Stage& st, const Q6Out& o, int t, int64_t m0, int64_t M,
                                               int64_t c0, int64_t nblk_c) {
  // the per-lane store addresses are formed here, per call, from an opaque copy of the thread index:
  // hoisted out of the sub-tile loop they are ~10 live 64-bit registers, which the head variant
  // spilled -- and a spill reload waits (vmcnt) behind the next sub-tile's prefetched loads
#ifndef Q6_STORE_HOIST   // A/B build knob: let the compiler hoist them
  asm volatile("" : "+v"(t));
#endif
  const int64_t blk0 = c0 / QB, mblk0 = m0 / QB;
#pragma unroll
  for (int it = 0; it < 2; ++it) {            // lo: 512 chunks each
    const int ch = t + 256 * it, i = ch >> 3, q = ch & 7;
    const uint4 rv = *reinterpret_cast<const uint4*>(&st.rlo[i][16 * (q ^ (i & 7))]);
    const uint4 cv = *reinterpret_cast<const uint4*>(&st.clo[i][16 * (q ^ (i & 7))]);
    if (m0 + i < M) *reinterpret_cast<uint4*>(o.rlo + ((m0 + i) * nblk_c + blk0) * 64 + 16 * q) = rv;
    *reinterpret_cast<uint4*>(o.clo + ((c0 + i) * o.nblk_m + mblk0) * 64 + 16 * q) = cv;
  }
  {                                           // hi: 256 chunks each
    const int i = t >> 2, q = t & 3;
    const uint4 rv = *reinterpret_cast<const uint4*>(&st.rhi[i][16 * (q ^ (i & 3))]);
    const uint4 cv = *reinterpret_cast<const uint4*>(&st.chi[i][16 * (q ^ (i & 3))]);
    if (m0 + i < M) *reinterpret_cast<uint4*>(o.rhi + ((m0 + i) * nblk_c + blk0) * 32 + 16 * q) = rv;
    *reinterpret_cast<uint4*>(o.chi + ((c0 + i) * o.nblk_m + mblk0) * 32 + 16 * q) = cv;
  }
  if (o.rres != nullptr && t < 128) {         // row residual planes: 32 B per row (blocks blk0, blk0+1)
    const int i = t >> 1, q = t & 1;
    const uint4 rv = *reinterpret_cast<const uint4*>(&st.rres[i][16 * (q ^ ((i >> 3) & 1))]);
    if (m0 + i < M) *reinterpret_cast<uint4*>(o.rres + ((m0 + i) * nblk_c + blk0) * 16 + 16 * q) = rv;
  }
  if (t < 8) {                                // row scales: rows m0 .. m0+63, blocks blk0, blk0+1
    *reinterpret_cast<uint4*>(o.rsc + (blk0 >> 1) * o.rsc_rows * 2 + m0 * 2 + 16 * t) =
        *reinterpret_cast<const uint4*>(&st.rsc[8 * t][0]);
  } else if (t < 16) {                        // column scales: columns c0 .. c0+63, blocks mblk0, +1
    *reinterpret_cast<uint4*>(o.csc + (mblk0 >> 1) * o.csc_rows * 2 + c0 * 2 + 16 * (t - 8)) =
        *reinterpret_cast<const uint4*>(&st.csc[8 * (t - 8)][0]);
  }
}

// NOUT > 0 (the fused head, bnn_bn_head_bwd_q6): dy is the head's output gradient dY4 [M][NOUT]
// and the gradient reaching the BatchNorm is dY4 . W4, formed per element (W4 [NOUT][C]).
template <int NOUT, bool Z16 = false, bool KB = false>
__global__ __launch_bounds__(256, (NOUT > 0 && !Z16) ? 2 : (NOUT > 0 ? Q6_HEAD_OCC : 3)) void bn_bwd_apply_q6_k(XIn xin, const float* __restrict__ dy,
                                                         int64_t M, int64_t C, const float* __restrict__ mean,
                                                         const float* __restrict__ mean_lo,
                                                         const float* __restrict__ invstd,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, int hardtanh,
                                                         const float* __restrict__ sg,
                                                         const float* __restrict__ sgx, float inv_n, Q6Out o,
                                                         Drop dp0, const float* __restrict__ w4, int rows_wg) {
  const Drop dp = drop_resolve(dp0);
  __shared__ __attribute__((aligned(16))) float tile[Q6T_SUB * Q6T_LD];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t c0 = (int64_t)blockIdx.x * Q6T_COLS;
  const int64_t mbase = (int64_t)blockIdx.y * rows_wg;
  const int64_t nblk_c = C / QB;
  // elementwise mapping: float4 f = t + 256 i of a 64 x 64 sub-tile: row f / 16, columns 4 (f % 16)
  const int cq = 4 * (t & 15);
  const int64_t c = c0 + cq;
  // the 16 column groups' BatchNorm parameters (and the head's W4 columns) live in LDS and are read
  // into registers for each sub-tile's dz phase only: dead during the quantisation phase, whose
  // conversion-unit digits need the registers -- every variant fits 3 waves per SIMD unspilled
  constexpr int NP = 7 + (NOUT > 0 ? NOUT : 0);
  __shared__ float4 prm[NP][16];
  if (t < 16) {
    const int64_t cg = c0 + 4 * t;
    const float4 s0 = ld4(sg + cg), s1 = ld4(sgx + cg);
    prm[0][t] = ld4(mean + cg);
    prm[1][t] = ld4(invstd + cg);
    prm[2][t] = ld4_or(mean_lo, cg, 0.f);
    prm[3][t] = ld4_or(gamma, cg, 1.f);
    prm[4][t] = ld4_or(beta, cg, 0.f);
    prm[5][t] = make_float4(s0.x * inv_n, s0.y * inv_n, s0.z * inv_n, s0.w * inv_n);
    prm[6][t] = make_float4(s1.x * inv_n, s1.y * inv_n, s1.z * inv_n, s1.w * inv_n);
    if constexpr (NOUT > 0) {
#pragma unroll
      for (int q = 0; q < NOUT; ++q) prm[7 + q][t] = ld4(w4 + q * C + cg);
    }
  }
  __syncthreads();
  const float4 xb = xin_bias4<Z16>(xin, c);
  double csum = 0.0;                      // waves 2-3: column lane, rows of block wave-2 of each sub-tile
  const int64_t mp = o.nblk_m * QB;
  // block maxima formed in the dz phase (|dz| bits, unsigned max: abs_bits / q6_block_pre) by LDS
  // atomics -- rmax[b][row] over the row's 32 columns of block b, cmax[b][col] over the column's 32
  // rows of block b -- so a quantising lane reads its block once; it zeroes its entry for the next
  // sub-tile.  (Shuffle reductions + plain stores instead measured no faster and pushed the head
  // variant into spills: ab/r03_q6_noatomics_bn2d_byrow.patch, tools/gpu_r03_q6b.sh; round 4's DPP
  // row-maximum trees + per-wave column partials: 1765 vs 1761 us, profiles/r04_ab_q6shfl_pixdiag.log.)  The
  // sub-tile's digit records are staged in LDS (Q6Stage) and written out as whole lines by all 256
  // threads.
  __shared__ uint32_t rmax[2][Q6T_SUB], cmax[2][Q6T_COLS];
  __shared__ __attribute__((aligned(16))) Q6Stage st;
  if (t < 2 * Q6T_SUB) rmax[t >> 6][t & 63] = 0u;
  else cmax[(t >> 6) - 2][t & 63] = 0u;
  constexpr int D4LD = NOUT > 0 ? (NOUT + 3) / 4 * 4 : 4;
  __shared__ __attribute__((aligned(16))) float d4s[NOUT > 0 ? Q6T_SUB * D4LD : 4];
  // software pipeline: sub-tile s+1's x (and dY) rows are loaded into registers before sub-tile s
  // is quantised, so their HBM latency hides behind the quantiser's VALU work
  constexpr int NI = Q6T_SUB / 16;
  // a thread's NI rows of a sub-tile: the head's 4 consecutive rows (half of one keep-bit word of the
  // forward's dropout mask), else rows 16 apart
  constexpr bool RC4 = NOUT > 0;
  static_assert(!KB || (RC4 && NI == 4), "keep bits: the head's row mapping (4 rows = half a word)");
  auto row_of = [&](int i) __attribute__((always_inline)) { return RC4 ? NI * (t >> 4) + i : (t >> 4) + 16 * i; };
  // prefetch depth: the bn2 form on z16 (int16 x + fp32 dY rows, 6 B per element in) loads two
  // sub-tiles ahead -- one quantise phase did not cover its loads' latency under the record-store
  // stream (phase stamps, profiles/r05_q6_stamps.log); the head form and the fp32-x form, at their
  // register limits (a second fp32 x set spills), one
#ifdef Q6_PREFETCH1
  constexpr int PD = 1;                         // timing-only A/B builds
#else
  constexpr int PD = (NOUT == 0 && Z16) ? 2 : 1;
#endif
  XRaw<Z16> xr[PD][NI];
  float4 gr[PD][NOUT > 0 ? 1 : NI];
  // this workgroup's rows end here: the prefetch past its last sub-tile loads nothing (it read the
  // next workgroup's rows -- 1/8 of the pass's input -- and threw them away)
  const int64_t mend = min(mp, mbase + (int64_t)rows_wg);
  // KB: the sub-tile's keep-bit words (8-row groups x 16 column groups), staged in LDS with dY4
  __shared__ uint32_t kbs[KB ? Q6T_SUB / 8 : 1][16];
  // the head's dY4 rows (and keep words) of the next sub-tile ride in registers with its x loads
  // (3 floats + 1 word per thread), written to LDS at the sub-tile's top: a load issued there had
  // the dz phase wait on its full HBM latency once per sub-tile
  constexpr int ND4 = NOUT > 0 ? (Q6T_SUB * D4LD + 255) / 256 : 1;
  float d4r[ND4];
  uint32_t kbr = 0u;
  auto load_sub = [&](int64_t m0n, auto slot_c) __attribute__((always_inline)) {
    constexpr int S = decltype(slot_c)::value;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int64_t r = m0n + row_of(i);
      if (m0n < mend && r < M) {
        xr[S][i] = xin_raw4<Z16>(xin, r * C + c);
        if constexpr (NOUT == 0) gr[S][i] = ld4(dy + r * C + c);
      }
    }
    if constexpr (NOUT > 0) {
#pragma unroll
      for (int u = 0; u < ND4; ++u) {
        const int i = t + 256 * u, rr = i / D4LD, q = i - rr * D4LD;
        d4r[u] = (m0n < mend && i < Q6T_SUB * D4LD && m0n + rr < M && q < NOUT) ? dy[(m0n + rr) * NOUT + q] : 0.f;
      }
      if constexpr (KB) {
        const int64_t r8 = m0n + 8 * (t >> 4);
        kbr = (m0n < mend && t < Q6T_SUB * 2 && r8 < M) ? dp.bits[keep_word(r8, c0 + 4 * (t & 15), C)] : 0u;
      }
    }
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, PD - 1>;
  load_sub(mbase, S0{});
  if constexpr (PD == 2) load_sub(mbase + Q6T_SUB, S1{});
  // the digit records of sub-tile s are stored one phase late -- after sub-tile s+1's dz phase, just
  // before its loads for s+2 are issued -- so they drain while s+1 is quantised: the vector-memory
  // counter retires in issue order, and loads issued behind a sub-tile's stores had to wait for those
  // stores first (the records stored at once cost 0.4-0.7 ms per wide-step pass: timing-only builds
  // without stores, profiles/r04_q6_diag.log)
  int64_t m_prev = -1;
  // one sub-tile; slot_c = its prefetch register set (compile-time: the loop runs PD sub-tiles per trip)
  auto sub_tile = [&](int sub, auto slot_c) __attribute__((always_inline)) {
    constexpr int S = decltype(slot_c)::value;
    const int64_t m0 = mbase + sub * Q6T_SUB;
    Q6_STAMP(sub, 0);
    if constexpr (NOUT > 0) {   // this sub-tile's dY4 rows, padded to float4 rows (prefetched)
#pragma unroll
      for (int u = 0; u < ND4; ++u)
        if (t + 256 * u < Q6T_SUB * D4LD) d4s[t + 256 * u] = d4r[u];
      if constexpr (KB) {
        if (t < Q6T_SUB * 2) kbs[t >> 4][t & 15] = kbr;
      }
      __syncthreads();
    }
    asm volatile("" ::: "memory");   // the table reads stay inside the loop
    const int pg = t & 15;
    const float4 mv = prm[0][pg], iv = prm[1][pg], lv = prm[2][pg], gav = prm[3][pg], bev = prm[4][pg];
    const float4 a0v = prm[5][pg], a1v = prm[6][pg];
    const float ms[4] = {mv.x, mv.y, mv.z, mv.w}, is[4] = {iv.x, iv.y, iv.z, iv.w};
    const float lo[4] = {lv.x, lv.y, lv.z, lv.w};
    const float ga[4] = {gav.x, gav.y, gav.z, gav.w}, be[4] = {bev.x, bev.y, bev.z, bev.w};
    const float a0[4] = {a0v.x, a0v.y, a0v.z, a0v.w}, a1[4] = {a1v.x, a1v.y, a1v.z, a1v.w};
    // KB: this thread's 4 rows are one half of a keep-bit word
    const uint32_t kb = KB ? kbs[(NI * (t >> 4)) >> 3][t & 15] >> (16 * ((t >> 4) & 1)) : 0u;
    // column-block maxima of this thread's 4 columns per 32-row block (CPR: pre-reduced in registers
    // and across the wave's lane groups, one atomic per column and wave; the head form, at its
    // register limit, keeps one atomic per element)
    constexpr bool CPR = NOUT == 0;
    uint32_t cmx[2][4] = {};
#pragma unroll
    for (int i = 0; i < Q6T_SUB / 16; ++i) {
      const int rr = row_of(i);
      const int64_t r = m0 + rr;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      float wc[NOUT > 0 ? NOUT : 1][4];     // the head's weight columns c..c+3, re-read per row (the
      if constexpr (NOUT > 0) {             // 40 registers would otherwise stay live: spills)
        asm volatile("" ::: "memory");
#pragma unroll
        for (int q = 0; q < NOUT; ++q) {
          const float4 f = prm[7 + q][pg];
          wc[q][0] = f.x, wc[q][1] = f.y, wc[q][2] = f.z, wc[q][3] = f.w;
        }
      }
      if (r < M) {
        const float4 xv = xin_cvt4<Z16>(xr[S][i], xb);
        float xs[4] = {xv.x, xv.y, xv.z, xv.w};
        float gs[4];
        if constexpr (NOUT > 0) {
          head_grad4<NOUT>(d4s + rr * D4LD, wc, gs);
        } else {
          const float4 gv = gr[S][i];
          gs[0] = gv.x, gs[1] = gv.y, gs[2] = gv.z, gs[3] = gv.w;
        }
        uint32_t km = 0u;
        if constexpr (KB) km = (kb >> (4 * i)) & 15u;
        else if (dp.on) km = drop_bits4(dp, (uint64_t)(r * C + c));
        drop4m(dp, km, xs);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          v[j] = bn_dz1(xs[j], gs[j], ms[j], lo[j], is[j], ga[j], be[j], a0[j], a1[j], hardtanh);
        drop4m(dp, km, v);
        if (o.dx) *reinterpret_cast<float4*>(o.dx + r * C + c) = make_float4(v[0], v[1], v[2], v[3]);
      }
      *reinterpret_cast<float4*>(tile + rr * Q6T_LD + cq) = make_float4(v[0], v[1], v[2], v[3]);
      const uint32_t a0b = abs_bits(v[0]), a1b = abs_bits(v[1]), a2b = abs_bits(v[2]), a3b = abs_bits(v[3]);
      // the row block's maximum over its 8 lanes (quad swaps, then the half-row mirror: DPP, no LDS
      // traffic) -- one lane writes it; the 8 lanes are the whole 32-column block, so no atomic
      uint32_t rm = max(max(a0b, a1b), max(a2b, a3b));
      rm = max(rm, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)rm, 0xB1, 0xF, 0xF, false));
      rm = max(rm, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)rm, 0x4E, 0xF, 0xF, false));
      rm = max(rm, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)rm, 0x141, 0xF, 0xF, false));
      if ((t & 7) == 0) rmax[(t & 15) >> 3][rr] = rm;
      if constexpr (CPR) {   // rows 16 apart: blocks i / 2
        const int cb = i >> 1;
        cmx[cb][0] = max(cmx[cb][0], a0b);
        cmx[cb][1] = max(cmx[cb][1], a1b);
        cmx[cb][2] = max(cmx[cb][2], a2b);
        cmx[cb][3] = max(cmx[cb][3], a3b);
      } else {
        atomicMax(&cmax[rr >> 5][cq], a0b);
        atomicMax(&cmax[rr >> 5][cq + 1], a1b);
        atomicMax(&cmax[rr >> 5][cq + 2], a2b);
        atomicMax(&cmax[rr >> 5][cq + 3], a3b);
      }
    }
    if constexpr (CPR) {
      // across the wave's 4 lane groups (the same columns, rows of the same blocks), then one atomic
      // per column, block and wave (the other waves merge into it)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uint32_t m = cmx[cb][j];
          m = max(m, (uint32_t)__shfl_xor((int)m, 16, 64));
          m = max(m, (uint32_t)__shfl_xor((int)m, 32, 64));
          if (lane < 16) atomicMax(&cmax[cb][cq + j], m);
        }
    }
    __syncthreads();
    Q6_STAMP(sub, 1);
    // whole-line stores of the PREVIOUS sub-tile: per row (column) its two adjacent blocks' records
    // are 128 (lo) + 64 (hi) contiguous bytes, its two scale bytes adjacent to the next row's
    if (m_prev >= 0) q6_stage_store(st, o, t, m_prev, M, c0, nblk_c);
    __syncthreads();                           // the staged records are read before they are rewritten
    Q6_STAMP(sub, 2);
    load_sub(m0 + PD * Q6T_SUB, slot_c);
    // this lane's block maximum (waves 0-1: row blocks, 2-3: column blocks), reset for the next sub-tile
    const int b = wave & 1;
    uint32_t* amp = wave < 2 ? &rmax[b][lane] : &cmax[b][lane];
    const uint32_t am = *amp;
    *amp = 0u;
    if (!Q6_DIAG_NOQUANT_ON) {
      if (wave < 2) {
        // row block (row m0 + lane, columns c0 + 32 b ..)
        Q6StageSink sink{st.rlo[lane], st.rhi[lane], &st.rsc[lane][b], lane, b, st.rres[lane]};
        double unused = 0.0;
        if (o.rres != nullptr)     // the dX operand's residual plane (block-uniform branch)
          q6_block_pre<1, false, Q6StageSink, true>(tile + lane * Q6T_LD + QB * b, am, sink, unused);
        else
          q6_block_pre<1, false>(tile + lane * Q6T_LD + QB * b, am, sink, unused);
      } else {
        // column block (column c0 + lane, rows m0 + 32 b ..): rows beyond M are zeros; its
        // elements are added to the column sum in row order while they are quantised
        Q6StageSink sink{st.clo[lane], st.chi[lane], &st.csc[lane][b], lane, b};
#ifdef Q6_DIAG_NOCSUM     // timing-only build: the column sums not formed
        q6_block_pre<Q6T_LD, false>(tile + QB * b * Q6T_LD + lane, am, sink, csum);
#else
        q6_block_pre<Q6T_LD, true>(tile + QB * b * Q6T_LD + lane, am, sink, csum);
#endif
      }
    }
    __syncthreads();
    Q6_STAMP(sub, 3);
    m_prev = m0;
  };
  for (int sub = 0; sub < rows_wg / Q6T_SUB; sub += PD) {
    if (mbase + sub * Q6T_SUB >= mp) break;     // block-uniform
    sub_tile(sub, S0{});
    if constexpr (PD == 2) {
      if (sub + 1 >= rows_wg / Q6T_SUB || mbase + (sub + 1) * Q6T_SUB >= mp) break;
      sub_tile(sub + 1, S1{});
    }
  }
  if (m_prev >= 0) q6_stage_store(st, o, t, m_prev, M, c0, nblk_c);
  if (o.part != nullptr) {
    // fixed-order fold of the two column waves' sums: deterministic
    __shared__ double cs[Q6T_COLS];
    if (wave == 3) cs[lane] = csum;
    __syncthreads();
    if (wave == 2) o.part[(int64_t)blockIdx.y * C + c0 + lane] = csum + cs[lane];
  }
}

// colsum[n] = sum_r part[r][n]: FF_COLS columns x FF_GROUPS chunk groups per workgroup, the
// groups folded in a fixed order (deterministic)
// ------------------------------------------------------------------ fused head: [drop ->] bn -> htanh -> Linear
// mnist-dist2.py:69-76: fc3 -> drop -> bn3 -> htanh3 -> fc4 (nn.Linear(C, 10)).  The fp32 hardtanh
// output h3 [M][C] is never written: the forward forms h3 tile by tile from z and multiplies it
// into the head on the f32 MFMA (v_mfma_f32_16x16x4_f32: exact f32 products, f32 accumulation,
// the numerics class of the reference's F.linear); the backward forms dh3 = dY4 . W4 per element
// inside the BatchNorm passes and accumulates dW4 = dY4^T . h3 there (h3 recomputed from z).
// Row pitches of the LDS images (floats).  W4's: = 2 mod 32, so the B-fragment reads -- lane (r, k)
// at row r = lane & 15, column k0 + (lane >> 4) -- fall on banks 2r + k, 32 distinct per 32-lane
// group (a pitch of 128 put W4's 10 rows on ONE bank: the head forward spent ~40 % of its time in
// LDS bank conflicts, profiles/r04_pmc_bn.txt).  h3's stays 132 (float4 stores; 2-way on reads).
constexpr int HD_ROWS = 64, HD_COLS = 128, HD_LD = HD_COLS + 4, HD_WLD = HD_COLS + 2;
// elementwise map of a 64 x 128 chunk: thread -> 4 columns 4 (t % 32), rows 8 (t / 32) + i (8
// consecutive rows: one keep-bit word per chunk)
constexpr int HD_CG = HD_COLS / 4, HD_RS = 256 / HD_CG, HD_NI = HD_ROWS / HD_RS;
static_assert(HD_NI == 8, "a thread's rows are one keep-bit word");

typedef float hf4 __attribute__((ext_vector_type(4)));

template <int NOUT, bool Z16 = false, bool KB = false>
#ifndef HFWD_OCC
#define HFWD_OCC 4             // waves per SIMD of the fused head's forward (z16 input)
#endif
__global__ __launch_bounds__(256, Z16 ? HFWD_OCC : 2) void bn_head_fwd_k(XIn xin, int64_t M, int64_t C,
                                                     const float* __restrict__ mean, const float* __restrict__ mean_lo,
                                                     const float* __restrict__ invstd, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, const float* __restrict__ w4,
                                                     const float* __restrict__ b4, float* __restrict__ y4, Drop dp0) {
  static_assert(NOUT <= 16, "one 16-column MFMA tile");
  __shared__ __attribute__((aligned(16))) float ht[HD_ROWS * HD_LD];
  // W4's NOUT real rows only (the MFMA's B columns NOUT..15 read as zero): with <= 128 registers
  // (4 waves per SIMD) the 1024 workgroups of a 65536-row batch are resident at once (4 per CU,
  // 38.4 KiB of LDS each) instead of running in two rounds at 3 per CU
  __shared__ float ws[NOUT * HD_WLD];
  const Drop dp = drop_resolve(dp0);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * HD_ROWS;
  const int cq = 4 * (t % HD_CG);
  hf4 acc = hf4{0.f, 0.f, 0.f, 0.f};
  // software pipeline: chunk c0 + 128's x rows are fetched into registers before chunk c0 is
  // normalised and multiplied (the pass is latency-bound otherwise); W4's columns and the BatchNorm
  // parameters of the chunk (L2-resident) are loaded at its top, ahead of the barrier
  XRaw<Z16> xn[HD_NI];
  const int64_t rt = r0 + HD_NI * (t / HD_CG);   // this thread's first row
  uint32_t kn = 0u;                               // its keep-bit word of the fetched chunk
  auto fetch_x = [&](int64_t c0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < HD_NI; ++i) {
      const int64_t r = rt + i;
      if (r < M) xn[i] = xin_raw4<Z16>(xin, r * C + c0 + cq);
    }
    if (KB && rt < M) kn = dp.bits[keep_word(rt, c0 + cq, C)];
  };
  fetch_x(0);
  for (int64_t c0 = 0; c0 < C; c0 += HD_COLS) {
    XRaw<Z16> xc[HD_NI];
#pragma unroll
    for (int i = 0; i < HD_NI; ++i) xc[i] = xn[i];
    const uint32_t kc = kn;
    if (c0 + HD_COLS < C) fetch_x(c0 + HD_COLS);
    const int64_t c = c0 + cq;
    const float4 xb = xin_bias4<Z16>(xin, c);
    float w4c[(NOUT * HD_COLS + 255) / 256];
#pragma unroll
    for (int u = 0; u < (NOUT * HD_COLS + 255) / 256; ++u) {
      const int i = t + 256 * u, q = i / HD_COLS, k = i - q * HD_COLS;
      w4c[u] = q < NOUT ? w4[q * C + c0 + k] : 0.f;
    }
    const float4 mv = ld4(mean + c), iv = ld4(invstd + c), lv = ld4_or(mean_lo, c, 0.f);
    const float4 gv = ld4_or(gamma, c, 1.f), bv = ld4_or(beta, c, 0.f);
    const float mu[4] = {mv.x, mv.y, mv.z, mv.w}, is[4] = {iv.x, iv.y, iv.z, iv.w};
    const float lo[4] = {lv.x, lv.y, lv.z, lv.w};
    const float ga[4] = {gv.x, gv.y, gv.z, gv.w}, be[4] = {bv.x, bv.y, bv.z, bv.w};
    __syncthreads();   // the previous chunk's fragment reads are done
#pragma unroll
    for (int i = 0; i < HD_NI; ++i) {
      const int rr = HD_NI * (t / HD_CG) + i;
      const int64_t r = r0 + rr;
      float h[4] = {0.f, 0.f, 0.f, 0.f};
      if (r < M) {
        const float4 xv = xin_cvt4<Z16>(xc[i], xb);
        float xs[4] = {xv.x, xv.y, xv.z, xv.w};
        if constexpr (KB) drop4m(dp, (kc >> (4 * i)) & 15u, xs);
        else drop4(dp, (uint64_t)(r * C + c), xs);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          h[j] = fminf(fmaxf(fmaf(((xs[j] - mu[j]) - lo[j]) * is[j], ga[j], be[j]), -1.f), 1.f);
      }
      *reinterpret_cast<float4*>(ht + rr * HD_LD + cq) = make_float4(h[0], h[1], h[2], h[3]);
    }
#pragma unroll
    for (int u = 0; u < (NOUT * HD_COLS + 255) / 256; ++u)
      if (t + 256 * u < NOUT * HD_COLS) {
        const int i = t + 256 * u, q = i / HD_COLS;
        ws[q * HD_WLD + (i - q * HD_COLS)] = w4c[u];
      }
    __syncthreads();
    // wave wv: rows 16 wv .. +15 of the tile; A = h3 rows, B = W4^T (16 x 16 of which NOUT real)
#pragma unroll
    for (int k0 = 0; k0 < HD_COLS; k0 += 4) {
      const float a = ht[(16 * wv + (lane & 15)) * HD_LD + k0 + (lane >> 4)];
      const float b = (lane & 15) < NOUT ? ws[(lane & 15) * HD_WLD + k0 + (lane >> 4)] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    }
  }
  const int col = lane & 15;
  if (col < NOUT) {
    const float bias = b4 ? b4[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t r = r0 + 16 * wv + 4 * (lane >> 4) + i;
      if (r < M) y4[r * NOUT + col] = acc[i] + bias;
    }
  }
}

// Statistics pass of the head's BatchNorm backward (bn_reduce_k MODE 1 with g = dY4 . W4 formed per
// element) plus the head's weight gradient partials dW4[q][c] over the chunk's rows (fp32 per chunk).
template <int NOUT, bool Z16 = false, bool KB = false>
__global__ __launch_bounds__(256, HRED_OCC) void bn_head_reduce_k(XIn xin, const float* __restrict__ d4,
                                                        const float* __restrict__ w4, int64_t M, int64_t C,
                                                        const float* __restrict__ mean, const float* __restrict__ mean_lo,
                                                        const float* __restrict__ invstd,
                                                        const float* __restrict__ gamma, const float* __restrict__ beta,
                                                        double* __restrict__ p0, double* __restrict__ p1,
                                                        float* __restrict__ pw, int64_t chunk_rows, Drop dp0) {
  const Drop dp = drop_resolve(dp0);
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t C4 = C / 4;
  const int64_t chunk = id / C4;
  const int64_t c = (id - chunk * C4) * 4;
  const int64_t r0 = chunk * chunk_rows;
  const int64_t r1 = (M < r0 + chunk_rows) ? M : r0 + chunk_rows;
  // C % 256 == 0 (host check): a wave's 64 column groups share one chunk, whose dY4 rows the wave
  // stages in its own LDS slice once (chunk_rows x NOUT floats) and then reads as broadcasts (per-row
  // scalar loads of dY4 left the loop waiting on the scalar cache: 677 -> 584 us on the wide step,
  // profiles/r04_ab_head_*)
  __shared__ float d4s[4][BN_ROWS * NOUT];
  float* myd4 = d4s[threadIdx.x >> 6];
  if (r0 < M)
    for (int64_t i = threadIdx.x & 63; i < (r1 - r0) * NOUT; i += 64) myd4[i] = d4[r0 * NOUT + i];
  __syncthreads();     // before any return: every wave of the workgroup reaches it
  if (r0 >= M) return;
  float mu[4], lo[4], is[4], ga[4], be[4];
  float wc[NOUT][4], aw[NOUT][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    mu[j] = mean[c + j];
    lo[j] = mean_lo ? mean_lo[c + j] : 0.f;
    is[j] = invstd[c + j];
    ga[j] = gamma ? gamma[c + j] : 1.f;
    be[j] = beta ? beta[c + j] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < NOUT; ++q)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      wc[q][j] = w4[q * C + c + j];
      aw[q][j] = 0.f;
    }
  double a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
  const float4 xbias = xin_bias4<Z16>(xin, c);
  for (int64_t r = r0; r < r1; r += 16) {
    float fa[4] = {0, 0, 0, 0}, fb[4] = {0, 0, 0, 0};
    const int64_t re = (r + 16 < r1) ? r + 16 : r1;
    constexpr int RB = 8;   // rows whose x loads are issued together (as bn_reduce_k; 4: slower)
    for (int64_t rb = r; rb < re; rb += RB) {
    float4 xv8[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) xv8[u] = xin_load4<Z16>(xin, (rb + u < re ? rb + u : re - 1) * C + c, xbias);
    // the forward's keep bits of these 8 rows (host: only with 8-row batches at multiples of 8)
    const uint32_t kw = KB ? dp.bits[keep_word(rb, c, C)] : 0u;
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int64_t rr = rb + u;
      if (rr >= re) break;
      const float4 xv = xv8[u];
      float xs[4] = {xv.x, xv.y, xv.z, xv.w};
      if constexpr (KB) drop4m(dp, (kw >> (4 * u)) & 15u, xs);
      else drop4(dp, (uint64_t)(rr * C + c), xs);
      float dq[NOUT];
#pragma unroll
      for (int q = 0; q < NOUT; ++q) dq[q] = myd4[(rr - r0) * NOUT + q];
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {   // column pairs: the q-sums on the packed FMA
        pf2 gs2 = {0.f, 0.f};
#pragma unroll
        for (int q = 0; q < NOUT; ++q)   // head_grad4's order
          gs2 = __builtin_elementwise_fma(pf2{dq[q], dq[q]}, pf2{wc[q][2 * jp], wc[q][2 * jp + 1]}, gs2);
        float hh[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int j = 2 * jp + e;
          const float xh = ((xs[j] - mu[j]) - lo[j]) * is[j];
          const float y = fmaf(xh, ga[j], be[j]);
          const bool in = y > -1.f && y < 1.f;
          const float g = in ? (e ? gs2.y : gs2.x) : 0.f;
          fa[j] += g;
          fb[j] = fmaf(g, xh, fb[j]);
          hh[e] = fminf(fmaxf(y, -1.f), 1.f);     // the forward's h3
        }
#pragma unroll
        for (int q = 0; q < NOUT; ++q) {
          const pf2 a2 = __builtin_elementwise_fma(pf2{dq[q], dq[q]}, pf2{hh[0], hh[1]},
                                                   pf2{aw[q][2 * jp], aw[q][2 * jp + 1]});
          aw[q][2 * jp] = a2.x;
          aw[q][2 * jp + 1] = a2.y;
        }
      }
    }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] += (double)fa[j];
      b[j] += (double)fb[j];
    }
  }
  const int64_t o = chunk * C + c;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    p0[o + j] = a[j];
    p1[o + j] = b[j];
  }
#pragma unroll
  for (int q = 0; q < NOUT; ++q)
    *reinterpret_cast<float4*>(pw + (chunk * NOUT + q) * C + c) = make_float4(aw[q][0], aw[q][1], aw[q][2], aw[q][3]);
}

// bn_head_reduce_k with 2 columns per thread instead of 4: half the per-thread weight columns,
// dW4 accumulators and BatchNorm parameters (~100 registers: 4 waves per SIMD where the 4-column
// form holds 2), 4-B row loads.  Every column's sums run over the same rows in the same order as
// bn_head_reduce_k's: bit-identical partials.
template <int NOUT, bool Z16 = false, bool KB = false>
__global__ __launch_bounds__(256, 4) void bn_head_reduce2_k(XIn xin, const float* __restrict__ d4,
                                                         const float* __restrict__ w4, int64_t M, int64_t C,
                                                         const float* __restrict__ mean, const float* __restrict__ mean_lo,
                                                         const float* __restrict__ invstd,
                                                         const float* __restrict__ gamma, const float* __restrict__ beta,
                                                         double* __restrict__ p0, double* __restrict__ p1,
                                                         float* __restrict__ pw, int64_t chunk_rows, Drop dp0) {
  const Drop dp = drop_resolve(dp0);
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t C2 = C / 2;
  const int64_t chunk = id / C2;
  const int64_t c = (id - chunk * C2) * 2;
  const int64_t r0 = chunk * chunk_rows;
  const int64_t r1 = (M < r0 + chunk_rows) ? M : r0 + chunk_rows;
  // C % 256 == 0 (host check): a wave's 64 column pairs share one chunk (its dY4 rows staged once)
  __shared__ float d4s[4][BN_ROWS * NOUT];
  float* myd4 = d4s[threadIdx.x >> 6];
  if (r0 < M)
    for (int64_t i = threadIdx.x & 63; i < (r1 - r0) * NOUT; i += 64) myd4[i] = d4[r0 * NOUT + i];
  __syncthreads();     // before any return: every wave of the workgroup reaches it
  if (r0 >= M) return;
  float mu[2], lo[2], is[2], ga[2], be[2], xb[2];
  float wc[NOUT][2], aw[NOUT][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    mu[j] = mean[c + j];
    lo[j] = mean_lo ? mean_lo[c + j] : 0.f;
    is[j] = invstd[c + j];
    ga[j] = gamma ? gamma[c + j] : 1.f;
    be[j] = beta ? beta[c + j] : 0.f;
    xb[j] = (Z16 && xin.bias != nullptr) ? xin.bias[c + j] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < NOUT; ++q)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      wc[q][j] = w4[q * C + c + j];
      aw[q][j] = 0.f;
    }
  double a[2] = {0, 0}, b[2] = {0, 0};
  const uint32_t ksh = (uint32_t)(c & 3);   // this pair's bits within a row's nibble
  for (int64_t r = r0; r < r1; r += 16) {
    float fa[2] = {0, 0}, fb[2] = {0, 0};
    const int64_t re = (r + 16 < r1) ? r + 16 : r1;
    constexpr int RB = 8;
    for (int64_t rb = r; rb < re; rb += RB) {
      uint32_t xr[Z16 ? RB : 2 * RB];
#pragma unroll
      for (int u = 0; u < RB; ++u) {
        const int64_t idx = (rb + u < re ? rb + u : re - 1) * C + c;
        if constexpr (Z16) {
          xr[u] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const int16_t*>(xin.p) + idx);
        } else {
          const float2 f = *reinterpret_cast<const float2*>(reinterpret_cast<const float*>(xin.p) + idx);
          xr[2 * u] = __float_as_uint(f.x);
          xr[2 * u + 1] = __float_as_uint(f.y);
        }
      }
      const uint32_t kw = KB ? dp.bits[keep_word(rb, c, C)] : 0u;
#pragma unroll
      for (int u = 0; u < RB; ++u) {
        const int64_t rr = rb + u;
        if (rr >= re) break;
        float xs[2];
        if constexpr (Z16) {
          xs[0] = (float)(int16_t)(xr[u] & 0xFFFFu) + xb[0];
          xs[1] = (float)(int16_t)(xr[u] >> 16) + xb[1];
        } else {
          xs[0] = __uint_as_float(xr[2 * u]);
          xs[1] = __uint_as_float(xr[2 * u + 1]);
        }
        if (dp.on) {
          uint32_t km;
          if constexpr (KB) {
            km = (kw >> (4 * u + ksh)) & 3u;
          } else {
            const uint32_t key = drop_key(dp.seed), h0 = (uint32_t)(rr * C + c) * 0x9E3779B1u;
            km = (uint32_t)(fmix32(h0 ^ key) < dp.thresh) | ((uint32_t)(fmix32((h0 + 0x9E3779B1u) ^ key) < dp.thresh) << 1);
          }
#pragma unroll
          for (int j = 0; j < 2; ++j) xs[j] = ((km >> j) & 1u) ? xs[j] * dp.scale : 0.f;
        }
        float dq[NOUT];
#pragma unroll
        for (int q = 0; q < NOUT; ++q) dq[q] = myd4[(rr - r0) * NOUT + q];
        pf2 gs2 = {0.f, 0.f};
#pragma unroll
        for (int q = 0; q < NOUT; ++q)   // head_grad4's order
          gs2 = __builtin_elementwise_fma(pf2{dq[q], dq[q]}, pf2{wc[q][0], wc[q][1]}, gs2);
        float hh[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const float xh = ((xs[e] - mu[e]) - lo[e]) * is[e];
          const float y = fmaf(xh, ga[e], be[e]);
          const bool in = y > -1.f && y < 1.f;
          const float g = in ? (e ? gs2.y : gs2.x) : 0.f;
          fa[e] += g;
          fb[e] = fmaf(g, xh, fb[e]);
          hh[e] = fminf(fmaxf(y, -1.f), 1.f);     // the forward's h3
        }
#pragma unroll
        for (int q = 0; q < NOUT; ++q) {
          const pf2 a2 = __builtin_elementwise_fma(pf2{dq[q], dq[q]}, pf2{hh[0], hh[1]}, pf2{aw[q][0], aw[q][1]});
          aw[q][0] = a2.x;
          aw[q][1] = a2.y;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      a[j] += (double)fa[j];
      b[j] += (double)fb[j];
    }
  }
  const int64_t o = chunk * C + c;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    p0[o + j] = a[j];
    p1[o + j] = b[j];
  }
#pragma unroll
  for (int q = 0; q < NOUT; ++q)
    *reinterpret_cast<float2*>(pw + (chunk * NOUT + q) * C + c) = make_float2(aw[q][0], aw[q][1]);
}

// dW4[q][c] = sum over chunks of the partials: FF_COLS elements x FF_GROUPS chunk groups per
// workgroup, groups folded in a fixed order (double, deterministic)
// HD_FF_COLS fp32 partials per chunk row = one 128-B line (FF_COLS = 16 read half lines); each
// element's sum order (chunks grp, grp + FF_GROUPS, ..., then the groups in order) is unchanged
constexpr int HD_FF_COLS = 32;
__global__ __launch_bounds__(HD_FF_COLS * FF_GROUPS) void head_dw_final_k(const float* __restrict__ pw, int64_t R,
                                                                          int64_t nq, int64_t C,
                                                                          float* __restrict__ dw4) {
  __shared__ double sa[FF_GROUPS][HD_FF_COLS];
  const int lc = threadIdx.x & (HD_FF_COLS - 1), grp = threadIdx.x / HD_FF_COLS;
  const int64_t e = (int64_t)blockIdx.x * HD_FF_COLS + lc, ne = nq * C;
  double s = 0.0;
  if (e < ne)
#pragma unroll 16
    for (int64_t r = grp; r < R; r += FF_GROUPS) s += (double)pw[r * ne + e];
  sa[grp][lc] = s;
  __syncthreads();
  if (grp != 0 || e >= ne) return;
  s = 0.0;
  for (int gI = 0; gI < FF_GROUPS; ++gI) s += sa[gI][lc];
  dw4[e] = (float)s;
}

__global__ __launch_bounds__(256) void q6_colsum_final_k(const double* __restrict__ part, int64_t R, int64_t N,
                                                         float* __restrict__ out) {
  __shared__ double sa[FF_GROUPS][FF_COLS];
  const int lc = threadIdx.x & (FF_COLS - 1), grp = threadIdx.x / FF_COLS;
  const int64_t n = (int64_t)blockIdx.x * FF_COLS + lc;
  double s = 0.0;
  if (n < N)
#pragma unroll 16
    for (int64_t r = grp; r < R; r += FF_GROUPS) s += part[r * N + n];
  sa[grp][lc] = s;
  __syncthreads();
  if (grp != 0 || n >= N) return;
  s = 0.0;
  for (int gI = 0; gI < FF_GROUPS; ++gI) s += sa[gI][lc];
  out[n] = (float)s;
}

inline int grid_for(int64_t n) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 16384));
}

bool bn_args_ok(const float* x, int64_t M, int64_t C) {
  return x && M > 0 && C > 0 && C % 4 == 0 && aligned16(x) && (C / 4) * bn_chunks(M, C) < (1LL << 31) &&
         (M + apply_rows(M, C) - 1) / apply_rows(M, C) <= 65535;
}

bool vec_ok(const float* p) { return p == nullptr || aligned16(p); }

// the int16 form (XIn z16): 8-B aligned values (4 per 8-B load), 16-B aligned bias or none
bool bn_args_ok16(const XIn& in, int64_t M, int64_t C) {
  return in.p && (reinterpret_cast<uintptr_t>(in.p) & 7) == 0 && vec_ok(in.bias) && M > 0 && C > 0 && C % 4 == 0 &&
         (C / 4) * bn_chunks(M, C) < (1LL << 31) && (M + apply_rows(M, C) - 1) / apply_rows(M, C) <= 65535;
}

// the s20 form (XIn XF 2): the int16 plane as above, the nibble plane 2-B aligned (4 per 2-B load)
bool bn_args_ok20(const XIn& in, int64_t M, int64_t C) {
  return bn_args_ok16(in, M, C) && in.hi && (reinterpret_cast<uintptr_t>(in.hi) & 1) == 0;
}

bool bn_args_okf(const XIn& in, int xf, int64_t M, int64_t C) {
  return xf == 2 ? bn_args_ok20(in, M, C)
                 : (xf == 1 ? bn_args_ok16(in, M, C) : bn_args_ok(reinterpret_cast<const float*>(in.p), M, C));
}


// ------------------------------------------------------------------ BatchNorm2d (+ Hardtanh, + MaxPool2d(2))
// NCHW [N][C][H][W] activations of the binarized CNN (conv -> BatchNorm2d -> Hardtanh -> MaxPool2d(2),
// the mnist-dist.py:31-51 template the build's BinCNN follows).  Per-channel statistics over N*H*W,
// same math and merge order as the 1d kernels above (chunk = CR images of one channel, one workgroup).
// pool = 2 fuses MaxPool2d(kernel 2, stride 2): forward writes only the pooled map; backward takes
// the pooled gradient and recomputes the window's argmax (torch's rule: first strictly greater
// value in (h, w) scan order, NaN wins), so neither the fp32 full-resolution output nor the
// max-pool indices are ever stored.

constexpr int BN2_T = 256;

inline int64_t bn2_chunk_images(int64_t N, int64_t C) {
  const int64_t R = std::max<int64_t>(1, std::min<int64_t>(N, (2048 + C - 1) / C));
  return (N + R - 1) / R;
}

__device__ __forceinline__ void block_sum2(double& a, double& b) {
  __shared__ double sa[BN2_T / 64], sb[BN2_T / 64];
  a = wave_sum(a);
  b = wave_sum(b);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sa[w] = a;
    sb[w] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ta = 0.0, tb = 0.0;
    for (int i = 0; i < BN2_T / 64; ++i) {   // fixed order: deterministic
      ta += sa[i];
      tb += sb[i];
    }
    a = ta;
    b = tb;
  }
}

// MODE 0: chunk (mean, M2) of x.  MODE 1: chunk (sum g, sum g*xhat), g = masked full-resolution
// gradient (POOL: routed to the window argmax from the pooled dy).
template <int MODE, int POOL, int XF = 0>
__global__ __launch_bounds__(BN2_T) void bn2d_reduce_k(X2 x, const float* __restrict__ dy,
                                                       int64_t N, int64_t C, int H, int W, int64_t CR,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ invstd,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, int hardtanh,
                                                       double* __restrict__ p0, double* __restrict__ p1) {
  const int64_t c = blockIdx.x, r = blockIdx.y;
  const int64_t n0 = r * CR, n1 = (n0 + CR < N) ? n0 + CR : N;
  const int64_t HW = (int64_t)H * W;
  const float xb = x2_bias<XF>(x, c);
  double a = 0.0, b = 0.0;
  float fa = 0.f, fb = 0.f;
  int cnt = 0;
  if (MODE == 0) {
    const float shift = x2_ld1<XF>(x, (n0 * C + c) * HW, xb);
    // thread -> (image lane li, 4-element group j): ipi images per sweep of the workgroup when a
    // plane has fewer than BN2_T groups, the index split paid once per thread (not per element)
    const int hw4 = (int)(HW / 4);
    const bool wide = hw4 >= BN2_T;
    const int ipi = wide ? 1 : BN2_T / hw4;
    const int li = wide ? 0 : (int)threadIdx.x / hw4;
    const int j0 = wide ? (int)threadIdx.x : (int)threadIdx.x - li * hw4;
    const int jstep = wide ? BN2_T : hw4;
    if (li < ipi) {
      for (int64_t n = n0 + li; n < n1; n += ipi) {
        const int64_t base = (n * C + c) * HW;
        for (int j = j0; j < hw4; j += jstep) {
          const float4 v = x2_ld4<XF, true>(x, base + 4 * j, xb);
          const float d[4] = {v.x - shift, v.y - shift, v.z - shift, v.w - shift};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            fa += d[q];
            fb = fmaf(d[q], d[q], fb);
          }
          if (++cnt == 8) {
            a += (double)fa;
            b += (double)fb;
            fa = fb = 0.f;
            cnt = 0;
          }
        }
      }
    }
    a += (double)fa;
    b += (double)fb;
    block_sum2(a, b);
    if (threadIdx.x == 0) {
      const double nb = (double)((n1 - n0) * HW), dm = a / nb;
      p0[r * C + c] = (double)shift * nb + a;   // chunk sum
      p1[r * C + c] = b - a * dm;
    }
    return;
  }
  const Bn2Chan k = bn2_chan(c, mean, invstd, gamma, beta);
  if (POOL) {
    const int PH = H / 2, PW = W / 2;
    const int64_t pp = (int64_t)PH * PW, total = (n1 - n0) * pp;
    for (int64_t i = threadIdx.x; i < total; i += BN2_T) {
      const int64_t n = n0 + i / pp, p = i - (i / pp) * pp;
      const int ph = (int)(p / PW), pw = (int)(p - (int64_t)ph * PW);
      const int64_t xo = (n * C + c) * HW + (int64_t)(2 * ph) * W + 2 * pw;
      const Win w = bn2_window(x2_ld2<XF>(x, xo, xb), x2_ld2<XF>(x, xo + W, xb), k, hardtanh);
      const float yv = w.y[w.arg];
      const float g = (!hardtanh || (yv > -1.f && yv < 1.f)) ? dy[(n * C + c) * pp + p] : 0.f;
      fa += g;
      fb = fmaf(g, w.xh[w.arg], fb);
      if (++cnt == 8) {
        a += (double)fa;
        b += (double)fb;
        fa = fb = 0.f;
        cnt = 0;
      }
    }
  } else {
    const int64_t hw4 = HW / 4, total = (n1 - n0) * hw4;
    for (int64_t i = threadIdx.x; i < total; i += BN2_T) {
      const int64_t n = n0 + i / hw4, j = i - (i / hw4) * hw4;
      const int64_t o = (n * C + c) * HW + 4 * j;
      const float4 xv = x2_ld4<XF>(x, o, xb), gv = ld4(dy + o);
      const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, gs[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float xh = (xs[q] - k.mu) * k.is;
        const float y = fmaf(xh, k.ga, k.be);
        const float g = (!hardtanh || (y > -1.f && y < 1.f)) ? gs[q] : 0.f;
        fa += g;
        fb = fmaf(g, xh, fb);
      }
      if (++cnt == 8) {
        a += (double)fa;
        b += (double)fb;
        fa = fb = 0.f;
        cnt = 0;
      }
    }
  }
  a += (double)fa;
  b += (double)fb;
  block_sum2(a, b);
  if (threadIdx.x == 0) {
    p0[r * C + c] = a;
    p1[r * C + c] = b;
  }
}

// Forward statistics (bn2d_reduce_k<0>'s chunk sum and M2 about the chunk's first element) with the
// chunk's (image, 4-element group) pairs flattened over the workgroup (no idle lanes when a plane
// has fewer than 256 groups: conv1's 196) and 4 groups' loads issued together; 32-bit index split.
template <int XF>
__global__ __launch_bounds__(BN2_T) void bn2d_fwd_stats_flat_k(X2 x, int64_t N, int64_t C, int HW, int64_t CR,
                                                               double* __restrict__ p0, double* __restrict__ p1) {
  constexpr int B = 4;
  const int64_t c = blockIdx.x, r = blockIdx.y;
  const int64_t n0 = r * CR, n1 = (n0 + CR < N) ? n0 + CR : N;
  const float xb = x2_bias<XF>(x, c);
  const float shift = x2_ld1<XF>(x, (n0 * C + c) * HW, xb);
  const int hw4 = HW / 4, total = (int)((n1 - n0) * hw4);
  double a = 0.0, b = 0.0;
  for (int i0 = threadIdx.x; i0 < total; i0 += B * BN2_T) {
    float4 v[B];
#pragma unroll
    for (int q = 0; q < B; ++q) {
      const int i = min(i0 + q * BN2_T, total - 1);   // clamped, unconditional: the loads batch
      const int im = i / hw4, gi = i - im * hw4;
      v[q] = x2_ld4<XF, true>(x, ((n0 + im) * C + c) * (int64_t)HW + 4 * gi, xb);
    }
    float fa = 0.f, fb = 0.f;
#pragma unroll
    for (int q = 0; q < B; ++q) {
      if (i0 + q * BN2_T >= total) break;
      const float d[4] = {v[q].x - shift, v[q].y - shift, v[q].z - shift, v[q].w - shift};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        fa += d[e];
        fb = fmaf(d[e], d[e], fb);
      }
    }
    a += (double)fa;
    b += (double)fb;
  }
  block_sum2(a, b);
  if (threadIdx.x == 0) {
    const double nb = (double)((n1 - n0) * HW), dm = a / nb;
    p0[r * C + c] = (double)shift * nb + a;   // chunk sum
    p1[r * C + c] = b - a * dm;
  }
}

// Backward statistics of a 2x2-pooled BatchNorm2d (bn2d_reduce_k<1, 2>'s sums) with thread =
// (image, pooled row): the PW windows' loads -- two x rows and one dy row -- are all issued before
// any is used (3 PW independent loads per thread; the window-per-trip loop waited on memory ~60 %
// of its cycles: profiles/r04_pmc_sq_cnn.txt).  Same per-window arithmetic; the fp32 partial of a
// row is folded into the double sums per row.
template <int PW, int XF>
__global__ __launch_bounds__(BN2_T) void bn2d_bwd_stats_rows_k(X2 x, const float* __restrict__ dy, int64_t N,
                                                               int64_t C, int H, int64_t CR,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ invstd,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, int hardtanh,
                                                               double* __restrict__ p0, double* __restrict__ p1) {
  constexpr int W = 2 * PW;
  const int64_t c = blockIdx.x, r = blockIdx.y;
  const int64_t n0 = r * CR, n1 = (n0 + CR < N) ? n0 + CR : N;
  const int PH = H / 2;
  const int64_t HW = (int64_t)H * W, pp = (int64_t)PH * PW;
  const float xb = x2_bias<XF>(x, c);
  const Bn2Chan k = bn2_chan(c, mean, invstd, gamma, beta);
  double a = 0.0, b = 0.0;
  const int64_t pairs = (n1 - n0) * PH;
  // XF = 2: each trip's 256 row pairs staged through LDS by address-ordered loads (Rows16)
  __shared__ uint2 lds[XF == 2 ? 256 * Rows16<PW>::LD : 1];
  const float inv_ph = 1.f / (float)PH;
  for (int64_t i0 = 0; i0 < pairs; i0 += BN2_T) {   // uniform trips: every thread reaches the barriers
    const int64_t i = i0 + threadIdx.x;
    const int64_t q0 = i / PH;
    const int ph = (int)(i - q0 * PH);
    const int64_t plane = (n0 + q0) * C + c;
    const int64_t xo = plane * HW + (int64_t)(2 * ph) * W, yo = plane * pp + (int64_t)ph * PW;
    float2 top[PW], bot[PW];
    if constexpr (XF == 2) {
      if (i0 > 0) __syncthreads();                     // the previous trip's LDS reads are done
      const int np = (int)((pairs - i0) < BN2_T ? (pairs - i0) : BN2_T);
      rows16_stage<PW>(x, np, [&](int pr) {
        // pair qq of the chunk -> (image qq / PH, pooled row); 32-bit quotient by a float
        // reciprocal, corrected (pairs < 2^22: off by at most one)
        const int qq = (int)i0 + pr;
        int qq0 = (int)((float)qq * inv_ph);
        qq0 += (qq0 + 1) * PH <= qq;
        qq0 -= qq0 * PH > qq;
        return 2 * (((n0 + qq0) * C + c) * HW + (int64_t)(qq - qq0 * PH) * (2 * W));
      }, lds);
      __syncthreads();
      if (i >= pairs) continue;
      rows16_unpack<PW>(lds, (int)threadIdx.x, xb, top, bot);
    } else {
      if (i >= pairs) continue;
      x2_rows<XF, PW>(x, xo, xb, top, bot);
    }
    float g[PW];
#pragma unroll
    for (int q = 0; q < PW; ++q) g[q] = dy[yo + q];
    float fa = 0.f, fb = 0.f;
#pragma unroll
    for (int q = 0; q < PW; ++q) {
      const Win w = bn2_window(top[q], bot[q], k, hardtanh);
      float yv = w.y[0], xa = w.xh[0];   // w.y[w.arg], w.xh[w.arg] as selects (no indexed private array)
#pragma unroll
      for (int j = 1; j < 4; ++j) {
        yv = w.arg == j ? w.y[j] : yv;
        xa = w.arg == j ? w.xh[j] : xa;
      }
      const float gg = (!hardtanh || (yv > -1.f && yv < 1.f)) ? g[q] : 0.f;
      fa += gg;
      fb = fmaf(gg, xa, fb);
    }
    a += (double)fa;
    b += (double)fb;
  }
  block_sum2(a, b);
  if (threadIdx.x == 0) {
    p0[r * C + c] = a;
    p1[r * C + c] = b;
  }
}

// The pooled forward / backward apply passes with thread = (plane, pooled row): one index split per
// row of PW windows (the window-per-thread forms split a 64-bit flat index three times per window)
// and all of a row's loads issued before use.  Per-window arithmetic identical to bn2d_apply_k /
// bn2d_bwd_apply_k<2> (bit-identical outputs).
template <int PW, int XF>
__global__ __launch_bounds__(256) void bn2d_apply_rows_k(X2 x, int64_t N, int64_t C, int H,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ invstd,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, int hardtanh,
                                                         float* __restrict__ y) {
  constexpr int W = 2 * PW;
  const int PH = H / 2;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float2 top[PW], bot[PW];
  // XF = 2: the workgroup's 256 row pairs are one contiguous 4 W * 256-byte run, staged through LDS
  // by address-ordered loads (Rows16) before any thread leaves
  __shared__ uint2 lds[XF == 2 ? 256 * Rows16<PW>::LD : 1];
  if constexpr (XF == 2) {
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x, total = N * C * PH;
    const int np = (int)((total - i0) < 256 ? (total - i0) : 256);
    rows16_stage<PW>(x, np, [&](int pr) { return (i0 + pr) * (int64_t)(4 * W); }, lds);
    __syncthreads();
  }
  if (i >= N * C * PH) return;
  const int64_t plane = i / PH;
  const int ph = (int)(i - plane * PH);
  const int64_t c = plane % C;
  const Bn2Chan k = bn2_chan(c, mean, invstd, gamma, beta);
  const float xb = x2_bias<XF>(x, c);
  const int64_t xo = plane * ((int64_t)H * W) + (int64_t)(2 * ph) * W;
  if constexpr (XF == 2)
    rows16_unpack<PW>(lds, (int)threadIdx.x, xb, top, bot);
  else
    x2_rows<XF, PW>(x, xo, xb, top, bot);
  float* yr = y + plane * ((int64_t)PH * PW) + (int64_t)ph * PW;
#pragma unroll
  for (int q = 0; q < PW; ++q) yr[q] = bn2_window(top[q], bot[q], k, hardtanh).out;
}

template <int PW, int XF>
__global__ __launch_bounds__(256) void bn2d_bwd_apply_rows_k(X2 x, const float* __restrict__ dy, int64_t N,
                                                             int64_t C, int H, const float* __restrict__ mean,
                                                             const float* __restrict__ invstd,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, int hardtanh,
                                                             const float* __restrict__ sg,
                                                             const float* __restrict__ sgx, float inv_n,
                                                             float* __restrict__ dx) {
  constexpr int W = 2 * PW;
  const int PH = H / 2;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * C * PH) return;
  const int64_t plane = i / PH;
  const int ph = (int)(i - plane * PH);
  const int64_t c = plane % C;
  const Bn2Chan k = bn2_chan(c, mean, invstd, gamma, beta);
  const float m0 = sg[c] * inv_n, m1 = sgx[c] * inv_n, sc = k.ga * k.is;
  const float xb = x2_bias<XF>(x, c);
  const int64_t xo = plane * ((int64_t)H * W) + (int64_t)(2 * ph) * W;
  const float* dr = dy + plane * ((int64_t)PH * PW) + (int64_t)ph * PW;
  float2 top[PW], bot[PW];
  float gp[PW];
  x2_rows<XF, PW>(x, xo, xb, top, bot);
#pragma unroll
  for (int q = 0; q < PW; ++q) gp[q] = dr[q];
#pragma unroll
  for (int q = 0; q < PW; ++q) {
    const Win w = bn2_window(top[q], bot[q], k, hardtanh);
    float o[4];
    bn2_window_dz(w, gp[q], m0, m1, sc, hardtanh, o);
    *reinterpret_cast<float2*>(dx + xo + 2 * q) = make_float2(o[0], o[1]);
    *reinterpret_cast<float2*>(dx + xo + W + 2 * q) = make_float2(o[2], o[3]);
  }
}

// Forward apply: y = clamp((x-mean)*invstd*gamma+beta) (POOL: max over each 2x2 window).
template <int POOL, int XF = 0>
__global__ __launch_bounds__(256) void bn2d_apply_k(X2 x, int64_t N, int64_t C, int H, int W,
                                                    const float* __restrict__ mean,
                                                    const float* __restrict__ invstd,
                                                    const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, int hardtanh,
                                                    float* __restrict__ y) {
  const int64_t HW = (int64_t)H * W;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (POOL) {
    const int PH = H / 2, PW = W / 2;
    const int64_t pp = (int64_t)PH * PW, total = N * C * pp;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
      const int64_t plane = i / pp, p = i - plane * pp;
      const int ph = (int)(p / PW), pw = (int)(p - (int64_t)ph * PW);
      const int64_t c = plane % C;
      const Bn2Chan k = bn2_chan(c, mean, invstd, gamma, beta);
      const float xb = x2_bias<XF>(x, c);
      const int64_t xo = plane * HW + (int64_t)(2 * ph) * W + 2 * pw;
      y[i] = bn2_window(x2_ld2<XF, true>(x, xo, xb), x2_ld2<XF, true>(x, xo + W, xb), k, hardtanh).out;
    }
    return;
  }
  const int64_t n4 = N * C * HW / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const int64_t c = ((4 * i) / HW) % C;
    const Bn2Chan k = bn2_chan(c, mean, invstd, gamma, beta);
    const float4 xv = x2_ld4<XF, true>(x, 4 * i, x2_bias<XF>(x, c));
    float v[4] = {fmaf((xv.x - k.mu) * k.is, k.ga, k.be), fmaf((xv.y - k.mu) * k.is, k.ga, k.be),
                  fmaf((xv.z - k.mu) * k.is, k.ga, k.be), fmaf((xv.w - k.mu) * k.is, k.ga, k.be)};
    if (hardtanh) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = fminf(fmaxf(v[j], -1.f), 1.f);
    }
    *reinterpret_cast<float4*>(y + 4 * i) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// Backward apply: dx = gamma*invstd*(g - sum_g/n - xhat*sum_gxhat/n), g routed/masked as in reduce.
template <int POOL, int XF = 0>
__global__ __launch_bounds__(256) void bn2d_bwd_apply_k(X2 x, const float* __restrict__ dy,
                                                        int64_t N, int64_t C, int H, int W,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ invstd,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, int hardtanh,
                                                        const float* __restrict__ sg,
                                                        const float* __restrict__ sgx, float inv_n,
                                                        float* __restrict__ dx) {
  // inv_n = 1/(N*H*W) with batch statistics; 0 in eval mode (running statistics: dx = gamma*invstd*g)
  const int64_t HW = (int64_t)H * W;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (POOL) {
    const int PH = H / 2, PW = W / 2;
    const int64_t pp = (int64_t)PH * PW, total = N * C * pp;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
      const int64_t plane = i / pp, p = i - plane * pp, c = plane % C;
      const int ph = (int)(p / PW), pw = (int)(p - (int64_t)ph * PW);
      const Bn2Chan k = bn2_chan(c, mean, invstd, gamma, beta);
      const float m0 = sg[c] * inv_n, m1 = sgx[c] * inv_n, sc = k.ga * k.is;
      const int64_t off = plane * HW + (int64_t)(2 * ph) * W + 2 * pw;
      const float xb = x2_bias<XF>(x, c);
      const Win w = bn2_window(x2_ld2<XF>(x, off, xb), x2_ld2<XF>(x, off + W, xb), k, hardtanh);
      float o[4];
      bn2_window_dz(w, dy[i], m0, m1, sc, hardtanh, o);
      *reinterpret_cast<float2*>(dx + off) = make_float2(o[0], o[1]);
      *reinterpret_cast<float2*>(dx + off + W) = make_float2(o[2], o[3]);
    }
    return;
  }
  const int64_t n4 = N * C * HW / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const int64_t c = ((4 * i) / HW) % C;
    const Bn2Chan k = bn2_chan(c, mean, invstd, gamma, beta);
    const float m0 = sg[c] * inv_n, m1 = sgx[c] * inv_n, sc = k.ga * k.is;
    const float4 xv = x2_ld4<XF>(x, 4 * i, x2_bias<XF>(x, c)), gv = ld4(dy + 4 * i);
    const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, gs[4] = {gv.x, gv.y, gv.z, gv.w};
    float o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float xh = (xs[j] - k.mu) * k.is;
      const float yv = fmaf(xh, k.ga, k.be);
      const float g = (!hardtanh || (yv > -1.f && yv < 1.f)) ? gs[j] : 0.f;
      o[j] = sc * (g - m0 - xh * m1);
    }
    *reinterpret_cast<float4*>(dx + 4 * i) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

bool bn2_args_ok(const float* x, int64_t N, int64_t C, int64_t H, int64_t W, int pool) {
  if (!x || N <= 0 || C <= 0 || H <= 0 || W <= 0 || !aligned16(x) || C > 65535) return false;
  if ((H * W) % 4 != 0) return false;
  if (pool != 0 && (pool != 2 || H % 2 != 0 || W % 2 != 0)) return false;
  return (N + bn2_chunk_images(N, C) - 1) / bn2_chunk_images(N, C) <= 65535;
}

}  // namespace
}  // namespace bnn

using namespace bnn;

namespace {
// The dropout keep-bit plane (Drop::bits, keep_word): the forward statistics pass writes it where
// its thread's 8-row load batches are whole words (chunks of a multiple of 8 rows), else
// keep_bits_k does; the statistics pass of the head backward reads it on the same condition.
inline bool keep_bits_fused(int64_t M, int64_t C) { return RED_RB == 8 && bn_chunk_rows(M, C) % 8 == 0; }

__global__ __launch_bounds__(256) void keep_bits_k(int64_t M, int64_t C, Drop d0, uint32_t* __restrict__ out) {
  const Drop d = drop_resolve(d0);
  const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x, C4 = C / 4;
  if (w >= keep_words(M, C)) return;
  const int64_t r0 = (w / C4) * 8, c = (w % C4) * 4;
  uint32_t kw = 0;
  for (int i = 0; i < 8 && r0 + i < M; ++i) kw |= drop_bits4(d, (uint64_t)((r0 + i) * C + c)) << (4 * i);
  out[w] = kw;
}
}  // namespace

BNN_API int64_t bnn_dropout_keep_bits_bytes(int64_t M, int64_t C) {
  return (M > 0 && C > 0 && C % 4 == 0) ? keep_words(M, C) * (int64_t)sizeof(uint32_t) : -1;
}

BNN_API int64_t bnn_bn_workspace(int64_t M, int64_t C) {
  // two double partial arrays [R][C] + two float vectors [C]
  return 2 * bn_chunks(M, C) * C * (int64_t)sizeof(double) + 2 * round_up(C * 4, 256);
}

static int bn_fwd_train_impl(XIn xin, bool z16, int64_t M, int64_t C, const float* gamma, const float* beta,
                             float* running_mean, float* running_var, float momentum, float eps,
                             float* save_mean, float* save_invstd, float* save_mean_lo, float* y,
                             int32_t hardtanh, void* work, void* stream, Drop dp, uint32_t* keep_bits = nullptr) {
  const float* x = reinterpret_cast<const float*>(xin.p);
  if (!(z16 ? bn_args_ok16(xin, M, C) : bn_args_ok(x, M, C)) || !save_mean || !save_invstd || !work || !vec_ok(y) ||
      !vec_ok(save_mean_lo) || (running_mean == nullptr) != (running_var == nullptr) || !vec_ok(gamma) ||
      !vec_ok(beta) || !aligned16(save_mean) || !aligned16(save_invstd) || (z16 && y != nullptr)) {
    set_error("bnn_bn_fwd_train: bad arguments (M=%lld C=%lld; C must be a multiple of 4, M > 0)",
              (long long)M, (long long)C);
    return kErrInval;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t R = bn_chunks(M, C);
  double* p0 = reinterpret_cast<double*>(work);
  double* p1 = p0 + R * C;
  // without a caller buffer the lo part of the mean lives in the workspace (the bwd's k0 slot)
  float* lo = save_mean_lo ? save_mean_lo : reinterpret_cast<float*>(p1 + R * C);
  // the keep-bit plane: written by the statistics pass where its row batches are whole words, else
  // by its own kernel
  Drop dps = dp;
  if (keep_bits != nullptr && dp.on) {
    if (keep_bits_fused(M, C)) dps.bits_out = keep_bits;
    else hipLaunchKernelGGL(keep_bits_k, dim3((unsigned)((keep_words(M, C) + 255) / 256)), dim3(256), 0, s, M, C, dp,
                            keep_bits);
  }
  if (z16)
    hipLaunchKernelGGL((bn_reduce_k<0, 1>), reduce_grid(M, C), dim3(256), 0, s, xin,
                       nullptr, M, C, nullptr, nullptr, nullptr, nullptr, nullptr, 0, p0, p1, bn_chunk_rows(M, C), dps);
  else
    hipLaunchKernelGGL((bn_reduce_k<0, 0>), reduce_grid(M, C), dim3(256), 0, s, xin,
                       nullptr, M, C, nullptr, nullptr, nullptr, nullptr, nullptr, 0, p0, p1, bn_chunk_rows(M, C), dps);
  hipLaunchKernelGGL(bn_fwd_final_k, ffin_grid(C), dim3(256), 0, s, p0, p1, M, C, R, momentum, eps, running_mean,
                     running_var, save_mean, save_invstd, lo, bn_chunk_rows(M, C), (int64_t)1);
  if (y != nullptr)   // y == NULL: statistics only (the fused apply+pack path writes no fp32 y)
    hipLaunchKernelGGL(bn_apply_k, apply_grid(M, C), dim3(256), 0, s, x, M, C, save_mean, lo, save_invstd,
                       gamma, beta, hardtanh, y, dp);
  return check_launch("bnn_bn_fwd_train");
}

// The forward statistics from chunk partials another kernel formed (bnn_gemm_i8_affine_bnstats):
// part = [2][R][C] doubles (chunk sums, M2 about the chunk means), chunk r = rows
// [r*chunk_rows, min((r+1)*chunk_rows, M)); the same final as bnn_bn_fwd_train
BNN_API int bnn_bn_fwd_final_parts(const double* part, int64_t R, int64_t chunk_rows, int64_t M, int64_t C,
                                   float* running_mean, float* running_var, float momentum, float eps,
                                   float* save_mean, float* save_invstd, float* save_mean_lo, void* stream) {
  if (!part || M <= 0 || C <= 0 || chunk_rows <= 0 || R != (M + chunk_rows - 1) / chunk_rows || !save_mean ||
      !save_invstd || !save_mean_lo || (running_mean == nullptr) != (running_var == nullptr)) {
    set_error("bnn_bn_fwd_final_parts: bad arguments (R=%lld chunk_rows=%lld M=%lld C=%lld)", (long long)R,
              (long long)chunk_rows, (long long)M, (long long)C);
    return kErrInval;
  }
  hipLaunchKernelGGL(bn_fwd_final_k, ffin_grid(C), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), part,
                     part + R * C, M, C, R, momentum, eps, running_mean, running_var, save_mean, save_invstd,
                     save_mean_lo, chunk_rows, (int64_t)1);
  return check_launch("bnn_bn_fwd_final_parts");
}

BNN_API int bnn_bn_fwd_train(const float* x, int64_t M, int64_t C, const float* gamma, const float* beta,
                             float* running_mean, float* running_var, float momentum, float eps,
                             float* save_mean, float* save_invstd, float* save_mean_lo, float* y, int32_t hardtanh,
                             void* work, void* stream) {
  return bn_fwd_train_impl(XIn{x, nullptr}, false, M, C, gamma, beta, running_mean, running_var, momentum, eps,
                           save_mean, save_invstd, save_mean_lo, y, hardtanh, work, stream, make_drop(0.f, 0));
}

BNN_API int bnn_bn_dropout_fwd_train(const float* x, int64_t M, int64_t C, const float* gamma, const float* beta,
                                     float* running_mean, float* running_var, float momentum, float eps,
                                     float* save_mean, float* save_invstd, float* save_mean_lo, float* y,
                                     int32_t hardtanh, float p, uint64_t seed, uint32_t* keep_bits, void* work,
                                     void* stream) {
  if (!(p >= 0.f && p < 1.f)) {
    set_error("bnn_bn_dropout_fwd_train: p must be in [0, 1) (got %g)", (double)p);
    return kErrInval;
  }
  return bn_fwd_train_impl(XIn{x, nullptr}, false, M, C, gamma, beta, running_mean, running_var, momentum, eps,
                           save_mean, save_invstd, save_mean_lo, y, hardtanh, work, stream, make_drop(p, seed),
                           keep_bits);
}

BNN_API int bnn_bn_fwd_train_i16(const int16_t* x16, const float* xbias, int64_t M, int64_t C, const float* gamma,
                                 const float* beta, float* running_mean, float* running_var, float momentum, float eps,
                                 float* save_mean, float* save_invstd, float* save_mean_lo, float p, uint64_t seed,
                                 uint32_t* keep_bits, void* work, void* stream) {
  if (!(p >= 0.f && p < 1.f)) {
    set_error("bnn_bn_fwd_train_i16: p must be in [0, 1) (got %g)", (double)p);
    return kErrInval;
  }
  return bn_fwd_train_impl(XIn{x16, xbias}, true, M, C, gamma, beta, running_mean, running_var, momentum, eps,
                           save_mean, save_invstd, save_mean_lo, nullptr, 0, work, stream, make_drop(p, seed),
                           keep_bits);
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
  hipLaunchKernelGGL(bn_apply_k, apply_grid(M, C), dim3(256), 0, s, x, M, C, running_mean, nullptr, istd, gamma,
                     beta, hardtanh, y);
  return check_launch("bnn_bn_fwd_eval");
}

static int bn_bwd_impl(const float* x, const float* dy, int64_t M, int64_t C, const float* gamma,
                       const float* beta, const float* save_mean, const float* save_invstd,
                       const float* save_mean_lo, int32_t hardtanh,
                       float* dx, float* dgamma, float* dbeta, void* work, void* stream, Drop dp,
                       bool batch_stats) {
  if (!bn_args_ok(x, M, C) || !dy || !aligned16(dy) || !save_mean || !save_invstd || !work ||
      (dx && !aligned16(dx)) || !vec_ok(gamma) || !vec_ok(beta) || !aligned16(save_mean) ||
      !aligned16(save_invstd) || !vec_ok(save_mean_lo)) {
    set_error("bnn_bn_bwd: bad arguments");
    return kErrInval;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t R = bn_chunks(M, C);
  double* p0 = reinterpret_cast<double*>(work);
  double* p1 = p0 + R * C;
  float* k0 = reinterpret_cast<float*>(p1 + R * C);
  float* k1 = reinterpret_cast<float*>(reinterpret_cast<char*>(k0) + round_up(C * 4, 256));
  hipLaunchKernelGGL((bn_reduce_k<1, 0>), reduce_grid(M, C), dim3(256), 0, s, XIn{x, nullptr}, dy,
                     M, C, save_mean, save_mean_lo, save_invstd, gamma, beta, hardtanh, p0, p1, bn_chunk_rows(M, C), dp);
  hipLaunchKernelGGL(bn_bwd_final_k, ffin_grid(C), dim3(256), 0, s, p0, p1, C, R, dgamma,
                     dbeta, k0, k1);
  if (dx) {
    hipLaunchKernelGGL(bn_bwd_apply_k, apply_grid(M, C), dim3(256), 0, s, x, dy, M, C, save_mean, save_mean_lo,
                       save_invstd, gamma, beta, hardtanh, k0, k1, batch_stats ? 1.f / (float)M : 0.f, dx, dp);
  }
  return check_launch("bnn_bn_bwd");
}

namespace bnn {
int64_t bn_workspace_bytes(int64_t M, int64_t C) { return bnn_bn_workspace(M, C); }
// where bn_bwd_sums / bnn_bn_bwd_stats_pre leave k0 = sum g, k1 = sum g*xhat in the workspace
void bn_stat_slots(void* work, int64_t M, int64_t C, const float** k0, const float** k1) {
  const int64_t R = bn_chunks(M, C);
  double* p1 = reinterpret_cast<double*>(work) + R * C;
  float* a = reinterpret_cast<float*>(p1 + R * C);
  *k0 = a;
  *k1 = reinterpret_cast<float*>(reinterpret_cast<char*>(a) + round_up(C * 4, 256));
}
int64_t bn_reduce_chunks(int64_t M, int64_t C) { return bn_chunks(M, C); }

// The statistics half of the training-mode backward (bnn_bn_bwd without its apply pass): k0 =
// sum g, k1 = sum g*xhat per column (and dgamma / dbeta) in `work` (bnn_bn_workspace bytes).
// For passes in other files that form dz themselves (bnn_bn_bwd_i8cols, bnn_pack.hip).
int bn_bwd_sums(XIn xin, int xf, const float* dy, int64_t M, int64_t C, const float* gamma, const float* beta,
                const float* save_mean, const float* save_invstd, const float* save_mean_lo, int32_t hardtanh,
                float* dgamma, float* dbeta, void* work, hipStream_t s, const float** k0_out, const float** k1_out,
                float* pmx, float* scale, int64_t* dsum) {
  if ((xf != 0 && xf != 2) || !bn_args_okf(xin, xf, M, C) || !dy || !aligned16(dy) || !save_mean || !save_invstd ||
      !work || !vec_ok(gamma) || !vec_ok(beta) || !aligned16(save_mean) || !aligned16(save_invstd) ||
      !vec_ok(save_mean_lo)) {
    set_error("bn_bwd_sums: bad arguments");
    return kErrInval;
  }
  const int64_t R = bn_chunks(M, C);
  double* p0 = reinterpret_cast<double*>(work);
  double* p1 = p0 + R * C;
  float* k0 = reinterpret_cast<float*>(p1 + R * C);
  float* k1 = reinterpret_cast<float*>(reinterpret_cast<char*>(k0) + round_up(C * 4, 256));
  if (pmx && !scale) {
    set_error("bn_bwd_sums: the bound pass needs the scale output");
    return kErrInval;
  }
  if (pmx && xf == 2)
    hipLaunchKernelGGL((bn_reduce_k<2, 2>), reduce_grid(M, C), dim3(256), 0, s, xin, dy, M, C,
                       save_mean, save_mean_lo, save_invstd, gamma, beta, hardtanh, p0, p1, bn_chunk_rows(M, C),
                       make_drop(0.f, 0), pmx);
  else if (pmx)
    hipLaunchKernelGGL((bn_reduce_k<2, 0>), reduce_grid(M, C), dim3(256), 0, s, xin, dy, M, C,
                       save_mean, save_mean_lo, save_invstd, gamma, beta, hardtanh, p0, p1, bn_chunk_rows(M, C),
                       make_drop(0.f, 0), pmx);
  else if (xf == 2)
    hipLaunchKernelGGL((bn_reduce_k<1, 2>), reduce_grid(M, C), dim3(256), 0, s, xin, dy, M, C,
                       save_mean, save_mean_lo, save_invstd, gamma, beta, hardtanh, p0, p1, bn_chunk_rows(M, C),
                       make_drop(0.f, 0));
  else
    hipLaunchKernelGGL((bn_reduce_k<1, 0>), reduce_grid(M, C), dim3(256), 0, s, xin, dy, M, C,
                       save_mean, save_mean_lo, save_invstd, gamma, beta, hardtanh, p0, p1, bn_chunk_rows(M, C),
                       make_drop(0.f, 0));
  hipLaunchKernelGGL(bn_bwd_final_k, ffin_grid(C), dim3(256), 0, s, p0, p1, C, R, dgamma, dbeta, k0, k1,
                     I8cBound{pmx, save_invstd, gamma, 1.f / (float)M, scale, dsum});
  *k0_out = k0;
  *k1_out = k1;
  return check_launch("bn_bwd_sums");
}
}  // namespace bnn

BNN_API int bnn_bn_bwd(const float* x, const float* dy, int64_t M, int64_t C, const float* gamma,
                       const float* beta, const float* save_mean, const float* save_invstd,
                       const float* save_mean_lo, int32_t hardtanh, float* dx, float* dgamma, float* dbeta,
                       void* work, void* stream) {
  return bn_bwd_impl(x, dy, M, C, gamma, beta, save_mean, save_invstd, save_mean_lo, hardtanh, dx, dgamma, dbeta,
                     work, stream, make_drop(0.f, 0), true);
}

BNN_API int bnn_bn_bwd_eval(const float* x, const float* dy, int64_t M, int64_t C, const float* gamma,
                            const float* beta, const float* running_mean, const float* invstd, int32_t hardtanh,
                            float* dx, float* dgamma, float* dbeta, void* work, void* stream) {
  return bn_bwd_impl(x, dy, M, C, gamma, beta, running_mean, invstd, nullptr, hardtanh, dx, dgamma, dbeta, work,
                     stream, make_drop(0.f, 0), false);
}

BNN_API int bnn_bn_dropout_bwd(const float* x, const float* dy, int64_t M, int64_t C, const float* gamma,
                               const float* beta, const float* save_mean, const float* save_invstd,
                               const float* save_mean_lo, int32_t hardtanh, float p, uint64_t seed, float* dx,
                               float* dgamma, float* dbeta, void* work, void* stream) {
  if (!(p >= 0.f && p < 1.f)) {
    set_error("bnn_bn_dropout_bwd: p must be in [0, 1) (got %g)", (double)p);
    return kErrInval;
  }
  return bn_bwd_impl(x, dy, M, C, gamma, beta, save_mean, save_invstd, save_mean_lo, hardtanh, dx, dgamma, dbeta,
                     work, stream, make_drop(p, seed), true);
}

// pre: the statistics are already in `work` (bnn_bn_bwd_stats_pre from the dX GEMM's epilogue
// partials): only the quantising apply pass runs
static int bn_bwd_q6_impl(XIn xin, bool z16, const float* dy, int64_t M, int64_t C, const float* gamma,
                          const float* beta, const float* save_mean, const float* save_invstd,
                          const float* save_mean_lo, int32_t hardtanh, float p, uint64_t seed, float* dx,
                          float* dgamma, float* dbeta, uint8_t* rlo, uint8_t* rhi, uint8_t* rsc, uint8_t* rres, uint8_t* clo,
                          uint8_t* chi, uint8_t* csc, float* colsum, void* work, void* stream, bool pre = false) {
  const float* x = reinterpret_cast<const float*>(xin.p);
  if (!(z16 ? bn_args_ok16(xin, M, C) : bn_args_ok(x, M, C)) || C % Q6T_COLS != 0 || !dy || !aligned16(dy) ||
      !save_mean || !save_invstd || !work || (dx && !aligned16(dx)) || !vec_ok(gamma) || !vec_ok(beta) ||
      !aligned16(save_mean) || !aligned16(save_invstd) || !vec_ok(save_mean_lo) || !rlo || !rhi || !rsc || !clo ||
      !chi || !csc || !aligned16(rlo) || !aligned16(rhi) || !aligned16(clo) || !aligned16(chi) ||
      (rres && !aligned16(rres)) || !(p >= 0.f && p < 1.f) || (M + Q6T_SUB - 1) / Q6T_SUB > 65535) {
    set_error("bnn_bn_bwd_q6: bad arguments (M=%lld C=%lld; C must be a multiple of 64, 0 <= p < 1)", (long long)M,
              (long long)C);
    return kErrInval;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const Drop dp = make_drop(p, seed);
  const int64_t R = bn_chunks(M, C);
  double* p0 = reinterpret_cast<double*>(work);
  double* p1 = p0 + R * C;
  float* k0 = reinterpret_cast<float*>(p1 + R * C);
  float* k1 = reinterpret_cast<float*>(reinterpret_cast<char*>(k0) + round_up(C * 4, 256));
  if (pre && p > 0.f) {
    set_error("bnn_bn_bwd_q6_pre: the epilogue statistics carry no dropout mask (p must be 0)");
    return kErrInval;
  }
  if (!pre) {
    if (z16)
      hipLaunchKernelGGL((bn_reduce_k<1, 1>), reduce_grid(M, C), dim3(256), 0, s, xin, dy, M, C, save_mean,
                         save_mean_lo, save_invstd, gamma, beta, hardtanh, p0, p1, bn_chunk_rows(M, C), dp);
    else
      hipLaunchKernelGGL((bn_reduce_k<1, 0>), reduce_grid(M, C), dim3(256), 0, s, xin, dy, M, C, save_mean,
                         save_mean_lo, save_invstd, gamma, beta, hardtanh, p0, p1, bn_chunk_rows(M, C), dp);
    hipLaunchKernelGGL(bn_bwd_final_k, ffin_grid(C), dim3(256), 0, s, p0, p1, C, R, dgamma, dbeta, k0, k1);
  }
  // p0 is free once bn_bwd_final_k has folded it: it takes the column-sum partials
  const int64_t mp = round_up(M, 64);
  Q6Out o{dx, rlo, rhi, rsc, q6_scale_rows(M), clo, chi, csc, q6_scale_rows(C), mp / QB, colsum ? p0 : nullptr};
  o.rres = rres;
  const int64_t qr = q6_rows(M, C);
  const dim3 g((unsigned)(C / Q6T_COLS), (unsigned)((M + qr - 1) / qr));
  if (z16)
    hipLaunchKernelGGL((bn_bwd_apply_q6_k<0, true>), g, dim3(256), 0, s, xin, dy, M, C, save_mean, save_mean_lo,
                       save_invstd, gamma, beta, hardtanh, k0, k1, 1.f / (float)M, o, dp, nullptr, (int)qr);
  else
    hipLaunchKernelGGL((bn_bwd_apply_q6_k<0, false>), g, dim3(256), 0, s, xin, dy, M, C, save_mean, save_mean_lo,
                       save_invstd, gamma, beta, hardtanh, k0, k1, 1.f / (float)M, o, dp, nullptr, (int)qr);
  if (colsum)
    hipLaunchKernelGGL(q6_colsum_final_k, ffin_grid(C), dim3(256), 0, s, p0, (M + qr - 1) / qr, C, colsum);
  return check_launch("bnn_bn_bwd_q6");
}

#if defined(Q6_DIAG_STAMPS)
BNN_API int bnn_q6_stamps_copy(void* dst, int64_t bytes) {
  if (bytes < (int64_t)sizeof(g_q6_stamps)) return kErrInval;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_q6_stamps), sizeof(g_q6_stamps), 0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0 : kErrInval;
}
#endif

BNN_API int bnn_bn_bwd_q6(const float* x, const float* dy, int64_t M, int64_t C, const float* gamma,
                          const float* beta, const float* save_mean, const float* save_invstd,
                          const float* save_mean_lo, int32_t hardtanh, float p, uint64_t seed, float* dx,
                          float* dgamma, float* dbeta, uint8_t* rlo, uint8_t* rhi, uint8_t* rsc, uint8_t* rres, uint8_t* clo,
                          uint8_t* chi, uint8_t* csc, float* colsum, void* work, void* stream) {
  return bn_bwd_q6_impl(XIn{x, nullptr}, false, dy, M, C, gamma, beta, save_mean, save_invstd, save_mean_lo, hardtanh,
                        p, seed, dx, dgamma, dbeta, rlo, rhi, rsc, rres, clo, chi, csc, colsum, work, stream);
}

BNN_API int bnn_bn_bwd_q6_pre(const float* x, const float* dy, int64_t M, int64_t C, const float* gamma,
                              const float* beta, const float* save_mean, const float* save_invstd,
                              const float* save_mean_lo, int32_t hardtanh, float p, uint64_t seed, float* dx,
                              float* dgamma, float* dbeta, uint8_t* rlo, uint8_t* rhi, uint8_t* rsc, uint8_t* rres, uint8_t* clo,
                              uint8_t* chi, uint8_t* csc, float* colsum, void* work, void* stream) {
  return bn_bwd_q6_impl(XIn{x, nullptr}, false, dy, M, C, gamma, beta, save_mean, save_invstd, save_mean_lo, hardtanh,
                        p, seed, dx, dgamma, dbeta, rlo, rhi, rsc, rres, clo, chi, csc, colsum, work, stream, true);
}

BNN_API int bnn_bn_bwd_q6_i16_pre(const int16_t* x16, const float* xbias, const float* dy, int64_t M, int64_t C,
                                  const float* gamma, const float* beta, const float* save_mean,
                                  const float* save_invstd, const float* save_mean_lo, int32_t hardtanh, float p,
                                  uint64_t seed, float* dx, float* dgamma, float* dbeta, uint8_t* rlo, uint8_t* rhi,
                                  uint8_t* rsc, uint8_t* rres, uint8_t* clo, uint8_t* chi, uint8_t* csc, float* colsum, void* work,
                                  void* stream) {
  return bn_bwd_q6_impl(XIn{x16, xbias}, true, dy, M, C, gamma, beta, save_mean, save_invstd, save_mean_lo, hardtanh,
                        p, seed, dx, dgamma, dbeta, rlo, rhi, rsc, rres, clo, chi, csc, colsum, work, stream, true);
}

// The statistics half of a training-mode BatchNorm(+Hardtanh) backward from the per-tile-row partials
// the FP6 dX GEMM's epilogue wrote (bnn_gemm_fp6_bnstats: part [2 or 4][R][C] floats): k0 = sum g,
// k1 = sum g*xhat into `work` (bnn_bn_workspace(M, C) bytes, where the *_pre apply entries read them),
// dgamma / dbeta, and (mode 2) the int8 column-digit scale from the max|g| / max|xhat| bound + zeroed
// digit sums, as bn_bwd_final_k does for bn_reduce_k's partials.
BNN_API int bnn_bn_bwd_stats_pre(const float* part, int64_t R, int64_t M, int64_t C, int32_t mode, const float* gamma,
                                 const float* save_invstd, float* dgamma, float* dbeta, float* scale, int64_t* dsum,
                                 void* work, void* stream) {
  if (!part || R <= 0 || M <= 0 || C <= 0 || (mode != 1 && mode != 2) || !work || (mode == 2 && (!scale || !save_invstd))) {
    set_error("bnn_bn_bwd_stats_pre: bad arguments");
    return kErrInval;
  }
  const int64_t Rb = bn_chunks(M, C);
  double* p1 = reinterpret_cast<double*>(work) + Rb * C;
  float* k0 = reinterpret_cast<float*>(p1 + Rb * C);
  float* k1 = reinterpret_cast<float*>(reinterpret_cast<char*>(k0) + round_up(C * 4, 256));
  const I8cBound ib = mode == 2 ? I8cBound{part + 2 * R * C, save_invstd, gamma, 1.f / (float)M, scale, dsum}
                                : I8cBound{nullptr, nullptr, nullptr, 0.f, nullptr, nullptr};
  hipLaunchKernelGGL(bn_bwd_final_pre_k, ffin_grid(C), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), part,
                     part + R * C, C, R, dgamma, dbeta, k0, k1, ib);
  return check_launch("bnn_bn_bwd_stats_pre");
}

BNN_API int bnn_bn_bwd_q6_i16(const int16_t* x16, const float* xbias, const float* dy, int64_t M, int64_t C,
                              const float* gamma, const float* beta, const float* save_mean, const float* save_invstd,
                              const float* save_mean_lo, int32_t hardtanh, float p, uint64_t seed, float* dx,
                              float* dgamma, float* dbeta, uint8_t* rlo, uint8_t* rhi, uint8_t* rsc, uint8_t* rres, uint8_t* clo,
                              uint8_t* chi, uint8_t* csc, float* colsum, void* work, void* stream) {
  return bn_bwd_q6_impl(XIn{x16, xbias}, true, dy, M, C, gamma, beta, save_mean, save_invstd, save_mean_lo, hardtanh,
                        p, seed, dx, dgamma, dbeta, rlo, rhi, rsc, rres, clo, chi, csc, colsum, work, stream);
}

constexpr int HEAD_NOUT = 10;   // the reference head: nn.Linear(C, 10) (mnist-dist2.py:73)

// columns per thread of the head's statistics pass (bnn_bn_set_head_reduce_cols): 2 (bn_head_reduce2_k,
// 4 waves per SIMD: 496 vs 527 us on the wide step, profiles/r05_kb2_*) or 4 (bn_head_reduce_k);
// bit-identical results
#ifndef BNN_HEAD_RED_COLS_DEFAULT
#define BNN_HEAD_RED_COLS_DEFAULT 2
#endif
static int g_head_red_cols = BNN_HEAD_RED_COLS_DEFAULT;

BNN_API int32_t bnn_bn_set_head_reduce_cols(int32_t cols) {
  if (cols < 0) return g_head_red_cols;
  if (cols != 2 && cols != 4) return kErrInval;
  g_head_red_cols = cols;
  return 0;
}

BNN_API int64_t bnn_bn_head_workspace(int64_t M, int64_t C, int32_t nout) {
  return bnn_bn_workspace(M, C) + round_up(bn_chunks(M, C) * (int64_t)nout * C * (int64_t)sizeof(float), 256);
}

static int bn_head_fwd_impl(XIn xin, bool z16, int64_t M, int64_t C, const float* mean, const float* invstd,
                            const float* mean_lo, const float* gamma, const float* beta, float p, uint64_t seed,
                            const uint32_t* keep_bits, const float* w4, int32_t nout, const float* b4, float* y4,
                            void* stream) {
  const float* x = reinterpret_cast<const float*>(xin.p);
  if (!(z16 ? bn_args_ok16(xin, M, C) : bn_args_ok(x, M, C)) || C % HD_COLS != 0 || !mean || !invstd || !w4 || !y4 ||
      nout != HEAD_NOUT || !aligned16(mean) || !aligned16(invstd) || !vec_ok(mean_lo) || !vec_ok(gamma) ||
      !vec_ok(beta) || !(p >= 0.f && p < 1.f)) {
    set_error("bnn_bn_head_fwd: bad arguments (M=%lld C=%lld nout=%d; C %% 128 == 0, nout == 10)", (long long)M,
              (long long)C, nout);
    return kErrInval;
  }
  const dim3 g((unsigned)((M + HD_ROWS - 1) / HD_ROWS));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  Drop dp = make_drop(p, seed);
  dp.bits = dp.on ? keep_bits : nullptr;
  auto k = z16 ? (dp.bits ? bn_head_fwd_k<HEAD_NOUT, true, true> : bn_head_fwd_k<HEAD_NOUT, true, false>)
               : (dp.bits ? bn_head_fwd_k<HEAD_NOUT, false, true> : bn_head_fwd_k<HEAD_NOUT, false, false>);
  hipLaunchKernelGGL(k, g, dim3(256), 0, s, xin, M, C, mean, mean_lo, invstd, gamma, beta, w4, b4, y4, dp);
  return check_launch("bnn_bn_head_fwd");
}

BNN_API int bnn_bn_head_fwd(const float* x, int64_t M, int64_t C, const float* mean, const float* invstd,
                            const float* mean_lo, const float* gamma, const float* beta, float p, uint64_t seed,
                            const uint32_t* keep_bits, const float* w4, int32_t nout, const float* b4, float* y4,
                            void* stream) {
  return bn_head_fwd_impl(XIn{x, nullptr}, false, M, C, mean, invstd, mean_lo, gamma, beta, p, seed, keep_bits, w4,
                          nout, b4, y4, stream);
}

BNN_API int bnn_bn_head_fwd_i16(const int16_t* x16, const float* xbias, int64_t M, int64_t C, const float* mean,
                                const float* invstd, const float* mean_lo, const float* gamma, const float* beta,
                                float p, uint64_t seed, const uint32_t* keep_bits, const float* w4, int32_t nout,
                                const float* b4, float* y4, void* stream) {
  return bn_head_fwd_impl(XIn{x16, xbias}, true, M, C, mean, invstd, mean_lo, gamma, beta, p, seed, keep_bits, w4,
                          nout, b4, y4, stream);
}

// Row chunks of the fused head's backward statistics pass: the BatchNorm chunks, but never fewer
// than 16 rows.  A narrow head (config 3: 768 columns at 4,096 rows) would otherwise get 4-row chunks
// (bn_chunk_rows fills the chip with threads) -- 1,024 chunk partials of dgamma / dbeta and of
// dW4's 10 x C products (31 MB) to write and fold -- and the keep-bit plane, whose words are 8 rows,
// would be re-hashed instead of read.  Fixed per shape (deterministic).
#ifndef HEAD_MIN_ROWS
#define HEAD_MIN_ROWS 16
#endif
inline int64_t head_chunk_rows(int64_t M, int64_t C) { return std::max<int64_t>(bn_chunk_rows(M, C), HEAD_MIN_ROWS); }
inline int64_t head_chunks(int64_t M, int64_t C) {
  const int64_t rows = head_chunk_rows(M, C);
  return std::max<int64_t>(1, (M + rows - 1) / rows);
}

static int bn_head_bwd_q6_impl(XIn xin, bool z16, const float* dy4, const float* w4, int32_t nout, int64_t M,
                               int64_t C, const float* gamma, const float* beta, const float* save_mean,
                               const float* save_invstd, const float* save_mean_lo, float p, uint64_t seed,
                               const uint32_t* keep_bits, float* dx, float* dgamma, float* dbeta, float* dw4,
                               uint8_t* rlo, uint8_t* rhi, uint8_t* rsc, uint8_t* rres, uint8_t* clo, uint8_t* chi,
                               uint8_t* csc, float* colsum, void* work, void* stream) {
  const float* x = reinterpret_cast<const float*>(xin.p);
  if (!(z16 ? bn_args_ok16(xin, M, C) : bn_args_ok(x, M, C)) || C % 256 != 0 || !dy4 || !w4 || !dw4 ||
      nout != HEAD_NOUT || !save_mean || !save_invstd || !work || (dx && !aligned16(dx)) || !vec_ok(gamma) ||
      !vec_ok(beta) || !aligned16(save_mean) || !aligned16(save_invstd) || !vec_ok(save_mean_lo) || !aligned16(w4) ||
      !rlo || !rhi || !rsc || !clo || !chi || !csc || !aligned16(rlo) || !aligned16(rhi) || !aligned16(clo) ||
      !aligned16(chi) || (rres && !aligned16(rres)) || !(p >= 0.f && p < 1.f) || (M + Q6T_SUB - 1) / Q6T_SUB > 65535) {
    set_error("bnn_bn_head_bwd_q6: bad arguments (M=%lld C=%lld nout=%d)", (long long)M, (long long)C, nout);
    return kErrInval;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  Drop dp = make_drop(p, seed);
  dp.bits = dp.on ? keep_bits : nullptr;   // the apply pass reads the forward's keep bits in any shape
  Drop dpr = dp;                           // the statistics pass where its 8-row batches are whole words
  const int64_t hrows = head_chunk_rows(M, C);
  if (!(RED_RB == 8 && hrows % 8 == 0)) dpr.bits = nullptr;
  const int64_t R = head_chunks(M, C);
  double* p0 = reinterpret_cast<double*>(work);
  double* p1 = p0 + R * C;
  float* k0 = reinterpret_cast<float*>(p1 + R * C);
  float* k1 = reinterpret_cast<float*>(reinterpret_cast<char*>(k0) + round_up(C * 4, 256));
  float* pw = reinterpret_cast<float*>(reinterpret_cast<char*>(work) + bnn_bn_workspace(M, C));
  if (g_head_red_cols == 2) {
    auto kr = z16 ? (dpr.bits ? bn_head_reduce2_k<HEAD_NOUT, true, true> : bn_head_reduce2_k<HEAD_NOUT, true, false>)
                  : (dpr.bits ? bn_head_reduce2_k<HEAD_NOUT, false, true> : bn_head_reduce2_k<HEAD_NOUT, false, false>);
    const dim3 g2((unsigned)(((C / 2) * R + 255) / 256));
    hipLaunchKernelGGL(kr, g2, dim3(256), 0, s, xin, dy4, w4, M, C, save_mean, save_mean_lo, save_invstd, gamma,
                       beta, p0, p1, pw, hrows, dpr);
  } else {
    auto kr = z16 ? (dpr.bits ? bn_head_reduce_k<HEAD_NOUT, true, true> : bn_head_reduce_k<HEAD_NOUT, true, false>)
                  : (dpr.bits ? bn_head_reduce_k<HEAD_NOUT, false, true> : bn_head_reduce_k<HEAD_NOUT, false, false>);
    hipLaunchKernelGGL(kr, dim3((unsigned)(((C / 4) * R + 255) / 256)), dim3(256), 0, s, xin, dy4, w4, M, C, save_mean,
                       save_mean_lo, save_invstd, gamma, beta, p0, p1, pw, hrows, dpr);
  }
  hipLaunchKernelGGL(bn_bwd_final_k, ffin_grid(C), dim3(256), 0, s, p0, p1, C, R, dgamma, dbeta, k0, k1);
  hipLaunchKernelGGL(head_dw_final_k, dim3((unsigned)((nout * C + HD_FF_COLS - 1) / HD_FF_COLS)),
                     dim3(HD_FF_COLS * FF_GROUPS), 0, s, pw, R,
                     (int64_t)nout, C, dw4);
  const int64_t mp = round_up(M, 64);
  Q6Out o{dx, rlo, rhi, rsc, q6_scale_rows(M), clo, chi, csc, q6_scale_rows(C), mp / QB, colsum ? p0 : nullptr};
  o.rres = rres;
  const int64_t qr = q6_rows(M, C);
  const dim3 g((unsigned)(C / Q6T_COLS), (unsigned)((M + qr - 1) / qr));
  auto ka = z16 ? (dp.bits ? bn_bwd_apply_q6_k<HEAD_NOUT, true, true> : bn_bwd_apply_q6_k<HEAD_NOUT, true, false>)
                : (dp.bits ? bn_bwd_apply_q6_k<HEAD_NOUT, false, true> : bn_bwd_apply_q6_k<HEAD_NOUT, false, false>);
  hipLaunchKernelGGL(ka, g, dim3(256), 0, s, xin, dy4, M, C, save_mean, save_mean_lo, save_invstd, gamma, beta, 1, k0,
                     k1, 1.f / (float)M, o, dp, w4, (int)qr);
  if (colsum)
    hipLaunchKernelGGL(q6_colsum_final_k, ffin_grid(C), dim3(256), 0, s, p0, (M + qr - 1) / qr, C, colsum);
  return check_launch("bnn_bn_head_bwd_q6");
}

BNN_API int bnn_bn_head_bwd_q6(const float* x, const float* dy4, const float* w4, int32_t nout, int64_t M, int64_t C,
                               const float* gamma, const float* beta, const float* save_mean,
                               const float* save_invstd, const float* save_mean_lo, float p, uint64_t seed,
                               const uint32_t* keep_bits, float* dx, float* dgamma, float* dbeta, float* dw4,
                               uint8_t* rlo, uint8_t* rhi, uint8_t* rsc, uint8_t* rres, uint8_t* clo, uint8_t* chi,
                               uint8_t* csc, float* colsum, void* work, void* stream) {
  return bn_head_bwd_q6_impl(XIn{x, nullptr}, false, dy4, w4, nout, M, C, gamma, beta, save_mean, save_invstd,
                             save_mean_lo, p, seed, keep_bits, dx, dgamma, dbeta, dw4, rlo, rhi, rsc, rres, clo, chi, csc, colsum,
                             work, stream);
}

BNN_API int bnn_bn_head_bwd_q6_i16(const int16_t* x16, const float* xbias, const float* dy4, const float* w4,
                                   int32_t nout, int64_t M, int64_t C, const float* gamma, const float* beta,
                                   const float* save_mean, const float* save_invstd, const float* save_mean_lo,
                                   float p, uint64_t seed, const uint32_t* keep_bits, float* dx, float* dgamma,
                                   float* dbeta, float* dw4, uint8_t* rlo, uint8_t* rhi, uint8_t* rsc, uint8_t* rres,
                                   uint8_t* clo, uint8_t* chi, uint8_t* csc, float* colsum, void* work, void* stream) {
  return bn_head_bwd_q6_impl(XIn{x16, xbias}, true, dy4, w4, nout, M, C, gamma, beta, save_mean, save_invstd,
                             save_mean_lo, p, seed, keep_bits, dx, dgamma, dbeta, dw4, rlo, rhi, rsc, rres, clo, chi, csc, colsum,
                             work, stream);
}

BNN_API int bnn_set_seed_counter(const int64_t* ctr) {
  g_seed_ctr = ctr;
  return 0;
}

__global__ __launch_bounds__(256) void dropout_mask_k(int64_t n, Drop d0, float* __restrict__ out) {
  const Drop d = drop_resolve(d0);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = (!d.on || drop_keep(d, (uint64_t)i)) ? d.scale : 0.f;   // p == 0: the fused passes never mask
}

BNN_API int bnn_dropout_mask(int64_t n, float p, uint64_t seed, float* out, void* stream) {
  if (n < 0 || (n > 0 && !out) || !(p >= 0.f && p < 1.f)) {
    set_error("bnn_dropout_mask: bad arguments");
    return kErrInval;
  }
  if (n == 0) return 0;
  const Drop d = make_drop(p, seed);   // p == 0: d.on = 0, scale 1 -> every element kept
  hipLaunchKernelGGL(dropout_mask_k, dim3(grid_for(n)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), n, d,
                     out);
  return check_launch("bnn_dropout_mask");
}

BNN_API int64_t bnn_bn2d_workspace(int64_t N, int64_t C) {
  const int64_t R = (std::max<int64_t>(N, 1) + bn2_chunk_images(std::max<int64_t>(N, 1), C) - 1) /
                    bn2_chunk_images(std::max<int64_t>(N, 1), C);
  return 2 * R * C * (int64_t)sizeof(double) + 2 * round_up(C * 4, 256);
}

#define BN2_POOL_SWITCH(pool, ...) \
  do { if (pool) { constexpr int P = 2; __VA_ARGS__; } else { constexpr int P = 0; __VA_ARGS__; } } while (0)
#define BN2_XF_SWITCH(xf, ...)                                               \
  do {                                                                       \
    if ((xf) == 1) { constexpr int XFV = 1; __VA_ARGS__; }                   \
    else if ((xf) == 2) { constexpr int XFV = 2; __VA_ARGS__; }              \
    else { constexpr int XFV = 0; __VA_ARGS__; }                             \
  } while (0)

// 1 (default): the pooled statistics and forward apply of 28- / 14-wide planes on the row kernels
// (bn2d_*_rows_k); 2: also the backward apply (slower: A/B only); 0: the window-per-thread kernels
static int g_bn2_rows = 1;

BNN_API int bnn_bn2d_set_rows(int32_t on) {
  g_bn2_rows = on < 0 ? 1 : (on > 2 ? 1 : on);
  return 0;
}

static int bn2d_fwd_train_impl(X2 x, int xf, int64_t N, int64_t C, int64_t H, int64_t W, const float* gamma,
                               const float* beta, float* running_mean, float* running_var, float momentum,
                               float eps, float* save_mean, float* save_invstd, float* y, int32_t hardtanh,
                               int32_t pool, void* work, void* stream) {
  if (!bn2_args_ok(reinterpret_cast<const float*>(x.p), N, C, H, W, pool) || !save_mean || !save_invstd || !work ||
      !y || (running_mean == nullptr) != (running_var == nullptr) || xf < 0 || xf > 2 || (xf == 0 && x.bias) ||
      (x.bias && !aligned16(x.bias)) || (xf != 0 && N * C * H * W * xf >= (1LL << 31))) {
    set_error("bnn_bn2d_fwd_train: bad arguments (N=%lld C=%lld H=%lld W=%lld pool=%d; H*W must be a multiple "
              "of 4, pool 0 or 2 with even H, W)", (long long)N, (long long)C, (long long)H, (long long)W, pool);
    return kErrInval;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t CR = bn2_chunk_images(N, C), R = (N + CR - 1) / CR;
  double* p0 = reinterpret_cast<double*>(work);
  double* p1 = p0 + R * C;
  if (g_bn2_rows && (H * W) % 4 == 0 && CR * (H * W / 4) < (1LL << 30)) {   // flattened, batched loads
    BN2_XF_SWITCH(xf, hipLaunchKernelGGL((bn2d_fwd_stats_flat_k<XFV>), dim3((unsigned)C, (unsigned)R), dim3(BN2_T), 0,
                                         s, x, N, C, (int)(H * W), CR, p0, p1));
  } else {
    BN2_XF_SWITCH(xf, hipLaunchKernelGGL((bn2d_reduce_k<0, 0, XFV>), dim3((unsigned)C, (unsigned)R), dim3(BN2_T), 0,
                                         s, x, nullptr, N, C, (int)H, (int)W, CR, nullptr, nullptr, nullptr, nullptr,
                                         0, p0, p1));
  }
  hipLaunchKernelGGL(bn_fwd_final_k, ffin_grid(C), dim3(256), 0, s, p0, p1, N, C, R,
                     momentum, eps, running_mean, running_var, save_mean, save_invstd, nullptr, CR, H * W);
  const int64_t outs = pool ? N * C * (H / 2) * (W / 2) : N * C * H * W / 4;
  if (pool && g_bn2_rows && (W == 28 || W == 14)) {   // the BinCNN's pooled layers: one row per thread
    const dim3 rg((unsigned)((N * C * (H / 2) + 255) / 256));
    if (W == 28)
      BN2_XF_SWITCH(xf, hipLaunchKernelGGL((bn2d_apply_rows_k<14, XFV>), rg, dim3(256), 0, s, x, N, C, (int)H,
                                           save_mean, save_invstd, gamma, beta, hardtanh, y));
    else
      BN2_XF_SWITCH(xf, hipLaunchKernelGGL((bn2d_apply_rows_k<7, XFV>), rg, dim3(256), 0, s, x, N, C, (int)H,
                                           save_mean, save_invstd, gamma, beta, hardtanh, y));
  } else {
    BN2_XF_SWITCH(xf, BN2_POOL_SWITCH(pool, hipLaunchKernelGGL((bn2d_apply_k<P, XFV>), dim3(grid_for(outs)), dim3(256),
                                                                 0, s, x, N, C, (int)H, (int)W, save_mean, save_invstd,
                                                                 gamma, beta, hardtanh, y)));
  }
  return check_launch("bnn_bn2d_fwd_train");
}

BNN_API int bnn_bn2d_fwd_train(const float* x, int64_t N, int64_t C, int64_t H, int64_t W, const float* gamma,
                               const float* beta, float* running_mean, float* running_var, float momentum,
                               float eps, float* save_mean, float* save_invstd, float* y, int32_t hardtanh,
                               int32_t pool, void* work, void* stream) {
  return bn2d_fwd_train_impl(X2{x, nullptr}, 0, N, C, H, W, gamma, beta, running_mean, running_var, momentum, eps,
                             save_mean, save_invstd, y, hardtanh, pool, work, stream);
}

BNN_API int bnn_bn2d_fwd_train_q(const void* xq, const float* xbias, int32_t xfmt, int64_t N, int64_t C, int64_t H,
                                 int64_t W, const float* gamma, const float* beta, float* running_mean,
                                 float* running_var, float momentum, float eps, float* save_mean, float* save_invstd,
                                 float* y, int32_t hardtanh, int32_t pool, void* work, void* stream) {
  if (xfmt != 1 && xfmt != 2) {
    set_error("bnn_bn2d_fwd_train_q: xfmt must be 1 (int8) or 2 (int16)");
    return kErrInval;
  }
  return bn2d_fwd_train_impl(X2{xq, xbias}, xfmt, N, C, H, W, gamma, beta, running_mean, running_var, momentum, eps,
                             save_mean, save_invstd, y, hardtanh, pool, work, stream);
}

BNN_API int bnn_bn2d_fwd_eval(const float* x, int64_t N, int64_t C, int64_t H, int64_t W, const float* gamma,
                              const float* beta, const float* running_mean, const float* running_var, float eps,
                              float* y, int32_t hardtanh, int32_t pool, void* work, void* stream) {
  if (!bn2_args_ok(x, N, C, H, W, pool) || !running_mean || !running_var || !y || !work) {
    set_error("bnn_bn2d_fwd_eval: bad arguments");
    return kErrInval;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* istd = reinterpret_cast<float*>(work);
  hipLaunchKernelGGL(bn_invstd_k, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, running_var, istd, C, eps);
  const int64_t outs = pool ? N * C * (H / 2) * (W / 2) : N * C * H * W / 4;
  BN2_POOL_SWITCH(pool, hipLaunchKernelGGL((bn2d_apply_k<P, 0>), dim3(grid_for(outs)), dim3(256), 0, s, X2{x, nullptr},
                                           N, C, (int)H, (int)W, running_mean, istd, gamma, beta, hardtanh, y));
  return check_launch("bnn_bn2d_fwd_eval");
}

static int bn2d_bwd_impl(X2 x, int xf, const float* dy, int64_t N, int64_t C, int64_t H, int64_t W,
                         const float* gamma, const float* beta, const float* save_mean, const float* save_invstd,
                         int32_t hardtanh, int32_t pool, float* dx, float* dgamma, float* dbeta, void* work,
                         void* stream, bool batch_stats, float* k0_out = nullptr, float* k1_out = nullptr) {
  if (!bn2_args_ok(reinterpret_cast<const float*>(x.p), N, C, H, W, pool) || !dy || !save_mean || !save_invstd ||
      !work || (dx && !aligned16(dx)) || (!pool && !aligned16(dy)) || xf < 0 || xf > 2 || (xf == 0 && x.bias) ||
      (x.bias && !aligned16(x.bias)) || (xf != 0 && N * C * H * W * xf >= (1LL << 31))) {
    set_error("bnn_bn2d_bwd: bad arguments");
    return kErrInval;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t CR = bn2_chunk_images(N, C), R = (N + CR - 1) / CR;
  double* p0 = reinterpret_cast<double*>(work);
  double* p1 = p0 + R * C;
  float* k0 = k0_out ? k0_out : reinterpret_cast<float*>(p1 + R * C);
  float* k1 = k1_out ? k1_out : reinterpret_cast<float*>(reinterpret_cast<char*>(p1 + R * C) + round_up(C * 4, 256));
  if (pool && g_bn2_rows && (W == 28 || W == 14)) {   // the BinCNN's pooled layers: row-batched loads
    if (W == 28)
      BN2_XF_SWITCH(xf, hipLaunchKernelGGL((bn2d_bwd_stats_rows_k<14, XFV>), dim3((unsigned)C, (unsigned)R),
                                           dim3(BN2_T), 0, s, x, dy, N, C, (int)H, CR, save_mean, save_invstd, gamma,
                                           beta, hardtanh, p0, p1));
    else
      BN2_XF_SWITCH(xf, hipLaunchKernelGGL((bn2d_bwd_stats_rows_k<7, XFV>), dim3((unsigned)C, (unsigned)R),
                                           dim3(BN2_T), 0, s, x, dy, N, C, (int)H, CR, save_mean, save_invstd, gamma,
                                           beta, hardtanh, p0, p1));
  } else {
    BN2_XF_SWITCH(xf, BN2_POOL_SWITCH(pool, hipLaunchKernelGGL((bn2d_reduce_k<1, P, XFV>), dim3((unsigned)C, (unsigned)R),
                                                                 dim3(BN2_T), 0, s, x, dy, N, C, (int)H, (int)W, CR,
                                                                 save_mean, save_invstd, gamma, beta, hardtanh, p0, p1)));
  }
  hipLaunchKernelGGL(bn_bwd_final_k, ffin_grid(C), dim3(256), 0, s, p0, p1, C, R, dgamma,
                     dbeta, k0, k1);
  if (dx) {
    const int64_t outs = pool ? N * C * (H / 2) * (W / 2) : N * C * H * W / 4;
    const float inv_n = batch_stats ? (float)(1.0 / ((double)N * (double)(H * W))) : 0.f;
    // (the row form, bn2d_bwd_apply_rows_k, is built for A/B only -- g_bn2_rows == 2: its two
    // full-resolution output rows per thread write 8-B pieces 224 B apart, 186 vs 70 us on the
    // BinCNN's first layer, profiles/r04_cnn_bn2d_rows.log)
    if (pool && g_bn2_rows == 2 && (W == 28 || W == 14)) {
      const dim3 rg((unsigned)((N * C * (H / 2) + 255) / 256));
      if (W == 28)
        BN2_XF_SWITCH(xf, hipLaunchKernelGGL((bn2d_bwd_apply_rows_k<14, XFV>), rg, dim3(256), 0, s, x, dy, N, C,
                                             (int)H, save_mean, save_invstd, gamma, beta, hardtanh, k0, k1, inv_n, dx));
      else
        BN2_XF_SWITCH(xf, hipLaunchKernelGGL((bn2d_bwd_apply_rows_k<7, XFV>), rg, dim3(256), 0, s, x, dy, N, C,
                                             (int)H, save_mean, save_invstd, gamma, beta, hardtanh, k0, k1, inv_n, dx));
    } else {
      BN2_XF_SWITCH(xf, BN2_POOL_SWITCH(pool, hipLaunchKernelGGL((bn2d_bwd_apply_k<P, XFV>), dim3(grid_for(outs)),
                                                                   dim3(256), 0, s, x, dy, N, C, (int)H, (int)W,
                                                                   save_mean, save_invstd, gamma, beta, hardtanh, k0,
                                                                   k1, inv_n, dx)));
    }
  }
  return check_launch("bnn_bn2d_bwd");
}

BNN_API int bnn_bn2d_bwd(const float* x, const float* dy, int64_t N, int64_t C, int64_t H, int64_t W,
                         const float* gamma, const float* beta, const float* save_mean, const float* save_invstd,
                         int32_t hardtanh, int32_t pool, float* dx, float* dgamma, float* dbeta, void* work,
                         void* stream) {
  return bn2d_bwd_impl(X2{x, nullptr}, 0, dy, N, C, H, W, gamma, beta, save_mean, save_invstd, hardtanh, pool, dx,
                       dgamma, dbeta, work, stream, true);
}

BNN_API int bnn_bn2d_bwd_q(const void* xq, const float* xbias, int32_t xfmt, const float* dy, int64_t N, int64_t C,
                           int64_t H, int64_t W, const float* gamma, const float* beta, const float* save_mean,
                           const float* save_invstd, int32_t hardtanh, int32_t pool, float* dx, float* dgamma,
                           float* dbeta, void* work, void* stream) {
  if (xfmt != 1 && xfmt != 2) {
    set_error("bnn_bn2d_bwd_q: xfmt must be 1 (int8) or 2 (int16)");
    return kErrInval;
  }
  return bn2d_bwd_impl(X2{xq, xbias}, xfmt, dy, N, C, H, W, gamma, beta, save_mean, save_invstd, hardtanh, pool, dx,
                       dgamma, dbeta, work, stream, true);
}

// The backward statistics only (no dx): dgamma, dbeta and sum g / sum g*xhat into sg / sgx (C
// floats each) -- for a consumer that forms dx itself (bnn_conv2d_bwd_filter_bn)
BNN_API int bnn_bn2d_bwd_stats_q(const void* xq, const float* xbias, int32_t xfmt, const float* dy, int64_t N,
                                 int64_t C, int64_t H, int64_t W, const float* gamma, const float* beta,
                                 const float* save_mean, const float* save_invstd, int32_t hardtanh, int32_t pool,
                                 float* dgamma, float* dbeta, float* sg, float* sgx, void* work, void* stream) {
  if ((xfmt != 1 && xfmt != 2) || !sg || !sgx) {
    set_error("bnn_bn2d_bwd_stats_q: xfmt must be 1 (int8) or 2 (int16); sg, sgx required");
    return kErrInval;
  }
  return bn2d_bwd_impl(X2{xq, xbias}, xfmt, dy, N, C, H, W, gamma, beta, save_mean, save_invstd, hardtanh, pool,
                       nullptr, dgamma, dbeta, work, stream, true, sg, sgx);
}

BNN_API int bnn_bn2d_bwd_eval(const float* x, const float* dy, int64_t N, int64_t C, int64_t H, int64_t W,
                              const float* gamma, const float* beta, const float* running_mean, const float* invstd,
                              int32_t hardtanh, int32_t pool, float* dx, float* dgamma, float* dbeta, void* work,
                              void* stream) {
  return bn2d_bwd_impl(X2{x, nullptr}, 0, dy, N, C, H, W, gamma, beta, running_mean, invstd, hardtanh, pool, dx,
                       dgamma, dbeta, work, stream, false);
}
