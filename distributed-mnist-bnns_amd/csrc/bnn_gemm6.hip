// fp32-operand GEMMs of the binarized layers on the block-scaled FP6 MFMA.
//
// The straight-through backward of BinarizeLinear (models/binarized_modules.py:80; autograd:
// dX = dY.W_b, dW = dY^T.X_b) and the first layer's forward (fp32 pixels x W_b) multiply an fp32
// operand by a ternary one.  Here the fp32 operand enters v_mfma_scale_f32_32x32x64_f8f6f4 as FOUR
// FP6 (e2m3) digit planes with one power-of-two scale per 32-element K-block (the instruction's
// own E8M0 block scales), the ternary operand as FP4 (e2m1, unit scale):
//
//   block b of row r (32 consecutive k):  e = exponent with max|x| in [2^(e-1), 2^e)
//   I = rint(x * 2^(19-e)), |I| <= 2^19, split into balanced base-32 digits
//   I = d0 + 32 d1 + 1024 d2 + 32768 d3,  d0..d2 in [-16, 15], d3 in [-16, 16]
//   plane j holds d_j / 8 (exact in e2m3: 0..15 in steps of 1/8 and 16/8 = 2.0) with block
//   scale 2^(e - 19 + 5j + 3), so the MFMA sums d_j * 2^(e-19+5j) * (+-1 or 0).
//
// All four planes of a k-block accumulate into ONE fp32 accumulator.  |x - I*2^(e-19)| <=
// 2^(e-20) <= max|x_block| * 2^-19, so the norm-wise relative error of a 32-element block is at
// most sqrt(32) * 2^-19 / ... <= 5.4e-6 (each block's norm is >= its max), ~1e-6 typical; the fp32
// accumulation over blocks rounds like an fp32 GEMM does (the reference's F.linear backward is
// one).  Cost: 4 FP6 MFMA passes at the FP4/FP6 rate (2x the int8 rate) = 2 int8-equivalent
// passes, against 3 for the int8 digit form (bnn_gemm.hip), with one accumulator instead of three.
//
// The residual plane (row operands of the dX GEMMs, whose fp32 precision the hidden BatchNorms' bias
// gradients need: they sum dX over the batch, where it nearly cancels -- tests/test_gpu_wide_step.py's
// calibration): three more bits of x as ONE FP4 (e2m1) plane, d = rint(x 2^(22-e)) - 8 I in [-4, 4]
// (bnn_fp6.h res4_code), scaled by 2^(e-21) (E8M0 byte = plane 0's - 5), a fifth MFMA pass into the
// same accumulator: |x - q| <= 2^(e-23) <= max|x_block| 2^-22.
//
// Operand layouts (K = padded reduction length, a multiple of 64; all rows 16-B aligned):
//   A digits "lo": [rows][K/32][64 B]  -- per block, 16 B per plane: dwords 0..3 of the plane's
//                                          6-dword MFMA operand (bits 0..127 of the 32 codes)
//   A digits "hi": [rows][K/32][32 B]  -- per block, 8 B per plane: dwords 4..5 (bits 128..191)
//   A scales:      [K/64][rows_pad][2] -- E8M0 byte of plane 0 (plane j adds 5j), per block
//   B ternary:     [rows][ldb bytes]   -- FP4 nibbles, element k in byte k/2 (low nibble even k)
//   A residual:    [rows][K/32][16 B]  -- per block, the 32 FP4 codes (element i at bits 4i); optional
// The MFMA operand map (checked by tools/probes/probe_fp6.hip on MI355X): lane l holds row l%32,
// k-block l/32 of the 64-k step, element j at bits 6j..6j+5; the lane's scale byte scales its 32.
#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstdio>

#include "bnn_fp6.h"

namespace bnn {
namespace {

// ------------------------------------------------------------------------------------------
// Row quantiser: x [M][K] (row stride ldx) -> lo, hi, scales; blocks beyond K are zero digits.
// 8 lanes per block (4 elements each: one 16-B load per lane), lane j < 4 of the group packs and
// writes plane j (lo 16 B + hi 8 B).  Grid: (rows, row blocks / 32); one wave = 8 blocks of a row.
__global__ __launch_bounds__(256) void quant6_rows_k(const float* __restrict__ x, int64_t M, int64_t K,
                                                     int64_t ldx, int64_t nblk, uint8_t* __restrict__ lo,
                                                     uint8_t* __restrict__ hi, uint8_t* __restrict__ sc,
                                                     int64_t sc_rows, int vec, uint8_t* __restrict__ res) {
  const int lane = threadIdx.x & 63, q = lane & 7;
  const int64_t row = blockIdx.x;
  const int64_t blk = ((int64_t)blockIdx.y * 4 + (threadIdx.x >> 6)) * 8 + (lane >> 3);
  if (blk >= nblk) return;   // whole 8-lane groups leave together
  const int64_t k0 = blk * QB + 4 * q;
  const float* xr = x + row * ldx;
  float v[4];
  if (vec && k0 + 4 <= K) {
    const float4 f = *reinterpret_cast<const float4*>(xr + k0);
    v[0] = f.x, v[1] = f.y, v[2] = f.z, v[3] = f.w;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (k0 + j < K) ? xr[k0 + j] : 0.f;
  }
  q6_block_store(v, lane, true, lo + (row * nblk + blk) * 64, hi + (row * nblk + blk) * 32,
                 sc + (blk >> 1) * sc_rows * 2 + row * 2 + (blk & 1), res ? res + (row * nblk + blk) * 16 : nullptr);
}

// ------------------------------------------------------------------------------------------
// Transposed column quantiser: x [M][N] -> the digits of x^T (rows n, k = m), blocks of 32
// consecutive m; plus per-256-row partial column sums (double) for the bias gradient
// dB = sum_B dY (binarized_modules.py:81-83).  Workgroup = 64 columns x 8 blocks (256 rows);
// thread (column t%64, block t/64) reads its block's 32 values column-wise (each wave reads 64
// consecutive columns of one row: 256 B) and writes the block's 96 digit bytes.
constexpr int QC_COLS = 64, QC_BLKS = 8;

__global__ __launch_bounds__(512) void quant6_cols_t_k(const float* __restrict__ x, int64_t M, int64_t N,
                                                       int64_t ldx, int64_t nblk, uint8_t* __restrict__ lo,
                                                       uint8_t* __restrict__ hi, uint8_t* __restrict__ sc,
                                                       int64_t sc_rows, double* __restrict__ part) {
  __shared__ double psum[QC_BLKS][QC_COLS];
  const int tc = threadIdx.x & (QC_COLS - 1), tb = threadIdx.x / QC_COLS;
  const int64_t n = (int64_t)blockIdx.x * QC_COLS + tc;
  const int64_t blk = (int64_t)blockIdx.y * QC_BLKS + tb;
  const int64_t m0 = blk * QB;
  float v[QB];
  float amax = 0.f;
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < QB; ++i) {
    const int64_t m = m0 + i;
    v[i] = (n < N && m < M) ? x[m * ldx + n] : 0.f;
    const float a = fabsf(v[i]);
    amax = (a == a) ? fmaxf(amax, a) : __builtin_inff();
    s += (double)v[i];
  }
  psum[tb][tc] = s;
  if (n < N && blk < nblk) {
    int shift;
    const int sbyte = block_scale(amax, &shift);
    uint32_t w[4][6];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 6; ++i) w[j][i] = 0;
#pragma unroll
    for (int i = 0; i < QB; ++i) {
      uint32_t cd[4];
      codes4(v[i], shift, cd);
      const int bit = 6 * i;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t c = cd[j];
        w[j][bit >> 5] |= c << (bit & 31);
        if ((bit & 31) > 26) w[j][(bit >> 5) + 1] |= c >> (32 - (bit & 31));
      }
    }
    uint8_t* lo_p = lo + (n * nblk + blk) * 64;
    uint8_t* hi_p = hi + (n * nblk + blk) * 32;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *reinterpret_cast<uint4*>(lo_p + 16 * j) = make_uint4(w[j][0], w[j][1], w[j][2], w[j][3]);
    *reinterpret_cast<uint4*>(hi_p) = make_uint4(w[0][4], w[0][5], w[1][4], w[1][5]);
    *reinterpret_cast<uint4*>(hi_p + 16) = make_uint4(w[2][4], w[2][5], w[3][4], w[3][5]);
    sc[(blk >> 1) * sc_rows * 2 + n * 2 + (blk & 1)] = (uint8_t)sbyte;
  }
  __syncthreads();
  if (part != nullptr && tb == 0 && n < N) {
    double t = 0.0;
#pragma unroll
    for (int b = 0; b < QC_BLKS; ++b) t += psum[b][tc];   // fixed order: deterministic
    part[(int64_t)blockIdx.y * N + n] = t;
  }
}

__global__ __launch_bounds__(256) void colsum_final_k(const double* __restrict__ part, int64_t R, int64_t N,
                                                      float* __restrict__ out) {
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  double s = 0.0;
#pragma unroll 8
  for (int64_t r = 0; r < R; ++r) s += part[r * N + n];
  out[n] = (float)s;
}

// ------------------------------------------------------------------------------------------
// FP4 panels: B [N][ldb] (row n = K/2 bytes of nibbles) -> [ceil(N/512)][K/64][512][32 B].  A GEMM
// stage reads 32 B of each of its BN rows per 64-k step: from row-major B that is one quarter of a
// 128-B line per row -- 4x the L2->L1 lines of the bytes used, 29 % of the FP6 GEMM's time
// (profiles/r03_fp6_staging_diag.log) -- from panels one contiguous BN x 32 B run.  Workgroup = 32
// rows x 4 k-steps (one 128-B line per source row, staged in LDS), written as 4 contiguous 1-KiB
// runs; the rows of the last panel beyond N are zeros.
constexpr int FP4_PANEL = 512;

__global__ __launch_bounds__(256) void fp4_panelize_k(const uint8_t* __restrict__ b, int64_t N, int64_t ldb,
                                                      int64_t nks, uint8_t* __restrict__ out) {
  __shared__ uint4 tile[32][8];
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.y * 32, ks0 = (int64_t)blockIdx.x * 4;
  {
    const int row = t >> 3, ch = t & 7;                 // 16-B chunk ch of the row's 128 B
    const int64_t n = r0 + row, ks = ks0 + (ch >> 1);
    uint4 v = make_uint4(0, 0, 0, 0);
    if (n < N && ks < nks) v = *reinterpret_cast<const uint4*>(b + n * ldb + ks * 32 + (ch & 1) * 16);
    tile[row][ch] = v;
  }
  __syncthreads();
  const int q = t >> 6, row = (t & 63) >> 1, half = t & 1;   // k-step q: 32 rows x 32 B = 1 KiB
  const int64_t ks = ks0 + q, n = r0 + row;
  if (ks < nks)
    *reinterpret_cast<uint4*>(out + ((n / FP4_PANEL) * nks + ks) * (FP4_PANEL * 32) + (n % FP4_PANEL) * 32 + half * 16) =
        tile[row][2 * q + half];
}

// ------------------------------------------------------------------------------------------
// GEMM: C[M][N] = sum_k A[m][k] B[n][k] (+ bias[n]); A = FP6 digits (lo, hi, scales), B = FP4.
struct Gemm6Params {
  const uint8_t* alo;   // [M][K/32][64]
  const uint8_t* ahi;   // [M][K/32][32]
  const uint8_t* asc;   // [K/64][asc_rows][2]
  const uint8_t* b;     // [N][ldb], or (b_panel) FP4 panels [N/512][K/64][512][32 B] (bnn_fp4_panelize)
  int64_t ldb, asc_rows;
  const float* bias;
  float* C;
  int64_t ldc;
  int M, N, K;
  int gm, gn;
  int group;   // raster group rows (tile6_of)
  // split-K (grids too small to fill the chip): workgroup bid computes k-steps
  // [split * kps, min((split + 1) * kps, K / 64)) of tile bid / ksplit, split = bid % ksplit, and
  // writes its fp32 partial (no bias) to part[split][M][N]; gemm6_splitk_sum_k folds the splits
  int ksplit, kps;
  float* part;
  int64_t bks;   // > 0: B in the panel layout with bks 64-k steps per panel (>= K / 64): every
                 // stage's B piece is one contiguous run of BN x 32 B
  // BatchNorm-backward statistics of C in the epilogue (bnn_gemm_fp6_bnstats; mode 0 = off): C is the
  // gradient dy reaching a training-mode BatchNorm(+Hardtanh) whose input x [M][N] (fp32, or int16
  // + xbias) is read here; per 128-row tile row tm and column n the epilogue writes
  // part[0][tm][n] = sum g, part[1] = sum g*xhat (mode 2: part[2] = max|g|, part[3] = max|xhat|),
  // g = dy masked by -1 < BN(x) < 1 -- bn_reduce_k's MODE 1 / 2 sums, without its pass over x and dy
  struct Bn {
    const void* x;
    const float* xbias;
    const float *mean, *mean_lo, *invstd, *gamma, *beta;
    float* part;
    int z16, hardtanh, mode;
  } bn;
  const uint8_t* ares = nullptr;   // the residual FP4 plane [M][K/32][16 B] (instances with RES = 1)
  // first-round stagger (bnn_gemm_fp6_set_half): workgroups stg_lo <= bid < stg_hi wait stg_ticks of
  // the 100 MHz realtime clock before their k loop, so the two workgroups sharing a CU run half a
  // tile apart and one's epilogue stores drain while the other's MFMAs run
  int stg_lo = 0, stg_hi = 0;
  int64_t stg_ticks = 0;
};

__device__ __forceinline__ void glds16_6(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// The same 16-B LDS-DMA in its saddr form: wave-uniform 64-bit base in SGPRs + per-lane 32-bit
// offset, LDS destination through M0 (as bnn_gemm.hip's glds16_s).
__device__ __forceinline__ void glds16_6s(const void* sbase, uint32_t voff, void* l) {
  const uint32_t la = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(l);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
               :
               : "s"(la), "v"(voff), "s"(sbase)
               : "memory", "m0");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt6() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

__device__ __forceinline__ void barrier6() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Bijective XCD remap + grouped raster (as bnn_gemm.hip's tile_of).
// G = tile rows per raster group: an XCD's ~32 co-resident workgroups then cover about G rows x
// 32/G columns, re-reading each A panel (3.1 B/element) once per 32/G columns and each B panel
// (0.5 B/element) once per G rows; 4 suits dX (K = 8192), 8 the long-K dW (tools/gpu_fp6_group.sh).
__device__ __forceinline__ void tile6_of(int bid, int gm, int gn, int G, int& tm, int& tn) {
  const int nwg = gm * gn;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int per_group = G * gn;
  const int g = L / per_group, first = g * G;
  const int gs = min(gm - first, G);
  const int in = L - g * per_group;
  tm = first + in % gs;
  tn = in / gs;
}

// LDS stage (BK = 64 = one MFMA k-step, 2 scale blocks):
//   A lo : BM rows x 128 B  (block 0: planes 0-3, block 1: planes 0-3), 16-B chunk c stored at
//          chunk c ^ ((row >> 1) & 7)
//   A hi : BM rows x  64 B  (block 0: planes 01, 23; block 1: ...), chunk c at c ^ ((row >> 2) & 3)
//   A sc : BM x 2 B        (row-major, plane-0 bytes of blocks 0, 1)
//   B    : BN rows x  32 B  (the 64 FP4 codes), chunk c at c ^ ((row >> 3) & 1)
// DIAG (timing-only builds, wrong results): 1 = no global->LDS staging, 2 = no LDS fragment reads,
// 3 / 4 = the MFMA stream alone (fragments read once) with / without the per-step barrier, 5 = B
// staged from contiguous per-k-step panels (as if B were stored [N/BN][K/64][BN][32 B]), 6 = 5 +
// A hi likewise ([M/BM][K/64][BM][64 B]): what whole-line staging loads would gain.
// OCC = waves per SIMD the register allocation must allow (2: one 512-thread workgroup per CU;
// 4: two, whose independent barriers let one's LDS-read phase overlap the other's MFMAs).
// PP = 1 (WM = 2, STAGES = 3): software-pipelined k loop.  Each k-step's two A tiles are split
// around a mid-step barrier: the MFMAs of tile 0 run while tile 1's fragments are read; then the
// barrier retires the NEXT stage and its B and tile-0 fragments are read into the second register
// set while tile 1's MFMAs run -- no k-step starts with the matrix pipe waiting on LDS.  All three
// ring slots are in flight: stage kt+1 is waited for at step kt with stage kt+2 still landing
// (two steps of cover), and stage kt+3 refills the slot stage kt has just left.
// RES = 1: A carries the residual FP4 plane (header): BM x 32 B more per stage (block c of row i at
// chunk c ^ ((i >> 3) & 1), as B's), a fifth MFMA per A fragment; the plain two-stage loop only.
template <int WAVES_M, int WAVES_N, int WM, int WN, int STAGES, int DIAG = 0, int OCC = 2, int PP = 0,
          int BNS = 0, int RES = 0>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N, OCC) void gemm_fp6_k(Gemm6Params p) {
  static_assert(PP != 1 || (WM == 2 && STAGES == 3 && DIAG == 0), "pipelined form 1: 2 tile rows, 3 stages");
  static_assert(PP != 2 || (WM == 1 && WN % 2 == 0 && STAGES == 3 && DIAG == 0),
                "pipelined form 2: 1 tile row, an even number of tile columns, 3 stages");
  static_assert(PP != 3 || (WAVES_M == 2 && WM == 2 && STAGES == 3 && DIAG == 0),
                "ping-pong form: 2 wave rows (the two groups), 2 tile rows, 3 stages");
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int BM = WAVES_M * WM * 32, BN = WAVES_N * WN * 32;
  constexpr int LO_ST = BM * 128, HI_ST = BM * 64, SC_ST = BM * 2, B_ST = BN * 32;
  constexpr int SC_PAD = (SC_ST + 1023) / 1024 * 1024;
  constexpr int R_ST = RES ? BM * 32 : 0;
  constexpr int ST = LO_ST + HI_ST + SC_PAD + B_ST + R_ST;
  static_assert(!RES || (PP == 0 && DIAG == 0 && STAGES == 2), "the residual plane: the plain two-stage loop");
  constexpr int I_LO = LO_ST / 1024, I_HI = HI_ST / 1024, I_SC = SC_PAD / 1024, I_B = B_ST / 1024;
  constexpr int PER_WAVE = (I_LO + I_HI + I_B) / NW + 1;   // wave 0 also issues the scale piece
  __shared__ __attribute__((aligned(16))) char smem[STAGES * ST];

  const int lane = threadIdx.x & 63, wave = wave_id();
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  if (p.stg_ticks > 0 && (int)blockIdx.x >= p.stg_lo && (int)blockIdx.x < p.stg_hi) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) < p.stg_ticks) __builtin_amdgcn_s_sleep(32);
  }
  int tm, tn;
  const int split = p.ksplit > 1 ? (int)(blockIdx.x % p.ksplit) : 0;
  tile6_of(p.ksplit > 1 ? (int)(blockIdx.x / p.ksplit) : (int)blockIdx.x, p.gm, p.gn, p.group, tm, tn);
  const int64_t nblk = p.K / QB;
  const int ks0 = split * p.kps;                          // this workgroup's first k-step
  const int nk = min(p.K / 64 - ks0, p.kps);
  // split-K: this split's partial, row pitch N, no bias (added once by the fold)
  float* const Cout = p.ksplit > 1 ? p.part + (int64_t)split * p.M * p.N : p.C;
  const int64_t ldo = p.ksplit > 1 ? p.N : p.ldc;
  const float* const bias = p.ksplit > 1 ? nullptr : p.bias;
  const int m0 = tm * BM, n0 = tn * BN;

  // One stage = I_LO + I_HI + I_SC + I_B LDS-DMA pieces of 1 KiB (64 lanes x 16 B): lo 8 rows per
  // piece, hi 16 rows, scales 512 rows of 2-B entries (only this tile's BM rows are loaded), B 32
  // rows.  Every wave issues the same compile-time number of lo / hi / B pieces (wave 0 also the
  // scale piece); each piece's per-lane source offset (row clamped to the last valid row -- its
  // results are never stored -- and the XOR-swizzled 16-B chunk: the LDS image stays linear) is
  // k-invariant and computed once, so a stage is a wave-uniform base advance + the saddr-form DMA.
  static_assert(I_LO % NW == 0 && I_HI % NW == 0 && I_B % NW == 0 && I_SC == 1, "piece split");
  constexpr int P_LO = I_LO / NW, P_HI = I_HI / NW, P_B = I_B / NW;
  uint32_t off_lo[P_LO], off_hi[P_HI], off_b[P_B];
#pragma unroll
  for (int ii = 0; ii < P_LO; ++ii) {
    const int i = wave + ii * NW;
    const int lrow = i * 8 + (lane >> 3), c = lane & 7;
    off_lo[ii] = (uint32_t)min(lrow, p.M - 1 - m0) * (uint32_t)(nblk * 64) + 16u * (uint32_t)(c ^ ((lrow >> 1) & 7));
  }
#pragma unroll
  for (int ii = 0; ii < P_HI; ++ii) {
    const int i = wave + ii * NW;
    const int lrow = i * 16 + (lane >> 2), c = lane & 3;
    off_hi[ii] = DIAG == 6 ? (uint32_t)lrow * 64u + 16u * (uint32_t)(c ^ ((lrow >> 2) & 3))
                           : (uint32_t)min(lrow, p.M - 1 - m0) * (uint32_t)(nblk * 32) + 16u * (uint32_t)(c ^ ((lrow >> 2) & 3));
  }
#pragma unroll
  for (int ii = 0; ii < P_B; ++ii) {
    const int i = wave + ii * NW;
    const int lrow = i * 32 + (lane >> 1), c = lane & 1;
    off_b[ii] = (DIAG >= 5 || p.bks > 0) ? (uint32_t)lrow * 32u + 16u * (uint32_t)(c ^ ((lrow >> 3) & 1))
                                         : (uint32_t)min(lrow, p.N - 1 - n0) * (uint32_t)p.ldb + 16u * (uint32_t)(c ^ ((lrow >> 3) & 1));
  }
  const uint8_t* lo_base = p.alo + (int64_t)m0 * nblk * 64 + (int64_t)ks0 * 128;
  const uint8_t* hi_base = p.ahi + (int64_t)m0 * nblk * 32 + (int64_t)ks0 * 64;
  const uint8_t* sc_base = p.asc + (int64_t)m0 * 2 + (int64_t)ks0 * p.asc_rows * 2;
  // panel layout: tile column n0 lies in panel n0 / 512 at row n0 % 512 (BN divides 512); rows
  // beyond N are the panel's padding, staged unclamped: zero in every producer's buffer
  // (bnn_fp4_panelize writes them, functional._qt_buffer zeroes them for the packing kernels) and
  // in any case only ever multiplied into output columns >= N, which are neither stored nor reduced
  const uint8_t* b_base = p.bks > 0 ? p.b + ((int64_t)(n0 / FP4_PANEL) * p.bks + ks0) * (FP4_PANEL * 32) + (n0 % FP4_PANEL) * 32
                                    : p.b + (int64_t)n0 * p.ldb + (int64_t)ks0 * 32;
  const int64_t b_step = (DIAG >= 5) ? BN * 32 : (p.bks > 0 ? FP4_PANEL * 32 : 32);
  // the residual plane: I_R pieces of 32 rows x 32 B, one per wave (waves >= I_R issue none; the
  // two-stage loop waits for every piece, so the per-wave counts need not match)
  constexpr int I_R = R_ST / 1024, P_R = (I_R + NW - 1) / NW;
  uint32_t off_r[P_R > 0 ? P_R : 1];
#pragma unroll
  for (int ii = 0; ii < P_R; ++ii) {
    const int lrow = (wave + ii * NW) * 32 + (lane >> 1), c = lane & 1;
    off_r[ii] = (uint32_t)min(lrow, p.M - 1 - m0) * (uint32_t)(nblk * 16) + 16u * (uint32_t)(c ^ ((lrow >> 3) & 1));
  }
  const uint8_t* r_base = RES ? p.ares + (int64_t)m0 * nblk * 16 + (int64_t)ks0 * 32 : nullptr;
  auto stage = [&](int kt, int buf) __attribute__((always_inline)) {
    if constexpr (DIAG == 1) return;
    char* base = smem + buf * ST;
#pragma unroll
    for (int ii = 0; ii < P_LO; ++ii)
      glds16_6s(lo_base + (int64_t)kt * 128, off_lo[ii], base + (wave + ii * NW) * 1024);
#pragma unroll
    for (int ii = 0; ii < P_HI; ++ii)
      glds16_6s(hi_base + (int64_t)kt * (DIAG == 6 ? BM * 64 : 64), off_hi[ii], base + LO_ST + (wave + ii * NW) * 1024);
#pragma unroll
    for (int ii = 0; ii < P_B; ++ii)
      glds16_6s(b_base + (int64_t)kt * b_step, off_b[ii], base + LO_ST + HI_ST + SC_PAD + (wave + ii * NW) * 1024);
    if (wave == 0)   // a whole 1-KiB piece (512 rows): the scale array has 512 rows of tail padding
      glds16_6(sc_base + (int64_t)kt * p.asc_rows * 2 + lane * 16, base + LO_ST + HI_ST);
    if constexpr (RES) {
#pragma unroll
      for (int ii = 0; ii < P_R; ++ii)
        if (wave + ii * NW < I_R)
          glds16_6s(r_base + (int64_t)kt * 32, off_r[ii], base + LO_ST + HI_ST + SC_PAD + B_ST + (wave + ii * NW) * 1024);
    }
  };
  // piece i (compile-time after unrolling) of stage(kt, buf): lo, hi, B, then wave 0's scale piece
  constexpr int NPIECE = P_LO + P_HI + P_B + 1;
  auto stage_piece = [&](int kt, int buf, int i) __attribute__((always_inline)) {
    char* base = smem + buf * ST;
    if (i < P_LO) {
      glds16_6s(lo_base + (int64_t)kt * 128, off_lo[i], base + (wave + i * NW) * 1024);
    } else if (i < P_LO + P_HI) {
      const int ii = i - P_LO;
      glds16_6s(hi_base + (int64_t)kt * 64, off_hi[ii], base + LO_ST + (wave + ii * NW) * 1024);
    } else if (i < P_LO + P_HI + P_B) {
      const int ii = i - P_LO - P_HI;
      glds16_6s(b_base + (int64_t)kt * b_step, off_b[ii], base + LO_ST + HI_ST + SC_PAD + (wave + ii * NW) * 1024);
    } else if (wave == 0) {   // asm form: the compiler must not order LDS reads behind it
      glds16_6s(sc_base + (int64_t)kt * p.asc_rows * 2, (uint32_t)lane * 16u, base + LO_ST + HI_ST);
    }
  };

  v16f acc[WM][WN];
#pragma unroll
  for (int t = 0; t < WM; ++t)
#pragma unroll
    for (int u = 0; u < WN; ++u) acc[t][u] = v16f{0};

  const int r = lane & 31, h = lane >> 5;
  // pieces this wave issues per stage (wave-uniform): the counted waits keep later stages in
  // flight while retiring one
  const int mine = wave == 0 ? PER_WAVE : PER_WAVE - 1;

  struct AFrag {      // the 4 planes' 6-dword MFMA operands (elements 6, 7 unused) + scale byte
    v8i a0, a1, a2, a3;
    int sb;
    v4i rr;           // RES: the residual plane's 4 dwords
  };
  auto read_a = [&](const char* base, int t, AFrag& f) __attribute__((always_inline)) {
    const int lrow = wm * WM * 32 + t * 32 + r;
    const char* sLo = base;
    const char* sHi = base + LO_ST;
    const uint8_t* sSc = reinterpret_cast<const uint8_t*>(base + LO_ST + HI_ST);
    const int sw = (lrow >> 1) & 7;
    const v4i l0 = *reinterpret_cast<const v4i*>(sLo + lrow * 128 + 16 * ((h * 4 + 0) ^ sw));
    const v4i l1 = *reinterpret_cast<const v4i*>(sLo + lrow * 128 + 16 * ((h * 4 + 1) ^ sw));
    const v4i l2 = *reinterpret_cast<const v4i*>(sLo + lrow * 128 + 16 * ((h * 4 + 2) ^ sw));
    const v4i l3 = *reinterpret_cast<const v4i*>(sLo + lrow * 128 + 16 * ((h * 4 + 3) ^ sw));
    const v4i h01 = *reinterpret_cast<const v4i*>(sHi + lrow * 64 + 16 * ((h * 2) ^ ((lrow >> 2) & 3)));
    const v4i h23 = *reinterpret_cast<const v4i*>(sHi + lrow * 64 + 16 * ((h * 2 + 1) ^ ((lrow >> 2) & 3)));
    f.a0 = v8i{l0.x, l0.y, l0.z, l0.w, h01.x, h01.y, 0, 0};
    f.a1 = v8i{l1.x, l1.y, l1.z, l1.w, h01.z, h01.w, 0, 0};
    f.a2 = v8i{l2.x, l2.y, l2.z, l2.w, h23.x, h23.y, 0, 0};
    f.a3 = v8i{l3.x, l3.y, l3.z, l3.w, h23.z, h23.w, 0, 0};
    f.sb = sSc[lrow * 2 + h];
    if constexpr (RES)
      f.rr = *reinterpret_cast<const v4i*>(base + LO_ST + HI_ST + SC_PAD + B_ST + lrow * 32 + 16 * (h ^ ((lrow >> 3) & 1)));
  };
  // B fragments: row n, 16 B = k-block h
  auto read_b = [&](const char* base, v4i (&bf)[WN]) __attribute__((always_inline)) {
    const char* sB = base + LO_ST + HI_ST + SC_PAD;
#pragma unroll
    for (int u = 0; u < WN; ++u) {
      const int lrow = wn * WN * 32 + u * 32 + r;
      bf[u] = *reinterpret_cast<const v4i*>(sB + lrow * 32 + 16 * (h ^ ((lrow >> 3) & 1)));
    }
  };
  // MFMAs of one A fragment against B fragments u0 .. u1-1
  auto mma_cols = [&](const AFrag& f, const v4i (&bf)[WN], v16f (&ac)[WN], int u0, int u1) __attribute__((always_inline)) {
    const v8i a0 = f.a0, a1 = f.a1, a2 = f.a2, a3 = f.a3;
    const int sb = f.sb;
    const int s0 = sb, s1 = sb == 255 ? 255 : sb + 5, s2 = sb == 255 ? 255 : sb + 10, s3 = sb == 255 ? 255 : sb + 15;
#pragma unroll
    for (int u = 0; u < WN; ++u) {
      if (u < u0 || u >= u1) continue;
      const v8i bb = {bf[u].x, bf[u].y, bf[u].z, bf[u].w, 0, 0, 0, 0};
      ac[u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a3, bb, ac[u], 2, 4, 0, s3, 0, 127);
      ac[u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a2, bb, ac[u], 2, 4, 0, s2, 0, 127);
      ac[u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a1, bb, ac[u], 2, 4, 0, s1, 0, 127);
      ac[u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a0, bb, ac[u], 2, 4, 0, s0, 0, 127);
    }
  };
  // B fragments u0 .. u1-1
  auto read_b_cols = [&](const char* base, v4i (&bf)[WN], int u0, int u1) __attribute__((always_inline)) {
    const char* sB = base + LO_ST + HI_ST + SC_PAD;
#pragma unroll
    for (int u = 0; u < WN; ++u) {
      if (u < u0 || u >= u1) continue;
      const int lrow = wn * WN * 32 + u * 32 + r;
      bf[u] = *reinterpret_cast<const v4i*>(sB + lrow * 32 + 16 * (h ^ ((lrow >> 3) & 1)));
    }
  };
  auto mma_tile = [&](const AFrag& f, const v4i (&bf)[WN], v16f (&ac)[WN]) __attribute__((always_inline)) {
    const v8i a0 = f.a0, a1 = f.a1, a2 = f.a2, a3 = f.a3;
    // a NaN block (255) stays NaN in every plane; otherwise plane j scale = sb + 5j (<= 254)
    const int sb = f.sb;
    const int s0 = sb, s1 = sb == 255 ? 255 : sb + 5, s2 = sb == 255 ? 255 : sb + 10, s3 = sb == 255 ? 255 : sb + 15;
#pragma unroll
    for (int u = 0; u < WN; ++u) {
      const v8i bb = {bf[u].x, bf[u].y, bf[u].z, bf[u].w, 0, 0, 0, 0};
      ac[u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a3, bb, ac[u], 2, 4, 0, s3, 0, 127);
      ac[u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a2, bb, ac[u], 2, 4, 0, s2, 0, 127);
      ac[u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a1, bb, ac[u], 2, 4, 0, s1, 0, 127);
      ac[u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a0, bb, ac[u], 2, 4, 0, s0, 0, 127);
      if constexpr (RES) {   // the residual FP4 plane at plane 0's scale / 32 (blocks below 2^-106: zeros)
        const int sr = sb == 255 ? 255 : (sb >= 5 ? sb - 5 : 0);
        const v8i ar = {f.rr.x, f.rr.y, f.rr.z, f.rr.w, 0, 0, 0, 0};
        ac[u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ar, bb, ac[u], 4, 4, 0, sr, 0, 127);
      }
    }
  };

  if constexpr (PP == 3) {
    // Ping-pong (cdna_hip_programming.md §5, the 8-phase template's stagger): wave row g = wm is a
    // group of 4 waves, one per SIMD; group 1 runs one barrier behind group 0, so between two
    // barriers one group issues its 16 MFMAs while the other issues its fragment reads (and LDS-DMA
    // pieces) -- every SIMD's matrix pipe is fed by one wave while its partner reads.  Per k-step a
    // wave runs two phases (A tile 0 with the B fragments, then A tile 1), each {reads, wait for
    // them, barrier X, MFMAs, barrier Y}.  Reads are waited for BEFORE X, so a slot is free for
    // the DMA one barrier later; stage kt+2 is issued at k-step kt's phase 0 into the slot of
    // stage kt-1 (read by both groups two or more barriers earlier); every wave's stage kt+1
    // pieces are waited for before its phase-1 X barrier, which precedes all reads of stage kt+1.
    // wave w runs on SIMD w % 4 (grouping by wave parity instead put both of a SIMD's waves in one
    // group and ran 28% slower): the wave rows are the groups
    const int grp = wm;
    auto bar = [&]() __attribute__((always_inline)) { barrier6(); };
    auto mma_tile_pl = [&](const AFrag& f, const v4i (&bf)[WN], v16f (&ac)[WN]) __attribute__((always_inline)) {
      const int sb = f.sb;
      const v8i av[4] = {f.a0, f.a1, f.a2, f.a3};
#pragma unroll
      for (int j = 3; j >= 0; --j) {
        const int sj = sb == 255 ? 255 : sb + 5 * j;
#pragma unroll
        for (int u = 0; u < WN; ++u) {
          const v8i bb = {bf[u].x, bf[u].y, bf[u].z, bf[u].w, 0, 0, 0, 0};
          ac[u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av[j], bb, ac[u], 2, 4, 0, sj, 0, 127);
        }
      }
    };
    auto buf_of = [&](int kt) __attribute__((always_inline)) { return smem + (kt % STAGES) * ST; };
    if (0 < nk) stage(0, 0);
    if (1 < nk) stage(1, 1);
    if (nk >= 2) {
      if (mine == PER_WAVE) wait_vmcnt6<PER_WAVE>(); else wait_vmcnt6<PER_WAVE - 1>();
    } else {
      wait_vmcnt6<0>();
    }
    bar();
    if (grp == 1) bar();    // the stagger
    v4i bf[WN];
    AFrag fa;
    for (int kt = 0; kt < nk; ++kt) {
      // phase 0: A tile 0 + B
      if (kt + 2 < nk) stage(kt + 2, (kt + 2) % STAGES);
      read_b(buf_of(kt), bf);
      read_a(buf_of(kt), 0, fa);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      bar();
      __builtin_amdgcn_s_setprio(1);
      mma_tile_pl(fa, bf, acc[0]);
      __builtin_amdgcn_s_setprio(0);
      bar();
      // phase 1: A tile 1 (same B)
      read_a(buf_of(kt), 1, fa);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (kt + 2 < nk) {     // stage kt+1 landed; stage kt+2 may still be in flight
        if (mine == PER_WAVE) wait_vmcnt6<PER_WAVE>(); else wait_vmcnt6<PER_WAVE - 1>();
      } else {
        wait_vmcnt6<0>();
      }
      bar();
      __builtin_amdgcn_s_setprio(1);
      mma_tile_pl(fa, bf, acc[1]);
      __builtin_amdgcn_s_setprio(0);
      bar();
    }
    if (grp == 0) bar();    // equal barrier counts: group 1 ran one extra at the start
  } else if constexpr (PP == 2) {
    // form 2: one A fragment per k-step; its MFMAs against B columns [0, WN/2) run while the
    // columns [WN/2, WN) are read, then the barrier retires the next stage and its A fragment and
    // first-half B columns are read while the second-half MFMAs run
    constexpr int HN = WN / 2;
    auto buf_of = [&](int kt) __attribute__((always_inline)) { return smem + (kt % STAGES) * ST; };
#pragma unroll
    for (int s = 0; s < STAGES; ++s)
      if (s < nk) stage(s, s);
    if (nk >= 3) {
      if (mine == PER_WAVE) wait_vmcnt6<2 * PER_WAVE>(); else wait_vmcnt6<2 * (PER_WAVE - 1)>();
    } else if (nk == 2) {
      if (mine == PER_WAVE) wait_vmcnt6<PER_WAVE>(); else wait_vmcnt6<PER_WAVE - 1>();
    } else {
      wait_vmcnt6<0>();
    }
    barrier6();
    v4i b0[WN], b1[WN];
    AFrag f0, f1;
    read_b_cols(buf_of(0), b0, 0, HN);
    read_a(buf_of(0), 0, f0);
#define BNN_FP6_STEP2(KT, BC, FC, BN, FN)                                                             \
  {                                                                                                  \
    read_b_cols(buf_of(KT), BC, HN, WN);                                                             \
    mma_cols(FC, BC, acc[0], 0, HN);                                                                 \
    if ((KT) + 1 < nk) {                                                                             \
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                             \
      if ((KT) + 2 < nk) {                                                                           \
        if (mine == PER_WAVE) wait_vmcnt6<PER_WAVE>(); else wait_vmcnt6<PER_WAVE - 1>();             \
      } else {                                                                                       \
        wait_vmcnt6<0>();                                                                            \
      }                                                                                              \
      barrier6();                                                                                    \
      if ((KT) + 3 < nk) stage((KT) + 3, ((KT) + 3) % STAGES);                                       \
      read_b_cols(buf_of((KT) + 1), BN, 0, HN);                                                      \
      read_a(buf_of((KT) + 1), 0, FN);                                                               \
    }                                                                                                \
    mma_cols(FC, BC, acc[0], HN, WN);                                                                \
  }
    for (int kt = 0; kt < nk; kt += 2) {
      BNN_FP6_STEP2(kt, b0, f0, b1, f1)
      if (kt + 1 < nk) BNN_FP6_STEP2(kt + 1, b1, f1, b0, f0)
    }
#undef BNN_FP6_STEP2
  } else if constexpr (PP == 1) {
    auto buf_of = [&](int kt) __attribute__((always_inline)) { return smem + (kt % STAGES) * ST; };
#pragma unroll
    for (int s = 0; s < STAGES; ++s)
      if (s < nk) stage(s, s);
    // stage 0 ready, stages 1 and 2 may still be landing
    if (nk >= 3) {
      if (mine == PER_WAVE) wait_vmcnt6<2 * PER_WAVE>(); else wait_vmcnt6<2 * (PER_WAVE - 1)>();
    } else if (nk == 2) {
      if (mine == PER_WAVE) wait_vmcnt6<PER_WAVE>(); else wait_vmcnt6<PER_WAVE - 1>();
    } else {
      wait_vmcnt6<0>();
    }
    barrier6();
    v4i b0[WN], b1[WN];
    AFrag f0, f1;
    read_b(buf_of(0), b0);
    read_a(buf_of(0), 0, f0);
    // one k-step (written out twice so each register set keeps a fixed name): (BC, FC) hold this
    // step's B and tile-0 fragments, (BN, FN) receive the next step's
#define BNN_FP6_STEP(KT, BC, FC, BN, FN)                                                              \
  {                                                                                                  \
    AFrag ft;                                                                                        \
    read_a(buf_of(KT), 1, ft);                                                                       \
    mma_tile(FC, BC, acc[0]);                                                                        \
    if ((KT) + 1 < nk) {                                                                             \
      /* tile 1's reads of this slot are complete before any wave may refill it */                   \
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                             \
      if ((KT) + 2 < nk) {                                                                           \
        if (mine == PER_WAVE) wait_vmcnt6<PER_WAVE>(); else wait_vmcnt6<PER_WAVE - 1>();             \
      } else {                                                                                       \
        wait_vmcnt6<0>();                                                                            \
      }                                                                                              \
      barrier6();                                                                                    \
      if ((KT) + 3 < nk) stage((KT) + 3, ((KT) + 3) % STAGES);                                       \
      read_b(buf_of((KT) + 1), BN);                                                                  \
      read_a(buf_of((KT) + 1), 0, FN);                                                               \
    }                                                                                                \
    mma_tile(ft, BC, acc[1]);                                                                        \
  }
    for (int kt = 0; kt < nk; kt += 2) {
      BNN_FP6_STEP(kt, b0, f0, b1, f1)
      if (kt + 1 < nk) BNN_FP6_STEP(kt + 1, b1, f1, b0, f0)
    }
#undef BNN_FP6_STEP
  } else if constexpr (PP == 4) {
    // Interleaved form (2 stages): after the barrier each wave reads ALL of this step's fragments
    // (B, A tile 0, A tile 1) at once -- tile 1's arrive while tile 0's MFMAs run -- and issues the
    // next stage's LDS-DMA pieces one at a time between its MFMA column groups (4 MFMAs each), so
    // neither the reads nor the DMA issue sit between the barrier and the first MFMA of the step
    // (the plain loop issues every piece, then the reads, then waits for them all).
    static_assert((STAGES == 2 || STAGES == 3) && WM == 2 && DIAG == 0 && NPIECE <= 9,
                  "interleaved form: 2 or 3 stages, 2 tile rows");
    // a tile's fragment as loaded: the 4 planes' lo chunks, the 2 hi chunks, the scale byte
    v4i al[2][4], ah[2][2];
    int asb[2];
    auto read_raw = [&](const char* base, int t) __attribute__((always_inline)) {
      const int lrow = wm * WM * 32 + t * 32 + r;
      const char* sLo = base + lrow * 128;
      const char* sHi = base + LO_ST + lrow * 64;
      const int sw = (lrow >> 1) & 7, sh = (lrow >> 2) & 3;
#pragma unroll
      for (int q = 0; q < 4; ++q) al[t][q] = *reinterpret_cast<const v4i*>(sLo + 16 * ((h * 4 + q) ^ sw));
#pragma unroll
      for (int q = 0; q < 2; ++q) ah[t][q] = *reinterpret_cast<const v4i*>(sHi + 16 * ((h * 2 + q) ^ sh));
    };
    // both tiles' scale bytes: read first, so the scale arithmetic the compiler places early waits
    // only for them, not for the operand reads behind them
    auto read_sb = [&](const char* base) __attribute__((always_inline)) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
        asb[t] = reinterpret_cast<const uint8_t*>(base + LO_ST + HI_ST)[(wm * WM * 32 + t * 32 + r) * 2 + h];
    };
    // STAGES - 1 stages ahead; every step issues one stage (near the end a re-load of the last one
    // into a slot nobody reads): no branch between the MFMA groups -- a conditional piece let the
    // compiler sink every MFMA below it -- and a constant count of pieces in flight
    if (nk > 0) {
      stage(0, 0);
      if constexpr (STAGES == 3) stage(min(1, nk - 1), 1);
    }
    for (int kt = 0; kt < nk; ++kt) {
      if constexpr (STAGES == 3) {   // stage kt landed; stage kt + 1 may still be in flight
        if (mine == PER_WAVE) wait_vmcnt6<PER_WAVE>(); else wait_vmcnt6<PER_WAVE - 1>();
      } else {
        wait_vmcnt6<0>();
      }
      barrier6();
      const char* base = smem + (kt % STAGES) * ST;
      const int kn = min(kt + STAGES - 1, nk - 1);
      const int nb = (kt + STAGES - 1) % STAGES;
      if (wave == 0) stage_piece(kn, nb, NPIECE - 1);   // the scale piece (a branch: before the block)
      v4i bf[WN];
      read_sb(base);
      __builtin_amdgcn_sched_barrier(0);
      read_b(base, bf);
      read_raw(base, 0);
      __builtin_amdgcn_sched_barrier(0);
      read_raw(base, 1);
      // group g = one plane of one tile against the WN columns (independent accumulators)
      auto mma_plane = [&](int t, int j, v16f (&ac)[WN]) __attribute__((always_inline)) {
        const v4i l = al[t][j], hh = ah[t][j >> 1];
        const v8i a = (j & 1) ? v8i{l.x, l.y, l.z, l.w, hh.z, hh.w, 0, 0} : v8i{l.x, l.y, l.z, l.w, hh.x, hh.y, 0, 0};
        const int sj = asb[t] == 255 ? 255 : asb[t] + 5 * j;
#pragma unroll
        for (int u = 0; u < WN; ++u) {
          const v8i bb = {bf[u].x, bf[u].y, bf[u].z, bf[u].w, 0, 0, 0, 0};
          ac[u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, bb, ac[u], 2, 4, 0, sj, 0, 127);
        }
      };
#pragma unroll
      for (int g = 0; g < 8; ++g) {           // tile g / 4, plane 3 - g % 4 (mma_tile's order)
        __builtin_amdgcn_sched_barrier(0);
        if (g < 4) mma_plane(0, 3 - g, acc[0]);
        else mma_plane(1, 7 - g, acc[1]);
        __builtin_amdgcn_sched_barrier(0);
        if (g < NPIECE - 1) stage_piece(kn, nb, g);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  } else if constexpr (DIAG == 3 || DIAG == 4) {
    // timing-only: fragments read once from stage 0 and reused by every k-step -- the MFMA
    // stream alone (3: with the per-k-step barrier, 4: without)
    stage(0, 0);
    wait_vmcnt6<0>();
    barrier6();
    v4i bf[WN];
    AFrag fr[WM];
    read_b(smem, bf);
#pragma unroll
    for (int t = 0; t < WM; ++t) read_a(smem, t, fr[t]);
    for (int kt = 0; kt < nk; ++kt) {
      if constexpr (DIAG == 3) barrier6();
#pragma unroll
      for (int t = 0; t < WM; ++t) mma_tile(fr[t], bf, acc[t]);
    }
  } else {
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) stage(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(STAGES - 2, nk - 1 - kt);
    if constexpr (STAGES >= 3) {
      if (ahead >= 1 && mine == PER_WAVE) wait_vmcnt6<PER_WAVE>();
      else if (ahead >= 1 && PER_WAVE > 1) wait_vmcnt6<(PER_WAVE > 1 ? PER_WAVE - 1 : 0)>();
      else wait_vmcnt6<0>();
    } else {
      wait_vmcnt6<0>();
    }
    barrier6();
    if (kt + STAGES - 1 < nk) stage(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
    const char* base = smem + (kt % STAGES) * ST;
    v4i bf[WN];
    read_b(base, bf);
#pragma unroll
    for (int t = 0; t < WM; ++t) {
      AFrag f;
      if constexpr (DIAG == 2) {
        f.a0 = v8i{lane, t, kt, 1, lane, t, 0, 0};
        f.a1 = v8i{t, lane, kt, 2, kt, lane, 0, 0};
        f.a2 = v8i{kt, t, lane, 3, t, kt, 0, 0};
        f.a3 = v8i{lane, kt, t, 4, lane, kt, 0, 0};
        f.sb = 100 + (lane & 7);
      } else {
        read_a(base, t, f);
      }
      mma_tile(f, bf, acc[t]);
    }
  }
  }

  // epilogue: C/D map of the 32x32 MFMA (reg i -> row (i&3)+8(i>>2)+4h, col lane&31), transposed
  // through a per-wave LDS patch and written as 16-B row segments (as bnn_gemm.hip); with p.bn.mode
  // the BatchNorm-backward column statistics of the tile ride along (Gemm6Params::Bn)
  wait_vmcnt6<0>();
  barrier6();
  float* patch = reinterpret_cast<float*>(smem) + wave * 1024;
  const bool vec_ok = ((ldo & 3) == 0) && ((reinterpret_cast<uintptr_t>(Cout) & 15) == 0);
  // the statistics epilogue exists in the 2-wave-row, 2-tile-row forms (the default 128 x 512 tile)
  // BNS = 1: its own instance (bnn_gemm_fp6_bnstats), so the default kernel carries none of it
  // (with the statistics code compiled in, the plain launches ran 17 % slower: 240 VGPRs, 94 SGPRs)
  constexpr bool BNE = BNS && WAVES_M == 2 && WM == 2 && DIAG == 0;
  const int bnmode = BNE ? p.bn.mode : 0;
  __shared__ float bnred[BNE ? 2 : 1][BNE ? WAVES_N : 1][BNE ? WN : 1][32][4];   // per wave row: its column statistics
#pragma unroll
  for (int u = 0; u < WN; ++u) {
    const int tcol0 = n0 + wn * WN * 32 + u * 32;
    const int col = tcol0 + r;
    const float bb = (bias && col < p.N) ? bias[col] : 0.f;
    const int c4 = lane & 7, cs = tcol0 + 4 * c4;          // this lane's 4 columns in the row phase
    float st0[4] = {0.f, 0.f, 0.f, 0.f}, st1[4] = {0.f, 0.f, 0.f, 0.f};
    float stg[4] = {0.f, 0.f, 0.f, 0.f}, stx[4] = {0.f, 0.f, 0.f, 0.f};
    float bm[4], bl[4], bi[4], bg[4], bbt[4], bx[4];
    if (bnmode && cs + 3 < p.N) {
      const float4 m4 = *reinterpret_cast<const float4*>(p.bn.mean + cs);
      const float4 i4 = *reinterpret_cast<const float4*>(p.bn.invstd + cs);
      const float4 l4 = p.bn.mean_lo ? *reinterpret_cast<const float4*>(p.bn.mean_lo + cs) : make_float4(0, 0, 0, 0);
      const float4 g4 = p.bn.gamma ? *reinterpret_cast<const float4*>(p.bn.gamma + cs) : make_float4(1, 1, 1, 1);
      const float4 b4 = p.bn.beta ? *reinterpret_cast<const float4*>(p.bn.beta + cs) : make_float4(0, 0, 0, 0);
      const float4 x4 = (p.bn.z16 && p.bn.xbias) ? *reinterpret_cast<const float4*>(p.bn.xbias + cs) : make_float4(0, 0, 0, 0);
      bm[0] = m4.x, bm[1] = m4.y, bm[2] = m4.z, bm[3] = m4.w;
      bi[0] = i4.x, bi[1] = i4.y, bi[2] = i4.z, bi[3] = i4.w;
      bl[0] = l4.x, bl[1] = l4.y, bl[2] = l4.z, bl[3] = l4.w;
      bg[0] = g4.x, bg[1] = g4.y, bg[2] = g4.z, bg[3] = g4.w;
      bbt[0] = b4.x, bbt[1] = b4.y, bbt[2] = b4.z, bbt[3] = b4.w;
      bx[0] = x4.x, bx[1] = x4.y, bx[2] = x4.z, bx[3] = x4.w;
    }
    // this lane's x values of both tile rows, all loads issued before any is used (one memory
    // latency per column group instead of one per row phase); rows past M clamped, never summed
    float xv[WM][4][4];
    if (bnmode && cs + 3 < p.N) {
#pragma unroll
      for (int t = 0; t < WM; ++t)
#pragma unroll
        for (int ps = 0; ps < 4; ++ps) {
          const int rr = m0 + wm * WM * 32 + t * 32 + (lane >> 3) + 8 * ps;
          const int64_t xi = (int64_t)(rr < p.M ? rr : p.M - 1) * p.N + cs;
          if (p.bn.z16) {
            const uint2 q = *reinterpret_cast<const uint2*>(reinterpret_cast<const int16_t*>(p.bn.x) + xi);
            xv[t][ps][0] = (float)(int16_t)(q.x & 0xFFFFu) + bx[0], xv[t][ps][1] = (float)(int16_t)(q.x >> 16) + bx[1];
            xv[t][ps][2] = (float)(int16_t)(q.y & 0xFFFFu) + bx[2], xv[t][ps][3] = (float)(int16_t)(q.y >> 16) + bx[3];
          } else {
            const float4 q = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p.bn.x) + xi);
            xv[t][ps][0] = q.x, xv[t][ps][1] = q.y, xv[t][ps][2] = q.z, xv[t][ps][3] = q.w;
          }
        }
    }
#pragma unroll
    for (int t = 0; t < WM; ++t) {
      const int trow0 = m0 + wm * WM * 32 + t * 32;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int lr = (i & 3) + 8 * (i >> 2) + 4 * h;
        float f = acc[t][u][i];
        if (bias) f += bb;
        patch[lr * 32 + ((((r >> 2) ^ (lr & 7)) << 2) | (r & 3))] = f;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int ps = 0; ps < 4; ++ps) {
        const int lr = (lane >> 3) + 8 * ps;
        const float4 v = *reinterpret_cast<const float4*>(patch + lr * 32 + ((c4 ^ (lr & 7)) << 2));
        const int row = trow0 + lr, c0 = cs;
        if (row >= p.M) continue;
        float* dst = Cout + (int64_t)row * ldo + c0;
        if (vec_ok && c0 + 3 < p.N) {
#ifdef GEMM6_DIAG_NOSTORE     // timing-only build: the epilogue without its global stores
          if (p.M > 0) continue;
#endif
          out_store4f(dst, v);
        } else {
          const float vs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (c0 + j < p.N) dst[j] = vs[j];
        }
        if (bnmode && c0 + 3 < p.N) {
          // bn_reduce_k MODE 1 / 2 on these 4 elements (the same xhat, y, mask and products)
          const float* xs = xv[t][ps];
          const float gs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float xh = ((xs[j] - bm[j]) - bl[j]) * bi[j];
            const float y = fmaf(xh, bg[j], bbt[j]);
            const float g = (!p.bn.hardtanh || (y > -1.f && y < 1.f)) ? gs[j] : 0.f;
            st0[j] += g;
            st1[j] = fmaf(g, xh, st1[j]);
            if (bnmode == 2) {   // NaN -> inf: the bound (and the scale) become non-finite
              const float ag = fabsf(g), ax = fabsf(xh);
              stg[j] = (ag == ag) ? fmaxf(stg[j], ag) : __builtin_inff();
              stx[j] = (ax == ax) ? fmaxf(stx[j], ax) : __builtin_inff();
            }
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (BNE && bnmode) {
      // the 8 lanes holding these columns (lane bits 3-5: 8 row phases): a fixed xor tree
#pragma unroll
      for (int o = 8; o < 64; o <<= 1)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          st0[j] += __shfl_xor(st0[j], o, 64);
          st1[j] += __shfl_xor(st1[j], o, 64);
          if (bnmode == 2) {
            stg[j] = fmaxf(stg[j], __shfl_xor(stg[j], o, 64));
            stx[j] = fmaxf(stx[j], __shfl_xor(stx[j], o, 64));
          }
        }
      if (lane < 8) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          bnred[wm][wn][u][4 * c4 + j][0] = st0[j];
          bnred[wm][wn][u][4 * c4 + j][1] = st1[j];
          bnred[wm][wn][u][4 * c4 + j][2] = stg[j];
          bnred[wm][wn][u][4 * c4 + j][3] = stx[j];
        }
      }
    }
  }
  if (BNE && bnmode) {
    __syncthreads();
    // wave row 0 folds the two wave rows (fixed order) and writes this tile row's partials
    if (wm == 0 && lane < 32) {
      const int64_t RN = (int64_t)p.gm * p.N;
#pragma unroll
      for (int u = 0; u < WN; ++u) {
        const int c = n0 + wn * WN * 32 + u * 32 + lane;
        if (c >= p.N) continue;
        float* pp = p.bn.part + (int64_t)tm * p.N + c;
        pp[0] = bnred[0][wn][u][lane][0] + bnred[1][wn][u][lane][0];
        pp[RN] = bnred[0][wn][u][lane][1] + bnred[1][wn][u][lane][1];
        if (bnmode == 2) {
          pp[2 * RN] = fmaxf(bnred[0][wn][u][lane][2], bnred[1][wn][u][lane][2]);
          pp[3 * RN] = fmaxf(bnred[0][wn][u][lane][3], bnred[1][wn][u][lane][3]);
        }
      }
    }
  }
}

// Persistent form of the default 128 x 512 tile (variant 7; RES = 1 with the residual plane): one
// workgroup per CU walks the tiles bid, bid + G, ... in the same XCD / raster order as the one-tile
// grid, and its fp32 epilogue no longer holds the CU.  The four waves of wave row 1 issue every
// global store of a tile (their own 32 x 32 patches and, through a separate LDS patch region, their
// row-0 partners'); the four of wave row 0 never store.  gfx9 counts loads and stores in one
// in-order vmcnt, so a wave waiting for its stage pieces also waits for every store issued before
// them: the first S_LD stages of each tile are issued by the row-0 waves alone (and the next tile's
// first stage during the current tile's last k-step), so the row-1 waves' stores drain under the
// next tile's first S_LD k-steps; from stage S_LD on all eight waves share the staging again.  Same fragments, MFMAs and accumulation order as gemm_fp6_k<2, 4, 2, 4, 2>:
// bit-identical C.  No bias, no split-K, no statistics (the host picks this form only then).
template <int RES>
__global__ __launch_bounds__(512, 2) void gemm_fp6_pers_k(Gemm6Params p) {
  constexpr int WAVES_N = 4, WM = 2, WN = 4, NL = 4;     // NL loading waves (wave row 0)
  constexpr int BM = 128, BN = 512;
  constexpr int LO_ST = BM * 128, HI_ST = BM * 64, SC_PAD = 1024, B_ST = BN * 32, R_ST = RES ? BM * 32 : 0;
  constexpr int ST = LO_ST + HI_ST + SC_PAD + B_ST + R_ST;
  constexpr int P_LO = LO_ST / 1024 / NL, P_HI = HI_ST / 1024 / NL, P_B = B_ST / 1024 / NL;
  static_assert(P_LO * NL * 1024 == LO_ST && P_HI * NL * 1024 == HI_ST && P_B * NL * 1024 == B_ST, "piece split");
  static_assert(R_ST / 1024 <= NL, "residual pieces: at most one per loading wave");
  // the first S_LD stages of a tile are issued by the loading waves alone (the storing waves' vmcnt
  // holds the previous tile's stores); from stage S_LD on every wave issues its one-tile share
  constexpr int S_LD = 16;
  using NLt = std::integral_constant<int, NL>;
  using NWt = std::integral_constant<int, 8>;
  __shared__ __attribute__((aligned(16))) char smem[2 * ST + 8 * 4096];
  float* const patches = reinterpret_cast<float*>(smem + 2 * ST);   // one 32 x 32 fp32 patch per wave

  const int lane = threadIdx.x & 63, wave = wave_id();
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const bool loader = wm == 0;
  const int r = lane & 31, h = lane >> 5;
  const int64_t nblk = p.K / QB;
  const int nk = p.K / 64, ntiles = p.gm * p.gn, G = (int)gridDim.x;
  int L = (int)blockIdx.x;
  if (L >= ntiles) return;

  // Stage issue (loading waves).  The host takes this form only for M % 128 == 0, N % 512 == 0 and B
  // in the panel layout, so no row is clamped: each piece's per-lane offset (row in tile and the
  // XOR-swizzled 16-B chunk) is a function of the lane alone, formed at issue from an opaque copy of
  // the lane index (so it is not hoisted into 11 registers held across the k loop), and the stage
  // bases are formed from (m0, n0, kt) in scalar registers -- the persistent loop has neither VGPRs
  // nor SGPRs to spare beside the 128 accumulators.
  const int64_t b_step = FP4_PANEL * 32;
  // NI = the number of waves issuing the stage (NL: the loading waves alone; NW: all eight, each a
  // one-tile share); wi = this wave's index among them
  auto stage = [&](auto ni_tag, int m0, int n0, int kt, int buf) __attribute__((always_inline)) {
    constexpr int NI = decltype(ni_tag)::value;
    constexpr int I_R = R_ST / 1024;
    constexpr int Q_LO = LO_ST / 1024 / NI, Q_HI = HI_ST / 1024 / NI, Q_B = B_ST / 1024 / NI, Q_R = (I_R + NI - 1) / NI;
    const int wi = wave;
    int ln;
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    char* base = smem + buf * ST;
    const uint8_t* lo_b = p.alo + (int64_t)m0 * nblk * 64 + (int64_t)kt * 128;
    const uint8_t* hi_b = p.ahi + (int64_t)m0 * nblk * 32 + (int64_t)kt * 64;
    const uint8_t* b_b = p.b + ((int64_t)(n0 / FP4_PANEL) * p.bks + kt) * b_step + (n0 % FP4_PANEL) * 32;
#pragma unroll
    for (int ii = 0; ii < Q_LO; ++ii) {
      const int lrow = (wi + ii * NI) * 8 + (ln >> 3), c = ln & 7;
      glds16_6s(lo_b, (uint32_t)lrow * (uint32_t)(nblk * 64) + 16u * (uint32_t)(c ^ ((lrow >> 1) & 7)),
                base + (wi + ii * NI) * 1024);
    }
#pragma unroll
    for (int ii = 0; ii < Q_HI; ++ii) {
      const int lrow = (wi + ii * NI) * 16 + (ln >> 2), c = ln & 3;
      glds16_6s(hi_b, (uint32_t)lrow * (uint32_t)(nblk * 32) + 16u * (uint32_t)(c ^ ((lrow >> 2) & 3)),
                base + LO_ST + (wi + ii * NI) * 1024);
    }
#pragma unroll
    for (int ii = 0; ii < Q_B; ++ii) {
      const int lrow = (wi + ii * NI) * 32 + (ln >> 1), c = ln & 1;
      glds16_6s(b_b, (uint32_t)lrow * 32u + 16u * (uint32_t)(c ^ ((lrow >> 3) & 1)),
                base + LO_ST + HI_ST + SC_PAD + (wi + ii * NI) * 1024);
    }
    if (wave == 0) glds16_6(p.asc + (int64_t)m0 * 2 + (int64_t)kt * p.asc_rows * 2 + ln * 16, base + LO_ST + HI_ST);
    if constexpr (RES) {
      const uint8_t* r_b = p.ares + (int64_t)m0 * nblk * 16 + (int64_t)kt * 32;
#pragma unroll
      for (int ii = 0; ii < Q_R; ++ii) {
        if (wi + ii * NI >= I_R) continue;   // the residual's pieces: one per wave of the first I_R
        const int lrow = (wi + ii * NI) * 32 + (ln >> 1), c = ln & 1;
        glds16_6s(r_b, (uint32_t)lrow * (uint32_t)(nblk * 16) + 16u * (uint32_t)(c ^ ((lrow >> 3) & 1)),
                  base + LO_ST + HI_ST + SC_PAD + B_ST + (wi + ii * NI) * 1024);
      }
    }
  };

  int tm, tn;
  tile6_of(L, p.gm, p.gn, p.group, tm, tn);
  if (loader) stage(NLt{}, tm * BM, tn * BN, 0, 0);
  int gk = 0;   // k-steps run so far (the ring slot of step kt of this tile is gk & 1)
  const bool vec_ok = ((p.ldc & 3) == 0) && ((reinterpret_cast<uintptr_t>(p.C) & 15) == 0);
  for (;;) {
    v16f acc[WM][WN];
#pragma unroll
    for (int t = 0; t < WM; ++t)
#pragma unroll
      for (int u = 0; u < WN; ++u) acc[t][u] = v16f{0};
    const int m0 = tm * BM, n0 = tn * BN;
    int ntm = 0, ntn = 0;
    const bool more = L + G < ntiles;
    if (more) tile6_of(L + G, p.gm, p.gn, p.group, ntm, ntn);
    for (int kt = 0; kt < nk; ++kt, ++gk) {
      // this wave's pieces of stage kt; a storing wave issues pieces only from stage S_LD on, by when
      // the previous tile's stores ahead of them in its vmcnt have drained
      if (loader || kt >= S_LD) wait_vmcnt6<0>();
      barrier6();
      const int buf = gk & 1;
      if (kt + 1 < nk) {
        if (kt + 1 >= S_LD) stage(NWt{}, m0, n0, kt + 1, buf ^ 1);
        else if (loader) stage(NLt{}, m0, n0, kt + 1, buf ^ 1);
      } else if (more && loader) {
        stage(NLt{}, ntm * BM, ntn * BN, 0, buf ^ 1);   // the next tile's first stage
      }
      const char* base = smem + buf * ST;
      v4i bf[WN];
      const char* sB = base + LO_ST + HI_ST + SC_PAD;
#pragma unroll
      for (int u = 0; u < WN; ++u) {
        const int lrow = wn * WN * 32 + u * 32 + r;
        bf[u] = *reinterpret_cast<const v4i*>(sB + lrow * 32 + 16 * (h ^ ((lrow >> 3) & 1)));
      }
#pragma unroll
      for (int t = 0; t < WM; ++t) {
        const int lrow = wm * WM * 32 + t * 32 + r;
        const char* sLo = base;
        const char* sHi = base + LO_ST;
        const uint8_t* sSc = reinterpret_cast<const uint8_t*>(base + LO_ST + HI_ST);
        const int sw = (lrow >> 1) & 7;
        const v4i l0 = *reinterpret_cast<const v4i*>(sLo + lrow * 128 + 16 * ((h * 4 + 0) ^ sw));
        const v4i l1 = *reinterpret_cast<const v4i*>(sLo + lrow * 128 + 16 * ((h * 4 + 1) ^ sw));
        const v4i l2 = *reinterpret_cast<const v4i*>(sLo + lrow * 128 + 16 * ((h * 4 + 2) ^ sw));
        const v4i l3 = *reinterpret_cast<const v4i*>(sLo + lrow * 128 + 16 * ((h * 4 + 3) ^ sw));
        const v4i h01 = *reinterpret_cast<const v4i*>(sHi + lrow * 64 + 16 * ((h * 2) ^ ((lrow >> 2) & 3)));
        const v4i h23 = *reinterpret_cast<const v4i*>(sHi + lrow * 64 + 16 * ((h * 2 + 1) ^ ((lrow >> 2) & 3)));
        const v8i a0 = v8i{l0.x, l0.y, l0.z, l0.w, h01.x, h01.y, 0, 0};
        const v8i a1 = v8i{l1.x, l1.y, l1.z, l1.w, h01.z, h01.w, 0, 0};
        const v8i a2 = v8i{l2.x, l2.y, l2.z, l2.w, h23.x, h23.y, 0, 0};
        const v8i a3 = v8i{l3.x, l3.y, l3.z, l3.w, h23.z, h23.w, 0, 0};
        const int sb = sSc[lrow * 2 + h];
        v4i rr = v4i{0, 0, 0, 0};
        if constexpr (RES)
          rr = *reinterpret_cast<const v4i*>(base + LO_ST + HI_ST + SC_PAD + B_ST + lrow * 32 + 16 * (h ^ ((lrow >> 3) & 1)));
        const int s0 = sb, s1 = sb == 255 ? 255 : sb + 5, s2 = sb == 255 ? 255 : sb + 10, s3 = sb == 255 ? 255 : sb + 15;
        const int sr = sb == 255 ? 255 : (sb >= 5 ? sb - 5 : 0);
#pragma unroll
        for (int u = 0; u < WN; ++u) {
          const v8i bb = {bf[u].x, bf[u].y, bf[u].z, bf[u].w, 0, 0, 0, 0};
          acc[t][u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a3, bb, acc[t][u], 2, 4, 0, s3, 0, 127);
          acc[t][u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a2, bb, acc[t][u], 2, 4, 0, s2, 0, 127);
          acc[t][u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a1, bb, acc[t][u], 2, 4, 0, s1, 0, 127);
          acc[t][u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a0, bb, acc[t][u], 2, 4, 0, s0, 0, 127);
          if constexpr (RES) {
            const v8i ar = {rr.x, rr.y, rr.z, rr.w, 0, 0, 0, 0};
            acc[t][u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ar, bb, acc[t][u], 4, 4, 0, sr, 0, 127);
          }
        }
      }
    }
    // epilogue: every wave transposes its 32 x 32 patches through its own slot of the patch region
    // (the ring holds the next tile's first stage); the storing wave of each column group writes its
    // partner's patch (rows 0..63 of the tile) and its own (rows 64..127) as 16-B row segments
    float* const mine = patches + wave * 1024;
    float* const partner = patches + (wave - NL) * 1024;   // storing waves only
#pragma unroll
    for (int u = 0; u < WN; ++u) {
      const int tcol0 = n0 + wn * WN * 32 + u * 32;
#pragma unroll
      for (int t = 0; t < WM; ++t) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int lr = (i & 3) + 8 * (i >> 2) + 4 * h;
          mine[lr * 32 + ((((r >> 2) ^ (lr & 7)) << 2) | (r & 3))] = acc[t][u][i];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier6();
        if (!loader) {
          const int c4 = lane & 7;
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            const float* src = half ? mine : partner;
            const int trow0 = m0 + half * WM * 32 + t * 32;
#pragma unroll
            for (int ps = 0; ps < 4; ++ps) {
              const int lr = (lane >> 3) + 8 * ps;
              const float4 v = *reinterpret_cast<const float4*>(src + lr * 32 + ((c4 ^ (lr & 7)) << 2));
              const int row = trow0 + lr, c0 = tcol0 + 4 * c4;
              if (row >= p.M) continue;
              float* dst = p.C + (int64_t)row * p.ldc + c0;
              if (vec_ok && c0 + 3 < p.N) {
                out_store4f(dst, v);
              } else {
                const float vs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 4; ++j)
                  if (c0 + j < p.N) dst[j] = vs[j];
              }
            }
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        barrier6();   // the slots are free for the next patch
      }
    }
    if (!more) break;
    L += G;
    tm = ntm;
    tn = ntn;
  }
}

// C = bias + sum over splits of the partials, in split order (deterministic); float4 per thread
__global__ __launch_bounds__(256) void gemm6_splitk_sum_k(const float* __restrict__ part, int S, int64_t M, int64_t N,
                                                          const float* __restrict__ bias, float* __restrict__ C,
                                                          int64_t ldc) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= M * N) return;
  const int64_t m = i / N, n = i - m * N;       // N % 4 == 0 (host check): 4 elements of one row
  float4 a = *reinterpret_cast<const float4*>(part + i);
  for (int sp = 1; sp < S; ++sp) {
    const float4 b = *reinterpret_cast<const float4*>(part + sp * M * N + i);
    a.x += b.x, a.y += b.y, a.z += b.z, a.w += b.w;
  }
  if (bias) a.x += bias[n], a.y += bias[n + 1], a.z += bias[n + 2], a.w += bias[n + 3];
  float* dst = C + m * ldc + n;
  if (((reinterpret_cast<uintptr_t>(dst)) & 15) == 0) {
    *reinterpret_cast<float4*>(dst) = a;
  } else {   // e.g. a gradient-bucket view at an odd offset: same sums, scalar stores
    dst[0] = a.x, dst[1] = a.y, dst[2] = a.z, dst[3] = a.w;
  }
}

template <int WAVES_M, int WAVES_N, int WM, int WN, int STAGES, int DIAG = 0, int OCC = 2, int PP = 0,
          int BNS = 0, int RES = 0>
int launch6(Gemm6Params p, hipStream_t s) {
  constexpr int BM = WAVES_M * WM * 32, BN = WAVES_N * WN * 32;
  p.gm = (p.M + BM - 1) / BM;
  p.gn = (p.N + BN - 1) / BN;
  if (p.part == nullptr) p.ksplit = 1;
  const int nk = p.K / 64;
  p.kps = (nk + p.ksplit - 1) / p.ksplit;
  p.ksplit = (nk + p.kps - 1) / p.kps;          // no empty split
  hipLaunchKernelGGL((gemm_fp6_k<WAVES_M, WAVES_N, WM, WN, STAGES, DIAG, OCC, PP, BNS, RES>),
                     dim3((unsigned)((int64_t)p.gm * p.gn * p.ksplit)), dim3(64 * WAVES_M * WAVES_N), 0, s, p);
  if (p.ksplit > 1)
    hipLaunchKernelGGL(gemm6_splitk_sum_k, dim3((unsigned)(((int64_t)p.M * p.N / 4 + 255) / 256)), dim3(256), 0, s,
                       p.part, p.ksplit, (int64_t)p.M, (int64_t)p.N, p.bias, p.C, p.ldc);
  return check_launch("bnn_gemm_fp6");
}

// The persistent form (gemm_fp6_pers_k) for grids of at least two rounds, no bias / split-K: measured
// slower than one workgroup per tile on both backward shapes (dX 8.52 vs 8.60 ms with the row-0
// waves staging every stage, dW 7.2-7.3 vs 6.85-6.89; sharing the staging again after the first 16
// k-steps: dX 9.27, dW 7.80 -- profiles/r05_fp6_persistent_ab.log), so off by default (A/B switch).
int g_fp6_pers = 0;

template <int RES>
int launch6_pers(Gemm6Params p, int ncu, hipStream_t s) {
  p.gm = (p.M + 127) / 128;
  p.gn = (p.N + 511) / 512;
  const int ntiles = p.gm * p.gn;
  hipLaunchKernelGGL((gemm_fp6_pers_k<RES>), dim3((unsigned)std::min(ntiles, ncu)), dim3(512), 0, s, p);
  return check_launch("bnn_gemm_fp6 (persistent)");
}

struct Variant6 {
  int id;
  const char* name;
  int (*fn)(Gemm6Params, hipStream_t);
  int bm;   // rows per tile (the scale array must hold round_up(M, bm) rows... see bnn_gemm_fp6)
  int bn;   // columns per tile
};

const Variant6 kVariants6[] = {
    {0, "gemm_fp6_k<2, 4, 4, 2, 2>", launch6<2, 4, 4, 2, 2>, 256, 256},
    {1, "gemm_fp6_k<2, 4, 2, 2, 3>", launch6<2, 4, 2, 2, 3>, 128, 256},
    {2, "gemm_fp6_k<2, 2, 2, 2, 3>", launch6<2, 2, 2, 2, 3>, 128, 128},
    {3, "gemm_fp6_k<4, 2, 2, 4, 2>", launch6<4, 2, 2, 4, 2>, 256, 256},
    {4, "gemm_fp6_k<2, 4, 2, 2, 4>", launch6<2, 4, 2, 2, 4>, 128, 256},
    // tall-N tiles: the FP6 operand costs 3 B/element against 0.5 for FP4, so BM x BN = 128 x 512
    // moves 29% fewer bytes per MAC than 256 x 256 and leaves room for a third stage
    {5, "gemm_fp6_k<2, 4, 2, 4, 3>", launch6<2, 4, 2, 4, 3>, 128, 512},
    {6, "gemm_fp6_k<1, 8, 4, 2, 3>", launch6<1, 8, 4, 2, 3>, 128, 512},
    {7, "gemm_fp6_k<2, 4, 2, 4, 2>", launch6<2, 4, 2, 4, 2>, 128, 512},
    // two workgroups per CU (OCC 4: <= 128 registers per lane)
    {8, "gemm_fp6_k<2, 4, 2, 2, 2, 0, 4>", launch6<2, 4, 2, 2, 2, 0, 4>, 128, 256},
    // software-pipelined k loop (PP): 128 x 512 and 128 x 256 tiles
    {10, "gemm_fp6_k<2, 4, 2, 4, 3, 0, 2, 1>", launch6<2, 4, 2, 4, 3, 0, 2, 1>, 128, 512},
    {11, "gemm_fp6_k<2, 4, 2, 2, 3, 0, 2, 1>", launch6<2, 4, 2, 2, 3, 0, 2, 1>, 128, 256},
    // pipelined form 2: 128 x 512 tile, every wave 32 rows x 256 columns (4 x 2 waves)
    {12, "gemm_fp6_k<4, 2, 1, 8, 3, 0, 2, 2>", launch6<4, 2, 1, 8, 3, 0, 2, 2>, 128, 512},
    {13, "gemm_fp6_k<4, 1, 1, 8, 3, 0, 2, 2>", launch6<4, 1, 1, 8, 3, 0, 2, 2>, 128, 256},
    // 4-wave workgroups small enough in LDS for two per CU: one workgroup's barrier wait or
    // epilogue overlaps the other's MFMAs
    {14, "gemm_fp6_k<1, 4, 2, 4, 2>", launch6<1, 4, 2, 4, 2>, 64, 512},
    {15, "gemm_fp6_k<2, 2, 2, 4, 2>", launch6<2, 2, 2, 4, 2>, 128, 256},
    // ping-pong: the two wave rows run a phase apart, one group's MFMAs beside the other's reads
    // (equal to variant 7 within 1% on the wide shapes: the MFMA-busy fraction stays ~0.6 --
    // profiles/r02_fp6_pingpong.txt)
    {16, "gemm_fp6_k<2, 4, 2, 4, 3, 0, 2, 3>", launch6<2, 4, 2, 4, 3, 0, 2, 3>, 128, 512},
    // interleaved form: all fragment reads right after the barrier, the next stage's DMA pieces
    // spread between the MFMA column groups
    {17, "gemm_fp6_k<2, 4, 2, 4, 2, 0, 2, 4>", launch6<2, 4, 2, 4, 2, 0, 2, 4>, 128, 512},
    {18, "gemm_fp6_k<2, 4, 2, 4, 3, 0, 2, 4>", launch6<2, 4, 2, 4, 3, 0, 2, 4>, 128, 512},
    // timing-only diagnostics of variant 5 (wrong results; never picked by default)
    {91, "diag: v5 without global->LDS staging", launch6<2, 4, 2, 4, 3, 1>, 128, 512},
    {92, "diag: v5 without LDS fragment reads", launch6<2, 4, 2, 4, 3, 2>, 128, 512},
    // timing-only diagnostics of variant 7 (the wide default)
    {93, "diag: v7 MFMA stream + barrier", launch6<2, 4, 2, 4, 2, 3>, 128, 512},
    {94, "diag: v7 MFMA stream only", launch6<2, 4, 2, 4, 2, 4>, 128, 512},
    {95, "diag: v7 without global->LDS staging", launch6<2, 4, 2, 4, 2, 1>, 128, 512},
    {96, "diag: v7 without LDS fragment reads", launch6<2, 4, 2, 4, 2, 2>, 128, 512},
    {97, "diag: v7 with B staged from contiguous panels", launch6<2, 4, 2, 4, 2, 5>, 128, 512},
    {98, "diag: v7 with B and A hi staged from contiguous panels", launch6<2, 4, 2, 4, 2, 6>, 128, 512},
};

int g_variant6 = -1;
// bnn_gemm_fp6_set_half: 0 = the 128 x 512 tile, one workgroup per CU; 1 (default) = the dX
// launches (residual plane) on 64 x 512 tiles, two 4-wave workgroups per CU; 2 = the dW launches
// (4 planes) too.  g_half_ticks: the first-round stagger of the second workgroup on each CU.
// Measured on the wide step's shapes (profiles/r06_b_fp6_half.log, one box, interleaved): dX + res
// 8.83 -> 8.31 ms with no stagger (40-200 us: 8.32-8.35), dW 7.12 -> 7.30-7.37 (kept on the 128 x
// 512 tile).  The two residents of a CU (blocks b and b + 256 in the first round,
// tools/probes/probe_wg_placement.hip) drift apart by themselves once their tiles' epilogues and
// barrier waits differ, so one's fp32 stores drain beside the other's MFMAs.
int g_fp6_half = 1;
int64_t g_half_ticks = 0;
int g_half_group = 0;   // raster group rows of the half-tile form (0: as the 128 x 512 tile's, 4 / 8)

const Variant6* find6(int id) {
  for (const Variant6& v : kVariants6)
    if (v.id == id) return &v;
  return &kVariants6[0];      // unknown id: the first entry (the sweep skips repeated names)
}

// Default per shape: the 128 x 512 tile (the FP6 operand is 6x the bytes of the FP4 one per row,
// so tall-N tiles move the fewest bytes per MAC) for every shape; grids below one round of the
// chip are split along K (plan6).
const Variant6* pick6(int64_t M, int64_t N) {
  (void)M, (void)N;
  return g_variant6 >= 0 ? find6(g_variant6) : find6(7);
}

inline hipStream_t S6(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace
}  // namespace bnn

using namespace bnn;

// scale-array row pitch: rows rounded up to 256, plus 512 rows of padding so the GEMM's per-stage
// 1-KiB scale piece (512 rows from the tile's first row) never reads past the slab
BNN_API int64_t bnn_quant6_scale_rows(int64_t rows) { return q6_scale_rows(rows); }

BNN_API int bnn_quant6_rows(const float* x, int64_t M, int64_t K, int64_t ldx, int64_t Kp, uint8_t* lo, uint8_t* hi,
                            uint8_t* sc, uint8_t* res, void* stream) {
  if (!x || !lo || !hi || !sc || M < 0 || K < 0 || ldx < K || Kp < K || Kp % 64 != 0 || Kp == 0 || !aligned16(lo) ||
      !aligned16(hi) || (res && !aligned16(res)) || M > 0x7fffffff || (Kp / QB + 31) / 32 > 65535) {
    set_error("bnn_quant6_rows: bad arguments (M=%lld K=%lld Kp=%lld)", (long long)M, (long long)K, (long long)Kp);
    return kErrInval;
  }
  if (M == 0) return 0;
  const int64_t nblk = Kp / QB;
  const int vec = aligned16(x) && (ldx % 4 == 0);
  hipLaunchKernelGGL(quant6_rows_k, dim3((unsigned)M, (unsigned)((nblk + 31) / 32)), dim3(256), 0, S6(stream), x, M,
                     K, ldx, nblk, lo, hi, sc, bnn_quant6_scale_rows(M), vec, res);
  return check_launch("bnn_quant6_rows");
}

BNN_API int64_t bnn_quant6_cols_workspace(int64_t M, int64_t N) {
  return ((M + 255) / 256) * N * (int64_t)sizeof(double);
}

BNN_API int bnn_quant6_cols_t(const float* x, int64_t M, int64_t N, int64_t ldx, int64_t Mp, uint8_t* lo,
                              uint8_t* hi, uint8_t* sc, float* colsum, void* work, void* stream) {
  if (!x || !lo || !hi || !sc || M < 0 || N < 0 || ldx < N || Mp < M || Mp % 64 != 0 || Mp == 0 || !aligned16(lo) ||
      !aligned16(hi) || (colsum && !work) || (Mp + 255) / 256 > 65535) {
    set_error("bnn_quant6_cols_t: bad arguments (M=%lld N=%lld Mp=%lld)", (long long)M, (long long)N, (long long)Mp);
    return kErrInval;
  }
  if (N == 0) return 0;
  const int64_t nblk = Mp / QB;
  const int64_t R = (nblk + QC_BLKS - 1) / QC_BLKS;
  double* part = colsum ? reinterpret_cast<double*>(work) : nullptr;
  hipLaunchKernelGGL(quant6_cols_t_k, dim3((unsigned)((N + QC_COLS - 1) / QC_COLS), (unsigned)R), dim3(512), 0,
                     S6(stream), x, M, N, ldx, nblk, lo, hi, sc, bnn_quant6_scale_rows(N), part);
  if (colsum)
    hipLaunchKernelGGL(colsum_final_k, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, S6(stream), part, R, N,
                       colsum);
  return check_launch("bnn_quant6_cols_t");
}

// Launch plan of the default kernel for a shape: the 128 x 512 tile, and a grid below one round of
// the chip (the MLP's backward GEMMs at batch 4096: 18-192 tiles) split along K into
// floor(CUs / tiles) parts of >= 4 k-steps each (the whole-round efficiency of the big tile beats a
// smaller tile's finer grid: stream-K on 128 x 256 tiles measured 27-55 us per GEMM against 44 for
// the unsplit 192-tile 128 x 512 grid, tools/gpu_r03_sk.sh).  Forced variants never split.
struct Fp6Plan {
  const Variant6* v;
  int ksplit;
};

static int device_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cus = n;
  }
  return cus;
}

#ifndef FP6_SPLIT_CAP
#define FP6_SPLIT_CAP 8
#endif
static Fp6Plan plan6(int64_t M, int64_t N, int64_t K) {
  if (g_variant6 >= 0) return Fp6Plan{find6(g_variant6), 1};
  const Variant6* v = find6(7);
  const int64_t tiles = ((M + v->bm - 1) / v->bm) * ((N + v->bn - 1) / v->bn), ncu = device_cus();
  const int64_t s = std::min<int64_t>(std::min<int64_t>(ncu / std::max<int64_t>(tiles, 1), (K / 64) / 4), FP6_SPLIT_CAP);
  return Fp6Plan{v, (int)std::max<int64_t>(1, s)};
}

BNN_API int64_t bnn_gemm_fp6_workspace(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 64 != 0) return 0;
  const Fp6Plan pl = plan6(M, N, K);
  return pl.ksplit > 1 && N % 4 == 0 ? (int64_t)pl.ksplit * M * N * (int64_t)sizeof(float) : 0;
}

static int gemm_fp6_impl(const uint8_t* alo, const uint8_t* ahi, const uint8_t* asc, int64_t asc_rows,
                         const uint8_t* ares, const uint8_t* b, int64_t ldb, const float* bias, float* C, int64_t ldc,
                         int64_t M, int64_t N, int64_t K, void* work, int64_t work_bytes, void* stream);

// Whether a launch takes the persistent form of the default tile (gemm_fp6_pers_k, selected by
// bnn_gemm_fp6_set_persistent): no bias, B in panels, whole K per tile, a 128 x 512-tiled shape of at
// least two rounds of tiles.  One predicate for gemm_fp6_impl and the name bnn_gemm_fp6_kernel_k reports.
// Whether a launch takes the half-tile form (bnn_gemm_fp6_set_half): mode 1 the residual-plane (dX)
// launches, mode 2 every launch; no bias, whole K per tile, 64 x 512-tiled shapes of >= 2 rounds of
// two workgroups per CU.
// FP6_HALF_SMALL: also an unsplit grid of under one round of 128 x 512 tiles (config 3's dX), where the
// half tiles double the workgroups that share the chip.
#ifndef FP6_HALF_SMALL
#define FP6_HALF_SMALL 0
#endif
static bool fp6_half_applies(int64_t M, int64_t N, int ksplit, bool has_bias, bool res) {
  if (g_fp6_half <= 0 || has_bias || ksplit > 1 || g_variant6 >= 0 || M % 64 != 0 || N % 512 != 0) return false;
  const int64_t tiles = (M / 64) * (N / 512);
  if (res || g_fp6_half > 1) return tiles >= 4 * device_cus();
  return FP6_HALF_SMALL && tiles < 2 * device_cus();
}

static bool fp6_pers_applies(int64_t M, int64_t N, int ksplit, bool has_bias, bool panel) {
  return g_fp6_pers && !has_bias && panel && ksplit <= 1 && g_variant6 < 0 && M % 128 == 0 && N % 512 == 0 &&
         (M / 128) * (N / 512) >= 2 * device_cus();
}

BNN_API int bnn_gemm_fp6(const uint8_t* alo, const uint8_t* ahi, const uint8_t* asc, int64_t asc_rows,
                         const uint8_t* ares, const uint8_t* b, int64_t ldb, const float* bias, float* C, int64_t ldc,
                         int64_t M, int64_t N, int64_t K, void* stream) {
  return gemm_fp6_impl(alo, ahi, asc, asc_rows, ares, b, ldb, bias, C, ldc, M, N, K, nullptr, 0, stream);
}

BNN_API int bnn_gemm_fp6_ws(const uint8_t* alo, const uint8_t* ahi, const uint8_t* asc, int64_t asc_rows,
                            const uint8_t* ares, const uint8_t* b, int64_t ldb, const float* bias, float* C,
                            int64_t ldc, int64_t M, int64_t N, int64_t K, void* work, int64_t work_bytes, void* stream) {
  return gemm_fp6_impl(alo, ahi, asc, asc_rows, ares, b, ldb, bias, C, ldc, M, N, K, work, work_bytes, stream);
}

static int gemm_fp6_impl(const uint8_t* alo, const uint8_t* ahi, const uint8_t* asc, int64_t asc_rows,
                         const uint8_t* ares, const uint8_t* b, int64_t ldb, const float* bias, float* C, int64_t ldc,
                         int64_t M, int64_t N, int64_t K, void* work, int64_t work_bytes, void* stream) {
  const bool panel = ldb < 0;   // bnn_gemm_fp6_panel_ws: ldb = -(k-steps per panel)
  if (!alo || !ahi || !asc || !b || !C || M < 0 || N < 0 || K <= 0 || K % 64 != 0 || (!panel && (ldb < K / 2 || ldb % 16 != 0)) ||
      ldc < N || asc_rows < bnn_quant6_scale_rows(M) || asc_rows % 256 != 0 || !aligned16(alo) || !aligned16(ahi) ||
      !aligned16(asc) || !aligned16(b) || (ares && !aligned16(ares)) || (ares && g_variant6 >= 0 && g_variant6 != 7) ||
      M > 0x7fffffff || N > 0x7fffffff || K > 0x7fffffff) {
    set_error("bnn_gemm_fp6: bad arguments (M=%lld N=%lld K=%lld ldb=%lld asc_rows=%lld; K a positive multiple of "
              "64, asc_rows a multiple of 256 >= bnn_quant6_scale_rows(M))",
              (long long)M, (long long)N, (long long)K, (long long)ldb, (long long)asc_rows);
    return kErrInval;
  }
  if (M == 0 || N == 0) return 0;
  // split-K only with a workspace of bnn_gemm_fp6_workspace bytes (else the whole K per tile); the
  // result depends on the shape only -- never on C's alignment or pitch: a gradient written straight
  // into a bucket view must equal the one AccumulateGrad would add
  const Fp6Plan pl = plan6(M, N, K);
  const int64_t need = bnn_gemm_fp6_workspace(M, N, K);
  const bool split = need > 0 && work != nullptr && aligned16(work) && work_bytes >= need;
  Gemm6Params p{alo, ahi, asc, b, ldb, asc_rows, bias, C, ldc, (int)M, (int)N, (int)K, 0, 0, K >= 32768 ? 8 : 4,
                split ? pl.ksplit : 1, 0, split ? reinterpret_cast<float*>(work) : nullptr, panel ? -ldb : 0, {}};

  const bool pers = fp6_pers_applies(M, N, p.ksplit, bias != nullptr, panel);
  // the half-tile form: 64 x 512 tiles, two workgroups per CU, the second resident of each CU in the
  // first round (blocks [CUs, 2 CUs): tools/probes/probe_wg_placement.hip) held back g_half_ticks
  const bool half = !pers && fp6_half_applies(M, N, p.ksplit, bias != nullptr, ares != nullptr);
  if (half) {
    p.stg_lo = device_cus();
    p.stg_hi = 2 * device_cus();
    p.stg_ticks = g_half_ticks;
    if (g_half_group > 0) p.group = g_half_group;
  }
  if (ares) {   // the residual plane runs on the default tile (variant 7) with its own instance
    p.ares = ares;
    if (pers) return launch6_pers<1>(p, device_cus(), S6(stream));
    if (half) return launch6<1, 4, 2, 4, 2, 0, 2, 0, 0, 1>(p, S6(stream));
    return launch6<2, 4, 2, 4, 2, 0, 2, 0, 0, 1>(p, S6(stream));
  }
  if (half) return launch6<1, 4, 2, 4, 2>(p, S6(stream));
  if (pers && pl.v->id == 7) return launch6_pers<0>(p, device_cus(), S6(stream));
  return pl.v->fn(p, S6(stream));
}

// 0 (default): one workgroup per tile.  1: the default tile runs persistent with split load / store
// roles on grids of two or more rounds (gemm_fp6_pers_k; measured slower on both backward shapes,
// DESIGN.md §5 -- kept for A/B).  on < 0 queries.
BNN_API int bnn_gemm_fp6_set_persistent(int32_t on) {
  if (on < 0) return g_fp6_pers;
  g_fp6_pers = on != 0;
  return 0;
}

// The FP6 GEMM's half-tile form (g_fp6_half above): mode 0 / 1 / 2, stagger in microseconds (the
// first-round wait of the second workgroup on each CU); mode < 0 queries the mode.
BNN_API int bnn_gemm_fp6_set_half(int32_t mode, double stagger_us) {
  if (mode < 0) return g_fp6_half;
  g_fp6_half = mode;
  g_half_ticks = (int64_t)(stagger_us * 100.0);
  return 0;
}

// Tuning hook: raster group (tile rows per group, tile6_of) of the half-tile form; 0 = default.
BNN_API int bnn_gemm_fp6_set_half_group(int32_t g) {
  g_half_group = g < 0 ? 0 : g;
  return 0;
}

BNN_API int64_t bnn_fp4_panel_bytes(int64_t N, int64_t Kp) {
  if (N <= 0 || Kp <= 0 || Kp % 64 != 0) return 0;
  return (N + FP4_PANEL - 1) / FP4_PANEL * FP4_PANEL * (Kp / 2);
}

BNN_API int bnn_fp4_panelize(const uint8_t* b, int64_t N, int64_t ldb, int64_t Kp, uint8_t* panels, void* stream) {
  if (!b || !panels || N <= 0 || Kp <= 0 || Kp % 64 != 0 || ldb < Kp / 2 || ldb % 16 != 0 || !aligned16(b) ||
      !aligned16(panels) || (Kp / 64 + 3) / 4 > 0x7fffffff) {
    set_error("bnn_fp4_panelize: bad arguments (N=%lld ldb=%lld Kp=%lld)", (long long)N, (long long)ldb, (long long)Kp);
    return kErrInval;
  }
  const int64_t nks = Kp / 64, rows = (N + FP4_PANEL - 1) / FP4_PANEL * FP4_PANEL;
  hipLaunchKernelGGL(fp4_panelize_k, dim3((unsigned)((nks + 3) / 4), (unsigned)(rows / 32)), dim3(256), 0, S6(stream),
                     b, N, ldb, nks, panels);
  return check_launch("bnn_fp4_panelize");
}

BNN_API int bnn_gemm_fp6_panel_ws(const uint8_t* alo, const uint8_t* ahi, const uint8_t* asc, int64_t asc_rows,
                                  const uint8_t* ares, const uint8_t* bpanels, int64_t bks, const float* bias, float* C,
                                  int64_t ldc, int64_t M, int64_t N, int64_t K, void* work, int64_t work_bytes,
                                  void* stream) {
  if ((g_variant6 >= 0 && 512 % find6(g_variant6)->bn != 0) || K <= 0 || bks < K / 64) {
    set_error("bnn_gemm_fp6_panel_ws: bad arguments (K=%lld bks=%lld; bks >= K/64, a tile width dividing 512)",
              (long long)K, (long long)bks);
    return kErrInval;
  }
  return gemm_fp6_impl(alo, ahi, asc, asc_rows, ares, bpanels, -bks, bias, C, ldc, M, N, K, work, work_bytes, stream);
}

// The panel GEMM with the BatchNorm-backward statistics of C in its epilogue (Gemm6Params::Bn), for
// the dX product that feeds a training-mode BatchNorm(+Hardtanh) backward: part = [2 or 4][gm][N]
// floats, gm = bnn_gemm_fp6_bnstats_rows(M) (one row per 128-row tile row); no bias, no split-K.
BNN_API int64_t bnn_gemm_fp6_bnstats_rows(int64_t M) { return (M + 127) / 128; }

BNN_API int bnn_gemm_fp6_bnstats(const uint8_t* alo, const uint8_t* ahi, const uint8_t* asc, int64_t asc_rows,
                                 const uint8_t* ares, const uint8_t* bpanels, int64_t bks, float* C, int64_t ldc,
                                 int64_t M, int64_t N,
                                 int64_t K, const void* x, const float* xbias, int32_t x_i16, const float* mean,
                                 const float* mean_lo, const float* invstd, const float* gamma, const float* beta,
                                 int32_t hardtanh, int32_t mode, float* part, void* stream) {
  const Fp6Plan pl = plan6(M, N, K);
  if (!x || !mean || !invstd || !part || (mode != 1 && mode != 2) || N % 4 != 0 || pl.ksplit != 1 ||
      pl.v->bm != 128 || pl.v->id != 7 || K <= 0 || bks < K / 64 || !aligned16(x) || !aligned16(mean) ||
      !aligned16(invstd) || (mean_lo && !aligned16(mean_lo)) || (gamma && !aligned16(gamma)) ||
      (beta && !aligned16(beta)) || (xbias && !aligned16(xbias)) || !aligned16(part)) {
    set_error("bnn_gemm_fp6_bnstats: bad arguments (M=%lld N=%lld K=%lld mode=%d; N %% 4 == 0, an unsplit 128x512 "
              "default plan, 16-B aligned vectors)", (long long)M, (long long)N, (long long)K, mode);
    return kErrInval;
  }
  if (!alo || !ahi || !asc || !bpanels || !C || M <= 0 || N <= 0 || K % 64 != 0 || ldc < N ||
      asc_rows < bnn_quant6_scale_rows(M) || asc_rows % 256 != 0 || !aligned16(alo) || !aligned16(ahi) ||
      !aligned16(asc) || !aligned16(bpanels) || (ares && !aligned16(ares)) || M > 0x7fffffff || N > 0x7fffffff ||
      K > 0x7fffffff) {
    set_error("bnn_gemm_fp6_bnstats: bad GEMM arguments");
    return kErrInval;
  }
  Gemm6Params p{alo, ahi, asc, bpanels, -bks, asc_rows, nullptr, C, ldc, (int)M, (int)N, (int)K, 0, 0,
                K >= 32768 ? 8 : 4, 1, 0, nullptr, bks};
  p.bn = Gemm6Params::Bn{x, xbias, mean, mean_lo, invstd, gamma, beta, part, x_i16 ? 1 : 0, hardtanh ? 1 : 0, mode};
  if (ares) {
    p.ares = ares;
    return launch6<2, 4, 2, 4, 2, 0, 2, 0, 1, 1>(p, S6(stream));
  }
  return launch6<2, 4, 2, 4, 2, 0, 2, 0, 1>(p, S6(stream));
}

BNN_API const char* bnn_gemm_fp6_kernel(int64_t M, int64_t N) { return pick6(M, N)->name; }

BNN_API const char* bnn_gemm_fp6_kernel_k(int64_t M, int64_t N, int64_t K) {
  const Fp6Plan pl = plan6(M, N, K);
  static thread_local char buf[96];
  // the name of what the backward GEMMs (no bias, B in panels) launch on this shape: the persistent
  // form where gemm_fp6_impl's predicate takes it; a residual-plane launch runs the default tile's
  // RES instance, which is variant 7 = the plan's choice on every unsplit shape of the wide step
  if (fp6_pers_applies(M, N, pl.ksplit, false, true)) return "gemm_fp6_pers_k<2, 4, 2, 4, 2>";
  if (pl.ksplit <= 1) return pl.v->name;
  snprintf(buf, sizeof buf, "%s split-K %d", pl.v->name, pl.ksplit);
  return buf;
}

// As bnn_gemm_fp6_kernel_k for a launch with (res != 0) or without the residual plane.
BNN_API const char* bnn_gemm_fp6_kernel_kr(int64_t M, int64_t N, int64_t K, int32_t res) {
  const Fp6Plan pl = plan6(M, N, K);
  if (!fp6_pers_applies(M, N, pl.ksplit, false, true) && fp6_half_applies(M, N, pl.ksplit, false, res != 0))
    return "gemm_fp6_k<1, 4, 2, 4, 2>";
  return bnn_gemm_fp6_kernel_k(M, N, K);
}

BNN_API int bnn_gemm_fp6_set_variant(int32_t v) {
  g_variant6 = v;
  return 0;
}
