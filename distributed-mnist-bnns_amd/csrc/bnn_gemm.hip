// Subsystem (2)+(3): the int8 MFMA GEMM behind BinarizeLinear (models/binarized_modules.py:80)
// and both GEMMs of its autograd (dX = dY.W_b, dW = dY^T.X_b).
//
//   C[m][n] = cvt( sum_{i,j} 2^(8(i+j)) sum_k A_i[m][k] B_j[n][k] ) * a_scale[m] * b_scale[n] + bias[n]
//
// Both operands are K-contiguous int8 ("NT" layout) -- exactly what v_mfma_i32_32x32x32_i8 wants
// for its A and B fragments.  Ternary x ternary sums are exact int32, so the (1,1) form followed by
// one fp32 bias add is bit-identical to the reference's F.linear(x_b, W_b) + bias.  fp32 operands
// arrive as 3 balanced base-256 digit planes with a power-of-two scale per row (bnn_pack.hip);
// their partial sums are exact int32 and are combined in fp64 in the epilogue (one fp32 rounding).
//
// Structure (CDNA4): 256-thread workgroups = 4 waves in 2x2; each wave owns WM x WN 32x32 output
// tiles; BK = 64 bytes of K per stage; operands staged global->LDS with global_load_lds_dwordx4
// (16 B per lane, LDS image lane-linear, chunk XOR-swizzle applied on the SOURCE address so the
// ds_read_b128 fragment reads are bank-conflict free); two LDS buffers; XCD-aware bijective
// block remap + grouped raster so blocks sharing an A panel run on one XCD's L2.
#include <algorithm>
#include <type_traits>

#include "bnn_common.h"

namespace bnn {
namespace {

constexpr int BK = 64;

struct GemmParams {
  const int8_t* A;
  const int8_t* B;
  int64_t lda, ldb, a_plane, b_plane;
  const float* a_scale;
  const float* b_scale;
  const float* bias;
  float* C;
  int64_t ldc;
  int M, N, K;
  int gm, gn;
  // optional integer offsets added to the raw sum before scaling (u8 pixel operands,
  // bnn_pixels.hip): sum + off_mul * (row_off[m] + col_off[n]), in double
  const int64_t* row_off;
  const int64_t* col_off;
  double off_mul;
  // int16 output (ternary x ternary forms without scales, offsets or bias): the exact dot products
  // |sum| <= K < 2^15 as int16 [M][ldc] instead of fp32 C (bnn_gemm_fp4_i16)
  int16_t* C16 = nullptr;
  // the next BatchNorm's forward statistics from the (1,1) 32x32 forms' epilogue
  // (bnn_gemm_i8_affine_bnstats): [2][stat_rows][N] doubles, chunk = this tile row's wave row
  double* stat = nullptr;
  int64_t stat_rows = 0;
  const float* stat_bias = nullptr;   // FP4 statistics form: z = fl(sum + stat_bias[n]) (the int16 carrier's bias)
  Drop stat_drop{0, 0u, 0, 1.f, nullptr};   // ... of drop(z) when a fused dropout precedes the BatchNorm
  // 1: row-major tile order (consecutive tiles along N: concurrent tiles write adjacent segments of
  // the same C rows) instead of the grouped raster
  int raster = 0;
  // s20 output of the u8-pixel statistics form (bnn_gemm_i8_affine_bnstats_s20): the exact integer
  // S = sum + off_mul * col_off[n] (integral off_mul, |S| < 2^19: host check) as its low 16 bits
  // [M][ldc] + high nibbles [M][ldc / 2] instead of fp32 C (XIn XF 2 in bnn_common.h)
  int16_t* S20lo = nullptr;
  uint8_t* S20hi = nullptr;
};

__device__ __forceinline__ double int_offset(const GemmParams& p, int row, int col) {
  double o = 0.0;
  if (p.row_off) o += (double)p.row_off[row];
  if (p.col_off) o += (double)p.col_off[col];
  return o * p.off_mul;
}

__device__ __forceinline__ void glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// The same 16-B LDS-DMA in its saddr form: wave-uniform 64-bit base in SGPRs + per-lane 32-bit
// offset (one VGPR), LDS destination through M0.  Written as asm because the compiler hoists
// base+offset into a 64-bit VGPR pair per piece.  The explicit wait_vmcnt_c() counts cover it.
__device__ __forceinline__ void glds16_s(const void* sbase, uint32_t voff, void* l) {
  const uint32_t la = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(l);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
               :
               : "s"(la), "v"(voff), "s"(sbase)
               : "memory", "m0");
}

// Bijective XCD remap (blocks b and b+8 share an XCD under round-robin dispatch: speed only)
// followed by a grouped raster (8 tile-rows per group) so an XCD works on neighbouring tiles.
__device__ __forceinline__ void tile_of(int bid, int gm, int gn, int& tm, int& tn) {
  const int nwg = gm * gn;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  constexpr int G = 8;
  const int per_group = G * gn;
  const int g = L / per_group, first = g * G;
  const int gs = min(gm - first, G);
  const int in = L - g * per_group;
  tm = first + in % gs;
  tn = in / gs;
}

template <int DA, int DB>
struct Cfg {
  static constexpr int NC = (DA == 1 && DB == 1) ? 1 : 3;  // accumulator classes
  static constexpr bool FLUSH = (DB == 3);                 // int32 -> f32 flush (digit x digit)
  static constexpr int FLUSH_KT = 512;                      // k-tiles per flush: 32768 k
};

template <int DA, int DB, int WM, int WN>
__global__ __launch_bounds__(256) void gemm_i8_k(GemmParams p) {
  constexpr int BM = 64 * WM, BN = 64 * WN;
  constexpr int A_ST = DA * BM * BK, B_ST = DB * BN * BK, ST = A_ST + B_ST;
  constexpr int NC = Cfg<DA, DB>::NC;
  constexpr bool FLUSH = Cfg<DA, DB>::FLUSH;
  __shared__ __attribute__((aligned(16))) char smem[2 * ST];

  const int lane = threadIdx.x & 63, wave = wave_id();
  const int wm = wave >> 1, wn = wave & 1;
  int tm, tn;
  tile_of(blockIdx.x, p.gm, p.gn, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- global -> LDS staging: one glds = 1 KiB = 16 rows x 64 B; lane i -> row i/4, slot i%4,
  // source chunk slot ^ ((row>>2)&3) (the swizzle lives on the source address: rule 21).
  const int srow = lane >> 2, sslot = lane & 3;
  const int schunk = sslot ^ ((srow >> 2) & 3);
  auto stage = [&](int kt, int buf) {
    char* sA = smem + buf * ST;
    char* sB = sA + A_ST;
    const int k0 = kt * BK + 16 * schunk;
#pragma unroll
    for (int j = wave; j < DA * BM / 16; j += 4) {
      const int d = j / (BM / 16), jr = j % (BM / 16);
      const int row = min(m0 + jr * 16 + srow, p.M - 1);
      glds16(p.A + d * p.a_plane + (int64_t)row * p.lda + k0, sA + d * BM * BK + jr * 1024);
    }
#pragma unroll
    for (int j = wave; j < DB * BN / 16; j += 4) {
      const int e = j / (BN / 16), jr = j % (BN / 16);
      const int row = min(n0 + jr * 16 + srow, p.N - 1);
      glds16(p.B + e * p.b_plane + (int64_t)row * p.ldb + k0, sB + e * BN * BK + jr * 1024);
    }
  };

  v16i acc[NC][WM][WN];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int t = 0; t < WM; ++t)
#pragma unroll
      for (int u = 0; u < WN; ++u) acc[c][t][u] = v16i{0};
  float facc[FLUSH ? WM : 1][FLUSH ? WN : 1][16];
  if constexpr (FLUSH) {
#pragma unroll
    for (int t = 0; t < WM; ++t)
#pragma unroll
      for (int u = 0; u < WN; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) facc[t][u][i] = 0.f;
  }

  const int r = lane & 31, h = lane >> 5, sw = (r >> 2) & 3;
  const int nk = p.K / BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, buf ^ 1);
    const char* sA = smem + buf * ST;
    const char* sB = sA + A_ST;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int off = 16 * ((2 * ks + h) ^ sw);
      v4i a[DA][WM], b[DB][WN];
#pragma unroll
      for (int d = 0; d < DA; ++d)
#pragma unroll
        for (int t = 0; t < WM; ++t)
          a[d][t] = *reinterpret_cast<const v4i*>(sA + d * BM * BK + (wm * WM * 32 + t * 32 + r) * BK + off);
#pragma unroll
      for (int e = 0; e < DB; ++e)
#pragma unroll
        for (int u = 0; u < WN; ++u)
          b[e][u] = *reinterpret_cast<const v4i*>(sB + e * BN * BK + (wn * WN * 32 + u * 32 + r) * BK + off);
#pragma unroll
      for (int t = 0; t < WM; ++t)
#pragma unroll
        for (int u = 0; u < WN; ++u) {
          if constexpr (DA == 1 && DB == 1) {
            acc[0][t][u] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[0][t], b[0][u], acc[0][t][u], 0, 0, 0);
          } else if constexpr (DB == 1) {
#pragma unroll
            for (int d = 0; d < DA; ++d)
              acc[d][t][u] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[d][t], b[0][u], acc[d][t][u], 0, 0, 0);
          } else {
#pragma unroll
            for (int i = 0; i < DA; ++i)
#pragma unroll
              for (int j = 0; j < DB; ++j)
                if (i + j >= 2)
                  acc[i + j - 2][t][u] =
                      __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i][t], b[j][u], acc[i + j - 2][t][u], 0, 0, 0);
          }
        }
    }
    if constexpr (FLUSH) {
      if ((kt + 1) % Cfg<DA, DB>::FLUSH_KT == 0 || kt + 1 == nk) {
#pragma unroll
        for (int t = 0; t < WM; ++t)
#pragma unroll
          for (int u = 0; u < WN; ++u) {
#pragma unroll
            for (int i = 0; i < 16; ++i)
              facc[t][u][i] += (float)((double)acc[2][t][u][i] * 65536.0 + (double)acc[1][t][u][i] * 256.0 +
                                       (double)acc[0][t][u][i]);
#pragma unroll
            for (int c = 0; c < NC; ++c) acc[c][t][u] = v16i{0};
          }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: C/D map of the 32x32 MFMA: reg i -> row (i&3)+8(i>>2)+4h, col = lane&31.
#pragma unroll
  for (int t = 0; t < WM; ++t)
#pragma unroll
    for (int u = 0; u < WN; ++u) {
      const int col = n0 + wn * WN * 32 + u * 32 + r;
      if (col >= p.N) continue;
      const float bs = p.b_scale ? p.b_scale[col] : 1.f;
      const float bb = p.bias ? p.bias[col] : 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = m0 + wm * WM * 32 + t * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (row >= p.M) continue;
        double v;
        if constexpr (DA == 1 && DB == 1) {
          v = (double)acc[0][t][u][i];
        } else if constexpr (DB == 1) {
          v = (double)acc[2][t][u][i] * 65536.0 + (double)acc[1][t][u][i] * 256.0 + (double)acc[0][t][u][i];
        } else {
          v = (double)facc[t][u][i] * 65536.0;
        }
        if (p.row_off || p.col_off) v += int_offset(p, row, col);
        if (p.a_scale) v *= (double)p.a_scale[row];
        v *= (double)bs;
        float f = (float)v;
        if (p.bias) f += bb;
        p.C[(int64_t)row * p.ldc + col] = f;
      }
    }
}

// ---------------------------------------------------------------------------------------------
// v2: WAVES_M x WAVES_N waves, STAGES-deep LDS ring filled by global_load_lds, counted vmcnt
// (the next STAGES-2 tiles stay in flight across the barrier), raw s_barrier (a __syncthreads()
// would drain every in-flight LDS-DMA with vmcnt(0)).
// s_waitcnt simm16 (gfx9 encoding): vmcnt[3:0] | expcnt[6:4]=7 | lgkmcnt[11:8]=15 | vmcnt_hi[15:14]
template <int N>
__device__ __forceinline__ void wait_vmcnt_c() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// Wait until at most `ahead` stages (PER_WAVE loads each) of this wave's LDS-DMA remain in flight.
template <int PER_WAVE, int MAX_AHEAD>
__device__ __forceinline__ void wait_stages(int ahead) {
  if constexpr (MAX_AHEAD >= 3) {
    if (ahead >= 3) { wait_vmcnt_c<3 * PER_WAVE>(); return; }
  }
  if constexpr (MAX_AHEAD >= 2) {
    if (ahead == 2) { wait_vmcnt_c<2 * PER_WAVE>(); return; }
  }
  if constexpr (MAX_AHEAD >= 1) {
    if (ahead == 1) { wait_vmcnt_c<PER_WAVE>(); return; }
  }
  wait_vmcnt_c<0>();
}

template <int S16, typename Acc>
__device__ __forceinline__ Acc mfma_i8(v4i a, v4i b, Acc c) {
  if constexpr (S16)
    return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void block_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int DA, int DB, int WAVES_M, int WAVES_N, int WM, int WN, int STAGES, int BKT, int IL = 0,
          int DIAG = 0, int F4 = 0, int S16 = 0, int BST = 0>
__device__ __forceinline__ void gemm_v2_body(const GemmParams& p) {
  // F4 = 1: both operands are ternary FP4 (e2m1) nibbles, 2 per byte; K and the LDS tiles are
  // counted in bytes (BKT bytes = 2*BKT elements); v_mfma_scale_f32_32x32x64_f8f6f4 with unit
  // E8M0 scales (127) multiplies 64 k per instruction -- twice the int8 rate on half the bytes --
  // and its fp32 accumulation of +-1 products is exact (|sum| < 2^24).
  // S16 = 1: the same WM x WN 32x32 wave tile computed as (2WM) x (2WN) 16x16 MFMA tiles
  // (v_mfma_i32_16x16x64_i8 / v_mfma_scale_f32_16x16x128_f8f6f4, 64 bytes of K per instruction):
  // equal cycles per op, but the chip holds a higher clock on the 16x16 shape under load
  // (MI355X_MICROARCH.md, DVFS give-back item 7).  Needs BKT = 128 for conflict-free reads.
  static_assert(!F4 || (DA == 1 && DB == 1), "FP4 mode is the ternary x ternary form");
  static_assert(!S16 || BKT == 128, "16x16 tiles use the BK=128 swizzle");
  constexpr int TS = S16 ? 16 : 32;            // MFMA tile edge
  constexpr int TM = S16 ? 2 * WM : WM, TN = S16 ? 2 * WN : WN;
  constexpr int TR = TS * TS / 64;             // accumulator registers per tile
  using AccT = typename std::conditional<
      S16 != 0, typename std::conditional<F4 != 0, v4f, v4i>::type,
      typename std::conditional<F4 != 0, v16f, v16i>::type>::type;
  // DIAG (timing-only builds, wrong results): 1 = no LDS fragment reads, 2 = no global->LDS staging;
  // DIAG = 3 is not a diagnostic: the 16x16 digit form with B fragments prefetched a k-step ahead
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int BM = WAVES_M * WM * 32, BN = WAVES_N * WN * 32;
  constexpr int A_ST = DA * BM * BKT, B_ST = DB * BN * BKT, ST = A_ST + B_ST;
  constexpr int RPI = 1024 / BKT;          // rows covered by one 1-KiB glds
  constexpr int CPR = BKT / 16;            // 16-B chunks per row
  constexpr int IA = DA * BM / RPI, IB = DB * BN / RPI;
  static_assert(IA % NW == 0 && IB % NW == 0, "glds instructions must split evenly over waves");
  constexpr int PER_WAVE = (IA + IB) / NW;
  constexpr int NC = Cfg<DA, DB>::NC;
  constexpr bool FLUSH = Cfg<DA, DB>::FLUSH;
  constexpr int KSTEPS = BKT / (S16 ? 64 : 32);
  constexpr int FLUSH_KT = Cfg<DA, DB>::FLUSH_KT * 64 / BKT;
  __shared__ __attribute__((aligned(16))) char smem[STAGES * ST];

  const int lane = threadIdx.x & 63, wave = wave_id();
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  int tm, tn;
  if (p.raster == 1) {   // XCD remap only, then row-major
    const int nwg = p.gm * p.gn, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
    const int L = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
    tm = L / p.gn;
    tn = L - tm * p.gn;
  } else {
    tile_of(blockIdx.x, p.gm, p.gn, tm, tn);
  }
  const int m0 = tm * BM, n0 = tn * BN;

  // chunk swizzle: BK=64 -> chunk ^ ((row>>2)&3); BK=128 -> chunk ^ ((row>>1)&7).  Applied to the
  // global source (LDS image stays lane-linear) and to the ds_read address.
  auto swz = [](int row) { return BKT == 64 ? ((row >> 2) & 3) : ((row >> 1) & 7); };
  // lane -> (row srow of the 1-KiB piece, 16-B slot sslot); the swizzle uses the tile-local row
  // (piece jr covers rows jr*RPI .. jr*RPI+RPI-1; with BK=128 bit 3 of the row comes from jr).
  const int srow = lane / CPR, sslot = lane % CPR;
  // Each piece's address = a wave-uniform 64-bit base (SGPRs: operand, plane, tile row, k-tile)
  // + a per-lane 32-bit offset (row in tile, clamped to the last valid row, and the swizzled
  // chunk), so the LDS-DMA issues in its saddr form with one VGPR of address; the loops have
  // compile-time trip counts (no branches between pieces).  The host guarantees BM*lda and
  // BN*ldb < 2^31 (bnn_gemm_i8 falls back to the v1 kernel otherwise).
  const int lim_a = p.M - 1 - m0, lim_b = p.N - 1 - n0;
  auto stage = [&](int kt, int buf) {
    if constexpr (DIAG == 2) return;
    char* sA = smem + buf * ST;
    char* sB = sA + A_ST;
#pragma unroll
    for (int i = 0; i < IA / NW; ++i) {
      const int j = wave + i * NW;
      const int d = j / (BM / RPI), jr = j % (BM / RPI);
      const int lrow = jr * RPI + srow;
      const uint32_t voff = (uint32_t)min(lrow, lim_a) * (uint32_t)p.lda + 16u * (uint32_t)(sslot ^ swz(lrow));
      const int8_t* base = p.A + d * p.a_plane + (int64_t)m0 * p.lda + (int64_t)kt * BKT;
      glds16_s(base, voff, sA + d * BM * BKT + jr * 1024);
    }
#pragma unroll
    for (int i = 0; i < IB / NW; ++i) {
      const int j = wave + i * NW;
      const int e = j / (BN / RPI), jr = j % (BN / RPI);
      const int lrow = jr * RPI + srow;
      const uint32_t voff = (uint32_t)min(lrow, lim_b) * (uint32_t)p.ldb + 16u * (uint32_t)(sslot ^ swz(lrow));
      const int8_t* base = p.B + e * p.b_plane + (int64_t)n0 * p.ldb + (int64_t)kt * BKT;
      glds16_s(base, voff, sB + e * BN * BKT + jr * 1024);
    }
  };

  AccT acc[NC][TM][TN];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u) acc[c][t][u] = AccT{0};
  float facc[FLUSH ? TM : 1][FLUSH ? TN : 1][TR];
  if constexpr (FLUSH) {
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int u = 0; u < TN; ++u)
#pragma unroll
        for (int i = 0; i < TR; ++i) facc[t][u][i] = 0.f;
  }

  // fragment lane map: 32x32 -> row lane&31, 16-B chunk (lane>>5) of a 32-B k-step;
  //                    16x16 -> row lane&15, 16-B chunk (lane>>4) of a 64-B k-step
  const int r = S16 ? (lane & 15) : (lane & 31), h = S16 ? (lane >> 4) : (lane >> 5), sw = swz(r);
#ifdef GEMM_DIAG_NOMAIN   // timing-only build: no k loop (the epilogue of zero accumulators)
  const int nk = p.K > (1 << 30) ? p.K / BKT : 0;
#else
  const int nk = p.K / BKT;
#endif
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) stage(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    if constexpr (IL == 2) {
      // IL = 2: the next stage is always issued (the last tile is re-loaded into the free buffer
      // near the end), so STAGES-2 stages are always in flight, the loop body has no branch and
      // its LDS-DMA pieces can be spread between the MFMAs by the schedule below.
      wait_stages<PER_WAVE, STAGES - 2>(STAGES - 2);
      block_barrier();
      stage(min(kt + STAGES - 1, nk - 1), (kt + STAGES - 1) % STAGES);
    } else {
      const int ahead = min(STAGES - 2, nk - 1 - kt);
      wait_stages<PER_WAVE, STAGES - 2>(ahead);
      block_barrier();
      if (kt + STAGES - 1 < nk) stage(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
    }
    const int buf = kt % STAGES;
    const char* sA = smem + buf * ST;
    const char* sB = sA + A_ST;
    // fragments of k-step ks+1 are read from LDS while the MFMAs of k-step ks run (register
    // double buffer; indices are compile-time after unrolling)
    v4i a[2][DA][TM], b[2][DB][TN];
    auto load_frags = [&](int ks, v4i (&fa)[DA][TM], v4i (&fb)[DB][TN]) {
      if constexpr (DIAG == 1) {
#pragma unroll
        for (int d = 0; d < DA; ++d)
#pragma unroll
          for (int t = 0; t < TM; ++t) fa[d][t] = v4i{lane + ks, d, t, kt};
#pragma unroll
        for (int e = 0; e < DB; ++e)
#pragma unroll
          for (int u = 0; u < TN; ++u) fb[e][u] = v4i{lane, e + ks, u, kt};
        return;
      }
      const int off = S16 ? 16 * ((4 * ks + h) ^ sw) : 16 * ((2 * ks + h) ^ sw);
#pragma unroll
      for (int d = 0; d < DA; ++d)
#pragma unroll
        for (int t = 0; t < TM; ++t)
          fa[d][t] = *reinterpret_cast<const v4i*>(sA + d * BM * BKT + (wm * WM * 32 + t * TS + r) * BKT + off);
#pragma unroll
      for (int e = 0; e < DB; ++e)
#pragma unroll
        for (int u = 0; u < TN; ++u)
          fb[e][u] = *reinterpret_cast<const v4i*>(sB + e * BN * BKT + (wn * WN * 32 + u * TS + r) * BKT + off);
    };
    if constexpr (S16 && DA == 3 && DB == 1 && (DIAG == 0 || DIAG == 3)) {
      constexpr bool BPF = DIAG == 3;   // B fragments of the next k-step read during the last tiles
      // 16x16 digit form: a full register double buffer of 64-B k-steps would not fit beside the
      // 192 accumulator registers, so B fragments are read once per k-step and A fragments are
      // streamed one 16-row tile ahead of the MFMAs that use them.
      v4i bfs[2][TN];
      auto load_b = [&](int ks, v4i (&fb)[TN]) {
        const int off = 16 * ((4 * ks + h) ^ sw);
#pragma unroll
        for (int u = 0; u < TN; ++u)
          fb[u] = *reinterpret_cast<const v4i*>(sB + (wn * WN * 32 + u * TS + r) * BKT + off);
      };
      if constexpr (BPF) load_b(0, bfs[0]);
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks) {
        const int off = 16 * ((4 * ks + h) ^ sw);
        v4i(&bf)[TN] = bfs[BPF ? (ks & 1) : 0];
        if constexpr (!BPF) load_b(ks, bf);
        v4i af[2][DA];
        auto load_a = [&](int t, v4i (&fa)[DA]) {
#pragma unroll
          for (int d = 0; d < DA; ++d)
            fa[d] = *reinterpret_cast<const v4i*>(sA + d * BM * BKT + (wm * WM * 32 + t * TS + r) * BKT + off);
        };
        load_a(0, af[0]);
#pragma unroll
        for (int t = 0; t < TM; ++t) {
          if (t + 1 < TM) load_a(t + 1, af[(t + 1) & 1]);
          if (BPF && t == TM - 2 && ks + 1 < KSTEPS) load_b(ks + 1, bfs[(ks + 1) & 1]);
#pragma unroll
          for (int u = 0; u < TN; ++u)
#pragma unroll
            for (int d = 0; d < DA; ++d) acc[d][t][u] = mfma_i8<S16>(af[t & 1][d], bf[u], acc[d][t][u]);
          if constexpr (IL == 1) {
            if (t + 1 < TM) {
#pragma unroll
              for (int q = 0; q < DA; ++q) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
              }
              __builtin_amdgcn_sched_group_barrier(0x008, TN * DA - DA, 0);
            }
          }
          if constexpr (IL == 2) {
            // the k-tile's PER_WAVE LDS-DMA pieces spread over its KSTEPS*TM (k-step, tile) slots
            constexpr int SLOTS = KSTEPS * TM;
            const int slot = ks * TM + t;
            const int nv = PER_WAVE * (slot + 1) / SLOTS - PER_WAVE * slot / SLOTS;
            const int nld = t + 1 < TM ? DA : 0;
            if (t == 0) __builtin_amdgcn_sched_group_barrier(0x100, TN + DA, 0);
#pragma unroll
            for (int q = 0; q < TN * DA; ++q) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              if (q < nld) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
              if (q < nv) __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
            }
          }
        }
      }
    } else {
    load_frags(0, a[0], b[0]);
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      if (ks + 1 < KSTEPS) load_frags(ks + 1, a[(ks + 1) & 1], b[(ks + 1) & 1]);
      const int cur = ks & 1;
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int u = 0; u < TN; ++u) {
          if constexpr (F4) {
            const v4i x = a[cur][0][t], y = b[cur][0][u];
            const v8i xa = {x.x, x.y, x.z, x.w, 0, 0, 0, 0}, yb = {y.x, y.y, y.z, y.w, 0, 0, 0, 0};
            if constexpr (S16)
              acc[0][t][u] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(xa, yb, acc[0][t][u], 4, 4, 0, 127,
                                                                              0, 127);
            else
              acc[0][t][u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(xa, yb, acc[0][t][u], 4, 4, 0, 127,
                                                                              0, 127);
          } else if constexpr (DA == 1 && DB == 1) {
            acc[0][t][u] = mfma_i8<S16>(a[cur][0][t], b[cur][0][u], acc[0][t][u]);
          } else if constexpr (DB == 1) {
#pragma unroll
            for (int d = 0; d < DA; ++d) acc[d][t][u] = mfma_i8<S16>(a[cur][d][t], b[cur][0][u], acc[d][t][u]);
          } else {
#pragma unroll
            for (int i = 0; i < DA; ++i)
#pragma unroll
              for (int j = 0; j < DB; ++j)
                if (i + j >= 2)
                  acc[i + j - 2][t][u] = mfma_i8<S16>(a[cur][i][t], b[cur][j][u], acc[i + j - 2][t][u]);
          }
        }
      if constexpr (IL == 1) {
        // interleave: one MFMA of step ks, then one LDS fragment read of step ks+1
        constexpr int NLD = DA * TM + DB * TN;
        constexpr int NMF = TM * TN * (DA == 1 ? 1 : (DB == 1 ? DA : 6));
        if (ks + 1 < KSTEPS) {
#pragma unroll
          for (int q = 0; q < NLD; ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, NMF - NLD, 0);
        }
      }
      if constexpr (IL == 2) {
        // one MFMA, then one LDS fragment read of step ks+1 and one of this tile's PER_WAVE
        // LDS-DMA pieces (spread evenly over the KSTEPS steps), then the remaining MFMAs
        constexpr int NLD = DA * TM + DB * TN;
        constexpr int NMF = TM * TN * (DA == 1 ? 1 : (DB == 1 ? DA : 6));
        constexpr int NV = (PER_WAVE + KSTEPS - 1) / KSTEPS;
        const int nv = min(NV, PER_WAVE - ks * NV);
        const int nld = ks + 1 < KSTEPS ? NLD : 0;
        if (ks == 0) __builtin_amdgcn_sched_group_barrier(0x100, NLD, 0);  // fragments of step 0
        const int nq = max(nld, nv);
        int used = 0;
#pragma unroll
        for (int q = 0; q < nq; ++q) {
          if (used < NMF) { __builtin_amdgcn_sched_group_barrier(0x008, 1, 0); ++used; }
          if (q < nld) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          if (q < nv) __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
        }
#pragma unroll
        for (int q = used; q < NMF; ++q) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
    }
    }
    if constexpr (FLUSH) {
      if ((kt + 1) % FLUSH_KT == 0 || kt + 1 == nk) {
#pragma unroll
        for (int t = 0; t < TM; ++t)
#pragma unroll
          for (int u = 0; u < TN; ++u) {
#pragma unroll
            for (int i = 0; i < TR; ++i)
              facc[t][u][i] += (float)((double)acc[2][t][u][i] * 65536.0 + (double)acc[1][t][u][i] * 256.0 +
                                       (double)acc[0][t][u][i]);
#pragma unroll
            for (int c = 0; c < NC; ++c) acc[c][t][u] = AccT{0};
          }
      }
    }
  }

  // ---- epilogue.  C/D map of the 32x32 MFMA: reg i -> tile row (i&3)+8(i>>2)+4h, col lane&31;
  // of the 16x16 MFMA: reg i -> tile row 4(lane>>4)+i, col lane&15.
  // Each 32x32 output patch (one 32x32 tile or 2x2 16x16 tiles) is finished in registers
  // (combine digits, scales, bias), transposed through a per-wave 4 KiB LDS patch (16-B chunks
  // XOR-swizzled by row: conflict-free both ways) and written as whole 128-B row segments with
  // 16-B stores (4 per lane instead of 16 dword stores).
  wait_vmcnt_c<0>();  // no LDS-DMA piece may land in the epilogue's patches
  block_barrier();  // every wave is done reading the last operand stage
  // BST = 1: the statistics instance (bnn_gemm_i8_affine_bnstats); the plain kernels carry none of it
  if constexpr (BST && DA == 1 && DB == 1 && !F4 && !S16 && DIAG == 0) {
    if (p.stat != nullptr) {
      // BatchNorm forward statistics of z = a*(S + coff) + b (the pixel layer; a = b_scale, no
      // a_scale / row_off: host check) per column over this wave row's WM*32 rows of the tile --
      // one chunk of bn_fwd_final_k: the chunk sum and the M2 about the chunk mean, formed in double
      // from the exact integer sums S (sum S, sum S^2 as int32 / int64), with no extra HBM traffic
      const int cr0 = m0 + wm * WM * 32;
      const int cnt = min(WM * 32, p.M - cr0);
      const int64_t chunk = (int64_t)tm * WAVES_M + wm, RN = p.stat_rows * (int64_t)p.N;
#pragma unroll
      for (int u = 0; u < TN; ++u) {
        const int col = n0 + wn * WN * 32 + u * 32 + r;
        // integer sums (|S| <= 128 K: a lane's 16 WM values fit int32, their squares int64)
        int i1 = 0;
        long long i2 = 0;
        if (cr0 + WM * 32 <= p.M) {              // a full chunk (wave-uniform): no row tests
#pragma unroll
          for (int t = 0; t < TM; ++t)
#pragma unroll
            for (int i = 0; i < TR; ++i) {
              const int v = (int)acc[0][t][u][i];
              i1 += v;
              i2 += (long long)v * v;
            }
        } else {
          const int lim = p.M - cr0 - 4 * h;     // this lane's rows below M: offsets < lim
#pragma unroll
          for (int t = 0; t < TM; ++t)
#pragma unroll
            for (int i = 0; i < TR; ++i) {
              const int v = (t * 32 + (i & 3) + 8 * (i >> 2)) < lim ? (int)acc[0][t][u][i] : 0;
              i1 += v;
              i2 += (long long)v * v;
            }
        }
        i1 += __shfl_xor(i1, 32, 64);
        i2 += __shfl_xor(i2, 32, 64);
        if (h == 0 && cnt > 0 && col < p.N) {
          const double s1 = (double)i1, s2 = (double)i2;
          const double a = p.b_scale ? (double)p.b_scale[col] : 1.0;
          const double coff = p.col_off ? (double)p.col_off[col] * p.off_mul : 0.0;
          const double b = p.bias ? (double)p.bias[col] : 0.0;
          p.stat[chunk * p.N + col] = a * (s1 + cnt * coff) + cnt * b;
          const double m2 = s2 - s1 * s1 / cnt;
          p.stat[RN + chunk * p.N + col] = a * a * (m2 > 0.0 ? m2 : 0.0);
        }
      }
    }
  }
  if constexpr (BST && F4 && DIAG == 0) {
    if (p.stat != nullptr) {
      // the next BatchNorm's forward statistics (bnn_gemm_fp4_bnstats): per column over this wave
      // row's WM*32 rows, the chunk sum of the stored z = fl(sum + b) (the value the C / C16 + bias
      // consumers see) and its M2 about the chunk mean, both from double sums in a fixed order --
      // the sum is exact as bn_reduce_k's is, so the batch mean is the same double
      const int cr0 = m0 + wm * WM * 32;
      const int cnt = min(WM * 32, p.M - cr0);
      const int64_t chunk = (int64_t)tm * WAVES_M + wm, RN = p.stat_rows * (int64_t)p.N;
      const bool full = cr0 + WM * 32 <= p.M;
      const int lim = p.M - cr0 - 4 * h;     // this lane's rows below M: offsets < lim
      const Drop dp = drop_resolve(p.stat_drop);
#pragma unroll
      for (int u = 0; u < TN; ++u) {
        const int col = n0 + wn * WN * 32 + u * TS + r;
        const float sb = (p.stat_bias && col < p.N) ? p.stat_bias[col] : 0.f;
        double s1 = 0.0, s2 = 0.0;
        if (dp.on) {
          // the BatchNorm sees drop(z): the element-index mask of its own passes, x * scale kept
#pragma unroll
          for (int t = 0; t < TM; ++t)
#pragma unroll
            for (int i = 0; i < TR; ++i) {
              const int off = S16 ? t * 16 + i : t * 32 + (i & 3) + 8 * (i >> 2);
              const int64_t idx = (int64_t)(cr0 + 4 * h + off) * p.N + col;
              const float xv = acc[0][t][u][i] + sb;
              const float xd = drop_keep(dp, (uint64_t)idx) ? xv * dp.scale : 0.f;
              const double d = (full || off < lim) ? (double)xd : 0.0;
              s1 += d;
              s2 = fma(d, d, s2);
            }
        } else if (full) {
#pragma unroll
          for (int t = 0; t < TM; ++t)
#pragma unroll
            for (int i = 0; i < TR; ++i) {
              const double d = (double)(acc[0][t][u][i] + sb);
              s1 += d;
              s2 = fma(d, d, s2);
            }
        } else {
#pragma unroll
          for (int t = 0; t < TM; ++t)
#pragma unroll
            for (int i = 0; i < TR; ++i) {
              const int off = S16 ? t * 16 + i : t * 32 + (i & 3) + 8 * (i >> 2);
              const double d = off < lim ? (double)(acc[0][t][u][i] + sb) : 0.0;
              s1 += d;
              s2 = fma(d, d, s2);
            }
        }
        if constexpr (S16) {
          s1 += __shfl_xor(s1, 16, 64);
          s2 += __shfl_xor(s2, 16, 64);
        }
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 32, 64);
        if (h == 0 && cnt > 0 && col < p.N) {
          p.stat[chunk * p.N + col] = s1;
          const double m2 = s2 - s1 * s1 / cnt;
          p.stat[RN + chunk * p.N + col] = m2 > 0.0 ? m2 : 0.0;
        }
      }
    }
  }
  float* patch = reinterpret_cast<float*>(smem) + wave * 1024;
  const bool vec_ok = ((p.ldc & 3) == 0) && ((reinterpret_cast<uintptr_t>(p.C) & 15) == 0);
  constexpr int SUB = S16 ? 2 : 1;   // MFMA tiles per patch edge
#pragma unroll
  for (int t = 0; t < WM; ++t) {
    const int trow0 = m0 + wm * WM * 32 + t * 32;
#pragma unroll
    for (int u = 0; u < WN; ++u) {
      const int tcol0 = n0 + wn * WN * 32 + u * 32;
#pragma unroll
      for (int sb = 0; sb < SUB; ++sb) {
        const int lc = sb * TS + r;    // patch column of this lane
        const int col = tcol0 + lc;
        const bool cin = col < p.N;
        const float bb = (p.bias && cin) ? p.bias[col] : 0.f;
        const double bs = (p.b_scale && cin) ? (double)p.b_scale[col] : 1.0;
        const bool offs = p.row_off || p.col_off;
        const double coff = (p.col_off && cin) ? (double)p.col_off[col] * p.off_mul : 0.0;
        const int icoff = (int)coff;   // s20: exact (host check)
#pragma unroll
        for (int sa = 0; sa < SUB; ++sa) {
          const int ti = t * SUB + sa, ui = u * SUB + sb;
#pragma unroll
          for (int i = 0; i < TR; ++i) {
            const int lr = S16 ? sa * 16 + 4 * h + i : (i & 3) + 8 * (i >> 2) + 4 * h;
            const int row = min(trow0 + lr, p.M - 1);
            float f;
            if constexpr (DA == 1 && DB == 1) {
              f = (float)acc[0][ti][ui][i];  // exact: |sum| <= K < 2^24
              if (p.S20lo != nullptr) {
                // the integer S travels through the patch as its bit pattern
                f = __int_as_float((int)acc[0][ti][ui][i] + icoff);
              } else if (offs) {
                double v = (double)acc[0][ti][ui][i] + coff;
                if (p.row_off) v += (double)p.row_off[row] * p.off_mul;
                f = (float)(v * (p.a_scale ? (double)p.a_scale[row] : 1.0) * bs);
              } else if (p.a_scale || p.b_scale)
                f = (float)((double)f * (p.a_scale ? (double)p.a_scale[row] : 1.0) * bs);
            } else {
              double v;
              if constexpr (DB == 1) {
                v = (double)acc[2][ti][ui][i] * 65536.0 + (double)acc[1][ti][ui][i] * 256.0 +
                    (double)acc[0][ti][ui][i];
              } else {
                v = (double)facc[ti][ui][i] * 65536.0;
              }
              if (offs) {
                v += coff;
                if (p.row_off) v += (double)p.row_off[row] * p.off_mul;
              }
              f = (float)(v * bs * (p.a_scale ? (double)p.a_scale[row] : 1.0));
            }
            if (p.bias && p.S20lo == nullptr) f += bb;
            patch[lr * 32 + ((((lc >> 2) ^ (lr & 7)) << 2) | (lc & 3))] = f;
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int ps = 0; ps < 4; ++ps) {
        const int lr = (lane >> 3) + 8 * ps, c4 = lane & 7;
        const float4 v = *reinterpret_cast<const float4*>(patch + lr * 32 + ((c4 ^ (lr & 7)) << 2));
        const int row = trow0 + lr, c0 = tcol0 + 4 * c4;
        if (row >= p.M) continue;
        if (p.S20lo != nullptr) {   // N % 4 == 0, ldc % 4 == 0 (host check): 8 B + 2 B per 4 sums
          const int64_t o = (int64_t)row * p.ldc + c0;
          if (c0 < p.N) {
            const int s0 = __float_as_int(v.x), s1 = __float_as_int(v.y), s2 = __float_as_int(v.z),
                      s3 = __float_as_int(v.w);
            out_store2u(p.S20lo + o, ((uint32_t)s0 & 0xFFFFu) | ((uint32_t)s1 << 16),
                        ((uint32_t)s2 & 0xFFFFu) | ((uint32_t)s3 << 16));
            *reinterpret_cast<uint16_t*>(p.S20hi + (o >> 1)) =
                (uint16_t)((((uint32_t)s0 >> 16) & 0xFu) | ((((uint32_t)s1 >> 16) & 0xFu) << 4) |
                           ((((uint32_t)s2 >> 16) & 0xFu) << 8) | ((((uint32_t)s3 >> 16) & 0xFu) << 12));
          }
          continue;
        }
        if (p.C16 != nullptr) {   // ldc % 4 == 0 (host check): one 8-B store of 4 exact sums
          int16_t* d16 = p.C16 + (int64_t)row * p.ldc + c0;
          if (c0 + 3 < p.N) {
            const uint32_t lo = (uint32_t)(uint16_t)(int16_t)v.x | ((uint32_t)(uint16_t)(int16_t)v.y << 16);
            const uint32_t hi = (uint32_t)(uint16_t)(int16_t)v.z | ((uint32_t)(uint16_t)(int16_t)v.w << 16);
            out_store2u(d16, lo, hi);
          } else {
            const float vs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (c0 + j < p.N) d16[j] = (int16_t)vs[j];
          }
          continue;
        }
        float* dst = p.C + (int64_t)row * p.ldc + c0;
#ifdef GEMM_DIAG_NOSTORE     // timing-only build: the epilogue without its global stores
        if (p.M > 0) continue;
#endif
        if (vec_ok && c0 + 3 < p.N) {
          out_store4f(dst, v);
        } else {
          const float vs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (c0 + j < p.N) dst[j] = vs[j];
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
}

template <int DA, int DB, int WAVES_M, int WAVES_N, int WM, int WN, int STAGES, int BKT, int IL = 0,
          int DIAG = 0, int S16 = 0, int BST = 0>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void gemm_i8_v2_k(GemmParams p) {
  gemm_v2_body<DA, DB, WAVES_M, WAVES_N, WM, WN, STAGES, BKT, IL, DIAG, 0, S16, BST>(p);
}

// FP4 (e2m1) ternary x ternary form: its own kernel name, so traces and the bench's peak lookup
// tell it apart from the int8 forms
template <int WAVES_M, int WAVES_N, int WM, int WN, int STAGES, int BKT, int IL = 0, int S16 = 0, int BST = 0>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void gemm_fp4_k(GemmParams p) {
  gemm_v2_body<1, 1, WAVES_M, WAVES_N, WM, WN, STAGES, BKT, IL, 0, 1, S16, BST>(p);
}

// The FP4 form held to <= 256 registers per lane (two waves per SIMD): 4-wave tiles small enough
// in LDS for two workgroups per CU, so one's epilogue stores drain beside the other's k loop
// (as the FP6 GEMM's half-tile form, bnn_gemm6.hip).
template <int WAVES_M, int WAVES_N, int WM, int WN, int STAGES, int BKT, int IL = 0, int S16 = 0, int BST = 0>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N, 2) void gemm_fp4_h_k(GemmParams p) {
  gemm_v2_body<1, 1, WAVES_M, WAVES_N, WM, WN, STAGES, BKT, IL, 0, 1, S16, BST>(p);
}

template <int WAVES_M, int WAVES_N, int WM, int WN, int STAGES, int BKT, int IL = 0, int S16 = 0, int BST = 0>
int launch_fp4h(GemmParams p, hipStream_t s) {
  constexpr int BM = WAVES_M * WM * 32, BN = WAVES_N * WN * 32;
  p.gm = (p.M + BM - 1) / BM;
  p.gn = (p.N + BN - 1) / BN;
  hipLaunchKernelGGL((gemm_fp4_h_k<WAVES_M, WAVES_N, WM, WN, STAGES, BKT, IL, S16, BST>),
                     dim3((unsigned)((int64_t)p.gm * p.gn)), dim3(64 * WAVES_M * WAVES_N), 0, s, p);
  return check_launch("bnn_gemm_fp4");
}

template <int DA, int DB, int WAVES_M, int WAVES_N, int WM, int WN, int STAGES, int BKT, int IL = 0,
          int DIAG = 0, int F4 = 0, int S16 = 0, int BST = 0>
int launch_v2(GemmParams p, hipStream_t s) {
  constexpr int BM = WAVES_M * WM * 32, BN = WAVES_N * WN * 32;
  p.gm = (p.M + BM - 1) / BM;
  p.gn = (p.N + BN - 1) / BN;
  const int64_t nblk = (int64_t)p.gm * p.gn;
  if constexpr (F4) {
    static_assert(DA == 1 && DB == 1 && DIAG == 0, "FP4 form");
    hipLaunchKernelGGL((gemm_fp4_k<WAVES_M, WAVES_N, WM, WN, STAGES, BKT, IL, S16, BST>), dim3((unsigned)nblk),
                       dim3(64 * WAVES_M * WAVES_N), 0, s, p);
    return check_launch("bnn_gemm_fp4");
  } else {
    hipLaunchKernelGGL((gemm_i8_v2_k<DA, DB, WAVES_M, WAVES_N, WM, WN, STAGES, BKT, IL, DIAG, S16, BST>),
                       dim3((unsigned)nblk), dim3(64 * WAVES_M * WAVES_N), 0, s, p);
    return check_launch("bnn_gemm_i8");
  }
}

int g_variant = -1;  // tuning hook (bnn_gemm_set_variant); -1 = default table
int g_raster = 0;    // tuning hook (bnn_gemm_set_raster): GemmParams::raster of the affine entry

template <int DA, int DB, int WM, int WN>
int launch(GemmParams p, hipStream_t s) {
  constexpr int BM = 64 * WM, BN = 64 * WN;
  p.gm = (p.M + BM - 1) / BM;
  p.gn = (p.N + BN - 1) / BN;
  const int64_t nblk = (int64_t)p.gm * p.gn;
  hipLaunchKernelGGL((gemm_i8_k<DA, DB, WM, WN>), dim3((unsigned)nblk), dim3(256), 0, s, p);
  return check_launch("bnn_gemm_i8");
}

// Kernel table; the default choice per digit configuration and shape comes from
// tools/gemm_sweep.py on MI355X (profiles/r01_gemm_sweep*.log).
struct Variant {
  int id;
  const char* name;  // as rocprofv3 lists the instance
  int (*fn)(GemmParams, hipStream_t);
  int bk;
};

const Variant kVariants[] = {
    {0, "gemm_i8_k<1, 1, 2, 2>", launch<1, 1, 2, 2>, 64},
    {1, "gemm_i8_v2_k<1, 1, 2, 2, 2, 2, 3, 64, 0, 0, 0>", launch_v2<1, 1, 2, 2, 2, 2, 3, 64>, 64},
    {2, "gemm_i8_v2_k<1, 1, 2, 4, 4, 2, 3, 64, 0, 0, 0>", launch_v2<1, 1, 2, 4, 4, 2, 3, 64>, 64},
    {3, "gemm_i8_v2_k<1, 1, 2, 4, 4, 2, 2, 128, 0, 0, 0>", launch_v2<1, 1, 2, 4, 4, 2, 2, 128>, 128},
    {4, "gemm_i8_v2_k<1, 1, 2, 2, 4, 4, 2, 64, 0, 0, 0>", launch_v2<1, 1, 2, 2, 4, 4, 2, 64>, 64},
    {5, "gemm_i8_v2_k<1, 1, 2, 4, 4, 2, 4, 64, 0, 0, 0>", launch_v2<1, 1, 2, 4, 4, 2, 4, 64>, 64},
    {6, "gemm_i8_v2_k<1, 1, 2, 4, 4, 2, 2, 128, 1, 0, 0>", launch_v2<1, 1, 2, 4, 4, 2, 2, 128, 1>, 128},
    // 16x16 MFMA shape (S16) of variants 3/6, 14, 33 (DVFS: higher clock held on 16x16)
    {7, "gemm_i8_v2_k<1, 1, 2, 4, 4, 2, 2, 128, 0, 0, 1>", launch_v2<1, 1, 2, 4, 4, 2, 2, 128, 0, 0, 0, 1>, 128},
    {8, "gemm_i8_v2_k<1, 1, 2, 4, 4, 2, 2, 128, 1, 0, 1>", launch_v2<1, 1, 2, 4, 4, 2, 2, 128, 1, 0, 0, 1>, 128},
    {17, "gemm_i8_v2_k<3, 1, 2, 4, 2, 2, 2, 128, 0, 0, 1>", launch_v2<3, 1, 2, 4, 2, 2, 2, 128, 0, 0, 0, 1>, 128},
    {18, "gemm_i8_v2_k<3, 1, 2, 4, 2, 2, 2, 128, 2, 0, 1>", launch_v2<3, 1, 2, 4, 2, 2, 2, 128, 2, 0, 0, 1>, 128},
    {34, "gemm_fp4_k<2, 4, 4, 2, 2, 128, 0, 1>", launch_v2<1, 1, 2, 4, 4, 2, 2, 128, 0, 0, 1, 1>, 128},
    {35, "gemm_fp4_k<2, 4, 4, 2, 2, 128, 1, 1>", launch_v2<1, 1, 2, 4, 4, 2, 2, 128, 1, 0, 1, 1>, 128},
    // IL = 2: LDS-DMA pieces spread between the MFMAs (9, 18, 36: 16x16; 19: 16x16 + B prefetch)
    {9, "gemm_i8_v2_k<1, 1, 2, 4, 4, 2, 2, 128, 2, 0, 1>", launch_v2<1, 1, 2, 4, 4, 2, 2, 128, 2, 0, 0, 1>, 128},
    {19, "gemm_i8_v2_k<3, 1, 2, 4, 2, 2, 2, 128, 0, 3, 1>", launch_v2<3, 1, 2, 4, 2, 2, 2, 128, 0, 3, 0, 1>, 128},
    {36, "gemm_fp4_k<2, 4, 4, 2, 2, 128, 2, 1>", launch_v2<1, 1, 2, 4, 4, 2, 2, 128, 2, 0, 1, 1>, 128},
    {77, "diag: v6 without LDS fragment reads", launch_v2<1, 1, 2, 4, 4, 2, 2, 128, 1, 1>, 128},
    {78, "diag: v6 without global->LDS staging", launch_v2<1, 1, 2, 4, 4, 2, 2, 128, 1, 2>, 128},
    {10, "gemm_i8_k<3, 1, 2, 2>", launch<3, 1, 2, 2>, 64},
    {11, "gemm_i8_v2_k<3, 1, 2, 2, 2, 2, 3, 64, 0, 0, 0>", launch_v2<3, 1, 2, 2, 2, 2, 3, 64>, 64},
    {12, "gemm_i8_v2_k<3, 1, 4, 2, 2, 2, 2, 64, 0, 0, 0>", launch_v2<3, 1, 4, 2, 2, 2, 2, 64>, 64},
    {13, "gemm_i8_v2_k<3, 1, 2, 4, 2, 1, 3, 64, 0, 0, 0>", launch_v2<3, 1, 2, 4, 2, 1, 3, 64>, 64},
    {14, "gemm_i8_v2_k<3, 1, 2, 4, 2, 2, 2, 128, 0, 0, 0>", launch_v2<3, 1, 2, 4, 2, 2, 2, 128>, 128},
    {15, "gemm_i8_v2_k<3, 1, 2, 4, 2, 2, 3, 64, 0, 0, 0>", launch_v2<3, 1, 2, 4, 2, 2, 3, 64>, 64},
    {16, "gemm_i8_v2_k<3, 1, 2, 4, 2, 2, 4, 64, 0, 0, 0>", launch_v2<3, 1, 2, 4, 2, 2, 4, 64>, 64},
    // timing-only diagnostics (wrong results; never picked by default)
    {97, "diag: v14 without LDS fragment reads", launch_v2<3, 1, 2, 4, 2, 2, 2, 128, 0, 1>, 128},
    {98, "diag: v14 without global->LDS staging", launch_v2<3, 1, 2, 4, 2, 2, 2, 128, 0, 2>, 128},
    {20, "gemm_i8_k<3, 3, 2, 1>", launch<3, 3, 2, 1>, 64},
    // FP4 (e2m1) ternary x ternary forms (bnn_gemm_fp4): K in bytes, 2 elements per byte
    {30, "gemm_fp4_k<2, 4, 4, 2, 2, 128, 1, 0>", launch_v2<1, 1, 2, 4, 4, 2, 2, 128, 1, 0, 1>, 128},
    {31, "gemm_fp4_k<2, 2, 2, 2, 3, 64, 0, 0>", launch_v2<1, 1, 2, 2, 2, 2, 3, 64, 0, 0, 1>, 64},
    {32, "gemm_fp4_k<2, 4, 4, 2, 3, 64, 0, 0>", launch_v2<1, 1, 2, 4, 4, 2, 3, 64, 0, 0, 1>, 64},
    {33, "gemm_fp4_k<2, 4, 4, 2, 2, 128, 0, 0>", launch_v2<1, 1, 2, 4, 4, 2, 2, 128, 0, 0, 1>, 128},
    // two workgroups per CU (A/B sweep, tools/fp4_half_ab.py): 128 x 256 tiles with BK 64 (3 / 2
    // stages), 128 x 128 tiles of 2 waves with BK 128 + 16x16 MFMAs
    {37, "gemm_fp4_h_k<1, 4, 4, 2, 3, 64, 0, 0>", launch_fp4h<1, 4, 4, 2, 3, 64, 0, 0>, 64},
    {38, "gemm_fp4_h_k<1, 4, 4, 2, 2, 64, 0, 0>", launch_fp4h<1, 4, 4, 2, 2, 64, 0, 0>, 64},
    {39, "gemm_fp4_h_k<1, 2, 4, 2, 2, 128, 2, 1>", launch_fp4h<1, 2, 4, 2, 2, 128, 2, 1>, 128},
    {21, "gemm_i8_v2_k<3, 3, 2, 2, 2, 1, 2, 64, 0, 0, 0>", launch_v2<3, 3, 2, 2, 2, 1, 2, 64>, 64},
    {22, "gemm_i8_v2_k<3, 3, 2, 4, 2, 1, 2, 64, 0, 0, 0>", launch_v2<3, 3, 2, 4, 2, 1, 2, 64>, 64},
};

const Variant* find_variant(int id) {
  for (const Variant& v : kVariants)
    if (v.id == id) return &v;
  return nullptr;
}

const Variant* pick_kernel(int a_digits, int b_digits, int64_t M, int64_t N, int64_t K) {
  if (a_digits == 0) {  // FP4 ternary form; K in bytes
    const bool big = ((M + 255) / 256) * ((N + 255) / 256) >= 512;
    int id = g_variant >= 0 ? 30 + g_variant : (big ? 36 : 31);   // sweep r01: 36 = 0.435 of FP4 peak
    const Variant* v = find_variant(id);
    if (v == nullptr) v = find_variant(31);
    if (K % v->bk != 0) v = find_variant(big ? 32 : 31);
    return v;
  }
  const int base = a_digits == 1 ? 0 : (b_digits == 1 ? 10 : 20);
  int id, alt;  // alt = the BK=64 sibling used when K % 128 != 0
  if (g_variant >= 0) {
    id = base + g_variant;
    alt = base + 1;
  } else if (a_digits == 1) {   // sweep r01: 256x256 BK128 16x16-MFMA + DMA spread 0.49 of peak; 128x128 on small grids
    const bool big = ((M + 255) / 256) * ((N + 255) / 256) >= 512;
    id = big ? 9 : 1;
    alt = big ? 2 : 1;
  } else if (b_digits == 1) {   // 128x256 BK128 8 waves 16x16-MFMA + DMA spread: 0.51-0.56 of peak on dX / dW
    const bool big = ((M + 127) / 128) * ((N + 255) / 256) >= 256;
    id = big ? 18 : 13;
    alt = big ? 15 : 13;
  } else {
    id = 22;
    alt = 22;
  }
  const Variant* v = find_variant(id);
  if (v == nullptr) v = find_variant(base + 1);
  if (K % v->bk != 0) v = find_variant(alt);
  return v;
}

}  // namespace
}  // namespace bnn

using namespace bnn;

BNN_API int bnn_gemm_i8_affine(const int8_t* A, int64_t lda, int64_t a_plane, int32_t a_digits,
                               const int8_t* B, int64_t ldb, int64_t b_plane, int32_t b_digits,
                               const float* a_scale, const float* b_scale, const float* bias,
                               const int64_t* row_off, const int64_t* col_off, double off_mul, float* C,
                               int64_t ldc, int64_t M, int64_t N, int64_t K, void* stream) {
  const bool cfg_ok = (a_digits == 1 && b_digits == 1) || (a_digits == 3 && b_digits == 1) ||
                      (a_digits == 3 && b_digits == 3);
  if (!A || !B || !C || !cfg_ok || M < 0 || N < 0 || K <= 0 || K % BK != 0 || lda < K || ldb < K ||
      lda % 16 != 0 || ldb % 16 != 0 || ldc < N || !aligned16(A) || !aligned16(B) ||
      M > 0x7fffffff || N > 0x7fffffff || K > 0x7fffffff ||
      (a_digits > 1 && (a_plane < M * lda || a_plane % 16 != 0)) ||
      (b_digits > 1 && (b_plane < N * ldb || b_plane % 16 != 0))) {
    set_error("bnn_gemm_i8_affine: bad arguments (M=%lld N=%lld K=%lld lda=%lld ldb=%lld digits=%d,%d; "
              "K must be a positive multiple of 64)",
              (long long)M, (long long)N, (long long)K, (long long)lda, (long long)ldb, a_digits,
              b_digits);
    return kErrInval;
  }
  if (M == 0 || N == 0) return 0;
  GemmParams p{A, B, lda, ldb, a_plane, b_plane, a_scale, b_scale, bias, C, ldc,
               (int)M, (int)N, (int)K, 0, 0, row_off, col_off, off_mul};
  p.raster = g_raster;
  // v2 kernels address a tile's rows with 32-bit per-lane offsets (< 256 rows x ld)
  if (lda * 256 >= (1LL << 31) || ldb * 256 >= (1LL << 31))
    return find_variant(a_digits == 1 ? 0 : (b_digits == 1 ? 10 : 20))->fn(p, reinterpret_cast<hipStream_t>(stream));
  return pick_kernel(a_digits, b_digits, M, N, K)->fn(p, reinterpret_cast<hipStream_t>(stream));
}

// The statistics form runs the 32x32 (1,1) kernels only: 128x128 tiles (64-row chunks) on grids
// below 512 of the 256x256 tiles (128-row chunks), as pick_kernel's BK=64 choices
// bnn_gemm_i8_bnstats_set_tile: 0 = by grid size (above), 1 = always the 128 x 128 tile, 2 = always
// 256 x 256 (A/B hook; the chunk query and the launch read the same setting)
static int g_i8_bnstats_tile = 0;

static const Variant* i8_bnstats_variant(int64_t M, int64_t N) {
  const bool big = ((M + 255) / 256) * ((N + 255) / 256) >= 512;
  if (g_i8_bnstats_tile != 0) return find_variant(g_i8_bnstats_tile == 2 ? 2 : 1);
  return find_variant(big ? 2 : 1);
}

BNN_API int32_t bnn_gemm_i8_bnstats_set_tile(int32_t tile) {
  if (tile < 0) return g_i8_bnstats_tile;
  if (tile > 2) return kErrInval;
  g_i8_bnstats_tile = tile;
  return 0;
}

BNN_API int64_t bnn_gemm_i8_bnstats_chunk(int64_t M, int64_t N) {
  return i8_bnstats_variant(M, N)->id == 2 ? 128 : 64;
}

// The shape bounds of the statistics form (the plain kernel has fallbacks where it has none)
static bool i8_bnstats_shape_ok(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb) {
  return M > 0 && N > 0 && K > 0 && K % BK == 0 && lda >= K && ldb >= K && lda % 16 == 0 && ldb % 16 == 0 &&
         M <= 0x7fffffff && N <= 0x7fffffff && K <= 0x7fffffff && lda * 256 < (1LL << 31) &&
         ldb * 256 < (1LL << 31) &&
         // |S| <= 128 K: sum S^2 over a column stays an exact double below 2^53
         (double)M * (128.0 * K) * (128.0 * K) < 9007199254740992.0;
}

BNN_API int bnn_gemm_i8_bnstats_ok(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb) {
  return i8_bnstats_shape_ok(M, N, K, lda, ldb) ? 1 : 0;
}

BNN_API int bnn_gemm_i8_affine_bnstats(const int8_t* A, int64_t lda, const int8_t* B, int64_t ldb,
                                       const float* b_scale, const float* bias, const int64_t* col_off,
                                       double off_mul, float* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                                       double* stat, int64_t stat_rows, void* stream) {
  const int64_t chunk = M > 0 ? bnn_gemm_i8_bnstats_chunk(M, N) : 1;
  if (!A || !B || !C || !stat || !i8_bnstats_shape_ok(M, N, K, lda, ldb) || ldc < N || !aligned16(A) ||
      !aligned16(B) || stat_rows != (M + chunk - 1) / chunk) {
    set_error("bnn_gemm_i8_affine_bnstats: bad arguments (M=%lld N=%lld K=%lld stat_rows=%lld; want %lld)",
              (long long)M, (long long)N, (long long)K, (long long)stat_rows, (long long)((M + chunk - 1) / chunk));
    return kErrInval;
  }
  GemmParams p{A, B, lda, ldb, 0, 0, nullptr, b_scale, bias, C, ldc,
               (int)M, (int)N, (int)K, 0, 0, nullptr, col_off, off_mul};
  p.stat = stat;
  p.stat_rows = stat_rows;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  return i8_bnstats_variant(M, N)->id == 2 ? launch_v2<1, 1, 2, 4, 4, 2, 3, 64, 0, 0, 0, 0, 1>(p, st)
                                           : launch_v2<1, 1, 2, 2, 2, 2, 3, 64, 0, 0, 0, 0, 1>(p, st);
}

// bnn_gemm_i8_affine_bnstats writing the s20 form of z (XIn XF 2): z = fl(fl(S * a) + bias) with
// S = sum + s0 * col_off[n] read back by the *_s20 BatchNorm entries, bit-identical to the fp32 z.
// Needs an integral s0 (ToTensor without Normalize) and |S| <= K (128 + |s0|) < 2^19; N % 4 == 0.
BNN_API int bnn_gemm_i8_s20_ok(int64_t M, int64_t N, int64_t K, int64_t k_true, double s0) {
  return (N % 4 == 0 && s0 == (double)(int64_t)s0 && k_true > 0 && k_true <= K &&
          (double)k_true * (128.0 + fabs(s0)) < 524288.0)
             ? 1
             : 0;
}

BNN_API int bnn_gemm_i8_affine_bnstats_s20(const int8_t* A, int64_t lda, const int8_t* B, int64_t ldb,
                                           const int64_t* col_off, double off_mul, int64_t k_true, int16_t* Slo,
                                           uint8_t* Shi, int64_t ldc, int64_t M, int64_t N, int64_t K, double* stat,
                                           int64_t stat_rows, const float* b_scale, const float* bias, void* stream) {
  const int64_t chunk = M > 0 ? bnn_gemm_i8_bnstats_chunk(M, N) : 1;
  if (!A || !B || !Slo || !Shi || !col_off || !stat || !i8_bnstats_shape_ok(M, N, K, lda, ldb) || ldc < N ||
      ldc % 4 != 0 || !aligned16(A) || !aligned16(B) || (reinterpret_cast<uintptr_t>(Slo) & 7) != 0 ||
      (reinterpret_cast<uintptr_t>(Shi) & 1) != 0 || !bnn_gemm_i8_s20_ok(M, N, K, k_true, off_mul) ||
      stat_rows != (M + chunk - 1) / chunk) {
    set_error("bnn_gemm_i8_affine_bnstats_s20: bad arguments (M=%lld N=%lld K=%lld k_true=%lld off_mul=%g "
              "stat_rows=%lld)", (long long)M, (long long)N, (long long)K, (long long)k_true, off_mul,
              (long long)stat_rows);
    return kErrInval;
  }
  // b_scale / bias enter only the statistics (the stored S carries neither)
  GemmParams p{A, B, lda, ldb, 0, 0, nullptr, b_scale, bias, nullptr, ldc,
               (int)M, (int)N, (int)K, 0, 0, nullptr, col_off, off_mul};
  p.stat = stat;
  p.stat_rows = stat_rows;
  p.S20lo = Slo;
  p.S20hi = Shi;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  return i8_bnstats_variant(M, N)->id == 2 ? launch_v2<1, 1, 2, 4, 4, 2, 3, 64, 0, 0, 0, 0, 1>(p, st)
                                           : launch_v2<1, 1, 2, 2, 2, 2, 3, 64, 0, 0, 0, 0, 1>(p, st);
}

BNN_API int bnn_gemm_i8(const int8_t* A, int64_t lda, int64_t a_plane, int32_t a_digits,
                        const int8_t* B, int64_t ldb, int64_t b_plane, int32_t b_digits,
                        const float* a_scale, const float* b_scale, const float* bias, float* C,
                        int64_t ldc, int64_t M, int64_t N, int64_t K, void* stream) {
  return bnn_gemm_i8_affine(A, lda, a_plane, a_digits, B, ldb, b_plane, b_digits, a_scale, b_scale, bias,
                            nullptr, nullptr, 0.0, C, ldc, M, N, K, stream);
}

BNN_API int bnn_gemm_fp4(const uint8_t* A, int64_t lda, const uint8_t* B, int64_t ldb, const float* bias,
                         float* C, int64_t ldc, int64_t M, int64_t N, int64_t K, void* stream) {
  if (!A || !B || !C || M < 0 || N < 0 || K <= 0 || K % BK != 0 || lda < K || ldb < K || lda % 16 != 0 ||
      ldb % 16 != 0 || ldc < N || !aligned16(A) || !aligned16(B) || M > 0x7fffffff || N > 0x7fffffff ||
      K > 0x7fffffff || lda * 256 >= (1LL << 31) || ldb * 256 >= (1LL << 31)) {
    set_error("bnn_gemm_fp4: bad arguments (M=%lld N=%lld K=%lld bytes; K must be a positive multiple of 64 "
              "and below 2^23 bytes)",
              (long long)M, (long long)N, (long long)K);
    return kErrInval;
  }
  if (M == 0 || N == 0) return 0;
  GemmParams p{reinterpret_cast<const int8_t*>(A), reinterpret_cast<const int8_t*>(B), lda, ldb, 0, 0,
               nullptr, nullptr, bias, C, ldc, (int)M, (int)N, (int)K, 0, 0, nullptr, nullptr, 0.0};
  return pick_kernel(0, 0, M, N, K)->fn(p, reinterpret_cast<hipStream_t>(stream));
}

BNN_API int bnn_gemm_fp4_i16(const uint8_t* A, int64_t lda, const uint8_t* B, int64_t ldb, int16_t* C16,
                             int64_t ldc, int64_t M, int64_t N, int64_t K, void* stream) {
  // K bytes = 2K ternary products per output: |sum| <= 2K must fit int16
  if (!C16 || ldc % 4 != 0 || (reinterpret_cast<uintptr_t>(C16) & 7) != 0 || 2 * K > 32767) {
    set_error("bnn_gemm_fp4_i16: bad arguments (ldc=%lld, K=%lld bytes; ldc %% 4 == 0, 8-B aligned output, "
              "2K <= 32767)", (long long)ldc, (long long)K);
    return kErrInval;
  }
  if (!A || !B || M < 0 || N < 0 || K <= 0 || K % BK != 0 || lda < K || ldb < K || lda % 16 != 0 ||
      ldb % 16 != 0 || ldc < N || !aligned16(A) || !aligned16(B) || M > 0x7fffffff || N > 0x7fffffff ||
      lda * 256 >= (1LL << 31) || ldb * 256 >= (1LL << 31)) {
    set_error("bnn_gemm_fp4_i16: bad arguments (M=%lld N=%lld K=%lld bytes)", (long long)M, (long long)N,
              (long long)K);
    return kErrInval;
  }
  if (M == 0 || N == 0) return 0;
  GemmParams p{reinterpret_cast<const int8_t*>(A), reinterpret_cast<const int8_t*>(B), lda, ldb, 0, 0,
               nullptr, nullptr, nullptr, nullptr, ldc, (int)M, (int)N, (int)K, 0, 0, nullptr, nullptr, 0.0, C16};
  return pick_kernel(0, 0, M, N, K)->fn(p, reinterpret_cast<hipStream_t>(stream));
}

// The FP4 forward with the next BatchNorm's forward statistics (its own instances of the default
// choices: 256x256 tiles with 128-row chunks on big grids, 128x128 with 64-row chunks otherwise)
// 0: no statistics form for this shape (the big-grid BK=64 fallback, K % 128 != 0, would spill)
BNN_API int64_t bnn_gemm_fp4_bnstats_chunk(int64_t M, int64_t N, int64_t K) {
  const int id = pick_kernel(0, 0, M, N, K)->id;
  return id == 31 ? 64 : (id == 36 ? 128 : 0);
}

BNN_API int bnn_gemm_fp4_bnstats(const uint8_t* A, int64_t lda, const uint8_t* B, int64_t ldb, const float* bias,
                                 float* C, int16_t* C16, int64_t ldc, const float* zbias, int64_t M, int64_t N,
                                 int64_t K, float drop_p, uint64_t drop_seed, double* stat, int64_t stat_rows,
                                 void* stream) {
  if (!(drop_p >= 0.f && drop_p < 1.f)) {
    set_error("bnn_gemm_fp4_bnstats: drop_p must be in [0, 1) (got %g)", (double)drop_p);
    return kErrInval;
  }
  const int64_t chunk = (M > 0 && N > 0 && K > 0) ? bnn_gemm_fp4_bnstats_chunk(M, N, K) : 1;
  const bool c16 = C16 != nullptr;
  if (chunk <= 0 || !A || !B || (C == nullptr) == (C16 == nullptr) || (c16 && bias) || !stat || M <= 0 || N <= 0 || K <= 0 ||
      K % BK != 0 || lda < K || ldb < K || lda % 16 != 0 || ldb % 16 != 0 || ldc < N || !aligned16(A) ||
      !aligned16(B) || M > 0x7fffffff || N > 0x7fffffff || lda * 256 >= (1LL << 31) || ldb * 256 >= (1LL << 31) ||
      (c16 && (ldc % 4 != 0 || (reinterpret_cast<uintptr_t>(C16) & 7) != 0 || 2 * K > 32767)) ||
      stat_rows != (M + chunk - 1) / chunk) {
    set_error("bnn_gemm_fp4_bnstats: bad arguments (M=%lld N=%lld K=%lld bytes, stat_rows=%lld; one of C / C16, "
              "no bias with C16)", (long long)M, (long long)N, (long long)K, (long long)stat_rows);
    return kErrInval;
  }
  GemmParams p{reinterpret_cast<const int8_t*>(A), reinterpret_cast<const int8_t*>(B), lda, ldb, 0, 0,
               nullptr, nullptr, bias, C, ldc, (int)M, (int)N, (int)K, 0, 0, nullptr, nullptr, 0.0, C16};
  p.stat = stat;
  p.stat_rows = stat_rows;
  p.stat_bias = zbias;
  p.stat_drop = make_drop(drop_p, drop_seed);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  return chunk == 128 ? launch_v2<1, 1, 2, 4, 4, 2, 2, 128, 2, 0, 1, 1, 1>(p, st)
                      : launch_v2<1, 1, 2, 2, 2, 2, 3, 64, 0, 0, 1, 0, 1>(p, st);
}

BNN_API const char* bnn_gemm_i8_kernel(int32_t a_digits, int32_t b_digits, int64_t M, int64_t N,
                                       int64_t K) {
  // same fallback rule as bnn_gemm_i8 (K here is the padded row length the caller passes as lda);
  // the FP4 form has no fallback (bnn_gemm_fp4 rejects such shapes)
  if (a_digits != 0 && K * 256 >= (1LL << 31)) return find_variant(a_digits == 1 ? 0 : (b_digits == 1 ? 10 : 20))->name;
  return pick_kernel(a_digits, b_digits, M, N, K)->name;
}

// Tuning hook: select a kernel variant for every later bnn_gemm_i8 call in this process
// (-1 = built-in default).  Not part of the stable ABI contract; used by tools/gemm_sweep.py.
BNN_API int bnn_gemm_set_raster(int32_t r) {
  g_raster = r;
  return 0;
}

BNN_API int bnn_gemm_set_variant(int32_t v) {
  g_variant = v;
  return 0;
}
