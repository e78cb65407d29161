/* libbnn -- MI355X (gfx950) binarized-network training hot path, C ABI.
 *
 * Drop-in boundary: the reference exposes no FFI; its operator API is the Python module
 * models/binarized_modules.py (Binarize :11-15, BinarizeLinear :68-85, BinarizeConv2d :87-107)
 * plus the DDP gradient exchange the trainers wrap around it (mnist-dist2.py:93, fires inside
 * loss.backward() at :130).  Each entry point below replaces the torch/ATen work that interface
 * triggers; the "replaces" line names the reference call site.  The Python mirror of the
 * operator API (distributed-mnist-bnns_amd/models/binarized_modules.py) binds these through
 * ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - Every pointer is a device pointer (hipMalloc / torch caching allocator) unless noted.
 *  - All sizes are element counts (int64).  Row-major; "ld" = row stride in elements.
 *  - `stream` is a hipStream_t (NULL = legacy default stream).  Calls are asynchronous,
 *    allocate nothing, never synchronise, and are safe to capture into a hipGraph.
 *  - Return value: 0 = ok; BNN_EINVAL (-1) = invalid argument (nothing launched);
 *    >0 = hipError_t of a failed launch.  bnn_last_error() describes the last failure
 *    (thread-local).
 *  - Ternary operands: int8 {-1,0,+1} = Tensor.sign() of fp32 (sign(0) = 0).
 *  - Digit operands (fp32 values entering a GEMM): D planes of int8 balanced base-256 digits
 *    plus one power-of-two scale per row; see DESIGN.md "fp32 operands on the int8 MFMA".
 */
#ifndef BNN_H_
#define BNN_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BNN_EINVAL (-1)

typedef void* bnn_stream_t; /* hipStream_t */

/* ---------------------------------------------------------------- library */
int bnn_version(void);
const char* bnn_last_error(void);

/* ---------------------------------------------------------------- (1) sign-and-pack
 * replaces: Binarize(tensor) = tensor.sign()   models/binarized_modules.py:11-13,
 *           as called on inputs (:76, :95) and latent weights (:79, :98).
 *
 * x fp32 [M][K] (row stride ldx) ->
 *   q   int8 [M][ldq]    ternary, columns K..ldq-1 zero-filled          (nullable)
 *   qt  int8 [K][ldqt]   ternary transpose, columns M..ldqt-1 zero-filled (nullable)
 * ldq >= round_up(K,64) and ldqt >= round_up(M,64), both multiples of 64; q, qt 16-B aligned. */
int bnn_sign_pack_i8(const float* x, int64_t M, int64_t K, int64_t ldx, int8_t* q, int64_t ldq,
                     int8_t* qt, int64_t ldqt, bnn_stream_t stream);

/* FP4 form of the ternary rows for bnn_gemm_fp4: q4 [M][ldq4 bytes], ldq4 a multiple of 128 with
 * 2*ldq4 >= round_up(K,256) (zero nibbles beyond K).  qt = the transpose [K][ldqt] for the
 * backward GEMMs: qt_fmt 0 = int8 as in bnn_sign_pack_i8; qt_fmt 1 = FP4 nibbles, ldqt BYTES (a
 * multiple of 128, 2*ldqt >= round_up(M,256)), the B operand of bnn_gemm_fp6; qt_fmt 2 = the same
 * nibbles in the panel layout of bnn_gemm_fp6_panel_ws ([ceil(K/512)][ldqt/32][512][32 B], bks =
 * ldqt/32; rows beyond K unspecified). */
int bnn_sign_pack_fp4(const float* x, int64_t M, int64_t K, int64_t ldx, uint8_t* q4, int64_t ldq4,
                      int8_t* qt, int64_t ldqt, int32_t qt_fmt, bnn_stream_t stream);

/* y[i] = sign(x[i]) as fp32 (the caller-visible `input.data = Binarize(input.data)` of :76/:95;
 * y may alias x). */
int bnn_sign_f32(const float* x, float* y, int64_t n, bnn_stream_t stream);

/* bnn_sign_pack_fp4 (ldx = K; q4 and qt both, qt_fmt 1 rows / 2 panels) that also writes the fp32
 * sign sout[m][k] = sign(x[m][k]) -- the BinarizeLinear input write-back of :76 -- from the same read
 * of x (256 x 256 tiles: K % 256 == 0, >= 1024 tiles; else the two passes).  sout may alias x. */
int bnn_sign_pack_fp4_out(const float* x, int64_t M, int64_t K, uint8_t* q4, int64_t ldq4, int8_t* qt,
                          int64_t ldqt, int32_t qt_fmt, float* sout, bnn_stream_t stream);

/* Bit-planes for the XNOR-popcount path: word w of row m holds k = 32w..32w+31 (bit k%32);
 * sbits = 1 where x<0, nzbits = 1 where x!=0.  ldw >= ceil(K/32) words, padding words zeroed. */
int bnn_sign_pack_bits(const float* x, int64_t M, int64_t K, int64_t ldx, uint32_t* sbits,
                       uint32_t* nzbits, int64_t ldw, bnn_stream_t stream);

/* ---------------------------------------------------------------- fp32 -> digit operands
 * Row-scaled digits: for each row m of x [M][K], scale[m] = 2^(E-22) with max|x[m,:]| in
 * [2^(E-1), 2^E), digits[d][m][k] (d = 0,1,2; plane stride `plane`) with
 * x ~= scale*(d2*65536 + d1*256 + d0).  Columns K..ldq-1 zero-filled.
 * replaces: the fp32 operand of F.linear / autograd (x of fc1 :80, dY of every backward). */
int bnn_quant_rows(const float* x, int64_t M, int64_t K, int64_t ldx, int8_t* digits, int64_t ldq,
                   int64_t plane, float* scale, bnn_stream_t stream);

/* Column-scaled, transposed digits: for each column n of x [M][N], scale[n] from max|x[:,n]|,
 * digits_t[d][n][m] (plane stride `plane`, row stride ldqt >= round_up(M,64), padding zeroed).
 * colsum (nullable) receives sum_m x[m,n] (double accumulation, fixed order): the bias
 * gradient dB = sum_B dY of BinarizeLinear (:81-83).  `work` is scratch of
 * bnn_quant_cols_workspace(M,N) bytes. */
int64_t bnn_quant_cols_workspace(int64_t M, int64_t N);
int bnn_quant_cols_t(const float* x, int64_t M, int64_t N, int64_t ldx, int8_t* digits_t,
                     int64_t ldqt, int64_t plane, float* scale, float* colsum, void* work,
                     bnn_stream_t stream);
/* bnn_quant_cols_t that also writes dsum[n] = sum_m (d2*2^16 + d1*2^8 + d0)[n][m], the exact
 * integer column sum of the digits (the T[n] of bnn_gemm_i8_affine's row_off); dsum nullable. */
int bnn_quant_cols_t_dsum(const float* x, int64_t M, int64_t N, int64_t ldx, int8_t* digits_t,
                          int64_t ldqt, int64_t plane, float* scale, float* colsum, int64_t* dsum,
                          void* work, bnn_stream_t stream);

/* ---------------------------------------------------------------- (2) forward GEMM, int8 MFMA
 * C[m][n] = cvt( sum_{i,j} 2^(8(i+j)) * sum_k A_i[m][k]*B_j[n][k] ) * a_scale[m] * b_scale[n]
 *           + bias[n]
 * A: a_digits planes (1 or 3) of int8 [M][lda] (plane stride a_plane), B: b_digits planes
 * (1 or 3) of int8 [N][ldb].  (a_digits,b_digits) in {(1,1),(3,1),(3,3)}.  K (the padded
 * reduction length) must be a multiple of 64 and <= lda, ldb; lda, ldb multiples of 16;
 * A, B 16-B aligned; a_scale/b_scale/bias nullable.  Integer sums are exact; the
 * (1,1) form with bias is bit-exact against F.linear(x_b, W_b) + bias (:80-83).
 * replaces: F.linear in BinarizeLinear.forward (:80) and the two GEMMs of its autograd
 * (dX = dY.W_b, dW = dY^T.X_b). */
int bnn_gemm_i8(const int8_t* A, int64_t lda, int64_t a_plane, int32_t a_digits,
                const int8_t* B, int64_t ldb, int64_t b_plane, int32_t b_digits,
                const float* a_scale, const float* b_scale, const float* bias, float* C,
                int64_t ldc, int64_t M, int64_t N, int64_t K, bnn_stream_t stream);

/* bnn_gemm_i8 with integer offsets folded into the raw sum before any rounding:
 * C[m][n] = (combine(sums) + off_mul * (row_off[m] + col_off[n])) * a_scale[m] * b_scale[n]
 *           + bias[n]        (the bracket and products in double, one rounding to fp32)
 * row_off / col_off nullable int64 (NULL both: this IS bnn_gemm_i8).  For u8 pixels
 * (bnn_pixels_pack, v = u - 128, off_mul = 128 for ToTensor): fc1 with col_off = R (bnn_row_sums
 * of the weight), dW1 with row_off = T (bnn_quant_cols_t_dsum of dY), so both are exact integer
 * sums over u before scaling. */
int bnn_gemm_i8_affine(const int8_t* A, int64_t lda, int64_t a_plane, int32_t a_digits,
                       const int8_t* B, int64_t ldb, int64_t b_plane, int32_t b_digits,
                       const float* a_scale, const float* b_scale, const float* bias,
                       const int64_t* row_off, const int64_t* col_off, double off_mul, float* C,
                       int64_t ldc, int64_t M, int64_t N, int64_t K, bnn_stream_t stream);

/* fc1 on u8 pixels (digits (1,1), no a_scale / row_off) that also hands the next BatchNorm its
 * forward statistics (mnist-dist2.py:64-65, fc1 -> bn1): stat = [2][stat_rows][N] doubles, per
 * column and chunk of bnn_gemm_i8_bnstats_chunk(M, N) rows the sum of z = b_scale*(S + off_mul*
 * col_off) + bias and its M2 about the chunk mean, formed in the GEMM epilogue from the exact
 * integer sums S (no pass over C); stat_rows = ceil(M / chunk).  Feed to bnn_bn_fwd_final_parts.
 * The statistics are those of the unrounded z (C holds its fp32 rounding). */
int64_t bnn_gemm_i8_bnstats_chunk(int64_t M, int64_t N);

/* The FP4 forward (bnn_gemm_fp4 with C, or bnn_gemm_fp4_i16 with C16 and bias NULL) that also hands
 * the next BatchNorm (mnist-dist2.py:66-67, fc2 -> bn2; or fc3 -> drop -> bn3 with drop_p > 0 and
 * the seed the fused dropout BatchNorm passes will use, :68-70) its forward statistics:
 * stat = [2][stat_rows][N] doubles, per column and chunk of bnn_gemm_fp4_bnstats_chunk(M, N, K)
 * rows the sum of the stored z = fl(sum + zbias[n]) (dropped: fl(z * 1/(1-p)) or 0, the mask of
 * bnn_bn_dropout_fwd_train) -- exact in double, as bnn_bn_fwd_train's -- and its M2 about the
 * chunk mean; stat_rows = ceil(M / chunk).
 * chunk 0 = no statistics form for the shape (use the statistics pass).  Feed the partials to
 * bnn_bn_fwd_final_parts. */
int64_t bnn_gemm_fp4_bnstats_chunk(int64_t M, int64_t N, int64_t K);
int bnn_gemm_fp4_bnstats(const uint8_t* A, int64_t lda, const uint8_t* B, int64_t ldb, const float* bias,
                         float* C, int16_t* C16, int64_t ldc, const float* zbias, int64_t M, int64_t N, int64_t K,
                         float drop_p, uint64_t drop_seed, double* stat, int64_t stat_rows, bnn_stream_t stream);
/* Tile of the u8-pixel statistics GEMM (bnn_gemm_i8_affine_bnstats[_s20] and its chunk query):
 * 0 = by grid size (default), 1 = 128 x 128, 2 = 256 x 256; tile < 0 returns the setting.  Set it
 * before the chunk query of a launch (both read it). */
int bnn_gemm_i8_bnstats_set_tile(int32_t tile);
int bnn_gemm_i8_affine_bnstats(const int8_t* A, int64_t lda, const int8_t* B, int64_t ldb,
                               const float* b_scale, const float* bias, const int64_t* col_off,
                               double off_mul, float* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                               double* stat, int64_t stat_rows, bnn_stream_t stream);
/* 1 when bnn_gemm_i8_affine_bnstats takes the shape (no 32-bit tile offsets overflow, the column
 * sum of S^2 stays an exact double: M (128 K)^2 < 2^53), else 0 -- then run bnn_gemm_i8_affine and
 * the statistics pass. */
int bnn_gemm_i8_bnstats_ok(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb);

/* The s20 form of fc1's output (compact pre-activation; mnist-dist2.py:64-65 fc1 -> bn1): the
 * statistics form above writing, instead of fp32 C, the exact integer S = sum + off_mul*col_off[n]
 * (|S| < 2^19) as 20-bit two's complement -- Slo [M][ldc] int16 (its low 16 bits, 8-B aligned) and
 * Shi [M][ldc/2] (its high nibbles, column 2j in the low nibble of byte j, 2-B aligned), 2.5 B per
 * element.  The *_s20 BatchNorm entries read z = fl(fl(S * b_scale) + bias), bit-identical to the
 * fp32 C of bnn_gemm_i8_affine_bnstats (b_scale a constant vector, its value passed to them as
 * xscale; bias as xbias).  bnn_gemm_i8_s20_ok: 1 when off_mul (the pixel offset s0) is integral,
 * N % 4 == 0 and k_true (128 + |s0|) < 2^19 (ToTensor without Normalize; any K <= 2048). */
int bnn_gemm_i8_s20_ok(int64_t M, int64_t N, int64_t K, int64_t k_true, double s0);
int bnn_gemm_i8_affine_bnstats_s20(const int8_t* A, int64_t lda, const int8_t* B, int64_t ldb,
                                   const int64_t* col_off, double off_mul, int64_t k_true, int16_t* Slo,
                                   uint8_t* Shi, int64_t ldc, int64_t M, int64_t N, int64_t K, double* stat,
                                   int64_t stat_rows, const float* b_scale, const float* bias, bnn_stream_t stream);

/* The fp32 images ToTensor makes (x = fl(u / 255), mnist-dist2.py:96-99) back to their bytes: u[i] =
 * rint(255 x[i]); *bad |= 1 (device int, zero it first) if any x[i] is not exactly fl(u / 255) for a
 * byte u.  Lets the drop-in's 784-input BinarizeLinear, handed fp32 images, run its u8-pixel GEMMs
 * (one exact int8 pass instead of three digit planes).  x 16-B aligned, u 4-B aligned.
 * replaces: nothing in the reference (transforms.ToTensor's inverse, for the pixel operands). */
int bnn_unit_to_pixels(const float* x, int64_t n, uint8_t* u, int32_t* bad, bnn_stream_t stream);
/* ---------------------------------------------------------------- u8 pixels (first layer)
 * Replaces the fp32 pixel tensor the reference's loader builds (ToTensor = u8/255, optionally
 * Normalize; mnist-dist2.py:96-99, mnist-distributed-BNNS2.py:82) as the operand of fc1
 * (models/binarized_modules.py:80, input kept because size(1) == 784): x = a*v + c with
 * v = u - 128 stored as int8, so fc1 and its weight gradient are exact int8 MFMA sums.
 * bnn_pixels_pack: x [M][ldx] bytes -> q [M][ldq] int8 rows v (zero for k >= K; ldq >=
 * round_up(K,64)) and/or qt [K][ldqt] = v^T (zero for m >= M; ldqt >= round_up(M,64)); either
 * output may be NULL, ld's multiples of 16, outputs 16-B aligned. */
int bnn_pixels_pack(const uint8_t* x, int64_t M, int64_t K, int64_t ldx, int8_t* q, int64_t ldq,
                    int8_t* qt, int64_t ldqt, bnn_stream_t stream);
/* out[n] = sum_{k<K} q[n][k] (exact int64): R[n] of the packed ternary weight rows. */
int bnn_row_sums(const int8_t* q, int64_t N, int64_t K, int64_t ldq, int64_t* out, bnn_stream_t stream);

/* Ternary x ternary GEMM on the FP4 (e2m1) block-scaled MFMA (unit scales): operands hold FP4
 * codes (+1 = 0x2, -1 = 0xA, 0 = 0x0), two elements per byte (element k in byte k/2, low nibble
 * for even k), rows of lda / ldb BYTES; K = padded reduction length in BYTES (multiple of 64,
 * zero nibbles beyond the true length).  C = sum + bias[n], bit-exact like the (1,1) int8 form,
 * at twice its MFMA rate on half the operand bytes.  Pack with bnn_sign_pack_fp4. */
int bnn_gemm_fp4(const uint8_t* A, int64_t lda, const uint8_t* B, int64_t ldb, const float* bias,
                 float* C, int64_t ldc, int64_t M, int64_t N, int64_t K, bnn_stream_t stream);

/* bnn_gemm_fp4 without bias, writing the exact dot products as int16 C16 [M][ldc] (ldc % 4 == 0,
 * 8-B aligned; 2K <= 32767 so |sum| fits): the compact pre-activation of a hidden BinarizeLinear
 * (its z = fl(C16 + bias) is formed by the BatchNorm passes that read it, the *_i16 entries
 * below), half the bytes of the fp32 output on every pass over it. */
int bnn_gemm_fp4_i16(const uint8_t* A, int64_t lda, const uint8_t* B, int64_t ldb, int16_t* C16, int64_t ldc,
                     int64_t M, int64_t N, int64_t K, bnn_stream_t stream);

/* Tuning hook (not part of the stable contract): select the bnn_gemm_i8 kernel variant for all
 * later calls in this process; -1 restores the built-in default table (tools/gemm_sweep.py). */
int bnn_gemm_set_variant(int32_t variant);
/* Tuning hook: tile order of later bnn_gemm_i8_affine calls (0 = grouped raster, 1 = row-major). */
int bnn_gemm_set_raster(int32_t raster);
/* Name of the kernel instance bnn_gemm_i8 launches for this configuration (as rocprofv3 lists
 * it), so host-side HIP-event timings can be matched with profiles; a_digits = b_digits = 0
 * names the bnn_gemm_fp4 kernel (K in bytes). */
const char* bnn_gemm_i8_kernel(int32_t a_digits, int32_t b_digits, int64_t M, int64_t N,
                               int64_t K);

/* ---------------------------------------------------------------- fp32 x ternary on the FP6 MFMA
 * The fp32 operand of the backward GEMMs (dY) and of the first layer's forward (pixels) as FOUR
 * FP6 (e2m3) planes of balanced base-32 digits with one E8M0 scale per 32-element k-block
 * (v_mfma_scale_f32_32x32x64_f8f6f4's own block scales), against the FP4 ternary operand:
 * |x - x_q| <= max|x_block| * 2^-19 per element, accumulated in fp32.
 * Layouts (Kp = padded reduction length, multiple of 64):
 *   lo  [rows][Kp/32][64 B]   per block and plane j: dwords 0..3 of the plane's MFMA operand
 *   hi  [rows][Kp/32][32 B]   per block: dwords 4..5 of planes 0,1,2,3
 *   sc  [Kp/64][bnn_quant6_scale_rows(rows)][2]  E8M0 byte of plane 0 per block (plane j: +5j;
 *       255 = NaN); the row pitch carries 512 rows of tail padding the GEMM may read
 *   res [rows][Kp/32][16 B]   optional residual plane (row operands of the dX GEMMs): the next 3
 *       bits, d = rint(x 2^(22-e)) - 8 rint(x 2^(19-e)) in [-4, 4] as FP4 (e2m1) codes of d/2
 *       (element i at bits 4i), scaled by plane 0's scale / 32: with it |x - x_q| <= max|x_block|
 *       * 2^-22 -- fp32-grade sums for the hidden BatchNorms' bias gradients
 * replaces: the fp32 GEMMs of BinarizeLinear's autograd (dX = dY.W_b, dW = dY^T.X_b) and the
 * first layer's F.linear(x, W_b) (models/binarized_modules.py:80). */
int64_t bnn_quant6_scale_rows(int64_t rows);
/* x [M][K] (row stride ldx) -> digits of its rows, blocks along K (zero digits for K..Kp-1). */
int bnn_quant6_rows(const float* x, int64_t M, int64_t K, int64_t ldx, int64_t Kp, uint8_t* lo, uint8_t* hi,
                    uint8_t* sc, uint8_t* res /* nullable */, bnn_stream_t stream);
/* x [M][N] -> digits of x^T (rows n, blocks along m, zero digits for M..Mp-1), plus colsum[n] =
 * sum_m x[m][n] (nullable; fixed-order double sums, `work` of bnn_quant6_cols_workspace bytes):
 * the bias gradient dB = sum_B dY (binarized_modules.py:81-83). */
int64_t bnn_quant6_cols_workspace(int64_t M, int64_t N);
int bnn_quant6_cols_t(const float* x, int64_t M, int64_t N, int64_t ldx, int64_t Mp, uint8_t* lo, uint8_t* hi,
                      uint8_t* sc, float* colsum, void* work, bnn_stream_t stream);
/* C[m][n] = sum_k A[m][k] B[n][k] (+ bias[n]): A as above (asc_rows = the sc row pitch; ares = its
 * residual plane or NULL: a fifth MFMA pass), B FP4 nibbles [N][ldb bytes] (ldb multiple of 16,
 * >= K/2; zero nibbles beyond the true length). */
int bnn_gemm_fp6(const uint8_t* alo, const uint8_t* ahi, const uint8_t* asc, int64_t asc_rows, const uint8_t* ares,
                 const uint8_t* b, int64_t ldb, const float* bias, float* C, int64_t ldc, int64_t M, int64_t N,
                 int64_t K, bnn_stream_t stream);
/* The same product with split-K when the tile grid is below one round of the chip (small M x N:
 * the MLP's backward GEMMs at batch 4096): `work` of bnn_gemm_fp6_workspace(M, N, K) bytes (0 = no
 * split for this shape) holds the per-split fp32 partials, folded in split order (deterministic,
 * shape-only) with the bias.  A smaller workspace falls back to the unsplit grid. */
int64_t bnn_gemm_fp6_workspace(int64_t M, int64_t N, int64_t K);
int bnn_gemm_fp6_ws(const uint8_t* alo, const uint8_t* ahi, const uint8_t* asc, int64_t asc_rows,
                    const uint8_t* ares, const uint8_t* b, int64_t ldb, const float* bias, float* C, int64_t ldc,
                    int64_t M, int64_t N, int64_t K, void* work, int64_t work_bytes, bnn_stream_t stream);
/* FP4 panels of a B operand: [N][ldb] -> [ceil(N/512)][Kp/64][512][32 B] (rows beyond N zero), so
 * each GEMM stage stages one contiguous run of B instead of 32 B from each of 512 rows (a quarter
 * line per row); bnn_gemm_fp6_panel_ws = bnn_gemm_fp6_ws with B in that layout, bks = the 64-k
 * steps stored per panel (>= K/64; Kp/64 of bnn_fp4_panelize, round_up(M,256)/64 of
 * bnn_bn_apply_pack's panel transpose). */
int64_t bnn_fp4_panel_bytes(int64_t N, int64_t Kp);
int bnn_fp4_panelize(const uint8_t* b, int64_t N, int64_t ldb, int64_t Kp, uint8_t* panels, bnn_stream_t stream);
int bnn_gemm_fp6_panel_ws(const uint8_t* alo, const uint8_t* ahi, const uint8_t* asc, int64_t asc_rows,
                          const uint8_t* ares, const uint8_t* bpanels, int64_t bks, const float* bias, float* C,
                          int64_t ldc, int64_t M, int64_t N, int64_t K, void* work, int64_t work_bytes,
                          bnn_stream_t stream);
/* bnn_gemm_fp6_panel_ws (no bias, the unsplit default plan only) with the BatchNorm-backward column
 * statistics of C in its epilogue: C is the dy of a training-mode BatchNorm(+Hardtanh) over x
 * [M][N] (fp32, or int16 + xbias when x_i16) with save_mean / mean_lo / invstd and gamma / beta;
 * part = [2 (mode 1) or 4 (mode 2)][bnn_gemm_fp6_bnstats_rows(M)][N] floats (sum g, sum g*xhat,
 * max|g|, max|xhat| per 128-row tile row), folded by bnn_bn_bwd_stats_pre. */
int64_t bnn_gemm_fp6_bnstats_rows(int64_t M);
int bnn_gemm_fp6_bnstats(const uint8_t* alo, const uint8_t* ahi, const uint8_t* asc, int64_t asc_rows,
                         const uint8_t* ares, const uint8_t* bpanels, int64_t bks, float* C, int64_t ldc, int64_t M,
                         int64_t N, int64_t K,
                         const void* x, const float* xbias, int32_t x_i16, const float* mean, const float* mean_lo,
                         const float* invstd, const float* gamma, const float* beta, int32_t hardtanh, int32_t mode,
                         float* part, bnn_stream_t stream);
const char* bnn_gemm_fp6_kernel(int64_t M, int64_t N);
const char* bnn_gemm_fp6_kernel_k(int64_t M, int64_t N, int64_t K);   /* + " split-K S" */
const char* bnn_gemm_fp6_kernel_kr(int64_t M, int64_t N, int64_t K, int32_t res);   /* with / without the residual plane */
int bnn_gemm_fp6_set_variant(int32_t variant);   /* tuning hook (-1 = default) */
/* 1: on grids of >= 2 rounds of 128 x 512 tiles with no bias, M % 128 == 0, N % 512 == 0 and B in
 * panels (the backward GEMMs), the default tile runs persistent -- one workgroup per CU, the waves
 * split into loading and storing roles so a tile's fp32 stores drain under the next tile's k loop
 * (gemm_fp6_pers_k); bit-identical to 0 (one workgroup per tile, the default: measured faster).
 * on < 0 queries. */
int bnn_gemm_fp6_set_persistent(int32_t on);
/* Half-tile form of the backward GEMMs: mode 1 runs the dX launches (residual plane) on 64 x 512
 * tiles, two 4-wave workgroups per CU, the second resident of each CU held back stagger_us in the
 * first round so one workgroup's fp32 epilogue drains while the other's MFMAs run; mode 2 also the
 * dW launches; 0 = the 128 x 512 tile.  Default 1 (dX + res 8.83 -> 8.31 ms; dW slower on half
 * tiles, profiles/r06_b_fp6_half.log).  Same fragments and accumulation order per output element:
 * bit-identical C.  mode < 0 queries. */
int bnn_gemm_fp6_set_half(int32_t mode, double stagger_us);
int bnn_gemm_fp6_set_half_group(int32_t group);   /* tuning hook: raster group rows of the half-tile form (0 = default) */

/* XNOR/AND-popcount VALU GEMM on bit-planes (same contract as the (1,1) form):
 * C[m][n] = sum_w popc(nzA&nzB) - 2*popc(nzA&nzB&(sA^sB)) + bias[n]; kw = words per row
 * (multiple of 32, <= lda/ldb in words). */
int bnn_gemm_xnor(const uint32_t* As, const uint32_t* Anz, int64_t lda, const uint32_t* Bs,
                  const uint32_t* Bnz, int64_t ldb, const float* bias, float* C, int64_t ldc,
                  int64_t M, int64_t N, int64_t kw, bnn_stream_t stream);

/* ---------------------------------------------------------------- binary conv2d (NCHW fp32)
 * replaces: F.conv2d(input, W_b, None, stride, padding, dilation, groups) + bias (:100-105)
 * and its autograd.  binarize_input != 0 -> sign(x) is used (the :94 rule is applied by the
 * caller).  w_latent [Co][Ci/groups][KH][KW] is binarised on the fly (sign). */
int bnn_conv2d_fwd(const float* x, int32_t binarize_input, const float* w_latent,
                   const float* bias, float* y, int64_t N, int64_t C, int64_t H, int64_t W,
                   int64_t Co, int64_t KH, int64_t KW, int32_t stride, int32_t pad,
                   int32_t dil, int32_t groups, bnn_stream_t stream);
/* The binary-input forward writing the exact sums I (no bias) as int8 (yfmt 1, C*KH*KW <= 127) or
 * int16 (yfmt 2, <= 32767) for a BatchNorm2d that reads fl(I + bias) (bnn_bn2d_*_q): stride 1,
 * dilation 1, groups 1, C == 1 (KW <= 8) or C % 16 == 0 (<= 64), Co <= 64; other shapes -1. */
int bnn_conv2d_fwd_q(const float* x, const float* w_latent, void* y, int32_t yfmt, int64_t N, int64_t C, int64_t H,
                     int64_t W, int64_t Co, int64_t KH, int64_t KW, int32_t stride, int32_t pad, int32_t dil,
                     int32_t groups, bnn_stream_t stream);
/* 1 when bnn_conv2d_fwd_q takes the shape (the same geometry checks, nothing launched; depends on
 * bnn_conv_set_mfma), else 0: the host asks before emitting a compact conv output. */
int bnn_conv2d_fwd_q_ok(int32_t yfmt, int64_t N, int64_t C, int64_t H, int64_t W, int64_t Co, int64_t KH, int64_t KW,
                        int32_t stride, int32_t pad, int32_t dil, int32_t groups);
int bnn_conv2d_bwd_data(const float* dy, const float* w_latent, float* dx, int64_t N, int64_t C,
                        int64_t H, int64_t W, int64_t Co, int64_t KH, int64_t KW, int32_t stride,
                        int32_t pad, int32_t dil, int32_t groups, bnn_stream_t stream);
/* dw = sum dy (x) x_used (x_used = sign(x) when binarize_input); db (nullable) = sum dy.
 * `work` scratch of bnn_conv2d_bwd_filter_workspace(...) bytes. */
int64_t bnn_conv2d_bwd_filter_workspace(int64_t N, int64_t C, int64_t Co, int64_t KH, int64_t KW,
                                        int32_t groups);
int bnn_conv2d_bwd_filter(const float* dy, const float* x, int32_t binarize_input, float* dw,
                          float* db, void* work, int64_t N, int64_t C, int64_t H, int64_t W,
                          int64_t Co, int64_t KH, int64_t KW, int32_t stride, int32_t pad,
                          int32_t dil, int32_t groups, bnn_stream_t stream);

/* The first BinarizeConv2d's weight gradient fused with its BatchNorm2d + Hardtanh + MaxPool2d(2)
 * backward (mnist-dist.py:31-51 template, binarized_modules.py:100-107): bnn_conv2d_bwd_filter with
 * dY = the BatchNorm2d backward of the pooled gradient dyp, formed per 2x2 window from the conv's
 * compact output zq (zfmt 1 int8 / 2 int16 sums + zbias, bnn_conv2d_fwd_q), the BatchNorm's
 * mean / invstd / gamma / beta and sg / sgx from bnn_bn2d_bwd_stats_q (inv_n = 1 / (N OH OW)) -- the
 * arithmetic of bnn_bn2d_bwd_q's dx, which is never written.  One input channel, stride 1, 3x3 or
 * 5x5, even OH, OW % 4 == 0 (bnn_conv2d_bwd_filter_bn_ok); work as bnn_conv2d_bwd_filter's. */
int bnn_conv2d_bwd_filter_bn_ok(int64_t N, int64_t C, int64_t H, int64_t W, int64_t Co, int64_t KH, int64_t KW,
                                int32_t stride, int32_t pad, int32_t dil, int32_t groups);
int bnn_conv2d_bwd_filter_bn(const void* zq, const float* zbias, int32_t zfmt, const float* dyp, const float* mean,
                             const float* invstd, const float* gamma, const float* beta, const float* sg,
                             const float* sgx, float inv_n, int32_t hardtanh, const float* x, int32_t binarize_input,
                             float* dw, float* db, void* work, int64_t N, int64_t C, int64_t H, int64_t W, int64_t Co,
                             int64_t KH, int64_t KW, int32_t stride, int32_t pad, int32_t dil, int32_t groups,
                             bnn_stream_t stream);

/* Convolution engine switch: 1 (default) = MFMA implicit-GEMM kernels for stride-1 ungrouped
 * shapes -- backward data on v_mfma_f32_16x16x32_bf16 with dY split exactly into three bf16
 * terms (exact products, fp32 accumulation), backward filter on v_mfma_f32_16x16x4_f32 (exact f32
 * products), forward with a binarised input and C % 16 == 0 on v_mfma_i32_16x16x64_i8 (exact
 * integer sums); 2 = as 1 but backward data on the f32 MFMA; 0 = the VALU LDS-tiled / generic
 * kernels.  Process-global; for cross-checks and the kernel sweep. */
int bnn_conv_set_mfma(int32_t mode);
/* 1 (default, with bnn_conv_set_mfma != 0): the filter gradient of a one-input-channel layer
 * (stride 1, 3x3 or 5x5, OW % 4 == 0, Co | 256, Co <= 64 -- the BinCNN's conv1) on a VALU kernel
 * that reads dY once with coalesced 16-B loads; 0: the MFMA kernels as for any layer. */
int bnn_conv_set_c1_filter(int32_t on);
/* Binarised-input forward engine (bnn_conv2d_fwd with binarize_input, bnn_conv2d_fwd_q): 1 = the
 * VALU popcount kernels (sign / nonzero bit planes, and + xor + v_bcnt per 32 taps, exact integer
 * sums) where they take the shape -- stride 1, dilation 1, one group, square odd K, pad <= K - 1, and
 * C == 16 (K <= 7) or C == 1 (K*K <= 32, W + 2 pad <= 32, H + 2 pad <= 40); 0 = the int8-MFMA / dot4
 * kernels.  The two write identical outputs; the default is the faster on the BinCNN's layers
 * (DESIGN.md §6).  Process-global; on < 0 only returns the current setting (0 / 1). */
int bnn_conv_set_popc(int32_t on);
/* 1 (default): the 2x2-pooled BatchNorm2d backward statistics and forward apply over 28- / 14-wide
 * planes (the BinCNN's layers) on the row kernels (one thread per pooled row, every load of the row
 * issued up front); 2: the backward apply too (slower; A/B); 0: the window-per-thread kernels.
 * Same per-element arithmetic (the backward statistics summed per row). */
int bnn_bn2d_set_rows(int32_t on);
/* Host-only plan query (needs no GPU): the bf16x3 backward kernels' LDS layouts for a shape.
 * out[9]: data kernel (pixel pitch ps, weight pitch ws, row tiles, LDS bytes), then filter kernel
 * (dY pitch Kd, copy channel stride CS, copy stride XL, LDS bytes, modelled cycles x 100 of its B
 * fragment ds_read_b128, 400 = conflict-free); -1 where the kernel does not take the shape. */
int bnn_conv_bf3_plan(int64_t N, int64_t C, int64_t H, int64_t W, int64_t Co, int64_t KH, int64_t KW,
                      int32_t stride, int32_t pad, int32_t dil, int32_t groups, int64_t* out);

/* ---------------------------------------------------------------- BatchNorm1d (+ Hardtanh)
 * The layers between the binarized GEMMs in the reference Net (mnist-dist2.py:52-74):
 * nn.BatchNorm1d (train: batch stats, biased var; running stats with the unbiased var and
 * `momentum`; eval: running stats) optionally followed by nn.Hardtanh (fused: y clamped to
 * [-1,1] in forward, gradient masked by -1 < y < 1 in backward, y recomputed from x).
 * x, y, dy, dx fp32 [M][C] row-major, C % 4 == 0, 16-B aligned; gamma/beta nullable (affine off);
 * running_mean/var nullable in train mode (track_running_stats off; momentum < 0 skips the update).
 * `work` scratch of bnn_bn_workspace(M, C) bytes.  Deterministic (fixed-order reductions).
 * bnn_bn_fwd_train with y == NULL computes the statistics only (for bnn_bn_apply_pack).
 * The batch mean is the batch sum taken in double (exact for integer-plus-bias pre-activations)
 * divided by M, returned as save_mean (fp32) + save_mean_lo (fp32, nullable: the rounding
 * remainder); every pass that normalises computes x - mean as (x - save_mean) - save_mean_lo,
 * so a value within an ulp of the mean (a BatchNorm near-tie, frequent when x is integer-valued)
 * gets the sign of the exact difference, as the reference's (double-accumulated) CPU BatchNorm
 * gives it.  Pass the same save_mean_lo to the backward / apply-pack calls (NULL = 0). */
int64_t bnn_bn_workspace(int64_t M, int64_t C);
int bnn_bn_fwd_train(const float* x, int64_t M, int64_t C, const float* gamma, const float* beta,
                     float* running_mean, float* running_var, float momentum, float eps,
                     float* save_mean, float* save_invstd, float* save_mean_lo, float* y, int32_t hardtanh,
                     void* work, bnn_stream_t stream);
/* bnn_bn_fwd_train's final step (mean hi/lo, invstd, running statistics) from chunk partials
 * another kernel formed: part = [2][R][C] doubles (chunk sums, then M2 about each chunk's mean),
 * chunk r = rows [r*chunk_rows, min((r+1)*chunk_rows, M)), R = ceil(M / chunk_rows). */
int bnn_bn_fwd_final_parts(const double* part, int64_t R, int64_t chunk_rows, int64_t M, int64_t C,
                           float* running_mean, float* running_var, float momentum, float eps,
                           float* save_mean, float* save_invstd, float* save_mean_lo, bnn_stream_t stream);
int bnn_bn_fwd_eval(const float* x, int64_t M, int64_t C, const float* gamma, const float* beta,
                    const float* running_mean, const float* running_var, float eps, float* y,
                    int32_t hardtanh, void* work, bnn_stream_t stream);
int bnn_bn_bwd(const float* x, const float* dy, int64_t M, int64_t C, const float* gamma,
               const float* beta, const float* save_mean, const float* save_invstd, const float* save_mean_lo,
               int32_t hardtanh, float* dx, float* dgamma, float* dbeta, void* work, bnn_stream_t stream);
/* Backward of the eval-mode forward (running statistics are constants, torch's
 * batch_norm_backward with training=False): dx = gamma*invstd*g, dgamma = sum g*xhat,
 * dbeta = sum g, with invstd = 1/sqrt(running_var + eps). */
int bnn_bn_bwd_eval(const float* x, const float* dy, int64_t M, int64_t C, const float* gamma,
                    const float* beta, const float* running_mean, const float* invstd, int32_t hardtanh,
                    float* dx, float* dgamma, float* dbeta, void* work, bnn_stream_t stream);

/* ---------------------------------------------------------------- BatchNorm2d (+ Hardtanh, + MaxPool2d(2))
 * The block after each BinarizeConv2d of the build's CNN (conv -> nn.BatchNorm2d -> nn.Hardtanh ->
 * nn.MaxPool2d(2, 2), the ConvNet template of mnist-dist.py:31-51 with the reference's BNN
 * activation): per-channel statistics over N*H*W with the BatchNorm1d semantics above.  x, dx fp32
 * NCHW [N][C][H][W], H*W % 4 == 0, 16-B aligned.  pool = 0: y, dy are [N][C][H][W]; pool = 2:
 * y, dy are the max-pooled [N][C][H/2][W/2] (H, W even) and the backward recomputes each
 * window's argmax (torch's rule: first strictly greater value in (h, w) order, NaN wins), so no
 * full-resolution output or pooling indices are stored.  `work` scratch of
 * bnn_bn2d_workspace(N, C) bytes.  Deterministic. */
int64_t bnn_bn2d_workspace(int64_t N, int64_t C);
int bnn_bn2d_fwd_train(const float* x, int64_t N, int64_t C, int64_t H, int64_t W, const float* gamma,
                       const float* beta, float* running_mean, float* running_var, float momentum,
                       float eps, float* save_mean, float* save_invstd, float* y, int32_t hardtanh,
                       int32_t pool, void* work, bnn_stream_t stream);
int bnn_bn2d_fwd_eval(const float* x, int64_t N, int64_t C, int64_t H, int64_t W, const float* gamma,
                      const float* beta, const float* running_mean, const float* running_var, float eps,
                      float* y, int32_t hardtanh, int32_t pool, void* work, bnn_stream_t stream);
int bnn_bn2d_bwd(const float* x, const float* dy, int64_t N, int64_t C, int64_t H, int64_t W,
                 const float* gamma, const float* beta, const float* save_mean, const float* save_invstd,
                 int32_t hardtanh, int32_t pool, float* dx, float* dgamma, float* dbeta, void* work,
                 bnn_stream_t stream);
/* Eval-mode backward (running statistics), as bnn_bn_bwd_eval. */
int bnn_bn2d_bwd_eval(const float* x, const float* dy, int64_t N, int64_t C, int64_t H, int64_t W,
                      const float* gamma, const float* beta, const float* running_mean, const float* invstd,
                      int32_t hardtanh, int32_t pool, float* dx, float* dgamma, float* dbeta, void* work,
                      bnn_stream_t stream);
/* The same training-mode passes on a compact input: xq = int8 (xfmt 1) or int16 (xfmt 2) sums
 * [N][C][H][W] of bnn_conv2d_fwd_q, xbias [C] (nullable, 16-B aligned) its bias, read as
 * x = fl(xq + xbias[c]) -- bit-identical to the fp32 entries on the conv's fp32 output. */
int bnn_bn2d_fwd_train_q(const void* xq, const float* xbias, int32_t xfmt, int64_t N, int64_t C, int64_t H, int64_t W,
                         const float* gamma, const float* beta, float* running_mean, float* running_var,
                         float momentum, float eps, float* save_mean, float* save_invstd, float* y, int32_t hardtanh,
                         int32_t pool, void* work, bnn_stream_t stream);
int bnn_bn2d_bwd_q(const void* xq, const float* xbias, int32_t xfmt, const float* dy, int64_t N, int64_t C, int64_t H,
                   int64_t W, const float* gamma, const float* beta, const float* save_mean, const float* save_invstd,
                   int32_t hardtanh, int32_t pool, float* dx, float* dgamma, float* dbeta, void* work,
                   bnn_stream_t stream);
/* bnn_bn2d_bwd_q's statistics only (no dx): dgamma, dbeta and the column sums sum g, sum g*xhat into
 * sg / sgx (C floats each), for bnn_conv2d_bwd_filter_bn. */
int bnn_bn2d_bwd_stats_q(const void* xq, const float* xbias, int32_t xfmt, const float* dy, int64_t N, int64_t C,
                         int64_t H, int64_t W, const float* gamma, const float* beta, const float* save_mean,
                         const float* save_invstd, int32_t hardtanh, int32_t pool, float* dgamma, float* dbeta,
                         float* sg, float* sgx, void* work, bnn_stream_t stream);

/* nn.Dropout(p) fused in front of BatchNorm1d (+ Hardtanh) (mnist-dist2.py:69-70: fc3 -> drop ->
 * bn3): x is the pre-dropout input; the keep mask is a counter-based hash of (seed, row*C + col)
 * regenerated by every pass, kept values scaled by 1/(1-p) as torch does; the backward's dx is
 * the gradient w.r.t. the pre-dropout input.  p in [0, 1).  bnn_dropout_mask writes the mask the
 * fused passes use (scale or 0 per element, n = M*C) for tests.
 * keep_bits (nullable; p > 0, C % 4 == 0): the forward statistics pass also stores the mask as a
 * bit plane of bnn_dropout_keep_bits_bytes(M, C) bytes -- word (r/8)*(C/4) + c/4 holds rows
 * (r & ~7) + i, columns (c & ~3) + j at bit 4i + j -- which bnn_bn_head_fwd / bnn_bn_head_bwd_q6
 * (and their _i16 forms) then read instead of evaluating the hash (same mask, bit-identical
 * results).  bnn_dropout_keep_bits_bytes returns -1 for M <= 0 or C % 4 != 0. */
int64_t bnn_dropout_keep_bits_bytes(int64_t M, int64_t C);
int bnn_bn_dropout_fwd_train(const float* x, int64_t M, int64_t C, const float* gamma, const float* beta,
                             float* running_mean, float* running_var, float momentum, float eps,
                             float* save_mean, float* save_invstd, float* save_mean_lo, float* y, int32_t hardtanh,
                             float p, uint64_t seed, uint32_t* keep_bits, void* work, bnn_stream_t stream);
int bnn_bn_dropout_bwd(const float* x, const float* dy, int64_t M, int64_t C, const float* gamma,
                       const float* beta, const float* save_mean, const float* save_invstd,
                       const float* save_mean_lo, int32_t hardtanh, float p, uint64_t seed, float* dx,
                       float* dgamma, float* dbeta, void* work, bnn_stream_t stream);

/* The BatchNorm(+Dropout) backward whose dz is the upstream gradient of an FP6-backward
 * BinarizeLinear (mnist-dist2.py:66-71 fc -> [drop ->] bn -> htanh -> fc): bnn_bn_bwd /
 * bnn_bn_dropout_bwd (p = 0: no dropout) that also writes both FP6 digit forms of dz -- rows
 * (lo/hi/sc as bnn_quant6_rows with Kp = C) and the transpose (as bnn_quant6_cols_t with
 * Mp = round_up(M, 64)) -- and colsum[n] = sum_m dz[m][n] (nullable), in the same pass, so dz is
 * never re-read; dx (the fp32 dz) is optional; rres (nullable) also the rows' residual plane
 * ([M][C/32][16 B], bnn_quant6_rows' res) for the dX GEMM.  C % 64 == 0; training statistics only.  Digits
 * are bit-identical to the standalone quantisers on the same dz. */
int bnn_bn_bwd_q6(const float* x, const float* dy, int64_t M, int64_t C, const float* gamma, const float* beta,
                  const float* save_mean, const float* save_invstd, const float* save_mean_lo, int32_t hardtanh,
                  float p, uint64_t seed, float* dx, float* dgamma, float* dbeta, uint8_t* rlo, uint8_t* rhi,
                  uint8_t* rsc, uint8_t* rres, uint8_t* clo, uint8_t* chi, uint8_t* csc, float* colsum, void* work,
                  bnn_stream_t stream);
int bnn_dropout_mask(int64_t n, float p, uint64_t seed, float* out, bnn_stream_t stream);

/* The network's head fused with its BatchNorm (mnist-dist2.py:69-76: fc3 -> drop -> bn3 -> htanh3
 * -> fc4 = nn.Linear(C, nout)), training mode, nout == 10, C % 256 == 0 (the forward: C % 128): the fp32 hardtanh
 * output h3 is never written.
 * bnn_bn_head_fwd: y4[m][q] = sum_c h3[m][c] W4[q][c] + b4[q] with h3 = clamp(BN(drop(x)), -1, 1)
 *   formed from x with the statistics of bnn_bn_dropout_fwd_train (y = NULL: statistics only);
 *   products exact in f32, f32 accumulation (v_mfma_f32_16x16x4_f32).
 * bnn_bn_head_bwd_q6: given dY4 [M][nout], the BatchNorm(+dropout) backward with the incoming
 *   gradient dh3 = dY4 . W4 formed per element, as bnn_bn_bwd_q6 (dx optional, both FP6 digit
 *   forms of dx, colsum of dx), plus dW4 = dY4^T . h3 [nout][C] (h3 recomputed from x).
 *   work: bnn_bn_head_workspace(M, C, nout) bytes.  The head's bias gradient is sum_m dY4.
 * keep_bits (nullable): the mask plane the statistics pass stored (bnn_bn_dropout_fwd_train), read
 *   instead of the hash; it must come from the same (M, C, p, seed) forward. */
int64_t bnn_bn_head_workspace(int64_t M, int64_t C, int32_t nout);
/* Columns per thread of bnn_bn_head_bwd_q6's statistics pass: 2 (default: half the registers, twice
 * the threads) or 4; identical results.  cols < 0 returns the current setting. */
int bnn_bn_set_head_reduce_cols(int32_t cols);
int bnn_bn_head_fwd(const float* x, int64_t M, int64_t C, const float* mean, const float* invstd,
                    const float* mean_lo, const float* gamma, const float* beta, float p, uint64_t seed,
                    const uint32_t* keep_bits, const float* w4, int32_t nout, const float* b4, float* y4,
                    bnn_stream_t stream);
int bnn_bn_head_bwd_q6(const float* x, const float* dy4, const float* w4, int32_t nout, int64_t M, int64_t C,
                       const float* gamma, const float* beta, const float* save_mean, const float* save_invstd,
                       const float* save_mean_lo, float p, uint64_t seed, const uint32_t* keep_bits, float* dx,
                       float* dgamma, float* dbeta,
                       float* dw4, uint8_t* rlo, uint8_t* rhi, uint8_t* rsc, uint8_t* rres, uint8_t* clo, uint8_t* chi,
                       uint8_t* csc, float* colsum, void* work, bnn_stream_t stream);

/* Fused BatchNorm-apply -> Hardtanh -> sign-pack for the next binarized layer (mnist-dist2.py:
 * 66-68: bn1 -> htanh1 -> fc2 binarises its input): y = ((x-mean)-mean_lo)*invstd*gamma+beta exactly as
 * bnn_bn_fwd_* computes it, written only as the next GEMM's ternary operand -- q rows in fmt 0
 * (int8, ldq >= round_up(C,64)) or fmt 1 (FP4 nibbles, ldq bytes >= round_up(C,256)/2, multiple
 * of 128) and/or the transpose qt for the weight gradient: qt_fmt 0 int8 [C][ldqt], 1 FP4
 * [C][ldqt bytes], 2 FP4 in the panel layout of bnn_gemm_fp6_panel_ws ([ceil(C/512)][ldqt/32][512]
 * [32 B], bks = ldqt/32; rows beyond C unspecified); no fp32 activation is
 * written (Hardtanh keeps the sign; its backward mask is recomputed from x by bnn_bn_bwd). */
int bnn_bn_apply_pack(const float* x, int64_t M, int64_t C, const float* mean, const float* invstd,
                      const float* mean_lo, const float* gamma, const float* beta, int32_t fmt, void* q,
                      int64_t ldq, int8_t* qt, int64_t ldqt, int32_t qt_fmt, bnn_stream_t stream);

/* The int16 form of the BatchNorm input (z16): x16 [M][C] the int16 dot products of
 * bnn_gemm_fp4_i16 (8-B aligned), xbias [C] that layer's bias (16-B aligned, nullable), read as
 * x = fl(x16 + xbias) -- the value the fp32 GEMM epilogue stores, so every result is bit-identical
 * to the fp32 entry on that x.  Training-mode statistics passes only:
 *   bnn_bn_fwd_train_i16     = bnn_bn_dropout_fwd_train with y = NULL (p = 0: no dropout)
 *   bnn_bn_apply_pack_i16    = bnn_bn_apply_pack, fmt 1 rows + qt_fmt 1 (qt_panel 0) or 2 (qt_panel 1)
 *                              transpose, C % 256 == 0
 *   bnn_bn_bwd_q6_i16        = bnn_bn_bwd_q6
 *   bnn_bn_head_fwd_i16      = bnn_bn_head_fwd
 *   bnn_bn_head_bwd_q6_i16   = bnn_bn_head_bwd_q6
 * replaces: the fp32 z = F.linear(sign(h), W_b) + bias (binarized_modules.py:80-83) that the
 * reference materialises between a hidden BinarizeLinear and its BatchNorm (mnist-dist2.py:66-70). */
int bnn_bn_fwd_train_i16(const int16_t* x16, const float* xbias, int64_t M, int64_t C, const float* gamma,
                         const float* beta, float* running_mean, float* running_var, float momentum, float eps,
                         float* save_mean, float* save_invstd, float* save_mean_lo, float p, uint64_t seed,
                         uint32_t* keep_bits, void* work, bnn_stream_t stream);
int bnn_bn_apply_pack_i16(const int16_t* x16, const float* xbias, int64_t M, int64_t C, const float* mean,
                          const float* invstd, const float* mean_lo, const float* gamma, const float* beta,
                          uint8_t* q, int64_t ldq, uint8_t* qt, int64_t ldqt, int32_t qt_panel,
                          bnn_stream_t stream);
int bnn_bn_bwd_q6_i16(const int16_t* x16, const float* xbias, const float* dy, int64_t M, int64_t C,
                      const float* gamma, const float* beta, const float* save_mean, const float* save_invstd,
                      const float* save_mean_lo, int32_t hardtanh, float p, uint64_t seed, float* dx, float* dgamma,
                      float* dbeta, uint8_t* rlo, uint8_t* rhi, uint8_t* rsc, uint8_t* rres, uint8_t* clo, uint8_t* chi,
                      uint8_t* csc, float* colsum, void* work, bnn_stream_t stream);
int bnn_bn_head_fwd_i16(const int16_t* x16, const float* xbias, int64_t M, int64_t C, const float* mean,
                        const float* invstd, const float* mean_lo, const float* gamma, const float* beta, float p,
                        uint64_t seed, const uint32_t* keep_bits, const float* w4, int32_t nout, const float* b4,
                        float* y4, bnn_stream_t stream);
int bnn_bn_head_bwd_q6_i16(const int16_t* x16, const float* xbias, const float* dy4, const float* w4, int32_t nout,
                           int64_t M, int64_t C, const float* gamma, const float* beta, const float* save_mean,
                           const float* save_invstd, const float* save_mean_lo, float p, uint64_t seed,
                           const uint32_t* keep_bits, float* dx, float* dgamma, float* dbeta, float* dw4, uint8_t* rlo, uint8_t* rhi, uint8_t* rsc, uint8_t* rres,
                           uint8_t* clo, uint8_t* chi, uint8_t* csc, float* colsum, void* work,
                           bnn_stream_t stream);

/* The BatchNorm(+Hardtanh) backward feeding the first BinarizeLinear's weight gradient on u8
 * pixels (mnist-dist2.py:52-54 fc1 -> bn1 -> htanh1; dW1 = dz^T . x on bnn_gemm_i8_affine): dz is
 * formed from (x, dy) exactly as bnn_bn_bwd writes it, but only delivered as what that GEMM reads --
 * bnn_quant_cols_t_dsum's outputs (3 int8 digit planes of dz^T, per-column scale, colsum = the
 * bias gradient, dsum = exact digit sums) -- bit-identical to bnn_bn_bwd + bnn_quant_cols_t_dsum,
 * without writing or re-reading dz.  Training statistics, no dropout; dgamma/dbeta as bnn_bn_bwd.
 * work: bnn_bn_bwd_i8cols_workspace(M, C) bytes. */
int64_t bnn_bn_bwd_i8cols_workspace(int64_t M, int64_t C);
int bnn_bn_bwd_i8cols(const float* x, const float* dy, int64_t M, int64_t C, const float* gamma, const float* beta,
                      const float* save_mean, const float* save_invstd, const float* save_mean_lo, int32_t hardtanh,
                      float* dgamma, float* dbeta, int8_t* digits_t, int64_t ldqt, int64_t plane, float* scale,
                      float* colsum, int64_t* dsum, void* work, bnn_stream_t stream);

/* The s20 form of the BatchNorm input (the u8-pixel layer's sums from bnn_gemm_i8_affine_bnstats_s20:
 * xlo / xhi, xbias [C] (16-B aligned, nullable), xscale), read as x = fl(fl(S * xscale) + xbias) --
 * bit-identical results to the fp32 entries on that x:
 *   bnn_bn_apply_pack_s20       = bnn_bn_apply_pack_i16 (FP4 rows + transpose, C % 256 == 0)
 *   bnn_bn_bwd_i8cols_s20[_pre] = bnn_bn_bwd_i8cols[_pre]
 * replaces: the fp32 z1 = F.linear(x, W_b) + bias of the first BinarizeLinear (binarized_modules.py:
 * 80-83, input kept at size(1) == 784) the reference materialises for bn1 (mnist-dist2.py:64-65). */
int bnn_bn_apply_pack_s20(const int16_t* xlo, const uint8_t* xhi, const float* xbias, float xscale, int64_t M,
                          int64_t C, const float* mean, const float* invstd, const float* mean_lo, const float* gamma,
                          const float* beta, uint8_t* q, int64_t ldq, uint8_t* qt, int64_t ldqt, int32_t qt_panel,
                          bnn_stream_t stream);
int bnn_bn_bwd_i8cols_s20(const int16_t* xlo, const uint8_t* xhi, const float* xbias, float xscale, const float* dy,
                          int64_t M, int64_t C, const float* gamma, const float* beta, const float* save_mean,
                          const float* save_invstd, const float* save_mean_lo, int32_t hardtanh, float* dgamma,
                          float* dbeta, int8_t* digits_t, int64_t ldqt, int64_t plane, float* scale, float* colsum,
                          int64_t* dsum, void* work, bnn_stream_t stream);
int bnn_bn_bwd_i8cols_s20_pre(const int16_t* xlo, const uint8_t* xhi, const float* xbias, float xscale,
                              const float* dy, int64_t M, int64_t C, const float* gamma, const float* beta,
                              const float* save_mean, const float* save_invstd, const float* save_mean_lo,
                              int32_t hardtanh, float* dgamma, float* dbeta, int8_t* digits_t, int64_t ldqt,
                              int64_t plane, float* scale, float* colsum, int64_t* dsum, void* work,
                              bnn_stream_t stream);

/* The BatchNorm(+Hardtanh) backward statistics from the FP6 dX GEMM's epilogue instead of their own
 * pass over (x, dy): bnn_gemm_fp6_bnstats (below) writes per-128-row-tile-row partials of sum g,
 * sum g*xhat (mode 2: + max|g|, max|xhat|) while it writes dy; bnn_bn_bwd_stats_pre folds them
 * (fixed order) into `work` (bnn_bn_workspace(M, C) bytes -- for i8cols the first
 * bnn_bn_workspace bytes of its workspace) with dgamma / dbeta (mode 2: the digit scale + zeroed
 * dsum); the *_pre entries then run only the apply pass (same arguments as their plain forms;
 * p = 0).  Same math as the plain entries, the statistics summed in another order.
 * replaces: the statistics reduction of BatchNorm1d's backward (mnist-dist2.py:66-74) */
int bnn_bn_bwd_stats_pre(const float* part, int64_t R, int64_t M, int64_t C, int32_t mode, const float* gamma,
                         const float* save_invstd, float* dgamma, float* dbeta, float* scale, int64_t* dsum,
                         void* work, bnn_stream_t stream);
int bnn_bn_bwd_q6_pre(const float* x, const float* dy, int64_t M, int64_t C, const float* gamma, const float* beta,
                      const float* save_mean, const float* save_invstd, const float* save_mean_lo, int32_t hardtanh,
                      float p, uint64_t seed, float* dx, float* dgamma, float* dbeta, uint8_t* rlo, uint8_t* rhi,
                      uint8_t* rsc, uint8_t* rres, uint8_t* clo, uint8_t* chi, uint8_t* csc, float* colsum, void* work,
                      bnn_stream_t stream);
int bnn_bn_bwd_q6_i16_pre(const int16_t* x16, const float* xbias, const float* dy, int64_t M, int64_t C,
                          const float* gamma, const float* beta, const float* save_mean, const float* save_invstd,
                          const float* save_mean_lo, int32_t hardtanh, float p, uint64_t seed, float* dx,
                          float* dgamma, float* dbeta, uint8_t* rlo, uint8_t* rhi, uint8_t* rsc, uint8_t* rres, uint8_t* clo,
                          uint8_t* chi, uint8_t* csc, float* colsum, void* work, bnn_stream_t stream);
int bnn_bn_bwd_i8cols_pre(const float* x, const float* dy, int64_t M, int64_t C, const float* gamma,
                          const float* beta, const float* save_mean, const float* save_invstd,
                          const float* save_mean_lo, int32_t hardtanh, float* dgamma, float* dbeta, int8_t* digits_t,
                          int64_t ldqt, int64_t plane, float* scale, float* colsum, int64_t* dsum, void* work,
                          bnn_stream_t stream);

/* ---------------------------------------------------------------- narrow fp32 Linear
 * The binarized CNN's classifier nn.Linear(7*7*32, 10) (BASELINE config 4; fp32, not binarized):
 * y = x.w^T + b for x [M][K], w [N][K], y [M][N] (N in {1,2,4,8,10,16}, K % 4 == 0, N*K <= 16384
 * (w is staged whole in LDS), x and w 16-B aligned, b nullable).  Backward: dx = dy.w, dw = dy^T.x,
 * db = column sums of dy (each output nullable); dw / db need `work` of
 * bnn_linear_nsmall_workspace(M, N, K) bytes.  fp32 products
 * and sums in a fixed order (deterministic), the numerics class of torch's F.linear. */
int64_t bnn_linear_nsmall_workspace(int64_t M, int64_t N, int64_t K);
int bnn_linear_nsmall_fwd(const float* x, int64_t M, int64_t K, const float* w, const float* b, int64_t N,
                          float* y, bnn_stream_t stream);
int bnn_linear_nsmall_bwd(const float* x, const float* w, const float* dy, int64_t M, int64_t K, int64_t N,
                          float* dx, float* dw, float* db, void* work, int64_t work_bytes, bnn_stream_t stream);
/* out[n] = sum over rows of y[m][n] (row-major, leading dimension ld) for a narrow matrix: N <= 16,
 * 0 < M <= 32768 -- the fused head's bias gradient db4 = dY4.sum(0) (mnist-dist2.py:76, fc4's
 * bias).  One workgroup, double sums in a fixed order (deterministic). */
int bnn_col_sums_narrow(const float* y, int64_t M, int64_t N, int64_t ld, float* out, void* stream);

/* The training step's loss (replaces criterion = nn.CrossEntropyLoss() on the nets' LogSoftmax
 * output, mnist-dist2.py:118-137): p [M][C] fp32 rows (C in {2, 10, 16, 32, 64}: the MNIST heads),
 * y [M] int64 targets.  fwd writes the mean loss to loss[0] (device) and keeps each row's
 * log-sum-exp and the kept-row count n in work (bnn_cross_entropy_workspace(M) bytes) for bwd,
 * which writes dp = go[0] / n * (softmax(p) - onehot(y)) with go read on the device.  Rows whose
 * target equals ignore_index (torch's default -100) are skipped as torch skips them: no loss term,
 * a zero gradient row, n counts the others (all ignored: loss NaN, gradient 0).  fp32 row
 * arithmetic as torch's log_softmax; the row losses summed in double in a fixed order
 * (deterministic); any other target outside [0, C) makes the loss NaN. */
int bnn_cross_entropy_ok(int64_t C);
int64_t bnn_cross_entropy_workspace(int64_t M);
int bnn_cross_entropy_fwd(const float* p, const int64_t* y, int64_t M, int64_t C, int64_t ignore_index, float* loss,
                          void* work, int64_t work_bytes, bnn_stream_t stream);
int bnn_cross_entropy_bwd(const float* p, const int64_t* y, int64_t M, int64_t C, int64_t ignore_index,
                          const float* go, const void* work, float* dp, bnn_stream_t stream);

/* ---------------------------------------------------------------- (3) STE backward helpers
 * Hardtanh backward: g_out = g_in * (-1 < x < 1) (strict), as nn.Hardtanh (mnist-dist2.py:51). */
int bnn_hardtanh_bwd(const float* x, const float* g, float* out, int64_t n, bnn_stream_t stream);

/* Fused latent update (replaces mnist-dist2.py:131-137 around torch.optim.Adam, :91):
 * p <- Adam(p, grad*grad_scale) with torch's bias-corrected formula, then, if clamp != 0,
 * p <- clamp(p, -1, 1).  step = 1-based Adam step count after this update. */
/* Tuning hook: 0 makes bnn_adam_clamp_pack use its 64 x 64-tile kernel even for whole 256 x 256
 * tiles (A/B timing and the equality test); 1 (default) the 1-KiB-run form for grids of >= 512 whole
 * tiles; 2 the 1-KiB-run form at every whole-tile shape. */
int bnn_adam_pack_set_tile256(int32_t on);
int bnn_adam_clamp(float* p, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                   float lr, float beta1, float beta2, float eps, int64_t step, float grad_scale,
                   int32_t clamp, bnn_stream_t stream);

/* The same update fused with the next forward's weight packing: p is a latent
 * weight [N][K] row-major (ld = K; grad, exp_avg, exp_avg_sq alike), updated in place exactly as
 * bnn_adam_clamp does (bit-identical p, m, v), and in the same pass sign(p_new) is written as the
 * ternary rows q -- fmt 0: int8 [N][ldq] (ldq multiple of 64 >= round_up(K,64)); fmt 1: FP4
 * nibbles [N][ldq bytes] (ldq multiple of 128, 2*ldq >= round_up(K,256)) -- and/or the int8
 * transpose qt [K][ldqt] (qt_fmt 0: int8, ldqt multiple of 64 >= round_up(N,64); qt_fmt 1 / 2: FP4
 * nibbles, ldqt bytes, rows or panels as in bnn_sign_pack_fp4); padding zero-filled, as
 * bnn_sign_pack_i8 / bnn_sign_pack_fp4 of p_new would write them.  q or qt may be NULL (not both).
 * replaces: p.data.copy_(p.org); Adam.step(); p.org.copy_(p.data.clamp_(-1,1)) (mnist-dist2.py:
 * 131-137) and the weight sign of the next forward (binarized_modules.py:79). */
int bnn_adam_clamp_pack(float* p, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t N,
                        int64_t K, float lr, float beta1, float beta2, float eps, int64_t step,
                        float grad_scale, int32_t clamp, int32_t fmt, void* q, int64_t ldq, int8_t* qt,
                        int64_t ldqt, int32_t qt_fmt, bnn_stream_t stream);

/* ---------------------------------------------------------------- device-step form (HIP graphs)
 * A captured training step replays with frozen kernel arguments, so the per-step quantities the
 * host passes by value (Adam's bias corrections, the dropout seed) are read from device memory:
 * ctr[0] = the step index since the counter was created, advanced by bnn_counter_add at the end
 * of each optimizer step (inside the graph).
 * bnn_adam_schedule: host-only; out[2i], out[2i+1] = the (step_size, sqrt(1 - beta2^s)) that
 * bnn_adam_clamp computes for step s = step0 + i (same double arithmetic, bit-identical).
 * bnn_adam_clamp_sched / bnn_adam_clamp_pack_sched: bnn_adam_clamp / bnn_adam_clamp_pack with
 * those two values taken from sched[2 * ctr[0]] on the device.
 * bnn_set_seed_counter: process-wide; while non-NULL every dropout launch (bnn_bn_dropout_*,
 * bnn_bn_bwd_q6, bnn_dropout_mask) draws its mask from seed + ctr[0] * 0xD1B54A32D192ED03. */
int bnn_adam_schedule(float lr, float beta1, float beta2, int64_t step0, int64_t n, float* out);
/* bnn_adam_clamp (or, with sched/ctr non-NULL, bnn_adam_clamp_sched) over up to 16 tensors in one
 * launch: host arrays of `count` device pointers, element counts, Adam step counts and clamp
 * flags.  Bit-identical per tensor to the single-tensor entries; one launch for a network's small
 * parameters (biases, BatchNorm affine parameters, the head) instead of one each. */
int bnn_adam_clamp_multi(int32_t count, float* const* p, const float* const* grad, float* const* exp_avg,
                         float* const* exp_avg_sq, const int64_t* n, const int64_t* step, const int32_t* clamp,
                         float lr, float beta1, float beta2, float eps, const float* sched, const int64_t* ctr,
                         float grad_scale, bnn_stream_t stream);
int bnn_adam_clamp_sched(float* p, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float beta1,
                         float beta2, float eps, const float* sched, const int64_t* ctr, float grad_scale,
                         int32_t clamp, bnn_stream_t stream);
int bnn_adam_clamp_pack_sched(float* p, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t N, int64_t K,
                              float beta1, float beta2, float eps, const float* sched, const int64_t* ctr,
                              float grad_scale, int32_t clamp, int32_t fmt, void* q, int64_t ldq, int8_t* qt,
                              int64_t ldqt, int32_t qt_fmt, bnn_stream_t stream);
int bnn_counter_add(int64_t* ctr, int64_t v, bnn_stream_t stream);
int bnn_set_seed_counter(const int64_t* ctr);

#ifdef __cplusplus
}
#endif
#endif /* BNN_H_ */
