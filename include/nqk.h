/*
 * nqk.h — C ABI of libnqk.so, the MI355X (gfx950) backend for numpy-quant's
 * quantized per-node execution hot path.
 *
 * The reference has no FFI of its own: its operator boundary is
 *   onnx_operator_implementation(op, inputs, attrs)   numpy_quant/model.py:65-213
 * plus the L1 array functions in numpy_quant/numpy_quantization.py:7-72 and
 * numpy_quant/numpy_helper.py:73-112.  Each entry point below replaces one of
 * those (cited per function); the Python host (numpy-quant_amd/numpy_quant/_lib.py)
 * binds them with ctypes exactly as INTEGRATION.md shows.
 *
 * Conventions
 *   - plain pointers and sizes only; device pointers come from nqk_malloc;
 *   - every call is asynchronous on the library's single stream for the current
 *     device (one process per GPU), except the *_sync / memcpy_d2h calls;
 *   - kernels never allocate; callers own every buffer;
 *   - return 0 on success, <0 on error; nqk_last_error() describes the last error
 *     of the calling thread (the Python layer raises ValueError / RuntimeError);
 *   - dtype codes (NQK_*) select the storage of integer tensors:
 *       quantized values of bit width bw live in the narrowest of i8/i16/i32/i64
 *       that holds [-2^(bw-1), 2^(bw-1)-1] (the reference stores int64 always,
 *       tensor.py:158-166; values are identical, storage is narrower).
 *   - "zero point term" of a MatMul output (numpy_quantization.py:49-61) is never
 *     materialised: it is rebuilt on the fly from per-row sums of A and per-column
 *     sums of B:  zpt[b,m,n] = row[a(b),m]*zpb + col[b(b),n]*zpa - zpa*zpb*K,
 *     with the terms enabled by NQK_ZP_ROW / NQK_ZP_COL / NQK_ZP_SCALAR flags.
 *   - batch map (broadcast batch dims of np.matmul, numpy_quantization.py:47): the
 *     output batch index b is split as (bo, bi) = (b / inner, b % inner) and the
 *     A / B matrix index is bo*ao + bi*ai / bo*bo_ + bi*bi_ (in matrices); `bmap`
 *     is a HOST array of 5 int64 (NULL = no broadcast: every operand has `batch`).
 */
#ifndef NQK_H
#define NQK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum nqk_dtype { NQK_I8 = 1, NQK_I16 = 2, NQK_I32 = 3, NQK_I64 = 4, NQK_F32 = 5 };

enum nqk_zp_flags {
  NQK_ZP_NONE = 0,
  NQK_ZP_SCALAR = 1,  /* subtract a scalar zero point zp                       */
  NQK_ZP_ROW = 2,     /* + row[a(b), m] * zpb  (rowsum(A) term, zero_point_b)   */
  NQK_ZP_COL = 4,     /* + col[b(b), n] * zpa  (colsum(B) term, zero_point_a)   */
  NQK_ZP_KCONST = 8,  /* - zpa * zpb * K       (both operands asymmetric)       */
  NQK_ZP_FULL = 16    /* + row[i]: a materialised int64 zero-point array (flat) */
};

/* ---------------------------------------------------------------- runtime */
int nqk_init(int device);              /* select device, create the stream (idempotent) */
int nqk_device_count(int* count);
const char* nqk_last_error(void);
int nqk_malloc(void** ptr, size_t bytes);
int nqk_free(void* ptr);
int nqk_memcpy_h2d(void* dst, const void* src, size_t bytes);   /* returns when the copy is done */
int nqk_memcpy_d2h(void* dst, const void* src, size_t bytes);   /* stream-ordered, synchronous */
int nqk_memcpy_d2d(void* dst, const void* src, size_t bytes);   /* async */
int nqk_memset(void* ptr, int value, size_t bytes);             /* async */
int nqk_sync(void);
int nqk_stream(void** stream);         /* the library's hipStream_t */
/* side streams 1..3 for independent work (the fused plan's batch parts):
 * nqk_set_stream(s) routes every later call to stream s, nqk_set_stream(0) back;
 * nqk_stream_fork makes every side stream wait for all work issued so far on stream 0,
 * nqk_stream_join makes stream 0 wait for all work issued so far on the side streams. */
int nqk_set_stream(int which);
int nqk_stream_fork(void);
int nqk_stream_join(void);
/* stream timers: record start / stop events, nqk_timer_ms waits for stop */
int nqk_timer_start(void);
int nqk_timer_stop(void);
int nqk_timer_ms(float* ms);
/* events on the library stream (per-kernel timing inside bench.py) */
int nqk_event_create(void** event);
int nqk_event_record(void* event);
int nqk_event_elapsed(void* start, void* stop, float* ms);   /* waits for stop */
int nqk_event_destroy(void* event);
/* the current stream waits for the work an event recorded (cross-stream ordering of the fused
 * plan's batch parts: NQK_STREAM_LAG) */
int nqk_event_wait(void* event);
/* hipGraph capture of everything issued between begin and end (relaxed mode: the
 * caller's allocator may still allocate); abort drops a capture that failed part-way */
int nqk_graph_begin(void);
int nqk_graph_end(void** graph_exec);
int nqk_graph_abort(void);
int nqk_graph_launch(void* graph_exec);
int nqk_graph_destroy(void* graph_exec);

/* ------------------------------------------------- L1: quantization kernels */
/* quantize  numpy_quantization.py:24-34 (tensor.py:299-301 quantize_tensor)
 *   q = int(rint(clip(f64(zp) + f64(f32(x / s)), lo, hi)))   (has_zp)
 *   q = int(rint(clip(f32(x / s), f32(lo), f32(hi))))        (!has_zp)
 * optional rowsum (int64, per row of length row_len, may be NULL). */
int nqk_quantize(const float* x, void* q, int q_dtype, int64_t n, float scale,
                 int64_t zp, int has_zp, int bit_width, int64_t* rowsum, int64_t row_len);

/* dequantize  numpy_quantization.py:37-41, tensor.py:261-265
 *   out = f32( f64(q - zpt) * f64(s) ) over out[batch][M][N]; zpt from zp_flags.
 *   For a plain tensor pass batch=1, M=1, N=n and NQK_ZP_SCALAR or NONE. */
int nqk_dequantize(const void* q, int q_dtype, float* out, int64_t batch, int64_t M, int64_t N,
                   float scale, int zp_flags, int64_t zp, int64_t zpa, int64_t zpb, int64_t K,
                   const int64_t* row, const int64_t* col, const int64_t* bmap /* 5 */);

/* requantize  numpy_quantization.py:64-72 (+ QTensor.__add__ of the Gemm bias,
 * tensor.py:255-259, model.py:130):  d = dequantize(acc + bias[n]);
 *   q = int(clip(rint(f64(rz) + f64(f32(f32(1/rs) * d))), lo, hi)) */
int nqk_requantize(const void* acc, int acc_dtype, const void* bias, int bias_dtype,
                   void* out, int out_dtype, int64_t batch, int64_t M, int64_t N, float scale,
                   int zp_flags, int64_t zp, int64_t zpa, int64_t zpb, int64_t K,
                   const int64_t* row, const int64_t* col, const int64_t* bmap,
                   float res_scale, int64_t res_zp, int has_res_zp, int bit_width);

/* QTensor.relu  tensor.py:212-215:  out[i] = q[i] < zp ? zp : q[i]  (zp the tensor's scalar
 * zero point; out may be wider than q when zp lies outside q's storage range) */
int nqk_relu_q(const void* q, int q_dtype, void* out, int out_dtype, int64_t n, int64_t zp);

/* row / column sums of an integer matrix batch (the q_matmul zero-point terms,
 * numpy_quantization.py:52,55,58-59), int64: row[b][m] = sum_k A[b][m][k] (row-major,
 * lda), col[b][n] = sum_k B[b][k][n] (B given TRANSPOSED as Bt[b][n][k], ldb). */
int nqk_rowsum(const void* a, int dtype, int64_t* out, int64_t batch, int64_t rows, int64_t k,
               int64_t ld, int64_t batch_stride);

/* ------------------------------------------------------ L1: q_matmul GEMMs */
/* q_matmul's integer product, numpy_quantization.py:47:
 *   C[b][m][n] = sum_k A[b'][m][k] * Bt[b''][n][k]     (int32 out)
 * int8 operands on v_mfma_i32_32x32x32_i8; lda/ldb multiples of 16 bytes; K is
 * zero-padded by the caller to a multiple of 16 (zeros add nothing). */
int nqk_qgemm_i8(const int8_t* a, const int8_t* bt, int32_t* c, int64_t batch, int64_t M,
                 int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc,
                 const int64_t* bmap /* 5: inner, ao, ai, bo, bi in matrices */,
                 int64_t a_mat_stride, int64_t b_mat_stride, int64_t c_mat_stride);
/* any-width integer operands (bit widths > 8, tiny shapes), int64 accumulation on
 * VALU; B[K][N] addressed by element strides (b_sk, b_sn) */
int nqk_qgemm_generic(const void* a, int a_dtype, const void* b, int b_dtype, int64_t* c,
                      int64_t batch, int64_t M, int64_t N, int64_t K, int64_t a_sm, int64_t a_sk,
                      int64_t b_sk, int64_t b_sn, int64_t ldc, const int64_t* bmap,
                      int64_t a_mat_stride, int64_t b_mat_stride, int64_t c_mat_stride);

/* ------------------------------------------- float32 GEMM (BLAS-order exact) */
/* C = A[M][K] . B[K][N] (element strides a_sm/a_sk, b_sk/b_sn).  Every output element is the
 * reference BLAS's summation: K is cut into OpenBLAS level-3 blocks (GEMM_Q=448
 * rule), each block a k-ordered fmaf chain from 0, blocks added in order.  Used
 * by Conv (numpy_helper.py:73-92 x.dot(w)) and by float MatMul/Gemm of the
 * calibration forward (model.py:153-157, 122-131 via np.matmul). */
int nqk_sgemm(const float* a, const float* b, float* c, int64_t batch, int64_t M, int64_t N,
              int64_t K, int64_t a_sm, int64_t a_sk, int64_t b_sk, int64_t b_sn, int64_t ldc,
              const int64_t* bmap, int64_t a_mat_stride, int64_t b_mat_stride, int64_t c_mat_stride);

/* One-row float product y[N] = x[1][K] . B[K][N] where B's columns are contiguous
 * (bt[N][ldb], the layout of the Gemm's w.T view, model.py:122-131): NumPy's matmul hands
 * that to OpenBLAS's GEMV-T (vector_matrix -> cblas_sgemv), and this reproduces its order
 * bit for bit — the N columns split over `threads` chunks as OpenBLAS's gemv threading does
 * (one chunk when K*N < 460800), 8-lane fma / 4-lane SSE kernels per column class, K blocks
 * of 4096, trailing rows (oracle/openblas_order.py); for K <= 8 with ldb == K, OpenBLAS's
 * small-m kernels in every chunk of at most 16 384 columns (their column classes identified
 * in round 6: k_sgemv_small).  `threads` = OpenBLAS's thread count of the NumPy being matched. */
int nqk_sgemv_t(const float* x, const float* bt, float* y, int64_t N, int64_t K, int64_t ldb, int64_t threads);

/* One-row float product y[N] = x[1][K] . B[K][N] with B row-major (b[K][ldb], ldb >= N: a MatMul's
 * weight, tensor.py:100-101 FTensor.matmul -> np.matmul): NumPy hands it to OpenBLAS's GEMV-N, and
 * this reproduces its order bit for bit (round 6, oracle/openblas_order.py sgemv_n: K <= 48 fma
 * chains; N < 4 pairs; else the outputs split over `threads` chunks, blocks of 4096 outputs, the
 * 8-row and 16-row kernels' groups of 8 products, trailing outputs as fma chains).  `threads` as
 * nqk_sgemv_t. */
int nqk_sgemv_n(const float* x, const float* b, float* y, int64_t N, int64_t K, int64_t ldb, int64_t threads);

/* A 1 x 1 one-row product of NumPy's matmul (model.py:122-131 Gemm / tensor.py:100-101
 * FTensor.matmul): cblas_sdot's order at every length (the SkylakeX vector kernel's
 * accumulators over the first K & -32 products, the tail's f32 products summed in double;
 * round 6).  N must be 1 (one-row products with N > 1: nqk_sgemv_t); bt is the K-vector. */
int nqk_sgemv_small(const float* x, const float* bt, float* y, int64_t N, int64_t K, int64_t ldb);

/* im2col for Conv (numpy_helper.py:18-70): x NCHW f32 -> cols[N*Ho*Wo][KH*KW*C]
 * (column order kh, kw, c), zero padding pads = (ph0, pw0, ph1, pw1). */
/* ViT patch embedding in one GEMM (plan.py FusedEmbed): Conv as im2col . W in the BLAS
 * order (nqk_sgemm), + bias, NCHW -> [B, HW, N] Reshape/Transpose, Concat behind the class
 * token, + position embedding (model.py Conv/Reshape/Transpose/Concat/Add, in the node
 * loop's rounding order):  out[b][0][n] = cls[n] + pos[0][n],
 *   out[b][1+t][n] = (sgemm(cols, w)[b*hw + t][n] + bias[n]) + pos[1+t][n].
 * cols [images*hw][K] (nqk_im2col), w [K][N], pos [hw+1][N], out [images][hw+1][N]; K even. */
int nqk_sgemm_embed(const float* cols, const float* w, const float* bias, const float* cls, const float* pos,
                    float* out, int64_t images, int64_t hw, int64_t N, int64_t K);
/* im2col of a patchify Conv (stride = kernel, no padding, numpy_helper.py:18-70) fused with
 * the dequantize of its int8 input (numpy_quantization.py:37-41):
 * cols[(b,oy,ox)][(ki,kj,ci)] = f32((q[b][ci][oy*kh+ki][ox*kw+kj] - zp) * scale). */
int nqk_patchify_dequant(const int8_t* q, float* cols, int64_t n, int64_t c, int64_t h, int64_t w, int64_t kh,
                         int64_t kw, float scale, int64_t zp);
/* The patch embedding of a quantized image without the im2col matrix (round 3): the
 * patchify + dequantize above folded into the A-operand load of the nqk_sgemm_embed GEMM,
 * same bits (model.py:95-100 Conv on the dequantized input, tensor.py:256-264 fconv2d,
 * numpy_helper.py:18-92 im2col, then the Reshape / Transpose / Concat / Add(pos) chain).
 * q: int8 [images][3][h][w], 16 x 16 patches; wt: the weights as [N][768] in the
 * (ki, kj, ci) order with every 16-block permuted to p = (k & 1) * 8 + (k >> 1)
 * (numpy_quant/plan.py FusedEmbed); N % 64 == 0. */
/* The order nqk_embed_q expects its weights in, per 16-k block: 32 -> p = (k & 1) * 8 + (k >> 1) (the
 * v_mfma_f32_32x32x2_f32 kernel), 16 -> p = (k & 3) * 4 + (k >> 2) (the v_mfma_f32_16x16x4_f32 kernel;
 * round 6).  Callers permute the weights by it (plan.py FusedEmbed). */
int nqk_embed_weight_order(void);
int nqk_embed_q(const int8_t* q, float scale, int64_t zp, const float* wt, const float* bias, const float* cls,
                const float* pos, float* out, int64_t images, int64_t c, int64_t h, int64_t w, int64_t kh,
                int64_t kw, int64_t N);
int nqk_im2col(const float* x, float* cols, int64_t n, int64_t c, int64_t h, int64_t w,
               int64_t kh, int64_t kw, int64_t ph0, int64_t pw0, int64_t sh, int64_t sw,
               int64_t ho, int64_t wo);

/* ------------------------------------------- float ops (model.py:65-213) */
enum nqk_binop { NQK_ADD = 0, NQK_SUB = 1, NQK_MUL = 2, NQK_DIV = 3 };
/* out[i] = a[ia] op b[ib] over an N-d broadcast (ndim <= 6; strides in elements) */
int nqk_binary_f32(int op, const float* a, const float* b, float* out, int ndim,
                   const int64_t* shape, const int64_t* a_strides, const int64_t* b_strides);
enum nqk_unop { NQK_NEG = 0, NQK_EXP = 1, NQK_ERF = 2, NQK_SQRT = 3, NQK_RELU = 4,
                NQK_SIGMOID = 5, NQK_RECIP = 6, NQK_TANH = 7 };
/* NumPy-exact where it matters: EXP is numpy's AVX512F float32 exp algorithm
 * (bit-identical to np.exp on all 2^32 inputs), ERF is numpy_helper.py:95-112. */
int nqk_unary_f32(int op, const float* x, float* out, int64_t n);
/* x + scalar (FTensor.__add__ with a Python float, tensor.py:158-164) */
int nqk_add_scalar_f32(const float* x, float s, float* out, int64_t n);
/* Softmax over the last axis (tensor.py:211-218): e = exp(x - max); e / pairwise_sum(e) */
int nqk_softmax_lastdim(const float* x, float* out, int64_t rows, int64_t cols);
/* LayerNormalization over the last axis (model.py:134-152), NumPy pairwise means */
int nqk_layernorm_lastdim(const float* x, const float* gamma, const float* beta, float* out,
                          int64_t rows, int64_t cols, float eps);
/* mean over the last axis with NumPy's pairwise summation (np.mean f32) */
int nqk_mean_lastdim(const float* x, float* out, int64_t rows, int64_t cols);
/* global min and max (calibration, model.py:333-336) -> out[0]=min, out[1]=max */
int nqk_minmax_f32(const float* x, int64_t n, float* out2, float* scratch, int64_t scratch_len);
/* N-d strided copy for Transpose / Concat / Slice / Expand / Gather / padding
 * (element size 1, 2, 4 or 8 bytes; ndim <= 6; strides in elements) */
int nqk_copy_strided(const void* src, void* dst, int elem_size, int ndim, const int64_t* shape,
                     const int64_t* src_strides, const int64_t* dst_strides);
/* where(cond, a, b) with broadcasting (tensor.py:323-325), f32 */
int nqk_where_f32(const int64_t* cond, const float* a, const float* b, float* out, int ndim,
                  const int64_t* shape, const int64_t* c_strides, const int64_t* a_strides,
                  const int64_t* b_strides);

/* ------------------------------------------- fused device plan (plan.py) */
/* Epilogue of nqk_qgemm_fused: the consumer chain of a q_matmul output as the
 * reference's node loop runs it (dequantize -> float ops -> quantize), per element. */
enum nqk_epi { NQK_EPI_QKV = 0, NQK_EPI_SCORES = 1, NQK_EPI_PV = 2, NQK_EPI_RESID = 3, NQK_EPI_GELU = 4,
               NQK_EPI_NULL = 5 /* diagnostic: no stores (main-loop timing) */ };
typedef struct nqk_epilogue {
  int32_t zp_flags, bit_width, group_cols, tokens, heads, hdim, ld_out;
  int32_t col_absmax;                  /* max |col[n]| if known (0: unknown); lets the   */
                                       /* epilogue dequantize in f32 when provably exact */
  int64_t zpa, zpb, kdim;              /* zero-point term: ROW / COL / KCONST flags; row  */
  const int64_t* row;                  /* sums of A and Bt are computed in-kernel unless  */
  const int64_t* col;                  /* `col` holds precomputed int64 column sums of B  */
  float s_acc[3];                       /* dequant scale s_a*s_b per column group       */
  float s_out[3];                       /* quantize scale of the consumer value         */
  int64_t zp_out[3];                    /* quantize zero point of the consumer value    */
  void* out[3];                         /* outputs per column group                     */
  const float* bias;                    /* dequantized bias [N] (EPI_QKV/RESID/GELU)    */
  const float* resid;                   /* residual [M][N] (EPI_RESID)                  */
  float div, add1, mul2;                /* Div constant (8 / sqrt 2), GELU +1 and *0.5  */
  int32_t b_packed;                     /* 1: bt is an nqk_pack_b image; 2: nqk_pack_b4  */
  const int32_t* colterm;               /* optional: col[n] * zpa as int32 (the persistent */
                                        /* projection GEMM needs it; NULL: not used)     */
  const int8_t* bt_pg;                  /* optional: the nqk_pack_pg image of the same Bt;  */
                                        /* when set, the 16x16x64 persistent GEMM (k_pg)  */
                                        /* runs the cases it takes (NULL: not used)       */
  const void* gelu_lut;                 /* optional (EPI_GELU with bt_pg): the table of    */
  float lut_k[5];                       /* nqk_gelu_lut_build, its bucket coordinate and   */
  int32_t lut_n;                        /* entry count; k_pg then looks the GELU chain's   */
                                        /* output bytes up instead of computing them       */
  int32_t col_l1max;                    /* optional: max over columns of sum_k |Bt[n][k]|  */
                                        /* (0: unknown); |acc| <= 2^(bw-1) col_l1max then  */
                                        /* bounds the f32-exactness test more tightly than */
                                        /* 2^(2bw-2) K (FFN-down at K = 3072)              */
  /* optional (EPI_RESID, round 6): the consumer LayerNormalization (model.py:134-152) fused
   * into the epilogue, quantized for ITS consumer MatMul (numpy_quantization.py:24-34):
   * ln_out [M][N] int8 = quantize(LN(y) * ln_gamma + ln_beta, ln_scale, ln_zp, bit_width) of
   * the f32 rows y the epilogue writes to out[0].  Whole rows per tile: N = 192 only (NumPy's
   * pairwise tree of two 96-column leaves, the ViT-Ti width); anything else fails.  Bit-identical
   * to nqk_ln_quant on out[0].  NULL: no LayerNorm. */
  const float* ln_gamma;
  const float* ln_beta;
  int8_t* ln_out;
  float ln_eps, ln_scale;
  int64_t ln_zp;
} nqk_epilogue;
/* int8 MFMA GEMM C = A . Bt^T (layouts as nqk_qgemm_i8) with a fused epilogue:
 *   QKV    model.py MatMul -> Add(bias) -> Reshape -> Transpose -> quantize, 3 groups
 *   SCORES MatMul(Q, K^T) -> Div(const)                          -> f32
 *   PV     MatMul(P, V) -> Transpose -> Reshape -> quantize      -> int8
 *   RESID  MatMul -> Add(bias) -> Add(residual)                  -> f32
 *   GELU   MatMul -> Add(bias) -> Div -> Erf -> Add -> Mul -> Mul -> quantize */
/* Tile-packed copy of a constant int8 weight operand Bt [N][K] (K % 64 == 0) for
 * nqk_qgemm_fused with b_packed = 1: [ceil(N/256)][K/64] blocks of 256 rows x 64 bytes in
 * the GEMM's LDS stage image (zero rows past N); out holds ceil(N/256)*256*K bytes.  The packed
 * operand is read as whole 128-byte lines (replaces no reference function: a layout of
 * the same numpy_quantization.py:44-61 q_matmul operand). */
int nqk_pack_b(const int8_t* bt, int8_t* out, int64_t N, int64_t K, int64_t ldb);
/* int4 weights (every value in [-8, 7], bit width <= 4): the same tiles nibble-packed,
 * ceil(N/256)*256*K/2 bytes; the GEMM unpacks them in registers after the LDS stage
 * (b_packed = 2).  BASELINE configs[4] ("int4 packed weights"). */
int nqk_pack_b4(const int8_t* bt, uint8_t* out, int64_t N, int64_t K, int64_t ldb);
/* Tile-packed copy of Bt [N][K] (K % 64 == 0) for the persistent 16x16x64 projection GEMM
 * (nqk_epilogue.bt_pg): [ceil(N/256)][K/64] stages of 256 rows x 64 bytes, 16-byte chunks
 * swizzled for conflict-free fragment reads; each wave's 64 columns permuted so that a lane's
 * MFMA results are 16 consecutive output columns (layout 0: QKV / GELU, int8 outputs) or
 * 4 x 4 columns whose 16-byte stores cover 64 contiguous bytes per row (layout 1: the
 * residual epilogues, f32 outputs); ceil(N/256)*256*K bytes (a layout of the
 * numpy_quantization.py:44-61 q_matmul operand, replaces no reference function). */
int nqk_pack_pg(const int8_t* bt, int8_t* out, int64_t N, int64_t K, int64_t ldb, int layout);
/* int4 weights (every value in [-8, 7], bit width <= 4): the same stages nibble-packed, 256 rows
 * x 32 bytes each, ceil(N/256)*256*K/2 bytes; k_pg unpacks them in registers after the LDS stage
 * (nqk_epilogue.b_packed = 2 with bt_pg = this image).  BASELINE configs[4]. */
int nqk_pack_pg4(const int8_t* bt, uint8_t* out, int64_t N, int64_t K, int64_t ldb, int layout);
/* The FFN-up epilogue's GELU chain as a table (round 4; up to 1024 entries since round 5): model.py Div -> Erf -> Add -> Mul ->
 * Mul on f32 (numpy_helper.py:95-112 erf) followed by numpy_quantization.py:24-34 quantize
 * with (s_out, zp_out, bit_width), as a step function of the dequantized, biased f32 value h:
 * at most 1024 buckets of 8 bytes in lut (a 16-byte aligned device buffer of nqk_gelu_lut_capacity()
 * bytes: 8 KiB since round 5, 4 KiB in round 4 — size it by the call, not a constant), the bucket
 * coordinate in k_out[5], the entry count in *n_out (the 128 x 256-tile k_pg takes tables of up
 * to 512 entries, the 256 x 256 one up to 1024; the builder prefers <= 512).  Every entry comes from the exact chain,
 * and the table is then compared with the exact chain on all 2^32 - 2^24 finite f32 inputs:
 * *n_out = 0 (return 0) when the table cannot represent the chain exactly, when the chain is
 * not the GELU of model.py (div = f32(sqrt 2), add1 = 1, mul2 = 0.5) or bit_width is not in
 * 2..8.  Blocking (plan build time). */
int nqk_gelu_lut_build(float s_out, int64_t zp_out, int32_t bit_width, float div, float add1, float mul2, void* lut,
                       float* k_out, int32_t* n_out);
/* Bytes nqk_gelu_lut_build may write to its lut buffer (the API version check of the table
 * size; k_pg itself reads only the 8 * lut_n bytes of the table it is given). */
int nqk_gelu_lut_capacity(void);
/* The number of finite f32 inputs on which a table (n entries, coordinate k) differs from the
 * exact chain (tests). */
int nqk_gelu_lut_check(float s_out, int64_t zp_out, int32_t bit_width, float div, float add1, float mul2,
                       const void* lut, const float* k, int32_t n, uint64_t* mismatches);
int nqk_qgemm_fused(int epi, const int8_t* a, const int8_t* bt, int64_t batch, int64_t M, int64_t N, int64_t K,
                    int64_t lda, int64_t ldb, const int64_t* bmap, int64_t a_mat_stride, int64_t b_mat_stride,
                    const nqk_epilogue* params);
/* Which kernel the last nqk_qgemm_fused call launched (tests / diagnostics): 0 small tiles
 * (k_qgemm_epi), 1 128x256 tiles (k_qgemm_big), 2 ping-pong 256x256 (k_qgemm_pp), 3 the
 * persistent projection GEMM with the epilogue overlapped (k_proj), 4 the persistent 16x16x64
 * GEMM with two workgroups per CU (k_pg), 5 k_pg on 256 x 256 tiles (one 512-thread workgroup
 * per CU, B shared by its two row halves), 6 / 7 the same two with the GELU table epilogue
 * (nqk_gelu_lut_build); -1 none yet. */
int nqk_qgemm_last_kernel(void);
/* LayerNormalization (model.py:134-152) fused with the consumer MatMul's quantize */
int nqk_ln_quant(const float* x, const float* gamma, const float* beta, int8_t* out, int64_t rows, int64_t cols,
                 float eps, float scale, int64_t zp, int bit_width);
/* Softmax (tensor.py:211-218) fused with quantize; out row stride ldo (zero pad), int64 row sums */
int nqk_softmax_quant(const float* x, int8_t* out, int64_t* rowsum, int64_t rows, int64_t cols, int64_t ldo,
                      float scale, int64_t zp, int bit_width);
/* int8 [nb][R][C] -> [nb][C][Rp] (zero padded) and rowsum[nb][C] = sum over R (may be NULL) */
int nqk_transpose_pad_i8(const int8_t* src, int8_t* dst, int64_t* rowsum, int64_t nb, int64_t R, int64_t C,
                         int64_t Rp);

/* Fused self-attention of one layer: MatMul(Q, K^T) -> Div -> Softmax -> quantize ->
 * MatMul(P, V) -> Transpose -> Reshape -> quantize (model.py:153-157 MatMul, tensor.py:139-146
 * softmax, numpy_quantization.py:24-61 quantize / q_matmul), bit-identical to
 * nqk_qgemm_fused(SCORES) + nqk_softmax_quant + nqk_qgemm_fused(PV).
 * q, k, v: int8 [batch_heads][tokens][64]; ctx: int8 [batch_heads / heads][tokens][ld_out],
 * head h at columns h*64.  tokens <= 224; |zq|,|zk| <= 4096, |zp_p|,|zv| <= 1024. */
typedef struct nqk_attention {
  int32_t heads, tokens, hdim, ld_out, bit_width, pad0;
  int64_t zq, zk;          /* zero points of the quantized Q and K^T                 */
  float s_qk, div;         /* f32(s_q * s_k), the scores Div constant                */
  float s_p, s_pv;         /* softmax-output scale, f32(s_p * s_v)                   */
  int64_t zp_p, zv;        /* zero points of P and V                                 */
  float s_ctx, pad1;       /* context quantization scale                             */
  int64_t zp_ctx;          /* context zero point                                     */
} nqk_attention;
int nqk_attention_fused(const int8_t* q, const int8_t* k, const int8_t* v, int8_t* ctx, int64_t batch_heads,
                        const nqk_attention* params);

/* Diagnostic: on the device, compares the fast-division variants of NumPy's exp and the
 * reference's erf (used by the fused kernels) with the IEEE-division ones on all 2^32
 * float inputs; adds the mismatch counts to counts_dev[0] (exp) / [1] (erf), and those of
 * the attention kernel's non-positive-argument exp against NumPy's exp to [2] and of its
 * packed two-lane variant to [3] (all 2^31 inputs x <= 0), and of the exponent-add variant
 * for softmax rows with arguments in [-86.5, 0] to [4].  counts_dev and examples_dev hold 5
 * entries each. */
int nqk_selftest_fastmath(unsigned long long* counts_dev, uint32_t* examples_dev);
/* Diagnostic: checks the error bound of the GELU filter's cheap approximation on all
 * 2^32 inputs; stats_dev[0] = violations, [1] = an example, [2 + e] = max error per
 * exponent in units of |h| * 2^-24 (258 entries, zero-initialised by the caller). */
int nqk_selftest_gelu_filter(unsigned long long* stats_dev);

/* ------------------------------------------------ multi-GPU replicas (RCCL) */
int nqk_comm_unique_id(void* id128);                         /* rank 0 */
int nqk_comm_init(const void* id128, int nranks, int rank);
int nqk_comm_bcast(void* buf, size_t bytes, int root);
int nqk_comm_gather(const void* send, void* recv, size_t bytes_per_rank, int root);
int nqk_comm_barrier(void);
int nqk_comm_destroy(void);

#ifdef __cplusplus
}
#endif
#endif /* NQK_H */
