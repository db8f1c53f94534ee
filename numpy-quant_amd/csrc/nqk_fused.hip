// Fused device plan kernels for the quantized node chains of QModel.__call__
// (numpy_quant/model.py:486-565).  Every fused chain computes, per element, exactly
// the float/integer operations the reference's node-by-node loop performs, in the
// same order, so the results are bit-identical to the eager path (and to the
// reference); only the HBM round trips of the intermediate values disappear.
//
//   k_qgemm_epi<EPI>  int8 MFMA GEMM (v_mfma_i32_32x32x32_i8, 128x128x128 tiles)
//                     with the consumer chain in the epilogue:
//       EPI_QKV     dequant + bias + Reshape/Transpose + quantize (3 column groups)
//       EPI_SCORES  dequant (full zero-point term) + Div by a constant  -> f32
//       EPI_PV      dequant (full term) + Transpose/Reshape + quantize  -> int8
//       EPI_RESID   dequant + bias + residual Add                       -> f32
//       EPI_GELU    dequant + bias + Div/Erf/Add/Mul/Mul + quantize     -> int8
//   k_ln_quant        LayerNormalization (NumPy pairwise means) + quantize
//   k_softmax_quant   Softmax (NumPy exp + pairwise sum) + quantize + row sums
//   k_transpose_pad   int8 [nb][R][C] -> [nb][C][Rp] zero padded, + row sums
#include "nqk_common.h"
#include "nqk_numerics.h"

namespace nqk {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int FBM = 128, FBN = 128, FBK = 128;

// 128-byte LDS rows (8 chunks of 16 B); chunk c of row r at c ^ ((r >> 1) & 7):
// each 16-lane ds_read_b128 group then covers all 16 bank slots.
__device__ __forceinline__ int swz128(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

__device__ __forceinline__ double qclip(double u, double lo, double hi) {
  u = u < lo ? lo : u;
  return u > hi ? hi : u;
}

// quantize one f32 value with (s, zp) like numpy_quantization.py:24-34 (zp given)
__device__ __forceinline__ int quant_zp(float x, float s, double zp, double lo, double hi) {
  float t = x / s;
  double u = zp + (double)t;
  if (u != u) return (int)lo;  // unreachable for finite calibrated scales
  return (int)__builtin_rint(qclip(u, lo, hi));
}

struct Epi {
  // zero-point term (see nqk.h): zpt = row[a(b)*M+m]*zpb + col[b(b)*N+n]*zpa - zpa*zpb*K
  int zp_flags;
  int64_t zpa, zpb, kdim;
  const int64_t* row;
  const int64_t* col;
  int group_cols;        // columns per output group (EPI_QKV), else N
  float s_acc[3];        // dequant scale per group
  const float* bias;     // dequantized bias [N] or null
  float s_out[3];        // quantize scale per group
  double zp_out[3];      // quantize zero point per group
  void* out[3];          // outputs per group
  const float* resid;    // residual [M][N]
  float div;             // EPI_SCORES divisor; EPI_GELU sqrt(2) constant
  float add1, mul2;      // EPI_GELU: + 1.0, * 0.5
  int tokens, heads, hdim, ld_out;
  double lo, hi;
};

enum { EPI_QKV = 0, EPI_SCORES = 1, EPI_PV = 2, EPI_RESID = 3, EPI_GELU = 4 };

template <int EPI>
__device__ __forceinline__ void epi_store(const Epi& e, const BatchMap& bm, int64_t b, int64_t gm, int64_t gn,
                                          int64_t M, int64_t N, int32_t acc) {
  int64_t v = (int64_t)acc;
  if (e.zp_flags & NQK_ZP_ROW) v -= e.row[map_a(bm, b) * M + gm] * e.zpb;
  if (e.zp_flags & NQK_ZP_COL) v -= e.col[map_b(bm, b) * N + gn] * e.zpa;
  if (e.zp_flags & NQK_ZP_KCONST) v += e.zpa * e.zpb * e.kdim;
  const int g = (EPI == EPI_QKV) ? (int)(gn / e.group_cols) : 0;
  const float d = (float)((double)v * (double)e.s_acc[g]);
  if constexpr (EPI == EPI_SCORES) {
    float* o = (float*)e.out[0];
    o[(b * M + gm) * N + gn] = d / e.div;
  } else if constexpr (EPI == EPI_RESID) {
    float* o = (float*)e.out[0];
    const int64_t i = gm * N + gn;
    o[i] = (e.bias[gn] + d) + e.resid[i];
  } else if constexpr (EPI == EPI_GELU) {
    const float h = e.bias[gn] + d;
    const float t = h / e.div;
    const float a = ref_erf(t) + e.add1;
    const float y = (h * a) * e.mul2;
    int8_t* o = (int8_t*)e.out[0];
    o[gm * N + gn] = (int8_t)quant_zp(y, e.s_out[0], e.zp_out[0], e.lo, e.hi);
  } else if constexpr (EPI == EPI_QKV) {
    const float h = e.bias[gn] + d;
    const int q = quant_zp(h, e.s_out[g], e.zp_out[g], e.lo, e.hi);
    const int64_t nl = gn - (int64_t)g * e.group_cols;
    const int64_t img = gm / e.tokens, t = gm - img * e.tokens;
    const int64_t hh = nl / e.hdim, dd = nl - hh * e.hdim;
    int8_t* o = (int8_t*)e.out[g];
    o[((img * e.heads + hh) * e.tokens + t) * e.hdim + dd] = (int8_t)q;  // [b, h, t, d]
  } else {  // EPI_PV: batch b = img*heads + h, row = token, col = d -> ctx[img*T + t][h*D + d]
    const int q = quant_zp(d, e.s_out[0], e.zp_out[0], e.lo, e.hi);
    const int64_t img = b / e.heads, hh = b - img * e.heads;
    int8_t* o = (int8_t*)e.out[0];
    o[(img * e.tokens + gm) * (int64_t)e.ld_out + hh * e.hdim + gn] = (int8_t)q;
  }
}

template <int EPI>
__global__ void __launch_bounds__(256)
k_qgemm_epi(const int8_t* __restrict__ A, const int8_t* __restrict__ Bt, int64_t M, int64_t N, int64_t K,
            int64_t lda, int64_t ldb, BatchMap bm, int64_t a_ms, int64_t b_ms, int tiles_m, int tiles_n, Epi e) {
  __shared__ __attribute__((aligned(16))) int8_t smem[2 * (FBM + FBN) * FBK];
#define AS(buf) (smem + (buf) * (FBM + FBN) * FBK)
#define BS(buf) (smem + (buf) * (FBM + FBN) * FBK + FBM * FBK)
  const int64_t bz = blockIdx.z;
  A += map_a(bm, bz) * a_ms;
  Bt += map_b(bm, bz) * b_ms;
  // XCD-aware tile order: consecutive tiles that share an A row panel land on one XCD
  const int nwg = tiles_m * tiles_n;
  int wg = blockIdx.x;
  if (nwg >= 8) {
    const int q = nwg / 8, r = nwg % 8, x = wg % 8;
    wg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + wg / 8;
  }
  const int tm = wg / tiles_n, tn = wg % tiles_n;
  const int64_t m0 = (int64_t)tm * FBM, n0 = (int64_t)tn * FBN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  v4i ra[4], rb[4];
  auto load_tile = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * 256, row = idx >> 3, ch = idx & 7;
      const int64_t kk = k0 + ch * 16;
      const int64_t gm = m0 + row, gn = n0 + row;
      const v4i z = {0, 0, 0, 0};
      ra[i] = (gm < M && kk < K) ? *reinterpret_cast<const v4i*>(A + gm * lda + kk) : z;
      rb[i] = (gn < N && kk < K) ? *reinterpret_cast<const v4i*>(Bt + gn * ldb + kk) : z;
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * 256, row = idx >> 3, ch = idx & 7;
      *reinterpret_cast<v4i*>(AS(buf) + swz128(row, ch)) = ra[i];
      *reinterpret_cast<v4i*>(BS(buf) + swz128(row, ch)) = rb[i];
    }
  };

  v16i acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;

  const int nk = (int)((K + FBK - 1) / FBK);
  load_tile(0);
  store_tile(0);
  __syncthreads();
  const int r32 = lane & 31, half = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tile((int64_t)(kt + 1) * FBK);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      v4i fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        fa[i] = *reinterpret_cast<const v4i*>(AS(cur) + swz128(wm * 64 + i * 32 + r32, 2 * s + half));
#pragma unroll
      for (int j = 0; j < 2; ++j)
        fb[j] = *reinterpret_cast<const v4i*>(BS(cur) + swz128(wn * 64 + j * 32 + r32, 2 * s + half));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }
#undef AS
#undef BS
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t gn = n0 + wn * 64 + j * 32 + r32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t gm = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (gm < M && gn < N) epi_store<EPI>(e, bm, bz, gm, gn, M, N, acc[i][j][r]);
      }
    }
}

// ------------------------------------------------------------------ LayerNorm + quantize
__global__ void __launch_bounds__(64)
k_ln_quant(const float* __restrict__ x, const float* __restrict__ g, const float* __restrict__ b,
           int8_t* __restrict__ out, int64_t rows, int64_t cols, float eps, PwPlan p, float s, double zp, double lo,
           double hi) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* v = sm;
  float* part = sm + cols;
  float* leafv = part + kMaxLeaves * 8;
  const int lane = threadIdx.x;
  const float fcols = (float)cols;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const float* xr = x + r * cols;
    for (int64_t i = lane; i < cols; i += 64) v[i] = xr[i];
    __syncthreads();
    const float mean = row_pairwise_sum(v, p, part, leafv) / fcols;
    const float nmean = -mean;
    for (int64_t i = lane; i < cols; i += 64) {
      float d = v[i] + nmean;
      v[i] = d * d;
    }
    __syncthreads();
    const float var = row_pairwise_sum(v, p, part, leafv) / fcols;
    const float inv = 1.0f / __builtin_sqrtf(var + eps);
    int8_t* orow = out + r * cols;
    for (int64_t i = lane; i < cols; i += 64) {
      float d = xr[i] + nmean;
      float y = ((d * inv) * g[i]) + b[i];
      orow[i] = (int8_t)quant_zp(y, s, zp, lo, hi);
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ Softmax + quantize
// one row per 64-lane block; output row stride ldo (>= cols, pad zero-filled), row sum
__global__ void __launch_bounds__(64)
k_softmax_quant(const float* __restrict__ x, int8_t* __restrict__ out, int64_t* __restrict__ rowsum, int64_t rows,
                int64_t cols, int64_t ldo, PwPlan p, float s, double zp, double lo, double hi) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* v = sm;
  float* part = sm + cols;
  float* leafv = part + kMaxLeaves * 8;
  const int lane = threadIdx.x;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const float* xr = x + r * cols;
    float mx = -__builtin_inff();
    for (int64_t i = lane; i < cols; i += 64) {
      float t = xr[i];
      v[i] = t;
      mx = t > mx ? t : mx;
    }
    for (int off = 32; off > 0; off >>= 1) {
      float o = __shfl_xor(mx, off, 64);
      mx = o > mx ? o : mx;
    }
    const float nm = -mx;
    for (int64_t i = lane; i < cols; i += 64) v[i] = np_expf(v[i] + nm);
    __syncthreads();
    const float ssum = row_pairwise_sum(v, p, part, leafv);
    int8_t* orow = out + r * ldo;
    int64_t acc = 0;
    for (int64_t i = lane; i < ldo; i += 64) {
      int q = 0;
      if (i < cols) {
        q = quant_zp(v[i] / ssum, s, zp, lo, hi);
        acc += q;
      }
      orow[i] = (int8_t)q;
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) rowsum[r] = acc;
    __syncthreads();
  }
}

// ------------------------------------------------------------------ int8 transpose + pad
// src [nb][R][C] -> dst [nb][C][Rp] (Rp >= R, pad columns zero), rowsum[nb][C] = sum_r src
__global__ void __launch_bounds__(256)
k_transpose_pad(const int8_t* __restrict__ src, int8_t* __restrict__ dst, int64_t* __restrict__ rowsum, int64_t nb,
                int64_t R, int64_t C, int64_t Rp) {
  __shared__ int8_t tile[64][65];
  const int64_t b = blockIdx.z;
  const int r0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int8_t* s = src + b * R * C;
  for (int i = ty; i < 64; i += 4) {
    int r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < R && c < C) ? s[(int64_t)r * C + c] : (int8_t)0;
  }
  __syncthreads();
  int8_t* d = dst + b * C * Rp;
  for (int i = ty; i < 64; i += 4) {
    int c = c0 + i, r = r0 + tx;
    if (c < C && r < Rp) d[(int64_t)c * Rp + r] = tile[tx][i];
  }
  if (rowsum && blockIdx.x == 0 && ty == 0) {
    // one lane per output row c: sum over all R (reads src directly; R is small)
    int c = c0 + tx;
    if (c < C) {
      int64_t acc = 0;
      for (int64_t r = 0; r < R; ++r) acc += s[r * C + c];
      rowsum[b * C + c] = acc;
    }
  }
}

}  // namespace
}  // namespace nqk

using namespace nqk;

static Epi make_epi(const nqk_epilogue* p) {
  Epi e{};
  e.zp_flags = p->zp_flags;
  e.zpa = p->zpa;
  e.zpb = p->zpb;
  e.kdim = p->kdim;
  e.row = p->row;
  e.col = p->col;
  e.group_cols = p->group_cols > 0 ? p->group_cols : 1;
  for (int g = 0; g < 3; ++g) {
    e.s_acc[g] = p->s_acc[g];
    e.s_out[g] = p->s_out[g];
    e.zp_out[g] = (double)p->zp_out[g];
    e.out[g] = p->out[g];
  }
  e.bias = p->bias;
  e.resid = p->resid;
  e.div = p->div;
  e.add1 = p->add1;
  e.mul2 = p->mul2;
  e.tokens = p->tokens;
  e.heads = p->heads;
  e.hdim = p->hdim;
  e.ld_out = p->ld_out;
  e.lo = -__builtin_ldexp(1.0, p->bit_width - 1);
  e.hi = __builtin_ldexp(1.0, p->bit_width - 1) - 1.0;
  return e;
}

extern "C" int nqk_qgemm_fused(int epi, const int8_t* a, const int8_t* bt, int64_t batch, int64_t M, int64_t N,
                               int64_t K, int64_t lda, int64_t ldb, const int64_t* bmap, int64_t a_mat_stride,
                               int64_t b_mat_stride, const nqk_epilogue* params) {
  if (batch <= 0 || M <= 0 || N <= 0) return 0;
  if ((lda & 15) || (ldb & 15) || (K & 15)) return fail("nqk_qgemm_fused: lda, ldb and K must be multiples of 16");
  if ((((uintptr_t)a) & 15) || (((uintptr_t)bt) & 15) || (a_mat_stride & 15) || (b_mat_stride & 15))
    return fail("nqk_qgemm_fused: operands must be 16-byte aligned");
  if (batch > 65535) return fail("nqk_qgemm_fused: batch > 65535");
  if (params->bit_width < 2 || params->bit_width > 8) return fail("nqk_qgemm_fused: int8 outputs need 2 <= bw <= 8");
  const int tiles_m = (int)((M + FBM - 1) / FBM), tiles_n = (int)((N + FBN - 1) / FBN);
  const BatchMap m = batch_map(bmap);
  const Epi e = make_epi(params);
  const dim3 grid(tiles_m * tiles_n, 1, (unsigned)batch);
  switch (epi) {
#define L(E) case E: hipLaunchKernelGGL(k_qgemm_epi<E>, grid, dim3(256), 0, stream(), a, bt, M, N, K, lda, ldb, m, \
                                        a_mat_stride, b_mat_stride, tiles_m, tiles_n, e); break;
    L(EPI_QKV) L(EPI_SCORES) L(EPI_PV) L(EPI_RESID) L(EPI_GELU)
#undef L
    default: return fail("nqk_qgemm_fused: unknown epilogue");
  }
  return launch_status("nqk_qgemm_fused");
}

extern "C" int nqk_ln_quant(const float* x, const float* gamma, const float* beta, int8_t* out, int64_t rows,
                            int64_t cols, float eps, float scale, int64_t zp, int bit_width) {
  if (rows <= 0) return 0;
  PwPlan p;
  if (row_plan(cols, p)) return -1;
  const double lo = -__builtin_ldexp(1.0, bit_width - 1), hi = __builtin_ldexp(1.0, bit_width - 1) - 1.0;
  hipLaunchKernelGGL(k_ln_quant, dim3(row_grid(rows)), dim3(64), row_smem(cols), stream(), x, gamma, beta, out, rows,
                     cols, eps, p, scale, (double)zp, lo, hi);
  return launch_status("nqk_ln_quant");
}

extern "C" int nqk_softmax_quant(const float* x, int8_t* out, int64_t* rowsum, int64_t rows, int64_t cols,
                                 int64_t ldo, float scale, int64_t zp, int bit_width) {
  if (rows <= 0) return 0;
  if (ldo < cols) return fail("nqk_softmax_quant: ldo < cols");
  PwPlan p;
  if (row_plan(cols, p)) return -1;
  const double lo = -__builtin_ldexp(1.0, bit_width - 1), hi = __builtin_ldexp(1.0, bit_width - 1) - 1.0;
  hipLaunchKernelGGL(k_softmax_quant, dim3(row_grid(rows)), dim3(64), row_smem(cols), stream(), x, out, rowsum, rows,
                     cols, ldo, p, scale, (double)zp, lo, hi);
  return launch_status("nqk_softmax_quant");
}

extern "C" int nqk_transpose_pad_i8(const int8_t* src, int8_t* dst, int64_t* rowsum, int64_t nb, int64_t R,
                                    int64_t C, int64_t Rp) {
  if (nb <= 0 || R <= 0 || C <= 0) return 0;
  if (Rp < R || nb > 65535) return fail("nqk_transpose_pad_i8: bad shape");
  const dim3 grid((unsigned)((Rp + 63) / 64), (unsigned)((C + 63) / 64), (unsigned)nb);
  hipLaunchKernelGGL(k_transpose_pad, grid, dim3(256), 0, stream(), src, dst, rowsum, nb, R, C, Rp);
  return launch_status("nqk_transpose_pad_i8");
}
