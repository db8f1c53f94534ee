// Quantize / dequantize / requantize / row sums — the elementwise half of the hot
// path (numpy_quant/numpy_quantization.py:24-72, tensor.py:189-199, 255-259).
//
// Every kernel reproduces NumPy 2.2's arithmetic bit for bit:
//   * f32 division is IEEE correctly rounded (hipcc default; built -ffp-contract=off),
//   * zero-point additions are done in f64 (NEP 50: int64 array + f32 -> f64),
//   * rint is round-half-even (v_rndne_f32 / v_rndne_f64),
//   * float -> int64 conversion of NaN or out-of-range values gives INT64_MIN,
//     which is what x86 `cvttsd2si` (NumPy's astype) produces.
// HBM-bound: 4 B in + 1 B out per element for quantize (int8), 1 B + 4 B for
// dequantize; vectorised 16-B loads on the contiguous paths.
#include "nqk_common.h"

namespace nqk {
namespace {

__device__ __forceinline__ int64_t f64_to_i64(double u) {
  // NaN / +-inf / |u| >= 2^63 -> INT64_MIN (x86 integer-indefinite), else exact.
  if (!(u > -9223372036854775808.0 && u < 9223372036854775808.0)) {
    if (u == -9223372036854775808.0) return INT64_MIN;
    return INT64_MIN;
  }
  return (int64_t)u;
}

template <typename T>
__device__ __forceinline__ T narrow(int64_t v) { return (T)v; }

struct QuantP {
  float scale;
  double zp;     // f64(zero point)
  int has_zp;
  double lo, hi; // Python-float bounds (f64 exact for bw <= 53)
  float flo, fhi;
};

__device__ __forceinline__ int64_t quant1(float x, const QuantP& p) {
  float t = x / p.scale;  // correctly rounded
  if (p.has_zp) {
    double u = p.zp + (double)t;
    if (u != u) return INT64_MIN;
    u = u < p.lo ? p.lo : u;
    u = u > p.hi ? p.hi : u;
    return f64_to_i64(__builtin_rint(u));
  }
  if (t != t) return INT64_MIN;
  t = t < p.flo ? p.flo : t;
  t = t > p.fhi ? p.fhi : t;
  return f64_to_i64((double)__builtin_rintf(t));
}

template <typename T>
__global__ void k_quantize_flat(const float* __restrict__ x, T* __restrict__ q, int64_t n, QuantP p) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 3 < n && (((uintptr_t)(x + i)) & 15) == 0) {
      float4 v = *reinterpret_cast<const float4*>(x + i);
      q[i] = narrow<T>(quant1(v.x, p));
      q[i + 1] = narrow<T>(quant1(v.y, p));
      q[i + 2] = narrow<T>(quant1(v.z, p));
      q[i + 3] = narrow<T>(quant1(v.w, p));
    } else {
      for (int64_t j = i; j < n && j < i + 4; ++j) q[j] = narrow<T>(quant1(x[j], p));
    }
  }
}

// one wave per row: quantize and accumulate the row sum of the quantized values
template <typename T>
__global__ void k_quantize_rows(const float* __restrict__ x, T* __restrict__ q, int64_t rows,
                                int64_t len, QuantP p, int64_t* __restrict__ rowsum) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = wave; r < rows; r += nwaves) {
    const float* xr = x + r * len;
    T* qr = q + r * len;
    int64_t s = 0;
    for (int64_t j = lane; j < len; j += 64) {
      int64_t v = quant1(xr[j], p);
      qr[j] = narrow<T>(v);
      s += v;
    }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) rowsum[r] = s;
  }
}

struct ZpT {
  int flags;
  int64_t zp, zpa, zpb, K, M, N;
  const int64_t* row;
  const int64_t* col;
  BatchMap bm;
};

__device__ __forceinline__ int64_t zp_term(const ZpT& z, int64_t b, int64_t m, int64_t n) {
  int64_t t = 0;
  if (z.flags & NQK_ZP_FULL) t += z.row[(b * z.M + m) * z.N + n];
  if (z.flags & NQK_ZP_SCALAR) t += z.zp;
  if (z.flags & NQK_ZP_ROW) t += z.row[map_a(z.bm, b) * z.M + m] * z.zpb;
  if (z.flags & NQK_ZP_COL) t += z.col[map_b(z.bm, b) * z.N + n] * z.zpa;
  if (z.flags & NQK_ZP_KCONST) t -= z.zpa * z.zpb * z.K;
  return t;
}

template <typename T>
__global__ void k_dequantize(const T* __restrict__ q, float* __restrict__ out, int64_t total, ZpT z,
                             double scale) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t MN = z.M * z.N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    int64_t v = (int64_t)q[i];
    if (z.flags) {
      int64_t b = i / MN, r = i - b * MN, m = r / z.N, n = r - m * z.N;
      v -= zp_term(z, b, m, n);
    }
    out[i] = (float)((double)v * scale);
  }
}

template <typename TA, typename TB, typename TO>
__global__ void k_requantize(const TA* __restrict__ acc, const TB* __restrict__ bias, TO* __restrict__ out,
                             int64_t total, ZpT z, double scale, float res_scale, double rz, int has_rz,
                             double lo, double hi, float flo, float fhi) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t MN = z.M * z.N;
  const float r = 1.0f / res_scale;  // Python `1 / res_scale` on a float32 scalar
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    int64_t b = i / MN, rem = i - b * MN, m = rem / z.N, n = rem - m * z.N;
    int64_t v = (int64_t)acc[i];
    if (bias) v += (int64_t)bias[n];
    if (z.flags) v -= zp_term(z, b, m, n);
    float d = (float)((double)v * scale);
    float vv = r * d;
    int64_t o;
    if (has_rz) {
      double u = __builtin_rint(rz + (double)vv);
      if (u != u) o = INT64_MIN;
      else { u = u < lo ? lo : u; u = u > hi ? hi : u; o = f64_to_i64(u); }
    } else {
      float u = __builtin_rintf(vv);
      if (u != u) o = INT64_MIN;
      else { u = u < flo ? flo : u; u = u > fhi ? fhi : u; o = f64_to_i64((double)u); }
    }
    out[i] = (TO)o;
  }
}

template <typename T>
__global__ void k_rowsum(const T* __restrict__ a, int64_t* __restrict__ out, int64_t batch, int64_t rows,
                         int64_t k, int64_t ld, int64_t bstride) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = wave; r < batch * rows; r += nwaves) {
    int64_t b = r / rows, m = r - b * rows;
    const T* ar = a + b * bstride + m * ld;
    int64_t s = 0;
    for (int64_t j = lane; j < k; j += 64) s += (int64_t)ar[j];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) out[r] = s;
  }
}

// QTensor.relu (tensor.py:212-215): q < zp -> zp, elementwise, any storage in / out
template <typename TI, typename TO>
__global__ void k_relu_q(const TI* __restrict__ q, TO* __restrict__ out, int64_t n, int64_t zp) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t v = (int64_t)q[i];
    out[i] = (TO)(v < zp ? zp : v);
  }
}

QuantP make_qp(float scale, int64_t zp, int has_zp, int bw) {
  QuantP p;
  p.scale = scale;
  p.zp = (double)zp;
  p.has_zp = has_zp;
  p.lo = -__builtin_ldexp(1.0, bw - 1);
  p.hi = __builtin_ldexp(1.0, bw - 1) - 1.0;
  p.flo = (float)p.lo;
  p.fhi = (float)p.hi;
  return p;
}

ZpT make_zp(int flags, int64_t zp, int64_t zpa, int64_t zpb, int64_t K, int64_t M, int64_t N,
            const int64_t* row, const int64_t* col, const int64_t* bmap) {
  ZpT z;
  z.flags = flags; z.zp = zp; z.zpa = zpa; z.zpb = zpb; z.K = K; z.M = M; z.N = N;
  z.row = row; z.col = col; z.bm = batch_map(bmap);
  return z;
}

}  // namespace
}  // namespace nqk

using namespace nqk;

extern "C" int nqk_quantize(const float* x, void* q, int q_dtype, int64_t n, float scale, int64_t zp,
                            int has_zp, int bit_width, int64_t* rowsum, int64_t row_len) {
  if (n <= 0) return 0;
  if (bit_width < 1 || bit_width > 64) return fail("bit_width out of range");
  QuantP p = make_qp(scale, zp, has_zp, bit_width);
  if (rowsum) {
    if (row_len <= 0 || n % row_len) return fail("quantize: n not a multiple of row_len");
    int64_t rows = n / row_len;
    unsigned g = grid_for(rows * 64);
    NQK_INT_DISPATCH(q_dtype, T, hipLaunchKernelGGL(k_quantize_rows<T>, dim3(g), dim3(kThreads), 0, stream(),
                                                      x, (T*)q, rows, row_len, p, rowsum));
  } else {
    unsigned g = grid_for((n + 3) / 4);
    NQK_INT_DISPATCH(q_dtype, T, hipLaunchKernelGGL(k_quantize_flat<T>, dim3(g), dim3(kThreads), 0, stream(),
                                                      x, (T*)q, n, p));
  }
  return launch_status("nqk_quantize");
}

extern "C" int nqk_dequantize(const void* q, int q_dtype, float* out, int64_t batch, int64_t M, int64_t N,
                              float scale, int zp_flags, int64_t zp, int64_t zpa, int64_t zpb, int64_t K,
                              const int64_t* row, const int64_t* col, const int64_t* bmap) {
  int64_t total = batch * M * N;
  if (total <= 0) return 0;
  ZpT z = make_zp(zp_flags, zp, zpa, zpb, K, M, N, row, col, bmap);
  unsigned g = grid_for(total);
  NQK_INT_DISPATCH(q_dtype, T, hipLaunchKernelGGL(k_dequantize<T>, dim3(g), dim3(kThreads), 0, stream(),
                                                    (const T*)q, out, total, z, (double)scale));
  return launch_status("nqk_dequantize");
}

extern "C" int nqk_requantize(const void* acc, int acc_dtype, const void* bias, int bias_dtype, void* out,
                              int out_dtype, int64_t batch, int64_t M, int64_t N, float scale, int zp_flags,
                              int64_t zp, int64_t zpa, int64_t zpb, int64_t K, const int64_t* row,
                              const int64_t* col, const int64_t* bmap, float res_scale, int64_t res_zp,
                              int has_res_zp, int bit_width) {
  int64_t total = batch * M * N;
  if (total <= 0) return 0;
  if (bit_width < 1 || bit_width > 64) return fail("bit_width out of range");
  ZpT z = make_zp(zp_flags, zp, zpa, zpb, K, M, N, row, col, bmap);
  QuantP p = make_qp(1.0f, 0, 0, bit_width);
  unsigned g = grid_for(total);
  if (!bias) bias_dtype = NQK_I64;
  NQK_INT_DISPATCH(acc_dtype, TA,
    NQK_INT_DISPATCH(bias_dtype, TB,
      NQK_INT_DISPATCH(out_dtype, TO,
        hipLaunchKernelGGL((k_requantize<TA, TB, TO>), dim3(g), dim3(kThreads), 0, stream(),
                           (const TA*)acc, (const TB*)bias, (TO*)out, total, z, (double)scale, res_scale,
                           (double)res_zp, has_res_zp, p.lo, p.hi, p.flo, p.fhi))));
  return launch_status("nqk_requantize");
}

extern "C" int nqk_rowsum(const void* a, int dtype, int64_t* out, int64_t batch, int64_t rows, int64_t k,
                          int64_t ld, int64_t batch_stride) {
  if (batch * rows <= 0) return 0;
  unsigned g = grid_for(batch * rows * 64);
  NQK_INT_DISPATCH(dtype, T, hipLaunchKernelGGL(k_rowsum<T>, dim3(g), dim3(kThreads), 0, stream(),
                                                  (const T*)a, out, batch, rows, k, ld, batch_stride));
  return launch_status("nqk_rowsum");
}

extern "C" int nqk_relu_q(const void* q, int q_dtype, void* out, int out_dtype, int64_t n, int64_t zp) {
  if (n <= 0) return 0;
  unsigned g = grid_for(n);
  NQK_INT_DISPATCH(q_dtype, TI,
    NQK_INT_DISPATCH(out_dtype, TO,
      hipLaunchKernelGGL((k_relu_q<TI, TO>), dim3(g), dim3(kThreads), 0, stream(), (const TI*)q, (TO*)out, n, zp)));
  return launch_status("nqk_relu_q");
}
