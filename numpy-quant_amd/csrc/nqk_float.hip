// Float32 operators of the QModel node loop (numpy_quant/model.py:65-213,
// tensor.py:119-225) — the "else" branch of QModel.__call__ (model.py:528-538)
// runs these on dequantized inputs.  They are written to be NumPy-exact:
//   * elementwise f32 +,-,*,/ and sqrt are IEEE correctly rounded, no contraction
//     (-ffp-contract=off) — the same as NumPy's SIMD loops;
//   * exp is NumPy's AVX512F float32 algorithm (Cody-Waite reduction, 5/2 rational
//     minimax, scalef), bit-identical to np.exp on every one of the 2^32 inputs
//     (checked exhaustively on the host, tests/test_numerics.py on the GPU);
//   * sums / means over the last axis follow NumPy's pairwise summation
//     (blocks of <= 128 with 8 interleaved accumulators, recursive halving at
//     multiples of 8), so LayerNormalization and Softmax match bit for bit.
#include "nqk_common.h"
#include "nqk_numerics.h"

namespace nqk {
namespace {

template <int OP>
__device__ __forceinline__ float unary(float x) {
  if constexpr (OP == NQK_NEG) return -x;
  else if constexpr (OP == NQK_EXP) return np_expf(x);
  else if constexpr (OP == NQK_ERF) return ref_erf(x);
  else if constexpr (OP == NQK_SQRT) return __builtin_sqrtf(x);
  else if constexpr (OP == NQK_RELU) return (x > 0.0f ? 1.0f : 0.0f) * x;   // (x > 0) * x
  else if constexpr (OP == NQK_SIGMOID) return 1.0f / (np_expf(-x) + 1.0f);  // tensor.py:205-206
  else if constexpr (OP == NQK_RECIP) return 1.0f / x;
  else return tanhf(x);
}

template <int OP>
__global__ void k_unary(const float* __restrict__ x, float* __restrict__ y, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) y[i] = unary<OP>(x[i]);
}

__global__ void k_add_scalar(const float* __restrict__ x, float s, float* __restrict__ y, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) y[i] = x[i] + s;
}

struct Nd {
  int ndim, small;  // small: every index and extent < 2^31 -> 32-bit magic-number divmod
  int64_t shape[6];
  int64_t s0[6], s1[6], s2[6];
  uint32_t mag[6], ext[6];
  int sh1[6], sh2[6];
};

// n / d for 32-bit unsigned n with a precomputed magic (Granlund-Montgomery round-up)
__device__ __forceinline__ uint32_t magic_div(uint32_t n, uint32_t mag, int sh1, int sh2) {
  const uint32_t t = __umulhi(mag, n);
  return (t + ((n - t) >> sh1)) >> sh2;
}

__device__ __forceinline__ void nd_offsets(const Nd& d, int64_t i, int64_t& o0, int64_t& o1, int64_t& o2) {
  o0 = o1 = o2 = 0;
  if (d.small) {
    uint32_t u = (uint32_t)i;
    for (int k = d.ndim - 1; k >= 0; --k) {
      const uint32_t q = magic_div(u, d.mag[k], d.sh1[k], d.sh2[k]);
      const int64_t c = (int64_t)(u - q * d.ext[k]);
      u = q;
      o0 += c * d.s0[k];
      o1 += c * d.s1[k];
      o2 += c * d.s2[k];
    }
    return;
  }
  for (int k = d.ndim - 1; k >= 0; --k) {
    int64_t c = i % d.shape[k];
    i /= d.shape[k];
    o0 += c * d.s0[k];
    o1 += c * d.s1[k];
    o2 += c * d.s2[k];
  }
}

template <int OP>
__global__ void k_binary(const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ out,
                         int64_t total, Nd d) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    int64_t oa, ob, unused;
    nd_offsets(d, i, oa, ob, unused);
    float x = a[oa], y = b[ob], r;
    if constexpr (OP == NQK_ADD) r = x + y;
    else if constexpr (OP == NQK_SUB) r = x - y;
    else if constexpr (OP == NQK_MUL) r = x * y;
    else r = x / y;
    out[i] = r;
  }
}

__global__ void k_where(const int64_t* __restrict__ c, const float* __restrict__ a, const float* __restrict__ b,
                        float* __restrict__ out, int64_t total, Nd d, Nd d2) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    int64_t oc, oa, ob, u;
    nd_offsets(d, i, oc, oa, ob);
    (void)u;
    out[i] = c[oc] ? a[oa] : b[ob];
  }
}

template <typename T>
__global__ void k_copy_nd(const T* __restrict__ src, T* __restrict__ dst, int64_t total, Nd d) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    int64_t os, od, u;
    nd_offsets(d, i, os, od, u);
    dst[od] = src[os];
  }
}

__global__ void __launch_bounds__(64)
k_softmax(const float* __restrict__ x, float* __restrict__ out, int64_t rows, int64_t cols, PwPlan p) {
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
    float s = row_pairwise_sum(v, p, part, leafv);
    float* orow = out + r * cols;
    for (int64_t i = lane; i < cols; i += 64) orow[i] = v[i] / s;
    __syncthreads();
  }
}

__global__ void __launch_bounds__(64)
k_layernorm(const float* __restrict__ x, const float* __restrict__ g, const float* __restrict__ b,
            float* __restrict__ out, int64_t rows, int64_t cols, float eps, PwPlan p) {
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
    float* orow = out + r * cols;
    for (int64_t i = lane; i < cols; i += 64) {
      float d = xr[i] + nmean;
      orow[i] = ((d * inv) * g[i]) + b[i];
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(64)
k_mean_rows(const float* __restrict__ x, float* __restrict__ out, int64_t rows, int64_t cols, PwPlan p) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* v = sm;
  float* part = sm + cols;
  float* leafv = part + kMaxLeaves * 8;
  const int lane = threadIdx.x;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    for (int64_t i = lane; i < cols; i += 64) v[i] = x[r * cols + i];
    __syncthreads();
    float s = row_pairwise_sum(v, p, part, leafv);
    if (lane == 0) out[r] = s / (float)cols;
    __syncthreads();
  }
}

// ------------------------------------------------------------------ min / max (calibration)
__global__ void k_minmax_partial(const float* __restrict__ x, int64_t n, float* __restrict__ part) {
  float mn = __builtin_inff(), mx = -__builtin_inff();
  bool nan = false;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float t = x[i];
    nan |= (t != t);
    mn = t < mn ? t : mn;
    mx = t > mx ? t : mx;
  }
  for (int off = 32; off > 0; off >>= 1) {
    float a = __shfl_xor(mn, off, 64), b = __shfl_xor(mx, off, 64);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  unsigned long long anynan = __ballot(nan);
  __shared__ float smn[4], smx[4];
  __shared__ int snan[4];
  int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { smn[w] = mn; smx[w] = mx; snan[w] = anynan != 0; }
  __syncthreads();
  if (threadIdx.x == 0) {
    int nw = blockDim.x >> 6;
    bool nn = false;
    for (int i = 0; i < nw; ++i) { mn = smn[i] < mn ? smn[i] : mn; mx = smx[i] > mx ? smx[i] : mx; nn |= snan[i] != 0; }
    if (nn) { mn = __builtin_nanf(""); mx = mn; }
    part[2 * blockIdx.x] = mn;
    part[2 * blockIdx.x + 1] = mx;
  }
}

__global__ void __launch_bounds__(256) k_minmax_final(const float* __restrict__ part, int nparts, float* __restrict__ out) {
  float mn = __builtin_inff(), mx = -__builtin_inff();
  bool nan = false;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
    const float a = part[2 * i], b = part[2 * i + 1];
    nan |= (a != a) || (b != b);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  for (int off = 32; off > 0; off >>= 1) {
    const float a = __shfl_xor(mn, off, 64), b = __shfl_xor(mx, off, 64);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  const unsigned long long anynan = __ballot(nan);
  __shared__ float smn[4], smx[4];
  __shared__ int snan[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { smn[w] = mn; smx[w] = mx; snan[w] = anynan != 0; }
  __syncthreads();
  if (threadIdx.x == 0) {
    bool nn = false;
    for (int i = 0; i < 4; ++i) { mn = smn[i] < mn ? smn[i] : mn; mx = smx[i] > mx ? smx[i] : mx; nn |= snan[i] != 0; }
    if (nn) { mn = __builtin_nanf(""); mx = mn; }
    out[0] = mn;
    out[1] = mx;
  }
}

// exhaustive check: fast vs IEEE-division variants of np_expf / ref_erf on all 2^32
// bit patterns; counts[0] / counts[1] = mismatching exp / erf inputs, counts[2] / counts[3]
// = non-positive inputs where np_expf_nonpos / np_expf_nonpos2 (both lanes) differ from
// np_expf; ex[k] = an example
__global__ void k_fastmath_check(unsigned long long* counts, uint32_t* ex) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  unsigned long long ce = 0, cr = 0, cn = 0, cp = 0, cs = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (uint64_t(1) << 32); i += stride) {
    const float x = __uint_as_float((uint32_t)i);
    const float a = np_expf_t<true>(x), b = np_expf_t<false>(x);
    if (__float_as_uint(a) != __float_as_uint(b) && !(a != a && b != b)) { ++ce; ex[0] = (uint32_t)i; }
    const float c = ref_erf_t<true>(x), d = ref_erf_t<false>(x);
    if (__float_as_uint(c) != __float_as_uint(d) && !(c != c && d != d)) { ++cr; ex[1] = (uint32_t)i; }
    if (x <= 0.0f && __float_as_uint(np_expf_nonpos(x)) != __float_as_uint(b)) { ++cn; ex[2] = (uint32_t)i; }
    if (x <= 0.0f) {
      const v2f_t p = np_expf_nonpos2(v2f_t{x, x});
      if (__float_as_uint(p[0]) != __float_as_uint(b) || __float_as_uint(p[1]) != __float_as_uint(b)) {
        ++cp;
        ex[3] = (uint32_t)i;
      }
    }
    if (x <= 0.0f && x >= NP_EXP_SAFE_LO) {
      const v2f_t p = np_expf_safe2(v2f_t{x, x});
      if (__float_as_uint(p[0]) != __float_as_uint(b) || __float_as_uint(p[1]) != __float_as_uint(b)) {
        ++cs;
        ex[4] = (uint32_t)i;
      }
    }
  }
  if (ce) atomicAdd(counts, ce);
  if (cr) atomicAdd(counts + 1, cr);
  if (cn) atomicAdd(counts + 2, cn);
  if (cp) atomicAdd(counts + 3, cp);
  if (cs) atomicAdd(counts + 4, cs);
}

// exhaustive check of the GELU filter bound (nqk_numerics.h gelu_fast) for the graph
// constants div = sqrt2 (as f32), add1 = 1, mul2 = 0.5: st[0] = violations, st[1] = an
// example input; st[2 + e] = max over inputs with biased exponent e of the error in units
// of |h| * 2^-24 (diagnostic)
__global__ void k_gelu_filter_check(unsigned long long* st) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const double rdiv = 1.0 / (double)1.41421354f;
  unsigned long long bad = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (uint64_t(1) << 32); i += stride) {
    const float h = __uint_as_float((uint32_t)i);
    if (!(__builtin_fabsf(h) < 0x1p64f)) continue;  // NaN, inf and huge |h| take the exact path
    const float a = gelu_fast(h), b = gelu_ref(h, rdiv, 1.0f, 0.5f);
    const float d = __builtin_fabsf(a - b);
    const bool ok = (double)d <= (double)GELU_REL * __builtin_fabs((double)h) + (double)GELU_ABS;
    if (!ok) { ++bad; st[1] = i; }
    const int ex = (int)((i >> 23) & 0xff);
    const double units = __builtin_fabs((double)h) > 0 ? (double)d / (__builtin_fabs((double)h) * 0x1p-24) : 0.0;
    const unsigned long long u = (unsigned long long)(units < 1e18 ? units : 1e18);
    if (u) atomicMax(st + 2 + ex, u);
  }
  if (bad) atomicAdd(st, bad);
}

// drop extent-1 dimensions and merge neighbours that are contiguous for every operand
// (the output / destination index is always row-major), then precompute magic divisors
Nd make_nd(int ndim, const int64_t* shape, const int64_t* s0, const int64_t* s1, const int64_t* s2) {
  Nd d{};
  int n = 0;
  for (int k = 0; k < ndim; ++k) {
    if (shape[k] == 1) continue;
    const int64_t a0 = s0 ? s0[k] : 0, a1 = s1 ? s1[k] : 0, a2 = s2 ? s2[k] : 0;
    if (n > 0 && d.s0[n - 1] == a0 * shape[k] && d.s1[n - 1] == a1 * shape[k] && d.s2[n - 1] == a2 * shape[k]) {
      d.shape[n - 1] *= shape[k];
      d.s0[n - 1] = a0;
      d.s1[n - 1] = a1;
      d.s2[n - 1] = a2;
      continue;
    }
    d.shape[n] = shape[k];
    d.s0[n] = a0;
    d.s1[n] = a1;
    d.s2[n] = a2;
    ++n;
  }
  d.ndim = n;
  int64_t total = 1;
  for (int k = 0; k < n; ++k) total *= d.shape[k];
  d.small = total < (int64_t(1) << 31);
  for (int k = 0; k < n && d.small; ++k) {
    const uint32_t dv = (uint32_t)d.shape[k];
    int l = 0;
    while ((uint64_t(1) << l) < dv) ++l;
    d.mag[k] = (uint32_t)(((uint64_t(1) << 32) * ((uint64_t(1) << l) - dv)) / dv + 1);
    d.sh1[k] = l < 1 ? l : 1;
    d.sh2[k] = l > 1 ? l - 1 : 0;
    d.ext[k] = dv;
  }
  return d;
}

int64_t nd_total(int ndim, const int64_t* shape) {
  int64_t t = 1;
  for (int k = 0; k < ndim; ++k) t *= shape[k];
  return t;
}

}  // namespace
}  // namespace nqk

using namespace nqk;

extern "C" int nqk_binary_f32(int op, const float* a, const float* b, float* out, int ndim, const int64_t* shape,
                              const int64_t* a_strides, const int64_t* b_strides) {
  if (ndim < 0 || ndim > 6) return fail("nqk_binary_f32: ndim > 6");
  int64_t total = nd_total(ndim, shape);
  if (total <= 0) return 0;
  Nd d = make_nd(ndim, shape, a_strides, b_strides, nullptr);
  unsigned g = grid_for(total);
  switch (op) {
    case NQK_ADD: hipLaunchKernelGGL(k_binary<NQK_ADD>, dim3(g), dim3(kThreads), 0, stream(), a, b, out, total, d); break;
    case NQK_SUB: hipLaunchKernelGGL(k_binary<NQK_SUB>, dim3(g), dim3(kThreads), 0, stream(), a, b, out, total, d); break;
    case NQK_MUL: hipLaunchKernelGGL(k_binary<NQK_MUL>, dim3(g), dim3(kThreads), 0, stream(), a, b, out, total, d); break;
    case NQK_DIV: hipLaunchKernelGGL(k_binary<NQK_DIV>, dim3(g), dim3(kThreads), 0, stream(), a, b, out, total, d); break;
    default: return fail("nqk_binary_f32: bad op");
  }
  return launch_status("nqk_binary_f32");
}

extern "C" int nqk_selftest_fastmath(unsigned long long* counts_dev, uint32_t* examples_dev) {
  hipLaunchKernelGGL(k_fastmath_check, dim3(256 * 64), dim3(256), 0, stream(), counts_dev, examples_dev);
  return launch_status("nqk_selftest_fastmath");
}

extern "C" int nqk_selftest_gelu_filter(unsigned long long* stats_dev) {
  hipLaunchKernelGGL(k_gelu_filter_check, dim3(256 * 64), dim3(256), 0, stream(), stats_dev);
  return launch_status("nqk_selftest_gelu_filter");
}

extern "C" int nqk_unary_f32(int op, const float* x, float* out, int64_t n) {
  if (n <= 0) return 0;
  unsigned g = grid_for(n);
  switch (op) {
#define U(OPC) case OPC: hipLaunchKernelGGL(k_unary<OPC>, dim3(g), dim3(kThreads), 0, stream(), x, out, n); break;
    U(NQK_NEG) U(NQK_EXP) U(NQK_ERF) U(NQK_SQRT) U(NQK_RELU) U(NQK_SIGMOID) U(NQK_RECIP) U(NQK_TANH)
#undef U
    default: return fail("nqk_unary_f32: bad op");
  }
  return launch_status("nqk_unary_f32");
}

extern "C" int nqk_add_scalar_f32(const float* x, float s, float* out, int64_t n) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_add_scalar, dim3(grid_for(n)), dim3(kThreads), 0, stream(), x, s, out, n);
  return launch_status("nqk_add_scalar_f32");
}

extern "C" int nqk_softmax_lastdim(const float* x, float* out, int64_t rows, int64_t cols) {
  if (rows <= 0) return 0;
  PwPlan p;
  if (row_plan(cols, p)) return -1;
  hipLaunchKernelGGL(k_softmax, dim3(row_grid(rows)), dim3(64), row_smem(cols), stream(), x, out, rows, cols, p);
  return launch_status("nqk_softmax_lastdim");
}

extern "C" int nqk_layernorm_lastdim(const float* x, const float* gamma, const float* beta, float* out, int64_t rows,
                                     int64_t cols, float eps) {
  if (rows <= 0) return 0;
  PwPlan p;
  if (row_plan(cols, p)) return -1;
  hipLaunchKernelGGL(k_layernorm, dim3(row_grid(rows)), dim3(64), row_smem(cols), stream(), x, gamma, beta, out,
                     rows, cols, eps, p);
  return launch_status("nqk_layernorm_lastdim");
}

extern "C" int nqk_mean_lastdim(const float* x, float* out, int64_t rows, int64_t cols) {
  if (rows <= 0) return 0;
  PwPlan p;
  if (row_plan(cols, p)) return -1;
  hipLaunchKernelGGL(k_mean_rows, dim3(row_grid(rows)), dim3(64), row_smem(cols), stream(), x, out, rows, cols, p);
  return launch_status("nqk_mean_lastdim");
}

extern "C" int nqk_minmax_f32(const float* x, int64_t n, float* out2, float* scratch, int64_t scratch_len) {
  if (n <= 0) return fail("nqk_minmax_f32: empty tensor");
  int64_t parts = scratch_len / 2;
  if (parts < 1) return fail("nqk_minmax_f32: scratch too small");
  unsigned g = grid_for(n, 256, parts < 2048 ? parts : 2048);
  hipLaunchKernelGGL(k_minmax_partial, dim3(g), dim3(256), 0, stream(), x, n, scratch);
  hipLaunchKernelGGL(k_minmax_final, dim3(1), dim3(256), 0, stream(), scratch, (int)g, out2);
  return launch_status("nqk_minmax_f32");
}

extern "C" int nqk_copy_strided(const void* src, void* dst, int elem_size, int ndim, const int64_t* shape,
                                const int64_t* src_strides, const int64_t* dst_strides) {
  if (ndim < 0 || ndim > 6) return fail("nqk_copy_strided: ndim > 6");
  int64_t total = nd_total(ndim, shape);
  if (total <= 0) return 0;
  Nd d = make_nd(ndim, shape, src_strides, dst_strides, nullptr);
  unsigned g = grid_for(total);
  switch (elem_size) {
    case 1: hipLaunchKernelGGL(k_copy_nd<int8_t>, dim3(g), dim3(kThreads), 0, stream(), (const int8_t*)src, (int8_t*)dst, total, d); break;
    case 2: hipLaunchKernelGGL(k_copy_nd<int16_t>, dim3(g), dim3(kThreads), 0, stream(), (const int16_t*)src, (int16_t*)dst, total, d); break;
    case 4: hipLaunchKernelGGL(k_copy_nd<int32_t>, dim3(g), dim3(kThreads), 0, stream(), (const int32_t*)src, (int32_t*)dst, total, d); break;
    case 8: hipLaunchKernelGGL(k_copy_nd<int64_t>, dim3(g), dim3(kThreads), 0, stream(), (const int64_t*)src, (int64_t*)dst, total, d); break;
    default: return fail("nqk_copy_strided: element size must be 1, 2, 4 or 8");
  }
  return launch_status("nqk_copy_strided");
}

extern "C" int nqk_where_f32(const int64_t* cond, const float* a, const float* b, float* out, int ndim,
                             const int64_t* shape, const int64_t* c_strides, const int64_t* a_strides,
                             const int64_t* b_strides) {
  if (ndim < 0 || ndim > 6) return fail("nqk_where_f32: ndim > 6");
  int64_t total = nd_total(ndim, shape);
  if (total <= 0) return 0;
  Nd d = make_nd(ndim, shape, c_strides, a_strides, b_strides);
  hipLaunchKernelGGL(k_where, dim3(grid_for(total)), dim3(kThreads), 0, stream(), cond, a, b, out, total, d, d);
  return launch_status("nqk_where_f32");
}
