// NumPy-exact float building blocks shared by nqk_float.hip and nqk_fused.hip:
// numpy's AVX512F float32 exp, the reference's A&S erf (numpy_helper.py:95-112) and
// NumPy's pairwise summation plan (used by mean / sum / LayerNorm / Softmax).
#pragma once
#include "nqk_common.h"

namespace nqk {
namespace {

// ------------------------------------------------------------------ division
// a / b: FAST = v_rcp_f32 estimate + one residual correction (4 VALU instead of the ~10
// of the IEEE sequence).  It is NOT correctly rounded for every (a, b); it is used only
// inside np_expf_t / ref_erf_t, where nqk_selftest_fastmath proves on the GPU, over all
// 2^32 float inputs, that the fast and the IEEE variants of the two functions return
// identical bits (tests/test_gpu_kernels.py::test_fast_division_exp_erf_exhaustive).
template <bool FAST>
__device__ __forceinline__ float div_t(float a, float b) {
  if constexpr (FAST) {
    const float r = __builtin_amdgcn_rcpf(b);
    const float q = a * r;
    const float e = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(e, r, q);
  } else {
    return a / b;
  }
}

// ------------------------------------------------------------------ numpy float32 exp
template <bool FAST>
__device__ __forceinline__ float np_expf_t(float x) {
  const float xmax = 88.72283935546875f, xmin = -103.97208404541015625f;
  const bool over = x >= xmax, under = x <= xmin;
  float xx = (over || under) ? 0.0f : x;
  float q = xx * 1.442695040888963407359924681001892137f;
  q = q + 0x1.800000p+23f;
  q = q - 0x1.800000p+23f;
  float r = __builtin_fmaf(q, -6.93145752e-1f, xx);
  r = __builtin_fmaf(q, -1.42860677e-6f, r);
  r = __builtin_fmaf(q, 0.0f, r);
  float num = __builtin_fmaf(5.082762527590693718096e-04f, r, 6.757896990527504603057e-03f);
  num = __builtin_fmaf(num, r, 5.114512081637298353406e-02f);
  num = __builtin_fmaf(num, r, 2.473615434895520810817e-01f);
  num = __builtin_fmaf(num, r, 7.257664613233124478488e-01f);
  num = __builtin_fmaf(num, r, 9.999999999980870924916e-01f);
  float den = __builtin_fmaf(2.159509375685829852307e-02f, r, -2.742335390411667452936e-01f);
  den = __builtin_fmaf(den, r, 1.0f);
  float poly = div_t<FAST>(num, den);
  poly = __builtin_ldexpf(poly, (int)q);
  poly = over ? __builtin_inff() : poly;
  poly = under ? 0.0f : poly;
  return x != x ? x : poly;  // NaN passes through (selects, no branch)
}

// the fast-division variant everywhere: bit-identical on all 2^32 inputs (see div_t)
__device__ __forceinline__ float np_expf(float x) { return np_expf_t<true>(x); }

// np_expf for x <= 0 (including -inf; softmax arguments y - max): no overflow or NaN
// selects, no zeroing of the argument before the reduction (an underflowing x only
// produces a value the final select replaces by 0), and without the third Cody-Waite step
// fma(q, 0, r), which can only turn a -0 remainder into +0 and the rational function does
// not see the sign of a zero.  Equal to np_expf on all 2^31 non-positive inputs
// (nqk_selftest_fastmath, counts[2]).
__device__ __forceinline__ float np_expf_nonpos(float x) {
  const bool under = x <= -103.97208404541015625f;
  // rint by v_rndne_f32: the same integer as NumPy's magic-number add / subtract for
  // |x log2 e| < 2^22, and every larger |q| belongs to an x the final select zeroes
  const float q = __builtin_rintf(x * 1.442695040888963407359924681001892137f);
  float r = __builtin_fmaf(q, -6.93145752e-1f, x);
  r = __builtin_fmaf(q, -1.42860677e-6f, r);
  float num = __builtin_fmaf(5.082762527590693718096e-04f, r, 6.757896990527504603057e-03f);
  num = __builtin_fmaf(num, r, 5.114512081637298353406e-02f);
  num = __builtin_fmaf(num, r, 2.473615434895520810817e-01f);
  num = __builtin_fmaf(num, r, 7.257664613233124478488e-01f);
  num = __builtin_fmaf(num, r, 9.999999999980870924916e-01f);
  float den = __builtin_fmaf(2.159509375685829852307e-02f, r, -2.742335390411667452936e-01f);
  den = __builtin_fmaf(den, r, 1.0f);
  const float poly = __builtin_ldexpf(div_t<true>(num, den), (int)q);
  return under ? 0.0f : poly;
}

// np_expf_nonpos on two values with packed f32 arithmetic (v_pk_fma / v_pk_mul: per lane
// the same IEEE operations as the scalar code) for the softmax of the fused attention.
// Instead of the underflow select, x is clamped to -128 first: NumPy's underflow region
// x <= -103.97... has q <= -150 and, at q = -150, a remainder r <= 0 (so |poly| <= 1 and
// poly 2^-150 rounds to 0), and every q <= -151 scales |poly| <= 2^0.5 below half the
// smallest subnormal; the clamp also keeps -inf (padded score columns) out of the
// reduction.  Equal to np_expf on all 2^31 non-positive inputs (nqk_selftest_fastmath,
// counts[3]).
typedef float v2f_t __attribute__((ext_vector_type(2)));
// element-pair arithmetic, packed (v_pk_*) or as two scalar instructions (PK = false: the same
// IEEE operation per element; without the SLP vectorizer the pair stays unpacked)
template <bool PK>
__device__ __forceinline__ v2f_t vmul2(v2f_t a, v2f_t b) {
  if constexpr (PK) return a * b;
  else return v2f_t{a[0] * b[0], a[1] * b[1]};
}
template <bool PK>
__device__ __forceinline__ v2f_t vadd2(v2f_t a, v2f_t b) {
  if constexpr (PK) return a + b;
  else return v2f_t{a[0] + b[0], a[1] + b[1]};
}
template <bool PK>
__device__ __forceinline__ v2f_t vsub2(v2f_t a, v2f_t b) {
  if constexpr (PK) return a - b;
  else return v2f_t{a[0] - b[0], a[1] - b[1]};
}
template <bool PK>
__device__ __forceinline__ v2f_t vfma2(v2f_t a, v2f_t b, v2f_t c) {
  if constexpr (PK) return __builtin_elementwise_fma(a, b, c);
  else return v2f_t{__builtin_fmaf(a[0], b[0], c[0]), __builtin_fmaf(a[1], b[1], c[1])};
}
__device__ __forceinline__ v2f_t np_expf_nonpos2(v2f_t x) {
  const v2f_t xc = v2f_t{__builtin_fmaxf(x[0], -128.0f), __builtin_fmaxf(x[1], -128.0f)};
  const float l2e = 1.442695040888963407359924681001892137f;
  const v2f_t t = xc * v2f_t{l2e, l2e};
  const v2f_t q = v2f_t{__builtin_rintf(t[0]), __builtin_rintf(t[1])};
  v2f_t r = __builtin_elementwise_fma(q, v2f_t{-6.93145752e-1f, -6.93145752e-1f}, xc);
  r = __builtin_elementwise_fma(q, v2f_t{-1.42860677e-6f, -1.42860677e-6f}, r);
  auto c2 = [](float c) { return v2f_t{c, c}; };
  v2f_t num = __builtin_elementwise_fma(c2(5.082762527590693718096e-04f), r, c2(6.757896990527504603057e-03f));
  num = __builtin_elementwise_fma(num, r, c2(5.114512081637298353406e-02f));
  num = __builtin_elementwise_fma(num, r, c2(2.473615434895520810817e-01f));
  num = __builtin_elementwise_fma(num, r, c2(7.257664613233124478488e-01f));
  num = __builtin_elementwise_fma(num, r, c2(9.999999999980870924916e-01f));
  v2f_t den = __builtin_elementwise_fma(c2(2.159509375685829852307e-02f), r, c2(-2.742335390411667452936e-01f));
  den = __builtin_elementwise_fma(den, r, c2(1.0f));
  // div_t<true> on both lanes
  const v2f_t rc = v2f_t{__builtin_amdgcn_rcpf(den[0]), __builtin_amdgcn_rcpf(den[1])};
  const v2f_t qq = num * rc;
  const v2f_t e = __builtin_elementwise_fma(-den, qq, num);
  const v2f_t res = __builtin_elementwise_fma(e, rc, qq);
  return v2f_t{__builtin_ldexpf(res[0], (int)q[0]), __builtin_ldexpf(res[1], (int)q[1])};
}

// np_expf_nonpos2 for x in [NP_EXP_SAFE_LO, 0] (the softmax rows whose smallest argument
// is there: a wave-uniform test in the attention kernel): q = RN(RN(x log2 e) + 1.5 2^23) -
// 1.5 2^23 is NumPy's own magic-number rounding (the same integer as v_rndne here), q >= -125
// keeps poly 2^q normal, so the scaling is an integer add of q << 23 to poly's bits — and
// q << 23 is the rounded sum's bit pattern shifted left by 23 (1.5 2^23's low 9 bits are
// zero).  No clamp, no v_cvt / v_ldexp.  Equal to np_expf on every float of the domain
// (nqk_selftest_fastmath, counts[4]).
constexpr float NP_EXP_SAFE_LO = -86.5f;
template <bool PK = true>
__device__ __forceinline__ v2f_t np_expf_safe2(v2f_t x) {
  const float l2e = 1.442695040888963407359924681001892137f;
  const v2f_t mg = v2f_t{0x1.8p23f, 0x1.8p23f};
  const v2f_t s = vadd2<PK>(vmul2<PK>(x, v2f_t{l2e, l2e}), mg);
  const v2f_t q = vsub2<PK>(s, mg);
  v2f_t r = vfma2<PK>(q, v2f_t{-6.93145752e-1f, -6.93145752e-1f}, x);
  r = vfma2<PK>(q, v2f_t{-1.42860677e-6f, -1.42860677e-6f}, r);
  auto c2 = [](float c) { return v2f_t{c, c}; };
  v2f_t num = vfma2<PK>(c2(5.082762527590693718096e-04f), r, c2(6.757896990527504603057e-03f));
  num = vfma2<PK>(num, r, c2(5.114512081637298353406e-02f));
  num = vfma2<PK>(num, r, c2(2.473615434895520810817e-01f));
  num = vfma2<PK>(num, r, c2(7.257664613233124478488e-01f));
  num = vfma2<PK>(num, r, c2(9.999999999980870924916e-01f));
  v2f_t den = vfma2<PK>(c2(2.159509375685829852307e-02f), r, c2(-2.742335390411667452936e-01f));
  den = vfma2<PK>(den, r, c2(1.0f));
  const v2f_t rc = v2f_t{__builtin_amdgcn_rcpf(den[0]), __builtin_amdgcn_rcpf(den[1])};
  const v2f_t qq = vmul2<PK>(num, rc);
  const v2f_t e = vfma2<PK>(-den, qq, num);
  const v2f_t res = vfma2<PK>(e, rc, qq);
  return v2f_t{__uint_as_float(__float_as_uint(res[0]) + (__float_as_uint(s[0]) << 23)),
               __uint_as_float(__float_as_uint(res[1]) + (__float_as_uint(s[1]) << 23))};
}

// Round-and-pack of an element pair on the fast path.  c = clamp(x, lo - zp, hi - zp) (med3;
// clamping before rounding is the same as after for integer bounds), s = RN(c + MAGIC) with
// MAGIC = 1.5 2^23 + zp: s lies in [2^23, 2^24) where the f32 spacing is 1, so s = rint(c) +
// MAGIC exactly and the low mantissa byte of s is the two's complement byte of rint(c) + zp.
// (At an exact tie an odd zp flips the even choice, but then |dd| = 0.5 fails every filter
// limit and the element takes the exact chain.)
// dd = c - (s - MAGIC) is the filter's distance to the rounded value (exact).  Replaces
// v_rndne + add zp + med3 + v_cvt_pk_u8 + xor 0x80 per element (nqk_fused.hip
// quant_filter); used by the GELU GEMM and the attention epilogues.
template <bool PK = true>
__device__ __forceinline__ v2f_t round_magic2(v2f_t x, float qlo, float qhi, float magic, v2f_t& dd) {
  const v2f_t c = v2f_t{__builtin_amdgcn_fmed3f(x[0], qlo, qhi), __builtin_amdgcn_fmed3f(x[1], qlo, qhi)};
  const v2f_t s = vadd2<PK>(c, v2f_t{magic, magic});
  dd = vsub2<PK>(c, vsub2<PK>(s, v2f_t{magic, magic}));
  return s;
}
// the low bytes of four rounded values (round_magic2) as one dword
__device__ __forceinline__ uint32_t pack4_low(v2f_t s01, v2f_t s23) {
  const uint32_t x = __builtin_amdgcn_perm(__float_as_uint(s01[1]), __float_as_uint(s01[0]), 0x0c0c0400u);
  const uint32_t y = __builtin_amdgcn_perm(__float_as_uint(s23[1]), __float_as_uint(s23[0]), 0x04000c0cu);
  return x | y;
}

// numpy_helper.py:95-112 (A&S 7.1.26), float32 throughout
template <bool FAST>
__device__ __forceinline__ float ref_erf_t(float x) {
  float sgn = (x > 0.0f) ? 1.0f : ((x < 0.0f) ? -1.0f : (x == 0.0f ? 0.0f : x));
  float ax = __builtin_fabsf(x);
  const float den = 1.0f + 0.3275911f * ax;
  // FAST: 1 / inf must stay 0 (the residual step would make it NaN)
  float t = FAST ? (den == __builtin_inff() ? 0.0f : div_t<true>(1.0f, den)) : 1.0f / den;
  float p = 1.061405429f * t + -1.453152027f;
  p = p * t;
  p = p + 1.421413741f;
  p = p * t + -0.284496736f;
  p = p * t + 0.254829592f;
  float y = 1.0f - p * t * np_expf_t<FAST>(-ax * ax);
  return sgn * y;
}
__device__ __forceinline__ float ref_erf(float x) { return ref_erf_t<true>(x); }

// ------------------------------------------------------------------ GELU filter
// The FFN chain of the ViT graphs, h -> (h * (erf(h / sqrt2) + 1)) * 0.5 (model.py Div,
// Erf, Add, Mul, Mul on f32; numpy_helper.py:95-112 erf), as the fused kernels run it:
__device__ __forceinline__ float gelu_ref(float h, double rdiv, float add1, float mul2) {
  const float a = ref_erf((float)((double)h * rdiv)) + add1;
  return (h * a) * mul2;
}
// and a cheap approximation of it (hardware rcp / exp2).  nqk_selftest_gelu_filter
// checks on the GPU, for every one of the 2^32 f32 inputs with |h| < 2^64, that
// |gelu_fast(h) - gelu_ref(h)| <= GELU_REL * |h| + GELU_ABS; the GEMM epilogue only
// trusts gelu_fast where that bound cannot move the quantized value (nqk_fused.hip).
// (measured worst case: 7 |h| 2^-24 at exponents -10..-3, tests/test_gpu_kernels.py)
constexpr float GELU_REL = 0x1p-21f, GELU_ABS = 0x1p-60f;
// With A&S 7.1.26 erf(x) = 1 - P(t) t e^{-x^2}, t = 1 / (1 + p|x|), x = h / sqrt2, the
// GELU h (1 + erf(x)) / 2 is max(h, 0) - |h| q with q = P(t) t e^{-h^2/2} / 2 (the 1/2
// and 1/sqrt2 folded into the constants): 11 VALU + v_rcp + v_exp.
__device__ __forceinline__ float gelu_fast(float h) {
  const float ah = __builtin_fabsf(h);
  const float t = __builtin_amdgcn_rcpf(__builtin_fmaf(0.3275911f * 0.70710677f, ah, 1.0f));
  float p = __builtin_fmaf(0.5f * 1.061405429f, t, 0.5f * -1.453152027f);
  p = __builtin_fmaf(p, t, 0.5f * 1.421413741f);
  p = __builtin_fmaf(p, t, 0.5f * -0.284496736f);
  p = __builtin_fmaf(p, t, 0.5f * 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(h * (h * -0.72134752f));  // e^{-h^2/2}
  const float q = (p * t) * e;
  return __builtin_fmaf(-ah, q, __builtin_fmaxf(h, 0.0f));  // one rounding for max(h, 0) - |h| q
}

// ------------------------------------------------------------------ NumPy pairwise sum
// The recursion of NumPy's pairwise_sum (n < 8: sequential; n <= 128: 8 interleaved
// accumulators combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) then the n % 8 tail;
// else split at n/2 rounded down to a multiple of 8) depends only on n, so the host
// flattens it into leaves + a post-order combine program shared by every row.
constexpr int kMaxLeaves = 64;
struct PwPlan {
  int nleaf, nops, balanced;  // balanced: nleaf = 2^k and a complete binary combine tree
  int start[kMaxLeaves], len[kMaxLeaves];
  signed char ops[2 * kMaxLeaves];  // >= 0: push leaf; -1: pop b, pop a, push a + b
};

static int build_plan(int64_t n, int64_t s, PwPlan& p) {
  if (n <= 128) {
    if (p.nleaf >= kMaxLeaves) return -1;
    p.start[p.nleaf] = (int)s;
    p.len[p.nleaf] = (int)n;
    p.ops[p.nops++] = (signed char)p.nleaf++;
    return 0;
  }
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  if (build_plan(n2, s, p) || build_plan(n - n2, s + n2, p)) return -1;
  p.ops[p.nops++] = -1;
  return 0;
}

// one 64-lane block per row; `v` is the row in LDS, scratch holds 8 partials per leaf
__device__ float row_pairwise_sum(const float* v, const PwPlan& p, float* part, float* leafv) {
  const int lane = threadIdx.x;
  for (int c = lane; c < p.nleaf * 8; c += 64) {
    int l = c >> 3, j = c & 7;
    int L = p.len[l], s = p.start[l];
    float r = 0.0f;
    if (L >= 8) {
      r = v[s + j];
      int end = L - (L % 8);
      for (int i = 8 + j; i < end; i += 8) r = r + v[s + i];
    }
    part[c] = r;
  }
  __syncthreads();
  for (int l = lane; l < p.nleaf; l += 64) {
    int L = p.len[l], s = p.start[l];
    float res;
    if (L < 8) {
      res = 0.0f;
      for (int i = 0; i < L; ++i) res = res + v[s + i];
    } else {
      const float* r = part + l * 8;
      res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
      for (int i = L - (L % 8); i < L; ++i) res = res + v[s + i];
    }
    leafv[l] = res;
  }
  __syncthreads();
  float* total = leafv + kMaxLeaves;
  if (lane == 0) {
    float st[16];
    int sp = 0;
    for (int o = 0; o < p.nops; ++o) {
      int op = p.ops[o];
      if (op >= 0) st[sp++] = leafv[op];
      else { float b = st[--sp]; float a = st[--sp]; st[sp++] = a + b; }
    }
    *total = st[0];
  }
  __syncthreads();
  float t = *total;
  __syncthreads();
  return t;
}

// wave-local LDS visibility: this wave's LDS writes are complete and ordered before
// its later LDS reads (all lanes of a wave execute in lock step)
__device__ __forceinline__ void wave_lds_sync() {
  __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// NumPy pairwise sum of v[0..n) by ONE wave (any number of waves per block, each
// with its own v / part / leafv regions; no block barrier).  part: 8*kMaxLeaves,
// leafv: kMaxLeaves + 4 floats.
__device__ float wave_pairwise_sum(const float* v, const PwPlan& p, float* part, float* leafv) {
  const int lane = threadIdx.x & 63;
  for (int c = lane; c < p.nleaf * 8; c += 64) {
    const int l = c >> 3, j = c & 7;
    const int L = p.len[l], s = p.start[l];
    float r = 0.0f;
    if (L >= 8) {
      r = v[s + j];
      const int end = L - (L % 8);
      for (int i = 8 + j; i < end; i += 8) r = r + v[s + i];
    }
    part[c] = r;
  }
  wave_lds_sync();
  for (int l = lane; l < p.nleaf; l += 64) {
    const int L = p.len[l], s = p.start[l];
    float res;
    if (L < 8) {
      res = 0.0f;
      for (int i = 0; i < L; ++i) res = res + v[s + i];
    } else {
      const float* r = part + l * 8;
      res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
      for (int i = L - (L % 8); i < L; ++i) res = res + v[s + i];
    }
    leafv[l] = res;
  }
  wave_lds_sync();
  if (p.balanced) {
    for (int cnt = p.nleaf; cnt > 1; cnt >>= 1) {
      const int h = cnt >> 1;
      float val = 0.0f;
      if (lane < h) val = leafv[2 * lane] + leafv[2 * lane + 1];
      wave_lds_sync();
      if (lane < h) leafv[lane] = val;
      wave_lds_sync();
    }
  } else if (lane == 0) {
    float* st = part;  // the partials are consumed: reuse as the combine stack
    int sp = 0;
    for (int o = 0; o < p.nops; ++o) {
      const int op = p.ops[o];
      if (op >= 0) st[sp++] = leafv[op];
      else { const float b = st[--sp]; const float a = st[--sp]; st[sp++] = a + b; }
    }
    leafv[0] = st[0];
  }
  wave_lds_sync();
  const float t = leafv[0];
  wave_lds_sync();
  return t;
}

int row_plan(int64_t cols, PwPlan& p) {
  p.nleaf = 0;
  p.nops = 0;
  p.balanced = 0;
  if (cols <= 0 || build_plan(cols, 0, p)) return fail("row length not supported by the pairwise-sum plan (max 8192)");
  // balanced iff the post-order equals that of a complete tree over nleaf = 2^k leaves
  if ((p.nleaf & (p.nleaf - 1)) == 0) {
    signed char ref[2 * kMaxLeaves];
    int n = 0, leaf = 0;
    struct R { static void go(int cnt, signed char* ref, int& n, int& leaf) {
      if (cnt == 1) { ref[n++] = (signed char)leaf++; return; }
      go(cnt / 2, ref, n, leaf); go(cnt / 2, ref, n, leaf); ref[n++] = -1; } };
    R::go(p.nleaf, ref, n, leaf);
    p.balanced = (n == p.nops);
    for (int k = 0; k < n && p.balanced; ++k) p.balanced = (ref[k] == p.ops[k]);
  }
  return 0;
}


static size_t row_smem(int64_t cols) { return (size_t)(cols + kMaxLeaves * 8 + kMaxLeaves + 4) * sizeof(float); }
static unsigned row_grid(int64_t rows) { return (unsigned)(rows < 65536 * 4 ? rows : 65536 * 4); }

}  // namespace
}  // namespace nqk
