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
#include <type_traits>

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

// RN32(x / c) from the f64 reciprocal rc = RN64(1/c): bit-identical to the IEEE f32
// division.  The quotient of two normal floats lies at least 2^-49 (relative) away
// from every float32 rounding midpoint, while RN64(x * rc) is within 2^-52 of x/c, so
// both round to the same float.  Results near the subnormal range take the division.
__device__ __forceinline__ float div_rc(float x, float c, double rc) {
  const float t = (float)((double)x * rc);
  return __builtin_fabsf(t) < 0x1p-125f ? x / c : t;
}

// quantize one f32 value with (s, zp) like numpy_quantization.py:24-34 (zp given);
// rs = RN64(1/s)
__device__ __forceinline__ int quant_zp(float x, float s, double rs, double zp, double lo, double hi) {
  const float t = div_rc(x, s, rs);
  const double u = zp + (double)t;
  if (u != u) return (int)lo;  // unreachable for finite calibrated scales
  return (int)__builtin_rint(qclip(u, lo, hi));
}

// LayerNorm output quantize (numpy_quantization.py:24-34): t = RN32(RN64(y rs)) exactly as the
// reference's f64 product, then q = rint(clip(zp + t, lo, hi)) by the magic number instead of
// f64 arithmetic (round 5): c = med3(t, lo - zp, hi - zp) clamps in t's space (integer bounds:
// the same as clamping zp + t), and RN32(c + 1.5 2^23 + zp) lies in [2^23, 2^24), where the f32
// spacing is 1, so it is rint(c + zp) with ties to even (1.5 2^23 is even) — the low byte of its
// bits is the output byte.  Exact for |zp| <= 2^20 and bit widths <= 8 (host-checked, LNQ);
// 3 f32 + 2 f64-rate instructions per element instead of 9 mostly f64-rate ones.
struct LnQ {
  float qlo, qhi, magic;
};
template <bool PK = false>
__device__ __forceinline__ uint32_t ln_quant4(const float (&y)[4], double rs, const LnQ& m) {
  float sv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) sv[k] = __builtin_amdgcn_fmed3f((float)((double)y[k] * rs), m.qlo, m.qhi);
  if constexpr (PK) {  // the magic-number adds as two packed pairs
    const v2f_t s01 = v2f_t{sv[0], sv[1]} + v2f_t{m.magic, m.magic}, s23 = v2f_t{sv[2], sv[3]} + v2f_t{m.magic, m.magic};
    sv[0] = s01[0], sv[1] = s01[1], sv[2] = s23[0], sv[3] = s23[1];
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) sv[k] = sv[k] + m.magic;
  }
  const uint32_t x01 = __builtin_amdgcn_perm(__float_as_uint(sv[1]), __float_as_uint(sv[0]), 0x0c0c0400u);
  const uint32_t x23 = __builtin_amdgcn_perm(__float_as_uint(sv[3]), __float_as_uint(sv[2]), 0x04000c0cu);
  return x01 | x23;
}

struct Epi {
  // zero-point term (see nqk.h): zpt = rowsumA[m]*zpb + rowsumBt[n]*zpa - zpa*zpb*K; the
  // row sums of A and of Bt are accumulated inside the kernel from the staged tiles
  int zp_flags;
  int64_t zpa, zpb, kdim;
  const int64_t* colsum; // precomputed column sums of B (constant weights), or null
  int group_cols;        // columns per output group (EPI_QKV), else >= N
  float s_acc[3];        // dequant scale per group
  const float* bias;     // dequantized bias [N] or null
  float s_out[3];        // quantize scale per group
  double rs_out[3];      // RN64(1 / s_out)
  double zp_out[3];      // quantize zero point per group
  void* out[3];          // outputs per group
  const float* resid;    // residual [M][N]
  float div;             // EPI_SCORES divisor; EPI_GELU sqrt(2) constant
  double rdiv;           // RN64(1 / div)
  float add1, mul2;      // EPI_GELU: + 1.0, * 0.5
  int tokens, heads, hdim, ld_out;
  double lo, hi;
  int gelu_filter;           // EPI_GELU: constants are the ViT GELU's (sqrt2, 1, 0.5)
  float rsf[3], zpf[3];      // f32 RN(1/s_out), zp_out per group, for the rounding filters
  float lof, hif;            // lo, hi as f32
  float g_rel, g_abs, g_lim;  // GELU filter error terms, in units of t; g_lim = (0.5 - g_abs) rounded down
  int b_packed;              // Bt is the tile-packed image of nqk_pack_b
  const int32_t* colterm;    // int32 col * zpa (k_proj), or null
  // EPI_RESID with the consumer LayerNorm fused (nqk_epilogue.ln_out, round 6; k_qgemm_big<LN>)
  const float* ln_g;
  const float* ln_b;
  int8_t* ln_out;
  float ln_eps;
  int ln_mq;                 // 1: the magic-number output quantize (exact, host-checked as nqk_ln_quant's)
  double ln_rs, ln_zp, ln_lo, ln_hi;
  LnQ ln_q;
  int xcds;                  // XCDs of the device (xcd_tile's band count)
};

enum { EPI_QKV = 0, EPI_SCORES = 1, EPI_PV = 2, EPI_RESID = 3, EPI_GELU = 4, EPI_NULL = 5 };

__device__ __forceinline__ int sum16(v4i c) {
  int s = __builtin_amdgcn_sdot4(c[0], 0x01010101, 0, false);
  s = __builtin_amdgcn_sdot4(c[1], 0x01010101, s, false);
  s = __builtin_amdgcn_sdot4(c[2], 0x01010101, s, false);
  return __builtin_amdgcn_sdot4(c[3], 0x01010101, s, false);
}

// ---------------------------------------------------------------- shared epilogue
struct EpiCol {
  int64_t colterm;  // col-sum term minus the K constant (fits int32 when the kernel's I32 holds)
  float bias;
  int gn, g, hh, dd;
  bool valid;
};

template <int EPI>
__device__ __forceinline__ EpiCol epi_col(const Epi& e, int gn, int N, int64_t colsum_b, int64_t kconst) {
  EpiCol c;
  c.valid = gn < N;
  c.gn = gn;
  c.colterm = ((e.zp_flags & NQK_ZP_COL) ? colsum_b * e.zpa : 0) - kconst;
  c.bias = (e.bias != nullptr && c.valid) ? e.bias[gn] : 0.0f;
  c.g = 0;
  c.hh = 0;
  c.dd = gn;
  if constexpr (EPI == EPI_QKV) {
    c.g = gn / e.group_cols;
    const int nloc = gn - c.g * e.group_cols;
    c.hh = nloc / e.hdim;
    c.dd = nloc - c.hh * e.hdim;
  }
  return c;
}

// one output element: v = acc - zpt -> dequant -> the consumer chain -> store
template <int EPI, bool I32>
__device__ __forceinline__ void epi_elem(const Epi& e, int bz, int gm, int M, int N, int64_t rowterm, int img, int t,
                                         int img_b, int head_b, const EpiCol& c, int32_t acc, float resid, bool ok) {
  double vd;
  if constexpr (I32) {
    vd = (double)(acc - (int32_t)rowterm - (int32_t)c.colterm);  // host-checked: no int32 overflow
  } else {
    vd = (double)((int64_t)acc - rowterm - c.colterm);
  }
  const int g = c.g;
  const float d = (float)(vd * (double)e.s_acc[g]);
  const int gn = c.gn;
  if constexpr (EPI == EPI_SCORES) {
    const float y = div_rc(d, e.div, e.rdiv);
    if (ok) ((float*)e.out[0])[((int64_t)bz * M + gm) * N + gn] = y;
  } else if constexpr (EPI == EPI_RESID) {
    const float y = (c.bias + d) + resid;
    if (ok) ((float*)e.out[0])[(int64_t)gm * N + gn] = y;
  } else if constexpr (EPI == EPI_GELU) {
    const float h = c.bias + d;
    const float a = ref_erf(div_rc(h, e.div, e.rdiv)) + e.add1;
    const float y = (h * a) * e.mul2;
    const int q = quant_zp(y, e.s_out[0], e.rs_out[0], e.zp_out[0], e.lo, e.hi);
    if (ok) ((int8_t*)e.out[0])[(int64_t)gm * N + gn] = (int8_t)q;
  } else if constexpr (EPI == EPI_QKV) {
    const int q = quant_zp(c.bias + d, e.s_out[g], e.rs_out[g], e.zp_out[g], e.lo, e.hi);
    if (ok) ((int8_t*)e.out[g])[(((int64_t)img * e.heads + c.hh) * e.tokens + t) * e.hdim + c.dd] = (int8_t)q;
  } else if constexpr (EPI == EPI_NULL) {  // diagnostic: keeps the accumulators alive, stores nothing
    if (ok && acc == (int32_t)0x80000001) ((int32_t*)e.out[0])[0] = acc;
  } else {  // EPI_PV
    const int q = quant_zp(d, e.s_out[0], e.rs_out[0], e.zp_out[0], e.lo, e.hi);
    if (ok) ((int8_t*)e.out[0])[((int64_t)img_b * e.tokens + gm) * e.ld_out + head_b * e.hdim + gn] = (int8_t)q;
  }
}

// ---------------------------------------------------------------- 4-column epilogue
// (row-major staged tiles: one lane, one row, 4 consecutive columns of one head/group)
struct EpiCol4 {
  int64_t colterm[4];
  float bias[4];
  float s_acc, s_out;  // per-lane copies of the column group's scalars (no dynamic
  double rs_out, zp;   // indexing into the kernel-argument struct inside the row loop)
  float rsf, zpf;
  int8_t* out;
  int hh, dd;
};

template <int EPI>
__device__ __forceinline__ EpiCol4 epi_col4(const Epi& e, int gn0, bool ok) {
  EpiCol4 c;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    c.colterm[k] = (ok && (e.zp_flags & NQK_ZP_COL)) ? e.colsum[gn0 + k] * e.zpa : 0;
    c.bias[k] = (ok && e.bias != nullptr) ? e.bias[gn0 + k] : 0.0f;
  }
  int g = 0;
  c.hh = 0;
  c.dd = gn0;
  if constexpr (EPI == EPI_QKV) {
    g = gn0 / e.group_cols;
    const int nloc = gn0 - g * e.group_cols;
    c.hh = nloc / e.hdim;
    c.dd = nloc - c.hh * e.hdim;
  }
  g = g > 2 ? 2 : g;
  c.s_acc = g == 0 ? e.s_acc[0] : (g == 1 ? e.s_acc[1] : e.s_acc[2]);
  c.s_out = g == 0 ? e.s_out[0] : (g == 1 ? e.s_out[1] : e.s_out[2]);
  c.rs_out = g == 0 ? e.rs_out[0] : (g == 1 ? e.rs_out[1] : e.rs_out[2]);
  c.zp = g == 0 ? e.zp_out[0] : (g == 1 ? e.zp_out[1] : e.zp_out[2]);
  c.out = (int8_t*)(g == 0 ? e.out[0] : (g == 1 ? e.out[1] : e.out[2]));
  c.rsf = g == 0 ? e.rsf[0] : (g == 1 ? e.rsf[1] : e.rsf[2]);
  c.zpf = g == 0 ? e.zpf[0] : (g == 1 ? e.zpf[1] : e.zpf[2]);
  return c;
}

// RN32(x / c) from rc = RN64(1/c) without div_rc's subnormal fallback.  Used by the
// big-tile epilogues only for quotients whose exact rounding below 2^-125 cannot reach
// the output (nqk_attn.hip div_rc_w): t = y / s_out feeds rint(zp + t) (host check:
// s_out in [2^-100, 2^100]), and GELU's h / sqrt(2) feeds erf(), whose value for any
// |x| < 2^-125 only perturbs h * (erf + 1) * 0.5 at |h| < 2^-124, which quantizes to zp.
__device__ __forceinline__ float div_rc_u(float x, float c, double rc) {
  (void)c;
  return (float)((double)x * rc);
}

// quantize (numpy_quantization.py:24-34) with max/min clipping: a NaN clips to lo, as
// quant_zp returns; finite values are identical to the compare-based clip
__device__ __forceinline__ int quant_zp_u(float x, float s, double rs, double zp, double lo, double hi) {
  const float t = div_rc_u(x, s, rs);
  const double u = zp + (double)t;
  return (int)__builtin_rint(__builtin_fmin(__builtin_fmax(u, lo), hi));
}

// dequantize one accumulator: f32( f64(acc - zero-point term) * f64(s) )
template <bool I32>
__device__ __forceinline__ float dequant_elem(int32_t acc, int64_t colterm, float s_acc) {
  double vd;
  if constexpr (I32) vd = (double)(acc - (int32_t)colterm);
  else vd = (double)((int64_t)acc - colterm);
  return (float)(vd * (double)s_acc);
}

// rint(zp + t) for t = RN32(y / s) approximated by tf = RN32(y * RN32(1/s)) (|t - tf| <=
// |tf| 2^-22.4): decided by tf when the rounding boundary is farther than |tf| 2^-21 (zp is
// an integer, so zp + t rounds like t away from ties, and clipping to the integer bounds
// commutes with rounding); else *slow is set and the caller recomputes exactly
// quant_filter's decision room > |tf| 2^-21 + 2^-126 as |tf - r| + |tf| 2^-21 < Q_LIM in one
// fma: Q_LIM = (0.5 - 2^-126)(1 - 2^-23) rounded down, so a rounded-down sum that passes
// means the exact sum passes too
constexpr float Q_LIM = 0x1.fffffcp-2f;
__device__ __forceinline__ int quant_filter(float tf, float zpf, float lof, float hif, bool* slow) {
  const float r = __builtin_rintf(tf);
  const float room = 0.5f - __builtin_fabsf(tf - r);
  *slow = !(room > __builtin_fabsf(tf) * 0x1p-21f + 0x1p-126f);
  return (int)__builtin_amdgcn_fmed3f(r + zpf, lof, hif);
}

// F32X (host-checked: |acc - zero-point term| < 2^24 for every element, |zp_out| <= 2^20):
// the f32 dequantize (float)v * s_acc equals the f64 one (v and s_acc exact in f32, one
// rounding), so the QKV and GELU epilogues run in f32 with rounding filters.
template <int EPI, bool I32, bool F32X>
__device__ __forceinline__ void epi_row4(const Epi& e, int gm, int img, int t, int N, const EpiCol4& c, v4i a,
                                         float4 r) {
  float d[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    d[k] = (EPI == EPI_GELU || (EPI == EPI_QKV && F32X)) ? 0.0f : dequant_elem<I32>(a[k], c.colterm[k], c.s_acc);
  if constexpr (EPI == EPI_RESID) {
    const int64_t o = (int64_t)gm * N + c.dd;
    float4 y;
    y.x = (c.bias[0] + d[0]) + r.x;
    y.y = (c.bias[1] + d[1]) + r.y;
    y.z = (c.bias[2] + d[2]) + r.z;
    y.w = (c.bias[3] + d[3]) + r.w;
    *reinterpret_cast<float4*>((float*)e.out[0] + o) = y;
  } else if constexpr (EPI == EPI_NULL) {
    if (a[0] == (int32_t)0x80000001) ((int32_t*)e.out[0])[0] = (int)d[1];
  } else {
    uint32_t packed = 0;
    if constexpr (EPI == EPI_GELU) {
      if (F32X || e.gelu_filter) {  // F32X is only chosen with the filter (host)
        // filter: gelu_fast is within GELU_REL*|h| + GELU_ABS of the exact chain (checked
        // on all 2^32 inputs); h comes from an f32 dequant, which equals the f64 one for
        // |v| < 2^24 (v and s_acc exact in f32, one rounding); t = y / s from an f32
        // product (within |t| 2^-22.9 of RN32(y / s)).  Where those errors cannot reach a
        // rounding boundary of t (zp is an integer, so zp + t rounds like t away from
        // ties), rint(zp + t) is decided by the cheap value; all other elements (|v| >=
        // 2^24, NaN, |h| >= 2^64) take the exact chain in a wave-uniform branch.
        // the byte of q = clamp(rint(tf) + zp) straight from v_cvt_pk_u8_f32(q + 128)
        // (q + 128 in [0, 255]; ^ 0x80 per byte afterwards gives two's complement)
        const float zp128 = c.zpf + 128.0f, lo128 = e.lof + 128.0f, hi128 = e.hif + 128.0f;
        // the filter's decision per element; F32X keeps only the batch's largest measure
        // as an unsigned max of its bits (measure >= 0 or NaN: NaN / inf order above every
        // finite) and recomputes the decisions, identically, when any element may be slow
        auto decide = [&](int k, float& r, uint32_t& m) __attribute__((always_inline)) {
          int32_t vi;
          if constexpr (I32) vi = a[k] - (int32_t)c.colterm[k];
          else vi = (int32_t)__builtin_fmin(__builtin_fmax((double)((int64_t)a[k] - c.colterm[k]), -2147483520.0), 2147483520.0);
          const float df = (float)vi * c.s_acc;
          const float hf = c.bias[k] + df;
          const float tf = gelu_fast(hf) * c.rsf;
          r = __builtin_rintf(tf);
          if constexpr (F32X) {
            // g_rel also covers the product's |tf| 2^-22 (|gelu(h)| <= |h|), and
            // |s_out| <= 2^20 makes err > 0.5 for every |h| >= 2^64 (host); the test
            // |tf - r| + err < 0.5 in one fma (g_lim: 0.5 - g_abs, rounded down by 2^-23)
            m = __float_as_uint(__builtin_fmaf(__builtin_fabsf(hf), e.g_rel, __builtin_fabsf(tf - r)));
            return m >= __float_as_uint(e.g_lim);
          } else {
            const float room = 0.5f - __builtin_fabsf(tf - r);
            const float err = __builtin_fmaf(__builtin_fabsf(hf), e.g_rel, e.g_abs) + __builtin_fabsf(tf) * 0x1p-22f;
            m = 0;
            return !((room > err) & (err < 0.25f) & (__builtin_fabsf(hf) < 0x1p64f) & (vi < (1 << 24)) &
                     (vi > -(1 << 24)));
          }
        };
        bool slow[4], any_slow = false;
        uint32_t worst = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float r;
          uint32_t m;
          slow[k] = decide(k, r, m);
          if constexpr (F32X) worst = __builtin_elementwise_max(worst, m);
          else any_slow |= slow[k];
          packed = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_amdgcn_fmed3f(r + zp128, lo128, hi128), k, packed);
        }
        if constexpr (F32X) any_slow = worst >= __float_as_uint(e.g_lim);
        packed ^= 0x80808080u;
        if (__builtin_expect(__any(any_slow), 0)) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            float r;
            uint32_t m;
            if constexpr (F32X) slow[k] = decide(k, r, m);
          }
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (slow[k]) {
              const float h = c.bias[k] + dequant_elem<I32>(a[k], c.colterm[k], c.s_acc);
              const float aa = ref_erf(div_rc_u(h, e.div, e.rdiv)) + e.add1;
              const int q = quant_zp_u((h * aa) * e.mul2, c.s_out, c.rs_out, c.zp, e.lo, e.hi);
              packed = (packed & ~(0xffu << (8 * k))) | ((uint32_t)(q & 0xff) << (8 * k));
            }
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float h = c.bias[k] + dequant_elem<I32>(a[k], c.colterm[k], c.s_acc);
          const float aa = ref_erf(div_rc_u(h, e.div, e.rdiv)) + e.add1;
          const int q = quant_zp_u((h * aa) * e.mul2, c.s_out, c.rs_out, c.zp, e.lo, e.hi);
          packed |= ((uint32_t)(q & 0xff)) << (8 * k);
        }
      }
    } else if constexpr (F32X) {  // EPI_QKV, f32 with the rounding filter (quant_filter's
      // test in one fma, bytes by v_cvt_pk_u8_f32 as for GELU)
      const float zp128 = c.zpf + 128.0f, lo128 = e.lof + 128.0f, hi128 = e.hif + 128.0f;
      float y[4];
      bool slow[4], any_slow = false;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        y[k] = c.bias[k] + (float)(a[k] - (int32_t)c.colterm[k]) * c.s_acc;
        const float tf = y[k] * c.rsf;
        const float r = __builtin_rintf(tf);
        slow[k] = !(__builtin_fmaf(__builtin_fabsf(tf), 0x1p-21f, __builtin_fabsf(tf - r)) < Q_LIM);
        any_slow |= slow[k];
        packed = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_amdgcn_fmed3f(r + zp128, lo128, hi128), k, packed);
      }
      packed ^= 0x80808080u;
      if (__builtin_expect(__any(any_slow), 0)) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (slow[k]) {
            const int q = quant_zp_u(y[k], c.s_out, c.rs_out, c.zp, e.lo, e.hi);
            packed = (packed & ~(0xffu << (8 * k))) | ((uint32_t)(q & 0xff) << (8 * k));
          }
      }
    } else {  // EPI_QKV
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int q = quant_zp_u(c.bias[k] + d[k], c.s_out, c.rs_out, c.zp, e.lo, e.hi);
        packed |= ((uint32_t)(q & 0xff)) << (8 * k);
      }
    }
    if constexpr (EPI == EPI_GELU) {
      *reinterpret_cast<uint32_t*>(c.out + (int64_t)gm * N + c.dd) = packed;
    } else {
      *reinterpret_cast<uint32_t*>(c.out + (((int64_t)img * e.heads + c.hh) * e.tokens + t) * e.hdim + c.dd) = packed;
    }
  }
}

template <int EPI, bool I32>
__global__ void __launch_bounds__(256)
k_qgemm_epi(const int8_t* __restrict__ A, const int8_t* __restrict__ Bt, int M, int N, int K, int lda, int ldb,
            BatchMap bm, int64_t a_ms, int64_t b_ms, int tiles_m, int tiles_n, Epi e) {
  __shared__ __attribute__((aligned(16))) int8_t smem[2 * (FBM + FBN) * FBK];
#define AS(buf) (smem + (buf) * (FBM + FBN) * FBK)
#define BS(buf) (smem + (buf) * (FBM + FBN) * FBK + FBM * FBK)
  const int bz = blockIdx.z;
  A += map_a(bm, bz) * a_ms;
  Bt += map_b(bm, bz) * b_ms;
  // XCD-aware tile order: consecutive tiles that share an A row panel land on one XCD
  const int nwg = tiles_m * tiles_n;
  int wg = blockIdx.x;
  const int xc = e.xcds;
  if (nwg >= xc && xc > 0) {
    const int q = nwg / xc, r = nwg % xc, x = wg % xc;
    wg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + wg / xc;
  }
  const int tm = wg / tiles_n, tn = wg % tiles_n;
  const int m0 = tm * FBM, n0 = tn * FBN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const bool need_ra = (e.zp_flags & NQK_ZP_ROW) != 0, need_rb = (e.zp_flags & NQK_ZP_COL) != 0;

  v4i ra[4], rb[4];
  int psa[4] = {0, 0, 0, 0}, psb[4] = {0, 0, 0, 0};  // partial row sums of the staged chunks
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * 256, row = idx >> 3, ch = idx & 7;
      const int kk = k0 + ch * 16;
      const int gm = m0 + row, gn = n0 + row;
      const v4i z = {0, 0, 0, 0};
      ra[i] = (gm < M && kk < K) ? *reinterpret_cast<const v4i*>(A + (int64_t)gm * lda + kk) : z;
      rb[i] = (gn < N && kk < K) ? *reinterpret_cast<const v4i*>(Bt + (int64_t)gn * ldb + kk) : z;
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * 256, row = idx >> 3, ch = idx & 7;
      *reinterpret_cast<v4i*>(AS(buf) + swz128(row, ch)) = ra[i];
      *reinterpret_cast<v4i*>(BS(buf) + swz128(row, ch)) = rb[i];
      if (need_ra) psa[i] += sum16(ra[i]);
      if (need_rb) psb[i] += sum16(rb[i]);
    }
  };

  v16i acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;

  const int nk = (K + FBK - 1) / FBK;
  load_tile(0);
  store_tile(0);
  __syncthreads();
  const int r32 = lane & 31, half = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tile((kt + 1) * FBK);
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
  // row sums of the A and Bt rows of this tile (8 lanes share a row), kept in LDS
  int* rsA = reinterpret_cast<int*>(smem);
  int* rsB = rsA + FBM;
  if (need_ra || need_rb) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int sa = psa[i], sb = psb[i];
      sa += __shfl_xor(sa, 1, 64); sa += __shfl_xor(sa, 2, 64); sa += __shfl_xor(sa, 4, 64);
      sb += __shfl_xor(sb, 1, 64); sb += __shfl_xor(sb, 2, 64); sb += __shfl_xor(sb, 4, 64);
      if ((tid & 7) == 0) {
        const int row = (tid + i * 256) >> 3;
        rsA[row] = sa;
        rsB[row] = sb;
      }
    }
    __syncthreads();
  }

  // ---------------- epilogue: per-column values hoisted, per-row values once per row
  const int64_t kconst = (e.zp_flags & NQK_ZP_KCONST) ? e.zpa * e.zpb * e.kdim : 0;
  EpiCol cols[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int nl = wn * 64 + j * 32 + r32;
    cols[j] = epi_col<EPI>(e, n0 + nl, N, need_rb ? (int64_t)rsB[nl] : 0, kconst);
  }
  int img_b = 0, head_b = 0;
  if constexpr (EPI == EPI_PV) {
    img_b = bz / e.heads;
    head_b = bz - img_b * e.heads;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    float res[16][2];
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        res[r][j] = 0.0f;
        if constexpr (EPI == EPI_RESID) {
          const int gm = min(m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half, M - 1);
          res[r][j] = e.resid[(int64_t)gm * N + min(cols[j].gn, N - 1)];
        }
      }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ml = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
      const int gm = m0 + ml;
      const bool rok = gm < M;
      const int64_t rowterm = need_ra ? (int64_t)rsA[min(ml, FBM - 1)] * e.zpb : 0;
      int img = 0, t = 0;
      if constexpr (EPI == EPI_QKV) {
        img = gm / e.tokens;
        t = gm - img * e.tokens;
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
        epi_elem<EPI, I32>(e, bz, gm, M, N, rowterm, img, t, img_b, head_b, cols[j], acc[i][j][r], res[r][j],
                      rok && cols[j].valid);
    }
  }
}

// ---------------------------------------------------------------------------------------
// Projection GEMMs (A [M][K] activations x constant weights Bt [N][K]), batch 1, on
// v_mfma_i32_32x32x32_i8.  Every wave owns a 128 x 64 output block (4 x 2 tiles of
// 32x32); BK = 64; the stages are filled by global_load_lds_dwordx4 (LDS-DMA, 1 KiB
// pieces of 16 rows x 64 B, lane-linear LDS image, the conflict-free chunk swizzle applied
// to the SOURCE address) behind counted vmcnt waits and raw s_barriers.  A lane's 32
// k-bytes of one MFMA pair are contiguous (k chunk 2*half + s): integer sums do not depend
// on the k order, as long as A and B use the same one.  Both need K % 64 == 0 and
// precomputed weight column sums (zero-point COL term only).
//   k_qgemm_big: 128x256 tiles, 4 waves, a 3-stage ring with one barrier per k-step, two
//                blocks per CU (K % 192 == 0: the k loop is unrolled by the ring depth).
//   k_qgemm_pp:  256x256 tiles, 8 waves in two groups of 4 that alternate roles every
//                half k-step ("ping-pong"): while one group runs its 16 MFMAs on stage s,
//                the other reads its stage-s fragments from LDS and issues its share of
//                stage s+2, so each SIMD (one wave of each group) keeps its matrix pipe
//                busy while the partner loads; a third fewer LDS-DMA bytes per MFMA.
constexpr int GBN = 256, GBK = 64, GST = 3;
constexpr int G_RP = 32;                          // epilogue rows per pass and wave
constexpr int BIG_LDS = GST * (128 + GBN) * GBK;  // 72 KiB (>= 4 waves' staging, 36 KiB)
#ifndef NQK_PP_PD
#define NQK_PP_PD 2  // ping-pong ring: stages in flight ahead of the one being read
#endif
constexpr int PP_LDS = (NQK_PP_PD + 1) * (256 + GBN) * GBK;  // 96 KiB at depth 2 (>= 72 KiB staging)
// Diagnostic builds only (tools/gemm_diag.sh, never the shipped library): bit 1 = no
// global loads in the k loop, 2 = no LDS fragment reads, 4 = no k-step barrier, 8 = no MFMA
// (k_qgemm_big).
#ifndef NQK_DIAG
#define NQK_DIAG 0
#endif
#ifndef NQK_BIG_RPRE
#define NQK_BIG_RPRE 0  // 1: k_qgemm_big<RESID> issues pass 0's residual rows before the k loop (round 6 A/B: no gain)
#endif
#ifndef NQK_GLDS_FIRST
#define NQK_GLDS_FIRST 0  // diagnostic builds: issue the next stage's LDS-DMA before the reads
#endif

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

__device__ __forceinline__ int swz64(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4); }

// ---- epilogue of both projection GEMMs, staged through LDS (no longer read by the main
// loop): each wave owns a G_RP x 72-int32 slice; 128 / G_RP passes of G_RP rows.  Read
// back row-major, a lane takes 4 consecutive columns of one row, so bias / column terms
// are per lane and the outputs leave as 4-byte (int8) or 16-byte (f32) stores.
// LN (EPI_RESID, N = 192 = two NumPy leaves of 96: ViT-Ti; round 6): the consumer LayerNorm of every
// output row, fused.  Each pass's 32 rows of y go, besides their f32 stores, into a row image in LDS
// (after the four waves' staging slices; leaf 1 shifted by 16 floats and rows LN_IMGS floats apart,
// so the tree reads below hit 32 different banks per lane group), then — after a workgroup barrier —
// all four waves (wave 3 holds no columns at N = 192) normalize 8 rows each, 4 at a time with 16
// lanes per row: lane (row, leaf, j) sums NumPy's accumulator j of its leaf (columns leaf 96 + 8 i + j,
// in increasing i), the ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) combine and the leaf sum
// are xor butterflies 1, 2, 4, 8 (float addition commutes; only the grouping matters) — the same
// IEEE operations in the same order as k_ln_quant_lds<2> on the rows this kernel just wrote; then
// each lane normalizes, scales and quantizes 12 contiguous columns and stores them as 12 bytes.
constexpr int LN_IMGS = 232;  // floats per image row: 192 + 16 (leaf shift) + 24; 232 = 8 mod 32
__device__ __forceinline__ int ln_ipos(int c) { return c + (c >= 96 ? 16 : 0); }
template <int CTRL>  // v of another lane of the 16-lane row (DPP: no LDS round trip)
__device__ __forceinline__ float ln_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
// the residual rows of pass `pass` of a 128-row tile (rows mw + 32 pass + 4 it + (lane >> 4), the
// lane's 4 columns gn0 ..): proj_epilogue's loads, also issued by k_qgemm_big before its k loop
__device__ __forceinline__ void proj_res_load(const Epi& e, int mw, int gn0, bool cok, int M, int N, int lane, int pass,
                                              float4 (&dst)[G_RP / 4]) {
#pragma unroll
  for (int it = 0; it < G_RP / 4; ++it) {
    const int gm = min(mw + pass * G_RP + it * 4 + (lane >> 4), M - 1);
    dst[it] = cok ? *reinterpret_cast<const float4*>(e.resid + (int64_t)gm * N + gn0) : make_float4(0, 0, 0, 0);
  }
}
// PRE0 (round 6): pass 0's residual rows were loaded by the caller before its k loop (rv0)
template <int EPI, bool I32, bool F32X, int ASH = 0, bool LN = false, bool PRE0 = false>
__device__ __forceinline__ void proj_epilogue(int8_t* lds, v16i (&acc)[4][2], const Epi& e, int mw, int ncol0,
                                              int M, int N, int wave, int lane, const float4 (*rv0)[G_RP / 4] = nullptr) {
  constexpr int RP = G_RP;
  static_assert(!LN || EPI == EPI_RESID, "proj_epilogue: the LayerNorm fuses into the residual epilogue");
  const int r32 = lane & 31, half = lane >> 5;
  int32_t* stg = reinterpret_cast<int32_t*>(lds) + wave * (RP * 72);
  float* const lnimg = reinterpret_cast<float*>(lds + 4 * RP * 72 * 4);  // LN: the pass's 32 rows of y
  const int c4 = (lane & 15) * 4;
  const int gn0 = ncol0 + c4;
  const bool cok = gn0 < N;  // N % 4 == 0 (host-checked): the 4 columns are valid together
  EpiCol4 cc = epi_col4<EPI>(e, gn0, cok);
  // LN: this lane's 12 contiguous columns 12 c16 .. (gamma, beta), the same in every row
  float lg[12], lb[12];
  if constexpr (LN) {
    const int c12 = 12 * (lane & 15);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float4 g4 = *reinterpret_cast<const float4*>(e.ln_g + c12 + 4 * k);
      const float4 b4 = *reinterpret_cast<const float4*>(e.ln_b + c12 + 4 * k);
      lg[4 * k] = g4.x, lg[4 * k + 1] = g4.y, lg[4 * k + 2] = g4.z, lg[4 * k + 3] = g4.w;
      lb[4 * k] = b4.x, lb[4 * k + 1] = b4.y, lb[4 * k + 2] = b4.z, lb[4 * k + 3] = b4.w;
    }
  }
  // residual rows: pass 0's in flight while its tile is staged, every later pass's
  // issued right after the previous pass is staged (two register sets; the staged
  // accumulators of earlier passes are dead by then)
  float4 rv[2][RP / 4];
  auto load_res = [&](int pass, float4 (&dst)[RP / 4]) { proj_res_load(e, mw, gn0, cok, M, N, lane, pass, dst); };
  if constexpr (EPI == EPI_RESID) {
    if constexpr (PRE0) {
#pragma unroll
      for (int it = 0; it < RP / 4; ++it) rv[0][it] = (*rv0)[it];
    } else {
      load_res(0, rv[0]);
    }
  }
#pragma unroll
  for (int pass = 0; pass < 128 / RP; ++pass) {
#pragma unroll
    for (int ii = 0; ii < RP / 32; ++ii)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          stg[(ii * 32 + (r & 3) + 8 * (r >> 2) + 4 * half) * 72 + j * 32 + r32] = acc[pass * (RP / 32) + ii][j][r] >> ASH;
    wave_lds_sync();
    if constexpr (EPI == EPI_RESID)
      if (pass + 1 < 128 / RP) load_res(pass + 1, rv[(pass + 1) & 1]);
    // image / token of this lane's row, advanced incrementally (4 rows per step)
    int gm = mw + pass * RP + (lane >> 4);
    int img = 0, t = 0;
    if constexpr (EPI == EPI_QKV) {
      img = gm / e.tokens;
      t = gm - img * e.tokens;
    }
    auto row_acc = [&](int it) { return *reinterpret_cast<const v4i*>(stg + (it * 4 + (lane >> 4)) * 72 + c4); };
    auto row_step = [&](v4i a4, float4 r4) {
      if (gm < M && cok) epi_row4<EPI, I32, F32X>(e, gm, img, t, N, cc, a4, r4);
      gm += 4;
      if constexpr (EPI == EPI_QKV) {
        t += 4;
        while (t >= e.tokens) { t -= e.tokens; ++img; }
      }
    };
    if constexpr (LN) {
      // the residual rows as in epi_row4, and each row of y also into the LDS image
#pragma unroll
      for (int it = 0; it < RP / 4; ++it) {
        const v4i a4 = row_acc(it);
        const float4 r4 = rv[pass & 1][it];
        float4 y;
        y.x = (cc.bias[0] + dequant_elem<I32>(a4[0], cc.colterm[0], cc.s_acc)) + r4.x;
        y.y = (cc.bias[1] + dequant_elem<I32>(a4[1], cc.colterm[1], cc.s_acc)) + r4.y;
        y.z = (cc.bias[2] + dequant_elem<I32>(a4[2], cc.colterm[2], cc.s_acc)) + r4.z;
        y.w = (cc.bias[3] + dequant_elem<I32>(a4[3], cc.colterm[3], cc.s_acc)) + r4.w;
        if (gm < M && cok) *reinterpret_cast<float4*>((float*)e.out[0] + (int64_t)gm * N + cc.dd) = y;
        if (cok) *reinterpret_cast<float4*>(lnimg + (it * 4 + (lane >> 4)) * LN_IMGS + ln_ipos(gn0)) = y;
        gm += 4;
      }
      __syncthreads();  // the pass's 32 rows of y are in the image
      const int jr = lane >> 4, leaf = (lane >> 3) & 1, j = lane & 7, c16 = lane & 15;
      // the wave's 8 rows as two independent groups of 4 (their chains interleave); the butterfly
      // steps by DPP inside each 16-lane row: after step 1 the values are uniform per lane pair, after
      // step 2 per quad, after step 3 per leaf, so quad_perm [1,0,3,2], quad_perm [2,3,0,1],
      // row_half_mirror and row_mirror pair exactly the NumPy partners (xor 1, 2, 4, 8)
      float xv[2][12];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const float* irow = lnimg + (8 * wave + 4 * h2 + jr) * LN_IMGS;
#pragma unroll
        for (int i = 0; i < 12; ++i) xv[h2][i] = irow[ln_ipos(leaf * 96 + 8 * i + j)];
      }
      auto tree16 = [&](float a) __attribute__((always_inline)) {
        a = a + ln_dpp<0xB1>(a);
        a = a + ln_dpp<0x4E>(a);
        a = a + ln_dpp<0x141>(a);
        return a + ln_dpp<0x140>(a);
      };
      // the two row groups' chains as one packed pair per lane (row 0 in .x, row 1 in .y): per lane the
      // same IEEE operations in the same order as the scalar chains, one issue slot for both rows
      v2f_t nm2, inv2;
      {
        v2f_t sa = v2f_t{xv[0][0], xv[1][0]};
#pragma unroll
        for (int i = 1; i < 12; ++i) sa = sa + v2f_t{xv[0][i], xv[1][i]};
        const float s0 = tree16(sa[0]), s1 = tree16(sa[1]);
        nm2 = v2f_t{-(s0 / 192.0f), -(s1 / 192.0f)};
        v2f_t d = v2f_t{xv[0][0], xv[1][0]} + nm2;
        v2f_t va = d * d;
#pragma unroll
        for (int i = 1; i < 12; ++i) {
          d = v2f_t{xv[0][i], xv[1][i]} + nm2;
          va = va + d * d;
        }
        const float v0 = tree16(va[0]), v1 = tree16(va[1]);
        inv2 = v2f_t{1.0f / __builtin_sqrtf(v0 / 192.0f + e.ln_eps), 1.0f / __builtin_sqrtf(v1 / 192.0f + e.ln_eps)};
      }
      // normalize + affine of 12 contiguous columns of both rows (inside one leaf: 96 = 8 x 12), pairs (row 0, row 1)
      float yv[2][12];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float4 a4 = *reinterpret_cast<const float4*>(lnimg + (8 * wave + jr) * LN_IMGS + ln_ipos(12 * c16) + 4 * k);
        const float4 b4 = *reinterpret_cast<const float4*>(lnimg + (8 * wave + 4 + jr) * LN_IMGS + ln_ipos(12 * c16) + 4 * k);
        const float xa[4] = {a4.x, a4.y, a4.z, a4.w}, xb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const v2f_t y2 = (((v2f_t{xa[q], xb[q]} + nm2) * inv2) * v2f_t{lg[4 * k + q], lg[4 * k + q]}) +
                           v2f_t{lb[4 * k + q], lb[4 * k + q]};
          yv[0][4 * k + q] = y2[0];
          yv[1][4 * k + q] = y2[1];
        }
      }
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int rr = 8 * wave + 4 * h2 + jr;  // row of the pass
        uint32_t pk[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float y4[4] = {yv[h2][4 * k], yv[h2][4 * k + 1], yv[h2][4 * k + 2], yv[h2][4 * k + 3]};
          if (e.ln_mq) {
            pk[k] = ln_quant4(y4, e.ln_rs, e.ln_q);
          } else {
            uint32_t w = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float t = (float)((double)y4[q] * e.ln_rs);
              const double uu = e.ln_zp + (double)t;
              const int qv = (int)__builtin_rint(__builtin_fmin(__builtin_fmax(uu, e.ln_lo), e.ln_hi));
              w |= ((uint32_t)(qv & 0xff)) << (8 * q);
            }
            pk[k] = w;
          }
        }
        const int grow = mw + pass * RP + rr;
        if (grow < M) {
          uint32_t* o = reinterpret_cast<uint32_t*>(e.ln_out + (int64_t)grow * 192 + 12 * c16);
          o[0] = pk[0];
          o[1] = pk[1];
          o[2] = pk[2];
        }
      }
      __syncthreads();  // every wave has read the image: the next pass may overwrite it
    } else if constexpr (EPI == EPI_RESID) {
#pragma unroll
      for (int it = 0; it < RP / 4; ++it) row_step(row_acc(it), rv[pass & 1][it]);
    } else {
      // the next row's accumulators are read from LDS while this row is computed
      v4i nxt = row_acc(0);
#pragma unroll 2
      for (int it = 0; it < RP / 4; ++it) {
        const v4i cur = nxt;
        if (it + 1 < RP / 4) nxt = row_acc(it + 1);
        row_step(cur, make_float4(0, 0, 0, 0));
      }
    }
    wave_lds_sync();
  }
}

// XCD-aware tile order: XCD x (= blockIdx % XCDs) walks one contiguous band of tiles, so
// the blocks that share an A row panel share one L2
#ifndef NQK_STAGGER
#define NQK_STAGGER 0
#endif
#ifndef NQK_LN_DIAG
#define NQK_LN_DIAG 0
#endif
#ifndef NQK_TILE_ORDER
#define NQK_TILE_ORDER 0  // diagnostic builds: 1 = plain block order, 2 = column-panel bands
#endif
__device__ __forceinline__ int xcd_tile(int nwg, int xc) {
  int wg = blockIdx.x;
  if (NQK_TILE_ORDER != 1 && nwg >= xc && xc > 0) {
    const int q = nwg / xc, r = nwg % xc, x = wg % xc;
    wg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + wg / xc;
  }
  return wg;
}
// tile (tm, tn) of tile id wg: row-panel-major (blocks with consecutive ids share A rows)
__device__ __forceinline__ void tile_of(int wg, int tiles_m, int tiles_n, int& tm, int& tn) {
  if (NQK_TILE_ORDER == 2) {
    tn = wg / tiles_m;
    tm = wg - tn * tiles_m;
  } else {
    tm = wg / tiles_n;
    tn = wg - tm * tiles_n;
  }
}

// B4: the weights are int4 (|w| <= 8), nibble-packed by nqk_pack_b4: a B row of one
// k-step is 32 bytes, so a stage moves half the B bytes.  A lane's 16 k-values of one
// MFMA operand are 8 packed bytes (ds_read_b64) that unpack with two AND masks into
// bytes 16 * w (the nibble lands in the high half, its sign bit on the byte's): the
// MFMA then accumulates 16 * acc exactly (|acc| <= 2^11 K), and the epilogue takes
// acc >> 4.
template <int EPI, bool I32, bool F32X, bool B4 = false, bool LN = false>
__global__ void __launch_bounds__(256, 2)
k_qgemm_big(const int8_t* __restrict__ A, const int8_t* __restrict__ Bt, int M, int N, int K, int lda, int ldb,
            int tiles_m, int tiles_n, Epi e) {
  constexpr int GBM = 128;
  constexpr int BROW = B4 ? GBK / 2 : GBK;     // bytes of one B row per k-step
  constexpr int AP = GBM * GBK / 1024 / 4;     // A pieces per wave per stage (2)
  constexpr int BP = GBN * BROW / 1024 / 4;    // B pieces per wave per stage (4 / 2)
  constexpr int PW = AP + BP;                  // LDS-DMA ops per wave per stage (6 / 4)
  constexpr int STAGE = GBM * GBK + GBN * BROW;  // 24 / 16 KiB
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
#if NQK_STAGGER
  // diagnostic: the second block of each CU in the first dispatch round starts late
  if (blockIdx.x >= 256 && blockIdx.x < 512)
    for (int i = 0; i < NQK_STAGGER; ++i) __builtin_amdgcn_s_sleep(127);
#endif
  int tm, tn;
  tile_of(xcd_tile(tiles_m * tiles_n, e.xcds), tiles_m, tiles_n, tm, tn);
  const int m0 = tm * GBM, n0 = tn * GBN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave;  // 4 waves along N
  const int r32 = lane & 31, half = lane >> 5;

  // LDS-DMA sources: this lane's row / chunk for each 1 KiB piece (16 rows x 64 B)
  const int prow = lane >> 2, ppos = lane & 3;
  const int8_t* asrc[AP];
  const int8_t* bsrc[BP];
#pragma unroll
  for (int p = 0; p < AP; ++p) {
    const int row = (wave * AP + p) * 16 + prow;
    asrc[p] = A + (int64_t)min(m0 + row, M - 1) * lda + (ppos ^ ((row >> 2) & 3)) * 16;
  }
  // B: row-major Bt, or the tile-packed image of nqk_pack_b (every LDS-DMA piece one
  // contiguous KiB = eight full 128-B lines, the swizzle already applied)
  const bool bpk = B4 || e.b_packed != 0;
  const int64_t bstep = bpk ? (int64_t)GBN * BROW : GBK;
#pragma unroll
  for (int p = 0; p < BP; ++p) {
    const int row = (wave * BP + p) * 16 + prow;
    bsrc[p] = bpk ? Bt + (int64_t)tn * (K / GBK) * (GBN * BROW) + (wave * BP + p) * 1024 + lane * 16
                  : Bt + (int64_t)min(n0 + row, N - 1) * ldb + (ppos ^ ((row >> 2) & 3)) * 16;
  }
  auto issue = [&](int st, auto SLOT) {
    constexpr int sl = decltype(SLOT)::value;
    if constexpr ((NQK_DIAG & 1) != 0) return;
    int8_t* slot = lds + sl * STAGE;
    const int k0 = st * GBK;
    const int64_t kb = st * bstep;
#pragma unroll
    for (int p = 0; p < AP; ++p)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(asrc[p] + k0), (lds_ptr_t)(slot + (wave * AP + p) * 1024), 16, 0, 0);
#pragma unroll
    for (int p = 0; p < BP; ++p)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(bsrc[p] + kb),
                                       (lds_ptr_t)(slot + GBM * GBK + (wave * BP + p) * 1024), 16, 0, 0);
  };

  v16i acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;

  // one barrier per k-step: after it every wave has finished reading slot (kt-1)%3,
  // which the same step refills with stage kt+2 (loads spread between the MFMAs)
  auto kstep = [&](int kt, auto SLOT, auto refill, auto drain) {
    constexpr int sl = decltype(SLOT)::value;
    if constexpr (decltype(drain)::value) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW) : "memory");  // stage kt+1 may fly
    }
    if constexpr ((NQK_DIAG & 4) == 0) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const int8_t* sa = lds + sl * STAGE;
    const int8_t* sb = sa + GBM * GBK;
    if constexpr (NQK_GLDS_FIRST && decltype(refill)::value) issue(kt + 2, std::integral_constant<int, (sl + 2) % GST>{});
    v4i fa[2][4], fb[2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if constexpr ((NQK_DIAG & 2) != 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[s][i] = v4i{kt + i, lane, s, 1};
#pragma unroll
        for (int j = 0; j < 2; ++j) fb[s][j] = v4i{kt + j, lane, s, 2};
        continue;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[s][i] = *reinterpret_cast<const v4i*>(sa + swz64(i * 32 + r32, 2 * half + s));
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (B4) {
          // row of 4 x 8-byte chunks, chunk c at c ^ ((row >> 3) & 3): conflict-free b64 reads
          const int row = wn * 64 + j * 32 + r32, c = 2 * half + s;
          const uint2 w = *reinterpret_cast<const uint2*>(sb + row * 32 + ((c ^ ((row >> 3) & 3)) << 3));
          fb[s][j] = v4i{(int)((w.x << 4) & 0xF0F0F0F0u), (int)(w.x & 0xF0F0F0F0u), (int)((w.y << 4) & 0xF0F0F0F0u),
                         (int)(w.y & 0xF0F0F0F0u)};
        } else {
          fb[s][j] = *reinterpret_cast<const v4i*>(sb + swz64(wn * 64 + j * 32 + r32, 2 * half + s));
        }
      }
    }
    if constexpr (!NQK_GLDS_FIRST && decltype(refill)::value) issue(kt + 2, std::integral_constant<int, (sl + 2) % GST>{});
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if constexpr ((NQK_DIAG & 8) == 0)
            acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[s][i], fb[s][j], acc[i][j], 0, 0, 0);
          else
            acc[i][j][0] ^= fa[s][i][0] ^ fb[s][j][1];
        }
    // issue order: the s=0 fragment reads, then the MFMAs with the s=1 reads and the
    // next stage's loads spread between them
#if NQK_GLDS_FIRST
    if constexpr (decltype(refill)::value) __builtin_amdgcn_sched_group_barrier(0x020, PW, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
    for (int g = 0; g < 6; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 10, 0);
    return;
#endif
    __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
    for (int g = 0; g < 6; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    if constexpr (decltype(refill)::value) {
#pragma unroll
      for (int g = 0; g < PW; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 10 - (decltype(refill)::value ? PW : 0), 0);
    static_assert(PW <= 10, "LDS-DMA ops per stage must fit between the MFMAs");
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;
  const int nk = K / GBK;  // a multiple of 3 (host-checked): the ring slot of step kt is kt % 3
  // RESID (NQK_BIG_RPRE=1, opt-in; round 6, no gain: profiles/r06_big_rpre_dropped.txt): pass 0's residual rows issued before the k loop, so
  // the epilogue does not open on their HBM latency (ViT-Ti's residual GEMMs: 2 workgroups per CU
  // at most, latency-bound); the vmcnt waits of the loop count LDS-DMA operations only, so these
  // older loads are waited for with the first stage (vmcnt is in order)
  constexpr bool RPRE = EPI == EPI_RESID && NQK_BIG_RPRE;
  float4 rv0[G_RP / 4];
  if constexpr (RPRE) {
    const int gn0 = n0 + wn * 64 + (lane & 15) * 4;
    proj_res_load(e, m0, gn0, gn0 < N, M, N, lane, 0, rv0);
  }
  issue(0, S0{});
  issue(1, S1{});
  for (int kt = 0; kt + 3 < nk; kt += 3) {  // every step refills (stage kt + 4 < nk)
    kstep(kt, S0{}, T_{}, F_{});
    kstep(kt + 1, S1{}, T_{}, F_{});
    kstep(kt + 2, S2{}, T_{}, F_{});
  }
  kstep(nk - 3, S0{}, T_{}, F_{});
  kstep(nk - 2, S1{}, F_{}, F_{});
  kstep(nk - 1, S2{}, F_{}, T_{});
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if constexpr (RPRE) proj_epilogue<EPI, I32, F32X, B4 ? 4 : 0, LN, true>(lds, acc, e, m0, n0 + wn * 64, M, N, wave, lane, &rv0);
  else proj_epilogue<EPI, I32, F32X, B4 ? 4 : 0, LN>(lds, acc, e, m0, n0 + wn * 64, M, N, wave, lane);
}

template <int EPI, bool I32, bool F32X>
__global__ void __launch_bounds__(512, 1)
k_qgemm_pp(const int8_t* __restrict__ A, const int8_t* __restrict__ Bt, int M, int N, int K, int lda, int ldb,
           int tiles_m, int tiles_n, Epi e) {
  constexpr int BM = 256;
  constexpr int STAGE = (BM + GBN) * GBK;  // 32 KiB
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  int tm, tn;
  tile_of(xcd_tile(tiles_m * tiles_n, e.xcds), tiles_m, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * GBN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: scalar branches
  const int grp = wave >> 2, wn = wave & 3;
  const int r32 = lane & 31, half = lane >> 5;

  // LDS-DMA: each wave moves 2 A and 2 B pieces (16 rows x 64 B) of every stage
  const int prow = lane >> 2, ppos = lane & 3;
  const int8_t* asrc[2];
  const int8_t* bsrc[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int row = (wave * 2 + p) * 16 + prow;  // 0..255
    const int sw = (ppos ^ ((row >> 2) & 3)) * 16;
    asrc[p] = A + (int64_t)min(m0 + row, M - 1) * lda + sw;
    bsrc[p] = Bt + (int64_t)min(n0 + row, N - 1) * ldb + sw;
  }
  auto issue = [&](int st, int slot) {
    int8_t* sl = lds + slot * STAGE;
    const int k0 = st * GBK;
#pragma unroll
    for (int p = 0; p < 2; ++p)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(asrc[p] + k0), (lds_ptr_t)(sl + (wave * 2 + p) * 1024), 16, 0, 0);
#pragma unroll
    for (int p = 0; p < 2; ++p)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(bsrc[p] + k0),
                                       (lds_ptr_t)(sl + BM * GBK + (wave * 2 + p) * 1024), 16, 0, 0);
  };

  v16i acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;
  v4i fa[2][4], fb[2][2];
  const int nk = K / GBK;
  // load segment: this wave's fragments of stage st from its slot, then its share of
  // stage st+2 into slot (st+2) % 3 (last read two half-steps ago); lgkmcnt(0) before the
  // barrier that ends the segment (fragments in registers, slot reads retired)
  auto load_seg = [&](int st, int slot) {
    const int8_t* sa = lds + slot * STAGE;
    const int8_t* sb = sa + BM * GBK;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fa[s][i] = *reinterpret_cast<const v4i*>(sa + swz64(grp * 128 + i * 32 + r32, 2 * half + s));
#pragma unroll
      for (int j = 0; j < 2; ++j)
        fb[s][j] = *reinterpret_cast<const v4i*>(sb + swz64(wn * 64 + j * 32 + r32, 2 * half + s));
    }
    if (st + NQK_PP_PD < nk) issue(st + NQK_PP_PD, slot == 0 ? NQK_PP_PD : slot - 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  // compute segment: 16 MFMAs on the fragments of the last load segment; s_setprio keeps
  // the cluster between its barriers and ahead of the partner's loads on the SIMD
  auto compute_seg = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[s][i], fb[s][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto barrier = [&]() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
  };
  // stage st+1 complete for this wave: after each segment, the wave's own pieces of the
  // stage after the one it reads next have landed (at most stage st+2's 4 in flight)
  auto wait_next = [&](int st) {  // allow this wave's pieces of stages st+2 .. st+PD
    const int n = min(st + NQK_PP_PD, nk - 1) - (st + 1);
    if (n >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (n == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  issue(0, 0);
  for (int st = 1; st < NQK_PP_PD && st < nk; ++st) issue(st, st);
  wait_next(-1);
  barrier();
  // the stagger: group 1 runs one half-step behind group 0, so in every barrier interval
  // one group loads while the other computes; both run the same segment sequence
  if (grp == 1) barrier();
  int slot = 0;
  for (int st = 0; st < nk; ++st) {
    load_seg(st, slot);
    wait_next(st);
    barrier();
    compute_seg();
    wait_next(st);
    barrier();
    slot = slot == NQK_PP_PD ? 0 : slot + 1;
  }
  if (grp == 0) barrier();  // same barrier count for both groups
  // every load segment ended (lgkmcnt(0)) before the last barrier: the ring is free
  proj_epilogue<EPI, I32, F32X>(lds, acc, e, m0 + grp * 128, n0 + wn * 64, M, N, wave, lane);
}

// ---------------------------------------------------------------------------------------
// k_proj: persistent projection GEMM with 256 x 256 tiles, A [M][K] int8 x a tile-packed
// constant weight image (nqk_pack_b / nqk_pack_b4), K = 64 NK (NK = 12: K 768, NK = 48:
// K 3072), M % 256 == 0, N % 256 == 0.  One 512-thread workgroup per CU walks its tiles in
// order (every XCD owns a contiguous band of tile ids: the tiles in flight on one XCD
// share A row panels in its L2).  8 waves as 2 (M) x 4 (N), each owning 128 x 64 outputs
// (4 x 2 tiles of v_mfma_i32_32x32x32_i8, 128 accumulators).
//
// What bounds these GEMMs on MI355X (measured, tools/micro and DESIGN.md): the LDS-DMA
// stream from L2 delivers ~24 B per clock per CU, and on one SIMD the matrix pipe and the
// vector pipe do not overlap across waves.  So the tile is as large as the registers
// allow (256 x 256: 32 KiB staged per 1024 MFMA cycles, half the bytes per MFMA of the
// 128 x 256 kernel), the k loop keeps MFMAs issuing (the next k-step's fragment reads
// and stage publication sit between the two MFMA halves of a step), and the epilogue
// runs after the k loop with the next tile's first two stages already in flight.
// Epilogue values leave straight from the MFMA layout: QKV / GELU tiles are computed
// transposed (lane = row, 4 consecutive columns per register group: 4-byte stores of 4
// int8 values), RESID tiles not (lane = column: 2 rows x 128 B of f32 per store).  The
// column constants (int32 zero-point column terms, biases) and the residual arrive by
// LDS-DMA / buffer LDS-DMA and every VMEM operation is counted by the compile-time vmcnt
// waits (an ordinary VGPR load in the loop would make the compiler drain the LDS-DMA
// queue at its first use).
// LDS: ring of P2_DEPTH stages (4 x 32 KiB int8, 4 x 24 KiB int4 weights; EPI_RESID 3
// stages) | column constants 2 KiB | EPI_RESID: residual, 8 waves x 2 slots x 2 KiB =
// 32 KiB.  The ring depth is what the k loop's speed comes from: L2 delivers ~57 B per
// clock per CU into LDS (tools/micro/l2bw.hip) only with ~100 KiB in flight per CU; a
// 3-deep ring (one stage of lead) left the loop at ~24 B per clock.
constexpr int p2_depth(int epi) { return epi == EPI_RESID ? 3 : 4; }
constexpr int p2_stage(bool b4) { return 256 * GBK + GBN * (b4 ? GBK / 2 : GBK); }
constexpr int p2_colp(int epi, bool b4) { return p2_depth(epi) * p2_stage(b4); }
constexpr int p2_res(int epi, bool b4) { return p2_colp(epi, b4) + 2048; }
constexpr int p2_lds(int epi, bool b4) { return p2_res(epi, b4) + (epi == EPI_RESID ? 8 * 2 * 2048 : 0); }

template <int I>
using ic = std::integral_constant<int, I>;
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(ic<B>{});
    static_for<B + 1, E>(f);
  }
}

// LDS reads the compiler cannot see: a visible read of LDS-DMA'd bytes may get an
// s_waitcnt vmcnt(0) (it cannot prove the read misses the DMA in flight), which would
// drain the operand ring; the caller waits lgkmcnt
__device__ __forceinline__ int lds_read4(const void* p) {
  int v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)(lds_ptr_t)p));
  return v;
}
__device__ __forceinline__ v4i lds_read16(const void* p) {
  v4i v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)(lds_ptr_t)p));
  return v;
}
__device__ __forceinline__ void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
// the value of this register in the partner lane (lane ^ 32): v_permlane32_swap + a select
__device__ __forceinline__ uint32_t pswap32(uint32_t x) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return (threadIdx.x & 32) ? (uint32_t)r[0] : (uint32_t)r[1];
}

typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// 16-byte buffer LDS-DMA (a device function: used from a kernel's lambdas the builtin
// made the host pass drop the kernel's launch stub)
__device__ __forceinline__ void buf_lds16(rsrc_t r, void* l, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)l, 16, voff, soff, 0, 0);
}

#ifndef NQK_PJ_DIAG
#define NQK_PJ_DIAG 0  // diagnostic builds only: 1 = no epilogue stores, 2 = trivial epilogue math,
                      // 4 = no operand loads, 8 = no k-loop barriers, 16 = no fragment reads,
                      // 32 = no epilogue (results garbage)
#endif

// QKV / GELU epilogue of NG register groups of a transposed tile: group x = accumulators
// a[x][0..3] = 4 consecutive columns (column terms ct[x], biases bs[x]) of this lane's
// row; per element the operations of epi_row4 with the F32X rounding filters.  The fast
// path of all groups is one basic block (independent chains), then one wave-wide check
// sends the elements the filter could not decide through the exact chain.  Returns the
// 4 int8 results of each group packed in a dword.
template <int EPI, int ASH, int NG>
__device__ __forceinline__ void p2_quant(const Epi& e, const int (&a)[NG][4], const v4i (&ct)[NG],
                                         const v4i (&bs)[NG], float sacc, float rsf, float zpf, float s_out,
                                         double rs_out, double zp, uint32_t (&packed)[NG]) {
  constexpr int E = 4 * NG;
  // bytes as in epi_row4: v_cvt_pk_u8_f32(q + 128), ^ 0x80 per byte; the filters' tests
  // in one fma each (Q_LIM / g_lim)
  const float zp128 = zpf + 128.0f, lo128 = e.lof + 128.0f, hi128 = e.hif + 128.0f;
  // the filter's measure d = (distance to the rounding boundary's complement) + error bound
  // (>= 0, or NaN); the element is decided when d < lim.  The fast path keeps only the
  // largest d of the batch, as an unsigned max of the bit patterns (NaN and inf order
  // above every finite), one instruction per element; a batch with any undecided element
  // recomputes the same d per element (same operations, same values) for the exact chain
  const float lim = EPI == EPI_GELU ? e.g_lim : Q_LIM;
  auto measure = [&](float h, float& r) __attribute__((always_inline)) {
    float tf;
    if constexpr (EPI == EPI_GELU) tf = gelu_fast(h) * rsf;
    else tf = h * rsf;
    r = __builtin_rintf(tf);
    if constexpr (EPI == EPI_GELU) return __builtin_fmaf(__builtin_fabsf(h), e.g_rel, __builtin_fabsf(tf - r));
    else return __builtin_fmaf(__builtin_fabsf(tf), 0x1p-21f, __builtin_fabsf(tf - r));
  };
  float hv[E];
  uint32_t worst = 0;
#pragma unroll
  for (int g = 0; g < NG; ++g) packed[g] = 0;
#pragma unroll
  for (int x = 0; x < E; ++x) {
    const int v = (a[x >> 2][x & 3] >> ASH) - ct[x >> 2][x & 3];
    const float h = __int_as_float(bs[x >> 2][x & 3]) + (float)v * sacc;  // the f64 dequantize, exactly (F32X)
    hv[x] = h;
    if constexpr ((NQK_PJ_DIAG & 2) != 0) {
      packed[x >> 2] = __builtin_amdgcn_cvt_pk_u8_f32((float)(v & 255), x & 3, packed[x >> 2]);
      continue;
    }
    float r;
    const float d = measure(h, r);
    worst = __builtin_elementwise_max(worst, __float_as_uint(d));
    packed[x >> 2] = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_amdgcn_fmed3f(r + zp128, lo128, hi128), x & 3,
                                                    packed[x >> 2]);
  }
#pragma unroll
  for (int g = 0; g < NG; ++g) packed[g] ^= 0x80808080u;
  if (__builtin_expect(__any(worst >= __float_as_uint(lim)), 0)) {
#pragma unroll
    for (int x = 0; x < E; ++x) {
      float r;
      const bool slow = !(measure(hv[x], r) < lim);
      if (__any(slow)) {
        if (slow) {
          float y = hv[x];
          if constexpr (EPI == EPI_GELU) {
            const float aa = ref_erf(div_rc_u(y, e.div, e.rdiv)) + e.add1;
            y = (y * aa) * e.mul2;
          }
          const int q = quant_zp_u(y, s_out, rs_out, zp, e.lo, e.hi);
          packed[x >> 2] = (packed[x >> 2] & ~(0xffu << (8 * (x & 3)))) | ((uint32_t)(q & 0xff) << (8 * (x & 3)));
        }
      }
    }
  }
}

template <int EPI, bool F32X, int NK, bool B4>
__global__ void __launch_bounds__(512, 1)
k_proj(const int8_t* __restrict__ A, const int8_t* __restrict__ Bp, int M, int N, int lda, int tiles_n, int ntiles,
       Epi e) {
  constexpr bool RESID = EPI == EPI_RESID;
  constexpr bool TRANS = !RESID;               // lane = row (QKV / GELU) or lane = column (RESID)
  constexpr int BROW = B4 ? GBK / 2 : GBK;     // bytes of one B row per k-step
  constexpr int BPW = GBN * BROW / 1024 / 8;   // B pieces per wave per stage (2 / 1)
  constexpr int PW = 2 + BPW;                  // ring pieces per wave per stage
  constexpr int STG = 256 * GBK + GBN * BROW;
  constexpr int RD = p2_depth(EPI);
  static_assert(NK % RD == 0 && NK >= 2 * RD, "k_proj: NK a multiple of the ring depth");
  static_assert(p2_lds(EPI, B4) <= 160 * 1024, "k_proj: LDS");
  // VMEM operations of one epilogue: QKV / GELU 8 16-byte stores; RESID 15 x 8 residual
  // loads + 16 x 8 stores (the counter never holds more than 63).  Exact: the k loop's
  // vmcnt waits count the epilogue's operations as younger than the prefetched stages
  constexpr int EOPS = RESID ? 248 : 8;
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int r32 = lane & 31, half = lane >> 5;

  // this workgroup's tiles: XCD label x = blockIdx % X owns the band [lo, hi) of tile ids
  // and its workgroups take every nx-th tile from lo + jx (X = 8, fewer on a small grid)
  const int G = gridDim.x, X = G < 8 ? G : 8, x = blockIdx.x % X, jx = blockIdx.x / X;
  const int nx = (G - x + X - 1) / X;
  const int lo = (int)((int64_t)ntiles * x / X), hi = (int)((int64_t)ntiles * (x + 1) / X);
  const int first = lo + jx;
  if (first >= hi) return;
  const int cnt = (hi - first + nx - 1) / nx;
  const int64_t bstride = (int64_t)NK * GBN * BROW;

  // operands by buffer LDS-DMA: per lane one 32-bit offset each (A: the row and swizzled
  // 16-byte chunk this lane fetches; B: its 16 bytes of a 1 KiB piece), the tile and the
  // k-step in scalar offsets
  const rsrc_t r_a = make_rsrc(A, (uint32_t)((uint64_t)M * lda));
  const rsrc_t r_b = make_rsrc(Bp, (uint32_t)((uint64_t)tiles_n * bstride));
  const uint32_t va = [&] {
    const int row0 = wave * 32 + (lane >> 2), pos = lane & 3;
    return (uint32_t)(row0 * lda + ((pos ^ ((row0 >> 2) & 3)) << 4));
  }();
  const uint32_t vb = (uint32_t)(wave * BPW * 1024 + lane * 16);
  struct Src { uint32_t sa, sb; int r0, tn; };  // r0: the tile's first row
  auto src_of = [&](int tile) __attribute__((always_inline)) {
    Src s;
    const int tm = tile / tiles_n;
    s.tn = tile - tm * tiles_n;
    // a ragged last tile row is computed as rows M - 256 .. M - 1 (QKV / GELU only, host:
    // the rows it shares with the tile above are written twice with the same bytes)
    s.r0 = tm * 256 < M - 256 ? tm * 256 : M - 256;
    s.sa = (uint32_t)s.r0 * (uint32_t)lda;
    s.sb = (uint32_t)s.tn * (uint32_t)bstride;
    return s;
  };
  auto issue_stage = [&](const Src& s, auto KT, int slot) __attribute__((always_inline)) {
    constexpr int kt = decltype(KT)::value;
    if constexpr ((NQK_PJ_DIAG & 4) != 0) return;  // diagnostic: no operand loads
    int8_t* st = lds + slot * STG;
    // rows row0 and row0 + 16 (same swizzle: (row >> 2) & 3 repeats every 16 rows)
    buf_lds16(r_a, st + (2 * wave) * 1024, va, s.sa + kt * GBK);
    buf_lds16(r_a, st + (2 * wave + 1) * 1024, va, s.sa + 16u * (uint32_t)lda + kt * GBK);
#pragma unroll
    for (int p = 0; p < BPW; ++p)
      buf_lds16(r_b, st + 256 * GBK + (wave * BPW + p) * 1024, vb, s.sb + (uint32_t)(kt * GBN * BROW + p * 1024));
  };
  int8_t* const colp = lds + p2_colp(EPI, B4);
  auto issue_colp = [&](int tn) __attribute__((always_inline)) {  // waves 0 (ct) and 1 (bias)
    const int n0 = tn * GBN;
    if (wave == 0) {
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(reinterpret_cast<const int8_t*>(e.colterm + n0) + lane * 16),
                                       (lds_ptr_t)colp, 16, 0, 0);
    } else if (wave == 1 && e.bias != nullptr) {
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(reinterpret_cast<const int8_t*>(e.bias + n0) + lane * 16),
                                       (lds_ptr_t)(colp + 1024), 16, 0, 0);
    }
  };
  const rsrc_t r_res = make_rsrc(e.resid, RESID ? (uint32_t)((uint64_t)M * N * 4) : 0u);
  // RESID chunk c (0..15): MFMA tile (i, j) = (c >> 2, (c >> 1) & 1), registers 8 (c & 1) ..
  // + 7 = rows rb + 8 (el >> 2) + (el & 3) of column n
  auto res_slot = [&](int c) __attribute__((always_inline)) { return lds + p2_res(EPI, B4) + (wave * 2 + (c & 1)) * 2048; };
  auto issue_res = [&](const Src& s, int c) __attribute__((always_inline)) {
    if constexpr (RESID) {
      const int i = c >> 2, j = (c >> 1) & 1, hs = c & 1;
      const uint32_t rb = s.r0 + wm * 128 + i * 32 + 16 * hs + 4 * half;
      const uint32_t n = s.tn * GBN + wn * 64 + j * 32 + r32;
      const uint32_t o = (rb * (uint32_t)N + n) * 4u;
#pragma unroll
      for (int el = 0; el < 8; ++el)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r_res, (lds_ptr_t)(res_slot(c) + el * 256), 4, o,
                                                 (8 * (el >> 2) + (el & 3)) * N * 4, 0, 0);
    }
  };

  v16i acc[4][2];
  v4i f0a[4], f0b[2], f1a[4], f1b[2];  // the two k halves' fragments
  // fragment q of k half s from ring slot `slot`: q 0..3 the A rows of M-subtile q, 4..5
  // the B rows of N-subtile q - 4
  auto read_frag = [&](int slot, int s, int q, v4i (&fa)[4], v4i (&fb)[2]) __attribute__((always_inline)) {
    const int8_t* sa = lds + slot * STG;
    const int8_t* sb = sa + 256 * GBK;
    if constexpr ((NQK_PJ_DIAG & 16) != 0) return;  // diagnostic: no fragment reads
    if (q < 4) {
      fa[q] = *reinterpret_cast<const v4i*>(sa + swz64(wm * 128 + q * 32 + r32, 2 * half + s));
    } else {
      const int j = q - 4, row = wn * 64 + j * 32 + r32, c = 2 * half + s;
      if constexpr (B4) {
        // nibbles (inline asm read: see lds_read4); unpacked after an lgkmcnt wait
        uint2 w;
        asm volatile("ds_read_b64 %0, %1" : "=v"(w)
                     : "v"((uint32_t)(uintptr_t)(lds_ptr_t)(sb + row * 32 + ((c ^ ((row >> 3) & 3)) << 3))));
        fb[j] = v4i{(int)w.x, (int)w.y, 0, 0};
      } else {
        fb[j] = *reinterpret_cast<const v4i*>(sb + swz64(row, c));
      }
    }
  };
  auto read_frags = [&](int slot, int s, v4i (&fa)[4], v4i (&fb)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 6; ++q) read_frag(slot, s, q, fa, fb);
  };
  auto unpack = [&](v4i (&fb)[2]) __attribute__((always_inline)) {
    if constexpr (B4) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t wx = (uint32_t)fb[j][0], wy = (uint32_t)fb[j][1];
        fb[j] = v4i{(int)((wx << 4) & 0xF0F0F0F0u), (int)(wx & 0xF0F0F0F0u), (int)((wy << 4) & 0xF0F0F0F0u),
                    (int)(wy & 0xF0F0F0F0u)};
      }
    }
  };
  // the 8 MFMAs of one k half, with fn(q) issued after MFMA q (LDS reads and LDS-DMA
  // between MFMAs: one wave's in-order issue keeps the matrix pipe fed while they go out)
  auto mfmas = [&](const v4i (&fa)[4], const v4i (&fb)[2], auto&& fn) __attribute__((always_inline)) {
    static_for<0, 8>([&](auto Q) __attribute__((always_inline)) {
      constexpr int q = decltype(Q)::value, i = q >> 1, j = q & 1;
      if constexpr (TRANS) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fb[j], fa[i], acc[i][j], 0, 0, 0);
      else acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      fn(Q);
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  // ---- the epilogue of tile s (accumulators in acc)
  auto epilogue = [&](const Src& s) __attribute__((always_inline)) {
    const int r0 = s.r0, n0 = s.tn * GBN;
    if constexpr ((NQK_PJ_DIAG & 32) != 0) {  // diagnostic: no epilogue
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(acc[i][j][0]));
      return;
    }
    if constexpr (RESID) {
      int ct[2];
      float bias[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int cl = wn * 64 + j * 32 + r32;
        ct[j] = lds_read4(colp + cl * 4);
        bias[j] = e.bias ? __int_as_float(lds_read4(colp + 1024 + cl * 4)) : 0.0f;
      }
      const rsrc_t out = make_rsrc(e.out[0], (uint32_t)((uint64_t)M * N * 4));
      static_for<0, 16>([&](auto CI) __attribute__((always_inline)) {
        constexpr int c = decltype(CI)::value;
        constexpr int i = c >> 2, j = (c >> 1) & 1, hs = c & 1;
        // residual of chunk c landed (issued before the previous chunk's stores; chunk 0:
        // at the last k-step, before the RD - 1 prefetched stages)
        if constexpr (c == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((p2_depth(EPI) - 1) * PW) : "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        float res[8];
#pragma unroll
        for (int el = 0; el < 8; ++el) res[el] = __int_as_float(lds_read4(res_slot(c) + el * 256 + lane * 4));
        lgkm_wait();
        if constexpr (c + 1 < 16) issue_res(s, c + 1);
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t rb = r0 + wm * 128 + i * 32 + 16 * hs + 4 * half;
        const uint32_t o = (rb * (uint32_t)N + (uint32_t)(n0 + wn * 64 + j * 32 + r32)) * 4u;
        const int ctj = ct[j];
        float y[8];
#pragma unroll
        for (int el = 0; el < 8; ++el) {
          const int v = (acc[i][j][8 * hs + el] >> (B4 ? 4 : 0)) - ctj;
          const float d = F32X ? (float)v * e.s_acc[0] : (float)((double)v * (double)e.s_acc[0]);
          y[el] = (bias[j] + d) + res[el];
        }
#pragma unroll
        for (int el = 0; el < 8; ++el)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y[el]), out, o, (8 * (el >> 2) + (el & 3)) * N * 4, 0);
      });
    } else {
      // transposed tile: lane = row m of M-subtile i, group (j, g) = 4 consecutive columns
      // n_local = wn * 64 + j * 32 + 8 g + 4 half .. + 3
      const int cw = n0 + wn * 64;  // the wave's 64 columns: one head, one column group (host)
      int g3 = 0;
      uint32_t rowoff[4];
      if constexpr (EPI == EPI_QKV) {
        g3 = cw / e.group_cols;
        g3 = g3 > 2 ? 2 : g3;
        const int hh = (cw - g3 * e.group_cols) / e.hdim;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = r0 + wm * 128 + i * 32 + r32;
          const int img = m / e.tokens, t = m - img * e.tokens;
          rowoff[i] = (uint32_t)(((img * e.heads + hh) * e.tokens + t) * e.hdim) + 16 * half;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) rowoff[i] = (uint32_t)(r0 + wm * 128 + i * 32 + r32) * (uint32_t)N + cw + 16 * half;
      }
      const float sacc = g3 == 0 ? e.s_acc[0] : (g3 == 1 ? e.s_acc[1] : e.s_acc[2]);
      const float rsf = g3 == 0 ? e.rsf[0] : (g3 == 1 ? e.rsf[1] : e.rsf[2]);
      const float zpf = g3 == 0 ? e.zpf[0] : (g3 == 1 ? e.zpf[1] : e.zpf[2]);
      const float s_out = g3 == 0 ? e.s_out[0] : (g3 == 1 ? e.s_out[1] : e.s_out[2]);
      const double rs_out = g3 == 0 ? e.rs_out[0] : (g3 == 1 ? e.rs_out[1] : e.rs_out[2]);
      const double zp = g3 == 0 ? e.zp_out[0] : (g3 == 1 ? e.zp_out[1] : e.zp_out[2]);
      void* op = g3 == 0 ? e.out[0] : (g3 == 1 ? e.out[1] : e.out[2]);
      const rsrc_t out = make_rsrc(op, (uint32_t)(EPI == EPI_QKV ? (uint64_t)M * e.group_cols : (uint64_t)M * N));
      // batches of NG register groups (QKV: a whole MFMA tile, 16 values; GELU, whose
      // fast path holds more temporaries: half a tile), j-major: the column constants of
      // the lane's 4 column groups of N-subtile j are read at its first batch
      constexpr int NG = EPI == EPI_GELU ? 2 : 4, NB = 32 / NG;
      v4i ct[4], bs[4];
      uint32_t pk[4];  // the 4 column groups of MFMA tile (i, j), gathered over its batches
      static_for<0, NB>([&](auto BI) __attribute__((always_inline)) {
        constexpr int b = decltype(BI)::value, j = b / (NB / 2), i = (b % (NB / 2)) / (4 / NG),
                      g0 = (b % (4 / NG)) * NG;
        if constexpr (b % (NB / 2) == 0) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int cl = wn * 64 + j * 32 + 8 * g + 4 * half;
            ct[g] = lds_read16(colp + cl * 4);
            bs[g] = e.bias ? lds_read16(colp + 1024 + cl * 4) : v4i{0, 0, 0, 0};
          }
          lgkm_wait();
        }
        int a[NG][4];
        v4i cg[NG], bg[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          cg[g] = ct[g0 + g];
          bg[g] = bs[g0 + g];
#pragma unroll
          for (int k = 0; k < 4; ++k) a[g][k] = acc[i][j][4 * (g0 + g) + k];
        }
        uint32_t packed[NG];
        p2_quant<EPI, B4 ? 4 : 0, NG>(e, a, cg, bg, sacc, rsf, zpf, s_out, rs_out, zp, packed);
#pragma unroll
        for (int g = 0; g < NG; ++g) pk[g0 + g] = packed[g];
        if constexpr (g0 + NG == 4) {
          // lane (r, h) holds columns 8g + 4h .. + 3 of its row for g = 0..3; one exchange
          // with the partner half-lane gives half 0 columns 0..15 and half 1 columns
          // 16..31 of the tile: one 16-byte store per lane instead of four 4-byte ones
          const uint32_t x0 = pswap32(half ? pk[0] : pk[2]), x1 = pswap32(half ? pk[1] : pk[3]);
          const v4u st = half ? v4u{x0, pk[2], x1, pk[3]} : v4u{pk[0], x0, pk[1], x1};
          if constexpr ((NQK_PJ_DIAG & 1) != 0) {
            asm volatile("" ::"v"(st[0] ^ st[1] ^ st[2] ^ st[3]));
          } else {
            __builtin_amdgcn_raw_buffer_store_b128(st, out, rowoff[i] + j * 32, 0, 0);
          }
        }
      });
    }
  };

  // ---- the persistent loop.  Stages PF = RD - 1 ahead: the stage read at step kt + PF
  // goes into the slot step kt - 1 read (every wave's reads of it retired before the
  // barrier in the middle of step kt - 1)
  constexpr int PF = RD - 1;
  auto cap = [](int n) constexpr { return n > 63 ? 63 : n; };
  Src cur = src_of(first);
  static_for<0, PF>([&](auto S) __attribute__((always_inline)) { issue_stage(cur, S, decltype(S)::value); });
  for (int it = 0; it < cnt; ++it) {
    const Src nxt = src_of(first + (it + 1 < cnt ? it + 1 : it) * nx);
    // stage 0 of this tile landed (younger: stages 1 .. PF - 1 and the previous
    // epilogue's operations)
    if (it == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((PF - 1) * PW) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(cap((PF - 1) * PW + EOPS)) : "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    read_frags(0, 0, f0a, f0b);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;
    static_for<0, NK>([&](auto KT) __attribute__((always_inline)) {
      constexpr int kt = decltype(KT)::value;
      // first k half: F0 (read one barrier ago) in the MFMAs; between them the second
      // half's fragments (slot kt % RD), the column constants (step 0), the residual of
      // the epilogue's first chunk (last step) and the ring stage kt + PF
      if constexpr (B4) {
        lgkm_wait();
        unpack(f0b);
      }
      mfmas(f0a, f0b, [&](auto Q) __attribute__((always_inline)) {
        constexpr int q = decltype(Q)::value;
        if constexpr (q < 6) read_frag(kt % RD, 1, q, f1a, f1b);
        if constexpr (q == 6) {
          if constexpr (kt == 0) issue_colp(cur.tn);
          if constexpr (RESID && kt == NK - 1) issue_res(cur, 0);
          if constexpr (kt + PF < NK) issue_stage(cur, ic<kt + PF>{}, (kt + PF) % RD);
        }
      });
      if constexpr (kt + 1 < NK) {
        // stage kt + 1 landed (younger: the stages kt + 2 .. kt + PF issued; for the
        // stages prefetched before the previous epilogue also its operations) and this
        // step's fragment reads retired; then the barrier publishes stage kt + 1
        constexpr int last = kt + PF < NK ? kt + PF : NK - 1;
        constexpr int younger = (last >= kt + 2 ? last - kt - 1 : 0) * PW;
        if (kt + 1 <= PF - 1 && it > 0)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(cap(younger + EOPS)) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(younger) : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr ((NQK_PJ_DIAG & 8) == 0) __builtin_amdgcn_s_barrier();  // diagnostic: none
        __builtin_amdgcn_sched_barrier(0);
      } else if constexpr (B4) {
        lgkm_wait();
      }
      if constexpr (B4) unpack(f1b);
      // second k half, the next step's first-half fragments read between its MFMAs
      mfmas(f1a, f1b, [&](auto Q) __attribute__((always_inline)) {
        constexpr int q = decltype(Q)::value;
        if constexpr (kt + 1 < NK && q < 6) read_frag((kt + 1) % RD, 0, q, f0a, f0b);
      });
    });
    // the next tile's first PF stages fly during the epilogue (slot s was last read at
    // step NK - RD + s <= NK - 2, whose middle barrier every wave has passed)
    static_for<0, PF>([&](auto S) __attribute__((always_inline)) { issue_stage(nxt, S, decltype(S)::value); });
    __builtin_amdgcn_sched_barrier(0);
    epilogue(cur);
    cur = nxt;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Tile-packed image of a constant weight operand Bt [N][K] for k_qgemm_big: for column
// panel tn (256 rows, zero padded past N) and k-step kt (64 bytes), one 16 KiB block whose
// byte row*64 + pos*16 + b holds Bt[tn*256 + row][kt*64 + (pos ^ ((row >> 2) & 3))*16 + b]:
// the lane-linear LDS image of the stage, so each LDS-DMA piece is one contiguous KiB.
__global__ void k_pack_b(const int8_t* __restrict__ bt, int8_t* __restrict__ out, int64_t N, int64_t K, int64_t ldb,
                         int64_t chunks) {
  const int64_t nk = K / GBK;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < chunks; c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t blk = c >> 10, w = c & 1023;  // 1024 16-B chunks per 16 KiB block
    const int64_t tn = blk / nk, kt = blk - tn * nk;
    const int row = (int)(w >> 2), pos = (int)(w & 3);
    const int64_t n = tn * GBN + row;
    v4i v = {0, 0, 0, 0};
    if (n < N) v = *reinterpret_cast<const v4i*>(bt + n * ldb + kt * GBK + ((pos ^ ((row >> 2) & 3)) << 4));
    *reinterpret_cast<v4i*>(out + c * 16) = v;
  }
}

// nibble-packed int4 image of a weight Bt [N][K] with every value in [-8, 7], for
// k_qgemm_big<B4>: per column panel tn and k-step kt a 256 x 32-byte block; row chunk c
// (k = 16c .. 16c + 15) at chunk position c ^ ((row >> 3) & 3); inside a chunk byte b of
// word h (h = 0, 1) holds k = 16c + 8h + b in its low nibble and k = 16c + 8h + 4 + b in
// its high nibble (the order the unpack masks of the kernel produce).
__global__ void k_pack_b4(const int8_t* __restrict__ bt, uint8_t* __restrict__ out, int64_t N, int64_t K,
                          int64_t ldb, int64_t total) {
  const int64_t nk = K / GBK;
  for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += (int64_t)gridDim.x * blockDim.x) {
    const int64_t blk = o >> 13, w = o & 8191;  // 8 KiB per block
    const int64_t tn = blk / nk, kt = blk - tn * nk;
    const int row = (int)(w >> 5), pos = (int)((w >> 3) & 3), bb = (int)(w & 7);
    const int c = pos ^ ((row >> 3) & 3), h = bb >> 2, b = bb & 3;
    const int64_t n = tn * GBN + row;
    uint8_t v = 0;
    if (n < N) {
      const int8_t* src = bt + n * ldb + kt * GBK + 16 * c + 8 * h;
      v = (uint8_t)((src[b] & 0xF) | ((src[4 + b] & 0xF) << 4));
    }
    out[o] = v;
  }
}

// ------------------------------------------------------------------ LayerNorm + quantize
// 4 waves per block, one row per wave; per-wave LDS slice of row_smem(cols) bytes
__global__ void __launch_bounds__(256)
k_ln_quant(const float* __restrict__ x, const float* __restrict__ g, const float* __restrict__ b,
           int8_t* __restrict__ out, int64_t rows, int64_t cols, float eps, PwPlan p, float s, double zp, double lo,
           double hi, int64_t slice) {
  const double rs = 1.0 / (double)s;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float* v = sm + w * slice;
  float* part = v + cols;
  float* leafv = part + kMaxLeaves * 8;
  const float fcols = (float)cols;
  for (int64_t r = (int64_t)blockIdx.x * 4 + w; r < rows; r += (int64_t)gridDim.x * 4) {
    const float* xr = x + r * cols;
    for (int64_t i = lane; i < cols; i += 64) v[i] = xr[i];
    wave_lds_sync();
    const float mean = wave_pairwise_sum(v, p, part, leafv) / fcols;
    const float nmean = -mean;
    for (int64_t i = lane; i < cols; i += 64) {
      const float d = v[i] + nmean;
      v[i] = d * d;
    }
    wave_lds_sync();
    const float var = wave_pairwise_sum(v, p, part, leafv) / fcols;
    const float inv = 1.0f / __builtin_sqrtf(var + eps);
    int8_t* orow = out + r * cols;
    for (int64_t i = lane; i < cols; i += 64) {
      const float d = xr[i] + nmean;
      const float y = ((d * inv) * g[i]) + b[i];
      orow[i] = (int8_t)quant_zp(y, s, rs, zp, lo, hi);
    }
    wave_lds_sync();
  }
}

// LayerNorm + quantize with the whole NumPy pairwise tree in registers, for rows whose
// plan is a complete binary tree of NL equal leaves of 96 columns (768 = 8 x 96 for
// ViT-Base): lane (leaf, g) owns NumPy's accumulators r[4g..4g+3] of that leaf, i.e.
// columns leaf*96 + 8i + 4g + (0..3) — one float4 per i, summed in increasing i; the
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) combine and the leaf tree are xor-butterflies
// (float addition is commutative, only the grouping matters).  2*NL lanes per row,
// 64 / (2*NL) rows per wave; every load and store is 16 / 4 bytes per lane.
#ifndef NQK_LN_LB
#define NQK_LN_LB 1
#endif
template <int NL, bool MQ = false>
__global__ void __launch_bounds__(256, NQK_LN_LB)
k_ln_quant_reg(const float* __restrict__ x, const float* __restrict__ g, const float* __restrict__ b,
               int8_t* __restrict__ out, int64_t rows, float eps, float s, double rs, double zp, double lo,
               double hi, LnQ mq) {
  constexpr int LF = 96, LPR = NL * 2, NI = LF / 8, COLS = NL * LF;
  const int lane = threadIdx.x & 63;
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int u = lane % LPR, leaf = u >> 1, grp = u & 1;
  const bool ok = row < rows;
  const int c0 = leaf * LF + 4 * grp;
  const float* xr = x + (ok ? row : 0) * COLS + c0;
  float4 xv[NI];
#if NQK_LN_DIAG
  // diagnostic only (wrong values): fully coalesced loads of the wave's rows
  const float* wbase = x + (((int64_t)blockIdx.x * 256 + (threadIdx.x & ~63)) / LPR) * COLS;
#pragma unroll
  for (int i = 0; i < NI; ++i) xv[i] = *reinterpret_cast<const float4*>(wbase + (i * 64 + lane) * 4);
#else
#pragma unroll
  for (int i = 0; i < NI; ++i) xv[i] = *reinterpret_cast<const float4*>(xr + 8 * i);
#endif
  float a0 = xv[0].x, a1 = xv[0].y, a2 = xv[0].z, a3 = xv[0].w;
#pragma unroll
  for (int i = 1; i < NI; ++i) {
    a0 = a0 + xv[i].x; a1 = a1 + xv[i].y; a2 = a2 + xv[i].z; a3 = a3 + xv[i].w;
  }
  float acc = (a0 + a1) + (a2 + a3);
#pragma unroll
  for (int m = 1; m < LPR; m <<= 1) acc = acc + __shfl_xor(acc, m, 64);
  const float fcols = (float)COLS;
  const float nmean = -(acc / fcols);
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    xv[i].x = xv[i].x + nmean; xv[i].y = xv[i].y + nmean; xv[i].z = xv[i].z + nmean; xv[i].w = xv[i].w + nmean;
  }
  a0 = xv[0].x * xv[0].x; a1 = xv[0].y * xv[0].y; a2 = xv[0].z * xv[0].z; a3 = xv[0].w * xv[0].w;
#pragma unroll
  for (int i = 1; i < NI; ++i) {
    a0 = a0 + xv[i].x * xv[i].x; a1 = a1 + xv[i].y * xv[i].y;
    a2 = a2 + xv[i].z * xv[i].z; a3 = a3 + xv[i].w * xv[i].w;
  }
  float v2 = (a0 + a1) + (a2 + a3);
#pragma unroll
  for (int m = 1; m < LPR; m <<= 1) v2 = v2 + __shfl_xor(v2, m, 64);
  const float var = v2 / fcols;
  const float inv = 1.0f / __builtin_sqrtf(var + eps);
  if (!ok) return;
  int8_t* orow = out + row * COLS + c0;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const float4 gg = *reinterpret_cast<const float4*>(g + c0 + 8 * i);
    const float4 bb = *reinterpret_cast<const float4*>(b + c0 + 8 * i);
    const float y[4] = {((xv[i].x * inv) * gg.x) + bb.x, ((xv[i].y * inv) * gg.y) + bb.y,
                        ((xv[i].z * inv) * gg.z) + bb.z, ((xv[i].w * inv) * gg.w) + bb.w};
    uint32_t packed = 0;
    if constexpr (MQ) {
      packed = ln_quant4(y, rs, mq);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float t = (float)((double)y[k] * rs);
        const double uu = zp + (double)t;
        const int q = (int)__builtin_rint(__builtin_fmin(__builtin_fmax(uu, lo), hi));
        packed |= ((uint32_t)(q & 0xff)) << (8 * k);
      }
    }
    *reinterpret_cast<uint32_t*>(orow + 8 * i) = packed;
  }
}

// The same register tree, with the rows moved through LDS so that every global load and
// store of a wave is one contiguous 1 KiB (the tree's lane layout reads 16 B at a 32-B
// stride: 8 segments per row and instruction).  A wave's RW = 64 / (2 NL) rows are
// contiguous in memory: loaded linearly into the wave's own LDS image (16 B of pad per
// 96-column leaf: conflict-free reads in the tree layout), read in the tree layout,
// and the packed int8 results written back into LDS (784-B rows: conflict-free dword
// writes) and stored linearly.  No workgroup barrier: each wave owns its LDS image.
// (Measured slower and dropped in round 4: an f32 rounding filter in front of the f64
// quantize chain, 40.9 vs 39.3 us per launch at 50432 x 768, profiles/r04_ln_filter_dropped.txt;
// two row groups per wave with the second group's loads under the first's work, 40.8 vs
// 39.7 us, profiles/r04_ln_gpw_dropped.txt.)
#ifndef NQK_LN_PK
#define NQK_LN_PK 1  // 1: the f32 element arithmetic of the LDS variant as packed pairs (round 5)
#endif
#ifndef NQK_LN_NT
#define NQK_LN_NT 0  // 1: the f32 row loads non-temporal (read once; A/B variant, round 5)
#endif
#ifndef NQK_LN_DMA
#define NQK_LN_DMA 1  // 1: the rows by LDS-DMA (buffer_load ... lds) into an XOR-swizzled image (round 5)
#endif
// NQK_LN_DMA: LDS-DMA writes a wave's 64 x 16 B contiguously, so the image cannot carry the
// per-leaf pad; instead 16-B chunk c of row r sits at position c ^ 2 h (bits 1-2 flipped, inside
// the leaf's aligned 8-chunk blocks: an involution), h = (leaf >> 1) & 3 for 8 leaves, r & 3 for
// 4 and 2.  A tree read (chunk 24 leaf + 2 i + grp of each lane's row) then puts the 16 lanes of
// every ds_read_b128 lane group on 16 different 4-bank slots (rows of 24 NL chunks = 0 mod 16;
// checked for every i and lane group of MI355X_MICROARCH.md's table by tests/test_host.py)
__host__ __device__ constexpr int ln_swz(int nl, int r, int c) {
  return c ^ ((nl == 8 ? ((c / 24) >> 1) & 3 : r & 3) << 1);
}
template <int NL, bool MQ = false, int WPB = 4>  // WPB: waves (row groups) per workgroup
__global__ void __launch_bounds__(64 * WPB)
k_ln_quant_lds(const float* __restrict__ x, const float* __restrict__ g, const float* __restrict__ b,
               int8_t* __restrict__ out, int64_t rows, float eps, float s, double rs, double zp, double lo,
               double hi, LnQ mq) {
  constexpr int LF = 96, LPR = NL * 2, NI = LF / 8, COLS = NL * LF, RW = 64 / LPR;
  constexpr int CH = COLS / 4;                      // 16-B chunks per row
  constexpr bool DMA = NQK_LN_DMA;
  constexpr int RSI = COLS * 4 + (DMA ? 0 : NL * 16);  // LDS bytes per input row
  constexpr int RSO = COLS + 16;                    // LDS bytes per output row
  constexpr int WLDS = RW * RSI;                    // >= RW * RSO
  constexpr int NLD = RW * CH / 64, NST = RW * COLS / 16 / 64;
  static_assert(RW * CH % 64 == 0 && RW * COLS % 1024 == 0, "k_ln_quant_lds: shape");
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int8_t* const wl = lds + wave * WLDS;
  const int64_t row0 = ((int64_t)blockIdx.x * WPB + wave) * RW;
  if (row0 >= rows) return;  // (uniform per wave; no workgroup barrier follows)
  // ---- linear loads (rows past the end read the last row; not stored)
  if constexpr (DMA) {
    // position P = 64 k + lane of the image <- row P / CH, chunk ln_swz(P % CH)
    const rsrc_t rx = make_rsrc(x, (uint32_t)((uint64_t)rows * COLS * 4));
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int P = k * 64 + lane, r = P / CH, c = ln_swz(NL, r, P - r * CH);
      const int64_t gr = row0 + r < rows ? row0 + r : rows - 1;
      buf_lds16(rx, wl + k * 1024, (uint32_t)(gr * COLS + c * 4) * 4u, 0u);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  float4 ld[NLD];
#pragma unroll
  for (int k = 0; k < NLD && !DMA; ++k) {
    const int C = k * 64 + lane, r = C / CH, c = C - r * CH;
    const int64_t gr = row0 + r < rows ? row0 + r : rows - 1;
    if constexpr (NQK_LN_NT) {
      typedef float v4f_nt __attribute__((ext_vector_type(4)));
      const v4f_nt v = __builtin_nontemporal_load(reinterpret_cast<const v4f_nt*>(x + gr * COLS + c * 4));
      ld[k] = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      ld[k] = *reinterpret_cast<const float4*>(x + gr * COLS + c * 4);
    }
  }
#pragma unroll
  for (int k = 0; k < NLD && !DMA; ++k) {
    const int C = k * 64 + lane, r = C / CH, c = C - r * CH;
    *reinterpret_cast<float4*>(wl + r * RSI + c * 16 + (c / (LF / 4)) * 16) = ld[k];
  }
  if constexpr (!DMA) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  // ---- the tree layout: lane (row r, leaf, grp) holds columns leaf*96 + 8i + 4grp + 0..3
  const int r = lane / LPR, u = lane % LPR, leaf = u >> 1, grp = u & 1;
  const int c0 = leaf * LF + 4 * grp;
  float4 xv[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i)
    xv[i] = *reinterpret_cast<const float4*>(
        wl + r * RSI + (DMA ? ln_swz(NL, r, leaf * (LF / 4) + 2 * i + grp) * 16 : (leaf * (LF / 4) + 2 * i + grp) * 16 + leaf * 16));
  float inv, nmean;
  v2f_t xl[NI], xh[NI];  // NQK_LN_PK: xv[i] as the pairs (x, y), (z, w), centred in place
  if constexpr (NQK_LN_PK) {
    // element pairs as packed f32 (v_pk_add / v_pk_mul: per lane the same IEEE operations in
    // the same order as the scalar form below, one issue slot for two elements)
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      xl[i] = v2f_t{xv[i].x, xv[i].y};
      xh[i] = v2f_t{xv[i].z, xv[i].w};
    }
    v2f_t al = xl[0], ah = xh[0];
#pragma unroll
    for (int i = 1; i < NI; ++i) {
      al = al + xl[i];
      ah = ah + xh[i];
    }
    float acc = (al[0] + al[1]) + (ah[0] + ah[1]);
#pragma unroll
    for (int m = 1; m < LPR; m <<= 1) acc = acc + __shfl_xor(acc, m, 64);
    nmean = -(acc / (float)COLS);
    const v2f_t nm2 = v2f_t{nmean, nmean};
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      xl[i] = xl[i] + nm2;
      xh[i] = xh[i] + nm2;
    }
    al = xl[0] * xl[0];
    ah = xh[0] * xh[0];
#pragma unroll
    for (int i = 1; i < NI; ++i) {
      al = al + xl[i] * xl[i];
      ah = ah + xh[i] * xh[i];
    }
    float v2 = (al[0] + al[1]) + (ah[0] + ah[1]);
#pragma unroll
    for (int m = 1; m < LPR; m <<= 1) v2 = v2 + __shfl_xor(v2, m, 64);
    inv = 1.0f / __builtin_sqrtf(v2 / (float)COLS + eps);
  } else {
    float a0 = xv[0].x, a1 = xv[0].y, a2 = xv[0].z, a3 = xv[0].w;
  #pragma unroll
    for (int i = 1; i < NI; ++i) {
      a0 = a0 + xv[i].x; a1 = a1 + xv[i].y; a2 = a2 + xv[i].z; a3 = a3 + xv[i].w;
    }
    float acc = (a0 + a1) + (a2 + a3);
  #pragma unroll
    for (int m = 1; m < LPR; m <<= 1) acc = acc + __shfl_xor(acc, m, 64);
    const float fcols = (float)COLS;
    nmean = -(acc / fcols);
  #pragma unroll
    for (int i = 0; i < NI; ++i) {
      xv[i].x = xv[i].x + nmean; xv[i].y = xv[i].y + nmean; xv[i].z = xv[i].z + nmean; xv[i].w = xv[i].w + nmean;
    }
    a0 = xv[0].x * xv[0].x; a1 = xv[0].y * xv[0].y; a2 = xv[0].z * xv[0].z; a3 = xv[0].w * xv[0].w;
  #pragma unroll
    for (int i = 1; i < NI; ++i) {
      a0 = a0 + xv[i].x * xv[i].x; a1 = a1 + xv[i].y * xv[i].y;
      a2 = a2 + xv[i].z * xv[i].z; a3 = a3 + xv[i].w * xv[i].w;
    }
    float v2 = (a0 + a1) + (a2 + a3);
  #pragma unroll
    for (int m = 1; m < LPR; m <<= 1) v2 = v2 + __shfl_xor(v2, m, 64);
    const float var = v2 / fcols;
    inv = 1.0f / __builtin_sqrtf(var + eps);
  }
  // every lane's tree reads are done before the image is overwritten (in-order LDS)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const float4 gg = *reinterpret_cast<const float4*>(g + c0 + 8 * i);
    const float4 bb = *reinterpret_cast<const float4*>(b + c0 + 8 * i);
    float y[4];
    if constexpr (NQK_LN_PK) {
      const v2f_t i2 = v2f_t{inv, inv};
      const v2f_t yl = ((xl[i] * i2) * v2f_t{gg.x, gg.y}) + v2f_t{bb.x, bb.y};
      const v2f_t yh = ((xh[i] * i2) * v2f_t{gg.z, gg.w}) + v2f_t{bb.z, bb.w};
      y[0] = yl[0], y[1] = yl[1], y[2] = yh[0], y[3] = yh[1];
    } else {
      y[0] = ((xv[i].x * inv) * gg.x) + bb.x, y[1] = ((xv[i].y * inv) * gg.y) + bb.y;
      y[2] = ((xv[i].z * inv) * gg.z) + bb.z, y[3] = ((xv[i].w * inv) * gg.w) + bb.w;
    }
    uint32_t packed = 0;
    if constexpr (MQ) {
      packed = ln_quant4<NQK_LN_PK>(y, rs, mq);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float t = (float)((double)y[k] * rs);
        const double uu = zp + (double)t;
        const int q = (int)__builtin_rint(__builtin_fmin(__builtin_fmax(uu, lo), hi));
        packed |= ((uint32_t)(q & 0xff)) << (8 * k);
      }
    }
    *reinterpret_cast<uint32_t*>(wl + r * RSO + c0 + 8 * i) = packed;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  // ---- linear stores
#pragma unroll
  for (int k = 0; k < NST; ++k) {
    const int C = k * 64 + lane, rr = C / (COLS / 16), c = C - rr * (COLS / 16);
    const v4i v = *reinterpret_cast<const v4i*>(wl + rr * RSO + c * 16);
    if (row0 + rr < rows) *reinterpret_cast<v4i*>(out + (row0 + rr) * COLS + c * 16) = v;
  }
}
// Persistent form (round 5, NQK_LN_PERS): one-wave workgroups, LN_PERS_W per CU, each walking
// row groups g, g + grid, ... with the next group's rows loaded by LDS-DMA into the second half
// of a double-buffered image while the current group is reduced, quantized and stored (the
// single-shot kernel's waves load, then compute, then store: in a grid that is one or a few
// waves per slot those phases line up across the chip).  gamma / beta stay in registers (a
// lane's columns are the same in every group).  Same arithmetic as k_ln_quant_lds with
// NQK_LN_PK / NQK_LN_DMA.
template <int NL, bool MQ>
__global__ void __launch_bounds__(64)
k_ln_quant_pers(const float* __restrict__ x, const float* __restrict__ g, const float* __restrict__ b,
                int8_t* __restrict__ out, int64_t rows, float eps, double rs, double zp, double lo, double hi, LnQ mq) {
  constexpr int LF = 96, LPR = NL * 2, NI = LF / 8, COLS = NL * LF, RW = 64 / LPR;
  constexpr int CH = COLS / 4, RSI = COLS * 4, RSO = COLS + 16, WLDS = RW * RSI;
  constexpr int NLD = RW * CH / 64, NST = RW * COLS / 16 / 64;
  static_assert(RW * CH % 64 == 0 && RW * COLS % 1024 == 0 && RW * RSO <= WLDS, "k_ln_quant_pers: shape");
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  const int lane = threadIdx.x;
  const int64_t ngroups = (rows + RW - 1) / RW;
  int64_t grp = blockIdx.x;
  if (grp >= ngroups) return;
  // rx0: an empty buffer (loads return 0, no memory access) for the pieces issued after the
  // last group, so every iteration issues the same NLD pieces (uniform counted waits: the
  // compiler's own wait for the previous stores' data registers is then vmcnt(NLD), not 0)
  const rsrc_t rx = make_rsrc(x, (uint32_t)((uint64_t)rows * COLS * 4)), rx0 = make_rsrc(x, 0u);
  auto issue = [&](int64_t gi, int8_t* img, rsrc_t rr) {
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      const int P = k * 64 + lane, r = P / CH, c = ln_swz(NL, r, P - r * CH);
      const int64_t gr = gi * RW + r < rows ? gi * RW + r : rows - 1;
      buf_lds16(rr, img + k * 1024, (uint32_t)(gr * COLS + c * 4) * 4u, 0u);
    }
  };
  const int r = lane / LPR, u = lane % LPR, leaf = u >> 1, gq = u & 1;
  const int c0 = leaf * LF + 4 * gq;
  v2f_t gl[NI], gh[NI], bl[NI], bh[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const float4 gg = *reinterpret_cast<const float4*>(g + c0 + 8 * i);
    const float4 bb = *reinterpret_cast<const float4*>(b + c0 + 8 * i);
    gl[i] = v2f_t{gg.x, gg.y}, gh[i] = v2f_t{gg.z, gg.w}, bl[i] = v2f_t{bb.x, bb.y}, bh[i] = v2f_t{bb.z, bb.w};
  }
  // the parameters are in registers before any LDS-DMA is counted (the loop's waits are exact)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < NI; ++i) asm volatile("" : "+v"(gl[i]), "+v"(gh[i]), "+v"(bl[i]), "+v"(bh[i]));
  issue(grp, lds, rx);
  for (int cur = 0; grp < ngroups; grp += gridDim.x, cur ^= 1) {
    int8_t* const wl = lds + cur * WLDS;
    const int64_t nxt = grp + gridDim.x;
    // the other half held the previous group's staged output, read (lgkmcnt 0) before its stores;
    // vmcnt(NLD): this group's pieces (and the previous group's stores, issued before the next
    // pieces) are done, the next group's NLD pieces stay in flight
    issue(nxt < ngroups ? nxt : grp, lds + (cur ^ 1) * WLDS, nxt < ngroups ? rx : rx0);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NLD) : "memory");
    __builtin_amdgcn_wave_barrier();
    // the tree reads by inline asm, their lgkmcnt wait tied to the values: a compiler-visible LDS
    // read is given an s_waitcnt vmcnt(0) for the LDS-DMA in flight (it cannot tell the halves
    // apart), which would drain the next group's pieces
    typedef float v4f_t __attribute__((ext_vector_type(4)));
    v4f_t tv[NI];
    static_assert(NI == 12, "k_ln_quant_pers: 12 tree reads");
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const uint32_t a = (uint32_t)(uintptr_t)(lds_ptr_t)(wl + r * RSI + ln_swz(NL, r, leaf * (LF / 4) + 2 * i + gq) * 16);
      asm volatile("ds_read_b128 %0, %1" : "=v"(tv[i]) : "v"(a));
    }
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(tv[0]), "+v"(tv[1]), "+v"(tv[2]), "+v"(tv[3]), "+v"(tv[4]), "+v"(tv[5]), "+v"(tv[6]),
                   "+v"(tv[7]), "+v"(tv[8]), "+v"(tv[9]), "+v"(tv[10]), "+v"(tv[11])::"memory");
    v2f_t xl[NI], xh[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) xl[i] = v2f_t{tv[i][0], tv[i][1]}, xh[i] = v2f_t{tv[i][2], tv[i][3]};
    v2f_t al = xl[0], ah = xh[0];
#pragma unroll
    for (int i = 1; i < NI; ++i) al = al + xl[i], ah = ah + xh[i];
    float acc = (al[0] + al[1]) + (ah[0] + ah[1]);
#pragma unroll
    for (int m = 1; m < LPR; m <<= 1) acc = acc + __shfl_xor(acc, m, 64);
    const float nmean = -(acc / (float)COLS);
    const v2f_t nm2 = v2f_t{nmean, nmean};
#pragma unroll
    for (int i = 0; i < NI; ++i) xl[i] = xl[i] + nm2, xh[i] = xh[i] + nm2;
    al = xl[0] * xl[0], ah = xh[0] * xh[0];
#pragma unroll
    for (int i = 1; i < NI; ++i) al = al + xl[i] * xl[i], ah = ah + xh[i] * xh[i];
    float v2 = (al[0] + al[1]) + (ah[0] + ah[1]);
#pragma unroll
    for (int m = 1; m < LPR; m <<= 1) v2 = v2 + __shfl_xor(v2, m, 64);
    const float inv = 1.0f / __builtin_sqrtf(v2 / (float)COLS + eps);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // tree reads done before the staging overwrites
    __builtin_amdgcn_wave_barrier();
    const v2f_t i2 = v2f_t{inv, inv};
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const v2f_t yl = ((xl[i] * i2) * gl[i]) + bl[i], yh = ((xh[i] * i2) * gh[i]) + bh[i];
      const float y[4] = {yl[0], yl[1], yh[0], yh[1]};
      uint32_t packed = 0;
      if constexpr (MQ) {
        packed = ln_quant4<true>(y, rs, mq);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float t = (float)((double)y[k] * rs);
          const int q = (int)__builtin_rint(__builtin_fmin(__builtin_fmax(zp + (double)t, lo), hi));
          packed |= ((uint32_t)(q & 0xff)) << (8 * k);
        }
      }
      *reinterpret_cast<uint32_t*>(wl + r * RSO + c0 + 8 * i) = packed;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const int64_t row0 = grp * RW;
    v4i sv[NST];
#pragma unroll
    for (int k = 0; k < NST; ++k) {
      const int C = k * 64 + lane, rr = C / (COLS / 16), c = C - rr * (COLS / 16);
      sv[k] = *reinterpret_cast<const v4i*>(wl + rr * RSO + c * 16);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // staging read before the next issue refills it
#pragma unroll
    for (int k = 0; k < NST; ++k) {
      const int C = k * 64 + lane, rr = C / (COLS / 16), c = C - rr * (COLS / 16);
      if (row0 + rr < rows) *reinterpret_cast<v4i*>(out + (row0 + rr) * COLS + c * 16) = sv[k];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the wave's LDS is released
}
constexpr int ln_lds_bytes(int nl, int wpb = 4) { return wpb * (64 / (2 * nl)) * (nl * 96 * 4 + (NQK_LN_DMA ? 0 : nl * 16)); }

// ------------------------------------------------------------------ Softmax + quantize
// one row per wave; output row stride ldo (>= cols, pad zero-filled); optional row sums
__global__ void __launch_bounds__(256)
k_softmax_quant(const float* __restrict__ x, int8_t* __restrict__ out, int64_t* __restrict__ rowsum, int64_t rows,
                int64_t cols, int64_t ldo, PwPlan p, float s, double zp, double lo, double hi, int64_t slice) {
  const double rs = 1.0 / (double)s;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float* v = sm + w * slice;
  float* part = v + cols;
  float* leafv = part + kMaxLeaves * 8;
  for (int64_t r = (int64_t)blockIdx.x * 4 + w; r < rows; r += (int64_t)gridDim.x * 4) {
    const float* xr = x + r * cols;
    float mx = -__builtin_inff();
    for (int64_t i = lane; i < cols; i += 64) {
      const float t = xr[i];
      v[i] = t;
      mx = t > mx ? t : mx;
    }
    for (int off = 32; off > 0; off >>= 1) {
      const float o = __shfl_xor(mx, off, 64);
      mx = o > mx ? o : mx;
    }
    const float nm = -mx;
    for (int64_t i = lane; i < cols; i += 64) v[i] = np_expf(v[i] + nm);
    wave_lds_sync();
    const float ssum = wave_pairwise_sum(v, p, part, leafv);
    const double rsum = 1.0 / (double)ssum;
    int8_t* orow = out + r * ldo;
    int64_t acc = 0;
    for (int64_t i = lane; i < ldo; i += 64) {
      int q = 0;
      if (i < cols) {
        q = quant_zp(div_rc(v[i], ssum, rsum), s, rs, zp, lo, hi);
        acc += q;
      }
      orow[i] = (int8_t)q;
    }
    if (rowsum) {
      for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
      if (lane == 0) rowsum[r] = acc;
    }
    wave_lds_sync();
  }
}

// ------------------------------------------------------------------ int8 transpose + pad
// src [nb][R][C] -> dst [nb][C][Rp] (Rp >= R, pad zero); block = (64 columns, one matrix),
// loops over R in 64-row tiles; optional rowsum[nb][C] = sum over R.
__global__ void __launch_bounds__(256)
k_transpose_pad(const int8_t* __restrict__ src, int8_t* __restrict__ dst, int64_t* __restrict__ rowsum, int64_t nb,
                int64_t R, int64_t C, int64_t Rp) {
  __shared__ int8_t tile[64][65];
  __shared__ int colsum[4][64];
  const int64_t b = blockIdx.y;
  const int c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int8_t* s = src + b * R * C;
  int8_t* d = dst + b * C * Rp;
  int csum = 0;
  for (int r0 = 0; r0 < Rp; r0 += 64) {
    for (int i = ty; i < 64; i += 4) {
      const int r = r0 + i, c = c0 + tx;
      const int8_t val = (r < R && c < C) ? s[(int64_t)r * C + c] : (int8_t)0;
      tile[i][tx] = val;
      csum += val;
    }
    __syncthreads();
    for (int i = ty; i < 64; i += 4) {
      const int c = c0 + i, r = r0 + tx;
      if (c < C && r < Rp) d[(int64_t)c * Rp + r] = tile[tx][i];
    }
    __syncthreads();
  }
  if (rowsum) {
    colsum[ty][tx] = csum;
    __syncthreads();
    if (ty == 0 && c0 + tx < C)
      rowsum[b * C + c0 + tx] = (int64_t)colsum[0][tx] + colsum[1][tx] + colsum[2][tx] + colsum[3][tx];
  }
}

}  // namespace
}  // namespace nqk

using namespace nqk;

// projection GEMM kernel: the 128x256 one; NQK_GEMM_PP=1 selects the ping-pong 256x256
// one (measured no faster: the k loop is bound by the LDS-DMA latency, not the issue)
static bool gemm_pingpong() {
  const char* v = getenv("NQK_GEMM_PP");
  return v && atoi(v) == 1;
}

template <int EPI, bool I32, bool F32X>
static void launch_big(bool pp, const int8_t* a, const int8_t* bt, int64_t M, int64_t N, int64_t K, int64_t lda,
                       int64_t ldb, const Epi& e) {
  const int tn = (int)((N + GBN - 1) / GBN);
  if constexpr (EPI == EPI_RESID && !F32X) {
    if (e.ln_out != nullptr) {  // the consumer LayerNorm fused (N = 192, host-checked)
      const int tm = (int)((M + 127) / 128);
      if (e.b_packed == 2)
        hipLaunchKernelGGL((k_qgemm_big<EPI, I32, F32X, true, true>), dim3(tm * tn), dim3(256), BIG_LDS, stream(), a,
                           bt, (int)M, (int)N, (int)K, (int)lda, (int)ldb, tm, tn, e);
      else
        hipLaunchKernelGGL((k_qgemm_big<EPI, I32, F32X, false, true>), dim3(tm * tn), dim3(256), BIG_LDS, stream(), a,
                           bt, (int)M, (int)N, (int)K, (int)lda, (int)ldb, tm, tn, e);
      return;
    }
  }
  if constexpr (I32 && EPI != EPI_NULL) {
    if (e.b_packed == 2) {  // int4 nibble image (nqk_pack_b4)
      const int tm = (int)((M + 127) / 128);
      hipLaunchKernelGGL((k_qgemm_big<EPI, I32, F32X, true>), dim3(tm * tn), dim3(256), BIG_LDS, stream(), a, bt,
                         (int)M, (int)N, (int)K, (int)lda, (int)ldb, tm, tn, e);
      return;
    }
  }
  if (pp) {
    const int tm = (int)((M + 255) / 256);
    hipLaunchKernelGGL((k_qgemm_pp<EPI, I32, F32X>), dim3(tm * tn), dim3(512), PP_LDS, stream(), a, bt, (int)M,
                       (int)N, (int)K, (int)lda, (int)ldb, tm, tn, e);
  } else {
    const int tm = (int)((M + 127) / 128);
    hipLaunchKernelGGL((k_qgemm_big<EPI, I32, F32X>), dim3(tm * tn), dim3(256), BIG_LDS, stream(), a, bt, (int)M,
                       (int)N, (int)K, (int)lda, (int)ldb, tm, tn, e);
  }
}

static int g_last_gemm = -1;  // nqk_qgemm_last_kernel: 0 small tiles, 1 big tile, 2 ping-pong, 3 persistent, 4 k_pg,
                              // 5 k_pg 256 x 256 (WM = 2), 6 / 7 the same two with the GELU table
namespace nqk {
int pg_launch(int epi, const int8_t* a, const int8_t* bp, int64_t M, int64_t N, int64_t K, int64_t lda,
              const nqk_epilogue* p, bool f32x);  // nqk_pgemm.hip
}

static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}

template <int EPI, bool F32X, int NK, bool B4>
static void launch_proj(const int8_t* a, const int8_t* bp, int64_t M, int64_t N, int64_t lda, const Epi& e) {
  const int tn = (int)(N / GBN), nt = (int)((M + 255) / 256) * tn;
  // workgroups (one per CU): all CUs, or NQK_PROJ_CUS of them (diagnostic: a persistent
  // GEMM of one stream's half batch leaving CUs to the other stream)
  static const int cus = [] {
    const char* v = getenv("NQK_PROJ_CUS");
    const int n = v ? atoi(v) : 0;
    return n > 0 && n < num_cus() ? n : num_cus();
  }();
  const int grid = nt < cus ? nt : cus;
  const size_t shm = p2_lds(EPI, B4);
  hipLaunchKernelGGL((k_proj<EPI, F32X, NK, B4>), dim3(grid), dim3(512), shm, stream(), a, bp, (int)M, (int)N, (int)lda,
                     tn, nt, e);
}

static Epi make_epi(const nqk_epilogue* p) {
  Epi e{};
  e.zp_flags = p->zp_flags;
  e.zpa = p->zpa;
  e.zpb = p->zpb;
  e.kdim = p->kdim;
  e.colsum = p->col;
  e.group_cols = p->group_cols > 0 ? p->group_cols : 1;
  for (int g = 0; g < 3; ++g) {
    e.s_acc[g] = p->s_acc[g];
    e.s_out[g] = p->s_out[g];
    e.rs_out[g] = 1.0 / (double)p->s_out[g];
    e.zp_out[g] = (double)p->zp_out[g];
    e.out[g] = p->out[g];
  }
  e.bias = p->bias;
  e.resid = p->resid;
  e.div = p->div;
  e.rdiv = 1.0 / (double)p->div;
  e.add1 = p->add1;
  e.mul2 = p->mul2;
  e.tokens = p->tokens;
  e.heads = p->heads;
  e.hdim = p->hdim;
  e.ld_out = p->ld_out;
  e.lo = -__builtin_ldexp(1.0, p->bit_width - 1);
  e.hi = __builtin_ldexp(1.0, p->bit_width - 1) - 1.0;
  // the GELU filter's bound is proven for these constants only (nqk_selftest_gelu_filter)
  e.gelu_filter = p->div == 1.41421354f && p->add1 == 1.0f && p->mul2 == 0.5f && p->zp_out[0] >= -(1 << 20) &&
                  p->zp_out[0] <= (1 << 20) && __builtin_fabsf(p->s_out[0]) >= 0x1p-60f &&
                  __builtin_fabsf(p->s_out[0]) <= 0x1p20f && !(getenv("NQK_NO_GELU_FILTER"));
  for (int g = 0; g < 3; ++g) {
    e.rsf[g] = (p->s_out[g] != 0.0f) ? (float)(1.0 / (double)p->s_out[g]) : 0.0f;
    e.zpf[g] = (float)p->zp_out[g];
  }
  // GELU filter error in units of t: |gelu_fast - gelu| <= GELU_REL |h| + GELU_ABS, and
  // the product t = y * rsf adds |t| 2^-22 <= |h| |1/s| 2^-21.9 (|gelu(h)| <= |h|;
  // 0x1.13p-22 > 2^-21.9); 2 % margin on 1/s
  const double ars = __builtin_fabs(1.0 / (double)p->s_out[0]) * 1.02;
  e.g_rel = (float)(((double)GELU_REL + 0x1.13p-22) * ars);
  e.g_abs = (float)(GELU_ABS * ars) + 0x1p-100f;
  // |tf - r| + |h| g_rel + g_abs < 0.5 tested as RN(|h| g_rel + |tf - r|) < g_lim: a
  // rounded-down sum below g_lim = (0.5 - g_abs)(1 - 2^-22) keeps the exact one below
  // 0.5 - g_abs
  e.g_lim = (float)((0.5 - (double)e.g_abs) * (1.0 - 0x1p-22));
  e.b_packed = p->b_packed;
  e.colterm = p->colterm;
  e.lof = (float)e.lo;
  e.hif = (float)e.hi;
  e.xcds = [] {
    static int n = 0;
    if (n == 0) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeNumberOfXccs, dev) != hipSuccess ||
          n <= 0)
        n = 8;
    }
    return n;
  }();
  e.ln_g = p->ln_gamma;
  e.ln_b = p->ln_beta;
  e.ln_out = p->ln_out;
  e.ln_eps = p->ln_eps;
  if (p->ln_out != nullptr) {
    e.ln_rs = 1.0 / (double)p->ln_scale;
    e.ln_zp = (double)p->ln_zp;
    e.ln_lo = e.lo;
    e.ln_hi = e.hi;
    // nqk_ln_quant's conditions for the magic-number quantize (NQK_LN_F64Q=1 keeps the f64 chain)
    e.ln_mq = p->bit_width >= 1 && p->bit_width <= 8 && p->ln_zp >= -(1 << 20) && p->ln_zp <= (1 << 20) &&
              !getenv("NQK_LN_F64Q");
    e.ln_q = LnQ{(float)(e.lo - (double)p->ln_zp), (float)(e.hi - (double)p->ln_zp), 0x1.8p23f + (float)p->ln_zp};
  }
  return e;
}

static int64_t pack_b_bytes(int64_t N, int64_t K) { return (N + GBN - 1) / GBN * GBN * K; }

extern "C" int nqk_pack_b(const int8_t* bt, int8_t* out, int64_t N, int64_t K, int64_t ldb) {
  if (N <= 0 || K <= 0) return 0;
  if (K % GBK) return fail("nqk_pack_b: K must be a multiple of 64");
  if ((((uintptr_t)bt) & 15) || (ldb & 15) || (((uintptr_t)out) & 15)) return fail("nqk_pack_b: unaligned operand");
  const int64_t chunks = pack_b_bytes(N, K) / 16;
  hipLaunchKernelGGL(k_pack_b, dim3(grid_for(chunks)), dim3(kThreads), 0, stream(), bt, out, N, K, ldb, chunks);
  return launch_status("nqk_pack_b");
}

extern "C" int nqk_pack_b4(const int8_t* bt, uint8_t* out, int64_t N, int64_t K, int64_t ldb) {
  if (N <= 0 || K <= 0) return 0;
  if (K % GBK) return fail("nqk_pack_b4: K must be a multiple of 64");
  const int64_t total = pack_b_bytes(N, K) / 2;
  hipLaunchKernelGGL(k_pack_b4, dim3(grid_for(total)), dim3(kThreads), 0, stream(), bt, out, N, K, ldb, total);
  return launch_status("nqk_pack_b4");
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
  if (M > (1 << 30) || N > (1 << 30) || K > (1 << 30) || lda > (1 << 30) || ldb > (1 << 30))
    return fail("nqk_qgemm_fused: dimensions beyond int32");
  if (params->zp_flags & (NQK_ZP_SCALAR | NQK_ZP_FULL))
    return fail("nqk_qgemm_fused: only row / column / K-constant zero-point terms");
  const Epi e = make_epi(params);
  // int32 zero-point algebra when |acc| + |row term| + |col term| + |K term| < 2^31
  const double za = (double)(params->zpa < 0 ? -params->zpa : params->zpa);
  const double zb = (double)(params->zpb < 0 ? -params->zpb : params->zpb);
  const double kk = (double)(params->kdim > K ? params->kdim : K);
  const double bound = 16384.0 * kk + 128.0 * kk * (za + zb) + za * zb * kk;
  const bool i32 = bound < 2147483647.0 * 0.98;
  const bool pp = gemm_pingpong();
  const bool big = batch == 1 && (K % (pp ? GBK : GST * GBK)) == 0 && K > 0 && (N % 4) == 0 && params->zp_flags == NQK_ZP_COL &&
                   params->col != nullptr && (epi != EPI_QKV || (params->hdim % 4 == 0 && params->group_cols % 4 == 0)) &&
                   (epi == EPI_QKV || epi == EPI_RESID || epi == EPI_GELU || epi == EPI_NULL);
  // staged epilogue stores 4 columns at once: 16-byte (f32) / 4-byte (int8) aligned outputs
  auto al = [](const void* q, uintptr_t n) { return q == nullptr || (((uintptr_t)q) & (n - 1)) == 0; };
  const bool aligned = (epi == EPI_RESID) ? (al(params->out[0], 16) && al(params->resid, 16))
                                          : (al(params->out[0], 4) && al(params->out[1], 4) && al(params->out[2], 4));
  auto normal = [](float x) { return __builtin_fabsf(x) >= 0x1p-100f && __builtin_fabsf(x) <= 0x1p100f; };
  bool scales_ok = normal(params->s_out[0]) || epi == EPI_RESID || epi == EPI_NULL;
  if (epi == EPI_QKV) scales_ok = normal(params->s_out[0]) && normal(params->s_out[1]) && normal(params->s_out[2]);
  if (epi == EPI_GELU) scales_ok = scales_ok && normal(params->div);
  if (params->b_packed == 2 && (!i32 || epi == EPI_NULL))
    return fail("nqk_qgemm_fused: int4 packed weights need the int32 zero-point algebra");
  if (params->ln_out != nullptr) {
    // the fused LayerNorm: the one-tile-per-workgroup kernel with whole 192-column rows per tile
    if (!(epi == EPI_RESID && N == 192 && big && aligned && params->ln_gamma && params->ln_beta &&
          (((uintptr_t)params->ln_gamma | (uintptr_t)params->ln_beta) & 15) == 0 && (((uintptr_t)params->ln_out) & 3) == 0 &&
          __builtin_fabsf(params->ln_scale) >= 0x1p-100f && __builtin_fabsf(params->ln_scale) <= 0x1p100f &&
          !pp && !getenv("NQK_PROJ_RESID")))
      return fail("nqk_qgemm_fused: a fused LayerNorm needs the residual epilogue at N = 192 on the big-tile path "
                  "(16-byte aligned gamma / beta, a normal ln_scale)");
  }
  if (params->b_packed && !(big && aligned && scales_ok && (K % (GST * GBK)) == 0))
    return fail("nqk_qgemm_fused: a packed B operand needs the big-tile path (K % 192 == 0, N % 4 == 0, "
                "COL zero-point term, aligned outputs)");
  if (big && aligned && scales_ok) {
    // f32 epilogue arithmetic when every |acc - col term| < 2^24 (int8 operands:
    // |acc| <= 2^14 K) and the output zero points are exact in f32 with room to spare
    const double cmax = params->col_absmax > 0 ? (double)params->col_absmax : 128.0 * (double)K;
    // |sum_k a b| <= 2^14 K for int8 operands, or 128 max_n sum_k |b| when the host gave the
    // weights' largest column L1 norm (|a| <= 128)
    const double abound = params->col_l1max > 0 && !getenv("NQK_NO_L1")
                              ? std::min(16384.0 * (double)K, 128.0 * (double)params->col_l1max)
                              : 16384.0 * (double)K;
    const int ng = epi == EPI_QKV ? 3 : 1;
    bool zp_small = true;
    for (int g = 0; g < ng; ++g) zp_small = zp_small && params->zp_out[g] >= -(1 << 20) && params->zp_out[g] <= (1 << 20);
    const bool f32x = i32 && (epi == EPI_QKV || (epi == EPI_GELU && e.gelu_filter)) && zp_small &&
                      abound + cmax * za < 16777216.0 && !getenv("NQK_NO_F32X");
    const bool use_pp = pp && !params->b_packed;
    // the persistent 16x16x64 GEMM (nqk_pgemm.hip) where it takes the case (never with a fused
    // LayerNorm: its residual epilogue needs whole 256-column tiles)
    if (params->bt_pg != nullptr && params->ln_out == nullptr) {
      const bool f32x_r = i32 && epi == EPI_RESID && abound + cmax * za < 16777216.0 && !getenv("NQK_NO_F32X");
      const int rc = pg_launch(epi, a, params->bt_pg, M, N, K, lda, params, f32x || f32x_r);
      if (rc < 0) return rc;
      if (rc > 0) {
        g_last_gemm = rc;
        return 0;
      }
    }
    // the persistent 256 x 256 kernel where it takes the shape: QKV by default; FFN-up +
    // GELU with NQK_PROJ_GELU=1 and the residual epilogues with NQK_PROJ_RESID=1 (faster
    // alone, not inside the two-stream forward, DESIGN.md "Projection GEMM variants");
    // NQK_NO_PROJ=1 keeps the one-tile-per-workgroup kernel everywhere
    const bool f32x_r = i32 && epi == EPI_RESID && abound + cmax * za < 16777216.0 && !getenv("NQK_NO_F32X");
    const bool proj_shape = params->b_packed && i32 && params->colterm != nullptr && M >= 256 && (M % 256 == 0 || epi != EPI_RESID) && N % GBN == 0 &&
                            (K == 768 || K == 3072) && (double)M * N * 4.0 < 4294967295.0 && (double)M * lda < 4294967295.0 &&
                            !getenv("NQK_NO_PROJ") &&
                            (epi == EPI_RESID || (al(params->out[0], 16) && al(params->out[1], 16) && al(params->out[2], 16))) &&
                            ((epi == EPI_RESID && !(params->b_packed == 2 && K == 768) && getenv("NQK_PROJ_RESID")) ||
                             (f32x && K == 768 &&
                              ((epi == EPI_GELU && getenv("NQK_PROJ_GELU")) ||
                               (epi == EPI_QKV && params->tokens >= 64 && params->hdim == 64 && params->group_cols % 128 == 0 &&
                                (double)M * params->heads * params->hdim < 2147483647.0))));
    if (proj_shape) {
      const bool b4 = params->b_packed == 2;
      const int key = epi * 8 + (b4 ? 4 : 0) + (K == 3072 ? 2 : 0) + (f32x || f32x_r ? 1 : 0);
      switch (key) {
#define LP(E, B, NKV, X) case E * 8 + (B ? 4 : 0) + (NKV == 48 ? 2 : 0) + (X ? 1 : 0): \
        launch_proj<E, X, NKV, B>(a, bt, M, N, lda, e); break;
        LP(EPI_QKV, false, 12, true) LP(EPI_QKV, true, 12, true)
        LP(EPI_GELU, false, 12, true) LP(EPI_GELU, true, 12, true)
        LP(EPI_RESID, false, 12, true) LP(EPI_RESID, false, 12, false)
        LP(EPI_RESID, false, 48, false) LP(EPI_RESID, true, 48, false)
        LP(EPI_RESID, false, 48, true) LP(EPI_RESID, true, 48, true)
#undef LP
        default: return fail("nqk_qgemm_fused: no persistent kernel for this case");
      }
      g_last_gemm = 3;
      return launch_status("nqk_qgemm_fused(proj)");
    }
    switch (epi * 3 + (f32x ? 2 : (i32 ? 1 : 0))) {
#define LB(E) \
      case E * 3 + 0: launch_big<E, false, false>(use_pp, a, bt, M, N, K, lda, ldb, e); break; \
      case E * 3 + 1: launch_big<E, true, false>(use_pp, a, bt, M, N, K, lda, ldb, e); break;
      LB(EPI_QKV) LB(EPI_RESID) LB(EPI_GELU) LB(EPI_NULL)
#undef LB
      case EPI_QKV * 3 + 2: launch_big<EPI_QKV, true, true>(use_pp, a, bt, M, N, K, lda, ldb, e); break;
      case EPI_GELU * 3 + 2: launch_big<EPI_GELU, true, true>(use_pp, a, bt, M, N, K, lda, ldb, e); break;
      default: return fail("nqk_qgemm_fused: no big-tile kernel for this epilogue");
    }
    g_last_gemm = use_pp ? 2 : 1;
    return launch_status("nqk_qgemm_fused(big)");
  }
  g_last_gemm = 0;
  const int tiles_m = (int)((M + FBM - 1) / FBM), tiles_n = (int)((N + FBN - 1) / FBN);
  const BatchMap m = batch_map(bmap);
  const dim3 grid(tiles_m * tiles_n, 1, (unsigned)batch);
  switch (epi) {
#define L(E) case E: if (i32) hipLaunchKernelGGL((k_qgemm_epi<E, true>), grid, dim3(256), 0, stream(), a, bt, (int)M, \
                                 (int)N, (int)K, (int)lda, (int)ldb, m, a_mat_stride, b_mat_stride, tiles_m, tiles_n, e); \
                      else hipLaunchKernelGGL((k_qgemm_epi<E, false>), grid, dim3(256), 0, stream(), a, bt, (int)M, \
                                 (int)N, (int)K, (int)lda, (int)ldb, m, a_mat_stride, b_mat_stride, tiles_m, tiles_n, e); break;
    L(EPI_QKV) L(EPI_SCORES) L(EPI_PV) L(EPI_RESID) L(EPI_GELU) L(EPI_NULL)
#undef L
    default: return fail("nqk_qgemm_fused: unknown epilogue");
  }
  return launch_status("nqk_qgemm_fused");
}

extern "C" int nqk_qgemm_last_kernel(void) { return g_last_gemm; }

extern "C" int nqk_ln_quant(const float* x, const float* gamma, const float* beta, int8_t* out, int64_t rows,
                            int64_t cols, float eps, float scale, int64_t zp, int bit_width) {
  if (rows <= 0) return 0;
  PwPlan p;
  if (row_plan(cols, p)) return -1;
  const double lo = -__builtin_ldexp(1.0, bit_width - 1), hi = __builtin_ldexp(1.0, bit_width - 1) - 1.0;
  // register-tree kernel: balanced plan of equal leaves of 96 columns (768 = ViT-Base,
  // 192 = ViT-Tiny, 384 = ViT-Small); the quotient t = y / s only feeds rint(zp + t), so
  // the RN64(1/s) product needs no subnormal fallback (see nqk_attn.hip div_rc_w)
  bool eq = p.balanced && p.nleaf >= 1;
  for (int l = 0; eq && l < p.nleaf; ++l) eq = p.len[l] == 96;
  const bool snormal = __builtin_fabsf(scale) >= 0x1p-100f && __builtin_fabsf(scale) <= 0x1p100f;
  const bool al = ((((uintptr_t)x) | ((uintptr_t)gamma) | ((uintptr_t)beta)) & 15) == 0 && (((uintptr_t)out) & 3) == 0;
  if (eq && snormal && al && (p.nleaf == 8 || p.nleaf == 4 || p.nleaf == 2)) {
    const double rs = 1.0 / (double)scale;
    // the magic-number quantize (ln_quant4) where it is exact; NQK_LN_F64Q=1 keeps the f64 chain
    const bool mq = bit_width >= 1 && bit_width <= 8 && zp >= -(1 << 20) && zp <= (1 << 20) && !getenv("NQK_LN_F64Q");
    const LnQ lq{(float)(lo - (double)zp), (float)(hi - (double)zp), 0x1.8p23f + (float)zp};
    const int64_t lanes = rows * p.nleaf * 2;
    const unsigned grid = (unsigned)((lanes + 255) / 256);
    // rows through LDS: linear 1 KiB loads / stores per wave (the LDS-DMA form addresses x by 32-bit
    // buffer offsets: larger inputs take the register-tree kernel)
    const bool dma_ok = !NQK_LN_DMA || rows * cols * 4 < (int64_t(1) << 31);
    const char* pe = getenv("NQK_LN_PERS");
    if (NQK_LN_DMA && dma_ok && pe && atoi(pe) > 0 && mq && !getenv("NQK_LN_REG")) {
      // persistent double-buffered form: NQK_LN_PERS waves per CU (1-wave workgroups, 24 KiB each)
      const int64_t ngroups = (rows + 32 / p.nleaf - 1) / (32 / p.nleaf);
      const int64_t w = std::min<int64_t>(ngroups, (int64_t)std::min(6, atoi(pe)) * num_cus());
      const int lb = 2 * (32 / p.nleaf) * p.nleaf * 96 * 4;
#define LNP(NLV)                                                                                                 \
  hipLaunchKernelGGL((k_ln_quant_pers<NLV, true>), dim3((unsigned)w), dim3(64), lb, stream(), x, gamma, beta, out, \
                     rows, eps, rs, (double)zp, lo, hi, lq)
      switch (p.nleaf) {
        case 8: LNP(8); break;
        case 4: LNP(4); break;
        default: LNP(2); break;
      }
#undef LNP
      return launch_status("nqk_ln_quant(pers)");
    }
    if (!getenv("NQK_LN_REG") && dma_ok) {
      // WPB waves of 64 / (2 nleaf) rows per workgroup; NQK_LN_WPB = 1 / 2 / 4 (default: 4 for 8 leaves,
      // 1 for fewer — ViT-Ti's 192-column rows +1.3 % whole-bench, ViT-Base's -0.5 %, within noise:
      // profiles/r05_ln_variants.txt)
      const char* we = getenv("NQK_LN_WPB");
      const int wpb = we ? (atoi(we) == 1 ? 1 : atoi(we) == 2 ? 2 : 4) : (p.nleaf == 8 ? 4 : 1);
      const int64_t rpw = wpb * 32 / p.nleaf;
      const unsigned gl = (unsigned)((rows + rpw - 1) / rpw);
#define LNL2(NLV, W)                                                                                               \
  if (mq)                                                                                                          \
    hipLaunchKernelGGL((k_ln_quant_lds<NLV, true, W>), dim3(gl), dim3(64 * W), ln_lds_bytes(NLV, W), stream(), x,  \
                       gamma, beta, out, rows, eps, scale, rs, (double)zp, lo, hi, lq);                            \
  else                                                                                                             \
    hipLaunchKernelGGL((k_ln_quant_lds<NLV, false, W>), dim3(gl), dim3(64 * W), ln_lds_bytes(NLV, W), stream(), x, \
                       gamma, beta, out, rows, eps, scale, rs, (double)zp, lo, hi, lq)
#define LNL(NLV)                \
  if (wpb == 1) LNL2(NLV, 1);   \
  else if (wpb == 2) LNL2(NLV, 2); \
  else LNL2(NLV, 4)
      switch (p.nleaf) {
        case 8: LNL(8); break;
        case 4: LNL(4); break;
        default: LNL(2); break;
      }
#undef LNL2
#undef LNL
      return launch_status("nqk_ln_quant(lds)");
    }
    switch (p.nleaf) {
      case 8: hipLaunchKernelGGL((k_ln_quant_reg<8>), dim3(grid), dim3(256), 0, stream(), x, gamma, beta, out, rows,
                                 eps, scale, rs, (double)zp, lo, hi, lq); break;
      case 4: hipLaunchKernelGGL((k_ln_quant_reg<4>), dim3(grid), dim3(256), 0, stream(), x, gamma, beta, out, rows,
                                 eps, scale, rs, (double)zp, lo, hi, lq); break;
      default: hipLaunchKernelGGL((k_ln_quant_reg<2>), dim3(grid), dim3(256), 0, stream(), x, gamma, beta, out,
                                  rows, eps, scale, rs, (double)zp, lo, hi, lq); break;
    }
    return launch_status("nqk_ln_quant(reg)");
  }
  const int64_t slice = (int64_t)(row_smem(cols) / sizeof(float) + 3) / 4 * 4;
  const unsigned grid = (unsigned)(((rows + 3) / 4) < 65536 * 4 ? (rows + 3) / 4 : 65536 * 4);
  hipLaunchKernelGGL(k_ln_quant, dim3(grid), dim3(256), 4 * slice * sizeof(float), stream(), x, gamma, beta, out,
                     rows, cols, eps, p, scale, (double)zp, lo, hi, slice);
  return launch_status("nqk_ln_quant");
}

extern "C" int nqk_softmax_quant(const float* x, int8_t* out, int64_t* rowsum, int64_t rows, int64_t cols,
                                 int64_t ldo, float scale, int64_t zp, int bit_width) {
  if (rows <= 0) return 0;
  if (ldo < cols) return fail("nqk_softmax_quant: ldo < cols");
  PwPlan p;
  if (row_plan(cols, p)) return -1;
  const double lo = -__builtin_ldexp(1.0, bit_width - 1), hi = __builtin_ldexp(1.0, bit_width - 1) - 1.0;
  const int64_t slice = (int64_t)(row_smem(cols) / sizeof(float) + 3) / 4 * 4;
  const unsigned grid = (unsigned)(((rows + 3) / 4) < 65536 * 4 ? (rows + 3) / 4 : 65536 * 4);
  hipLaunchKernelGGL(k_softmax_quant, dim3(grid), dim3(256), 4 * slice * sizeof(float), stream(), x, out, rowsum,
                     rows, cols, ldo, p, scale, (double)zp, lo, hi, slice);
  return launch_status("nqk_softmax_quant");
}

extern "C" int nqk_transpose_pad_i8(const int8_t* src, int8_t* dst, int64_t* rowsum, int64_t nb, int64_t R,
                                    int64_t C, int64_t Rp) {
  if (nb <= 0 || R <= 0 || C <= 0) return 0;
  if (Rp < R || nb > 65535) return fail("nqk_transpose_pad_i8: bad shape");
  const dim3 grid((unsigned)((C + 63) / 64), (unsigned)nb, 1);
  hipLaunchKernelGGL(k_transpose_pad, grid, dim3(256), 0, stream(), src, dst, rowsum, nb, R, C, Rp);
  return launch_status("nqk_transpose_pad_i8");
}
