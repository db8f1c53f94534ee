// Fused self-attention of one quantized encoder layer (QModel.__call__, model.py:486-565,
// on the ViT attention block: MatMul(Q, K^T) -> Div -> Softmax -> MatMul(P, V) ->
// Transpose -> Reshape -> quantize for the output projection).
//
// One workgroup per (image, head); the scores never leave the CU:
//   S   = dequant(Q K^T - zero-point term) / div    v_mfma_i32_32x32x32_i8, K from LDS
//   P   = quantize(softmax(S))                      NumPy exp, NumPy pairwise row sums
//   ctx = quantize(dequant(P V - zero-point term))  v_mfma_i32_32x32x32_i8, V^T from LDS
// Every element goes through exactly the float / integer operations of the node loop
// (same as nqk_qgemm_fused EPI_SCORES + nqk_softmax_quant + EPI_PV), so the context is
// bit-identical to the unfused chain; only the f32 scores (B*H*T*T*4 bytes) and the
// int8 probabilities stop travelling through HBM.
//
// LDS (T = 197: NT = 7 score tiles of 32 columns):
//   Ks   [NT*32][64]     int8, 16-byte chunks XOR-swizzled (conflict-free A reads)
//   Vt   [64][PST]       int8 V^T, zero padded to NT*32 tokens; PST = NT*32 + 16, and dims
//                        16c .. 16c + 15 shifted by 64 c bytes (vt_row): conflict-free dword
//                        writes of the transposed staging
//   colK [NT*32], colV [64]   int32 zero-point column terms
// 30 KiB per workgroup: three workgroups (12 waves) per CU; everything else is in VGPRs.
#include <type_traits>

#include "nqk_common.h"
#include "nqk_numerics.h"

#ifndef NQK_ATTN_DIAG
#define NQK_ATTN_DIAG 0
#endif
#ifndef NQK_ATTN_EXPW
#define NQK_ATTN_EXPW 4
#endif
#ifndef NQK_ATTN_PK
#define NQK_ATTN_PK 1  // FAST path on element pairs with packed f32 arithmetic (0: scalar, for A/B)
#endif
#ifndef NQK_ATTN_PQ2
#define NQK_ATTN_PQ2 1  // 1: P quantize without the clamp when no row can reach it, by fma rounding
#endif
#ifndef NQK_ATTN_EXP2
#define NQK_ATTN_EXP2 1  // 1: rows whose arguments all lie in [-86.5, 0] take np_expf_safe2
#endif
#ifndef NQK_ATTN_PREL
#define NQK_ATTN_PREL 1  // 1: P filter margin per element (|tf| 2^-21) instead of the row's (kpf 2^-20)
#endif
// P filter margins (NQK_ATTN_PREL), per element: the reference's t = RN(RN(e / tot) / s_p) is within
// (2u + u^2)|x| of x = e / (tot s_p) (u = 2^-24), kpf = RN(rtot rs_p) within (u + 3 2^-53)|x| / e.
// Clamp-free path: r = rint(e kpf) exactly, so |t - e kpf| <= 3.0001 u |x| <= 4.5002 u |r| for |r| >= 1
// (|x| <= |r| + 0.5 + ...; r = 0: 1.5 u, under the limit's 2 u): margin 4.75 u |r|.
// Clamped path: tf = RN(e kpf) adds u, |t - tf| <= 4.0001 u |x| <= 4.002 u |tf|: margin 4.125 u |tf|.
// Both then pass only below 0.5 - 2u, which also takes dd's and the measure's own roundings
// (0.25 u each).  (Round 3 used 8 u for both: about twice the fallbacks.)
#ifndef NQK_ATTN_PM_R
#define NQK_ATTN_PM_R 0x1.3p-22f
#endif
#ifndef NQK_ATTN_PM_T
#define NQK_ATTN_PM_T 0x1.08p-22f
#endif
#ifndef NQK_ATTN_PKL
#define NQK_ATTN_PKL 0  // 1: clamped path tf = RN(e kpf + RN(e kpl)) (kpf + kpl = the double product):
                        // |t - tf| <= 3.001 u |tf|, margin 3.125 u |tf| (A/B variant)
#endif
#ifndef NQK_ATTN_PSUM
#define NQK_ATTN_PSUM 1  // 1: the pairwise-sum accumulators as packed pairs (v_pk_add_f32)
#endif

namespace nqk {
#if (NQK_ATTN_DIAG & 128)
// diagnostic builds: per launch, wave-tiles that took [0] the clamped exp (some argument below
// -86.5), [1] the clamped P quantize, [2] the P exact fallback, [3] the context exact fallback
__device__ unsigned long long g_attn_stats[4];
extern "C" int nqk_attn_diag_stats(unsigned long long* out, int reset) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_attn_stats), 4 * sizeof(unsigned long long));
  const unsigned long long z[4] = {0, 0, 0, 0};
  if (reset) (void)hipMemcpyToSymbol(HIP_SYMBOL(g_attn_stats), z, sizeof(z));
  return 0;
}
#define NQK_ATTN_COUNT(i) \
  do { if ((threadIdx.x & 63) == 0) atomicAdd(&g_attn_stats[i], 1ull); } while (0)
#else
#define NQK_ATTN_COUNT(i) do { } while (0)
#endif
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

struct AttnArgs {
  int T, H, ld_out, EST, PST, n2;
  int zq, zk, zp, zv;  // zero points (host-checked: every int32 intermediate is exact)
  int kq, kp;          // zq*zk*64, zp*zv*T
  float s_qk, div, s_p, s_pv, s_ctx;
  double rdiv, rs_p, zp_p, rs_ctx, zp_ctx, lo, hi;
  float inv_div, rs_ctx_f, zp_p_f, zp_ctx_f, lo_f, hi_f;  // FAST path constants
  float s_qkd;  // s_qk / div (div a power of two, s_qk / div in [2^-100, 2^100]: exact)
};

__device__ __forceinline__ int swz64a(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4); }

__device__ __forceinline__ int sum16a(v4i c) {
  int s = __builtin_amdgcn_sdot4(c[0], 0x01010101, 0, false);
  s = __builtin_amdgcn_sdot4(c[1], 0x01010101, s, false);
  s = __builtin_amdgcn_sdot4(c[2], 0x01010101, s, false);
  return __builtin_amdgcn_sdot4(c[3], 0x01010101, s, false);
}

// RN32(x / c) from rc = RN64(1/c): x * rc is within 2^-52 (relative) of x / c while a
// quotient of two floats is at least 2^-48 away from every float32 rounding midpoint,
// except for exact midpoints in the subnormal range (|x / c| < 2^-126).  Here every
// such quotient only feeds a rounding that cannot see it: (a) the scores y = d / div
// enter exp(y - max), where a |y| < 2^-125 either vanishes next to max or leaves an
// argument |x| < 2^-24 whose NumPy exp is exactly 1; (b) p = e / sum and t = p / s_p
// enter rint(zp + t), and |t| < 2^-25 (host check: s >= 2^-100) rounds to zp for any
// candidate.  So no exact-division fallback is needed (nqk_fused.hip keeps one).
__device__ __forceinline__ float div_rc_w(float x, double rc) { return (float)((double)x * rc); }

__device__ __forceinline__ int quant_w(float x, float s, double rs, double zp, double lo, double hi) {
  const float t = div_rc_w(x, rs);
  const double u = zp + (double)t;
  return (int)__builtin_rint(__builtin_fmin(__builtin_fmax(u, lo), hi));
}

// value of the partner lane (lane ^ 32): one v_permlane32_swap + a select
__device__ __forceinline__ int xor32i(int x) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return (threadIdx.x & 32) ? (int)r[0] : (int)r[1];
}
__device__ __forceinline__ float xor32f(float x) { return __int_as_float(xor32i(__float_as_int(x))); }

// The scores are computed transposed, S^T = K Q^T (A = K rows from LDS, B = Q rows from
// HBM), so a lane holds one query row: lane (r32, h) has S[m0 + r32][n] for the 112
// (NT = 7) key positions n = 32c + 8q + 4h + j' (c < NT, q < 4, j' < 4) of its half
// and the partner lane (lane ^ 32) has the other half.  Row max, NumPy's pairwise sum
// (accumulator j = n % 8 lives in half j / 4; chains in increasing n), division and
// quantize are all in-lane; one cross-half exchange combines them.  The context is
// computed transposed as well (O^T = V^T P^T), so each lane stores 4 consecutive
// head dimensions of its query row at once.
// FAST: the dequantized scores / context are formed in f32 (exact: every |acc - term| <
// 2^24, host-checked), the scores Div is a power of two (an exact f32 multiply), and the
// P / context quantizations go through a rounding filter (t from one f32 product, exact
// chain for any element within the product's error bound of a rounding boundary).
#ifndef NQK_ATTN_WPE
#define NQK_ATTN_WPE 0  // diagnostic builds: amdgpu_waves_per_eu(NQK_ATTN_WPE) occupancy target
#endif
#if NQK_ATTN_WPE
#define NQK_ATTN_OCC __attribute__((amdgpu_waves_per_eu(NQK_ATTN_WPE, NQK_ATTN_WPE)))
#else
#define NQK_ATTN_OCC
#endif
// three workgroups (12 waves) per CU: the register budget is 168 per lane (the exp /
// quantize phases are VALU-issue-bound, so the third wave per SIMD pays for a few spills)
#ifndef NQK_ATTN_MINB
#define NQK_ATTN_MINB 3
#endif
#ifndef NQK_ATTN_TAIL
#define NQK_ATTN_TAIL 0  // 1: the last row tile of T = 193 .. 200 by the row-parallel path (round 5; measured no faster,
                         // profiles/r05_attn_tail_dropped.txt: opt-in build)
#endif
constexpr int ATTN_TSTR = 232;
// the row-parallel tail path applies: the shipped FAST configuration, T > 128 with at most 8 real
// rows in the last tile and both pairwise-sum leaves of equal group counts (T = 193 .. 200)
template <int NT, int TC, bool FAST>
constexpr bool attn_tail() {
  constexpr int TR = TC > 0 ? TC - 32 * (NT - 1) : 32;
  constexpr int N2 = TC > 128 ? TC / 2 - (TC / 2) % 8 : 0;
  return NQK_ATTN_TAIL && FAST && NQK_ATTN_PK && NQK_ATTN_EXP2 && NQK_ATTN_PQ2 && NQK_ATTN_PREL && !NQK_ATTN_PKL &&
         NQK_ATTN_DIAG == 0 && TC > 128 && TR >= 1 && TR <= 8 && N2 / 8 == (TC - N2) / 8;
}
template <int NT, int TC, bool FAST>
constexpr size_t attn_tail_lds() {
  return attn_tail<NT, TC, FAST>() ? (size_t)(TC - 32 * (NT - 1)) * (ATTN_TSTR * 4 + NT * 32) : 0;
}
template <int NT, int TC, bool FAST>  // TC: compile-time token count (0: runtime a.T)
__global__ void __launch_bounds__(256, NQK_ATTN_MINB) NQK_ATTN_OCC
k_attention(const int8_t* __restrict__ Qg, const int8_t* __restrict__ Kg, const int8_t* __restrict__ Vg,
            int8_t* __restrict__ ctx, AttnArgs a) {
  constexpr int TP = NT * 32;  // padded tokens (score columns / PV contraction)
  constexpr int G = TP / 8;    // 8-column groups of a score row
  // group qq of score tile c (columns c*32 + 8qq .. + 7 of both halves) past the last
  // token: known at compile time when the token count is
  auto pad_group = [](int c, int qq) constexpr { return TC > 0 && c * 32 + 8 * qq >= TC; };
  // NQK_ATTN_TAIL: the last row tile's TR real rows by the row-parallel path (below); its LDS: the
  // rows' scores tS [TR][TSTR] f32 (rows 8 banks apart for ds_read_b32) and P bytes tP [TR][TP]
  constexpr int TR = TC > 0 ? TC - 32 * (NT - 1) : 32;
  constexpr int N2 = TC > 128 ? TC / 2 - (TC / 2) % 8 : 0, NG0 = N2 / 8, NG1 = (TC - N2) / 8, NG = NG0 + NG1;
  constexpr int TL1 = TC - N2 - 8 * NG1;
  constexpr bool TAILR = attn_tail<NT, TC, FAST>();
  constexpr int TSTR = ATTN_TSTR;
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  const int T = TC ? TC : a.T, PST = TC ? NT * 32 + 16 : a.PST;
  int8_t* Ks = lds;
  int8_t* Vt = Ks + TP * 64;
  auto vt_row = [&](int d) { return d * PST + (d >> 4) * 64; };  // byte offset of V^T row d
  int* colK = reinterpret_cast<int*>(Vt + 64 * PST + 256);  // rowsum(K[n]) * zq - zq*zk*64
  int* colV = colK + TP;                              // colsum(V[:, d]) * zp - zp*zv*T
  float* const tS = reinterpret_cast<float*>(colV + 64);  // NQK_ATTN_TAIL scratch
  int8_t* const tP = reinterpret_cast<int8_t*>(tS + (TAILR ? TR * TSTR : 0));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bh = blockIdx.x;
  const int img = bh / a.H, head = bh - img * a.H;
  const int8_t* q = Qg + (int64_t)bh * T * 64;
  const int8_t* k = Kg + (int64_t)bh * T * 64;
  const int8_t* v = Vg + (int64_t)bh * T * 64;

  // ---- K (swizzled) and V^T (zero padded) into LDS, zero-point column terms
  for (int idx = tid; idx < TP * 4; idx += 256) {
    const int row = idx >> 2, ch = idx & 3;
    const v4i z = {0, 0, 0, 0};
    // (diagnostic 64: no K loads)
    const v4i kv = (row < T && (NQK_ATTN_DIAG & 64) == 0) ? *reinterpret_cast<const v4i*>(k + row * 64 + ch * 16) : z;
    *reinterpret_cast<v4i*>(Ks + swz64a(row, ch)) = kv;
  }
  // V^T by blocks of 4 tokens x 16 dims: four 16-B row loads, a 4 x 4 byte transpose per
  // dword column (v_perm_b32), sixteen 4-byte writes of 4 consecutive tokens of one dim
  // (consecutive lanes: consecutive token blocks of one 16-dim chunk)
  for (int blk = tid; blk < TP; blk += 256) {  // TP / 4 token blocks x 4 dim chunks
    const int c = blk / (TP / 4), rb = blk - c * (TP / 4);
    v4i w[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int tok = 4 * rb + r;
      // (diagnostic 64: no K / V loads; 4096: no V loads)
      w[r] = (tok < T && (NQK_ATTN_DIAG & (64 | 4096)) == 0) ? *reinterpret_cast<const v4i*>(v + tok * 64 + c * 16)
                                                               : v4i{0, 0, 0, 0};
    }
#if NQK_ATTN_DIAG & 1  // diagnostic builds only (wrong results): 1 = V^T staging skipped, 2 = exp
                      // replaced by one add, 4 = P quantize replaced by a convert
    if (blk == 0) Vt[0] = (int8_t)(w[0][0] ^ w[1][1] ^ w[2][2] ^ w[3][3]);
#else
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      // out_k = [w0.byte k, w1.byte k, w2.byte k, w3.byte k] of dword column g
      const uint32_t lo01 = __builtin_amdgcn_perm((uint32_t)w[1][g], (uint32_t)w[0][g], 0x05010400u);
      const uint32_t hi01 = __builtin_amdgcn_perm((uint32_t)w[1][g], (uint32_t)w[0][g], 0x07030602u);
      const uint32_t lo23 = __builtin_amdgcn_perm((uint32_t)w[3][g], (uint32_t)w[2][g], 0x05010400u);
      const uint32_t hi23 = __builtin_amdgcn_perm((uint32_t)w[3][g], (uint32_t)w[2][g], 0x07030602u);
      const uint32_t o[4] = {__builtin_amdgcn_perm(lo23, lo01, 0x05040100u), __builtin_amdgcn_perm(lo23, lo01, 0x07060302u),
                             __builtin_amdgcn_perm(hi23, hi01, 0x05040100u), __builtin_amdgcn_perm(hi23, hi01, 0x07060302u)};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) *reinterpret_cast<uint32_t*>(Vt + vt_row(16 * c + 4 * g + kk) + 4 * rb) = o[kk];
    }
#endif
  }
  if constexpr ((NQK_ATTN_DIAG & 1024) == 0) __syncthreads();  // (diagnostic 1024: no workgroup barriers)
  for (int row = tid; row < TP; row += 256) {
    const v4i* kr = reinterpret_cast<const v4i*>(Ks + row * 64);
    colK[row] = (sum16a(kr[0]) + sum16a(kr[1]) + sum16a(kr[2]) + sum16a(kr[3])) * a.zq - a.kq;
  }
  {
    const int d = tid >> 2, part = tid & 3;
    int s = 0;
    for (int c = part; c < NT * 2; c += 4) s += sum16a(*reinterpret_cast<const v4i*>(Vt + vt_row(d) + c * 16));
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (part == 0) colV[d] = s * a.zp - a.kp;
  }
  if constexpr ((NQK_ATTN_DIAG & 1024) == 0) __syncthreads();

  // pairwise-sum plan of a row (uniform): leaf l = [s0_l, s0_l + L_l), main part of
  // ng_l whole 8-groups from group g0_l, then a tail of tl_l < 8 columns
  const int n2 = TC ? (TC > 128 ? (TC / 2) - (TC / 2) % 8 : 0) : a.n2;
  const int L0 = n2 ? n2 : T, L1 = n2 ? T - n2 : 0;
  const int g0_0 = 0, g0_1 = n2 >> 3;
  const int ng0 = L0 >= 8 ? L0 >> 3 : 0, ng1 = L1 >= 8 ? L1 >> 3 : 0;
  const int tl0 = L0 - 8 * ng0, tl1 = L1 - 8 * ng1;
  const int gt0 = g0_0 + ng0, gt1 = g0_1 + ng1;  // tail groups

  const int r32 = lane & 31, h = lane >> 5;
  // (NT = 7 row tiles on 4 waves: wave 3 holds one.  Rotating that light wave over the
  // waves by blockIdx measured 2 % slower, profiles/r04_attn_variants_ab.txt)
  // per row tile: the lane's query row m (clamped to the last token): Q fragments and minus the row term
  auto q_rows = [&](int m, v4i (&qb)[2]) __attribute__((always_inline)) {
      {
        // (Q rows by LDS-DMA at the workgroup's start instead: no faster on the bench's data,
        // profiles/r04_attn_real_data.txt)
        const int qrow = min(m, T - 1);
        if constexpr ((NQK_ATTN_DIAG & 2048) != 0) {  // (diagnostic 2048: Q rows from the LDS K image, no Q loads)
          qb[0] = *reinterpret_cast<const v4i*>(Ks + swz64a(qrow, h));
          qb[1] = *reinterpret_cast<const v4i*>(Ks + swz64a(qrow, 2 + h));
        } else {
          qb[0] = *reinterpret_cast<const v4i*>(q + qrow * 64 + h * 16);
          qb[1] = *reinterpret_cast<const v4i*>(q + qrow * 64 + (2 + h) * 16);
        }
      }
      int rq = sum16a(qb[0]) + sum16a(qb[1]);
      rq += xor32i(rq);
      // minus the row term: acc init = nrowterm - colterm, one v_sub per element (the empty asm
      // keeps the compiler from re-associating it into -(rowterm + colterm): an add and a sub)
      int nrowterm = -(rq * a.zk);
      asm volatile("" : "+v"(nrowterm));
    return nrowterm;
  };
  // dequant + quantize (EPI_PV) of a row tile's context -> ctx[img][m][head * 64 + d], 4 dims per store
  auto ctx_store = [&](int m, int rp, const v16i (&acc2)[2]) __attribute__((always_inline)) {
    const int rowp = rp * a.zv;
    int8_t* orow = ctx + ((int64_t)img * T + m) * a.ld_out + head * 64;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int d0 = j * 32 + 8 * qq + 4 * h;
        const v4i cv = *reinterpret_cast<const v4i*>(colV + d0);
        uint32_t packed = 0;
        int qs[4];
        float o[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int vv = acc2[j][4 * qq + jj] - rowp - cv[jj];
          o[jj] = FAST ? (float)vv * a.s_pv : (float)((double)vv * (double)a.s_pv);
        }
        if constexpr ((NQK_ATTN_DIAG & 16) != 0) {  // (diagnostic 16: context bytes without the quantize)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) qs[jj] = (int)o[jj];
        } else if constexpr (FAST) {
          // rint(zp + t) for t = RN(o / s_ctx) approximated by tf = o rs (|t - tf| <= |tf| 2^-21),
          // on pairs: one v_pk_mul, clamp + magic-number rounding (round_magic2), and the
          // measure |tf| 2^-21 + |dd| of the four elements: below 0.5 - 2^-23 every element's
          // rounding boundary is farther than the error, else the exact chain (quant_w)
          v2f_t dd0, dd1;
          const v2f_t t0 = v2f_t{o[0], o[1]} * v2f_t{a.rs_ctx_f, a.rs_ctx_f};
          const v2f_t t1 = v2f_t{o[2], o[3]} * v2f_t{a.rs_ctx_f, a.rs_ctx_f};
          const v2f_t s0 = round_magic2(t0, a.lo_f - a.zp_ctx_f, a.hi_f - a.zp_ctx_f, 0x1.8p23f + a.zp_ctx_f, dd0);
          const v2f_t s1 = round_magic2(t1, a.lo_f - a.zp_ctx_f, a.hi_f - a.zp_ctx_f, 0x1.8p23f + a.zp_ctx_f, dd1);
          const float m0 = __builtin_fmaf(__builtin_fabsf(t0[0]), 0x1p-21f, __builtin_fabsf(dd0[0]));
          const float m1 = __builtin_fmaf(__builtin_fabsf(t0[1]), 0x1p-21f, __builtin_fabsf(dd0[1]));
          const float m2 = __builtin_fmaf(__builtin_fabsf(t1[0]), 0x1p-21f, __builtin_fabsf(dd1[0]));
          const float m3 = __builtin_fmaf(__builtin_fabsf(t1[1]), 0x1p-21f, __builtin_fabsf(dd1[1]));
          // NaN / inf order above every finite measure as unsigned bits
          const uint32_t wm = __builtin_elementwise_max(__builtin_elementwise_max(__float_as_uint(m0), __float_as_uint(m1)),
                                                        __builtin_elementwise_max(__float_as_uint(m2), __float_as_uint(m3)));
          packed = pack4_low(s0, s1);
          if (__builtin_expect(__any(wm >= __float_as_uint(0x1.fffffcp-2f)), 0)) {
            NQK_ATTN_COUNT(3);
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              const int qv = quant_w(o[jj], a.s_ctx, a.rs_ctx, a.zp_ctx, a.lo, a.hi);
              packed = (packed & ~(0xffu << (8 * jj))) | ((uint32_t)(qv & 0xff) << (8 * jj));
            }
          }
          if (m < T) *reinterpret_cast<uint32_t*>(orow + d0) = packed;
          __builtin_amdgcn_sched_barrier(0);
          continue;
        } else {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) qs[jj] = quant_w(o[jj], a.s_ctx, a.rs_ctx, a.zp_ctx, a.lo, a.hi);
        }
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) packed |= ((uint32_t)(qs[jj] & 0xff)) << (8 * jj);
        if (m < T) *reinterpret_cast<uint32_t*>(orow + d0) = packed;
        __builtin_amdgcn_sched_barrier(0);
      }
  };
  for (int rt = wave; rt < (TAILR ? NT - 1 : NT); rt += 4) {
    const int m0 = rt * 32, m = m0 + r32;
    v4i qb[2];
    const int nrowterm = q_rows(m, qb);
    int rp;
    v16i acc2[2];
    // ---- per score tile c: S^T = K Q^T (two MFMAs), dequant + Div (EPI_SCORES), row
    // max; only one tile's accumulators are live
    float e[NT][16];
    float mx = -__builtin_inff();
    float mn = __builtin_inff();  // NQK_ATTN_EXP2: the smallest score of the whole groups
    // whole groups: max / min of the integers (y = RN(v s_qkd) is monotone in v for s_qkd > 0,
    // host-checked on the FAST path), one v_max3_i32 / v_min3_i32 per pair; converted once
    int imx = INT32_MIN, imn = INT32_MAX;
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      // the accumulators start at -(row term + column term): the MFMAs then leave the
      // zero-point-corrected integer v = acc - terms itself (int32, exact in any order)
      v16i acc;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        if (pad_group(c, qq)) {
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[4 * qq + j] = 0;
          continue;
        }
        const v4i ck = *reinterpret_cast<const v4i*>(colK + c * 32 + 8 * qq + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[4 * qq + j] = nrowterm - ck[j];
      }
#pragma unroll
      for (int s = 0; s < 2 && (NQK_ATTN_DIAG & 8) == 0; ++s) {  // (diagnostic 8: no score MFMAs)
        const v4i ka = *reinterpret_cast<const v4i*>(Ks + swz64a(c * 32 + r32, 2 * s + h));
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(ka, qb[s], acc, 0, 0, 0);
      }
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        if (pad_group(c, qq)) {  // every column of the group is padding (compile time)
#pragma unroll
          for (int j = 0; j < 4; ++j) e[c][4 * qq + j] = 0.0f;
          continue;
        }
        if constexpr (FAST && NQK_ATTN_PK) {
          // pairs: one v_pk_mul for the dequantize + Div, a v_max3 for the row max; the
          // -inf of padded columns only where the group straddles T (runtime lane half)
          const bool full = TC > 0 && c * 32 + 8 * qq + 8 <= TC;
#pragma unroll
          for (int j = 0; j < 4; j += 2) {
            const int r = 4 * qq + j, n = c * 32 + 8 * qq + 4 * h + j;
            v2f_t y = v2f_t{(float)acc[r], (float)acc[r + 1]} * v2f_t{a.s_qkd, a.s_qkd};
            if (!full) y = y + v2f_t{n < T ? 0.0f : -__builtin_inff(), n + 1 < T ? 0.0f : -__builtin_inff()};
            e[c][r] = y[0];
            e[c][r + 1] = y[1];
            if (full) {
              imx = max(imx, max(acc[r], acc[r + 1]));
              if (NQK_ATTN_EXP2) imn = min(imn, min(acc[r], acc[r + 1]));
            } else {
              mx = __builtin_fmaxf(mx, __builtin_fmaxf(y[0], y[1]));
            }
          }
          __builtin_amdgcn_sched_barrier(0);
          continue;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 4 * qq + j, n = c * 32 + 8 * qq + 4 * h + j;
          const int vv = acc[r];
          float y;
          // FAST: RN(v s) / 2^k == RN(v (s / 2^k)) while both are normal (host-checked)
          if constexpr (FAST) y = (float)vv * a.s_qkd;
          else y = div_rc_w((float)((double)vv * (double)a.s_qk), a.rdiv);
          // -inf for padded columns: an add of a selected constant, so no branch
          y = y + (n < T ? 0.0f : -__builtin_inff());
          e[c][r] = y;
          mx = y > mx ? y : mx;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (FAST && NQK_ATTN_PK) {
      if (imx != INT32_MIN) mx = __builtin_fmaxf(mx, (float)imx * a.s_qkd);
      if (NQK_ATTN_EXP2 && imn != INT32_MAX) mn = (float)imn * a.s_qkd;
    }
    {
      const float o = xor32f(mx);
      mx = o > mx ? o : mx;
    }
    const float nm = -mx;
    // NQK_ATTN_EXP2: every argument y - max of the whole groups in [-86.5, 0] in all lanes
    // (RN(mn - mx) is the smallest; straddling groups keep np_expf_nonpos2 for their -inf pads)
    const bool esafe = NQK_ATTN_EXP2 && __all(mn + nm >= NP_EXP_SAFE_LO);
    if (!esafe) NQK_ATTN_COUNT(0);
    if (FAST && NQK_ATTN_PK && NQK_ATTN_EXP2 && TC > 0 && (NQK_ATTN_DIAG & 2) == 0) {
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        if (esafe) {
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            if (pad_group(c, r >> 2)) continue;  // stays 0
            const v2f_t xa = v2f_t{e[c][r], e[c][r + 1]} + v2f_t{nm, nm};
            const v2f_t x = (TC > 0 && c * 32 + 8 * (r >> 2) + 8 <= TC) ? np_expf_safe2(xa) : np_expf_nonpos2(xa);
            e[c][r] = x[0];
            e[c][r + 1] = x[1];
            if ((r % NQK_ATTN_EXPW) == NQK_ATTN_EXPW - 2) __builtin_amdgcn_sched_barrier(0);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            if (pad_group(c, r >> 2)) continue;  // stays 0
            const v2f_t x = np_expf_nonpos2(v2f_t{e[c][r], e[c][r + 1]} + v2f_t{nm, nm});
            e[c][r] = x[0];
            e[c][r + 1] = x[1];
            if ((r % NQK_ATTN_EXPW) == NQK_ATTN_EXPW - 2) __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
    } else if constexpr (FAST && NQK_ATTN_PK && (NQK_ATTN_DIAG & 2) == 0) {
#pragma unroll
      for (int c = 0; c < NT; ++c)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          if (pad_group(c, r >> 2)) continue;  // stays 0
          const v2f_t x = np_expf_nonpos2(v2f_t{e[c][r], e[c][r + 1]} + v2f_t{nm, nm});
          e[c][r] = x[0];
          e[c][r + 1] = x[1];
          if ((r % NQK_ATTN_EXPW) == NQK_ATTN_EXPW - 2) __builtin_amdgcn_sched_barrier(0);
        }
    } else
#pragma unroll
    for (int c = 0; c < NT; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (pad_group(c, r >> 2)) continue;  // stays 0
        if constexpr ((NQK_ATTN_DIAG & 2) != 0) e[c][r] = e[c][r] + nm;
        else e[c][r] = np_expf_nonpos(e[c][r] + nm);  // y - max <= 0; -inf pads -> 0
        // scheduling window of NQK_ATTN_EXPW independent exp chains
        if ((r % NQK_ATTN_EXPW) == NQK_ATTN_EXPW - 1) __builtin_amdgcn_sched_barrier(0);
      }
    // ---- NumPy pairwise sum: accumulators r[4h + j] of each leaf, in increasing n
    float ra[2][4], tv[2][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) ra[0][j] = ra[1][j] = tv[0][j] = tv[1][j] = 0.0f;
    if constexpr (NQK_ATTN_PSUM && TC > 0) {
      // accumulators j, j + 1 as one packed pair: per lane the same IEEE adds in the same order
      v2f_t pa[2][2], pt[2][2];
#pragma unroll
      for (int l = 0; l < 2; ++l) pa[l][0] = pa[l][1] = pt[l][0] = pt[l][1] = v2f_t{0.0f, 0.0f};
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int c = g >> 2, qq = g & 3;
        const bool f0 = g == g0_0, in0 = g < g0_0 + ng0;
        const bool f1 = g == g0_1, in1 = g >= g0_1 && g < g0_1 + ng1;
        const v2f_t x01 = v2f_t{e[c][4 * qq], e[c][4 * qq + 1]}, x23 = v2f_t{e[c][4 * qq + 2], e[c][4 * qq + 3]};
        if (in0) {
          pa[0][0] = f0 ? x01 : pa[0][0] + x01;
          pa[0][1] = f0 ? x23 : pa[0][1] + x23;
        }
        if (in1) {
          pa[1][0] = f1 ? x01 : pa[1][0] + x01;
          pa[1][1] = f1 ? x23 : pa[1][1] + x23;
        }
        if (g == gt0) {
          pt[0][0] = x01;
          pt[0][1] = x23;
        }
        if (g == gt1) {
          pt[1][0] = x01;
          pt[1][1] = x23;
        }
      }
#pragma unroll
      for (int l = 0; l < 2; ++l)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          ra[l][j] = pa[l][j >> 1][j & 1];
          tv[l][j] = pt[l][j >> 1][j & 1];
        }
    } else
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int c = g >> 2, qq = g & 3;
      const bool f0 = g == g0_0, in0 = g < g0_0 + ng0;
      const bool f1 = g == g0_1, in1 = g >= g0_1 && g < g0_1 + ng1;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x = e[c][4 * qq + j];
        ra[0][j] = in0 ? (f0 ? x : ra[0][j] + x) : ra[0][j];
        ra[1][j] = in1 ? (f1 ? x : ra[1][j] + x) : ra[1][j];
        tv[0][j] = g == gt0 ? x : tv[0][j];
        tv[1][j] = g == gt1 ? x : tv[1][j];
      }
    }
    float leaf[2];
#pragma unroll
    for (int l = 0; l < 2; ++l) {
      const int ng = l ? ng1 : ng0, tl = l ? tl1 : tl0;
      float res = 0.0f;
      if (ng > 0) {
        const float mine = (ra[l][0] + ra[l][1]) + (ra[l][2] + ra[l][3]);
        const float other = xor32f(mine);
        res = h ? other + mine : mine + other;
      }
      // tail columns t < tl: t = 0..3 in half 0, 4..7 in half 1, added in order
      float x = res;
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (t < tl) x = x + tv[l][t];
      const float x0 = xor32f(x);  // half 1 receives half 0's running sum
      float y = x0;
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (4 + t < tl) y = y + tv[l][t];
      const float y1 = xor32f(y);  // half 0 receives half 1's result
      leaf[l] = h ? y : y1;
    }
    const float tot = n2 ? leaf[0] + leaf[1] : leaf[0];
    const double rtot = 1.0 / (double)tot;
    const double kpd = rtot * a.rs_p;
    const float kpf = (float)kpd;  // t = e / tot / s_p within |t| 2^-22 of e * kpf
    const float kpl = NQK_ATTN_PKL ? (float)(kpd - (double)kpf) : 0.0f;
    constexpr float PM_T = NQK_ATTN_PKL ? 0x1.9p-23f : NQK_ATTN_PM_T;
    // the filter's bound for the whole row (|tf| <= kpf (1 + 2^-23)), with margin
    const float plim = 0.5f - 2.0f * __builtin_fmaf(kpf, 0x1p-21f, 0x1p-126f);
    const float zp128 = a.zp_p_f + 128.0f, lo128 = a.lo_f + 128.0f, hi128 = a.hi_f + 128.0f;
    const float pqlo = a.lo_f - a.zp_p_f, pqhi = a.hi_f - a.zp_p_f, pmagic = 0x1.8p23f + a.zp_p_f;
    // ---- per score tile c: P = quantize(e / tot) (4 packed bytes per group, row sums),
    // then at once its share of O^T = V^T P^T (B operand = P row m, 16 consecutive tokens
    // per half), so only one tile's packed P is live
    rp = 0;
    // NQK_ATTN_PQ2: when every lane's kpf <= pqhi (and pqlo <= 0), e kpf in [0, kpf] never
    // reaches a clamp (wave-uniform): s = RN(e kpf + pmagic) is rint(e kpf) + pmagic from
    // the exact product (one rounding fewer than tf = RN(e kpf), so still within |t| 2^-22 of
    // t), dd = RN(e kpf - (s - pmagic)) within 2^-25 of the exact distance (the limit takes
    // 2^-24 off for it)
    // (diagnostic 512: the clamp-free path on every row, wrong results where a clamp is reached)
    const bool pq_nc = NQK_ATTN_PQ2 && ((NQK_ATTN_DIAG & 512) != 0 || (pqlo <= 0.0f && __all(kpf <= pqhi)));
    const float plim2 = plim - 0x1p-24f;
    if (!pq_nc) NQK_ATTN_COUNT(1);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc2[j][r] = 0;
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      int dw[4];
      if constexpr (FAST && (NQK_ATTN_DIAG & 4) == 0) {
        // t = e / tot / s_p is within thr of tf = e * kpf (|tf| <= kpf: e <= 1); where tf
        // is farther than that from a rounding boundary, rint(tf) is rint(t).  Per
        // element: the product, rint, the distance test, then v + 128 (v = the clamped
        // integer, in [0, 255]) converted straight into its byte (v_cvt_pk_u8_f32) and
        // the bytes flipped to two's complement at once (^ 0x80 each).
        // the tile's largest distance |tf - r| (tf finite: e in [0, 1], kpf finite),
        // one v_max per element; a tile with any element at or past plim recomputes the
        // same tf per element and sends those elements through the exact chain
        float worst = 0.0f;
        if (NQK_ATTN_PQ2 && NQK_ATTN_PK && pq_nc) {
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            if (pad_group(c, qq)) {
              dw[qq] = 0;
              continue;
            }
            const v2f_t k2 = v2f_t{kpf, kpf}, m2 = v2f_t{pmagic, pmagic};
            const v2f_t e0 = v2f_t{e[c][4 * qq], e[c][4 * qq + 1]}, e1 = v2f_t{e[c][4 * qq + 2], e[c][4 * qq + 3]};
            const v2f_t s0 = __builtin_elementwise_fma(e0, k2, m2), s1 = __builtin_elementwise_fma(e1, k2, m2);
            const v2f_t dd0 = __builtin_elementwise_fma(e0, k2, -(s0 - m2));
            const v2f_t dd1 = __builtin_elementwise_fma(e1, k2, -(s1 - m2));
            if constexpr (NQK_ATTN_PREL) {
              // |t - e kpf| <= 3 2^-24 |x|: the margin NQK_ATTN_PM_R |r| (r = the rounded value; at
              // r = 0 the limit itself covers it), the limit 0.5 - 2^-23 absorbs dd's own rounding
              const v2f_t r0 = s0 - m2, r1 = s1 - m2;
              worst = __builtin_fmaxf(worst, __builtin_fmaxf(__builtin_fmaf(__builtin_fabsf(r0[0]), NQK_ATTN_PM_R, __builtin_fabsf(dd0[0])),
                                                             __builtin_fmaf(__builtin_fabsf(r0[1]), NQK_ATTN_PM_R, __builtin_fabsf(dd0[1]))));
              worst = __builtin_fmaxf(worst, __builtin_fmaxf(__builtin_fmaf(__builtin_fabsf(r1[0]), NQK_ATTN_PM_R, __builtin_fabsf(dd1[0])),
                                                             __builtin_fmaf(__builtin_fabsf(r1[1]), NQK_ATTN_PM_R, __builtin_fabsf(dd1[1]))));
            } else {
              worst = __builtin_fmaxf(worst, __builtin_fmaxf(__builtin_fabsf(dd0[0]), __builtin_fabsf(dd0[1])));
              worst = __builtin_fmaxf(worst, __builtin_fmaxf(__builtin_fabsf(dd1[0]), __builtin_fabsf(dd1[1])));
            }
            uint32_t w = pack4_low(s0, s1);
            if (!(TC > 0 && c * 32 + 8 * qq + 8 <= TC)) {  // padded columns: 0
              const int n = c * 32 + 8 * qq + 4 * h;
              uint32_t keep = 0;
#pragma unroll
              for (int j = 0; j < 4; ++j) keep |= (n + j < T ? 0xffu : 0u) << (8 * j);
              w &= keep;
            }
            dw[qq] = (int)w;
          }
          // (diagnostic 256: the exact fallbacks skipped)
          if ((NQK_ATTN_DIAG & 256) == 0 && __builtin_expect(__any(!(worst < (NQK_ATTN_PREL ? 0x1.fffff8p-2f : plim2))), 0)) {
            NQK_ATTN_COUNT(2);
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
              if (pad_group(c, qq)) continue;
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const int n = c * 32 + 8 * qq + 4 * h + j;
                const float x = e[c][4 * qq + j];
                const float rr = __builtin_fmaf(x, kpf, pmagic) - pmagic;
                const float d = __builtin_fmaf(x, kpf, -rr);
                if (!(NQK_ATTN_PREL ? __builtin_fmaf(__builtin_fabsf(rr), NQK_ATTN_PM_R, __builtin_fabsf(d)) < 0x1.fffff8p-2f
                                    : __builtin_fabsf(d) < plim2)) {
                  const int qv = n < T ? quant_w(div_rc_w(x, rtot), a.s_p, a.rs_p, a.zp_p, a.lo, a.hi) : 0;
                  dw[qq] = (int)(((uint32_t)dw[qq] & ~(0xffu << (8 * j))) | ((uint32_t)(qv & 0xff) << (8 * j)));
                }
              }
            }
          }
        } else {
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          if (pad_group(c, qq)) {
            dw[qq] = 0;
            continue;
          }
          if constexpr (NQK_ATTN_PK) {
            // pairs: one v_pk_mul for tf, the clamp / magic-number rounding + byte pack of
            // round_magic2 / pack4_low (nqk_numerics.h), |dd| into the tile's worst
            v2f_t dd0, dd1;
            const v2f_t ea = v2f_t{e[c][4 * qq], e[c][4 * qq + 1]}, eb = v2f_t{e[c][4 * qq + 2], e[c][4 * qq + 3]};
            const v2f_t k2 = v2f_t{kpf, kpf}, kl2 = v2f_t{kpl, kpl};
            const v2f_t tf0 = NQK_ATTN_PKL ? __builtin_elementwise_fma(ea, k2, ea * kl2) : ea * k2;
            const v2f_t tf1 = NQK_ATTN_PKL ? __builtin_elementwise_fma(eb, k2, eb * kl2) : eb * k2;
            const v2f_t s0 = round_magic2(tf0, pqlo, pqhi, pmagic, dd0);
            const v2f_t s1 = round_magic2(tf1, pqlo, pqhi, pmagic, dd1);
            if constexpr (NQK_ATTN_PREL) {
              // |t - tf| <= 4 2^-24 |x|: the margin NQK_ATTN_PM_T |tf| per element (clamped elements:
              // dd = 0, and the clamp decides them either way)
              worst = __builtin_fmaxf(worst, __builtin_fmaxf(__builtin_fmaf(__builtin_fabsf(tf0[0]), PM_T, __builtin_fabsf(dd0[0])),
                                                             __builtin_fmaf(__builtin_fabsf(tf0[1]), PM_T, __builtin_fabsf(dd0[1]))));
              worst = __builtin_fmaxf(worst, __builtin_fmaxf(__builtin_fmaf(__builtin_fabsf(tf1[0]), PM_T, __builtin_fabsf(dd1[0])),
                                                             __builtin_fmaf(__builtin_fabsf(tf1[1]), PM_T, __builtin_fabsf(dd1[1]))));
            } else {
              worst = __builtin_fmaxf(worst, __builtin_fmaxf(__builtin_fabsf(dd0[0]), __builtin_fabsf(dd0[1])));
              worst = __builtin_fmaxf(worst, __builtin_fmaxf(__builtin_fabsf(dd1[0]), __builtin_fabsf(dd1[1])));
            }
            uint32_t w = pack4_low(s0, s1);
            if (!(TC > 0 && c * 32 + 8 * qq + 8 <= TC)) {  // padded columns: 0
              const int n = c * 32 + 8 * qq + 4 * h;
              uint32_t keep = 0;
#pragma unroll
              for (int j = 0; j < 4; ++j) keep |= (n + j < T ? 0xffu : 0u) << (8 * j);
              w &= keep;
            }
            dw[qq] = (int)w;
            continue;
          }
          uint32_t packed = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int n = c * 32 + 8 * qq + 4 * h + j;
            const float tf = e[c][4 * qq + j] * kpf;
            const float r = __builtin_rintf(tf);
            worst = __builtin_fmaxf(worst, __builtin_fabsf(tf - r));
            float v = __builtin_amdgcn_fmed3f(r + zp128, lo128, hi128);
            v = n < T ? v : 128.0f;  // padded columns: 0
            packed = __builtin_amdgcn_cvt_pk_u8_f32(v, j, packed);
          }
          dw[qq] = (int)(packed ^ 0x80808080u);
        }
        const bool prel = NQK_ATTN_PREL && NQK_ATTN_PK;
        if ((NQK_ATTN_DIAG & 256) == 0 && __builtin_expect(__any(!(worst < (prel ? 0x1.fffff8p-2f : plim))), 0)) {
          NQK_ATTN_COUNT(2);
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            if (pad_group(c, qq)) continue;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int n = c * 32 + 8 * qq + 4 * h + j;
              const float ej = e[c][4 * qq + j];
              const float tf = NQK_ATTN_PKL ? __builtin_fmaf(ej, kpf, ej * kpl) : ej * kpf;
              const float cf = prel ? __builtin_amdgcn_fmed3f(tf, pqlo, pqhi) : tf;  // (the clamp as in the fast path)
              const float dv = __builtin_fabsf(cf - __builtin_rintf(cf));
              if (!(prel ? __builtin_fmaf(__builtin_fabsf(tf), PM_T, dv) < 0x1.fffff8p-2f : dv < plim)) {
                const int qv = n < T ? quant_w(div_rc_w(e[c][4 * qq + j], rtot), a.s_p, a.rs_p, a.zp_p, a.lo, a.hi) : 0;
                dw[qq] = (int)(((uint32_t)dw[qq] & ~(0xffu << (8 * j))) | ((uint32_t)(qv & 0xff) << (8 * j)));
              }
            }
          }
        }
        }
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
          if (!pad_group(c, qq)) rp = __builtin_amdgcn_sdot4(dw[qq], 0x01010101, rp, false);
      } else {
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        if (pad_group(c, qq)) {
          dw[qq] = 0;
          continue;
        }
        uint32_t packed = 0;
        int qs[4];
        if constexpr ((NQK_ATTN_DIAG & 4) != 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j) qs[j] = (int)e[c][4 * qq + j];
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            qs[j] = quant_w(div_rc_w(e[c][4 * qq + j], rtot), a.s_p, a.rs_p, a.zp_p, a.lo, a.hi);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = c * 32 + 8 * qq + 4 * h + j;
          const int qv = qs[j] & -(int)(n < T);  // padded columns: 0
          rp += qv;
          packed |= ((uint32_t)(qv & 0xff)) << (8 * j);
        }
        dw[qq] = (int)packed;
        __builtin_amdgcn_sched_barrier(0);
      }
      }
      // half 0 needs tokens 0..15 of the tile = [own g0, partner g0, own g1, partner g1];
      // half 1 needs 16..31 = [partner g2, own g2, partner g3, own g3]
      const int xa = xor32i(h ? dw[0] : dw[2]);
      const int xb = xor32i(h ? dw[1] : dw[3]);
      v4i pb;
      if (h) { pb[0] = xa; pb[1] = dw[2]; pb[2] = xb; pb[3] = dw[3]; }
      else   { pb[0] = dw[0]; pb[1] = xa; pb[2] = dw[1]; pb[3] = xb; }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const v4i va = *reinterpret_cast<const v4i*>(Vt + vt_row(j * 32 + r32) + (2 * c + h) * 16);
        if constexpr ((NQK_ATTN_DIAG & 32) != 0) acc2[j][c] ^= va[0] ^ pb[j];  // (diagnostic 32: no PV MFMAs)
        else acc2[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(va, pb, acc2[j], 0, 0, 0);
      }
    }
    rp += xor32i(rp);
    ctx_store(m, rp, acc2);
  }
  if constexpr (TAILR) {
    if (wave == (NT - 1) % 4) {
      const int rt = NT - 1, m = rt * 32 + r32;
      v4i qb[2];
      const int nrowterm = q_rows(m, qb);
      int rp;
      v16i acc2[2];
      // ---- the last row tile (NQK_ATTN_TAIL): TR real query rows of 32.  The scores of those
      // rows go to LDS, and the softmax / P quantize run with one lane per (row, NumPy
      // accumulator n % 8) — NG + 1 elements a lane instead of 112 — then P comes back to the
      // MFMA layout for P V.  Same operations per element as the full tile, the pairwise sum's
      // accumulator chains and combination tree unchanged (every add of the tree is commutative).
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        v16i acc;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          if (pad_group(c, qq)) {
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[4 * qq + j] = 0;
            continue;
          }
          const v4i ck = *reinterpret_cast<const v4i*>(colK + c * 32 + 8 * qq + 4 * h);
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[4 * qq + j] = nrowterm - ck[j];
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const v4i ka = *reinterpret_cast<const v4i*>(Ks + swz64a(c * 32 + r32, 2 * s + h));
          acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(ka, qb[s], acc, 0, 0, 0);
        }
        if (r32 < TR) {
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            if (pad_group(c, qq)) continue;
            const v2f_t y01 = v2f_t{(float)acc[4 * qq], (float)acc[4 * qq + 1]} * v2f_t{a.s_qkd, a.s_qkd};
            const v2f_t y23 = v2f_t{(float)acc[4 * qq + 2], (float)acc[4 * qq + 3]} * v2f_t{a.s_qkd, a.s_qkd};
            *reinterpret_cast<float4*>(tS + r32 * TSTR + c * 32 + 8 * qq + 4 * h) = make_float4(y01[0], y01[1], y23[0], y23[1]);
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      // lane (ti, tj): row ti (rows >= TR mirror row TR - 1: computed, never stored), elements
      // n = 8 g + tj (g < NG: NG0 groups of leaf 0, NG1 of leaf 1) and the tail element 8 NG + tj
      const int ti = min(lane >> 3, TR - 1), tj = lane & 7, tb = lane & ~7;
      const bool real = (lane >> 3) < TR;
      float* const srow = tS + ti * TSTR;
      // (streamed through LDS in three passes, so the path holds no per-element registers: the
      // kernel's full tiles keep their register budget)
      const float xt = tj < TL1 ? srow[8 * NG + tj] : -__builtin_inff();
      float mxl = xt, mnl = tj < TL1 ? xt : __builtin_inff();
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const float v = srow[8 * g + tj];
        mxl = __builtin_fmaxf(mxl, v), mnl = __builtin_fminf(mnl, v);
      }
#pragma unroll
      for (int sh = 1; sh < 8; sh <<= 1) {
        mxl = __builtin_fmaxf(mxl, __shfl_xor(mxl, sh, 64));
        mnl = __builtin_fminf(mnl, __shfl_xor(mnl, sh, 64));
      }
      const float nm = -mxl;
      const bool esafe = __all(mnl + nm >= NP_EXP_SAFE_LO);
      // exp of elements g (leaf 0) and NG0 + g (leaf 1) as a pair, written back over the scores;
      // NumPy's pairwise sum: accumulator tj of each leaf in increasing n (the pair's lanes), the
      // 8 accumulators of a leaf combined ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) by xor
      // butterflies, leaf 1's tail elements added in order, then leaf 0 + leaf 1
      v2f_t ls;
#pragma unroll
      for (int g = 0; g < NG0; ++g) {
        const v2f_t xa = v2f_t{srow[8 * g + tj], srow[8 * (NG0 + g) + tj]} + v2f_t{nm, nm};
        const v2f_t ex = esafe ? np_expf_safe2(xa) : np_expf_nonpos2(xa);
        ls = g == 0 ? ex : ls + ex;
        if (real) srow[8 * g + tj] = ex[0], srow[8 * (NG0 + g) + tj] = ex[1];
      }
      const float et = np_expf_nonpos2(v2f_t{xt + nm, xt + nm})[0];  // (no tail element: -inf -> 0)
#pragma unroll
      for (int sh = 1; sh < 8; sh <<= 1) ls = ls + v2f_t{__shfl_xor(ls[0], sh, 64), __shfl_xor(ls[1], sh, 64)};
      float leaf1 = ls[1];
#pragma unroll
      for (int t = 0; t < TL1; ++t) leaf1 = leaf1 + __shfl(et, tb + t, 64);
      const float tot = ls[0] + leaf1;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      const double rtot = 1.0 / (double)tot;
      const float kpf = (float)(rtot * a.rs_p);
      const float pqlo = a.lo_f - a.zp_p_f, pqhi = a.hi_f - a.zp_p_f, pmagic = 0x1.8p23f + a.zp_p_f;
      const bool pq_nc = pqlo <= 0.0f && __all(kpf <= pqhi);
      // P = quantize(e / tot) by the full tile's filtered fast path, exact chain where it cannot decide
      const v2f_t k2 = v2f_t{kpf, kpf}, m2 = v2f_t{pmagic, pmagic};
      constexpr int NPW = (NG + 4) / 4;
      uint32_t pw[NPW];  // the lane's P bytes, 4 to a word: element g in byte g % 4 of word g / 4
#pragma unroll
      for (int w = 0; w < NPW; ++w) pw[w] = 0u;
      auto put = [&](int g, int q) __attribute__((always_inline)) {
        pw[g >> 2] = (pw[g >> 2] & ~(0xffu << (8 * (g & 3)))) | ((uint32_t)(q & 0xff) << (8 * (g & 3)));
      };
      auto get = [&](int g) __attribute__((always_inline)) { return (int)(int8_t)(pw[g >> 2] >> (8 * (g & 3))); };
      uint32_t fails = 0;
      auto quant_pair = [&](v2f_t e2, int& q0, int& q1, uint32_t& f0, uint32_t& f1) __attribute__((always_inline)) {
        v2f_t s2, dd, mag;
        if (pq_nc) {
          s2 = __builtin_elementwise_fma(e2, k2, m2);
          const v2f_t r2 = s2 - m2;
          dd = __builtin_elementwise_fma(e2, k2, -r2);
          mag = r2;
        } else {
          const v2f_t tf = e2 * k2;
          s2 = round_magic2(tf, pqlo, pqhi, pmagic, dd);
          mag = tf;
        }
        const float mr = pq_nc ? NQK_ATTN_PM_R : NQK_ATTN_PM_T;
        f0 = !(__builtin_fmaf(__builtin_fabsf(mag[0]), mr, __builtin_fabsf(dd[0])) < 0x1.fffff8p-2f);
        f1 = !(__builtin_fmaf(__builtin_fabsf(mag[1]), mr, __builtin_fabsf(dd[1])) < 0x1.fffff8p-2f);
        q0 = (int)(int8_t)(__float_as_uint(s2[0]) & 0xffu);
        q1 = (int)(int8_t)(__float_as_uint(s2[1]) & 0xffu);
      };
#pragma unroll
      for (int g = 0; g < NG; g += 2) {
        uint32_t f0, f1;
        int q0, q1;
        quant_pair(v2f_t{srow[8 * g + tj], srow[8 * (g + 1) + tj]}, q0, q1, f0, f1);
        put(g, q0);
        put(g + 1, q1);
        fails |= (f0 << g) | (f1 << (g + 1));
      }
      {
        uint32_t f0, f1;
        int q0, qd;
        quant_pair(v2f_t{et, et}, q0, qd, f0, f1);
        put(NG, tj < TL1 ? q0 : 0);  // (no tail element: 0, so the byte sum below needs no mask)
        fails |= (tj < TL1 ? f0 : 0u) << NG;
      }
      if (__builtin_expect(__any(fails != 0), 0)) {
        NQK_ATTN_COUNT(2);
#pragma unroll
        for (int g = 0; g <= NG; ++g)
          if ((fails >> g) & 1u) put(g, quant_w(div_rc_w(g < NG ? srow[8 * g + tj] : et, rtot), a.s_p, a.rs_p, a.zp_p, a.lo, a.hi));
      }
      int rps = 0;
#pragma unroll
      for (int w = 0; w < NPW; ++w) rps = __builtin_amdgcn_sdot4((int)pw[w], 0x01010101, rps, false);  // signed bytes
#pragma unroll
      for (int sh = 1; sh < 8; sh <<= 1) rps += __shfl_xor(rps, sh, 64);
      if ((lane >> 3) < TR) {
        int8_t* prow = tP + (lane >> 3) * TP;
#pragma unroll
        for (int g = 0; g < NG; ++g) prow[8 * g + tj] = (int8_t)get(g);
        if (tj < TL1) prow[8 * NG + tj] = (int8_t)get(NG);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      // ---- P back in the MFMA layout (rows >= TR and columns >= T: 0), then P V as the full tile
      rp = __shfl(rps, min(r32, TR - 1) * 8, 64);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc2[j][r] = 0;
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        int dw[4];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          if (pad_group(c, qq)) {
            dw[qq] = 0;
            continue;
          }
          const int n = c * 32 + 8 * qq + 4 * h;
          uint32_t w = r32 < TR ? *reinterpret_cast<const uint32_t*>(tP + r32 * TP + n) : 0u;
          if (!(c * 32 + 8 * qq + 8 <= TC)) {
            uint32_t keep = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) keep |= (n + j < T ? 0xffu : 0u) << (8 * j);
            w &= keep;
          }
          dw[qq] = (int)w;
        }
        const int xa = xor32i(h ? dw[0] : dw[2]);
        const int xb = xor32i(h ? dw[1] : dw[3]);
        v4i pb;
        if (h) { pb[0] = xa; pb[1] = dw[2]; pb[2] = xb; pb[3] = dw[3]; }
        else   { pb[0] = dw[0]; pb[1] = xa; pb[2] = dw[1]; pb[3] = xb; }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const v4i va = *reinterpret_cast<const v4i*>(Vt + vt_row(j * 32 + r32) + (2 * c + h) * 16);
          acc2[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(va, pb, acc2[j], 0, 0, 0);
        }
      }
      ctx_store(m, rp, acc2);
    }
  }
}


// ---------------------------------------------------------------------------------------------
// k_attn16 (round 6): the T = 197 FAST attention on v_mfma_i32_16x16x64_i8, FOUR lanes per query
// row (k_attention: 32x32x32, two lanes per row).  Why: k_attention holds a query's 112 scores per
// lane (168 VGPRs: three waves per SIMD) and its waves sit 30 % dependency-stalled and 33 % parked
// (profiles/r05_attn_diag.txt) — VALU-issue is 40 % busy.  Here a lane holds 52 scores (13 tiles of
// 16 keys x 4): fewer registers, more waves per SIMD to hide the same chains; the key dimension pads
// to 208 instead of 224 (7 % less exp / quantize work on pads); and the probabilities P feed the
// P V MFMAs from the lane that computed them (no cross-lane exchange).
//
// Key order.  Score tile c, position p = 4 g + r (g = lane >> 4, the lane group; r the accumulator
// register) holds key n(c, p) = 16 c + 8 (r >> 1) + 2 g + (r & 1): lane group g owns exactly NumPy's
// pairwise accumulators j = 2 g and 2 g + 1 (keys n = j mod 8), so every accumulator chain runs
// in-lane in increasing n (two tiles' t = 0, 1 halves in order), and the ((r0 + r1) + (r2 + r3)) +
// ((r4 + r5) + (r6 + r7)) combine is an in-lane add and two lane-group swaps (v_permlane16_swap,
// v_permlane32_swap).  T = 197: leaf 0 = keys 0..95 = tiles 0..5, leaf 1 = keys 96..191 (tiles
// 6..11) + the tail 192..196 (tile 12: group 0's r = 0, 1, group 1's r = 0, 1, group 2's r = 0),
// added in order in group 0's lanes and broadcast.  K rows are staged in LDS in this order.
// P V: the contraction index kappa = 16 lg + 4 q + r of a 64-key chunk ch is (tile 4 ch + q, position
// 4 lg + r), so lane (query, lg)'s B operand is its own P dwords of tiles 4 ch .. 4 ch + 3; V^T is
// staged in LDS in that key order (64 B rows per (chunk, dim), 16-B chunks swizzled as k_pg's).
// Every element goes through exactly k_attention<7, 197, true>'s operations (the same exps, sums,
// P / context filters and exact fallbacks), so the context bytes are bit-identical to it
// (tests/test_gpu_attention.py compares the two kernels).
#ifndef NQK_ATTN16_QPF
#define NQK_ATTN16_QPF 1
#endif
#ifndef NQK_ATTN16_MINB
#define NQK_ATTN16_MINB 4  // workgroups (= waves per SIMD) per CU the register budget is sized for
#endif
constexpr int A16_T = 197, A16_NT = 13, A16_KP = 208, A16_VT = 4 * 64 * 64;
__host__ __device__ constexpr int a16_sw(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }  // = pg_sw
__device__ __forceinline__ int a16_key(int c, int p) { return 16 * c + 8 * ((p >> 1) & 1) + 2 * (p >> 2) + (p & 1); }
__device__ __forceinline__ int xor16i(int x) {
  const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  return (threadIdx.x & 16) ? (int)r[0] : (int)r[1];
}
__device__ __forceinline__ float xor16f(float x) { return __int_as_float(xor16i(__float_as_int(x))); }
constexpr size_t attn16_lds() { return (size_t)A16_KP * 64 + A16_VT + (size_t)A16_KP * 4 + 64 * 4; }

// NW: waves per workgroup, each taking row tiles wave, wave + NW, ... of the 13: 4 (ViT-Base: 3 072
// (image, head) workgroups, 3 rounds of 4 per CU) or 5 (few (image, head) pairs, ViT-Ti: a
// workgroup's life is ceil(13 / 5) = 3 row tiles instead of 4; round-6 A/B)
template <int NW>
__global__ void __launch_bounds__(64 * NW, NQK_ATTN16_MINB)
k_attn16(const int8_t* __restrict__ Qg, const int8_t* __restrict__ Kg, const int8_t* __restrict__ Vg,
         int8_t* __restrict__ ctx, AttnArgs a) {
  constexpr int T = A16_T, NT = A16_NT;
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  int8_t* const Ks = lds;                      // [208][64], chunk c of row R at c ^ a16_sw(R & 15)
  int8_t* const Vt = Ks + A16_KP * 64;         // [4 chunks][64 dims][64 kappa]
  int* const colK = reinterpret_cast<int*>(Vt + A16_VT);  // rowsum(K[n]) zq - zq zk 64, per position
  int* const colV = colK + A16_KP;                         // colsum(V[:, d]) zp - zp zv T
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bh = blockIdx.x;
  const int img = bh / a.H, head = bh - img * a.H;
  const int8_t* q = Qg + (int64_t)bh * T * 64;
  const int8_t* k = Kg + (int64_t)bh * T * 64;
  const int8_t* v = Vg + (int64_t)bh * T * 64;
  const int l15 = lane & 15, g = lane >> 4;

  // ---- K rows in key order n(c, p), V^T in kappa order
  for (int idx = tid; idx < A16_KP * 4; idx += 64 * NW) {
    const int R = idx >> 2, ch = idx & 3;
    const int n = a16_key(R >> 4, R & 15);
    const v4i kv = n < T ? *reinterpret_cast<const v4i*>(k + n * 64 + ch * 16) : v4i{0, 0, 0, 0};
    *reinterpret_cast<v4i*>(Ks + R * 64 + 16 * (ch ^ a16_sw(R & 15))) = kv;
  }
  if (tid < 256) {  // (NW = 5: the fifth wave skips the V^T staging and the colV sums)
    // item tid = (chunk ch, tile-in-chunk qq, lane group lg, 16-dim block dm): keys k0, k0 + 1, k0 + 8,
    // k0 + 9 (k0 = 16 (4 ch + qq) + 2 lg) = kappa 16 lg + 4 qq + 0..3 of chunk ch, 16 dims
    const int ch = tid >> 6, qq = (tid >> 4) & 3, lg = (tid >> 2) & 3, dm = tid & 3;
    const int k0 = 16 * (4 * ch + qq) + 2 * lg;
    const int keys[4] = {k0, k0 + 1, k0 + 8, k0 + 9};
    v4i w[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) w[r] = keys[r] < T ? *reinterpret_cast<const v4i*>(v + keys[r] * 64 + dm * 16) : v4i{0, 0, 0, 0};
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      const uint32_t lo01 = __builtin_amdgcn_perm((uint32_t)w[1][gq], (uint32_t)w[0][gq], 0x05010400u);
      const uint32_t hi01 = __builtin_amdgcn_perm((uint32_t)w[1][gq], (uint32_t)w[0][gq], 0x07030602u);
      const uint32_t lo23 = __builtin_amdgcn_perm((uint32_t)w[3][gq], (uint32_t)w[2][gq], 0x05010400u);
      const uint32_t hi23 = __builtin_amdgcn_perm((uint32_t)w[3][gq], (uint32_t)w[2][gq], 0x07030602u);
      const uint32_t o[4] = {__builtin_amdgcn_perm(lo23, lo01, 0x05040100u), __builtin_amdgcn_perm(lo23, lo01, 0x07060302u),
                             __builtin_amdgcn_perm(hi23, hi01, 0x05040100u), __builtin_amdgcn_perm(hi23, hi01, 0x07060302u)};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int d = 16 * dm + 4 * gq + kk;
        *reinterpret_cast<uint32_t*>(Vt + (ch * 64 + d) * 64 + 16 * (lg ^ a16_sw(d & 15)) + 4 * qq) = o[kk];
      }
    }
  }
  __syncthreads();
  if (tid < A16_KP) {
    const int8_t* kr = Ks + tid * 64;  // (the chunk order does not matter for the sum)
    colK[tid] = (sum16a(*reinterpret_cast<const v4i*>(kr)) + sum16a(*reinterpret_cast<const v4i*>(kr + 16)) +
                 sum16a(*reinterpret_cast<const v4i*>(kr + 32)) + sum16a(*reinterpret_cast<const v4i*>(kr + 48))) * a.zq -
                a.kq;
  }
  if (tid < 256) {
    const int d = tid >> 2, ch = tid & 3;
    const int8_t* vr = Vt + (ch * 64 + d) * 64;
    int s = sum16a(*reinterpret_cast<const v4i*>(vr)) + sum16a(*reinterpret_cast<const v4i*>(vr + 16)) +
            sum16a(*reinterpret_cast<const v4i*>(vr + 32)) + sum16a(*reinterpret_cast<const v4i*>(vr + 48));
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (ch == 0) colV[d] = s * a.zp - a.kp;
  }
  __syncthreads();

  const int fo = l15 * 64 + 16 * (g ^ a16_sw(l15));  // fragment offset: row l15 of a 16-row block, chunk g
  const float pqlo = a.lo_f - a.zp_p_f, pqhi = a.hi_f - a.zp_p_f, pmagic = 0x1.8p23f + a.zp_p_f;
  auto q_frag = [&](int rt) __attribute__((always_inline)) {
    const int mq = rt * 16 + l15;
    return *reinterpret_cast<const v4i*>(q + (mq < T ? mq : T - 1) * 64 + g * 16);
  };
  v4i qnext = q_frag(wave);  // NQK_ATTN16_QPF: the next row tile's Q fragment loads under this one's work
  for (int rt = wave; rt < NT; rt += NW) {
    const int m = rt * 16 + l15;  // the lane's query row
    const v4i qb = NQK_ATTN16_QPF ? qnext : q_frag(rt);
    int nrowterm;
    {
      int rq = sum16a(qb);
      rq += xor16i(rq);
      rq += xor32i(rq);
      nrowterm = -(rq * a.zk);
      asm volatile("" : "+v"(nrowterm));
    }
    // ---- scores S^T tile by tile: e[c][r] = key n(c, 4 g + r) of the lane's query
    float e[NT][4];
    int imx = INT32_MIN, imn = INT32_MAX;
    float mx = -__builtin_inff();
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      const v4i ck = *reinterpret_cast<const v4i*>(colK + 16 * c + 4 * g);
      v4i acc = v4i{nrowterm - ck[0], nrowterm - ck[1], nrowterm - ck[2], nrowterm - ck[3]};
      const v4i ka = *reinterpret_cast<const v4i*>(Ks + c * 1024 + fo);
      acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(ka, qb, acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        v2f_t y = v2f_t{(float)acc[r], (float)acc[r + 1]} * v2f_t{a.s_qkd, a.s_qkd};
        if (c == NT - 1) {  // the tile with pads (keys 197 .. 207): -inf, float max
          const int n0 = 192 + 8 * (r >> 1) + 2 * g;
          y = y + v2f_t{n0 < T ? 0.0f : -__builtin_inff(), n0 + 1 < T ? 0.0f : -__builtin_inff()};
          mx = __builtin_fmaxf(mx, __builtin_fmaxf(y[0], y[1]));
        } else {
          imx = max(imx, max(acc[r], acc[r + 1]));
          imn = min(imn, min(acc[r], acc[r + 1]));
        }
        e[c][r] = y[0];
        e[c][r + 1] = y[1];
      }
    }
    if (NQK_ATTN16_QPF && rt + NW < NT) qnext = q_frag(rt + NW);
    mx = __builtin_fmaxf(mx, (float)imx * a.s_qkd);
    mx = __builtin_fmaxf(mx, xor16f(mx));
    mx = __builtin_fmaxf(mx, xor32f(mx));
    const float nm = -mx;
    const float mn = (float)imn * a.s_qkd;
    // every argument of tiles 0..11 in [-86.5, 0] in all lanes: NumPy's exp by np_expf_safe2;
    // tile 12 (pads: -inf) and any other row by np_expf_nonpos2 (both equal NumPy's exp)
    const bool esafe = __all(mn + nm >= NP_EXP_SAFE_LO);
    // (tile by tile, pair by pair: a two-pair form with both chains interleaved in the source (s_nop
    // 495 -> 70 in the kernel) and one branch hoisted over tiles 0..11 measured slower, 143 -> 165 us:
    // profiles/r06_attn16.txt — at four waves per SIMD the other waves fill the hazard wait states)
#pragma unroll
    for (int c = 0; c < NT; ++c) {
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const v2f_t xa = v2f_t{e[c][r], e[c][r + 1]} + v2f_t{nm, nm};
        const v2f_t x = (c < NT - 1 && esafe) ? np_expf_safe2(xa) : np_expf_nonpos2(xa);
        e[c][r] = x[0];
        e[c][r + 1] = x[1];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- NumPy's pairwise sum: leaf 0 = tiles 0..5, leaf 1 = tiles 6..11 + keys 192..196
    float tot;
    {
      v2f_t a0 = v2f_t{e[0][0], e[0][1]}, a1 = v2f_t{e[6][0], e[6][1]};
      a0 = a0 + v2f_t{e[0][2], e[0][3]};
      a1 = a1 + v2f_t{e[6][2], e[6][3]};
#pragma unroll
      for (int c = 1; c < 6; ++c) {
        a0 = a0 + v2f_t{e[c][0], e[c][1]};
        a0 = a0 + v2f_t{e[c][2], e[c][3]};
        a1 = a1 + v2f_t{e[c + 6][0], e[c + 6][1]};
        a1 = a1 + v2f_t{e[c + 6][2], e[c + 6][3]};
      }
      float s0 = a0[0] + a0[1], s1 = a1[0] + a1[1];  // r_2g + r_2g+1
      s0 = s0 + xor16f(s0);
      s1 = s1 + xor16f(s1);
      s0 = s0 + xor32f(s0);
      s1 = s1 + xor32f(s1);
      // the tail of leaf 1 in order (correct in lane group 0: 192, 193 its own, 194, 195 group 1's,
      // 196 group 2's), then the total broadcast from group 0
      const float x0 = e[NT - 1][0], x1 = e[NT - 1][1];
      const float p0 = xor16f(x0), p1 = xor16f(x1), z0 = xor32f(x0);
      s1 = ((((s1 + x0) + x1) + p0) + p1) + z0;
      float t0 = s0 + s1;
      const float t1 = xor16f(t0);
      t0 = g == 1 ? t1 : t0;
      const float t2 = xor32f(t0);
      tot = g >= 2 ? t2 : t0;
    }
    const double rtot = 1.0 / (double)tot;
    const float kpf = (float)(rtot * a.rs_p);
    // ---- P = quantize(e / tot) (k_attention's two FAST forms and filters), 4 bytes per tile
    const bool pq_nc = pqlo <= 0.0f && __all(kpf <= pqhi);
    uint32_t dw[NT];
    int rp = 0;
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      const v2f_t e0 = v2f_t{e[c][0], e[c][1]}, e1 = v2f_t{e[c][2], e[c][3]};
      float worst;
      uint32_t w;
      if (pq_nc) {
        const v2f_t k2 = v2f_t{kpf, kpf}, m2 = v2f_t{pmagic, pmagic};
        const v2f_t s0 = __builtin_elementwise_fma(e0, k2, m2), s1 = __builtin_elementwise_fma(e1, k2, m2);
        const v2f_t dd0 = __builtin_elementwise_fma(e0, k2, -(s0 - m2));
        const v2f_t dd1 = __builtin_elementwise_fma(e1, k2, -(s1 - m2));
        const v2f_t r0 = s0 - m2, r1 = s1 - m2;
        worst = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaf(__builtin_fabsf(r0[0]), NQK_ATTN_PM_R, __builtin_fabsf(dd0[0])),
                                                __builtin_fmaf(__builtin_fabsf(r0[1]), NQK_ATTN_PM_R, __builtin_fabsf(dd0[1]))),
                                __builtin_fmaxf(__builtin_fmaf(__builtin_fabsf(r1[0]), NQK_ATTN_PM_R, __builtin_fabsf(dd1[0])),
                                                __builtin_fmaf(__builtin_fabsf(r1[1]), NQK_ATTN_PM_R, __builtin_fabsf(dd1[1]))));
        w = pack4_low(s0, s1);
      } else {
        v2f_t dd0, dd1;
        const v2f_t tf0 = e0 * v2f_t{kpf, kpf}, tf1 = e1 * v2f_t{kpf, kpf};
        const v2f_t s0 = round_magic2(tf0, pqlo, pqhi, pmagic, dd0);
        const v2f_t s1 = round_magic2(tf1, pqlo, pqhi, pmagic, dd1);
        worst = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaf(__builtin_fabsf(tf0[0]), NQK_ATTN_PM_T, __builtin_fabsf(dd0[0])),
                                                __builtin_fmaf(__builtin_fabsf(tf0[1]), NQK_ATTN_PM_T, __builtin_fabsf(dd0[1]))),
                                __builtin_fmaxf(__builtin_fmaf(__builtin_fabsf(tf1[0]), NQK_ATTN_PM_T, __builtin_fabsf(dd1[0])),
                                                __builtin_fmaf(__builtin_fabsf(tf1[1]), NQK_ATTN_PM_T, __builtin_fabsf(dd1[1]))));
        w = pack4_low(s0, s1);
      }
      if (c == NT - 1) {  // pad keys: P = 0
        uint32_t keep = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) keep |= (192 + 8 * (r >> 1) + 2 * g + (r & 1) < T ? 0xffu : 0u) << (8 * r);
        w &= keep;
      }
      if (__builtin_expect(__any(!(worst < 0x1.fffff8p-2f)), 0)) {
        // the exact chain for the elements the filter could not decide (k_attention's fallbacks)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = 16 * c + 8 * (r >> 1) + 2 * g + (r & 1);
          const float x = e[c][r];
          bool slow;
          if (pq_nc) {
            const float rr = __builtin_fmaf(x, kpf, pmagic) - pmagic;
            const float d = __builtin_fmaf(x, kpf, -rr);
            slow = !(__builtin_fmaf(__builtin_fabsf(rr), NQK_ATTN_PM_R, __builtin_fabsf(d)) < 0x1.fffff8p-2f);
          } else {
            const float tf = x * kpf;
            const float cf = __builtin_amdgcn_fmed3f(tf, pqlo, pqhi);
            const float dv = __builtin_fabsf(cf - __builtin_rintf(cf));
            slow = !(__builtin_fmaf(__builtin_fabsf(tf), NQK_ATTN_PM_T, dv) < 0x1.fffff8p-2f);
          }
          if (slow) {
            const int qv = n < T ? quant_w(div_rc_w(x, rtot), a.s_p, a.rs_p, a.zp_p, a.lo, a.hi) : 0;
            w = (w & ~(0xffu << (8 * r))) | ((uint32_t)(qv & 0xff) << (8 * r));
          }
        }
      }
      dw[c] = w;
      rp = __builtin_amdgcn_sdot4((int)w, 0x01010101, rp, false);
    }
    rp += xor16i(rp);
    rp += xor32i(rp);
    // ---- context O^T = V^T P^T: chunk ch of 64 keys = this lane's P dwords of tiles 4 ch .. 4 ch + 3
    v4i acc2[4];
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) acc2[mm] = v4i{0, 0, 0, 0};
#pragma unroll
    for (int ch = 0; ch < 4; ++ch) {
      const v4i pb = v4i{(int)dw[4 * ch], 4 * ch + 1 < NT ? (int)dw[4 * ch + 1] : 0, 4 * ch + 2 < NT ? (int)dw[4 * ch + 2] : 0,
                         4 * ch + 3 < NT ? (int)dw[4 * ch + 3] : 0};
#pragma unroll
      for (int mm = 0; mm < 4; ++mm) {
        const v4i va = *reinterpret_cast<const v4i*>(Vt + (ch * 64 + 16 * mm) * 64 + fo);
        acc2[mm] = __builtin_amdgcn_mfma_i32_16x16x64_i8(va, pb, acc2[mm], 0, 0, 0);
      }
    }
    // ---- dequantize + quantize the context (k_attention's ctx_store): dims 16 mm + 4 g .. + 3
    const int rowp = rp * a.zv;
    int8_t* orow = ctx + ((int64_t)img * T + m) * a.ld_out + head * 64;
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) {
      const int d0 = 16 * mm + 4 * g;
      const v4i cv = *reinterpret_cast<const v4i*>(colV + d0);
      float o[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) o[jj] = (float)(acc2[mm][jj] - rowp - cv[jj]) * a.s_pv;
      v2f_t dd0, dd1;
      const v2f_t t0 = v2f_t{o[0], o[1]} * v2f_t{a.rs_ctx_f, a.rs_ctx_f};
      const v2f_t t1 = v2f_t{o[2], o[3]} * v2f_t{a.rs_ctx_f, a.rs_ctx_f};
      const v2f_t s0 = round_magic2(t0, a.lo_f - a.zp_ctx_f, a.hi_f - a.zp_ctx_f, 0x1.8p23f + a.zp_ctx_f, dd0);
      const v2f_t s1 = round_magic2(t1, a.lo_f - a.zp_ctx_f, a.hi_f - a.zp_ctx_f, 0x1.8p23f + a.zp_ctx_f, dd1);
      const float m0 = __builtin_fmaf(__builtin_fabsf(t0[0]), 0x1p-21f, __builtin_fabsf(dd0[0]));
      const float m1 = __builtin_fmaf(__builtin_fabsf(t0[1]), 0x1p-21f, __builtin_fabsf(dd0[1]));
      const float m2 = __builtin_fmaf(__builtin_fabsf(t1[0]), 0x1p-21f, __builtin_fabsf(dd1[0]));
      const float m3 = __builtin_fmaf(__builtin_fabsf(t1[1]), 0x1p-21f, __builtin_fabsf(dd1[1]));
      const uint32_t wm = __builtin_elementwise_max(__builtin_elementwise_max(__float_as_uint(m0), __float_as_uint(m1)),
                                                    __builtin_elementwise_max(__float_as_uint(m2), __float_as_uint(m3)));
      uint32_t packed = pack4_low(s0, s1);
      if (__builtin_expect(__any(wm >= __float_as_uint(0x1.fffffcp-2f)), 0)) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int qv = quant_w(o[jj], a.s_ctx, a.rs_ctx, a.zp_ctx, a.lo, a.hi);
          packed = (packed & ~(0xffu << (8 * jj))) | ((uint32_t)(qv & 0xff) << (8 * jj));
        }
      }
      if (m < T) *reinterpret_cast<uint32_t*>(orow + d0) = packed;
    }
  }
}
}  // namespace
}  // namespace nqk

using namespace nqk;

extern "C" int nqk_attention_fused(const int8_t* q, const int8_t* k, const int8_t* v, int8_t* ctx,
                                   int64_t batch_heads, const nqk_attention* p) {
  if (batch_heads <= 0) return 0;
  const int T = p->tokens;
  if (p->hdim != 64) return fail("nqk_attention_fused: head dimension 64 expected");
  if (T < 1 || T > 224) return fail("nqk_attention_fused: 1 <= tokens <= 224 expected");
  if (p->heads < 1 || batch_heads % p->heads) return fail("nqk_attention_fused: batch_heads % heads != 0");
  if (p->ld_out < p->heads * 64) return fail("nqk_attention_fused: ld_out < heads * 64");
  if (p->bit_width < 2 || p->bit_width > 8) return fail("nqk_attention_fused: 2 <= bit_width <= 8 expected");
  auto small = [](int64_t z, int64_t lim) { return z >= -lim && z <= lim; };
  if (!small(p->zq, 4096) || !small(p->zk, 4096) || !small(p->zp_p, 1024) || !small(p->zv, 1024))
    return fail("nqk_attention_fused: zero points beyond the int32-exact range");
  if ((((uintptr_t)q) | ((uintptr_t)k) | ((uintptr_t)v)) & 15) return fail("nqk_attention_fused: unaligned Q/K/V");
  if ((((uintptr_t)ctx) & 3) || (p->ld_out & 3)) return fail("nqk_attention_fused: ctx / ld_out not 4-byte aligned");
  auto normal = [](float x) { return __builtin_fabsf(x) >= 0x1p-100f && __builtin_fabsf(x) <= 0x1p100f; };
  if (!normal(p->s_p) || !normal(p->s_ctx) || !normal(p->div))
    return fail("nqk_attention_fused: scales / divisor outside [2^-100, 2^100]");
  if (batch_heads > 0x7fffffff) return fail("nqk_attention_fused: too many (image, head) pairs");
  const int NT = (T + 31) / 32;
  AttnArgs a{};
  a.T = T;
  a.H = p->heads;
  a.ld_out = p->ld_out;
  int est = (T + 3) / 4 * 4;
  if (((est / 4) & 1) == 0) est += 4;  // odd multiple of 4 floats: conflict-free b128 row reads
  a.EST = est;
  a.PST = NT * 32 + 16;
  a.n2 = 0;
  if (T > 128) {
    a.n2 = T / 2;
    a.n2 -= a.n2 % 8;
  }
  a.zq = (int)p->zq;
  a.zk = (int)p->zk;
  a.zp = (int)p->zp_p;
  a.zv = (int)p->zv;
  a.kq = a.zq * a.zk * 64;
  a.kp = a.zp * a.zv * T;
  a.s_qk = p->s_qk;
  a.div = p->div;
  a.rdiv = 1.0 / (double)p->div;
  a.s_p = p->s_p;
  a.rs_p = 1.0 / (double)p->s_p;
  a.zp_p = (double)p->zp_p;
  a.s_pv = p->s_pv;
  a.s_ctx = p->s_ctx;
  a.rs_ctx = 1.0 / (double)p->s_ctx;
  a.zp_ctx = (double)p->zp_ctx;
  a.lo = -__builtin_ldexp(1.0, p->bit_width - 1);
  a.hi = __builtin_ldexp(1.0, p->bit_width - 1) - 1.0;
  a.inv_div = 1.0f / p->div;
  a.s_qkd = p->s_qk * a.inv_div;
  a.rs_ctx_f = (float)a.rs_ctx;
  a.zp_p_f = (float)p->zp_p;
  a.zp_ctx_f = (float)p->zp_ctx;
  a.lo_f = (float)a.lo;
  a.hi_f = (float)a.hi;
  // FAST: |acc - zero-point term| < 2^24 for the scores and the context (f32 dequant is
  // then the f64 one), the Div is an exact power of two, |zp_ctx| small
  const double qm = __builtin_ldexp(1.0, p->bit_width - 1);
  const double bs = 64.0 * (qm * qm + qm * (double)(llabs(p->zq) + llabs(p->zk)) + (double)llabs(p->zq * p->zk));
  const double bp = (double)T * (qm * qm + qm * (double)(llabs(p->zp_p) + llabs(p->zv)) + (double)llabs(p->zp_p * p->zv));
  int dexp = 0;
  const float dm = frexpf(p->div, &dexp);
  const bool fast = bs < 16777216.0 && bp < 16777216.0 && dm == 0.5f && llabs(p->zp_ctx) < (1 << 20) &&
                    normal(a.s_qkd) && normal(p->s_qk) && a.s_qkd > 0.0f &&
                    !getenv("NQK_ATTN_EXACT");
  const size_t shm = (size_t)NT * 32 * 64 + (size_t)64 * a.PST + 256 + (size_t)(NT * 32 + 64) * 4;
  const dim3 grid((unsigned)batch_heads);
  const size_t shm_tail = shm + attn_tail_lds<7, 197, true>();
  // round 6: the 16x16x64 four-lanes-per-row kernel for T = 197 FAST (NQK_ATTN16=0 keeps k_attention;
  // on the bench's data 154 -> 143 us, profiles/r06_attn16.txt)
  const char* a16v = getenv("NQK_ATTN16");
  const bool a16 = a16v == nullptr || atoi(a16v) != 0;
  if (T == 197 && fast && a16) {
    // NQK_ATTN16_NW=5: five waves per workgroup (A/B variant)
    const char* nwv = getenv("NQK_ATTN16_NW");
    const int nw = nwv ? atoi(nwv) : 4;
    if (nw == 5)
      hipLaunchKernelGGL(k_attn16<5>, grid, dim3(320), attn16_lds(), stream(), q, k, v, ctx, a);
    else
      hipLaunchKernelGGL(k_attn16<4>, grid, dim3(256), attn16_lds(), stream(), q, k, v, ctx, a);
    return launch_status("nqk_attention_fused(16)");
  }
  switch (T == 197 ? (fast ? -1 : 0) : NT) {
#define A(n) case n: hipLaunchKernelGGL((k_attention<n, 0, false>), grid, dim3(256), shm, stream(), q, k, v, ctx, a); break;
    case -1:  // ViT at 224 px (196 patches + CLS): the pairwise plan and pads fold at compile time
      hipLaunchKernelGGL((k_attention<7, 197, true>), grid, dim3(256), shm_tail, stream(), q, k, v, ctx, a);
      break;
    case 0:
      hipLaunchKernelGGL((k_attention<7, 197, false>), grid, dim3(256), shm, stream(), q, k, v, ctx, a);
      break;
    A(1) A(2) A(3) A(4) A(5) A(6) A(7)
#undef A
    default: return fail("nqk_attention_fused: bad tile count");
  }
  return launch_status("nqk_attention_fused");
}
