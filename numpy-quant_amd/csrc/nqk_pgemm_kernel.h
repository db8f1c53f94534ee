// nqk_pgemm_kernel.h — k_pg, the kernel template; its instantiations are spread over
// nqk_pg_inst_*.hip (parallel builds), the host launcher and the weight packers are nqk_pgemm.hip.
//
// k_pg: the round-3 persistent projection GEMM of the fused ViT layer (the hot loop of
// numpy_quantization.py:44-61 q_matmul for every act x W MatMul, with the consumer chain of
// model.py:486-565 in the epilogue: QKV head split + quantize, FFN-up + GELU + quantize,
// out-projection / FFN-down + bias + residual).
//
// Why this shape (measured on MI355X, tools/micro/fill.hip, tools/micro/xwave.hip,
// profiles/r03_*):
//  * v_mfma_i32_16x16x64_i8 sustains 3.9 POPS on random operands against 3.26 for the
//    32x32x32 form: the chip holds ~1.95 GHz under it instead of ~1.6 (same cycles per op).
//  * A SIMD overlaps one wave's MFMAs with VALU work (its own or another wave's) up to
//    ~4-6 VALU per 32x32x32-equivalent; past that the VALU issue (≈4 cycles each) sets
//    the pace.  The epilogues are VALU work, so: two independent 4-wave workgroups per CU
//    (128 x 256 tiles), the second started half a tile later, so that one workgroup's
//    epilogue runs beside the other's k loop; and epilogues with fewer VALU per element
//    (zero-point column term as the MFMA's initial accumulator, one fma for the QKV
//    rescale, a single measure per element for the rounding filter).
//
// Layout: 4 waves side by side along N, each 128 rows x 64 columns = 8 x 4 MFMA tiles of
// 16 x 16 (acc[i][j], 4 registers).  The products are computed transposed (Bt fragment as
// the MFMA's A operand), and the weight image stores the 64 columns of a wave permuted
// (bperm), so that lane l holds, for M-subtile i, row 16 i + (l & 15) and the 16
// CONSECUTIVE columns 16 (l >> 4) + 4 j + r: one 16-byte store per subtile (int8 outputs)
// or four (f32), straight from the accumulators.
// A [M][K] int8 (activations) and the tile-packed weight image both go HBM/L2 -> LDS by
// buffer LDS-DMA into a 3-stage ring (24 KiB per 64-deep k-step); the 16-B chunks are
// XOR-swizzled (sw) so the fragment reads are conflict-free ds_read_b128.  Every VMEM
// operation of the loop is counted by compile-time vmcnt waits; LDS reads are inline asm
// (a compiler-visible read of LDS-DMA'd bytes gets a vmcnt(0) that would drain the ring).
#pragma once
#include <type_traits>

#include "nqk_common.h"
#include "nqk_numerics.h"
#include "nqk_glut.h"

namespace nqk {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
typedef float v2f __attribute__((ext_vector_type(2)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int PG_BM = 128, PG_BN = 256, PG_BK = 64, PG_RD = 3;
constexpr int PG_ASTG = PG_BM * PG_BK;           // 8 KiB
constexpr int PG_STG = PG_ASTG + PG_BN * PG_BK;  // 24 KiB
constexpr int PG_COLP = PG_RD * PG_STG;          // 2 slots x (ct[256] int32 | bias[256] f32)
constexpr int PG_LDS = PG_COLP + 2 * 2048;       // 76 KiB: two workgroups per CU
constexpr int PG_PW = 2 + 4;                      // LDS-DMA pieces per wave per stage

enum { PG_QKV = 0, PG_RESID = 3, PG_GELU = 4 };  // = the EPI_* codes of nqk_fused.hip
constexpr int PG_GLUT = 5;  // GELU by table lookup (nqk_glut.h): launched for PG_GELU when a table is given
constexpr int PG_GLUT1 = 6;  // ... with a single-line bucket coordinate (round 5: one pk_fma + the max fewer)
constexpr bool pg_is_glut(int epi) { return epi == PG_GLUT || epi == PG_GLUT1; }
// k_pg's LDS: a 3-stage ring of A (128 x 64 B) + B (256 rows x 64 B, or 32 B of int4
// nibbles) per stage, the column constants (2 x 2 KiB), then the GELU table (PG_GLUT, 4 KiB)
// or, for int4 weights, the residual epilogue's transpose scratch (int8: ring slot 2)
constexpr int PG_TR_ROW = 272;  // bytes per staged residual row (256 + 16: conflict-free b128 writes)
// WM = 2 (round 5): one 512-thread workgroup per CU on 256 x 256 tiles — waves 0..3 rows 0..127,
// waves 4..7 rows 128..255 of the tile, both halves reading the SAME B stage: 32 KiB per k step
// per CU for 2 x 128 x 256 outputs instead of 2 x 24 KiB (the operand stream measured ~1/3 of
// FFN-down's time, profiles/r04_pg_operand_probe.txt); the residual transposes get their own LDS
#ifndef NQK_PG_WM2_RD
#define NQK_PG_WM2_RD 3  // ring depth of the 256 x 256 form's non-residual instances (4 fits its LDS)
#endif
// ring depth: 3 stages, or NQK_PG_WM2_RD for the 256 x 256 form where K is a multiple of 4 k steps
constexpr int pg_rd(int epi, int wm, int nk) { return (wm == 2 && epi != PG_RESID && nk % 4 == 0) ? NQK_PG_WM2_RD : PG_RD; }
constexpr int pg_stg(bool b4, int wm = 1) { return (wm ? PG_ASTG * wm : PG_ASTG / 2) + PG_BN * (b4 ? PG_BK / 2 : PG_BK); }
constexpr int pg_colp(bool b4, int wm = 1, int rd = PG_RD) { return rd * pg_stg(b4, wm); }
constexpr int pg_lds_bytes(int epi, bool b4, int wm = 1, int nk = 12) {
  return pg_colp(b4, wm, pg_rd(epi, wm, nk)) + 4096 + (pg_is_glut(epi) ? 8 * (wm == 2 ? GLUT_MAX : GLUT_CAP1) : 0) +
         ((b4 || wm == 2) && epi == PG_RESID ? 4 * wm * 16 * PG_TR_ROW : 0);
}

#ifndef NQK_PG_STAUX
#define NQK_PG_STAUX 2  // cache-policy bits of the epilogue's output stores: nt (profiles/r03c_*: out-proj
                        // 77 -> 60 us; 16 = sc1, the line leaves L2: no gain)
#endif
#ifndef NQK_PG_STAUX_RESID
#define NQK_PG_STAUX_RESID 0  // the residual epilogues' f32 output stores: plain, so the LayerNorm that
                              // reads the rows next finds them in the Infinity Cache (same-box bench A/B,
                              // profiles/r03_store_policy_ab.txt: LN 46.4 -> 42.1 us, residual GEMMs equal)
#endif
#ifndef NQK_PG_RLAUX
#define NQK_PG_RLAUX -1  // cache-policy bits of the RESID epilogue's residual loads: -1 = nt for K = 3072
                         // (FFN-down 144 -> 138 us) and plain for K = 768 (nt: out-proj 59 -> 70 us)
#endif
#ifndef NQK_PG_RESQ
#define NQK_PG_RESQ 3  // the residual epilogue's subtiles of residual rows in flight (round 6 A/B: 4)
#endif
#ifndef NQK_PG_RDIRECT
#define NQK_PG_RDIRECT 0  // 1: the residual epilogue straight from the accumulator layout (no LDS transposes),
                          // so ring slot 2 is free and all three stages of the next tile go out before the
                          // epilogue's stores (round 6 A/B)
#endif
#ifndef NQK_PG_SPREAD
#define NQK_PG_SPREAD 0  // 1: the stage's LDS-DMA pieces spread over the first half step (A/B variant)
#endif
#ifndef NQK_PG_GELU4
#define NQK_PG_GELU4 1  // GELU epilogue two element pairs at a time, the chains interleaved
#endif
#ifndef NQK_PG_NOPK
#define NQK_PG_NOPK 1  // 1: the QKV epilogue without packed f32 instructions (MI355X_MICROARCH.md:
                       // beside MFMAs a v_pk_fma_f32 costs more than two v_fma_f32): QKV 97 -> 92 us
#endif

#ifndef NQK_PG_PRIO
#define NQK_PG_PRIO 3  // 3: s_setprio 1 in the epilogue, 0 in the k loop (the epilogue's VALU ahead of the
                       // other workgroup's k loop on the SIMD: -2..-4 %, profiles/r03c_*); 1: the reverse;
                       // 2: static prio 1 for the second workgroup of a CU; 0: none
#endif
#ifndef NQK_PG_DIAG
#define NQK_PG_DIAG 0  // diagnostic builds only (tools/pg_diag.sh): 1 = no epilogue stores,
                       // 2 = trivial epilogue math, 4 = no operand loads, 8 = no barriers,
                       // 16 = no fragment reads, 4096 = no residual loads (zeros)
#endif

// physical 16-B chunk of logical chunk c in 64-B LDS row r is c ^ pg_sw(r): the 16 lanes of
// each ds_read_b128 lane group (rows 16 i + (l & 15), chunk l >> 4) then hit 16 different
// 4-bank slots
__host__ __device__ constexpr int pg_sw(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }
// column (within the wave's 64) held by the wave's LDS B row rw = 16 j + c.  Layout 0 (int8
// outputs): lane (l & 15, lg = l >> 4) gets columns 16 lg + 4 j + r, 16 consecutive bytes;
// layout 1 (f32 outputs): columns 16 j + 4 lg + r, so each 16-B store instruction j covers
// 64 contiguous bytes of a row with the 4 lanes of that row
__host__ __device__ constexpr int pg_bperm(int rw, int layout) {
  return layout == 0 ? 16 * ((rw & 15) >> 2) + 4 * (rw >> 4) + (rw & 3) : rw;
}

template <int I>
using ic = std::integral_constant<int, I>;
template <int B, int E, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < E) {
    f(ic<B>{});
    sfor<B + 1, E>(f);
  }
}

__device__ __forceinline__ rsrc_t pg_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void pg_dma16(rsrc_t r, void* l, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)l, 16, voff, soff, 0, 0);
}
// LDS reads are compiler-visible (it places the lgkmcnt waits; an async load's destination
// register must never be copied before its wait, which only the compiler can guarantee);
// the compiler does not order them behind LDS-DMA, the explicit vmcnt waits + barriers do
__device__ __forceinline__ v4i pg_lds16(const void* p) {
  return *reinterpret_cast<const v4i*>(p);  // p points into the kernel's LDS array: ds_read_b128
}
// ds_read_b128 at base + a compile-time byte offset (the instruction's 16-bit offset field:
// one address VGPR for every fragment read of the loop)
#ifndef NQK_PG_ASMREAD
#define NQK_PG_ASMREAD 0  // diagnostic: fragment reads by inline asm
#endif
template <int OFF>
__device__ __forceinline__ v4i pg_lds16o(const int8_t* base) {
  static_assert(OFF >= 0 && (OFF < 65536 || !NQK_PG_ASMREAD), "ds_read offset");
  if constexpr (NQK_PG_ASMREAD) {
    v4i v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"((uint32_t)(uintptr_t)(lds_ptr_t)base), "n"(OFF));
    return v;
  } else {
    return *reinterpret_cast<const v4i*>(base + OFF);  // the offset folds into the instruction
  }
}
// ds_read_b64 at base + a compile-time byte offset (the int4 weight fragments)
template <int OFF>
__device__ __forceinline__ v2u pg_lds8o(const int8_t* base) {
  return *reinterpret_cast<const v2u*>(base + OFF);
}
__device__ __forceinline__ void pg_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
// lgkmcnt(0) that the values read by pg_lds16 pass through: their uses cannot be moved
// above the wait (a plain wait orders only memory operations)
__device__ __forceinline__ void pg_lgkm_tie(v4i& a, v4i& b, v4i& c, v4i& d) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d)::"memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void pg_lgkm_tie_a4(v4i (&a)[4], v2u (&b)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3])::"memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void pg_lgkm_tie8(v4i (&a)[4], v4i (&b)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3])::"memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <int N>
__device__ __forceinline__ void pg_vmcnt_tie(v4u (&a)[4]) {
  asm volatile("s_waitcnt vmcnt(%4)" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]) : "n"(N > 63 ? 63 : N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <int N>
__device__ __forceinline__ void pg_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N > 63 ? 63 : N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
// 16-byte buffer load to VGPRs (compiler-visible: it places the vmcnt wait before the use)
template <int AUX = 0>
__device__ __forceinline__ v4u pg_load16(rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, AUX);
}
__device__ __forceinline__ v4u pg_load16(rsrc_t r, uint32_t voff, uint32_t soff, int aux) {
  return aux == 2 ? pg_load16<2>(r, voff, soff) : pg_load16<0>(r, voff, soff);
}

struct PgEpi {
  float sacc[3];      // dequant scale per column group
  float rsf[3];       // RN32(1 / s_out)
  float c1[3];        // RN32(sacc * rsf)            (QKV fast path)
  float k1[3];        // |c1| 6.25 2^-24             (QKV filter: rounding error per |v|)
  float zp128[3];     // zp_out + 128 (f32)        (QKV: v_rndne + v_cvt_pk_u8 rounding)
  float qlo[3], qhi[3], magic[3];  // lo - zp, hi - zp, 1.5 2^23 + zp (GELU: pg_round2)
  float s_out[3];
  double rs_out[3], zp_out[3];
  void* out[3];
  const float* bias;
  const float* resid;
  const int32_t* colterm;  // col[n] * zpa (int32)
  double lo, hi;
  int group_cols, tokens, heads, hdim;
  float g_rel, g_lim;  // GELU filter (nqk_fused.hip make_epi)
  float div, add1, mul2;
  double rdiv;
  int ldo;  // row stride (elements) of the GELU / RESID output
  const void* lut;  // PG_GLUT: the GELU table (nqk_gelu_lut_build) and its bucket coordinate
  uint32_t lut_bytes;  // 8 * lut_n rounded up to 16: the table's buffer range
  GLutK gk;
  float blo, bhi;   // QKV: the clamp of v + 128 ([lo + 128, hi + 128] of the bit width)
  int xcds;         // XCDs of the device (the band count of the XCD-aware tile order)
};

// quantize (numpy_quantization.py:24-34) with f64 zero-point add and clipping
__device__ __forceinline__ int pg_quant_exact(float x, float s, double rs, double zp, double lo, double hi) {
  (void)s;
  const float t = (float)((double)x * rs);  // RN32(x / s) (s normal, host-checked)
  const double u = zp + (double)t;
  return (int)__builtin_rint(__builtin_fmin(__builtin_fmax(u, lo), hi));
}

// per-column-group constants of the exact fallback
struct PgFix {
  float c1, k1, rsf, sacc, lim, s_out;
  double rs_out, zp;
};
// The rounding filter's exact fallback for element q of one epilogue step: recheck the
// element's filter measure, and run the reference chain where it could not decide.
// av: the int32 accumulators; xv: QKV the column bias, GELU h = RN(bias + RN(v sacc)).
template <int EPI>
__device__ __forceinline__ void pg_exact_fix1(int q, const int (&av)[16], const float (&xv)[16], uint32_t (&pk)[4],
                                              const PgFix& f, const PgEpi& e) {
  const float vf = (float)av[q];
  const float x = xv[q];
  bool slow;
  if constexpr (EPI == PG_QKV) {
    const float u = __builtin_fmaf(vf, f.c1, x * f.rsf);
    const float r = __builtin_rintf(u);
    slow = !(__builtin_fmaf(__builtin_fabsf(vf), f.k1, __builtin_fabsf(u - r)) < f.lim);
  } else {
    const float tf = gelu_fast(x) * f.rsf;
    const float r = __builtin_rintf(tf);
    slow = !(__builtin_fmaf(__builtin_fabsf(x), e.g_rel, __builtin_fabsf(tf - r)) < f.lim);
  }
  if (__any(slow)) {
    if (slow) {
      float y;
      if constexpr (EPI == PG_QKV) {
        y = x + vf * f.sacc;  // F32X: the f64 dequantize, exactly
      } else {
        y = x;
        const float aa = ref_erf((float)((double)y * e.rdiv)) + e.add1;
        y = (y * aa) * e.mul2;
      }
      const int qv = pg_quant_exact(y, f.s_out, f.rs_out, f.zp, e.lo, e.hi);
      const int sh = 8 * (q & 3);
      pk[q >> 2] = (pk[q >> 2] & ~(0xffu << sh)) | ((uint32_t)(qv & 0xff) << sh);
    }
  }
}
// ... for all 16 elements of the step (entered when any lane's worst measure fails).  GELU:
// a loop that is not unrolled (av / xv / pk indexed by the wave-uniform q stay in VGPRs via
// relative moves), so the long exact chain is not duplicated per element and per step; QKV:
// unrolled (its exact chain is short; measured faster, profiles/r03_pg_micro.txt).
// gm (QKV, and GELU with NQK_PG_GELU4): bit g set when some lane's filter measure of elements
// 4 g .. 4 g + 3 failed; the other groups are skipped (their elements all passed)
template <int EPI>
__device__ __forceinline__ void pg_exact_fix(const int (&av)[16], const float (&xv)[16], uint32_t (&pk)[4],
                                             const PgFix& f, const PgEpi& e, uint32_t gm = 15u) {
  if constexpr (EPI == PG_QKV) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if ((gm >> g) & 1u) {
#pragma unroll
        for (int j = 0; j < 4; ++j) pg_exact_fix1<EPI>(4 * g + j, av, xv, pk, f, e);
      }
    }
  } else {
#pragma clang loop unroll(disable)
    for (int q = 0; q < 16; ++q) {
      if ((gm >> (q >> 2)) & 1u) pg_exact_fix1<EPI>(q, av, xv, pk, f, e);
    }
  }
}

// gelu_fast (nqk_numerics.h) on two values with packed f32 arithmetic (v_pk_fma / v_pk_mul:
// one instruction for both lanes of the pair, the same IEEE operations in the same order as
// the scalar function, so the same bits: the epilogues are VALU-issue-bound and a packed
// instruction issues at the scalar rate, tools/micro/valu.hip)
__device__ __forceinline__ v2f gelu_fast2(v2f h) {
  const v2f ah = __builtin_elementwise_abs(h);
  const v2f d = __builtin_elementwise_fma(v2f{0.3275911f * 0.70710677f, 0.3275911f * 0.70710677f}, ah, v2f{1.0f, 1.0f});
  const v2f t = v2f{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  v2f p = __builtin_elementwise_fma(v2f{0.5f * 1.061405429f, 0.5f * 1.061405429f}, t,
                                    v2f{0.5f * -1.453152027f, 0.5f * -1.453152027f});
  p = __builtin_elementwise_fma(p, t, v2f{0.5f * 1.421413741f, 0.5f * 1.421413741f});
  p = __builtin_elementwise_fma(p, t, v2f{0.5f * -0.284496736f, 0.5f * -0.284496736f});
  p = __builtin_elementwise_fma(p, t, v2f{0.5f * 0.254829592f, 0.5f * 0.254829592f});
  const v2f ea = h * (h * v2f{-0.72134752f, -0.72134752f});
  const v2f ex = v2f{__builtin_amdgcn_exp2f(ea[0]), __builtin_amdgcn_exp2f(ea[1])};
  const v2f q = (p * t) * ex;
  return __builtin_elementwise_fma(-ah, q, __builtin_elementwise_max(h, v2f{0.0f, 0.0f}));
}

// gelu_fast2 on two element pairs with every step of the two chains side by side: the
// dependent packed instructions of one chain leave hazard wait states (s_nop) that the other
// chain's instruction fills (same operations per lane, same bits)
__device__ __forceinline__ void gelu_fast2x2(v2f h0, v2f h1, v2f& g0, v2f& g1) {
  const v2f c1 = v2f{0.3275911f * 0.70710677f, 0.3275911f * 0.70710677f}, one = v2f{1.0f, 1.0f};
  const v2f ah0 = __builtin_elementwise_abs(h0), ah1 = __builtin_elementwise_abs(h1);
  const v2f d0 = __builtin_elementwise_fma(c1, ah0, one), d1 = __builtin_elementwise_fma(c1, ah1, one);
  const v2f hc0 = h0 * v2f{-0.72134752f, -0.72134752f}, hc1 = h1 * v2f{-0.72134752f, -0.72134752f};
  const v2f t0 = v2f{__builtin_amdgcn_rcpf(d0[0]), __builtin_amdgcn_rcpf(d0[1])};
  const v2f t1 = v2f{__builtin_amdgcn_rcpf(d1[0]), __builtin_amdgcn_rcpf(d1[1])};
  const v2f ea0 = h0 * hc0, ea1 = h1 * hc1;
  const v2f k5 = v2f{0.5f * 1.061405429f, 0.5f * 1.061405429f}, k4 = v2f{0.5f * -1.453152027f, 0.5f * -1.453152027f};
  const v2f k3 = v2f{0.5f * 1.421413741f, 0.5f * 1.421413741f}, k2 = v2f{0.5f * -0.284496736f, 0.5f * -0.284496736f};
  const v2f k1 = v2f{0.5f * 0.254829592f, 0.5f * 0.254829592f};
  v2f p0 = __builtin_elementwise_fma(k5, t0, k4), p1 = __builtin_elementwise_fma(k5, t1, k4);
  const v2f ex0 = v2f{__builtin_amdgcn_exp2f(ea0[0]), __builtin_amdgcn_exp2f(ea0[1])};
  const v2f ex1 = v2f{__builtin_amdgcn_exp2f(ea1[0]), __builtin_amdgcn_exp2f(ea1[1])};
  p0 = __builtin_elementwise_fma(p0, t0, k3);
  p1 = __builtin_elementwise_fma(p1, t1, k3);
  p0 = __builtin_elementwise_fma(p0, t0, k2);
  p1 = __builtin_elementwise_fma(p1, t1, k2);
  p0 = __builtin_elementwise_fma(p0, t0, k1);
  p1 = __builtin_elementwise_fma(p1, t1, k1);
  const v2f pt0 = p0 * t0, pt1 = p1 * t1;
  const v2f q0 = pt0 * ex0, q1 = pt1 * ex1;
  const v2f z = v2f{0.0f, 0.0f};
  g0 = __builtin_elementwise_fma(-ah0, q0, __builtin_elementwise_max(h0, z));
  g1 = __builtin_elementwise_fma(-ah1, q1, __builtin_elementwise_max(h1, z));
}

// Q_LIM = (0.5 - 2^-126)(1 - 2^-23) rounded down: a rounded fma measure below it keeps the
// exact one below 0.5 - 2^-126 (nqk_fused.hip quant_filter)
constexpr float PG_QLIM = 0x1.fffffcp-2f;
// QKV filter margin (round 4): |u - t| <= 6 units (2^-24) of |v c1| + 5 of |c2| to first order —
// the roundings of c1 = RN(sacc rsf), rsf = RN(1/s) and the fma on the fast side, of v sacc,
// + bias and / s_out on the reference's — so 6.25 and 5.25 units (round 3 used 8 and 16)
#ifndef NQK_PG_QK1
#define NQK_PG_QK1 0x1.9p-22f  // 6.25 2^-24 per |v c1|
#endif
#ifndef NQK_PG_QKC2
#define NQK_PG_QKC2 0x1.5p-22f  // 5.25 2^-24 per |c2|
#endif


// B4: int4 weights (every value in [-8, 7]) as the nibble image of nqk_pack_pg4: a stage's
// B part is 256 rows x 32 bytes (half the LDS-DMA pieces and LDS bytes); a lane's 16 k-values
// of one MFMA operand are 8 bytes (ds_read_b64) that unpack with two AND masks into bytes
// 16 w (the nibble in the high half, its sign bit on the byte's; as nqk_fused.hip
// k_qgemm_big), so the MFMAs accumulate 16 acc exactly (initial accumulators 16 x the column
// terms, host-checked to fit int32) and the epilogue takes acc >> 4.
// S8 (QKV with 8-bit outputs): v_cvt_pk_u8_f32 saturates to [0, 255] (tools/micro/cvtu8.hip:
// every integral f32 in [-2^24, 2^24], profiles/r04_cvtu8.txt), which is then the clamp, so the
// v_med3 before it goes.
// RB (round 5, K = 192 = three k steps: ViT-Ti): the whole K of a tile fits the ring, so the
// weight panel stays RESIDENT — tiles are numbered column-panel major, a workgroup reloads B only
// when its next tile is in another panel, and streams only A (24 KiB -> 8 KiB of operand bytes
// per tile: one third); the k loop runs without loads or barriers, the next tile's A is issued
// right after it, under the epilogue.
// WM = 0 (round 5, K = 192: ViT-Ti's QKV and FFN-up; opt-in NQK_PG_WM0=1): 64-row tiles — twice
// the tiles, for a less partial last pass of the persistent grid (ViT-Ti B = 256: 2 364 tiles = 4.6
// passes instead of 1 182 = 2.3); one A piece per wave per stage, the k step's 16 MFMAs (subtiles
// 0..3) split 8 + 8 around the stage wait.  Measured slower (the 128-row form's time is linear in its
// tiles; 64-row tiles read B twice per output), profiles/r05_pg_rows64_dropped.txt.
template <int EPI, int NK, bool F32X, bool B4, bool S8 = false, int WM = 1, bool RB = false>
__global__ void __launch_bounds__(256 * (WM == 2 ? 2 : 1), WM == 2 ? 1 : 2)
k_pg(const int8_t* __restrict__ A, const int8_t* __restrict__ Bp, int M, int N, int lda, int tiles_n, int ntiles,
     PgEpi e) {
  constexpr int RD = RB ? PG_RD : pg_rd(EPI, WM, NK);  // ring stages
  static_assert(NK % RD == 0 && (NK >= 2 * RD || NK == RD), "k_pg: NK a multiple of the ring depth");
  static_assert(RD == PG_RD || EPI != PG_RESID, "k_pg: the residual epilogue borrows ring slot 2 (3 stages)");
  static_assert(WM == 0 || WM == 1 || WM == 2, "k_pg: a 64-row tile, or one or two 128-row halves per tile");
  static_assert(WM != 0 || (!B4 && !RB && EPI != PG_RESID), "k_pg<WM = 0>: int8, QKV / GELU only");
  constexpr int WQ = WM == 2 ? 2 : 1;            // 4-wave groups per workgroup
  constexpr int APW = WM == 0 ? 1 : 2;           // A LDS-DMA pieces per wave per stage
  constexpr int MS = WM == 0 ? 4 : 8;            // 16-row subtiles of a wave
  static_assert(!RB || (NK == PG_RD && !B4 && EPI != PG_RESID), "k_pg<RB>: K = 3 k steps, int8, not residual");
  constexpr bool RESID = EPI == PG_RESID;
  constexpr int BM = WM ? PG_BM * WM : 64;      // tile rows
  constexpr int ASTG = WM ? PG_ASTG * WM : PG_ASTG / 2;  // A bytes of a stage
  constexpr int BROW = B4 ? PG_BK / 2 : PG_BK;  // bytes of one B row per k-step
  constexpr int NBP = (B4 ? 2 : 4) / WQ;        // B LDS-DMA pieces per wave per stage
  constexpr int STG = pg_stg(B4, WM), COLP = pg_colp(B4, WM, RD), LUTO = COLP + 4096;
  constexpr int PW = APW + NBP;                 // LDS-DMA pieces per wave per stage
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) & (4 * WQ - 1));
  const int wn = wave & 3, wm = WM == 2 ? wave >> 2 : 0;  // column quarter / row half of the tile
  const int l15 = lane & 15, lg = lane >> 4;

  // tiles: the workgroups with blockIdx % 8 == x (one XCD under round-robin placement)
  // walk the band [lo, hi) of tile ids, every nx-th tile from lo + jx; tile ids are
  // row-panel major, so the tiles in flight on an XCD share A row panels in its L2.
  const int G = gridDim.x, X = G < e.xcds ? G : e.xcds, x = blockIdx.x % X;
  const int nx = (G - x + X - 1) / X;
  const int lo = (int)((int64_t)ntiles * x / X), hi = (int)((int64_t)ntiles * (x + 1) / X);
  const int first = lo + (int)(blockIdx.x / X);
  const int iters = first < hi ? (hi - first + nx - 1) / nx : 0;
  if (iters == 0) return;
  auto tile_at = [&](int it) { return first + (it < iters ? it : iters - 1) * nx; };

  constexpr int64_t BSTRIDE = (int64_t)NK * PG_BN * BROW;  // bytes of one column panel
  const rsrc_t r_a = pg_rsrc(A, (uint32_t)((uint64_t)M * lda));
  const rsrc_t r_b = pg_rsrc(Bp, (uint32_t)((uint64_t)tiles_n * BSTRIDE));
  // LDS-DMA sources: A piece pp of wave w = rows 32 w + 16 pp + (l >> 2), physical chunk l & 3
  const uint32_t va = (uint32_t)((16 * APW * wave + (lane >> 2)) * lda + 16 * ((lane & 3) ^ pg_sw(lane >> 2)));
  const uint32_t vb = (uint32_t)(NBP * 1024 * wave + 16 * lane);
  // fragment offsets: row (l & 15) of a 16-row subtile, logical chunk l >> 4 (B4: 8-byte
  // chunks of 32-byte rows, chunk ^ 2 in rows 8..15 of a subtile: conflict-free b64 reads)
  const int f_off = l15 * 64 + 16 * (lg ^ pg_sw(l15));
  const int f_off4 = l15 * 32 + 8 * (lg ^ (2 * ((l15 >> 3) & 1)));

  struct Src { uint32_t sa, sb; int r0, tn; };
  auto src_of = [&](int tile) __attribute__((always_inline)) {
    Src s;
    int tm;
    if constexpr (RB) {  // column-panel major: consecutive tiles share their weight panel
      const int tms = ntiles / tiles_n;
      s.tn = tile / tms;
      tm = tile - s.tn * tms;
    } else {
      tm = tile / tiles_n;
      s.tn = tile - tm * tiles_n;
    }
    // a ragged last tile row is computed as rows M - BM .. M - 1 (the rows it shares
    // with the tile above are written twice with the same values; host: out != resid)
    s.r0 = tm * BM < M - BM ? tm * BM : M - BM;
    s.sa = (uint32_t)s.r0 * (uint32_t)lda;
    s.sb = (uint32_t)((int64_t)s.tn * BSTRIDE);
    return s;
  };
  // LDS-DMA piece p of a stage (0, 1: A; 2 .. PW - 1: B)
  auto issue_piece = [&](const Src& s, int kt, int slot, int p) __attribute__((always_inline)) {
    if constexpr ((NQK_PG_DIAG & 4) != 0) return;
    int8_t* st = lds + slot * STG;
    if (p < APW) {
      if constexpr ((NQK_PG_DIAG & 512) != 0) {
        // (diagnostic 512, wrong values: the A piece as 8 rows x 128 B — whole cache lines, rows
        // 8 (kt & 1) .. + 7 of the piece's 16 at the k-pair's 128-B block — the same bytes per step in
        // half the L1 -> L2 requests)
        const uint32_t v512 = (uint32_t)((32 * wave + 16 * p + 8 * (kt & 1) + (lane >> 3)) * lda + (lane & 7) * 16);
        pg_dma16(r_a, st + (APW * wave + p) * 1024, v512, s.sa + (uint32_t)(kt & ~1) * PG_BK);
      } else if constexpr ((NQK_PG_DIAG & 256) == 0)  // (diagnostic 256: no A pieces, 128: no B pieces)
        pg_dma16(r_a, st + (APW * wave + p) * 1024, va, s.sa + (uint32_t)p * 16u * (uint32_t)lda + kt * PG_BK);
    } else {
      if constexpr ((NQK_PG_DIAG & 128) == 0)
        pg_dma16(r_b, st + ASTG + (NBP * wave + p - APW) * 1024, vb,
                 s.sb + (uint32_t)(kt * (PG_BN * BROW) + (p - APW) * 1024));
    }
  };
  auto issue_stage = [&](const Src& s, int kt, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < PW; ++p) issue_piece(s, kt, slot, p);
  };
  // column constants of a tile (ct[256] | bias[256], 2 KiB): wave w moves bytes
  // [512 w, 512 w + 512) with lanes 0..31 (WM = 2: [256 w, 256 w + 256) with lanes 0..15);
  // one VMEM operation per wave, like every wave
  const rsrc_t r_ct = pg_rsrc(e.colterm, (uint32_t)((uint64_t)N * 4));
  const rsrc_t r_bias = pg_rsrc(e.bias, e.bias ? (uint32_t)((uint64_t)N * 4) : 0u);
  auto issue_colp = [&](int tn, int cslot) __attribute__((always_inline)) {
    constexpr int CB = 512 / WQ, CL = 32 / WQ;  // bytes / lanes per wave
    int8_t* dst = lds + COLP + cslot * 2048 + wave * CB;
    const uint32_t voff = (uint32_t)((tn * PG_BN + (wave % (2 * WQ)) * (CB / 4) + (lane & (CL - 1)) * 4) * 4);
    if (lane < CL) {
      if (wave < 2 * WQ) pg_dma16(r_ct, dst, voff, 0);
      else pg_dma16(r_bias, dst, voff, 0);  // bias == null: the descriptor returns zeros
    }
  };

  v4i acc[8][4];
  v4i a_lo[4], a_hi[4], b0[4], b1[4];
  v2u p0[4], p1[4];  // B4: the packed fragments of the current / next step (b0 holds the unpacked ones)
  const int8_t* const fa_base = lds + f_off + PG_ASTG * wm;  // the wave's 128-row half of the A stage
  const int8_t* const fb_base = B4 ? lds + f_off4 + 2048 * wn : lds + f_off + 4096 * wn;
  // fragment reads: A subtile i (rows 16 i ..), B subtile j of the wave (rows 64 w + 16 j ..)
  auto rd_a = [&](v4i (&dst)[4], auto SLOT, auto I0, auto Q) __attribute__((always_inline)) {
    if constexpr ((NQK_PG_DIAG & 16) != 0) return;
    constexpr int q = decltype(Q)::value;
    dst[q] = pg_lds16o<decltype(SLOT)::value * STG + (decltype(I0)::value + q) * 1024>(fa_base);
  };
  auto rd_b = [&](v4i (&dst)[4], auto SLOT, auto Q) __attribute__((always_inline)) {
    if constexpr ((NQK_PG_DIAG & 16) != 0) return;
    constexpr int q = decltype(Q)::value;
    dst[q] = pg_lds16o<decltype(SLOT)::value * STG + ASTG + q * 1024>(fb_base);
  };
  // B4: 8 nibble bytes per fragment into the packed double buffer; unpack_b expands the
  // current step's after its wait into b0 (the only unpacked set)
  auto rd_b4 = [&](v2u (&dst)[4], auto SLOT, auto Q) __attribute__((always_inline)) {
    if constexpr ((NQK_PG_DIAG & 16) != 0) return;
    constexpr int q = decltype(Q)::value;
    dst[q] = pg_lds8o<decltype(SLOT)::value * STG + ASTG + q * 512>(fb_base);
  };
  auto unpack_b = [&](const v2u (&p)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      b0[q] = v4i{(int)((p[q][0] << 4) & 0xF0F0F0F0u), (int)(p[q][0] & 0xF0F0F0F0u), (int)((p[q][1] << 4) & 0xF0F0F0F0u),
                  (int)(p[q][1] & 0xF0F0F0F0u)};
  };
  // 16 MFMAs of one half step (M-subtiles 4 h .. 4 h + 3) with fn(q) after MFMA q
  auto half = [&](auto H, auto FIRST, const v4i (&aa)[4], const v4i (&bb)[4], const v4i (&ci)[4], auto&& fn)
      __attribute__((always_inline)) {
    constexpr int h = decltype(H)::value;
    sfor<0, 16>([&](auto Q) __attribute__((always_inline)) {
      constexpr int q = decltype(Q)::value, ii = q >> 2, j = q & 3;
      if constexpr (decltype(FIRST)::value)
        acc[4 * h + ii][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(bb[j], aa[ii], ci[j], 0, 0, 0);
      else
        acc[4 * h + ii][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(bb[j], aa[ii], acc[4 * h + ii][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      fn(Q);
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  // 8 MFMAs (subtiles 2 qi, 2 qi + 1) with fn(q) after MFMA q: the 64-row form (WM = 0)
  auto quarter = [&](auto QI, auto FIRST, const v4i (&aa)[4], const v4i (&bb)[4], const v4i (&ci)[4], auto&& fn)
      __attribute__((always_inline)) {
    constexpr int qi = decltype(QI)::value;
    sfor<0, 8>([&](auto Q) __attribute__((always_inline)) {
      constexpr int q = decltype(Q)::value, ii = 2 * qi + (q >> 2), j = q & 3;
      if constexpr (decltype(FIRST)::value)
        acc[ii][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(bb[j], aa[ii], ci[j], 0, 0, 0);
      else
        acc[ii][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(bb[j], aa[ii], acc[ii][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      fn(Q);
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  // ---------------------------------------------------------------- epilogue of a tile
  // rows r0 + 128 wm + 16 i + (l & 15), columns n0 + 64 wn + 16 (l >> 4) + 0..15
  auto epilogue = [&](const Src& s, int cslot) __attribute__((always_inline)) {
    const int n0 = s.tn * PG_BN;
    const int cw = n0 + 64 * wn;  // the wave's 64 columns: one head, one column group (host)
    const int col0 = cw + 16 * lg;
    const int8_t* cp = lds + COLP + cslot * 2048;
    // PG_GLUT: LDS byte address of entry 0 minus bits(GLUT_MAGIC) * 8 (one v_lshl_add per lookup)
    const uint32_t lut_base = (uint32_t)(uintptr_t)(lds_ptr_t)(lds + LUTO) - (GLUT_MAGIC_BITS << 3);
    float bias[16];
    {
      v4i bb[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) bb[g] = pg_lds16(cp + 1024 + (64 * wn + 16 * lg + 4 * g) * 4);
      pg_lgkm_tie(bb[0], bb[1], bb[2], bb[3]);
#pragma unroll
      for (int q = 0; q < 16; ++q) bias[q] = __int_as_float(bb[q >> 2][q & 3]);
    }
    {
      int g3 = 0;
      if constexpr (EPI == PG_QKV) {
        g3 = cw / e.group_cols;
        g3 = g3 > 2 ? 2 : g3;
      }
      const float sacc = g3 == 0 ? e.sacc[0] : (g3 == 1 ? e.sacc[1] : e.sacc[2]);
      const float rsf = g3 == 0 ? e.rsf[0] : (g3 == 1 ? e.rsf[1] : e.rsf[2]);
      const float c1 = g3 == 0 ? e.c1[0] : (g3 == 1 ? e.c1[1] : e.c1[2]);
      const float k1 = g3 == 0 ? e.k1[0] : (g3 == 1 ? e.k1[1] : e.k1[2]);
      const float zp128 = g3 == 0 ? e.zp128[0] : (g3 == 1 ? e.zp128[1] : e.zp128[2]);
      const float qlo = g3 == 0 ? e.qlo[0] : (g3 == 1 ? e.qlo[1] : e.qlo[2]);
      const float qhi = g3 == 0 ? e.qhi[0] : (g3 == 1 ? e.qhi[1] : e.qhi[2]);
      const float magic = g3 == 0 ? e.magic[0] : (g3 == 1 ? e.magic[1] : e.magic[2]);
      const float s_out = g3 == 0 ? e.s_out[0] : (g3 == 1 ? e.s_out[1] : e.s_out[2]);
      const double rs_out = g3 == 0 ? e.rs_out[0] : (g3 == 1 ? e.rs_out[1] : e.rs_out[2]);
      const double zp = g3 == 0 ? e.zp_out[0] : (g3 == 1 ? e.zp_out[1] : e.zp_out[2]);
      void* op = g3 == 0 ? e.out[0] : (g3 == 1 ? e.out[1] : e.out[2]);
      // QKV: the head-layout buffer holds whole images, ceil(M / tokens) of them
      // N % 256 != 0 (ViT-tiny): a wave whose 64 columns lie past N stores through a
      // zero-size descriptor (dropped; its VMEM count stays that of every wave)
      const rsrc_t r_out = pg_rsrc(
          op, cw >= N ? 0u
                      : (uint32_t)(EPI == PG_QKV ? (uint64_t)((M + e.tokens - 1) / e.tokens) * e.tokens * e.heads * e.hdim
                                                 : (uint64_t)M * e.ldo));
      // QKV: u = v c1 + c2 with c2 = RN(bias rsf): within |v| k1 + kb of zp + 128 + t,
      // t = RN(RN(RN(v sacc) + bias) / s_out) (DESIGN.md §4.3 error bound); kb from the
      // lane's largest |c2|, folded into the lane's limit
      float c2[16];
      float lim = PG_QLIM;
      if constexpr (EPI == PG_QKV) {
        float cm = 0.0f;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          c2[q] = bias[q] * rsf;
          cm = __builtin_fmaxf(cm, __builtin_fabsf(c2[q]));
        }
        lim = (PG_QLIM - cm * NQK_PG_QKC2) - 0x1p-22f;  // conservative: every rounding down
      } else {
        lim = e.g_lim;
      }
      int hh = 0;
      if constexpr (EPI == PG_QKV) hh = (cw - g3 * e.group_cols) / e.hdim;
      sfor<0, MS>([&](auto I) __attribute__((always_inline)) {
        constexpr int i = decltype(I)::value;
        const int m = s.r0 + PG_BM * wm + 16 * i + l15;
        uint32_t off;
        if constexpr (EPI == PG_QKV) {
          const int img = m / e.tokens, t = m - img * e.tokens;
          off = (uint32_t)(((img * e.heads + hh) * e.tokens + t) * e.hdim + 16 * lg);
        } else {
          off = (uint32_t)(m * e.ldo + col0);
        }
        if constexpr (pg_is_glut(EPI)) {
          // GELU by table lookup: h exactly as the reference (F32X), its bucket entry from
          // the LDS table (one ds_read_b64 per element), the output byte selected by one
          // compare (nqk_glut.h); no filter and no fallback path
          float hv[16];
          uint2 ent[16];
#pragma unroll
          for (int q = 0; q < 16; q += 2) {
            const v4i& av4 = acc[i][q >> 2];
            // (packed: the unpacked form measured 146 -> 157 us, profiles/r04_glut_unpacked_dropped.txt)
            const v2f vf = v2f{(float)av4[q & 3], (float)av4[(q & 3) + 1]};
            const v2f h = v2f{bias[q], bias[q + 1]} + vf * v2f{sacc, sacc};
            const v2f r = __builtin_elementwise_fma(h, v2f{e.gk.iwR, e.gk.iwR}, v2f{e.gk.cR, e.gk.cR});
            // PG_GLUT1: one line over both branches (the table's L line is -inf: max(R, L) = R)
            const v2f l = EPI == PG_GLUT1 ? r : __builtin_elementwise_fma(h, v2f{e.gk.iwL, e.gk.iwL}, v2f{e.gk.cL, e.gk.cL});
            hv[q] = h[0];
            hv[q + 1] = h[1];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const float u = __builtin_amdgcn_fmed3f(EPI == PG_GLUT1 ? r[j] : __builtin_fmaxf(r[j], l[j]), GLUT_MAGIC, e.gk.uhi);
              const uint32_t a = (__float_as_uint(u) << 3) + lut_base;
              const v2u t = *(const __attribute__((address_space(3))) v2u*)(uintptr_t)a;
              ent[q + j] = make_uint2(t[0], t[1]);
            }
          }
          uint32_t pk[4] = {0, 0, 0, 0};
          uint64_t slow = 0;  // lanes with an element in its entry's window
          sfor<0, 16>([&](auto Q) __attribute__((always_inline)) {
            constexpr int q = decltype(Q)::value;
            pk[q >> 2] = glut_sel<q & 3>(pk[q >> 2], hv[q], ent[q].x, ent[q].y, slow);
          });
          if (__builtin_expect(slow != 0, 0) && (NQK_PG_DIAG & 32) == 0) {
            // the exact chain for the elements inside a window (wave-uniform branch; a loop
            // that is not unrolled keeps the chain's code once)
            // (element q picked by compile-time selects: no runtime-indexed arrays, no scratch)
#pragma clang loop unroll(disable)
            for (int q = 0; q < 16; ++q) {
              float hq = 0.0f;
              uint32_t tq = 0u, iq = 0u;
              sfor<0, 16>([&](auto Q) __attribute__((always_inline)) {
                constexpr int c = decltype(Q)::value;
                hq = q == c ? hv[c] : hq;
                tq = q == c ? ent[c].x : tq;
                iq = q == c ? ent[c].y : iq;
              });
              if (glut_in_window(hq, tq, iq)) {
                const uint32_t qv =
                    (uint32_t)glut_exact(hq, e.rdiv, e.add1, e.mul2, e.rs_out[0], e.zp_out[0], e.lo, e.hi) & 0xffu;
                sfor<0, 4>([&](auto G) __attribute__((always_inline)) {
                  constexpr int g = decltype(G)::value;
                  const int sh = 8 * (q & 3);
                  if ((q >> 2) == g) pk[g] = (pk[g] & ~(0xffu << sh)) | (qv << sh);
                });
              }
            }
          }
          const v4u st = v4u{pk[0], pk[1], pk[2], pk[3]};
          // (diagnostic 8192, wrong layout: the wave's 16 rows x 64 B of a subtile as 1 KiB contiguous
          // — whole lines per instruction, the same bytes per launch: does the half-line row pattern cost?)
          if constexpr ((NQK_PG_DIAG & 8192) != 0)
            off = (uint32_t)((s.r0 + PG_BM * wm + 16 * i) * e.ldo + (s.tn * 4 + wn) * 1024 + 16 * lane);
          if constexpr ((NQK_PG_DIAG & 1) != 0) asm volatile("" ::"v"(st[0] ^ st[1] ^ st[2] ^ st[3]));
          else __builtin_amdgcn_raw_buffer_store_b128(st, r_out, off, 0, NQK_PG_STAUX);
          return;
        }
        uint32_t pk[4] = {0, 0, 0, 0};
        uint32_t worst = 0;
        uint32_t wgr[4] = {0, 0, 0, 0};  // QKV, GELU4: the measure's maximum per group of 4 elements
        float hv[16];
        v2f sprev;
        // GELU, two pairs at a time (NQK_PG_GELU4): the two chains interleaved
        if constexpr (EPI == PG_GELU && NQK_PG_GELU4 && (NQK_PG_DIAG & 2) == 0) {
#pragma unroll
          for (int q = 0; q < 16; q += 4) {
            const v4i& av4 = acc[i][q >> 2];
            const v2f vf0 = v2f{(float)av4[0], (float)av4[1]}, vf1 = v2f{(float)av4[2], (float)av4[3]};
            const v2f h0 = v2f{bias[q], bias[q + 1]} + vf0 * v2f{sacc, sacc};
            const v2f h1 = v2f{bias[q + 2], bias[q + 3]} + vf1 * v2f{sacc, sacc};
            hv[q] = h0[0];
            hv[q + 1] = h0[1];
            hv[q + 2] = h1[0];
            hv[q + 3] = h1[1];
            v2f g0, g1;
            gelu_fast2x2(h0, h1, g0, g1);
            const v2f tf0 = g0 * v2f{rsf, rsf}, tf1 = g1 * v2f{rsf, rsf};
            v2f dd0, dd1;
            const v2f s0 = round_magic2(tf0, qlo, qhi, magic, dd0);
            const v2f s1 = round_magic2(tf1, qlo, qhi, magic, dd1);
            const float m0 = __builtin_fmaf(__builtin_fabsf(h0[0]), e.g_rel, __builtin_fabsf(dd0[0]));
            const float m1 = __builtin_fmaf(__builtin_fabsf(h0[1]), e.g_rel, __builtin_fabsf(dd0[1]));
            const float m2 = __builtin_fmaf(__builtin_fabsf(h1[0]), e.g_rel, __builtin_fabsf(dd1[0]));
            const float m3 = __builtin_fmaf(__builtin_fabsf(h1[1]), e.g_rel, __builtin_fabsf(dd1[1]));
            wgr[q >> 2] = __builtin_elementwise_max(__builtin_elementwise_max(__float_as_uint(m0), __float_as_uint(m1)),
                                                    __builtin_elementwise_max(__float_as_uint(m2), __float_as_uint(m3)));
            worst = __builtin_elementwise_max(worst, wgr[q >> 2]);
            pk[q >> 2] = pack4_low(s0, s1);
          }
        }
        // the fast paths on element pairs (packed f32 arithmetic where an instruction exists)
#pragma unroll
        for (int q = 0; q < 16 && (NQK_PG_DIAG & 2) == 0 && !(EPI == PG_GELU && NQK_PG_GELU4); q += 2) {
          const v2f vf = v2f{(float)acc[i][q >> 2][q & 3], (float)acc[i][q >> 2][(q & 3) + 1]};
          v2f dd, sv;
          float m0, m1;
          if constexpr (EPI == PG_QKV) {  // (pg_round2 measured slower here: a longer dependent chain)
            v2f u, rr, b;
            if constexpr (NQK_PG_NOPK) {  // the same IEEE operations per element, unpacked
#pragma unroll
              for (int j = 0; j < 2; ++j) {
                u[j] = __builtin_fmaf(vf[j], c1, c2[q + j]);
                rr[j] = __builtin_rintf(u[j]);
                dd[j] = u[j] - rr[j];
                b[j] = rr[j] + zp128;
              }
            } else {
              u = __builtin_elementwise_fma(vf, v2f{c1, c1}, v2f{c2[q], c2[q + 1]});
              rr = v2f{__builtin_rintf(u[0]), __builtin_rintf(u[1])};
              dd = u - rr;
              b = rr + v2f{zp128, zp128};
            }
            m0 = __builtin_fmaf(__builtin_fabsf(vf[0]), k1, __builtin_fabsf(dd[0]));
            m1 = __builtin_fmaf(__builtin_fabsf(vf[1]), k1, __builtin_fabsf(dd[1]));
            pk[q >> 2] = __builtin_amdgcn_cvt_pk_u8_f32(S8 ? b[0] : __builtin_amdgcn_fmed3f(b[0], e.blo, e.bhi), q & 3,
                                                        pk[q >> 2]);
            pk[q >> 2] = __builtin_amdgcn_cvt_pk_u8_f32(S8 ? b[1] : __builtin_amdgcn_fmed3f(b[1], e.blo, e.bhi),
                                                        (q & 3) + 1, pk[q >> 2]);
          } else {  // GELU: h exactly as the reference (F32X), then the filtered fast chain
            const v2f h = v2f{bias[q], bias[q + 1]} + vf * v2f{sacc, sacc};
            hv[q] = h[0];
            hv[q + 1] = h[1];
            const v2f tf = gelu_fast2(h) * v2f{rsf, rsf};
            sv = round_magic2(tf, qlo, qhi, magic, dd);
            m0 = __builtin_fmaf(__builtin_fabsf(h[0]), e.g_rel, __builtin_fabsf(dd[0]));
            m1 = __builtin_fmaf(__builtin_fabsf(h[1]), e.g_rel, __builtin_fabsf(dd[1]));
          }
          if constexpr (EPI == PG_QKV)
            wgr[q >> 2] = __builtin_elementwise_max(wgr[q >> 2], __builtin_elementwise_max(__float_as_uint(m0), __float_as_uint(m1)));
          else
            worst = __builtin_elementwise_max(worst, __builtin_elementwise_max(__float_as_uint(m0), __float_as_uint(m1)));
          if constexpr (EPI != PG_QKV) {
            if (q & 2) pk[q >> 2] = pack4_low(sprev, sv);
            sprev = sv;
          }
        }
        if constexpr (EPI == PG_QKV) {
#pragma unroll
          for (int g = 0; g < 4; ++g) pk[g] ^= 0x80808080u;  // offset bytes to two's complement
          worst = __builtin_elementwise_max(__builtin_elementwise_max(wgr[0], wgr[1]),
                                            __builtin_elementwise_max(wgr[2], wgr[3]));
        }
#pragma unroll
        for (int q = 0; q < 16 && (NQK_PG_DIAG & 2) != 0; ++q)  // diagnostic: no epilogue math
          pk[q >> 2] = __builtin_amdgcn_cvt_pk_u8_f32((float)(acc[i][q >> 2][q & 3] & 255), q & 3, pk[q >> 2]);
        if constexpr ((NQK_PG_DIAG & 34) == 0) {  // (diagnostic 32: no exact fallback)
          if (__builtin_expect(__any(worst >= __float_as_uint(lim)), 0)) {
            int av[16];
            float xv[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
              av[q] = acc[i][q >> 2][q & 3];
              xv[q] = EPI == PG_QKV ? bias[q] : hv[q];
            }
            uint32_t gm = 15u;
            if constexpr (EPI == PG_QKV || (EPI == PG_GELU && NQK_PG_GELU4)) {
              gm = 0u;
#pragma unroll
              for (int g = 0; g < 4; ++g) gm |= __any(wgr[g] >= __float_as_uint(lim)) ? 1u << g : 0u;
            }
            pg_exact_fix<EPI>(av, xv, pk, PgFix{c1, k1, rsf, sacc, lim, s_out, rs_out, zp}, e, gm);
          }
        }
        const v4u st = v4u{pk[0], pk[1], pk[2], pk[3]};
        if constexpr ((NQK_PG_DIAG & 1) != 0) asm volatile("" ::"v"(st[0] ^ st[1] ^ st[2] ^ st[3]));
        else __builtin_amdgcn_raw_buffer_store_b128(st, r_out, off, 0, NQK_PG_STAUX);
      });
    }
  };

  // RESID epilogue: y = (bias + RN(v sacc)) + residual, f32 stores, with whole 128-B lines
  // per instruction: each subtile's accumulators go through the wave's part of ring slot 2
  // (free from the barrier after the k loop until the next tile's step 0 refills it), row-
  // major [16 rows][64 columns] int32 with 272-B rows, and come back transposed: lane
  // (a = l & 15, b = l >> 4) takes row 4 k + b, columns 4 a .. 4 a + 3 for k = 0..3, so the
  // 16 lanes of a row load / store its 256 contiguous bytes.  Residual loads of subtile i + 2
  // are issued after subtile i's stores (0 and 1 before the next tile's stages); the
  // compiler places their waits (compiler-visible loads).
  const rsrc_t r_res = pg_rsrc(RESID ? e.resid : nullptr, RESID ? (uint32_t)((uint64_t)M * e.ldo * 4) : 0u);
  const rsrc_t r_nul = pg_rsrc(RESID ? e.resid : nullptr, 0u);  // columns past N: loads return 0, stores drop
  constexpr int TR_ROW = PG_TR_ROW;
  int8_t* const tr = lds + (B4 || WM == 2 ? COLP + 4096 : 2 * STG) + wave * (16 * TR_ROW);
  const int ta = lane & 15, tb = lane >> 4;
  constexpr int RQ = NQK_PG_RESQ;  // residual subtiles in flight (register slots)
  // DIRECT (NQK_PG_RDIRECT): no transposes, ring slot 2 stays free, PRE = the last stage of the next
  // tile issued before this tile's epilogue (RD - 2 otherwise)
  constexpr bool DIRECT = RESID && NQK_PG_RDIRECT && !B4 && WM == 1 && !RB;
  constexpr int PRE = DIRECT ? RD - 1 : RD - 2;
  v4u resv[RQ][4];
  auto res_off = [&](const Src& s, int i, int k) __attribute__((always_inline)) {
    return (uint32_t)(((s.r0 + PG_BM * wm + 16 * i + 4 * k + tb) * e.ldo + s.tn * PG_BN + 64 * wn + 4 * ta) * 4);
  };
  // DIRECT: lane (l15, lg) of subtile i, column block j: row 16 i + l15, columns 16 j + 4 lg .. + 3 of
  // the wave's 64 — the accumulator layout itself (16 rows x 64 B per instruction)
  auto res_off_d = [&](const Src& s, int i, int j) __attribute__((always_inline)) {
    return (uint32_t)(((s.r0 + PG_BM * wm + 16 * i + l15) * e.ldo + s.tn * PG_BN + 64 * wn + 16 * j + 4 * lg) * 4);
  };
  auto res_issue = [&](const Src& s, auto I) __attribute__((always_inline)) {
    constexpr int i = decltype(I)::value;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      resv[i % RQ][k] = pg_load16(s.tn * PG_BN + 64 * wn < N && (NQK_PG_DIAG & 4096) == 0 ? r_res : r_nul,
                                 DIRECT ? res_off_d(s, i, k) : res_off(s, i, k), 0u,
                                 NQK_PG_RLAUX >= 0 ? NQK_PG_RLAUX : (NK == 48 ? 2 : 0));
  };
  auto epilogue_resid_direct = [&](const Src& s, int cslot) __attribute__((always_inline)) {
    const int8_t* cp = lds + COLP + cslot * 2048;
    v4i bj[4];  // bias of columns 16 j + 4 lg .. + 3
#pragma unroll
    for (int j = 0; j < 4; ++j) bj[j] = pg_lds16(cp + 1024 + (64 * wn + 16 * j + 4 * lg) * 4);
    const rsrc_t r_out = pg_rsrc(e.out[0], s.tn * PG_BN + 64 * wn < N ? (uint32_t)((uint64_t)M * e.ldo * 4) : 0u);
    const float sacc = e.sacc[0];
    sfor<0, 8>([&](auto I) __attribute__((always_inline)) {
      constexpr int i = decltype(I)::value;
      const v4u(&rv)[4] = resv[i % RQ];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const v4i t = acc[i][j];
        const v4i bb = bj[j];
        v4u st;
        if constexpr (F32X) {
          const v2f b01 = v2f{__int_as_float(bb[0]), __int_as_float(bb[1])};
          const v2f b23 = v2f{__int_as_float(bb[2]), __int_as_float(bb[3])};
          const v2f d01 = v2f{(float)t[0], (float)t[1]} * v2f{sacc, sacc};
          const v2f d23 = v2f{(float)t[2], (float)t[3]} * v2f{sacc, sacc};
          const v2f y01 = (b01 + d01) + v2f{__uint_as_float(rv[j][0]), __uint_as_float(rv[j][1])};
          const v2f y23 = (b23 + d23) + v2f{__uint_as_float(rv[j][2]), __uint_as_float(rv[j][3])};
          st = v4u{__float_as_uint(y01[0]), __float_as_uint(y01[1]), __float_as_uint(y23[0]), __float_as_uint(y23[1])};
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float d = (float)((double)t[r] * (double)sacc);
            st[r] = __float_as_uint((__int_as_float(bb[r]) + d) + __uint_as_float(rv[j][r]));
          }
        }
        if constexpr ((NQK_PG_DIAG & 1) != 0) asm volatile("" ::"v"(st[0] ^ st[1] ^ st[2] ^ st[3]));
        else __builtin_amdgcn_raw_buffer_store_b128(st, r_out, res_off_d(s, i, j), 0, NQK_PG_STAUX_RESID);
      }
      if constexpr (i + RQ - 1 < 8) res_issue(s, ic<i + RQ - 1>{});
    });
  };
  auto epilogue_resid = [&](const Src& s, int cslot) __attribute__((always_inline)) {
    const int8_t* cp = lds + COLP + cslot * 2048;
    const v4i bb = pg_lds16(cp + 1024 + (64 * wn + 4 * ta) * 4);  // columns 4 a .. 4 a + 3
    const v2f b01 = v2f{__int_as_float(bb[0]), __int_as_float(bb[1])};
    const v2f b23 = v2f{__int_as_float(bb[2]), __int_as_float(bb[3])};
    const rsrc_t r_out = pg_rsrc(e.out[0], s.tn * PG_BN + 64 * wn < N ? (uint32_t)((uint64_t)M * e.ldo * 4) : 0u);
    const float sacc = e.sacc[0];
    sfor<0, 8>([&](auto I) __attribute__((always_inline)) {
      constexpr int i = decltype(I)::value;
      // this lane's 16 accumulators: row l15, columns 16 j + 4 lg + r (layout 1)
#pragma unroll
      for (int j = 0; j < 4; ++j) *reinterpret_cast<v4i*>(tr + l15 * TR_ROW + (16 * j + 4 * lg) * 4) = acc[i][j];
      v4i t[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) t[k] = *reinterpret_cast<const v4i*>(tr + (4 * k + tb) * TR_ROW + 16 * ta);
      const v4u(&rv)[4] = resv[i % RQ];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v4u st;
        if constexpr (F32X) {  // (unpacked: within noise, profiles/r04_qkv_nopk_ab.txt)
          const v2f d01 = v2f{(float)t[k][0], (float)t[k][1]} * v2f{sacc, sacc};
          const v2f d23 = v2f{(float)t[k][2], (float)t[k][3]} * v2f{sacc, sacc};
          const v2f y01 = (b01 + d01) + v2f{__uint_as_float(rv[k][0]), __uint_as_float(rv[k][1])};
          const v2f y23 = (b23 + d23) + v2f{__uint_as_float(rv[k][2]), __uint_as_float(rv[k][3])};
          st = v4u{__float_as_uint(y01[0]), __float_as_uint(y01[1]), __float_as_uint(y23[0]), __float_as_uint(y23[1])};
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float d = (float)((double)t[k][r] * (double)sacc);
            st[r] = __float_as_uint((__int_as_float(bb[r]) + d) + __uint_as_float(rv[k][r]));
          }
        }
        if constexpr ((NQK_PG_DIAG & 1) != 0) asm volatile("" ::"v"(st[0] ^ st[1] ^ st[2] ^ st[3]));
        else __builtin_amdgcn_raw_buffer_store_b128(st, r_out, res_off(s, i, k), 0, NQK_PG_STAUX_RESID);
      }
      if constexpr (i + RQ - 1 < 8) res_issue(s, ic<i + RQ - 1>{});
    });
  };

  // ---------------------------------------------------------------- the persistent loop
  // VMEM operations per wave, in issue order: [colp(next)] at step 1; stage kt + 2 in step
  // kt's first half; after the k loop (RESID: residual of subtiles 0, 1), the next tile's
  // stages 0 and 1, then the epilogue's operations (EOPS)
  // RESID: 8 x 4 stores after the stages (counted conservatively without the 6 x 4 residual
  // loads, which the compiler may hoist above the stage issues: a smaller count only waits more)
  constexpr int EOPS = RESID ? 32 : MS;
  constexpr int PWA = PW;
  Src cur = src_of(tile_at(0));
  if constexpr (RB) {
    // VMEM operations per wave, in issue order: [B pieces when the panel changes], colp(next),
    // the next tile's A pieces (3 k steps), then the epilogue's EOPS stores: waiting for all but
    // EOPS waits for everything the next tile reads
    if constexpr (pg_is_glut(EPI)) pg_dma16(pg_rsrc(e.lut, e.lut_bytes), lds + LUTO + wave * 1024, 16 * lane, 1024u * wave);
    auto issue_b = [&](const Src& s) __attribute__((always_inline)) {
#pragma unroll
      for (int kt = 0; kt < NK; ++kt)
#pragma unroll
        for (int p = 2; p < PW; ++p) issue_piece(s, kt, kt, p);
    };
    auto issue_a = [&](const Src& s) __attribute__((always_inline)) {
#pragma unroll
      for (int kt = 0; kt < NK; ++kt)
#pragma unroll
        for (int p = 0; p < 2; ++p) issue_piece(s, kt, kt, p);
    };
    int ctn = cur.tn;
    issue_b(cur);
    issue_colp(cur.tn, 0);
    issue_a(cur);
    for (int it = 0; it < iters; ++it) {
      if constexpr (NQK_PG_PRIO == 3) __builtin_amdgcn_s_setprio(0);
      const bool more = it + 1 < iters;
      const Src nxt = src_of(tile_at(more ? it + 1 : it));
      const int cs = it & 1;
      if (it == 0) pg_vmcnt<0>();
      else pg_vmcnt<EOPS>();
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      v4i cinit[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) cinit[j] = pg_lds16(lds + COLP + cs * 2048 + (64 * wn + 16 * lg + 4 * j) * 4);
      sfor<0, 4>([&](auto Q) __attribute__((always_inline)) {
        rd_a(a_lo, ic<0>{}, ic<0>{}, Q);
        rd_b(b0, ic<0>{}, Q);
      });
      pg_lgkm_tie8(a_lo, b0);
      pg_lgkm_tie(cinit[0], cinit[1], cinit[2], cinit[3]);
#pragma unroll
      for (int j = 0; j < 4; ++j) cinit[j] = -cinit[j];
      sfor<0, NK>([&](auto KT) __attribute__((always_inline)) {
        constexpr int kt = decltype(KT)::value;
        v4i(&bc)[4] = (kt & 1) ? b1 : b0;
        v4i(&bn)[4] = (kt & 1) ? b0 : b1;
        if constexpr (kt > 0) pg_lgkm_tie8(a_lo, bc);
        half(ic<0>{}, std::integral_constant<bool, kt == 0>{}, a_lo, bc, cinit, [&](auto Q) __attribute__((always_inline)) {
          constexpr int q = decltype(Q)::value;
          if constexpr (q < 4) rd_a(a_hi, ic<kt>{}, ic<4>{}, Q);
        });
        pg_lgkm_tie(a_hi[0], a_hi[1], a_hi[2], a_hi[3]);
        half(ic<1>{}, std::integral_constant<bool, kt == 0>{}, a_hi, bc, cinit, [&](auto Q) __attribute__((always_inline)) {
          constexpr int q = decltype(Q)::value;
          if constexpr (kt + 1 < NK) {
            if constexpr (q < 4) rd_a(a_lo, ic<kt + 1>{}, ic<0>{}, Q);
            else if constexpr (q < 8) rd_b(bn, ic<kt + 1>{}, ic<q - 4>{});
          }
        });
      });
      // every wave is done reading this tile's A (and B, if the panel changes)
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (nxt.tn != ctn) {  // (wave-uniform; rare: a workgroup's tiles are mostly one panel)
        issue_b(nxt);
        ctn = nxt.tn;
      }
      issue_colp(nxt.tn, cs ^ 1);
      issue_a(nxt);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (NQK_PG_PRIO == 3) __builtin_amdgcn_s_setprio(1);
      epilogue(cur, cs);
      cur = nxt;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }
  // PG_GLUT: the 4 KiB GELU table into LDS, 1 KiB per wave (waited for with stage 0)
  // (WM = 2: the 8 KiB of a table of up to GLUT_MAX entries, 1 KiB per wave as well)
  // (the descriptor's range is the table's own 8 * lut_n bytes, rounded up to 16: the pieces past it
  // read zeros, so a caller's buffer of exactly the table's size is never over-read)
  if constexpr (pg_is_glut(EPI)) pg_dma16(pg_rsrc(e.lut, e.lut_bytes), lds + LUTO + wave * 1024, 16 * lane, 1024u * wave);
  issue_colp(cur.tn, 0);
  sfor<0, PRE + 1>([&](auto S) __attribute__((always_inline)) { issue_stage(cur, decltype(S)::value, decltype(S)::value); });
  if constexpr (NQK_PG_PRIO == 2) {
    if ((int)blockIdx.x >= G / 2) __builtin_amdgcn_s_setprio(1);
  }
  for (int it = 0; it < iters; ++it) {
    if constexpr (NQK_PG_PRIO == 1) __builtin_amdgcn_s_setprio(1);
    if constexpr (NQK_PG_PRIO == 3) __builtin_amdgcn_s_setprio(0);
    const bool more = it + 1 < iters;
    const Src nxt = src_of(tile_at(more ? it + 1 : it));
    const int cs = it & 1;
    // stage 0 and this tile's column constants landed (younger: stages 1 .. RD - 2, the previous
    // epilogue's operations)
    if (it == 0) pg_vmcnt<PRE * PWA>();
    else pg_vmcnt<PRE * PWA + EOPS>();
    if constexpr ((NQK_PG_DIAG & 8) == 0) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // initial accumulators: minus the zero-point column terms of the lane's 16 columns
    v4i cinit[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      cinit[j] = pg_lds16(lds + COLP + cs * 2048 + (64 * wn + (RESID ? 16 * j + 4 * lg : 16 * lg + 4 * j)) * 4);
    sfor<0, 4>([&](auto Q) __attribute__((always_inline)) {
      rd_a(a_lo, ic<0>{}, ic<0>{}, Q);
      if constexpr (B4) rd_b4(p0, ic<0>{}, Q);
      else rd_b(b0, ic<0>{}, Q);
    });
    if constexpr (B4) {
      pg_lgkm_tie_a4(a_lo, p0);
      unpack_b(p0);
    } else {
      pg_lgkm_tie8(a_lo, b0);
    }
    pg_lgkm_tie(cinit[0], cinit[1], cinit[2], cinit[3]);
#pragma unroll
    for (int j = 0; j < 4; ++j) cinit[j] = B4 ? -(cinit[j] << 4) : -cinit[j];
    sfor<0, NK>([&](auto KT) __attribute__((always_inline)) {
      constexpr int kt = decltype(KT)::value;
      constexpr int slot = kt % RD;
      v4i(&bc)[4] = B4 ? b0 : ((kt & 1) ? b1 : b0);
      v4i(&bn)[4] = (kt & 1) ? b0 : b1;
      v2u(&pc)[4] = (kt & 1) ? p1 : p0;
      v2u(&pn)[4] = (kt & 1) ? p0 : p1;
      if constexpr (WM == 0) {
        // 64-row form: this step's A fragments (subtiles 0..3) alternate between a_lo and a_hi;
        // MFMAs of subtiles 0, 1 (the refill of the slot step kt - 1 read after MFMA 4), the wait
        // for stage kt + 1, then subtiles 2, 3 with the next step's fragment reads between them
        v4i(&ac)[4] = (kt & 1) ? a_hi : a_lo;
        v4i(&an)[4] = (kt & 1) ? a_lo : a_hi;
        if constexpr (kt > 0) pg_lgkm_tie8(ac, bc);
        quarter(ic<0>{}, std::integral_constant<bool, kt == 0>{}, ac, bc, cinit, [&](auto Q) __attribute__((always_inline)) {
          if constexpr (kt + RD - 1 < NK && kt + RD - 1 > PRE && decltype(Q)::value == 4) issue_stage(cur, kt + RD - 1, (kt + RD - 1) % RD);
        });
        if constexpr (kt == 1) issue_colp(nxt.tn, cs ^ 1);
        if constexpr (kt + 1 < NK) {
          constexpr int hi_s = (kt + RD - 1 < NK ? kt + RD - 1 : NK - 1);
          constexpr int y = (hi_s >= kt + 2 ? (hi_s - kt - 1) * PWA : 0) + ((kt >= 1 && kt <= RD - 1) ? 1 : 0);
          if (kt + 1 <= PRE && it > 0) pg_vmcnt<y + EOPS>();
          else pg_vmcnt<y>();
          if constexpr ((NQK_PG_DIAG & 8) == 0) __builtin_amdgcn_s_barrier();
          __builtin_amdgcn_sched_barrier(0);
        }
        quarter(ic<1>{}, std::integral_constant<bool, kt == 0>{}, ac, bc, cinit, [&](auto Q) __attribute__((always_inline)) {
          constexpr int q = decltype(Q)::value;
          if constexpr (kt + 1 < NK) {
            if constexpr (q < 4) rd_a(an, ic<(kt + 1) % RD>{}, ic<0>{}, Q);
            else rd_b(bn, ic<(kt + 1) % RD>{}, ic<q - 4>{});
          }
        });
        return;
      }
      if constexpr (kt > 0) {  // this step's fragments (read in step kt - 1)
        if constexpr (B4) {
          pg_lgkm_tie_a4(a_lo, pc);
          unpack_b(pc);
        } else {
          pg_lgkm_tie8(a_lo, bc);
        }
      }
      // first half: subtiles 0..3; between the MFMAs the second half's A fragments and the
      // refill of the slot step kt - 1 read (stage kt + RD - 1)
      half(ic<0>{}, std::integral_constant<bool, kt == 0>{}, a_lo, bc, cinit, [&](auto Q) __attribute__((always_inline)) {
        constexpr int q = decltype(Q)::value;
        if constexpr (q < 4) rd_a(a_hi, ic<slot>{}, ic<4>{}, Q);
        // stage kt + 2: NQK_PG_SPREAD 0 = all pieces after MFMA 4; 1 = one piece every
        // other MFMA from MFMA 1 (a burst of LDS-DMA issues costs each piece more:
        // MI355X_MICROARCH.md, LDS-DMA piece issue cost)
        if constexpr (kt + RD - 1 < NK && kt + RD - 1 > PRE) {
          if constexpr (NQK_PG_SPREAD == 0) {
            if constexpr (q == 4) issue_stage(cur, kt + RD - 1, (kt + RD - 1) % RD);
          } else if constexpr ((q & 1) == 1 && (q >> 1) < PW) {
            issue_piece(cur, kt + RD - 1, (kt + RD - 1) % RD, q >> 1);
          }
        }
      });
      if constexpr (kt == 1) issue_colp(nxt.tn, cs ^ 1);
      if constexpr (kt + 1 < NK) {
        // stage kt + 1 landed; younger: stages kt + 2 .. kt + RD - 1 (those issued), colp (step 1,
        // after stage RD), and for the stages issued before this tile (kt + 1 <= RD - 2) the
        // previous tile's epilogue operations
        constexpr int hi_s = (kt + RD - 1 < NK ? kt + RD - 1 : NK - 1);
        constexpr int y = (hi_s >= kt + 2 ? (hi_s - kt - 1) * PWA : 0) + ((kt >= 1 && kt <= RD - 1) ? 1 : 0);
        if (kt + 1 <= PRE && it > 0) pg_vmcnt<y + EOPS>();
        else pg_vmcnt<y>();
        pg_lgkm_tie(a_hi[0], a_hi[1], a_hi[2], a_hi[3]);
        if constexpr ((NQK_PG_DIAG & 8) == 0) __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      } else {
        pg_lgkm_tie(a_hi[0], a_hi[1], a_hi[2], a_hi[3]);
      }
      half(ic<1>{}, std::integral_constant<bool, kt == 0>{}, a_hi, bc, cinit, [&](auto Q) __attribute__((always_inline)) {
        constexpr int q = decltype(Q)::value;
        if constexpr (kt + 1 < NK) {
          if constexpr (q < 4) rd_a(a_lo, ic<(kt + 1) % RD>{}, ic<0>{}, Q);
          else if constexpr (q < 8) {
            if constexpr (B4) rd_b4(pn, ic<(kt + 1) % RD>{}, ic<q - 4>{});
            else rd_b(bn, ic<(kt + 1) % RD>{}, ic<q - 4>{});
          }
        }
      });
    });
    // RESID: the residual rows of the first two subtiles, then the next tile's first
    // stages (slots 0 and 1: last read before step NK - 2's barrier); a barrier frees slot 2
    // (stage NK - 1) for the epilogue's transposes
    if constexpr (RESID) {
      sfor<0, RQ - 1>([&](auto R) __attribute__((always_inline)) { res_issue(cur, R); });
      if constexpr (!B4 && WM == 1) __builtin_amdgcn_s_barrier();  // (B4, WM = 2: the scratch is not in the ring)
    }
    // (the last tile re-stages its own first stages: never read, drained at the end; the
    // VMEM counts stay the same on every path)
    sfor<0, PRE + 1>([&](auto S) __attribute__((always_inline)) { issue_stage(nxt, decltype(S)::value, decltype(S)::value); });
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (NQK_PG_PRIO == 1) __builtin_amdgcn_s_setprio(0);
    if constexpr (NQK_PG_PRIO == 3) __builtin_amdgcn_s_setprio(1);
    if constexpr (B4) {  // the MFMAs accumulated 16 acc
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = acc[i][j] >> 4;
    }
    if constexpr (DIRECT) epilogue_resid_direct(cur, cs);
    else if constexpr (RESID) epilogue_resid(cur, cs);
    else epilogue(cur, cs);
    cur = nxt;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

// One k_pg launch (the host launcher fills it; the instantiation files' dispatchers take the
// cases they hold).  epi points at a PgEpi.
struct PgArgs {
  const int8_t* a;
  const int8_t* bp;
  int m, n, lda, tiles_n, ntiles, grid;
  const void* epi;
};
// the dispatchers (nqk_pg_inst_*.hip): launch the k_pg instance of `key` and return true,
// or false when the file holds no such instance
bool pg_dispatch_i8(int key, const PgArgs& x);
bool pg_dispatch_resid(int key, const PgArgs& x);
bool pg_dispatch_tiny(int key, const PgArgs& x);
bool pg_dispatch_i4(int key, const PgArgs& x);
bool pg_dispatch_wm2(int key, const PgArgs& x);

// launch keys: EPI * 16 + (K 3072: 2, K 192: 1, else 0) * 4 + F32X + 2 B4 + 256 S8 + 512 WM2 + 1024 RB + 2048 WM0
constexpr int pg_key(int epi, int nk, bool f32x, bool b4, bool s8, int wm, bool rb = false) {
  return epi * 16 + (nk == 48 ? 2 : (nk == 3 ? 1 : 0)) * 4 + (f32x ? 1 : 0) + (b4 ? 2 : 0) + (s8 ? 256 : 0) +
         (wm == 2 ? 512 : 0) + (rb ? 1024 : 0) + (wm == 0 ? 2048 : 0);
}
#define NQK_PG_CASE_RB(E, NKV, X, B, S, W, R)                                                                  \
  case pg_key(E, NKV, X, B, S, W, R):                                                                          \
    hipLaunchKernelGGL((k_pg<E, NKV, X, B, S, W, R>), dim3(x.grid), dim3(W == 2 ? 512 : 256), pg_lds_bytes(E, B, W, NKV), stream(), \
                       x.a, x.bp, x.m, x.n, x.lda, x.tiles_n, x.ntiles, *static_cast<const PgEpi*>(x.epi));    \
    return true;
#define NQK_PG_CASE(E, NKV, X, B, S, W) NQK_PG_CASE_RB(E, NKV, X, B, S, W, false)

}  // namespace nqk
