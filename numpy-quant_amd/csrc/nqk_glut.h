// GELU + quantize by table lookup (round 4): the map from the FFN-up GEMM's dequantized,
// biased value h (f32) to the quantized output of the GELU chain, i.e. model.py's
// Div -> Erf -> Add -> Mul -> Mul on f32 (numpy_helper.py:95-112 erf) followed by
// numpy_quantization.py:24-34 quantize.  For fixed quantization parameters that map is a
// step function of h with a few hundred steps, so the epilogue replaces ~21 VALU of a
// filtered approximation per element by a bucket index (2 fma + max + med3), one 8-byte
// LDS read and a compare + select.
//
// Buckets: u(h) = med3(max(R(h), L(h)), MAGIC, uhi) with two lines that meet at the GELU
// minimum hk ~ -0.7518 (R steep on the increasing branch, L shallow on the decreasing one);
// u is an integral float in [2^23 + 2^22, ...), so bits(u) - bits(MAGIC) is the entry index.
// Entry = {thr, info}, info = q0 | K << 8 | q1 << 16: the output byte is q0 for h < thr and
// q1 for h >= thr, except inside the entry's window of K + 1 consecutive floats anchored at
// thr (thr and the K floats above it when thr >= +0, the K floats below it when thr <= -0):
// there the f32 chain is not monotone at the ulp level (h (erf(h / sqrt2) + 1) on the
// decreasing branch alternates between two outputs over a few ulps), and the epilogue
// computes those elements with the exact chain (a wave-uniform branch; a window holds a few
// floats of the ~2^31 in play).  Window test: (bits(h) - bits(thr)) <= K, unsigned.
// nqk_gelu_lut_build (nqk_glut.hip) derives every entry from the exact chain and then checks
// the table against the exact chain on every finite f32 h outside the windows (all 2^32 bit
// patterns); a table that differs anywhere is not used.
#pragma once
#include "nqk_numerics.h"

namespace nqk {
namespace {

constexpr int GLUT_MAX = 1024;  // entries of 8 bytes: the builder's capacity (8 KiB)
constexpr int GLUT_CAP1 = 512;  // what the 128 x 256-tile k_pg holds in LDS (4 KiB; two workgroups
                                // per CU); the 256 x 256 one (WM = 2) holds GLUT_MAX
constexpr float GLUT_MAGIC = 0x1.8p23f;
constexpr uint32_t GLUT_MAGIC_BITS = 0x4B400000u;

struct GLutK {
  float iwR, cR, iwL, cL, uhi;
};

// bucket coordinate (the same IEEE operations as the epilogue's packed form)
__device__ __forceinline__ float glut_u(float h, const GLutK& k) {
  const float r = __builtin_fmaf(h, k.iwR, k.cR);
  const float l = __builtin_fmaf(h, k.iwL, k.cL);
  return __builtin_amdgcn_fmed3f(__builtin_fmaxf(r, l), GLUT_MAGIC, k.uhi);
}

// byte B of pk := (h >= thr) ? info[23:16] : info[7:0], the other bytes kept, and the lanes
// whose h lies in the entry's window OR-ed into `slow`: v_cmp + one SDWA v_cndmask that
// selects a word of info and writes one byte of pk, v_sub + an SDWA compare with info[15:8],
// s_or_b64 (a VALU-written SGPR read by SALU: interlocked, like v_cmp -> s_and_saveexec).
// The s_or_b64 writes SCC, so "scc" is a clobber: without it the compiler kept an s_cselect's
// SCC live across the block, and a build that scheduled one there (the unpacked epilogue of
// round-4 call Q / U) stored through a zero-size descriptor
template <int B>
__device__ __forceinline__ uint32_t glut_sel(uint32_t pk, float h, uint32_t thr, uint32_t info, uint64_t& slow) {
  static_assert(B >= 0 && B < 4, "byte");
  uint32_t d;
  uint64_t m;
#define NQK_GLUT_SEL(BS)                                                                                          \
  asm("v_cmp_ge_f32 vcc, %[h], %[t]\n\t"                                                                          \
      "v_cndmask_b32_sdwa %[pk], %[i], %[i], vcc dst_sel:" BS " dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 "    \
      "src1_sel:WORD_1\n\t"                                                                                      \
      "v_sub_u32 %[d], %[h], %[t]\n\t"                                                                            \
      "v_cmp_le_u32_sdwa %[m], %[d], %[i] src0_sel:DWORD src1_sel:BYTE_1\n\t"                                     \
      "s_or_b64 %[s], %[s], %[m]"                                                                                \
      : [pk] "+v"(pk), [d] "=&v"(d), [m] "=&s"(m), [s] "+s"(slow)                                                  \
      : [h] "v"(h), [t] "v"(thr), [i] "v"(info)                                                                  \
      : "vcc", "scc")
  if constexpr (B == 0) NQK_GLUT_SEL("BYTE_0");
  else if constexpr (B == 1) NQK_GLUT_SEL("BYTE_1");
  else if constexpr (B == 2) NQK_GLUT_SEL("BYTE_2");
  else NQK_GLUT_SEL("BYTE_3");
#undef NQK_GLUT_SEL
  return pk;
}
// the same decisions in plain code (the table builder / checker): the output byte outside
// the window, and the window test
__device__ __forceinline__ uint32_t glut_pick(float h, uint32_t thr, uint32_t info) {
  return (h >= __uint_as_float(thr) ? (info >> 16) : info) & 0xffu;
}
__device__ __forceinline__ bool glut_in_window(float h, uint32_t thr, uint32_t info) {
  return __float_as_uint(h) - thr <= ((info >> 8) & 0xffu);
}

// the exact map: GELU chain (gelu_ref) + quantize (clip, rint) of numpy_quantization.py:24-34
__device__ __forceinline__ int glut_exact(float h, double rdiv, float add1, float mul2, double rs, double zp, double lo,
                                          double hi) {
  const float y = gelu_ref(h, rdiv, add1, mul2);
  const float t = (float)((double)y * rs);  // RN32(y / s), s normal (host-checked)
  const double u = zp + (double)t;
  return (int)__builtin_rint(__builtin_fmin(__builtin_fmax(u, lo), hi));
}

}  // namespace
}  // namespace nqk
