// k_pg host side: the weight packers (nqk_pack_pg / nqk_pack_pg4) and the launcher; the
// kernel is nqk_pgemm_kernel.h, its instantiations nqk_pg_inst_*.hip.
#include "nqk_pgemm_kernel.h"

namespace nqk {
namespace {


// weight image of k_pg: [N / 256][K / 64] stages of 256 rows x 64 B in the LDS order of the
// stage (row rho: column 64 (rho >> 6) + pg_bperm(rho & 63) of the panel; physical chunk
// pc: logical chunk pc ^ pg_sw(rho)); columns past N are zero
__global__ void k_pack_pg(const int8_t* __restrict__ bt, int8_t* __restrict__ out, int64_t N, int64_t K, int64_t ldb,
                          int64_t chunks, int layout) {
  const int64_t nk = K / PG_BK;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < chunks; c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t blk = c >> 10, w = c & 1023;
    const int64_t tn = blk / nk, kt = blk - tn * nk;
    const int rho = (int)(w >> 2), pc = (int)(w & 3);
    const int64_t col = tn * PG_BN + 64 * (rho >> 6) + pg_bperm(rho & 63, layout);
    const int lc = pc ^ pg_sw(rho);
    int4 v = make_int4(0, 0, 0, 0);
    if (col < N) v = *reinterpret_cast<const int4*>(bt + col * ldb + kt * PG_BK + lc * 16);
    reinterpret_cast<int4*>(out)[c] = v;
  }
}

// int4 weight image of k_pg<B4> (every value in [-8, 7]): [N / 256][K / 64] stages of 256 rows
// x 32 B, row rho as in k_pack_pg; an 8-byte chunk c (physical chunk c ^ 2 in rows 8..15 of
// a 16-row subtile) holds k = 16 c .. 16 c + 15 of the stage as two words h: byte b of word h
// = k 16 c + 8 h + b in the low nibble, 16 c + 8 h + 4 + b in the high one (the order the
// kernel's AND masks produce: nqk_fused.hip k_pack_b4)
__global__ void k_pack_pg4(const int8_t* __restrict__ bt, uint32_t* __restrict__ out, int64_t N, int64_t K,
                           int64_t ldb, int64_t words, int layout) {
  const int64_t nk = K / PG_BK;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < words; c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t blk = c >> 11, w = c & 2047;  // 2048 words per stage (256 rows x 32 B)
    const int64_t tn = blk / nk, kt = blk - tn * nk;
    const int rho = (int)(w >> 3), pc = (int)((w >> 1) & 3), h = (int)(w & 1);
    const int64_t col = tn * PG_BN + 64 * (rho >> 6) + pg_bperm(rho & 63, layout);
    const int lc = pc ^ (2 * ((rho >> 3) & 1));
    uint32_t v = 0;
    if (col < N) {
      const int8_t* src = bt + col * ldb + kt * PG_BK + 16 * lc + 8 * h;
#pragma unroll
      for (int b = 0; b < 4; ++b) v |= (uint32_t)(((src[b] & 15) | ((src[4 + b] & 15) << 4)) & 0xff) << (8 * b);
    }
    out[c] = v;
  }
}

}  // namespace

// ------------------------------------------------------------------------------ host
extern "C" int nqk_pack_pg(const int8_t* bt, int8_t* out, int64_t N, int64_t K, int64_t ldb, int layout) {
  if (N <= 0 || K <= 0) return 0;
  if (layout != 0 && layout != 1) return fail("nqk_pack_pg: layout must be 0 (int8 outputs) or 1 (f32 outputs)");
  if (K % PG_BK) return fail("nqk_pack_pg: K must be a multiple of 64");
  if ((((uintptr_t)bt) & 15) || (ldb & 15) || (((uintptr_t)out) & 15)) return fail("nqk_pack_pg: unaligned operand");
  const int64_t chunks = (N + PG_BN - 1) / PG_BN * PG_BN * K / 16;
  hipLaunchKernelGGL(k_pack_pg, dim3(grid_for(chunks)), dim3(kThreads), 0, stream(), bt, out, N, K, ldb, chunks, layout);
  return launch_status("nqk_pack_pg");
}

extern "C" int nqk_pack_pg4(const int8_t* bt, uint8_t* out, int64_t N, int64_t K, int64_t ldb, int layout) {
  if (N <= 0 || K <= 0) return 0;
  if (layout != 0 && layout != 1) return fail("nqk_pack_pg4: layout must be 0 (int8 outputs) or 1 (f32 outputs)");
  if (K % PG_BK) return fail("nqk_pack_pg4: K must be a multiple of 64");
  if ((((uintptr_t)bt) & 15) || (ldb & 15) || (((uintptr_t)out) & 15)) return fail("nqk_pack_pg4: unaligned operand");
  const int64_t words = (N + PG_BN - 1) / PG_BN * PG_BN * K / 8;
  hipLaunchKernelGGL(k_pack_pg4, dim3(grid_for(words)), dim3(kThreads), 0, stream(), bt, (uint32_t*)out, N, K, ldb, words,
                     layout);
  return launch_status("nqk_pack_pg4");
}

static int pg_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}

static int pg_num_xcds() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeNumberOfXccs, dev) != hipSuccess ||
        n <= 0)
      n = 8;
  }
  return n;
}

// Launches k_pg for one projection GEMM when it takes the case; returns the kernel id for
// nqk_qgemm_last_kernel (4 k_pg, 6 k_pg with the GELU table) if launched, 0 if the caller
// must use another kernel, < 0 on error.  bp: the nqk_pack_pg image.  (Round 4's k_pg2 —
// the epilogue inside the next tile's k loop — measured slower and was removed)
int pg_launch(int epi, const int8_t* a, const int8_t* bp, int64_t M, int64_t N, int64_t K, int64_t lda,
              const nqk_epilogue* p, bool f32x) {
  if (getenv("NQK_NO_PG")) return 0;
  if (bp == nullptr || p->colterm == nullptr) return 0;
  // b_packed == 2: int4 weights; bp is then the nqk_pack_pg4 nibble image (k_pg<B4>)
  const bool b4 = p->b_packed == 2;
  if (b4 && !(p->bit_width <= 4 && p->col_absmax > 0 && 16.0 * (double)p->col_absmax * (double)llabs(p->zpa) < 2147483647.0))
    return 0;
  if (!(epi == PG_QKV || epi == PG_RESID || epi == PG_GELU)) return 0;
  // K = 192 / 768 / 3072 (ViT-Ti / ViT-B widths and MLP), N % 64 == 0 (a partial last column
  // tile: whole waves past N)
  if (!(K == 192 || K == 768 || K == 3072) || N % 64 != 0 || M < PG_BM) return 0;
  if ((double)M * N * 4.0 >= 4294967295.0 || (double)M * lda >= 4294967295.0) return 0;
  if ((epi == PG_QKV || epi == PG_GELU) && (!f32x || K == 3072)) return 0;
  // residual epilogues need whole 256-column tiles: at N = 192 (ViT-Ti) the 394 row-panel
  // tiles of B = 256 fill 77 % of the slots with a quarter of each tile idle, and the
  // one-tile-per-workgroup kernel is faster (29.1 vs 24.9 us, profiles/r03_vit_tiny_pg.txt)
  if (epi == PG_RESID && N % PG_BN != 0) return 0;
  if (epi == PG_QKV && !(p->hdim == 64 && p->tokens > 0 && p->heads > 0 && p->heads * p->hdim == p->group_cols &&
                         p->group_cols % 64 == 0 && (double)M * p->heads * p->hdim < 2147483647.0))
    return 0;
  // NQK_PG_NORESID=1 keeps the residual epilogues on k_qgemm_big (the round-2 kernel)
  if (epi == PG_RESID && (getenv("NQK_PG_NORESID") || p->resid == nullptr || (M % PG_BM != 0 && p->resid == p->out[0])))
    return 0;
  // WM = 2: 256 x 256 tiles, one 512-thread workgroup per CU, B shared by the two row halves
  // (NQK_PG_WM=1 / 2 forces one form where both exist)
  int wm = 1;
  {
    const char* wv = getenv("NQK_PG_WM");
    if (wv) wm = atoi(wv) == 2 ? 2 : 1;
    if (wm == 2 && (K == 192 || M < 2 * PG_BM || (epi == PG_RESID && M % (2 * PG_BM) != 0 && p->resid == p->out[0])))
      wm = 1;
  }
  if (epi == PG_GELU && !(p->div == 1.41421354f && p->add1 == 1.0f && p->mul2 == 0.5f)) return 0;
  auto al16 = [](const void* q) { return q == nullptr || (((uintptr_t)q) & 15) == 0; };
  if (!al16(p->out[0]) || !al16(p->out[1]) || !al16(p->out[2]) || !al16(p->resid) || !al16(p->colterm) ||
      !al16(p->bias) || !al16(a) || (lda & 15))
    return 0;
  // GELU with a table (nqk_gelu_lut_build): the table holds the exact chain's output bytes
  // (a table of more than GLUT_CAP1 entries needs the 256 x 256-tile form's LDS: ViT-Ti's FFN-up)
  bool glut = epi == PG_GELU && p->gelu_lut != nullptr && p->lut_n > 0 && p->lut_n <= GLUT_MAX &&
              (((uintptr_t)p->gelu_lut) & 15) == 0 && !getenv("NQK_NO_GLUT");
  if (glut && p->lut_n > GLUT_CAP1) {
    if (M >= 2 * PG_BM && !b4 && f32x && (K == 192 || K == 768)) wm = 2;
    else glut = false;
  }
  if (p->bit_width < 2 || p->bit_width > 8) return 0;  // int8 outputs
  const double qlo = -__builtin_ldexp(1.0, p->bit_width - 1), qhi = __builtin_ldexp(1.0, p->bit_width - 1) - 1.0;
  PgEpi e{};
  const int ng = epi == PG_QKV ? 3 : 1;
  for (int g = 0; g < 3; ++g) {
    const int gg = g < ng ? g : 0;
    const float s_out = p->s_out[gg];
    e.sacc[g] = p->s_acc[gg];
    e.s_out[g] = s_out;
    e.rs_out[g] = 1.0 / (double)s_out;
    e.zp_out[g] = (double)p->zp_out[gg];
    e.rsf[g] = s_out != 0.0f ? (float)(1.0 / (double)s_out) : 0.0f;
    e.c1[g] = e.sacc[g] * e.rsf[g];
    e.k1[g] = __builtin_fabsf(e.c1[g]) * NQK_PG_QK1;
    e.zp128[g] = (float)p->zp_out[gg] + 128.0f;
    e.qlo[g] = (float)qlo - (float)p->zp_out[gg];
    e.qhi[g] = (float)qhi - (float)p->zp_out[gg];
    e.magic[g] = 0x1.8p23f + (float)p->zp_out[gg];
    e.out[g] = p->out[gg];
    if (epi != PG_RESID) {
      if (!(__builtin_fabsf(s_out) >= 0x1p-100f && __builtin_fabsf(s_out) <= 0x1p100f)) return 0;
      if (p->zp_out[gg] < -(1 << 20) || p->zp_out[gg] > (1 << 20)) return 0;
    }
  }
  e.bias = p->bias;
  e.resid = p->resid;
  e.colterm = p->colterm;
  e.lo = qlo;
  e.hi = qhi;
  e.blo = (float)qlo + 128.0f;
  e.bhi = (float)qhi + 128.0f;
  e.group_cols = p->group_cols > 0 ? p->group_cols : (int)N;
  e.tokens = p->tokens;
  e.heads = p->heads;
  e.hdim = p->hdim;
  e.div = p->div;
  e.rdiv = 1.0 / (double)p->div;
  e.add1 = p->add1;
  e.mul2 = p->mul2;
  e.ldo = (int)N;
  e.xcds = pg_num_xcds();
  e.lut = glut ? p->gelu_lut : nullptr;
  e.lut_bytes = glut ? (uint32_t)((8 * p->lut_n + 15) & ~15) : 0u;
  e.gk = GLutK{p->lut_k[0], p->lut_k[1], p->lut_k[2], p->lut_k[3], p->lut_k[4]};
  if (epi == PG_GELU) {
    // the GELU filter of nqk_fused.hip make_epi: |gelu_fast - gelu| <= GELU_REL |h| +
    // GELU_ABS, plus the product t = y * rsf
    const double ars = __builtin_fabs(1.0 / (double)p->s_out[0]) * 1.02;
    e.g_rel = (float)(((double)GELU_REL + 0x1.13p-22) * ars);
    const float g_abs = (float)(GELU_ABS * ars) + 0x1p-100f;
    e.g_lim = (float)((0.5 - (double)g_abs) * (1.0 - 0x1p-22));
  }
  // K = 192 (three k steps): NQK_PG_RB=1 keeps the weight panel resident (RB; measured no faster
  // at the ViT-Ti shapes: QKV 23.4 vs 23.4 us, GELU table 34.6 vs 34.9, profiles/r05_tiny_rb_embed_ab.txt)
  const char* rbv = getenv("NQK_PG_RB");
  const bool rb = K == 192 && !b4 && epi != PG_RESID && rbv && atoi(rbv) != 0;
  // K = 192, QKV / GELU, int8: 64-row tiles with NQK_PG_WM0=1 (WM = 0; measured slower: the 128-row
  // form's time is linear in its tiles, a partial last pass costs nothing extra, and the 64-row
  // tiles read B twice per output — QKV 22.8 vs 19.2 us, profiles/r05_pg_rows64_dropped.txt)
  {
    const char* w0 = getenv("NQK_PG_WM0");
    if (K == 192 && wm == 1 && epi != PG_RESID && !b4 && !rb && w0 && atoi(w0) == 1) wm = 0;
  }
  const int bm = wm ? wm * PG_BM : PG_BM / 2;
  const int tiles_n = (int)((N + PG_BN - 1) / PG_BN), tiles_m = (int)((M + bm - 1) / bm);
  const int nt = tiles_m * tiles_n;
  // NQK_PG_WGPC=1: one workgroup per CU (the other half of the register file free for the other
  // stream's kernels: A/B switch with NQK_STREAM_LAG)
  const char* wgpc = getenv("NQK_PG_WGPC");
  const int slots = (wm == 2 || (wgpc && atoi(wgpc) == 1) ? 1 : 2) * pg_num_cus();
  const int kc = K == 3072 ? 2 : (K == 192 ? 1 : 0);
  // a single-line table (lut_k[2] == 0: the L line is -inf) takes the epilogue without it
  const int epi_k = glut ? (p->lut_k[2] == 0.0f ? PG_GLUT1 : PG_GLUT) : epi;
  const bool s8 = epi == PG_QKV && p->bit_width == 8 && !b4 && !getenv("NQK_PG_NOS8");
  const int key = pg_key(epi_k, K == 3072 ? 48 : (K == 192 ? 3 : 12), f32x, b4, s8, wm, rb);
  (void)kc;
  const PgArgs x{a, bp, (int)M, (int)N, (int)lda, tiles_n, nt, nt < slots ? nt : slots, &e};
  // (A tail split — the rows of the whole rounds in one launch, the last round's row panels
  // in a second launch with one workgroup per tile — measured slower: FFN-down 142 -> 176 us,
  // out-proj 77 -> 90 us, profiles/r04_pg_split_dropped.txt)
  if (!(pg_dispatch_i8(key, x) || pg_dispatch_resid(key, x) || pg_dispatch_tiny(key, x) || pg_dispatch_i4(key, x) ||
        pg_dispatch_wm2(key, x)))
    return 0;
  const int rc = launch_status("nqk_qgemm_fused(pg)");
  return rc < 0 ? rc : (glut ? (wm == 2 ? 7 : 6) : (wm == 2 ? 5 : 4));
}

}  // namespace nqk
