// GEMMs of the hot path.
//
//  * nqk_qgemm_i8     — q_matmul's integer product (numpy_quantization.py:47) for
//                       bit widths <= 8 on v_mfma_i32_32x32x32_i8.  int32
//                       accumulation is exact: |a|,|b| <= 128, K < 2^17.
//  * nqk_qgemm_generic — the same product for any storage width, int64 on VALU
//                       (bit widths 9..32, tiny shapes such as the MLP).
//  * nqk_sgemm        — float32 GEMM that reproduces the reference BLAS bit for
//                       bit: OpenBLAS (scipy-openblas 0.3.29, SkylakeX kernels, the
//                       one NumPy 2.2.6 ships on both hosts) cuts K into level-3
//                       blocks (GEMM_Q = 448; a remainder in (Q, 2Q) is halved),
//                       each block a k-ordered fmaf chain from 0, blocks summed in
//                       order.  Verified against np.matmul for K = 64 .. 3072
//                       (tests/test_host.py::test_blas_order_matches_numpy_matmul).
//  * nqk_im2col       — numpy_helper.py:18-70 sliding windows, NCHW input.
#include "nqk_common.h"

namespace nqk {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------------------
// int8 MFMA GEMM: C[b][m][n] = sum_k A[m][k] * Bt[n][k]; block tile 128x128, BK = 64,
// 4 waves (2x2), each wave 64x64 = 2x2 tiles of v_mfma_i32_32x32x32_i8.
// LDS rows are 64 B (4 chunks of 16 B); chunk c of row r sits at c ^ ((r >> 2) & 3) so
// that every ds_read_b128 lane group touches 16 distinct 16-B bank slots.
constexpr int BM = 128, BN = 128, BK = 64;

__device__ __forceinline__ int swz(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4); }

__global__ void __launch_bounds__(256)
k_qgemm_i8(const int8_t* __restrict__ A, const int8_t* __restrict__ Bt, int32_t* __restrict__ C,
           int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, BatchMap bm,
           int64_t a_ms, int64_t b_ms, int64_t c_ms, int tiles_n) {
  __shared__ __attribute__((aligned(16))) int8_t smem[2 * (BM + BN) * BK];
  // buffer `buf`: A tile at smem + buf*(BM+BN)*BK, B tile right after it
#define AS(buf) (smem + (buf) * (BM + BN) * BK)
#define BS(buf) (smem + (buf) * (BM + BN) * BK + BM * BK)

  const int64_t bz = blockIdx.z;
  A += map_a(bm, bz) * a_ms;
  Bt += map_b(bm, bz) * b_ms;
  C += bz * c_ms;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // staging: 512 chunks of 16 B per operand tile, 2 per thread
  v4i ra[2], rb[2];
  auto load_tile = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int idx = tid + i * 256, row = idx >> 2, ch = idx & 3;
      int64_t kk = k0 + ch * 16;
      int64_t gm = m0 + row, gn = n0 + row;
      v4i za = {0, 0, 0, 0};
      ra[i] = (gm < M && kk < K) ? *reinterpret_cast<const v4i*>(A + gm * lda + kk) : za;
      rb[i] = (gn < N && kk < K) ? *reinterpret_cast<const v4i*>(Bt + gn * ldb + kk) : za;
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int idx = tid + i * 256, row = idx >> 2, ch = idx & 3;
      *reinterpret_cast<v4i*>(AS(buf) + swz(row, ch)) = ra[i];
      *reinterpret_cast<v4i*>(BS(buf) + swz(row, ch)) = rb[i];
    }
  };

  v16i acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;

  const int nk = (int)((K + BK - 1) / BK);
  load_tile(0);
  store_tile(0);
  __syncthreads();
  const int r32 = lane & 31, half = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tile((int64_t)(kt + 1) * BK);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      v4i fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = *reinterpret_cast<const v4i*>(AS(cur) + swz(wm * 64 + i * 32 + r32, 2 * s + half));
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = *reinterpret_cast<const v4i*>(BS(cur) + swz(wn * 64 + j * 32 + r32, 2 * s + half));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      store_tile(cur ^ 1);
    }
    __syncthreads();
  }
  // C/D layout (gfx950, dtype independent): col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      int64_t gn = n0 + wn * 64 + j * 32 + r32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int64_t gm = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (gm < M && gn < N) C[gm * ldc + gn] = acc[i][j][r];
      }
    }
#undef AS
#undef BS
}

// ---------------------------------------------------------------------------------------
// generic integer GEMM (int64 accumulate): 16x16 threads, one output each, LDS k-tiles
template <typename TA, typename TB>
__global__ void __launch_bounds__(256)
k_qgemm_generic(const TA* __restrict__ A, const TB* __restrict__ B, int64_t* __restrict__ C, int64_t M,
                int64_t N, int64_t K, int64_t a_sm, int64_t a_sk, int64_t b_sk, int64_t b_sn, int64_t ldc,
                BatchMap bm, int64_t a_ms, int64_t b_ms, int64_t c_ms) {
  __shared__ int64_t sa[16][17], sb[16][17];
  const int64_t bz = blockIdx.z;
  A += map_a(bm, bz) * a_ms;
  B += map_b(bm, bz) * b_ms;
  C += bz * c_ms;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int64_t m = (int64_t)blockIdx.y * 16 + ty, n = (int64_t)blockIdx.x * 16 + tx;
  int64_t acc = 0;
  for (int64_t k0 = 0; k0 < K; k0 += 16) {
    int64_t am = (int64_t)blockIdx.y * 16 + ty, ak = k0 + tx;
    sa[ty][tx] = (am < M && ak < K) ? (int64_t)A[am * a_sm + ak * a_sk] : 0;
    int64_t bk = k0 + ty, bn = (int64_t)blockIdx.x * 16 + tx;
    sb[ty][tx] = (bk < K && bn < N) ? (int64_t)B[bk * b_sk + bn * b_sn] : 0;
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) acc += sa[ty][kk] * sb[kk][tx];
    __syncthreads();
  }
  if (m < M && n < N) C[m * ldc + n] = acc;
}

// ---------------------------------------------------------------------------------------
// float32 GEMM in the reference BLAS's summation order.  64x64 tile, 256 threads,
// 4x4 outputs per thread, LDS k-tiles of 16.  `kb` holds the K-block ends.
struct KBlocks { int n; int64_t end[24]; };

__global__ void __launch_bounds__(256)
k_sgemm_blas(const float* __restrict__ A, const float* __restrict__ B, float* __restrict__ C, int64_t M,
             int64_t N, int64_t K, int64_t a_sm, int64_t a_sk, int64_t b_sk, int64_t b_sn, int64_t ldc,
             BatchMap bm, int64_t a_ms, int64_t b_ms, int64_t c_ms, KBlocks kb) {
  __shared__ float sa[16][64 + 4], sb[16][64 + 4];
  const int64_t bz = blockIdx.z;
  A += map_a(bm, bz) * a_ms;
  B += map_b(bm, bz) * b_ms;
  C += bz * c_ms;
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int64_t m0 = (int64_t)blockIdx.y * 64, n0 = (int64_t)blockIdx.x * 64;
  float acc[4][4], tot[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) { acc[i][j] = 0.0f; tot[i][j] = 0.0f; }
  int blk = 0;
  int64_t bend = kb.end[0];
  for (int64_t k0 = 0; k0 < K; k0 += 16) {
    // stage A[m0..+64][k0..+16] and B[k0..+16][n0..+64]
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int idx = tid + i * 256;
      int r = idx >> 4, kk = idx & 15;   // A: 64 rows x 16 k
      int64_t gm = m0 + r, gk = k0 + kk;
      sa[kk][r] = (gm < M && gk < K) ? A[gm * a_sm + gk * a_sk] : 0.0f;
      int kr = idx >> 6, cc = idx & 63;  // B: 16 k x 64 cols
      int64_t bk = k0 + kr, bn = n0 + cc;
      sb[kr][cc] = (bk < K && bn < N) ? B[bk * b_sk + bn * b_sn] : 0.0f;
    }
    __syncthreads();
    const int kmax = (int)((K - k0) < 16 ? (K - k0) : 16);
    for (int kk = 0; kk < kmax; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = sa[kk][ty * 4 + i];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = sb[kk][tx * 4 + j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_fmaf(a[i], b[j], acc[i][j]);
      if (k0 + kk + 1 == bend) {  // end of an OpenBLAS K block: C += block sum
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) { tot[i][j] = tot[i][j] + acc[i][j]; acc[i][j] = 0.0f; }
        ++blk;
        bend = blk < kb.n ? kb.end[blk] : -1;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int64_t gm = m0 + ty * 4 + i;
    if (gm >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int64_t gn = n0 + tx * 4 + j;
      if (gn < N) C[gm * ldc + gn] = tot[i][j];
    }
  }
}

// float32 GEMM on v_mfma_f32_32x32x2_f32: each output is a k-ordered fmaf chain
// (the instruction's numerics, bit for bit — MI355X_MICROARCH.md / cdna_hip_programming.md
// 'FP32-input MFMA'), so the same BLAS-order K blocking as k_sgemm_blas gives the same
// bits at the MFMA rate.  128x128 tile, 4 waves (2x2, 64x64 each = 2x2 tiles of 32x32),
// k-tiles of 16 staged k-major in LDS (one f32 per lane per MFMA operand).  Needs every
// K-block end even (K even), since one MFMA consumes k and k+1.
// EMBED epilogue (ViT patch embedding, plan.py FusedEmbed): row m = image * HW + patch of
// the im2col GEMM goes to out[image][1 + patch][n] = (C + bias[n]) + pos[1 + patch][n],
// i.e. Conv's bias add, the NCHW -> [B, HW, C] Reshape/Transpose, the Concat behind the
// class token and the position-embedding Add, in the node loop's order of roundings.
struct EmbedEpi {
  const float* bias;
  const float* pos;  // [HW + 1][N]
  int64_t hw;
  int xcd;  // k_embed_q: the XCD count for the XCD-aware tile order (a row panel's column tiles on one XCD), 0 = off
};

template <bool EMBED, bool AL16, bool VEC = false>
__global__ void __launch_bounds__(256, 2)
k_sgemm_mfma(const float* __restrict__ A, const float* __restrict__ B, float* __restrict__ C, int64_t M,
             int64_t N, int64_t K, int64_t a_sm, int64_t a_sk, int64_t b_sk, int64_t b_sn, int64_t ldc,
             BatchMap bm, int64_t a_ms, int64_t b_ms, int64_t c_ms, KBlocks kb, EmbedEpi ee) {
  typedef float v16f __attribute__((ext_vector_type(16)));
  __shared__ float sa[2][16][128 + 4], sb[2][16][128 + 4];
  const int64_t bz = blockIdx.z;
  A += map_a(bm, bz) * a_ms;
  B += map_b(bm, bz) * b_ms;
  C += bz * c_ms;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, r32 = lane & 31, h = lane >> 5;
  const int64_t m0 = (int64_t)blockIdx.y * 128, n0 = (int64_t)blockIdx.x * 128;
  float ra[8], rb[8];
  // VEC (unit k stride of A, unit n stride of B, K % 16 == 0, N % 4 == 0, 16-byte
  // aligned rows): the same tiles by two 16-byte loads per operand and thread
  float4 va[2], vb[2];
  auto load = [&](int64_t k0) {
    if constexpr (VEC) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int idx = tid + i * 256;
        const int r = idx >> 2, c = idx & 3;      // A: row r, k 4c .. 4c + 3
        const int64_t gm = m0 + r;
        va[i] = gm < M ? *reinterpret_cast<const float4*>(A + gm * a_sm + k0 + 4 * c) : make_float4(0, 0, 0, 0);
        const int kr = idx >> 5, cc = (idx & 31) * 4;  // B: k row kr, columns cc .. cc + 3
        const int64_t bn = n0 + cc;
        vb[i] = bn < N ? *reinterpret_cast<const float4*>(B + (k0 + kr) * b_sk + bn) : make_float4(0, 0, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = tid + i * 256;
      const int kk = idx & 15, r = idx >> 4;  // A: 128 rows x 16 k (k fastest)
      const int64_t gm = m0 + r, gk = k0 + kk;
      ra[i] = (gm < M && gk < K) ? A[gm * a_sm + gk * a_sk] : 0.0f;
      const int kr = idx >> 7, cc = idx & 127;  // B: 16 k x 128 cols (cols fastest)
      const int64_t bk = k0 + kr, bn = n0 + cc;
      rb[i] = (bk < K && bn < N) ? B[bk * b_sk + bn * b_sn] : 0.0f;
    }
  };
  auto store = [&](int buf) {
    if constexpr (VEC) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int idx = tid + i * 256;
        const int r = idx >> 2, c = idx & 3;
        sa[buf][4 * c + 0][r] = va[i].x;
        sa[buf][4 * c + 1][r] = va[i].y;
        sa[buf][4 * c + 2][r] = va[i].z;
        sa[buf][4 * c + 3][r] = va[i].w;
        *reinterpret_cast<float4*>(&sb[buf][idx >> 5][(idx & 31) * 4]) = vb[i];
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int idx = tid + i * 256;
      sa[buf][idx & 15][idx >> 4] = ra[i];
      sb[buf][idx >> 7][idx & 127] = rb[i];
    }
  };
  v16f acc[2][2], tot[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = tot[i][j][r] = 0.0f;
  int blk = 0;
  int64_t bend = kb.n > 0 ? kb.end[0] : -1;
  const int64_t nk = (K + 15) / 16;
  load(0);
  store(0);
  __syncthreads();
  for (int64_t kt = 0; kt < nk; ++kt) {
    const int cur = (int)(kt & 1);
    if (kt + 1 < nk) load((kt + 1) * 16);
    const int64_t k0 = kt * 16;
    if constexpr (AL16) {
      // K and every BLAS block end are multiples of 16: a whole static k-tile, the block
      // boundary (if any) at its end
#pragma unroll
      for (int kk = 0; kk < 16; kk += 2) {
        float a[2], b[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = sa[cur][kk + h][wm * 64 + i * 32 + r32];
#pragma unroll
        for (int j = 0; j < 2; ++j) b[j] = sb[cur][kk + h][wn * 64 + j * 32 + r32];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
      }
      if (k0 + 16 == bend) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              tot[i][j][r] = tot[i][j][r] + acc[i][j][r];
              acc[i][j][r] = 0.0f;
            }
        ++blk;
        bend = blk < kb.n ? kb.end[blk] : -1;
      }
      if (kt + 1 < nk) store(cur ^ 1);
      __syncthreads();
      continue;
    }
    const int kmax = (int)((K - k0) < 16 ? (K - k0) : 16);  // even
    for (int kk = 0; kk < kmax; kk += 2) {
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = sa[cur][kk + h][wm * 64 + i * 32 + r32];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = sb[cur][kk + h][wn * 64 + j * 32 + r32];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
      if (k0 + kk + 2 == bend) {  // end of an OpenBLAS K block: C += block sum
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              tot[i][j][r] = tot[i][j][r] + acc[i][j][r];
              acc[i][j][r] = 0.0f;
            }
        ++blk;
        bend = blk < kb.n ? kb.end[blk] : -1;
      }
    }
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t gn = n0 + wn * 64 + j * 32 + r32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t gm = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (gm < M && gn < N) {
          if constexpr (EMBED) {
            const uint32_t img = (uint32_t)gm / (uint32_t)ee.hw, t = (uint32_t)gm - img * (uint32_t)ee.hw;
            const float y = tot[i][j][r] + ee.bias[gn];
            C[((int64_t)img * (ee.hw + 1) + 1 + t) * N + gn] = y + ee.pos[(1 + (int64_t)t) * N + gn];
          } else {
            C[gm * ldc + gn] = tot[i][j][r];
          }
        }
      }
    }
}

// Patch embedding with the patchify + dequantize folded into the A-operand load (round 3):
// the quantized image (int8, NCHW, 3 channels, 16 x 16 patches) is read directly and the
// dequantized im2col matrix never exists.  Same numerics as k_patchify_dequant +
// k_sgemm_mfma<EMBED>: A[m][k] = f32((q - zp) * s) with k = (ki, kj, ci); each output a
// k-ordered fmaf chain per BLAS K block (v_mfma_f32_32x32x2_f32 is one, tools/micro/f32mfma),
// blocks summed in order, then bias and position embedding.  128 x (64 WN) tiles, 4 waves
// (2 x 2), k-tiles of 16.  Operands sit in LDS as [row][16 k] with the k order permuted to
// p = (k & 1) * 8 + (k >> 1) and 20-float rows, so a lane's 8 k values of one MFMA sub-tile
// come in two conflict-free ds_read_b128 (k_sgemm_mfma: 32 ds_read_b32 per k-tile).  The
// weights are pre-arranged once per plan as wt[N][K] in that order (plan.py FusedEmbed).
// A: the thread of row r (tid & 127) and half hf (tid >> 7, wave-uniform) keeps the 3 channel
// rows (3 x 16 B) of its patch for the current kernel row ki (3 k-tiles) in registers and
// writes its 8 k values of each k-tile as two ds_write_b128.
// XCDs of the device (hipDeviceAttributeNumberOfXccs; 8 on MI355X): the round-robin unit of the
// XCD-aware tile orders (not a constant)
static int num_xcds() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeNumberOfXccs, dev) != hipSuccess ||
        n <= 0)
      n = 8;
  }
  return n;
}
constexpr int EQ_ROW = 20;  // floats per LDS operand row (16 + 4 padding)
#ifndef NQK_EMBED_PXD
#define NQK_EMBED_PXD 1
#endif
#ifndef NQK_EMBED_DIAG
#define NQK_EMBED_DIAG 0  // timing diagnostics (wrong results): 1 no k-tile barriers, 2 no A convert, 4 no stores
#endif
template <int WN>
__global__ void __launch_bounds__(256, 2)
k_embed_q(const int8_t* __restrict__ q, const float* __restrict__ wt, float* __restrict__ C, int64_t M, int64_t N,
          int64_t hw, int64_t wo, int64_t H, int64_t W, float s, float zpf, KBlocks kb, EmbedEpi ee) {
  typedef float v16f __attribute__((ext_vector_type(16)));
  typedef float v4f __attribute__((ext_vector_type(4)));
  constexpr int BN = 64 * WN, K = 768;
  __shared__ __attribute__((aligned(16))) float sa[2][128 * EQ_ROW];
  __shared__ __attribute__((aligned(16))) float sb[2][BN * EQ_ROW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, r32 = lane & 31, h = lane >> 5;
  // XCD-aware tile order (ee.xcd): blocks are dealt round-robin over the 8 XCDs (block b on XCD
  // b % 8, MI355X_MICROARCH.md), so the row-panel-major tile ids are split into 8 contiguous bands,
  // band x served by the blocks of XCD x: the column tiles of one row panel — which read the same
  // image rows — share an L2 instead of fetching the image once per XCD
  int64_t tm = blockIdx.y, tn = blockIdx.x;
  if (ee.xcd) {
    const int64_t gx = gridDim.x, T = gx * gridDim.y, b = (int64_t)blockIdx.y * gx + blockIdx.x;
    const int64_t XC = ee.xcd, x = b % XC, q8 = T / XC, r8 = T % XC;
    const int64_t tile = x * q8 + (x < r8 ? x : r8) + b / 8;
    tm = tile / gx;
    tn = tile - tm * gx;
  }
  const int64_t m0 = tm * 128, n0 = tn * BN;
  // A rows of this thread: patch m = image * hw + oy * wo + ox
  const int ar = tid & 127, hf = tid >> 7;
  const int64_t am = m0 + ar < M ? m0 + ar : M - 1;
  const int64_t img = am / hw, pt = am - img * hw, oy = pt / wo, ox = pt - oy * wo;
  const int8_t* qrow = q + ((img * 3) * H + oy * 16) * W + ox * 16;  // channel 0, kernel row 0
  const int64_t cstride = H * W;
  int4 px[3], pxn[3];
  auto load_px = [&](int ki, int4 (&d)[3]) {
#pragma unroll
    for (int ci = 0; ci < 3; ++ci) d[ci] = *reinterpret_cast<const int4*>(qrow + ci * cstride + (int64_t)ki * W);
  };
  // B: thread t moves column cb = t >> 2 (and cb + 64 for WN = 2), k quarter t & 3
  const int cb = tid >> 2, kq = tid & 3;
  v4f bv[WN];
  auto load_b = [&](int kt) {
#pragma unroll
    for (int u = 0; u < WN; ++u) {
      const int64_t n = n0 + cb + 64 * u;
      bv[u] = n < N ? *reinterpret_cast<const v4f*>(wt + n * K + kt * 16 + 4 * kq) : v4f{0, 0, 0, 0};
    }
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int u = 0; u < WN; ++u) *reinterpret_cast<v4f*>(&sb[buf][(cb + 64 * u) * EQ_ROW + 4 * kq]) = bv[u];
  };
  // A values of k-tile sub (0..2 within kernel row): k_local = 8 hf + e -> j = 16 sub + k_local,
  // kj = j / 3, ci = j % 3; written at p = (k_local & 1) * 8 + (k_local >> 1)
  // (hf is wave-uniform: a scalar branch picks the half, so each value is one SDWA byte
  // convert, a subtract and a multiply)
  auto conv_a = [&](auto SUB, auto HF, const int4 (&d)[3], float (&f)[8]) __attribute__((always_inline)) {
    constexpr int sub = decltype(SUB)::value, half = decltype(HF)::value;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int j = 16 * sub + 8 * half + e, kj = j / 3, c = j % 3;
      const int w = (kj >> 2) == 0 ? d[c].x : (kj >> 2) == 1 ? d[c].y : (kj >> 2) == 2 ? d[c].z : d[c].w;
      f[e] = ((float)(int)(int8_t)(w >> (8 * (kj & 3))) - zpf) * s;
    }
  };
  auto store_a = [&](int buf, auto SUB, const int4 (&d)[3]) __attribute__((always_inline)) {
    float f[8];
    if constexpr ((NQK_EMBED_DIAG & 2) != 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = __int_as_float(d[e % 3].x);
    } else if (hf) conv_a(SUB, std::integral_constant<int, 1>{}, d, f);
    else conv_a(SUB, std::integral_constant<int, 0>{}, d, f);
    float* dst = &sa[buf][ar * EQ_ROW + 4 * hf];
    *reinterpret_cast<v4f*>(dst) = v4f{f[0], f[2], f[4], f[6]};      // k_local even -> p = k_local / 2
    *reinterpret_cast<v4f*>(dst + 8) = v4f{f[1], f[3], f[5], f[7]};  // odd -> 8 + k_local / 2
  };
  v16f acc[2][WN], tot[2][WN];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = tot[i][j][r] = 0.0f;
  int blk = 0;
  int64_t bend = kb.n > 0 ? kb.end[0] : -1;
  load_px(0, px);
  load_b(0);
  store_a(0, std::integral_constant<int, 0>{}, px);
  store_b(0);
  __syncthreads();
  constexpr int NKT = K / 16;
  // one k-tile; SUB = kt % 3 at compile time (the kernel row ki = kt / 3 in px)
  auto step = [&](int kt, auto SUB) __attribute__((always_inline)) {
    constexpr int sub = decltype(SUB)::value;
    const int cur = kt & 1;
    const bool more = kt + 1 < NKT;
    if (more) {
      load_b(kt + 1);
      // the next kernel row's image bytes (HBM): NQK_EMBED_PXD 1 = issued at the row's first
      // k-tile, three k-tiles before their use; 0 = in the k-tile before it
      if constexpr (NQK_EMBED_PXD == 0 && sub == 2) load_px((kt + 1) / 3, pxn);
    }
    if constexpr (NQK_EMBED_PXD == 1 && sub == 0) {
      if (kt + 3 < NKT) load_px(kt / 3 + 1, pxn);
    }
    v4f fa[2][2], fb[WN][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float* src = &sa[cur][(wm * 64 + i * 32 + r32) * EQ_ROW + 8 * h];
      fa[i][0] = *reinterpret_cast<const v4f*>(src);
      fa[i][1] = *reinterpret_cast<const v4f*>(src + 4);
    }
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const float* src = &sb[cur][(wn * 32 * WN + j * 32 + r32) * EQ_ROW + 8 * h];
      fb[j][0] = *reinterpret_cast<const v4f*>(src);
      fb[j][1] = *reinterpret_cast<const v4f*>(src + 4);
    }
#pragma unroll
    for (int kk = 0; kk < 8; ++kk)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][kk >> 2][kk & 3], fb[j][kk >> 2][kk & 3], acc[i][j], 0, 0, 0);
    if ((int64_t)kt * 16 + 16 == bend) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            tot[i][j][r] = tot[i][j][r] + acc[i][j][r];
            acc[i][j][r] = 0.0f;
          }
      ++blk;
      bend = blk < kb.n ? kb.end[blk] : -1;
    }
    if (more) {
      if constexpr (sub == 2) {
#pragma unroll
        for (int ci = 0; ci < 3; ++ci) px[ci] = pxn[ci];
      }
      store_a(cur ^ 1, std::integral_constant<int, (sub + 1) % 3>{}, px);
      store_b(cur ^ 1);
    }
    if constexpr ((NQK_EMBED_DIAG & 1) == 0) __syncthreads();
  };
  for (int ki = 0; ki < NKT / 3; ++ki) {
    step(3 * ki, std::integral_constant<int, 0>{});
    step(3 * ki + 1, std::integral_constant<int, 1>{});
    step(3 * ki + 2, std::integral_constant<int, 2>{});
  }
  // epilogue: per output row gm its image im = gm / hw (a float reciprocal, corrected by one
  // either way: gm < 2^24), output row gm + im + 1 (after the image's class-token row),
  // position row gm - im hw + 1; bias once per column
  // (32-bit element offsets: (M + images) N < 2^31, host-checked)
  const int hwi = (int)ee.hw, Ni = (int)N, Mi = (int)M;
  const float rhw = 1.0f / (float)hwi;
  float bj[WN];
  int gnj[WN];
#pragma unroll
  for (int j = 0; j < WN; ++j) {
    gnj[j] = (int)n0 + wn * 32 * WN + j * 32 + r32;
    bj[j] = gnj[j] < Ni ? ee.bias[gnj[j]] : 0.0f;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int gm = (int)m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (gm >= Mi) continue;
      int im = (int)((float)gm * rhw);
      im = im * hwi > gm ? im - 1 : im;
      im = (im + 1) * hwi <= gm ? im + 1 : im;
      const int co = (gm + im + 1) * Ni, po = (gm - im * hwi + 1) * Ni;
#pragma unroll
      for (int j = 0; j < WN; ++j)
        if (gnj[j] < Ni) {
          const float v = (tot[i][j][r] + bj[j]) + ee.pos[po + gnj[j]];
          if constexpr ((NQK_EMBED_DIAG & 4) != 0) asm volatile("" ::"v"(v));
          else C[co + gnj[j]] = v;
        }
    }
}

// k_embed_q on v_mfma_f32_16x16x4_f32 (round 6).  Same tiles (128 x 64 WN, 4 waves 2 x 2, k-tiles of
// 16, double-buffered LDS), same numerics: one 16x16x4 instruction accumulates its 4 k-products in
// order with a rounding after each (an fmaf chain, tools/micro/f32mfma: 0 of 12 800 outputs differ),
// so every output is still the k-ordered chain per BLAS K block.  Why: the chip holds a higher clock
// under the 16x16 f32 form than under 32x32x2 with operands from LDS (MI355X_MICROARCH.md, DVFS item 7).
// A wave's 64 x 32 WN tile is 4 x 2 WN blocks of 16 x 16; lane (l16 = l & 15, g = l >> 4) supplies
// A[row l16][k0 + g] and B[k0 + g][col l16] for k0 = 0, 4, 8, 12, i.e. k = 4 q + g for q = 0..3: the
// LDS rows hold each 16-k tile permuted to p = (k & 3) * 4 + (k >> 2), so a lane's four values are one
// ds_read_b128 (24-float rows: conflict-free in every ds_read_b128 lane group); the weights come in
// that order (plan.py FusedEmbed, nqk.h).
constexpr int EQ16_ROW = 24;
template <int WN>
__global__ void __launch_bounds__(256, 2)
k_embed_q16(const int8_t* __restrict__ q, const float* __restrict__ wt, float* __restrict__ C, int64_t M, int64_t N,
            int64_t hw, int64_t wo, int64_t H, int64_t W, float s, float zpf, KBlocks kb, EmbedEpi ee) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  typedef float v2f __attribute__((ext_vector_type(2)));
  constexpr int BN = 64 * WN, K = 768, NJ = 2 * WN;
  __shared__ __attribute__((aligned(16))) float sa[2][128 * EQ16_ROW];
  __shared__ __attribute__((aligned(16))) float sb[2][BN * EQ16_ROW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, l16 = lane & 15, g = lane >> 4;
  int64_t tm = blockIdx.y, tn = blockIdx.x;
  if (ee.xcd) {  // XCD-aware tile order, as k_embed_q
    const int64_t gx = gridDim.x, T = gx * gridDim.y, b = (int64_t)blockIdx.y * gx + blockIdx.x;
    const int64_t XC = ee.xcd, x = b % XC, q8 = T / XC, r8 = T % XC;
    const int64_t tile = x * q8 + (x < r8 ? x : r8) + b / XC;
    tm = tile / gx;
    tn = tile - tm * gx;
  }
  const int64_t m0 = tm * 128, n0 = tn * BN;
  const int ar = tid & 127, hf = tid >> 7;
  const int64_t am = m0 + ar < M ? m0 + ar : M - 1;
  const int64_t img = am / hw, pt = am - img * hw, oy = pt / wo, ox = pt - oy * wo;
  const int8_t* qrow = q + ((img * 3) * H + oy * 16) * W + ox * 16;
  const int64_t cstride = H * W;
  int4 px[3], pxn[3];
  auto load_px = [&](int ki, int4 (&d)[3]) {
#pragma unroll
    for (int ci = 0; ci < 3; ++ci) d[ci] = *reinterpret_cast<const int4*>(qrow + ci * cstride + (int64_t)ki * W);
  };
  const int cb = tid >> 2, kq = tid & 3;
  v4f bv[WN];
  auto load_b = [&](int kt) {
#pragma unroll
    for (int u = 0; u < WN; ++u) {
      const int64_t n = n0 + cb + 64 * u;
      bv[u] = n < N ? *reinterpret_cast<const v4f*>(wt + n * K + kt * 16 + 4 * kq) : v4f{0, 0, 0, 0};
    }
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int u = 0; u < WN; ++u) *reinterpret_cast<v4f*>(&sb[buf][(cb + 64 * u) * EQ16_ROW + 4 * kq]) = bv[u];
  };
  // A values of k-tile sub: k_local = 8 hf + e, written at p = (e & 3) * 4 + 2 hf + (e >> 2): the
  // pairs (e, e + 4) are adjacent, four 8-byte stores
  auto conv_a = [&](auto SUB, auto HF, const int4 (&d)[3], float (&f)[8]) __attribute__((always_inline)) {
    constexpr int sub = decltype(SUB)::value, half = decltype(HF)::value;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int j = 16 * sub + 8 * half + e, kj = j / 3, c = j % 3;
      const int w = (kj >> 2) == 0 ? d[c].x : (kj >> 2) == 1 ? d[c].y : (kj >> 2) == 2 ? d[c].z : d[c].w;
      f[e] = ((float)(int)(int8_t)(w >> (8 * (kj & 3))) - zpf) * s;
    }
  };
  auto store_a = [&](int buf, auto SUB, const int4 (&d)[3]) __attribute__((always_inline)) {
    float f[8];
    if (hf) conv_a(SUB, std::integral_constant<int, 1>{}, d, f);
    else conv_a(SUB, std::integral_constant<int, 0>{}, d, f);
    float* dst = &sa[buf][ar * EQ16_ROW + 2 * hf];
#pragma unroll
    for (int e = 0; e < 4; ++e) *reinterpret_cast<v2f*>(dst + 4 * e) = v2f{f[e], f[e + 4]};
  };
  v4f acc[4][NJ], tot[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = tot[i][j] = v4f{0, 0, 0, 0};
  int blk = 0;
  int64_t bend = kb.n > 0 ? kb.end[0] : -1;
  load_px(0, px);
  load_b(0);
  store_a(0, std::integral_constant<int, 0>{}, px);
  store_b(0);
  __syncthreads();
  constexpr int NKT = K / 16;
  auto step = [&](int kt, auto SUB) __attribute__((always_inline)) {
    constexpr int sub = decltype(SUB)::value;
    const int cur = kt & 1;
    const bool more = kt + 1 < NKT;
    if (more) load_b(kt + 1);
    if constexpr (sub == 0) {
      if (kt + 3 < NKT) load_px(kt / 3 + 1, pxn);
    }
    v4f fb[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      fb[j] = *reinterpret_cast<const v4f*>(&sb[cur][(wn * 32 * WN + 16 * j + l16) * EQ16_ROW + 4 * g]);
    // row block by row block (one A fragment live at a time): 4 NJ MFMAs per block, the NJ
    // accumulators of a block in rotation
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const v4f fa = *reinterpret_cast<const v4f*>(&sa[cur][(wm * 64 + 16 * i + l16) * EQ16_ROW + 4 * g]);
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[qq], fb[j][qq], acc[i][j], 0, 0, 0);
    }
    if ((int64_t)kt * 16 + 16 == bend) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          tot[i][j] = tot[i][j] + acc[i][j];
          acc[i][j] = v4f{0, 0, 0, 0};
        }
      ++blk;
      bend = blk < kb.n ? kb.end[blk] : -1;
    }
    if (more) {
      if constexpr (sub == 2) {
#pragma unroll
        for (int ci = 0; ci < 3; ++ci) px[ci] = pxn[ci];
      }
      store_a(cur ^ 1, std::integral_constant<int, (sub + 1) % 3>{}, px);
      store_b(cur ^ 1);
    }
    __syncthreads();
  };
  for (int ki = 0; ki < NKT / 3; ++ki) {
    step(3 * ki, std::integral_constant<int, 0>{});
    step(3 * ki + 1, std::integral_constant<int, 1>{});
    step(3 * ki + 2, std::integral_constant<int, 2>{});
  }
  // epilogue (as k_embed_q): lane holds rows 16 i + 4 g + r, column 16 j + l16 of the wave tile
  const int hwi = (int)ee.hw, Ni = (int)N, Mi = (int)M;
  const float rhw = 1.0f / (float)hwi;
  float bj[NJ];
  int gnj[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    gnj[j] = (int)n0 + wn * 32 * WN + 16 * j + l16;
    bj[j] = gnj[j] < Ni ? ee.bias[gnj[j]] : 0.0f;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gm = (int)m0 + wm * 64 + 16 * i + 4 * g + r;
      if (gm >= Mi) continue;
      int im = (int)((float)gm * rhw);
      im = im * hwi > gm ? im - 1 : im;
      im = (im + 1) * hwi <= gm ? im + 1 : im;
      const int co = (gm + im + 1) * Ni, po = (gm - im * hwi + 1) * Ni;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        if (gnj[j] < Ni) C[co + gnj[j]] = (tot[i][j][r] + bj[j]) + ee.pos[po + gnj[j]];
    }
}

// class-token rows of the EMBED output: out[image][0][n] = cls[n] + pos[0][n]
__global__ void k_embed_cls(const float* __restrict__ cls, const float* __restrict__ pos, float* __restrict__ out,
                            int64_t images, int64_t hw, int64_t n) {
  const int64_t total = images * n, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int64_t img = i / n, c = i - img * n;
    out[img * (hw + 1) * n + c] = cls[c] + pos[c];
  }
}

// im2col of a patchify Conv (stride = kernel, no padding) fused with the dequantize of
// its quantized input (model.py: QModel dequantizes a QTensor before a float op):
// cols[(b, oy, ox)][(ki, kj, ci)] = f32((q[b][ci][oy*kh + ki][ox*kw + kj] - zp) * s).
// f32 (q - zp) * s is the f64 dequant exactly: |q - zp| < 2^24, one rounding.
// One thread per (patch row m, ki): kw * c consecutive outputs.
template <bool VEC16>
__global__ void k_patchify_dequant(const int8_t* __restrict__ q, float* __restrict__ cols, int64_t n, int64_t c,
                                   int64_t h, int64_t w, int64_t kh, int64_t kw, float s, float zpf) {
  const int64_t ho = h / kh, wo = w / kw, M = n * ho * wo;
  const int64_t total = M * kh, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int64_t m = i / kh, ki = i - m * kh;
    const int64_t b = m / (ho * wo), p = m - b * (ho * wo), oy = p / wo, ox = p - oy * wo;
    float* dst = cols + m * (kh * kw * c) + ki * kw * c;
    if constexpr (VEC16) {
      // c == 3 (RGB): the 48 outputs (kj, ci) are contiguous -> 12 float4 stores
      int wv[3][4];
#pragma unroll
      for (int ci = 0; ci < 3; ++ci) {
        const int4 v = *reinterpret_cast<const int4*>(q + ((b * 3 + ci) * h + oy * kh + ki) * w + ox * 16);
        wv[ci][0] = v.x; wv[ci][1] = v.y; wv[ci][2] = v.z; wv[ci][3] = v.w;
      }
#pragma unroll
      for (int o = 0; o < 12; ++o) {
        float f[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int j = 4 * o + e, kj = j / 3, ci = j % 3;
          const int qv = (int)(int8_t)(wv[ci][kj >> 2] >> (8 * (kj & 3)));
          f[e] = ((float)qv - zpf) * s;
        }
        *reinterpret_cast<float4*>(dst + 4 * o) = make_float4(f[0], f[1], f[2], f[3]);
      }
    } else {
      for (int64_t ci = 0; ci < c; ++ci) {
        const int8_t* src = q + ((b * c + ci) * h + oy * kh + ki) * w + ox * kw;
        for (int64_t kj = 0; kj < kw; ++kj) dst[kj * c + ci] = ((float)src[kj] - zpf) * s;
      }
    }
  }
}

__global__ void k_im2col(const float* __restrict__ x, float* __restrict__ cols, int64_t n, int64_t c, int64_t h,
                         int64_t w, int64_t kh, int64_t kw, int64_t ph0, int64_t pw0, int64_t sh, int64_t sw,
                         int64_t ho, int64_t wo) {
  const int64_t kcols = kh * kw * c;
  const int64_t total = n * ho * wo * kcols;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    int64_t row = i / kcols, col = i - row * kcols;
    int64_t ci = col % c, t = col / c, kj = t % kw, ki = t / kw;
    int64_t ox = row % wo, t2 = row / wo, oy = t2 % ho, b = t2 / ho;
    int64_t iy = oy * sh + ki - ph0, ix = ox * sw + kj - pw0;
    float v = 0.0f;
    if (iy >= 0 && iy < h && ix >= 0 && ix < w) v = x[((b * c + ci) * h + iy) * w + ix];
    cols[i] = v;
  }
}

// ---------------------------------------------------------------------------------------
// One-row float product y = x[1][K] . B[K][N] with B's columns contiguous (Bt[N][K]): NumPy
// hands it to OpenBLAS's GEMV-T (matmul.cpp vector_matrix -> cblas_sgemv(ColMajor, Trans)),
// whose order this kernel reproduces (oracle/openblas_order.py states it and pins it to
// np.matmul): the N columns split over `threads` chunks (gemv_thread.c); per chunk, groups
// of 4 columns by the AVX2 4x4 kernel (8 fma lanes), 2 leftover columns by the SSE 4x2
// kernel (4 mul+add lanes), 1 by the SSE 4x1 kernel (2 x 4 mul+add lanes); K in blocks of
// 4096 added to y in order; K % 4 trailing rows in scalar C with fma contraction.
// Eight lanes per column (one per accumulator lane of the CPU kernel), 8 columns per wave.
__device__ __forceinline__ int gemv_class(int64_t j, int64_t N, int threads) {
  // chunk [j0, j1) of column j: widths ceil(rem / threads left), at least 4
  int64_t j0 = 0, rem = N;
  for (int t = 0; rem > 0; ++t) {
    int64_t w = threads - t > 0 ? (rem + threads - t - 1) / (threads - t) : rem;
    w = w < 4 ? 4 : w;
    w = w > rem ? rem : w;
    if (j < j0 + w) {
      const int64_t n = w, n4 = n & ~(int64_t)3, loc = j - j0;
      if (loc < n4) return 0;              // 4x4
      if (((n - n4) & 2) && loc < n4 + 2) return 1;  // 4x2
      return 2;                            // 4x1
    }
    j0 += w;
    rem -= w;
  }
  return 0;
}

__global__ void __launch_bounds__(256)
k_sgemv_t(const float* __restrict__ x, const float* __restrict__ bt, float* __restrict__ y, int64_t N, int64_t K,
          int64_t ldb, int threads) {
  const int64_t j = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3;
  const int l = threadIdx.x & 7;
  const bool live = j < N;
  const int64_t jj = live ? j : N - 1;
  const float* col = bt + jj * ldb;
  const int cls = gemv_class(jj, N, threads);
  const int64_t m3 = K & 3;
  int64_t m1 = K & ~(int64_t)3;
  const int64_t m2 = (K & 4095) - m3;
  float yv = 0.0f;
  int64_t k0 = 0, nb = 4096;
  while (nb == 4096) {
    m1 -= nb;
    if (m1 < 0) {
      if (m2 == 0) break;
      nb = m2;
    }
    const float* a = col + k0;
    const float* xb = x + k0;
    float acc = 0.0f;
    int64_t i = 0;
    if (cls == 0) {  // lane l: an fma chain over rows l, l + 8, ... (after a 4-row prologue)
      if (nb & 4) {
        if (l < 4) acc = __builtin_fmaf(xb[l], a[l], acc);
        i = 4;
      }
      for (; i < nb; i += 8) acc = __builtin_fmaf(xb[i + l], a[i + l], acc);
    } else if (cls == 1) {  // lanes 0-3: rows r = l mod 4, multiply then add
      if (l < 4)
        for (; i < nb; i += 4) acc = acc + xb[i + l] * a[i + l];
    } else {  // lane l: set l / 4, row l % 4 of each 8-row step (prologue rows to set 0)
      if (nb & 4) {
        if (l < 4) acc = acc + xb[l] * a[l];
        i = 4;
      }
      for (; i < nb; i += 8) acc = acc + xb[i + l] * a[i + l];
    }
    // lanes (r + r+4), then ((0+1) + (2+3)); the 4x2 kernel has no upper lanes
    const float up = __shfl_down(acc, 4, 8);
    const float h = cls == 1 ? acc : acc + up;
    const float h1 = __shfl_down(h, 1, 8);
    const float p = h + h1;  // lanes 0 and 2: (h0 + h1), (h2 + h3)
    const float p2 = __shfl_down(p, 2, 8);
    const float s = p + p2;  // lane 0
    yv = yv + s;
    k0 += nb;
  }
  if (m3) {
    const float* a = col + k0;
    const float* xb = x + k0;
    if (m3 == 1) {
      yv = __builtin_fmaf(a[0], xb[0], yv);
    } else {
      float t = __builtin_fmaf(a[0], xb[0], a[1] * xb[1]);
      if (m3 == 3) t = __builtin_fmaf(a[2], xb[2], t);
      yv = yv + t;
    }
  }
  if (live && l == 0) y[j] = yv;
}

// One-row products outside the GEMV-T kernel above (round 6: every class identified against
// np.matmul, oracle/openblas_order.py sdot / small_modes, pinned by tests/test_host.py):
//  * N == 1 (NumPy's matmul takes cblas_sdot for a 1 x 1 result): the first n & -32 products by
//    the SkylakeX vector kernel — lane l of the wave is element l of its four 16-wide fma
//    accumulators over 64-element steps; folded to four 8-wide ones (low + high half), which
//    continue over 32-element steps; ((a0 + a1) + a2) + a3, low + high 4, two horizontal adds —
//    then the tail's f32 products added in double, the sum rounded once;
//  * K <= 8 (OpenBLAS's small-m GEMV-T kernels, per thread chunk of at most 16 384 columns;
//    wider chunks take the regular kernel's order, restated here for K <= 8): the column's
//    class by its place in its chunk (small_modes), one lane per column.
__device__ __forceinline__ void gemv_chunk(int64_t j, int64_t N, int threads, int64_t& j0, int64_t& w) {
  int64_t rem = N;
  j0 = 0;
  for (int t = 0; rem > 0; ++t) {
    int64_t c = threads - t > 0 ? (rem + threads - t - 1) / (threads - t) : rem;
    c = c < 4 ? 4 : c;
    c = c > rem ? rem : c;
    if (j < j0 + c) {
      w = c;
      return;
    }
    j0 += c;
    rem -= c;
  }
  w = rem;
}

__global__ void __launch_bounds__(256)
k_sgemv_small(const float* __restrict__ x, const float* __restrict__ bt, float* __restrict__ y, int64_t N, int64_t K,
              int64_t ldb, int threads) {
  if (N == 1) {  // cblas_sdot: one wave
    if (threadIdx.x >= 64) return;
    const int l = threadIdx.x;
    const float* w = bt;
    const int64_t n1 = K & ~(int64_t)31, n64 = K & ~(int64_t)63;
    float a = 0.0f;  // lane l: element l % 16 of 16-wide accumulator l / 16
    int64_t i = 0;
    for (; i < n64; i += 64) a = __builtin_fmaf(x[i + l], w[i + l], a);
    // fold to 8 wide: accumulator q = l / 8 (lanes 0..31), element e = l % 8
    const int q = (l >> 3) & 3, e = l & 7;
    float a8 = __shfl(a, 16 * q + e, 64) + __shfl(a, 16 * q + 8 + e, 64);
    if (l < 32)
      for (int64_t k = i; k < n1; k += 32) a8 = __builtin_fmaf(x[k + l], w[k + l], a8);
    // ((a0 + a1) + a2) + a3 per element e (lanes e, e + 8, e + 16, e + 24)
    const float s8 = ((__shfl(a8, e, 64) + __shfl(a8, 8 + e, 64)) + __shfl(a8, 16 + e, 64)) + __shfl(a8, 24 + e, 64);
    const float h = __shfl(s8, e & 3, 64) + __shfl(s8, (e & 3) + 4, 64);  // low + high 4
    const float h01 = __shfl(h, 0, 64) + __shfl(h, 1, 64), h23 = __shfl(h, 2, 64) + __shfl(h, 3, 64);
    if (l == 0) {
      double d = n1 ? (double)(h01 + h23) : 0.0;
      for (int64_t k = n1; k < K; ++k) {
        const float p = x[k] * w[k];  // -ffp-contract=off: the f32 product, then the double add
        d += (double)p;
      }
      y[0] = (float)d;
    }
    return;
  }
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= N) return;
  const float* w = bt + j * ldb;
  float p[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) p[k] = k < K ? x[k] * w[k] : 0.0f;
  auto F = [&](int k, float acc) { return __builtin_fmaf(x[k], w[k], acc); };
  int64_t j0, cw;
  gemv_chunk(j, N, threads, j0, cw);
  float r;
  if (cw > 16384) {  // the regular kernel (k_sgemv_t's order) at K <= 8
    const int m3 = (int)(K & 3);
    float yv = 0.0f;
    if (K == 8) yv = yv + (((p[0] + p[4]) + (p[1] + p[5])) + ((p[2] + p[6]) + (p[3] + p[7])));
    else if (K >= 4) yv = yv + ((p[0] + p[1]) + (p[2] + p[3]));
    const int k0 = K >= 4 ? 4 : 0;
    if (m3 == 1) {
      yv = __builtin_fmaf(w[k0], x[k0], yv);
    } else if (m3 > 1) {
      float t = __builtin_fmaf(w[k0], x[k0], w[k0 + 1] * x[k0 + 1]);
      if (m3 == 3) t = __builtin_fmaf(w[k0 + 2], x[k0 + 2], t);
      yv = yv + t;
    }
    r = yv;
  } else {
    // the small-m kernel's class of local column loc in a chunk of cw (oracle small_modes)
    const int64_t loc = j - j0;
    char c = 'M';
    if (K == 4) {
      c = loc < (cw & ~(int64_t)1) ? 'P' : 'M';
    } else if (K == 8) {
      const int64_t n4 = cw & ~(int64_t)3;
      c = loc < n4 ? 'c' : ((cw & 2) && loc < n4 + 2 ? 'a' : 'e');
    } else if (K == 1) {
      c = 'F';
    } else {
      const int64_t blk = K == 2 ? 16 : (K == 5 ? 4 : 8);
      const int64_t f_end = cw / blk * blk;
      int64_t rr = cw - f_end, lo = loc - f_end;
      if (loc < f_end) {
        c = 'F';
      } else {
        if ((K == 3 || K == 6 || K == 7) && rr >= 4) {
          if (lo < 4) c = 'b';
          rr -= 4;
          lo -= 4;
        }
        if (c != 'b' && K == 3) c = ((rr & 2) && lo < 2) ? 'M' : 'b';
      }
    }
    switch (c) {
      case 'F': {
        float acc = 0.0f;
        for (int k = 0; k < K; ++k) acc = F(k, acc);
        r = acc;
        break;
      }
      case 'P': r = (p[0] + p[1]) + (p[2] + p[3]); break;
      case 'b':
        if (K == 3) r = F(2, F(0, p[1]));
        else if (K == 6) r = (p[0] + F(1, p[2])) + (p[3] + F(4, p[5]));
        else r = (F(0, p[1]) + F(4, p[5])) + (F(2, p[3]) + p[6]);
        break;
      case 'c': r = ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7])); break;
      case 'a': r = ((p[0] + p[1]) + (p[4] + p[5])) + ((p[2] + p[3]) + (p[6] + p[7])); break;
      case 'e': r = (((p[0] + p[4]) + (p[1] + p[5])) + (p[2] + p[6])) + (p[3] + p[7]); break;
      default: {
        float acc = 0.0f;
        for (int k = 0; k < K; ++k) acc = acc + p[k];
        r = acc;
      }
    }
  }
  y[j] = r;
}

// One-row product y[N] = x[1][K] . B[K][N] with B row-major (ldb >= N): NumPy's matmul hands it to
// OpenBLAS's GEMV-N (vector_matrix -> cblas_sgemv on the row-major matrix; round 6: the order
// identified against np.matmul, oracle/openblas_order.py sgemv_n, pinned by tests/test_host.py):
//  * K <= 48: a k-ordered fma chain per output;
//  * N < 4: pairs — t = t + fma(x_k, b_k, RN(x_{k+1} b_{k+1})) over k = 0, 2, .. below K & -4, then
//    an fma chain over the rest;
//  * else the outputs split over `threads` chunks (gemv_thread.c, as GEMV-T's columns); per chunk of
//    w outputs, the last w & 3 are fma chains; the others go in blocks of 4 096 (the last block
//    (w & 4095) - (w & 3)), and in a block of NB the first NB % 16 outputs take the 8- / 4-row
//    kernel (groups of 8 products as two fma chains, even and odd, summed: y += a + b; a 4-group
//    the same; 2- and 1-groups one chain), the rest the 16-row kernel (groups of 8, 4, 2, 1
//    products as one fma chain each: y += chain).
// One lane per output, K products serially (column j of B: adjacent lanes read adjacent floats).
__global__ void __launch_bounds__(256)
k_sgemv_n(const float* __restrict__ x, const float* __restrict__ b, float* __restrict__ y, int64_t N, int64_t K,
          int64_t ldb, int threads) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= N) return;
  const float* c = b + j;
  auto prod = [&](int64_t k, float acc) { return __builtin_fmaf(x[k], c[k * ldb], acc); };
  auto chain = [&](int64_t k0, int64_t k1) {
    float acc = 0.0f;
    for (int64_t k = k0; k < k1; ++k) acc = prod(k, acc);
    return acc;
  };
  if (K <= 48) {
    y[j] = chain(0, K);
    return;
  }
  if (N < 4) {
    float t = 0.0f;
    int64_t k = 0;
    for (; k < (K & ~(int64_t)3); k += 2) t = t + prod(k, x[k + 1] * c[(k + 1) * ldb]);
    for (; k < K; ++k) t = prod(k, t);
    y[j] = t;
    return;
  }
  int64_t j0, w;
  gemv_chunk(j, N, threads, j0, w);
  const int64_t loc = j - j0, m3 = w & 3;
  if (loc >= w - m3) {
    y[j] = chain(0, K);
    return;
  }
  const int64_t nfull = (w & ~(int64_t)3) / 4096, bi = loc / 4096;
  const int64_t nb = bi < nfull ? 4096 : (w & 4095) - m3;
  const bool two = (loc - bi * 4096) < nb % 16;  // the 8- / 4-row kernel
  auto two_acc = [&](int64_t k0, int64_t size) {
    float a = 0.0f, e = 0.0f;
    for (int64_t q = 0; q < size; ++q) {
      if (q & 1) e = prod(k0 + q, e);
      else a = prod(k0 + q, a);
    }
    return a + e;
  };
  float yv = 0.0f;
  const int64_t k8 = K & ~(int64_t)7;
  for (int64_t g = 0; g < k8; g += 8) yv = yv + (two ? two_acc(g, 8) : chain(g, g + 8));
  int64_t k = k8;
  if (K & 4) {
    yv = yv + (two ? two_acc(k, 4) : chain(k, k + 4));
    k += 4;
  }
  if (K & 2) {
    yv = yv + chain(k, k + 2);
    k += 2;
  }
  if (K & 1) yv = yv + chain(k, k + 1);
  y[j] = yv;
}

}  // namespace

// OpenBLAS level-3 K blocking (driver/level3/level3.c): GEMM_Q = 448 for SkylakeX sgemm
// (identified against np.matmul: 384 agrees only while K <= 768)
static int blas_kblocks(int64_t K, KBlocks* kb) {
  const int64_t Q = 448, U = 2;
  int64_t ls = 0;
  kb->n = 0;
  while (ls < K) {
    int64_t min_l = K - ls;
    if (min_l >= 2 * Q) min_l = Q;
    else if (min_l > Q) min_l = ((min_l / 2 + U - 1) / U) * U;
    ls += min_l;
    if (kb->n >= 24) return -1;
    kb->end[kb->n++] = ls;
  }
  return 0;
}

}  // namespace nqk

using namespace nqk;

// K and every BLAS block end multiples of 16 (k_sgemm_mfma AL16; NQK_SGEMM_AL16=0 disables)
static bool kblocks_al16(int64_t K, const KBlocks& kb) {
  const char* v = getenv("NQK_SGEMM_AL16");
  if (v && atoi(v) == 0) return false;
  if (K % 16) return false;
  for (int i = 0; i < kb.n; ++i)
    if (kb.end[i] % 16) return false;
  return true;
}

extern "C" int nqk_qgemm_i8(const int8_t* a, const int8_t* bt, int32_t* c, int64_t batch, int64_t M, int64_t N,
                            int64_t K, int64_t lda, int64_t ldb, int64_t ldc, const int64_t* bmap,
                            int64_t a_mat_stride, int64_t b_mat_stride, int64_t c_mat_stride) {
  if (batch <= 0 || M <= 0 || N <= 0) return 0;
  if ((lda & 15) || (ldb & 15) || (K & 15)) return fail("nqk_qgemm_i8: lda, ldb and K must be multiples of 16");
  if ((((uintptr_t)a) & 15) || (((uintptr_t)bt) & 15) || (a_mat_stride & 15) || (b_mat_stride & 15))
    return fail("nqk_qgemm_i8: operands must be 16-byte aligned");
  if (batch > 65535) return fail("nqk_qgemm_i8: batch > 65535");
  int tiles_m = (int)((M + BM - 1) / BM), tiles_n = (int)((N + BN - 1) / BN);
  if ((int64_t)tiles_m * tiles_n > 0x7fffffff) return fail("nqk_qgemm_i8: too many tiles");
  BatchMap m = batch_map(bmap);
  hipLaunchKernelGGL(k_qgemm_i8, dim3(tiles_m * tiles_n, 1, (unsigned)batch), dim3(256), 0, stream(), a, bt, c, M,
                     N, K, lda, ldb, ldc, m, a_mat_stride, b_mat_stride, c_mat_stride, tiles_n);
  return launch_status("nqk_qgemm_i8");
}

extern "C" int nqk_qgemm_generic(const void* a, int a_dtype, const void* b, int b_dtype, int64_t* c,
                                 int64_t batch, int64_t M, int64_t N, int64_t K, int64_t a_sm, int64_t a_sk,
                                 int64_t b_sk, int64_t b_sn, int64_t ldc, const int64_t* bmap,
                                 int64_t a_mat_stride, int64_t b_mat_stride, int64_t c_mat_stride) {
  if (batch <= 0 || M <= 0 || N <= 0) return 0;
  if (batch > 65535 || (M + 15) / 16 > 65535) return fail("nqk_qgemm_generic: grid too large");
  BatchMap m = batch_map(bmap);
  dim3 grid((unsigned)((N + 15) / 16), (unsigned)((M + 15) / 16), (unsigned)batch);
  NQK_INT_DISPATCH(a_dtype, TA,
    NQK_INT_DISPATCH(b_dtype, TB,
      hipLaunchKernelGGL((k_qgemm_generic<TA, TB>), grid, dim3(256), 0, stream(), (const TA*)a, (const TB*)b, c,
                         M, N, K, a_sm, a_sk, b_sk, b_sn, ldc, m, a_mat_stride, b_mat_stride, c_mat_stride)));
  return launch_status("nqk_qgemm_generic");
}

extern "C" int nqk_sgemm(const float* a, const float* b, float* c, int64_t batch, int64_t M, int64_t N, int64_t K,
                         int64_t a_sm, int64_t a_sk, int64_t b_sk, int64_t b_sn, int64_t ldc, const int64_t* bmap,
                         int64_t a_mat_stride, int64_t b_mat_stride, int64_t c_mat_stride) {
  if (batch <= 0 || M <= 0 || N <= 0) return 0;
  if (batch > 65535 || (M + 63) / 64 > 65535) return fail("nqk_sgemm: grid too large");
  KBlocks kb;
  if (K <= 0) { kb.n = 0; kb.end[0] = -1; }
  else if (blas_kblocks(K, &kb)) return fail("nqk_sgemm: K too large for the BLAS blocking table");
  BatchMap m = batch_map(bmap);
  // MFMA path: same numerics (k-ordered fmaf chains), needs even K-block ends
  if ((K & 1) == 0 && K > 0 && M * N >= 128 * 128 && !getenv("NQK_SGEMM_VALU")) {
    dim3 g2((unsigned)((N + 127) / 128), (unsigned)((M + 127) / 128), (unsigned)batch);
    if ((M + 127) / 128 > 65535) return fail("nqk_sgemm: grid too large");
    const bool vec = a_sk == 1 && b_sn == 1 && (N % 4) == 0 && (a_sm % 4) == 0 && (b_sk % 4) == 0 &&
                     (a_mat_stride % 4) == 0 && (b_mat_stride % 4) == 0 &&
                     ((((uintptr_t)a) | ((uintptr_t)b)) & 15) == 0 && !getenv("NQK_SGEMM_SCALAR");
    if (kblocks_al16(K, kb) && vec)
      hipLaunchKernelGGL((k_sgemm_mfma<false, true, true>), g2, dim3(256), 0, stream(), a, b, c, M, N, K, a_sm, a_sk,
                         b_sk, b_sn, ldc, m, a_mat_stride, b_mat_stride, c_mat_stride, kb, EmbedEpi{nullptr, nullptr, 1});
    else if (kblocks_al16(K, kb))
      hipLaunchKernelGGL((k_sgemm_mfma<false, true>), g2, dim3(256), 0, stream(), a, b, c, M, N, K, a_sm, a_sk, b_sk,
                         b_sn, ldc, m, a_mat_stride, b_mat_stride, c_mat_stride, kb, EmbedEpi{nullptr, nullptr, 1});
    else
      hipLaunchKernelGGL((k_sgemm_mfma<false, false>), g2, dim3(256), 0, stream(), a, b, c, M, N, K, a_sm, a_sk, b_sk,
                         b_sn, ldc, m, a_mat_stride, b_mat_stride, c_mat_stride, kb, EmbedEpi{nullptr, nullptr, 1});
    return launch_status("nqk_sgemm(mfma)");
  }
  dim3 grid((unsigned)((N + 63) / 64), (unsigned)((M + 63) / 64), (unsigned)batch);
  hipLaunchKernelGGL(k_sgemm_blas, grid, dim3(256), 0, stream(), a, b, c, M, N, K, a_sm, a_sk, b_sk, b_sn, ldc, m,
                     a_mat_stride, b_mat_stride, c_mat_stride, kb);
  return launch_status("nqk_sgemm");
}

extern "C" int nqk_sgemm_embed(const float* cols, const float* w, const float* bias, const float* cls,
                               const float* pos, float* out, int64_t images, int64_t hw, int64_t N, int64_t K) {
  const int64_t M = images * hw;
  if (M <= 0 || N <= 0) return 0;
  if ((K & 1) || K <= 0) return fail("nqk_sgemm_embed: K must be even (MFMA k pairs)");
  if ((M + 127) / 128 > 65535) return fail("nqk_sgemm_embed: grid too large");
  KBlocks kb;
  if (blas_kblocks(K, &kb)) return fail("nqk_sgemm_embed: K too large for the BLAS blocking table");
  const BatchMap m = batch_map(nullptr);
  dim3 g2((unsigned)((N + 127) / 128), (unsigned)((M + 127) / 128), 1);
  const bool vec = (N % 4) == 0 && ((((uintptr_t)cols) | ((uintptr_t)w)) & 15) == 0 && !getenv("NQK_SGEMM_SCALAR");
  if (kblocks_al16(K, kb) && vec)
    hipLaunchKernelGGL((k_sgemm_mfma<true, true, true>), g2, dim3(256), 0, stream(), cols, w, out, M, N, K, K, (int64_t)1,
                       N, (int64_t)1, N, m, (int64_t)0, (int64_t)0, (int64_t)0, kb, EmbedEpi{bias, pos, hw, getenv("NQK_EMBED_NOXCD") ? 0 : num_xcds()});
  else if (kblocks_al16(K, kb))
    hipLaunchKernelGGL((k_sgemm_mfma<true, true>), g2, dim3(256), 0, stream(), cols, w, out, M, N, K, K, (int64_t)1, N,
                       (int64_t)1, N, m, (int64_t)0, (int64_t)0, (int64_t)0, kb, EmbedEpi{bias, pos, hw, getenv("NQK_EMBED_NOXCD") ? 0 : num_xcds()});
  else
    hipLaunchKernelGGL((k_sgemm_mfma<true, false>), g2, dim3(256), 0, stream(), cols, w, out, M, N, K, K, (int64_t)1,
                       N, (int64_t)1, N, m, (int64_t)0, (int64_t)0, (int64_t)0, kb, EmbedEpi{bias, pos, hw, getenv("NQK_EMBED_NOXCD") ? 0 : num_xcds()});
  if (int rc = launch_status("nqk_sgemm_embed")) return rc;
  hipLaunchKernelGGL(k_embed_cls, dim3(grid_for(images * N)), dim3(kThreads), 0, stream(), cls, pos, out, images, hw, N);
  return launch_status("nqk_sgemm_embed(cls)");
}

// which k_embed_q form nqk_embed_q runs, and so the order its weights must come in: 16 = the
// v_mfma_f32_16x16x4_f32 form (p = (k & 3) * 4 + (k >> 2) in every 16-k block), 32 = the 32x32x2
// form (p = (k & 1) * 8 + (k >> 1)).  NQK_EMBED_MFMA=16 / 32 selects (A/B; read per call, so a
// caller must not change it between permuting its weights and launching).
static bool embed_mfma16() {
  const char* e = getenv("NQK_EMBED_MFMA");
  return e && atoi(e) == 16;
}
extern "C" int nqk_embed_weight_order(void) { return embed_mfma16() ? 16 : 32; }

extern "C" int nqk_embed_q(const int8_t* q, float scale, int64_t zp, const float* wt, const float* bias,
                           const float* cls, const float* pos, float* out, int64_t images, int64_t c, int64_t h,
                           int64_t w, int64_t kh, int64_t kw, int64_t N) {
  if (images <= 0 || N <= 0) return 0;
  if (c != 3 || kh != 16 || kw != 16 || h % 16 || w % 16)
    return fail("nqk_embed_q: 3-channel images and 16 x 16 patches expected");
  if (N % 64) return fail("nqk_embed_q: N % 64 == 0 expected");
  if (zp < -(1 << 20) || zp > (1 << 20)) return fail("nqk_embed_q: zero point out of range");
  if ((((uintptr_t)q) | ((uintptr_t)wt)) & 15) return fail("nqk_embed_q: unaligned operands");
  const int64_t wo = w / 16, hw = (h / 16) * wo, M = images * hw, K = 768;
  if ((M + 127) / 128 > 65535) return fail("nqk_embed_q: grid too large");
  if ((double)(M + images) * (double)N >= 2147483647.0) return fail("nqk_embed_q: output too large");
  KBlocks kb;
  if (blas_kblocks(K, &kb) || !kblocks_al16(K, kb)) return fail("nqk_embed_q: K blocking");
  const float zpf = (float)zp;
  // (a 3-stage LDS ring with the next k-tile's fragments read under the MFMAs measured 1.5 %
  // slower: 634 vs 625 us, profiles/r04_embed_ring_dropped.txt)
  // (also dropped: one workgroup per CU, 256 x 128 tiles, one wave per SIMD — 768 vs 605 us,
  // profiles/r04_embed_1wg_streams_dropped.txt)
  // (NQK_EMBED_WN1=1: the 128 x 64 tiles at N % 128 == 0 as well — 150 VGPRs, 3 workgroups per CU
  // instead of 2, twice the tiles; round-6 A/B)
  if (embed_mfma16()) {  // the weights in the 16x16 kernel's order (nqk_embed_weight_order() == 16)
    if (N % 128 == 0 && !getenv("NQK_EMBED_WN1"))
      hipLaunchKernelGGL(k_embed_q16<2>, dim3((unsigned)(N / 128), (unsigned)((M + 127) / 128)), dim3(256), 0, stream(), q,
                         wt, out, M, N, hw, wo, h, w, scale, zpf, kb, EmbedEpi{bias, pos, hw, getenv("NQK_EMBED_NOXCD") ? 0 : num_xcds()});
    else
      hipLaunchKernelGGL(k_embed_q16<1>, dim3((unsigned)(N / 64), (unsigned)((M + 127) / 128)), dim3(256), 0, stream(), q,
                         wt, out, M, N, hw, wo, h, w, scale, zpf, kb, EmbedEpi{bias, pos, hw, getenv("NQK_EMBED_NOXCD") ? 0 : num_xcds()});
  } else if (N % 128 == 0 && !getenv("NQK_EMBED_WN1")) {
    hipLaunchKernelGGL(k_embed_q<2>, dim3((unsigned)(N / 128), (unsigned)((M + 127) / 128)), dim3(256), 0, stream(), q,
                       wt, out, M, N, hw, wo, h, w, scale, zpf, kb, EmbedEpi{bias, pos, hw, getenv("NQK_EMBED_NOXCD") ? 0 : num_xcds()});
  } else {
    hipLaunchKernelGGL(k_embed_q<1>, dim3((unsigned)(N / 64), (unsigned)((M + 127) / 128)), dim3(256), 0, stream(), q,
                       wt, out, M, N, hw, wo, h, w, scale, zpf, kb, EmbedEpi{bias, pos, hw, getenv("NQK_EMBED_NOXCD") ? 0 : num_xcds()});
  }
  if (int rc = launch_status("nqk_embed_q")) return rc;
  hipLaunchKernelGGL(k_embed_cls, dim3(grid_for(images * N)), dim3(kThreads), 0, stream(), cls, pos, out, images, hw, N);
  return launch_status("nqk_embed_q(cls)");
}

extern "C" int nqk_patchify_dequant(const int8_t* q, float* cols, int64_t n, int64_t c, int64_t h, int64_t w,
                                    int64_t kh, int64_t kw, float scale, int64_t zp) {
  if (kh <= 0 || kw <= 0 || h % kh || w % kw) return fail("nqk_patchify_dequant: the kernel must tile the image");
  if (zp < -(1 << 20) || zp > (1 << 20)) return fail("nqk_patchify_dequant: zero point out of range");
  const int64_t total = n * (h / kh) * (w / kw) * kh;
  if (total <= 0) return 0;
  const bool vec = kw == 16 && c == 3 && (w % 16) == 0 && (((uintptr_t)q) & 15) == 0 && (((uintptr_t)cols) & 15) == 0;
  if (vec)
    hipLaunchKernelGGL(k_patchify_dequant<true>, dim3(grid_for(total)), dim3(kThreads), 0, stream(), q, cols, n, c, h,
                       w, kh, kw, scale, (float)zp);
  else
    hipLaunchKernelGGL(k_patchify_dequant<false>, dim3(grid_for(total)), dim3(kThreads), 0, stream(), q, cols, n, c,
                       h, w, kh, kw, scale, (float)zp);
  return launch_status("nqk_patchify_dequant");
}

extern "C" int nqk_im2col(const float* x, float* cols, int64_t n, int64_t c, int64_t h, int64_t w, int64_t kh,
                          int64_t kw, int64_t ph0, int64_t pw0, int64_t sh, int64_t sw, int64_t ho, int64_t wo) {
  int64_t total = n * ho * wo * kh * kw * c;
  if (total <= 0) return 0;
  hipLaunchKernelGGL(k_im2col, dim3(grid_for(total)), dim3(kThreads), 0, stream(), x, cols, n, c, h, w, kh, kw, ph0,
                     pw0, sh, sw, ho, wo);
  return launch_status("nqk_im2col");
}

extern "C" int nqk_sgemv_t(const float* x, const float* bt, float* y, int64_t N, int64_t K, int64_t ldb,
                           int64_t threads) {
  if (N <= 0) return 0;
  if (K <= 0) return fail("nqk_sgemv_t: K >= 1 expected");
  if (ldb < K) return fail("nqk_sgemv_t: ldb < K");
  if (threads < 1 || threads > 1024) return fail("nqk_sgemv_t: 1 <= threads <= 1024 expected");
  // interface/gemv.c: one thread below m * n = 115200 * GEMM_MULTITHREAD_THRESHOLD (4)
  const int t = (K * N < 115200 * 4) ? 1 : (int)threads;
  if (K <= 8 && ldb == K && N > 1) {  // the small-m kernels (chunks <= 16 384 columns) and K <= 8 of the regular one
    hipLaunchKernelGGL(k_sgemv_small, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, stream(), x, bt, y, N, K, ldb, t);
    return launch_status("nqk_sgemv_t(small)");
  }
  const int64_t lanes = N * 8;
  hipLaunchKernelGGL(k_sgemv_t, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, stream(), x, bt, y, N, K, ldb, t);
  return launch_status("nqk_sgemv_t");
}

extern "C" int nqk_sgemv_n(const float* x, const float* b, float* y, int64_t N, int64_t K, int64_t ldb,
                           int64_t threads) {
  if (N <= 0) return 0;
  if (K <= 0) return fail("nqk_sgemv_n: K >= 1 expected");
  if (ldb < N) return fail("nqk_sgemv_n: ldb < N");
  if (threads < 1 || threads > 1024) return fail("nqk_sgemv_n: 1 <= threads <= 1024 expected");
  const int t = (K * N < 115200 * 4) ? 1 : (int)threads;  // interface/gemv.c, as nqk_sgemv_t
  hipLaunchKernelGGL(k_sgemv_n, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, stream(), x, b, y, N, K, ldb, t);
  return launch_status("nqk_sgemv_n");
}

extern "C" int nqk_sgemv_small(const float* x, const float* bt, float* y, int64_t N, int64_t K, int64_t ldb) {
  if (N <= 0) return 0;
  if (K <= 0) return fail("nqk_sgemv_small: K >= 1 expected");
  if (ldb < K) return fail("nqk_sgemv_small: ldb < K");
  if (N != 1) return fail("nqk_sgemv_small: N == 1 (cblas_sdot) expected; one-row products with N > 1 are nqk_sgemv_t's");
  hipLaunchKernelGGL(k_sgemv_small, dim3(1), dim3(64), 0, stream(), x, bt, y, N, K, ldb, 1);
  return launch_status("nqk_sgemv_small");
}
