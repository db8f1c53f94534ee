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
// LDS (T = 197: NT = 7 score tiles of 32 columns, 136 KiB, one workgroup per CU):
//   Ks   [NT*32][64]     int8, 16-byte chunks XOR-swizzled (conflict-free B reads)
//   Vt   [64][PST]       int8 V^T, zero padded to NT*32 tokens; PST = NT*32 + 16
//   csK  [NT*32], csV [64]   int32 row sums of K / column sums of V
//   per wave: E [32][EST] f32 exp values of its 32-row tile (P aliases it, PST stride)
//             rsQ [32], rsP [32] row sums of Q / P
#include "nqk_common.h"
#include "nqk_numerics.h"

namespace nqk {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

struct AttnArgs {
  int T, H, ld_out, EST, PST, n2;
  int zq, zk, zp, zv;  // zero points (host-checked: every int32 intermediate is exact)
  int kq, kp;          // zq*zk*64, zp*zv*T
  float s_qk, div, s_p, s_pv, s_ctx;
  double rdiv, rs_p, zp_p, rs_ctx, zp_ctx, lo, hi;
};

__device__ __forceinline__ int swz64a(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4); }

__device__ __forceinline__ int sum16a(v4i c) {
  int s = __builtin_amdgcn_sdot4(c[0], 0x01010101, 0, false);
  s = __builtin_amdgcn_sdot4(c[1], 0x01010101, s, false);
  s = __builtin_amdgcn_sdot4(c[2], 0x01010101, s, false);
  return __builtin_amdgcn_sdot4(c[3], 0x01010101, s, false);
}

// RN32(x / c) from rc = RN64(1/c) (see nqk_fused.hip div_rc); the exact division only in
// a wave-uniform branch for quotients near the subnormal range
__device__ __forceinline__ float div_rc_w(float x, float c, double rc) {
  float t = (float)((double)x * rc);
  const bool slow = __builtin_fabsf(t) < 0x1p-125f && x != 0.0f;
  if (__builtin_expect(__any(slow), 0)) t = slow ? x / c : t;
  return t;
}

__device__ __forceinline__ int quant_w(float x, float s, double rs, double zp, double lo, double hi) {
  const float t = div_rc_w(x, s, rs);
  const double u = zp + (double)t;
  return (int)__builtin_rint(__builtin_fmin(__builtin_fmax(u, lo), hi));
}

// NumPy pairwise_sum leaf (n <= 128): 8 interleaved accumulators, then the n % 8 tail
__device__ __forceinline__ float leaf_sum(const float* v, int L) {
  if (L < 8) {
    float res = 0.0f;
    for (int i = 0; i < L; ++i) res = res + v[i];
    return res;
  }
  const float4* v4 = reinterpret_cast<const float4*>(v);
  float4 a = v4[0], b = v4[1];
  float r0 = a.x, r1 = a.y, r2 = a.z, r3 = a.w, r4 = b.x, r5 = b.y, r6 = b.z, r7 = b.w;
  const int end = L - (L % 8);
  for (int i = 8; i < end; i += 8) {
    a = v4[i / 4];
    b = v4[i / 4 + 1];
    r0 = r0 + a.x; r1 = r1 + a.y; r2 = r2 + a.z; r3 = r3 + a.w;
    r4 = r4 + b.x; r5 = r5 + b.y; r6 = r6 + b.z; r7 = r7 + b.w;
  }
  float res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (int i = end; i < L; ++i) res = res + v[i];
  return res;
}

template <int NT>
__global__ void __launch_bounds__(256, 1)
k_attention(const int8_t* __restrict__ Qg, const int8_t* __restrict__ Kg, const int8_t* __restrict__ Vg,
            int8_t* __restrict__ ctx, AttnArgs a) {
  constexpr int TP = NT * 32;  // padded tokens (score columns / PV contraction)
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  const int T = a.T, PST = a.PST, EST = a.EST;
  int8_t* Ks = lds;
  int8_t* Vt = Ks + TP * 64;
  int* csK = reinterpret_cast<int*>(Vt + 64 * PST);
  int* csV = csK + TP;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int8_t* wreg = reinterpret_cast<int8_t*>(csV + 64) + wave * (32 * EST * 4 + 256);
  float* E = reinterpret_cast<float*>(wreg);
  int8_t* P = wreg;  // aliases E row by row (P row r ends before E row r + 1 starts)
  int* rsQ = reinterpret_cast<int*>(wreg + 32 * EST * 4);
  int* rsP = rsQ + 32;

  const int bh = blockIdx.x;
  const int img = bh / a.H, head = bh - img * a.H;
  const int8_t* q = Qg + (int64_t)bh * T * 64;
  const int8_t* k = Kg + (int64_t)bh * T * 64;
  const int8_t* v = Vg + (int64_t)bh * T * 64;

  // ---- K (swizzled) and V^T (zero padded) into LDS
  for (int idx = tid; idx < TP * 4; idx += 256) {
    const int row = idx >> 2, ch = idx & 3;
    const v4i z = {0, 0, 0, 0};
    const v4i kv = row < T ? *reinterpret_cast<const v4i*>(k + row * 64 + ch * 16) : z;
    const v4i vv = row < T ? *reinterpret_cast<const v4i*>(v + row * 64 + ch * 16) : z;
    *reinterpret_cast<v4i*>(Ks + swz64a(row, ch)) = kv;
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int b = 0; b < 4; ++b) Vt[(ch * 16 + w * 4 + b) * PST + row] = (int8_t)(vv[w] >> (8 * b));
  }
  __syncthreads();
  for (int row = tid; row < TP; row += 256) {
    const v4i* kr = reinterpret_cast<const v4i*>(Ks + row * 64);
    csK[row] = sum16a(kr[0]) + sum16a(kr[1]) + sum16a(kr[2]) + sum16a(kr[3]);
  }
  {
    const int d = tid >> 2, part = tid & 3;
    int s = 0;
    for (int c = part; c < NT * 2; c += 4) s += sum16a(*reinterpret_cast<const v4i*>(Vt + d * PST + c * 16));
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (part == 0) csV[d] = s;
  }
  __syncthreads();

  const int r32 = lane & 31, half = lane >> 5;
  for (int rt = wave; rt < NT; rt += 4) {
    const int m0 = rt * 32;
    // ---- S = Q K^T (raw int32) for rows m0..m0+31, all TP columns
    v4i qa[2];
    {
      const int qrow = min(m0 + r32, T - 1);
      qa[0] = *reinterpret_cast<const v4i*>(q + qrow * 64 + half * 16);
      qa[1] = *reinterpret_cast<const v4i*>(q + qrow * 64 + (2 + half) * 16);
    }
    int rq = sum16a(qa[0]) + sum16a(qa[1]);
    rq += __shfl_xor(rq, 32, 64);
    if (half == 0) rsQ[r32] = rq;
    v16i acc[NT];
#pragma unroll
    for (int c = 0; c < NT; ++c) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[c][r] = 0;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const v4i kb = *reinterpret_cast<const v4i*>(Ks + swz64a(c * 32 + r32, 2 * s + half));
        acc[c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(qa[s], kb, acc[c], 0, 0, 0);
      }
    }
    wave_lds_sync();
    // ---- dequant + Div (EPI_SCORES), row max, NumPy exp -> E
    float y[NT][16];
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      const int col = c * 32 + r32;
      const int colterm = csK[col] * a.zq - a.kq;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * half;
        const int vv = acc[c][r] - rsQ[row] * a.zk - colterm;
        const float d = (float)((double)vv * (double)a.s_qk);
        const float yy = div_rc_w(d, a.div, a.rdiv);
        y[c][r] = col < T ? yy : -__builtin_inff();
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float mx = y[0][r];
#pragma unroll
      for (int c = 1; c < NT; ++c) mx = y[c][r] > mx ? y[c][r] : mx;
#pragma unroll
      for (int off = 1; off < 32; off <<= 1) {
        const float o = __shfl_xor(mx, off, 64);
        mx = o > mx ? o : mx;
      }
      const float nm = -mx;
      const int row = (r & 3) + 8 * (r >> 2) + 4 * half;
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        const int col = c * 32 + r32;
        if (col < T) E[row * EST + col] = np_expf(y[c][r] + nm);
      }
    }
    wave_lds_sync();
    // ---- NumPy pairwise row sums: lane = (row, leaf)
    float tot;
    {
      const int s0 = half ? a.n2 : 0;
      const int L = a.n2 ? (half ? T - a.n2 : a.n2) : (half ? 0 : T);
      const float res = leaf_sum(E + r32 * EST + s0, L);
      const float other = __shfl_xor(res, 32, 64);
      tot = a.n2 ? (half ? other + res : res + other) : (half ? other : res);
    }
    // ---- P = quantize(E / sum), one row per step (lane: 4 columns), int8 into P
    const int c0 = lane * 4;
    for (int r = 0; r < 32; ++r) {
      if (m0 + r >= T) break;
      const float ssum = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tot), r));
      const double rsum = 1.0 / (double)ssum;
      if (c0 < TP) {
        float4 e4 = make_float4(0.f, 0.f, 0.f, 0.f);
        if (c0 < T) e4 = *reinterpret_cast<const float4*>(E + r * EST + c0);
        const float ev[4] = {e4.x, e4.y, e4.z, e4.w};
        uint32_t packed = 0;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          int qv = 0;
          if (c0 + kk < T) qv = quant_w(div_rc_w(ev[kk], ssum, rsum), a.s_p, a.rs_p, a.zp_p, a.lo, a.hi);
          packed |= ((uint32_t)(qv & 0xff)) << (8 * kk);
        }
        *reinterpret_cast<uint32_t*>(P + r * PST + c0) = packed;
      }
    }
    wave_lds_sync();
    // ---- ctx = P V (raw int32), P row sums
    v16i acc2[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc2[j][r] = 0;
    int rp = 0;
#pragma unroll
    for (int s = 0; s < NT; ++s) {
      const v4i pa = *reinterpret_cast<const v4i*>(P + r32 * PST + (2 * s + half) * 16);
      rp += sum16a(pa);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const v4i vb = *reinterpret_cast<const v4i*>(Vt + (j * 32 + r32) * PST + (2 * s + half) * 16);
        acc2[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(pa, vb, acc2[j], 0, 0, 0);
      }
    }
    rp += __shfl_xor(rp, 32, 64);
    wave_lds_sync();
    if (half == 0) rsP[r32] = rp;
    wave_lds_sync();
    // ---- dequant + quantize (EPI_PV) -> ctx[img][token][head * 64 + d]
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int d = j * 32 + r32;
      const int colterm = csV[d] * a.zp - a.kp;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * half;
        const int vv = acc2[j][r] - rsP[row] * a.zv - colterm;
        const float o = (float)((double)vv * (double)a.s_pv);
        const int qv = quant_w(o, a.s_ctx, a.rs_ctx, a.zp_ctx, a.lo, a.hi);
        if (m0 + row < T) ctx[((int64_t)img * T + m0 + row) * a.ld_out + head * 64 + d] = (int8_t)qv;
      }
    }
    wave_lds_sync();
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
  const size_t shm = (size_t)NT * 32 * 64 + (size_t)64 * a.PST + (size_t)(NT * 32 + 64) * 4 +
                     4 * ((size_t)32 * a.EST * 4 + 256);
  const dim3 grid((unsigned)batch_heads);
  switch (NT) {
#define A(n) case n: hipLaunchKernelGGL(k_attention<n>, grid, dim3(256), shm, stream(), q, k, v, ctx, a); break;
    A(1) A(2) A(3) A(4) A(5) A(6) A(7)
#undef A
    default: return fail("nqk_attention_fused: bad tile count");
  }
  return launch_status("nqk_attention_fused");
}
