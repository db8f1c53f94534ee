// Microbenchmark, second form: can a SIMD execute one wave's MFMAs while it issues another
// wave's VALU?  Waves 0-3 run MFMAs, waves 4-7 (the same SIMDs) run VALU, in one 512-thread
// workgroup per CU.  The VALU side uses 16 independent fma chains (issue-bound, not
// latency-bound).  MFMA kinds: i8 32x32x32 (accumulators in VGPRs or forced into AGPRs by
// inline asm), bf16 32x32x16.  Prints ns per iteration; "sum" vs "max" of the solo runs
// answers the question.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));

enum { M_NONE = 0, M_I8 = 1, M_I8_AGPR = 2, M_BF16 = 3 };

template <int MK, bool VALU>
__global__ void __launch_bounds__(512, 1) k(int iters, int* out) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  int res = 0;
  if (wave < 4) {
    if constexpr (MK == M_I8) {
      v16i acc[4];
      for (int i = 0; i < 4; ++i) for (int r = 0; r < 16; ++r) acc[i][r] = lane + r;
      v4i a = {lane, 1, 2, 3}, b = {3, lane, 1, 2};
      for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[i], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[i], 0, 0, 0);
      }
      for (int i = 0; i < 4; ++i) res += acc[i][lane & 15];
    } else if constexpr (MK == M_I8_AGPR) {
      v4i a = {lane, 1, 2, 3}, b = {3, lane, 1, 2};
      v16i c0, c1, c2, c3;
      for (int r = 0; r < 16; ++r) { c0[r] = lane + r; c1[r] = r; c2[r] = lane; c3[r] = 1; }
      for (int it = 0; it < iters; ++it) {
        asm volatile(
            "v_mfma_i32_32x32x32_i8 %0, %4, %5, %0\n\t"
            "v_mfma_i32_32x32x32_i8 %1, %4, %5, %1\n\t"
            "v_mfma_i32_32x32x32_i8 %2, %4, %5, %2\n\t"
            "v_mfma_i32_32x32x32_i8 %3, %4, %5, %3\n\t"
            "v_mfma_i32_32x32x32_i8 %0, %4, %5, %0\n\t"
            "v_mfma_i32_32x32x32_i8 %1, %4, %5, %1\n\t"
            "v_mfma_i32_32x32x32_i8 %2, %4, %5, %2\n\t"
            "v_mfma_i32_32x32x32_i8 %3, %4, %5, %3\n\t"
            : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3)
            : "v"(a), "v"(b));
      }
      res += c0[lane & 15] + c1[lane & 15] + c2[lane & 15] + c3[lane & 15];
    } else if constexpr (MK == M_BF16) {
      v16f acc[4];
      for (int i = 0; i < 4; ++i) for (int r = 0; r < 16; ++r) acc[i][r] = lane + r;
      v8bf a, b;
      for (int r = 0; r < 8; ++r) { a[r] = (__bf16)(float)(lane + r); b[r] = (__bf16)(float)r; }
      for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[i], 0, 0, 0);
      }
      for (int i = 0; i < 4; ++i) res += (int)acc[i][lane & 15];
    }
  } else if constexpr (VALU) {
    float x[16];
    for (int i = 0; i < 16; ++i) x[i] = lane * 0.001f + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = __builtin_fmaf(x[i], 0.999f, 0.5f);
    }
    for (int i = 0; i < 16; ++i) res += (int)x[i];
  }
  if (res == 0x12345678) out[0] = res;
}

template <int MK, bool VALU>
static float run(int iters, int* d) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((k<MK, VALU>), dim3(256), dim3(512), 0, 0, iters, d);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k<MK, VALU>), dim3(256), dim3(512), 0, 0, iters, d);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5 * 1e6f / iters;
}

int main() {
  int* d;
  hipMalloc(&d, 16);
  const int iters = 4000;
  for (int rep = 0; rep < 2; ++rep) {
    const float v = run<M_NONE, true>(iters, d);
    const float i8 = run<M_I8, false>(iters, d), i8v = run<M_I8, true>(iters, d);
    const float ag = run<M_I8_AGPR, false>(iters, d), agv = run<M_I8_AGPR, true>(iters, d);
    const float bf = run<M_BF16, false>(iters, d), bfv = run<M_BF16, true>(iters, d);
    if (!rep) continue;
    printf("valu only (64 fma, 16 chains): %7.1f ns/it\n", v);
    printf("i8 vgpr acc : mfma %7.1f  both %7.1f  (sum %7.1f, max %7.1f)\n", i8, i8v, i8 + v, i8 > v ? i8 : v);
    printf("i8 agpr acc : mfma %7.1f  both %7.1f  (sum %7.1f, max %7.1f)\n", ag, agv, ag + v, ag > v ? ag : v);
    printf("bf16        : mfma %7.1f  both %7.1f  (sum %7.1f, max %7.1f)\n", bf, bfv, bf + v, bf > v ? bf : v);
  }
  return 0;
}
