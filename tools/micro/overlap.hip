// Microbenchmark: do MFMA work on waves 0-3 and VALU work on waves 4-7 of one 512-thread
// workgroup (one of each per SIMD) overlap?  mode 0: both, 1: MFMA only, 2: VALU only,
// 3: VALU with packed f32, 4: both with packed VALU, 5: VALU only dependent-chain-light (8 chains)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float f2 __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(512, 1) k(int mode, int iters, int* out) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  int res = 0;
  if (wave < 4) {
    if (mode == 0 || mode == 1 || mode == 4) {
      v16i acc[8];
      for (int i = 0; i < 8; ++i) for (int r = 0; r < 16; ++r) acc[i][r] = lane + r;
      v4i a = {lane, 1, 2, 3}, b = {3, lane, 1, 2};
      for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[i], 0, 0, 0);
      }
      for (int i = 0; i < 8; ++i) res += acc[i][lane & 15];
    }
  } else {
    if (mode == 0 || mode == 2) {
      float x[8];
      for (int i = 0; i < 8; ++i) x[i] = lane * 0.001f + i;
      for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int i = 0; i < 8; ++i) x[i] = __builtin_fmaf(x[i], 0.999f, 0.5f);
      }
      for (int i = 0; i < 8; ++i) res += (int)x[i];
    } else if (mode == 3 || mode == 4) {
      f2 x[8];
      for (int i = 0; i < 8; ++i) x[i] = f2{lane * 0.001f + i, i * 0.5f};
      for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 8; ++i) x[i] = __builtin_elementwise_fma(x[i], (f2)(0.999f), (f2)(0.5f));
      }
      for (int i = 0; i < 8; ++i) res += (int)(x[i].x + x[i].y);
    } else if (mode == 5) {
      float x[8];
      for (int i = 0; i < 8; ++i) x[i] = lane * 0.001f + i;
      for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int i = 0; i < 8; ++i) x[i] = __builtin_amdgcn_exp2f(x[i]) * 0.5f;
      }
      for (int i = 0; i < 8; ++i) res += (int)x[i];
    }
  }
  if (res == 0x12345678) out[0] = res;
}

int main(int argc, char** argv) {
  int* d;
  hipMalloc(&d, 16);
  const int iters = 2000;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[] = {"mfma+valu", "mfma only", "valu only (64 fma/it)", "valu pk only (32 pk_fma/it)", "mfma+valu pk", "exp2+mul chains only"};
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 0; mode < 6; ++mode) {
      hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, mode, iters, d);
      hipEventRecord(a);
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, 0, mode, iters, d);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep) printf("%-28s %8.3f ms  (per iteration per wave: %.1f ns)\n", names[mode], ms / 5, ms / 5 * 1e6 / iters);
    }
  return 0;
}
