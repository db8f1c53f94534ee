// Microbenchmark (round 3): does a SIMD overlap one wave's int8 MFMAs with ANOTHER wave's
// VALU?  (Round 2's overlap2.hip said "sum", but it was built with the SLP vectorizer,
// which packs the VALU chains into v_pk_fma_f32 — an anti-lever beside MFMAs.)  Build with
// -fno-slp-vectorize.  512-thread workgroups, one per CU: waves 0-3 run MFMAs (one per
// SIMD), waves 4-7 (the same SIMDs) run scalar VALU chains.  Random operands, sustained
// launches, in-kernel clock.  Reports ns per iteration for MFMA alone, VALU alone, both.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// SHAPE 0: 8 x 32x32x32 per iteration; 1: 16 x 16x16x64.  NV VALU ops per iteration
// (per VALU wave), KIND 0 fma, 1 mix with exp2 / rint / cvt.  MODE bit0 MFMA waves on,
// bit1 VALU waves on.  PRIO: VALU waves at s_setprio PRIO.
template <int SHAPE, int NV, int KIND, int MODE, int PRIO>
__global__ void __launch_bounds__(512, 1) k(const int* __restrict__ rnd, int iters, int* out, long long* clk) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int res = 0;
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  if (wave < 4) {
    if constexpr ((MODE & 1) != 0) {
      v4i a[4], b[4];
      for (int s = 0; s < 4; ++s) {
        a[s] = *reinterpret_cast<const v4i*>(rnd + ((s * 64 + lane) * 4 + blockIdx.x * 7) % 65536);
        b[s] = *reinterpret_cast<const v4i*>(rnd + ((s * 64 + lane) * 4 + 4096 + threadIdx.x) % 65536);
      }
      if constexpr (SHAPE == 0) {
        v16i acc[4];
        for (int i = 0; i < 4; ++i)
          for (int r = 0; r < 16; ++r) acc[i][r] = lane + r;
        for (int it0 = 0; it0 < iters; it0 += 4) {
#pragma unroll
          for (int q = 0; q < 32; ++q)
            acc[q & 3] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[q & 3], b[((q & 7) + (q >> 3)) & 3], acc[q & 3], 0, 0, 0);
        }
        for (int i = 0; i < 4; ++i) res += acc[i][lane & 15];
      } else {
        v4i acc[8];
        for (int i = 0; i < 8; ++i)
          for (int r = 0; r < 4; ++r) acc[i][r] = lane + r;
        for (int it0 = 0; it0 < iters; it0 += 4) {
#pragma unroll
          for (int q = 0; q < 64; ++q)
            acc[q & 7] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[q & 3], b[((q & 15) / 4 + (q >> 4)) & 3], acc[q & 7], 0, 0, 0);
        }
        for (int i = 0; i < 8; ++i) res += acc[i][lane & 3];
      }
    }
  } else if constexpr ((MODE & 2) != 0) {
    if (PRIO) __builtin_amdgcn_s_setprio(PRIO);
    float x[16];
    for (int i = 0; i < 16; ++i) x[i] = __int_as_float(rnd[(lane + i * 64) % 65536] & 0x3fffffff) * 0.001f + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int c = v % 16;
        if constexpr (KIND == 0) x[c] = __builtin_fmaf(x[c], 0.999f, 0.5f);
        else {
          if (v % 8 == 7) x[c] = __builtin_amdgcn_exp2f(x[c]);
          else if (v % 8 == 5) x[c] = __builtin_rintf(x[c]);
          else if (v % 8 == 3) x[c] = (float)(int)x[c];
          else x[c] = __builtin_fmaf(x[c], 0.999f, 0.5f);
        }
      }
    }
    for (int i = 0; i < 16; ++i) res += (int)x[i];
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (res == 0x12345678) out[0] = res;
  if (threadIdx.x == 0) {
    clk[blockIdx.x * 2] = t1 - t0;
    clk[blockIdx.x * 2 + 1] = r1 - r0;
  }
}

template <int SHAPE, int NV, int KIND, int MODE, int PRIO>
static double run(const int* rnd, int* d, long long* clk, int iters, double* ghz) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int r = 0; r < 30; ++r) hipLaunchKernelGGL((k<SHAPE, NV, KIND, MODE, PRIO>), dim3(256), dim3(512), 0, 0, rnd, iters, d, clk);
  hipEventRecord(e0);
  const int reps = 15;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k<SHAPE, NV, KIND, MODE, PRIO>), dim3(256), dim3(512), 0, 0, rnd, iters, d, clk);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> h(512);
  (void)hipMemcpy(h.data(), clk, 512 * sizeof(long long), hipMemcpyDeviceToHost);
  std::vector<double> f;
  for (int g = 0; g < 256; ++g) f.push_back((double)h[2 * g] / (double)h[2 * g + 1] * 0.1);
  std::sort(f.begin(), f.end());
  *ghz = f[128];
  return ms * 1e6 / reps / iters;  // ns per iteration
}

template <int SHAPE, int NV, int KIND, int PRIO>
static void trio(const int* rnd, int* d, long long* clk, const char* tag) {
  const int iters = 16000;
  double g1, g2, g3;
  const double m = run<SHAPE, NV, KIND, 1, PRIO>(rnd, d, clk, iters, &g1);
  const double v = run<SHAPE, NV, KIND, 2, PRIO>(rnd, d, clk, iters, &g2);
  const double b = run<SHAPE, NV, KIND, 3, PRIO>(rnd, d, clk, iters, &g3);
  printf("%-22s NV %3d prio %d: mfma %6.1f ns (%.2f GHz)  valu %6.1f ns (%.2f GHz)  both %6.1f ns (%.2f GHz)  sum %6.1f max %6.1f\n",
         tag, NV, PRIO, m, g1, v, g2, b, g3, m + v, m > v ? m : v);
  fflush(stdout);
}

int main() {
  std::vector<int> h(65536);
  srand(1);
  for (auto& v : h) v = (rand() << 16) ^ rand();
  int *rnd, *d;
  long long* clk;
  (void)hipMalloc(&rnd, 65536 * 4);
  (void)hipMalloc(&d, 64);
  (void)hipMalloc(&clk, 256 * 2 * 8);
  (void)hipMemcpy(rnd, h.data(), 65536 * 4, hipMemcpyHostToDevice);
  trio<0, 32, 0, 0>(rnd, d, clk, "32x32x32 / fma");
  trio<0, 64, 0, 0>(rnd, d, clk, "32x32x32 / fma");
  trio<0, 64, 1, 0>(rnd, d, clk, "32x32x32 / mix");
  trio<1, 32, 0, 0>(rnd, d, clk, "16x16x64 / fma");
  trio<1, 64, 0, 0>(rnd, d, clk, "16x16x64 / fma");
  trio<1, 64, 1, 0>(rnd, d, clk, "16x16x64 / mix");
  trio<1, 64, 0, 1>(rnd, d, clk, "16x16x64 / fma");
  trio<0, 64, 0, 1>(rnd, d, clk, "32x32x32 / fma");
  return 0;
}
