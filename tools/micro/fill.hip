// Microbenchmark (round 3): how much VALU work hides between int8 MFMAs of the SAME wave,
// and what the chip's clock does with each MFMA shape.
//   shape 0: v_mfma_i32_32x32x32_i8 (32 cycles), 8 per iteration on 4 accumulators
//   shape 1: v_mfma_i32_16x16x64_i8 (16 cycles), 16 per iteration on 8 accumulators
// (the same int8 MACs per iteration).  NV independent VALU operations (fma chains; kind 1:
// an epilogue-like mix with a transcendental) are placed after every 32x32x32-equivalent of
// MFMA work, inside the same wave's instruction stream (sched_group_barrier).  WPS waves
// per SIMD (1: 256-thread workgroups, 2: 512).  Operands are random bytes and rotate over
// 4 register sets.  Prints ns per 32x32x32-equivalent per SIMD, effective TOPS and the
// in-kernel clock (s_memtime / s_memrealtime, 100 MHz).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int SHAPE, int NV, int KIND>
__global__ void __launch_bounds__(512, 1) k(const int* __restrict__ rnd, int iters, int* out, long long* clk) {
  const int lane = threadIdx.x & 63;
  v4i a[4], b[4];
  for (int s = 0; s < 4; ++s) {
    a[s] = *reinterpret_cast<const v4i*>(rnd + ((s * 64 + lane) * 4 + blockIdx.x * 7) % 65536);
    b[s] = *reinterpret_cast<const v4i*>(rnd + ((s * 64 + lane) * 4 + 4096 + threadIdx.x) % 65536);
  }
  float x[12];
  for (int i = 0; i < 12; ++i) x[i] = __int_as_float(rnd[(lane + i * 64) % 65536] & 0x3fffffff) * 0.001f + i;
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  int res = 0;
  if constexpr (SHAPE == 0) {
    v16i acc[4];
    for (int i = 0; i < 4; ++i)
      for (int r = 0; r < 16; ++r) acc[i][r] = lane + r;
    for (int it0 = 0; it0 < iters; it0 += 4) {
#pragma unroll
      for (int q = 0; q < 32; ++q) {
        acc[q & 3] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[q & 3], b[((q & 7) + (q >> 3)) & 3], acc[q & 3], 0, 0, 0);
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          const int c = (q * NV + v) % 12;
          if constexpr (KIND == 0) x[c] = __builtin_fmaf(x[c], 0.999f, 0.5f);
          else {
            if (v % 6 == 5) x[c] = __builtin_amdgcn_exp2f(x[c]);
            else if (v % 6 == 4) x[c] = __builtin_rintf(x[c]);
            else x[c] = __builtin_fmaf(x[c], 0.999f, 0.5f);
          }
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (NV) __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
      }
    }
    for (int i = 0; i < 4; ++i) res += acc[i][lane & 15];
  } else {
    v4i acc[8];
    for (int i = 0; i < 8; ++i)
      for (int r = 0; r < 4; ++r) acc[i][r] = lane + r;
    for (int it0 = 0; it0 < iters; it0 += 4) {
#pragma unroll
      for (int q = 0; q < 64; ++q) {
        acc[q & 7] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[q & 3], b[((q & 15) / 4 + (q >> 4)) & 3], acc[q & 7], 0, 0, 0);
        if (q & 1) {
#pragma unroll
          for (int v = 0; v < NV; ++v) {
            const int c = ((q >> 1) * NV + v) % 12;
            if constexpr (KIND == 0) x[c] = __builtin_fmaf(x[c], 0.999f, 0.5f);
            else {
              if (v % 6 == 5) x[c] = __builtin_amdgcn_exp2f(x[c]);
              else if (v % 6 == 4) x[c] = __builtin_rintf(x[c]);
              else x[c] = __builtin_fmaf(x[c], 0.999f, 0.5f);
            }
          }
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if ((q & 1) && NV) __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
      }
    }
    for (int i = 0; i < 8; ++i) res += acc[i][lane & 3];
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < 12; ++i) res += (int)x[i];
  if (res == 0x12345678) out[0] = res;
  if (threadIdx.x == 0) {
    clk[blockIdx.x * 2] = t1 - t0;
    clk[blockIdx.x * 2 + 1] = r1 - r0;
  }
}

template <int SHAPE, int NV, int KIND>
static void run(int wps, const int* rnd, int* d, long long* clk, const char* tag) {
  const int threads = 256 * wps, grid = 256;
  const int iters = 20000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  // warm: ~0.5 s of back-to-back launches
  for (int r = 0; r < 40; ++r) hipLaunchKernelGGL((k<SHAPE, NV, KIND>), dim3(grid), dim3(threads), 0, 0, rnd, iters, d, clk);
  hipEventRecord(e0);
  const int reps = 20;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k<SHAPE, NV, KIND>), dim3(grid), dim3(threads), 0, 0, rnd, iters, d, clk);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> h(grid * 2);
  hipMemcpy(h.data(), clk, grid * 2 * sizeof(long long), hipMemcpyDeviceToHost);
  std::vector<double> f;
  for (int g = 0; g < grid; ++g) f.push_back((double)h[2 * g] / (double)h[2 * g + 1] * 0.1);
  std::sort(f.begin(), f.end());
  // 32x32x32-equivalents per SIMD per launch: 8 per iteration per wave x wps waves
  const double eq = 8.0 * iters * wps;
  const double ns = ms * 1e6 / reps / eq;
  const double tops = 256.0 * 4 * eq * 65536.0 / (ms * 1e-3 / reps) / 1e12;
  printf("%-28s wps %d NV %2d: %6.2f ns per 32x32x32 per SIMD, %7.1f TOPS, clock %.2f GHz, %5.1f cyc/mfma@clk\n", tag,
         wps, NV, ns, tops, f[grid / 2], ns * f[grid / 2] / wps);
  fflush(stdout);
}

template <int SHAPE, int KIND>
static void sweep(int wps, const int* rnd, int* d, long long* clk, const char* tag) {
  run<SHAPE, 0, KIND>(wps, rnd, d, clk, tag);
  run<SHAPE, 2, KIND>(wps, rnd, d, clk, tag);
  run<SHAPE, 4, KIND>(wps, rnd, d, clk, tag);
  run<SHAPE, 6, KIND>(wps, rnd, d, clk, tag);
  run<SHAPE, 8, KIND>(wps, rnd, d, clk, tag);
  run<SHAPE, 12, KIND>(wps, rnd, d, clk, tag);
}

int main() {
  std::vector<int> h(65536);
  srand(1);
  for (auto& v : h) v = (rand() << 16) ^ rand();
  int *rnd, *d;
  long long* clk;
  hipMalloc(&rnd, 65536 * 4);
  hipMalloc(&d, 64);
  hipMalloc(&clk, 256 * 2 * 8);
  hipMemcpy(rnd, h.data(), 65536 * 4, hipMemcpyHostToDevice);
  for (int wps = 1; wps <= 2; ++wps) {
    sweep<0, 0>(wps, rnd, d, clk, "32x32x32 fma");
    sweep<1, 0>(wps, rnd, d, clk, "16x16x64 fma");
    sweep<0, 1>(wps, rnd, d, clk, "32x32x32 mix(exp,rint)");
    sweep<1, 1>(wps, rnd, d, clk, "16x16x64 mix(exp,rint)");
  }
  return 0;
}
