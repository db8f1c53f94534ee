// Microbenchmark (round 3): VALU issue throughput per SIMD with 1, 2, 4 waves per SIMD and no
// MFMA: does a second wave on the SIMD double the epilogue's VALU rate?  Ops: v_fma_f32,
// v_pk_fma_f32 (2 lanes of f32 per instruction), v_exp_f32, v_cvt_f32_i32 + v_rndne mix.
// Build: hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 valu.hip -o valu
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

typedef float v2f __attribute__((ext_vector_type(2)));

template <int OP>
__global__ void __launch_bounds__(1024, 1) k(int iters, float* out) {
  const int lane = threadIdx.x & 63;
  float x[16];
  v2f y[8];
  for (int i = 0; i < 16; ++i) x[i] = lane * 0.001f + i;
  for (int i = 0; i < 8; ++i) y[i] = v2f{lane * 0.002f + i, 0.5f * i};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if constexpr (OP == 0) {
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = __builtin_fmaf(x[i], 0.999f, 0.5f);
      } else if constexpr (OP == 1) {
#pragma unroll
        for (int i = 0; i < 8; ++i) y[i] = __builtin_elementwise_fma(y[i], v2f{0.999f, 0.998f}, v2f{0.5f, 0.25f});
#pragma unroll
        for (int i = 0; i < 8; ++i) y[i] = __builtin_elementwise_fma(y[i], v2f{0.997f, 0.996f}, v2f{0.5f, 0.25f});
      } else if constexpr (OP == 2) {
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = __builtin_amdgcn_exp2f(x[i]);
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = (i & 1) ? __builtin_rintf(x[i]) : (float)(int)x[i];
      }
    }
  }
  float s = 0;
  for (int i = 0; i < 16; ++i) s += x[i];
  for (int i = 0; i < 8; ++i) s += y[i][0] + y[i][1];
  if (s == 1234.5f) out[0] = s;
}

template <int OP>
static void run(int wps, float* d, const char* tag) {
  const int iters = 20000;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k<OP>), dim3(256), dim3(256 * wps), 0, 0, iters, d);
  hipEventRecord(a);
  for (int r = 0; r < 10; ++r) hipLaunchKernelGGL((k<OP>), dim3(256), dim3(256 * wps), 0, 0, iters, d);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  // wave-instructions per SIMD: 64 per iteration per wave (pk: 64 instructions = 128 fma)
  const double ins = 64.0 * iters * wps;
  printf("%-10s wps %d: %6.3f ns per wave-instruction per SIMD\n", tag, wps, ms * 1e6 / 10 / ins);
  fflush(stdout);
}

int main() {
  float* d;
  (void)hipMalloc(&d, 64);
  for (int wps = 1; wps <= 4; wps *= 2) {
    run<0>(wps, d, "v_fma");
    run<1>(wps, d, "v_pk_fma");
    run<2>(wps, d, "v_exp");
    run<3>(wps, d, "cvt/rndne");
  }
  return 0;
}
