// Microbenchmark + numerics probe (round 3): the two f32-input MFMA shapes for the
// BLAS-order patch-embedding GEMM.  (1) Numerics: is v_mfma_f32_16x16x4_f32 (4 k-products
// per instruction) a k-ordered fmaf chain per output, as v_mfma_f32_32x32x2_f32 is?
// Compares one instruction chain over K = 64 against a host fmaf chain, bit for bit.
// (2) Rate: a bare loop of each shape (4 independent accumulators, 2 waves per SIMD),
// TFLOP/s and the in-kernel clock.
// Build: hipcc -O3 --offload-arch=gfx950 f32mfma.hip -o f32mfma
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

// C[16][16] = sum_k A[16][K] B[K][16] with v_mfma_f32_16x16x4_f32, k in order
__global__ void k_num16(const float* A, const float* B, float* C, int K) {
  const int lane = threadIdx.x;  // 64 lanes
  // operand layout (16x16x4): lane l supplies A[row l % 16][k0 + l / 16], B[k0 + l / 16][col l % 16]
  v4f acc = {0, 0, 0, 0};
  for (int k0 = 0; k0 < K; k0 += 4) {
    const float a = A[(lane % 16) * K + k0 + lane / 16];
    const float b = B[(k0 + lane / 16) * 16 + lane % 16];
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  // output layout: lane l holds rows 4 (l / 16) + r, column l % 16
  for (int r = 0; r < 4; ++r) C[(4 * (lane / 16) + r) * 16 + lane % 16] = acc[r];
}
__global__ void k_num32(const float* A, const float* B, float* C, int K) {
  const int lane = threadIdx.x;
  v16f acc;
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  for (int k0 = 0; k0 < K; k0 += 2) {
    const float a = A[(lane % 32) * K + k0 + lane / 32];
    const float b = B[(k0 + lane / 32) * 32 + lane % 32];
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 16; ++r) C[((r & 3) + 8 * (r >> 2) + 4 * (lane / 32)) * 32 + lane % 32] = acc[r];
}

template <int SHAPE>
__global__ void __launch_bounds__(512, 1) k_rate(int iters, float* out, long long* clk) {
  const int lane = threadIdx.x & 63;
  float a = 1.0f + lane * 1e-3f, b = 0.5f - lane * 1e-3f;
  if constexpr (SHAPE >= 1000) {  // (round 6) random-looking operands: a hash of (lane, block), sign and exponent spread
    uint32_t h = (uint32_t)(threadIdx.x * 2654435761u) ^ (uint32_t)(blockIdx.x * 40503u);
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    a = __uint_as_float((h & 0x807fffffu) | 0x3f000000u);          // +-[0.5, 1)
    b = __uint_as_float(((h * 2246822519u) & 0x807fffffu) | 0x3e800000u);  // +-[0.25, 0.5)
  }
  long long t0 = __builtin_amdgcn_s_memtime();
  float s = 0.0f;
  if constexpr (SHAPE == 16) {
    v4f acc[4];
    for (int i = 0; i < 4; ++i) acc[i] = v4f{0, 0, 0, 0};
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[q & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[q & 3], 0, 0, 0);
    for (int i = 0; i < 4; ++i) s += acc[i][0];
  } else {
    // SHAPE 32: four independent accumulator chains in rotation; 322: two (round 6: the order the
    // compiler gives k_embed_q's loop); 321: one; 1032: four, random-looking operands whose bits
    // change every instruction (a, b rotated through 4 values per lane)
    constexpr int CH = (SHAPE == 32 || SHAPE == 1032) ? 4 : (SHAPE == 322 ? 2 : 1);
    v16f acc[4];
    for (int i = 0; i < 4; ++i)
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.0f;
    float av[4] = {a, -b, b * 1.75f, -a * 0.625f}, bv[4] = {b, a * 0.875f, -a, b * 1.5f};
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float aa = SHAPE == 1032 ? av[q] : a, bb = SHAPE == 1032 ? bv[(q + 1) & 3] : b;
        acc[q % CH] = __builtin_amdgcn_mfma_f32_32x32x2f32(aa, bb, acc[q % CH], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    for (int i = 0; i < 4; ++i) s += acc[i][0];
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
  if (s == 12345.0f) out[0] = s;
}

static float host_chain(const float* A, const float* B, int K, int i, int j, int n) {
  float acc = 0.0f;
  for (int k = 0; k < K; ++k) acc = fmaf(A[i * K + k], B[k * n + j], acc);
  return acc;
}

int main() {
  const int K = 64;
  for (int shape : {16, 32}) {
    const int n = shape;
    std::vector<float> A(n * K), B(K * n), C(n * n);
    srand(1);
    int bad = 0, trials = 50;
    for (int t = 0; t < trials; ++t) {
      for (auto& v : A) v = (float)((rand() / (double)RAND_MAX - 0.5) * pow(2.0, rand() % 20 - 10));
      for (auto& v : B) v = (float)((rand() / (double)RAND_MAX - 0.5) * pow(2.0, rand() % 20 - 10));
      float *dA, *dB, *dC;
      hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4); hipMalloc(&dC, C.size() * 4);
      hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
      hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
      if (shape == 16) hipLaunchKernelGGL(k_num16, dim3(1), dim3(64), 0, 0, dA, dB, dC, K);
      else hipLaunchKernelGGL(k_num32, dim3(1), dim3(64), 0, 0, dA, dB, dC, K);
      hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost);
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
          const float h = host_chain(A.data(), B.data(), K, i, j, n);
          if (memcmp(&h, &C[i * n + j], 4)) ++bad;
        }
      hipFree(dA); hipFree(dB); hipFree(dC);
    }
    printf("numerics %dx%d f32 MFMA vs k-ordered fmaf chain (K=%d): %d of %d outputs differ\n", shape, shape, K, bad,
           trials * n * n);
  }
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float* out; long long* clk;
  hipMalloc(&out, 4); hipMalloc(&clk, cus * 8);
  const int iters = 20000;
  for (int shape : {16, 32, 322, 321, 1032}) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0);
      if (shape == 16) hipLaunchKernelGGL(k_rate<16>, dim3(cus), dim3(512), 0, 0, iters, out, clk);
      else if (shape == 32) hipLaunchKernelGGL(k_rate<32>, dim3(cus), dim3(512), 0, 0, iters, out, clk);
      else if (shape == 322) hipLaunchKernelGGL(k_rate<322>, dim3(cus), dim3(512), 0, 0, iters, out, clk);
      else if (shape == 1032) hipLaunchKernelGGL(k_rate<1032>, dim3(cus), dim3(512), 0, 0, iters, out, clk);
      else hipLaunchKernelGGL(k_rate<321>, dim3(cus), dim3(512), 0, 0, iters, out, clk);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      // flops per wave: 16x16x4: 16 instr x 2048 flops per iter; 32x32x2: 4 x 4096
      const double flops = (double)cus * 8 * iters * (shape == 16 ? 16 * 2048.0 : 4 * 4096.0);  // (1032: as 32)
      long long c0; hipMemcpy(&c0, clk, 8, hipMemcpyDeviceToHost);
      printf("rate %dx%d f32: %.3f ms  %.1f TFLOP/s  (shader clock ~%.2f GHz from s_memtime)\n", shape, shape, ms,
             flops / ms / 1e9, c0 / (ms * 1e6));
    }
  }
  return 0;
}
