// Semantics probe (round 4): does v_cvt_pk_u8_f32 saturate?  For every integral float x in
// [-2^24, 2^24] and a few special values, compares the byte it writes with clamp(x, 0, 255)
// and prints the mismatch count and examples (the epilogues' med3 clamp before it is
// redundant for 8-bit outputs exactly when the count is 0).
// Build: hipcc -O3 --offload-arch=gfx950 cvtu8.hip -o cvtu8
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k(unsigned long long* bad, int* ex) {
  const int64_t n = (int64_t)1 << 25;  // x = i - 2^24
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += (int64_t)gridDim.x * blockDim.x) {
    const float x = (float)(i - ((int64_t)1 << 24));
    const uint32_t b = __builtin_amdgcn_cvt_pk_u8_f32(x, 1, 0u) >> 8;
    const float c = x < 0.0f ? 0.0f : (x > 255.0f ? 255.0f : x);
    if (b != (uint32_t)c) {
      atomicAdd(bad, 1ull);
      ex[0] = (int)x;
      ex[1] = (int)b;
    }
  }
}

__global__ void special(const float* v, uint32_t* out) {  // (values from memory: no constant folding)
  const int i = threadIdx.x;
  if (i < 8) out[i] = __builtin_amdgcn_cvt_pk_u8_f32(v[i], 0, 0u);
}

int main() {
  unsigned long long* bad;
  int* ex;
  uint32_t* sp;
  (void)hipMalloc(&bad, 8);
  (void)hipMalloc(&ex, 8);
  (void)hipMalloc(&sp, 32);
  (void)hipMemset(bad, 0, 8);
  (void)hipMemset(ex, 0, 8);
  hipLaunchKernelGGL(k, dim3(4096), dim3(256), 0, 0, bad, ex);
  const float hv[8] = {__builtin_inff(), -__builtin_inff(), __builtin_nanf(""), 255.49f, 255.5f, -0.49f, 3e9f, -3e9f};
  float* dv;
  (void)hipMalloc(&dv, 32);
  (void)hipMemcpy(dv, hv, 32, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(special, dim3(1), dim3(64), 0, 0, dv, sp);
  unsigned long long hb;
  int he[2];
  uint32_t hs[8];
  (void)hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(he, ex, 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hs, sp, 32, hipMemcpyDeviceToHost);
  printf("integral x in [-2^24, 2^24]: %llu bytes differ from clamp(x, 0, 255) (e.g. x = %d -> %d)\n", hb, he[0], he[1]);
  printf("inf %u  -inf %u  nan %u  255.49 %u  255.5 %u  -0.49 %u  3e9 %u  -3e9 %u\n", hs[0], hs[1], hs[2], hs[3], hs[4],
         hs[5], hs[6], hs[7]);
  return 0;
}
