// Microbenchmark: bytes per clock per CU from L2 into a CU, by path.  Every workgroup
// (512 threads, one per CU) streams a 1 MiB window of an L2-resident buffer (one window
// per XCD label, all the XCD's workgroups read the same bytes) again and again.
//   mode 0: global_load_dwordx4 into VGPRs (xor-reduced, 4 loads in flight per lane)
//   mode 1: global_load_lds_dwordx4 (LDS-DMA) into a 32 KiB LDS ring, vmcnt(16) window
//   mode 2: both: half the waves each way
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

__global__ void __launch_bounds__(512, 1) k(const int8_t* buf, int mode, int iters, int* out) {
  extern __shared__ __attribute__((aligned(16))) int8_t lds[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int8_t* win = buf + (blockIdx.x & 7) * (1 << 20);
  v4i acc = {0, 0, 0, 0};
  const bool lds_path = mode == 1 || (mode == 2 && wave >= 4);
  // per iteration each wave reads 4 x 1 KiB pieces
  for (int it = 0; it < iters; ++it) {
    const int base = ((it * 8 + wave) * 4096) & ((1 << 20) - 1);
    if (lds_path) {
#pragma unroll
      for (int p = 0; p < 4; ++p)
        __builtin_amdgcn_global_load_lds((gbl_ptr_t)(win + base + p * 1024 + lane * 16),
                                         (lds_ptr_t)(lds + ((wave * 4 + p) & 31) * 1024), 16, 0, 0);
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    } else {
      v4i v[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) v[p] = *reinterpret_cast<const v4i*>(win + base + p * 1024 + lane * 16);
#pragma unroll
      for (int p = 0; p < 4; ++p) acc ^= v[p];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc[0] == 0x12345678) out[0] = acc[1] + lds[lane];
}

int main() {
  int8_t* buf;
  int* d;
  hipMalloc(&buf, 8 << 20);
  hipMemset(buf, 1, 8 << 20);
  hipMalloc(&d, 16);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);  // kHz
  const int iters = 4000;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[] = {"global->VGPR", "global->LDS (DMA)", "half and half"};
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 0; mode < 3; ++mode) {
      hipLaunchKernelGGL(k, dim3(cus), dim3(512), 32768, 0, buf, mode, iters, d);
      hipEventRecord(a);
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(cus), dim3(512), 32768, 0, buf, mode, iters, d);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double bytes = (double)cus * 8 * 4 * 1024 * iters;  // per launch
      const double s = ms / 5 * 1e-3;
      if (rep)
        printf("%-20s %7.3f ms  %7.1f TB/s  %6.1f B/clk/CU (clock %d MHz)\n", names[mode], ms / 5, bytes / s / 1e12,
               bytes / s / cus / (clk * 1e3), clk / 1000);
    }
  return 0;
}
