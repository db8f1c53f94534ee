// Shared internals of libnqk.so (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include "../../include/nqk.h"

namespace nqk {

hipStream_t stream();                      // the library stream of the current device
int fail(const std::string& msg);          // record an error message, return -1
int check(hipError_t e, const char* what); // 0 or fail()
inline int launch_status(const char* what) { return check(hipGetLastError(), what); }

// 64-bit grid-stride helpers
constexpr int kThreads = 256;
inline unsigned grid_for(int64_t n, int threads = kThreads, int64_t cap = 256 * 16) {
  int64_t g = (n + threads - 1) / threads;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

struct BatchMap {  // see nqk.h: output batch b -> (b / inner, b % inner)
  int64_t inner, ao, ai, bo, bi;
};
inline BatchMap batch_map(const int64_t* p) {
  BatchMap m{1, 1, 0, 1, 0};
  if (p) { m.inner = p[0] > 0 ? p[0] : 1; m.ao = p[1]; m.ai = p[2]; m.bo = p[3]; m.bi = p[4]; }
  return m;
}
__host__ __device__ inline int64_t map_a(const BatchMap& m, int64_t b) { return (b / m.inner) * m.ao + (b % m.inner) * m.ai; }
__host__ __device__ inline int64_t map_b(const BatchMap& m, int64_t b) { return (b / m.inner) * m.bo + (b % m.inner) * m.bi; }

// typed load/store of the integer storage classes
template <typename T> struct DT;
template <> struct DT<int8_t>  { static constexpr int code = NQK_I8; };
template <> struct DT<int16_t> { static constexpr int code = NQK_I16; };
template <> struct DT<int32_t> { static constexpr int code = NQK_I32; };
template <> struct DT<int64_t> { static constexpr int code = NQK_I64; };

// dispatch a lambda templated on the integer type of `code`
#define NQK_INT_DISPATCH(code, T, ...)                                 \
  switch (code) {                                                      \
    case NQK_I8:  { using T = int8_t;  __VA_ARGS__; break; }           \
    case NQK_I16: { using T = int16_t; __VA_ARGS__; break; }           \
    case NQK_I32: { using T = int32_t; __VA_ARGS__; break; }           \
    case NQK_I64: { using T = int64_t; __VA_ARGS__; break; }           \
    default: return fail("unsupported integer dtype code");            \
  }

}  // namespace nqk
