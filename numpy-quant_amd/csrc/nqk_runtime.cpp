// Runtime half of the C ABI: device selection, the per-device stream, memory,
// timers and hipGraph capture (include/nqk.h "runtime").
#include "nqk_common.h"

#include <mutex>
#include <string>

namespace {
thread_local std::string g_err;
int g_device = -1;
hipStream_t g_streams[64] = {};
constexpr int kSide = 3;           // side streams 1..3 (nqk_set_stream)
hipStream_t g_side[64][kSide] = {};
int g_cur = 0;                     // current stream index of the (single) host thread
hipEvent_t g_fork[64] = {}, g_join[64][kSide] = {};  // per device, with that device's side streams
hipEvent_t g_t0 = nullptr, g_t1 = nullptr;
hipGraph_t g_capturing = nullptr;
std::mutex g_mu;
}  // namespace

namespace nqk {
int fail(const std::string& msg) { g_err = msg; return -1; }
int check(hipError_t e, const char* what) {
  if (e == hipSuccess) return 0;
  return fail(std::string(what) + ": " + hipGetErrorString(e));
}
hipStream_t stream() {
  if (g_device < 0) nqk_init(0);
  return g_cur ? g_side[g_device][g_cur - 1] : g_streams[g_device];
}
}  // namespace nqk

using namespace nqk;

extern "C" {

const char* nqk_last_error(void) { return g_err.c_str(); }

int nqk_device_count(int* count) { return check(hipGetDeviceCount(count), "hipGetDeviceCount"); }

int nqk_init(int device) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (device < 0 || device >= 64) return fail("bad device index");
  if (check(hipSetDevice(device), "hipSetDevice")) return -1;
  if (!g_streams[device]) {
    if (check(hipStreamCreateWithFlags(&g_streams[device], hipStreamNonBlocking), "hipStreamCreate")) return -1;
  }
  g_device = device;
  if (!g_t0) {
    if (check(hipEventCreate(&g_t0), "hipEventCreate") || check(hipEventCreate(&g_t1), "hipEventCreate")) return -1;
  }
  return 0;
}

int nqk_malloc(void** ptr, size_t bytes) {
  if (g_device < 0 && nqk_init(0)) return -1;
  return check(hipMalloc(ptr, bytes ? bytes : 16), "hipMalloc");
}
int nqk_free(void* ptr) { return check(hipFree(ptr), "hipFree"); }

int nqk_memcpy_h2d(void* dst, const void* src, size_t bytes) {
  if (!bytes) return 0;
  if (check(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream()), "memcpy h2d")) return -1;
  return check(hipStreamSynchronize(stream()), "memcpy h2d sync");
}
int nqk_memcpy_d2h(void* dst, const void* src, size_t bytes) {
  if (!bytes) return 0;
  if (check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, stream()), "memcpy d2h")) return -1;
  return check(hipStreamSynchronize(stream()), "memcpy d2h sync");
}
int nqk_memcpy_d2d(void* dst, const void* src, size_t bytes) {
  if (!bytes) return 0;
  return check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, stream()), "memcpy d2d");
}
int nqk_memset(void* ptr, int value, size_t bytes) {
  if (!bytes) return 0;
  return check(hipMemsetAsync(ptr, value, bytes, stream()), "memset");
}
int nqk_sync(void) {
  for (int i = 0; g_device >= 0 && i < kSide; ++i)
    if (g_side[g_device][i] && check(hipStreamSynchronize(g_side[g_device][i]), "hipStreamSynchronize")) return -1;
  return check(hipStreamSynchronize(g_device >= 0 ? g_streams[g_device] : stream()), "hipStreamSynchronize");
}

static int ensure_side() {
  if (g_device < 0 && nqk_init(0)) return -1;
  for (int i = 0; i < kSide; ++i) {
    if (!g_side[g_device][i] &&
        check(hipStreamCreateWithFlags(&g_side[g_device][i], hipStreamNonBlocking), "hipStreamCreate"))
      return -1;
    if (!g_join[g_device][i] &&
        check(hipEventCreateWithFlags(&g_join[g_device][i], hipEventDisableTiming), "hipEventCreate"))
      return -1;
  }
  if (!g_fork[g_device] && check(hipEventCreateWithFlags(&g_fork[g_device], hipEventDisableTiming), "hipEventCreate"))
    return -1;
  return 0;
}

int nqk_set_stream(int which) {
  if (which < 0 || which > kSide) return fail("nqk_set_stream: 0 .. 3");
  if (which && ensure_side()) return -1;
  g_cur = which;
  return 0;
}

int nqk_stream_fork(void) {
  if (ensure_side()) return -1;
  if (check(hipEventRecord(g_fork[g_device], g_streams[g_device]), "hipEventRecord")) return -1;
  for (int i = 0; i < kSide; ++i)
    if (check(hipStreamWaitEvent(g_side[g_device][i], g_fork[g_device], 0), "hipStreamWaitEvent")) return -1;
  return 0;
}

int nqk_stream_join(void) {
  if (ensure_side()) return -1;
  for (int i = 0; i < kSide; ++i) {
    if (check(hipEventRecord(g_join[g_device][i], g_side[g_device][i]), "hipEventRecord")) return -1;
    if (check(hipStreamWaitEvent(g_streams[g_device], g_join[g_device][i], 0), "hipStreamWaitEvent")) return -1;
  }
  return 0;
}
int nqk_stream(void** s) { *s = (void*)stream(); return 0; }

int nqk_timer_start(void) { return check(hipEventRecord(g_t0, stream()), "hipEventRecord"); }
int nqk_timer_stop(void) { return check(hipEventRecord(g_t1, stream()), "hipEventRecord"); }
int nqk_timer_ms(float* ms) {
  if (check(hipEventSynchronize(g_t1), "hipEventSynchronize")) return -1;
  return check(hipEventElapsedTime(ms, g_t0, g_t1), "hipEventElapsedTime");
}

int nqk_event_create(void** event) {
  hipEvent_t e = nullptr;
  if (check(hipEventCreate(&e), "hipEventCreate")) return -1;
  *event = (void*)e;
  return 0;
}
int nqk_event_record(void* event) { return check(hipEventRecord((hipEvent_t)event, stream()), "hipEventRecord"); }
int nqk_event_elapsed(void* start, void* stop, float* ms) {
  if (check(hipEventSynchronize((hipEvent_t)stop), "hipEventSynchronize")) return -1;
  return check(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop), "hipEventElapsedTime");
}
int nqk_event_destroy(void* event) { return check(hipEventDestroy((hipEvent_t)event), "hipEventDestroy"); }
int nqk_event_wait(void* event) { return check(hipStreamWaitEvent(stream(), (hipEvent_t)event, 0), "hipStreamWaitEvent"); }

int nqk_graph_begin(void) {
  // relaxed: the caching allocator may still hipMalloc a fresh block mid-capture
  // (the block lives outside the graph; graph.py pins it for the graph's lifetime)
  g_cur = 0;
  return check(hipStreamBeginCapture(stream(), hipStreamCaptureModeRelaxed), "hipStreamBeginCapture");
}
int nqk_graph_abort(void) {
  // a capture that failed part-way: join the side streams back (they may be part of the
  // capture after a fork), end the capture and drop the partial graph
  g_cur = 0;
  for (int i = 0; g_device >= 0 && i < kSide; ++i)
    if (g_side[g_device][i] && g_join[g_device][i]) {
      (void)hipEventRecord(g_join[g_device][i], g_side[g_device][i]);
      (void)hipStreamWaitEvent(g_streams[g_device], g_join[g_device][i], 0);
    }
  hipGraph_t g = nullptr;
  (void)hipStreamEndCapture(stream(), &g);
  if (g) (void)hipGraphDestroy(g);
  (void)hipGetLastError();
  return 0;
}
int nqk_graph_end(void** graph_exec) {
  hipGraph_t g = nullptr;
  if (check(hipStreamEndCapture(stream(), &g), "hipStreamEndCapture")) return -1;
  hipGraphExec_t ex = nullptr;
  if (check(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0), "hipGraphInstantiate")) return -1;
  (void)hipGraphDestroy(g);
  *graph_exec = (void*)ex;
  return 0;
}
int nqk_graph_launch(void* graph_exec) {
  return check(hipGraphLaunch((hipGraphExec_t)graph_exec, stream()), "hipGraphLaunch");
}
int nqk_graph_destroy(void* graph_exec) {
  return check(hipGraphExecDestroy((hipGraphExec_t)graph_exec), "hipGraphExecDestroy");
}

}  // extern "C"
