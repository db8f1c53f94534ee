// Multi-GPU replicas over RCCL (xGMI): one process per GPU, a one-time broadcast
// of the packed quantized weights + parameters from rank 0 and a gather of the
// per-rank outputs.  The reference is single-process NumPy and
// has no collective of its own; there is no exchange in the per-forward data path.
#include <rccl/rccl.h>
#include <stdlib.h>
#include <string.h>
#include <sched.h>
#include <time.h>

#include "nqk_common.h"

namespace {
ncclComm_t g_comm = nullptr;
int g_nranks = 1, g_rank = 0;
int nccl_check(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return 0;
  return nqk::fail(std::string(what) + ": " + ncclGetErrorString(r));
}
double now_s() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}
// The communicator is non-blocking (config.blocking = 0), so that a rank whose peer died
// before joining does not wait forever inside ncclCommInitRank: every call returns
// ncclInProgress until its host-side work is done, polled here against a deadline
// (NQK_COMM_TIMEOUT_S, default 120 s); past it the communicator is aborted and the call fails.
// The deadline covers the HOST side of a call (init, the enqueue of a collective).  A collective
// already enqueued on the stream whose peer then dies never completes on the GPU: nqk_comm_barrier
// (the only place this library waits for one) therefore polls the stream and the communicator's
// async error against the same deadline instead of blocking in hipStreamSynchronize.  A caller that
// synchronizes the stream itself (nqk_sync) is not covered: bench.py's parent kills such a rank.
double comm_deadline_s() {
  const char* v = getenv("NQK_COMM_TIMEOUT_S");
  const double d = v ? atof(v) : 120.0;
  return d > 0 ? d : 120.0;
}
// a polling loop's pause: the first 2 000 polls spin (sched_yield), so a grouped op that reports
// ncclInProgress for a few microseconds (ncclGather on a non-blocking communicator, every step)
// does not pay a timer slice; past that 0.2 ms sleeps (the sleep alone cost a step
// >= 0.2 ms)
void pause_after(long spins) {
  if (spins < 2000) {
    sched_yield();
  } else {
    timespec ts{0, 200000};  // 0.2 ms
    nanosleep(&ts, nullptr);
  }
}
int nccl_wait(ncclResult_t r, const char* what) {
  if (r != ncclSuccess && r != ncclInProgress) return nccl_check(r, what);
  const double t0 = now_s(), lim = comm_deadline_s();
  long spins = 0;
  while (r == ncclInProgress) {
    if (ncclCommGetAsyncError(g_comm, &r) != ncclSuccess) break;
    if (r != ncclInProgress) break;
    if (now_s() - t0 > lim) {
      ncclCommAbort(g_comm);
      g_comm = nullptr;
      return nqk::fail(std::string(what) + ": not complete after " + std::to_string((int)lim) +
                       " s (a peer rank is gone?); communicator aborted");
    }
    pause_after(++spins);
  }
  return nccl_check(r, what);
}
}  // namespace

extern "C" {

int nqk_comm_unique_id(void* id128) {
  ncclUniqueId id;
  if (nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId")) return -1;
  memcpy(id128, &id, sizeof(id));
  return 0;
}

int nqk_comm_init(const void* id128, int nranks, int rank) {
  ncclUniqueId id;
  memcpy(&id, id128, sizeof(id));
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  const ncclResult_t r = ncclCommInitRankConfig(&g_comm, nranks, id, rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) {
    g_comm = nullptr;
    return nccl_check(r, "ncclCommInitRankConfig");
  }
  if (nccl_wait(r, "ncclCommInitRankConfig")) return -1;
  g_nranks = nranks;
  g_rank = rank;
  return 0;
}

int nqk_comm_bcast(void* buf, size_t bytes, int root) {
  if (!g_comm) return nqk::fail("communicator not initialised");
  return nccl_wait(ncclBroadcast(buf, buf, bytes, ncclInt8, root, g_comm, nqk::stream()), "ncclBroadcast");
}

int nqk_comm_gather(const void* send, void* recv, size_t bytes_per_rank, int root) {
  if (!g_comm) return nqk::fail("communicator not initialised");
  return nccl_wait(ncclGather(send, recv, bytes_per_rank, ncclInt8, root, g_comm, nqk::stream()), "ncclGather");
}

int nqk_comm_barrier(void) {
  if (!g_comm) return 0;
  // a 4-byte all-reduce on the library stream, then a stream sync
  static void* scratch = nullptr;
  if (!scratch && nqk::check(hipMalloc(&scratch, 16), "hipMalloc")) return -1;
  if (nccl_wait(ncclAllReduce(scratch, scratch, 1, ncclInt32, ncclSum, g_comm, nqk::stream()), "ncclAllReduce"))
    return -1;
  // the stream drains when every rank joined the all-reduce: poll it (and the communicator's
  // async error) against the deadline rather than block forever on a dead peer
  const double t0 = now_s(), lim = comm_deadline_s();
  for (long spins = 0;; ++spins) {
    const hipError_t q = hipStreamQuery(nqk::stream());
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) return nqk::check(q, "hipStreamQuery");
    ncclResult_t ar = ncclSuccess;
    if (ncclCommGetAsyncError(g_comm, &ar) == ncclSuccess && ar != ncclSuccess && ar != ncclInProgress)
      return nccl_check(ar, "nqk_comm_barrier");
    if (now_s() - t0 > lim) {
      ncclCommAbort(g_comm);
      g_comm = nullptr;
      return nqk::fail("nqk_comm_barrier: the all-reduce did not complete after " + std::to_string((int)lim) +
                       " s (a peer rank is gone?); communicator aborted");
    }
    pause_after(spins);
  }
}

int nqk_comm_destroy(void) {
  if (!g_comm) return 0;
  // non-blocking communicator: finalize (polled), then destroy
  ncclResult_t r = ncclCommFinalize(g_comm);
  if (r == ncclSuccess || r == ncclInProgress) {
    if (nccl_wait(r, "ncclCommFinalize")) return -1;
  }
  r = ncclCommDestroy(g_comm);
  g_comm = nullptr;
  return nccl_check(r, "ncclCommDestroy");
}

}  // extern "C"
