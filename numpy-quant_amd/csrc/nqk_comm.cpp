// Multi-GPU replicas over RCCL (xGMI): one process per GPU, a one-time broadcast
// of the packed quantized weights + parameters from rank 0 and a gather of the
// per-rank outputs.  The reference is single-process NumPy and
// has no collective of its own; there is no exchange in the per-forward data path.
#include <rccl/rccl.h>
#include <string.h>

#include "nqk_common.h"

namespace {
ncclComm_t g_comm = nullptr;
int g_nranks = 1, g_rank = 0;
int nccl_check(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return 0;
  return nqk::fail(std::string(what) + ": " + ncclGetErrorString(r));
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
  if (nccl_check(ncclCommInitRank(&g_comm, nranks, id, rank), "ncclCommInitRank")) return -1;
  g_nranks = nranks;
  g_rank = rank;
  return 0;
}

int nqk_comm_bcast(void* buf, size_t bytes, int root) {
  if (!g_comm) return nqk::fail("communicator not initialised");
  return nccl_check(ncclBroadcast(buf, buf, bytes, ncclInt8, root, g_comm, nqk::stream()), "ncclBroadcast");
}

int nqk_comm_gather(const void* send, void* recv, size_t bytes_per_rank, int root) {
  if (!g_comm) return nqk::fail("communicator not initialised");
  return nccl_check(ncclGather(send, recv, bytes_per_rank, ncclInt8, root, g_comm, nqk::stream()), "ncclGather");
}

int nqk_comm_barrier(void) {
  if (!g_comm) return 0;
  // a 4-byte all-reduce on the library stream, then a stream sync
  static void* scratch = nullptr;
  if (!scratch && nqk::check(hipMalloc(&scratch, 16), "hipMalloc")) return -1;
  if (nccl_check(ncclAllReduce(scratch, scratch, 1, ncclInt32, ncclSum, g_comm, nqk::stream()), "ncclAllReduce"))
    return -1;
  return nqk::check(hipStreamSynchronize(nqk::stream()), "hipStreamSynchronize");
}

int nqk_comm_destroy(void) {
  if (!g_comm) return 0;
  ncclResult_t r = ncclCommDestroy(g_comm);
  g_comm = nullptr;
  return nccl_check(r, "ncclCommDestroy");
}

}  // extern "C"
