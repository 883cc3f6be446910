// wpt_comm.cpp — RCCL communicator of the multi-GPU path (wpt_comm.h).
#include "wpt_comm.h"

#include <rccl/rccl.h>

#include <string.h>

namespace wpt {

struct Comm {
  ncclComm_t comm = nullptr;
  uint32_t rank = 0, nranks = 1;
};

namespace {
bool nccl_ok(ncclResult_t r, const char* what, std::string& err) {
  if (r == ncclSuccess) return true;
  err = std::string(what) + " failed: " + ncclGetErrorString(r);
  return false;
}
}  // namespace

bool comm_unique_id(void* out128, std::string& err) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  ncclUniqueId id;
  if (!nccl_ok(ncclGetUniqueId(&id), "ncclGetUniqueId", err)) return false;
  memcpy(out128, &id, sizeof id);
  return true;
}

Comm* comm_create(uint32_t rank, uint32_t nranks, const void* id128, std::string& err) {
  if (nranks == 0 || rank >= nranks) {
    err = "bad rank";
    return nullptr;
  }
  ncclUniqueId id;
  memcpy(&id, id128, sizeof id);
  Comm* c = new Comm();
  c->rank = rank;
  c->nranks = nranks;
  if (!nccl_ok(ncclCommInitRank(&c->comm, (int)nranks, id, (int)rank), "ncclCommInitRank", err)) {
    delete c;
    return nullptr;
  }
  return c;
}

void comm_destroy(Comm* c) {
  if (!c) return;
  if (c->comm) (void)ncclCommDestroy(c->comm);
  delete c;
}

uint32_t comm_rank(const Comm* c) { return c->rank; }
uint32_t comm_size(const Comm* c) { return c->nranks; }

bool comm_allgather(Comm* c, const float4* send, float4* recv, uint64_t count, hipStream_t stream, std::string& err) {
  if (!nccl_ok(ncclAllGather(send, recv, 4 * count, ncclFloat, c->comm, stream), "ncclAllGather", err)) return false;
  const hipError_t e = hipStreamSynchronize(stream);
  if (e != hipSuccess) {
    err = std::string("hipStreamSynchronize failed: ") + hipGetErrorString(e);
    return false;
  }
  return true;
}

bool comm_gather(Comm* c, const float4* send, float4* recv, uint64_t count, uint32_t root, hipStream_t stream,
                 std::string& err) {
  if (root >= c->nranks) {
    err = "bad root";
    return false;
  }
  if (c->nranks > 1) {
    // point-to-point over xGMI: every rank's packed partition to the root
    if (!nccl_ok(ncclGroupStart(), "ncclGroupStart", err)) return false;
    if (c->rank == root) {
      for (uint32_t r = 0; r < c->nranks; r++) {
        if (r == root) continue;
        if (!nccl_ok(ncclRecv(recv + (size_t)r * count, 4 * count, ncclFloat, (int)r, c->comm, stream), "ncclRecv",
                     err)) {
          (void)ncclGroupEnd();
          return false;
        }
      }
    } else if (!nccl_ok(ncclSend(send, 4 * count, ncclFloat, (int)root, c->comm, stream), "ncclSend", err)) {
      (void)ncclGroupEnd();
      return false;
    }
    if (!nccl_ok(ncclGroupEnd(), "ncclGroupEnd", err)) return false;
  }
  const hipError_t e = hipStreamSynchronize(stream);
  if (e != hipSuccess) {
    err = std::string("hipStreamSynchronize failed: ") + hipGetErrorString(e);
    return false;
  }
  return true;
}

}  // namespace wpt
