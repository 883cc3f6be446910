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

void gather_plan(uint32_t rank, uint32_t nranks, uint32_t root, uint64_t count, std::vector<XferOp>& ops) {
  ops.clear();
  if (nranks < 2 || root >= nranks || rank >= nranks) return;
  if (rank == root) {
    for (uint32_t r = 0; r < nranks; r++)
      if (r != root) ops.push_back(XferOp{r, (uint64_t)r * count, count, true});
  } else {
    ops.push_back(XferOp{root, 0, count, false});
  }
}

bool comm_gather(Comm* c, const float4* send, float4* recv, uint64_t count, uint32_t root, hipStream_t stream,
                 std::string& err) {
  if (root >= c->nranks) {
    err = "bad root";
    return false;
  }
  std::vector<XferOp> ops;
  gather_plan(c->rank, c->nranks, root, count, ops);
  if (!ops.empty()) {
    // point-to-point over xGMI: every rank's packed partition to the root
    if (!nccl_ok(ncclGroupStart(), "ncclGroupStart", err)) return false;
    for (const XferOp& op : ops) {
      const ncclResult_t r = op.recv ? ncclRecv(recv + op.offset, 4 * op.count, ncclFloat, (int)op.peer, c->comm, stream)
                                     : ncclSend(send, 4 * op.count, ncclFloat, (int)op.peer, c->comm, stream);
      if (!nccl_ok(r, op.recv ? "ncclRecv" : "ncclSend", err)) {
        (void)ncclGroupEnd();
        return false;
      }
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
