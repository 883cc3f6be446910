// wpt_comm.h — RCCL communicator of the multi-GPU path.
//
// One process per GPU; every rank renders its interleaved-tile partition with
// no data-path communication. RCCL carries only
//   * the final frame gather to one rank (grouped ncclSend / ncclRecv of the
//     packed partitions over xGMI), and
//   * the adaptive-round frame exchange (ncclAllGather of the packed
//     partitions at each round boundary of an adaptive screen half).
// The reference has no collective at all (one worker); its README
// intends random pixel partitions over 8 workers (README.md:87).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <vector>

namespace wpt {

struct Comm;

// One transfer of a rooted gather of packed partitions (rank-major layout:
// rank r's `count` float4 at offset r * count of the root's buffer): the
// root receives from every other rank, every other rank sends to the root.
struct XferOp {
  uint32_t peer;    // the other rank
  uint64_t offset;  // float4 offset in the root's receive buffer (recv ops)
  uint64_t count;   // float4 moved
  bool recv;        // true: root receives from peer; false: this rank sends its buffer to peer
};
void gather_plan(uint32_t rank, uint32_t nranks, uint32_t root, uint64_t count, std::vector<XferOp>& ops);

// ncclGetUniqueId: 128 bytes, made by one rank and handed to all.
bool comm_unique_id(void* out128, std::string& err);
// ncclCommInitRank on the calling thread's current HIP device (collective).
Comm* comm_create(uint32_t rank, uint32_t nranks, const void* id128, std::string& err);
void comm_destroy(Comm* c);
uint32_t comm_rank(const Comm* c);
uint32_t comm_size(const Comm* c);
// Every rank's `count` float4 at `send` into `recv` (rank-major, nranks *
// count float4) on `stream`; returns after the stream has completed.
bool comm_allgather(Comm* c, const float4* send, float4* recv, uint64_t count, hipStream_t stream, std::string& err);
// Every rank's `count` float4 at `send` into root's `recv` (rank-major; the
// root's own slot is left untouched) on `stream`; returns after completion.
bool comm_gather(Comm* c, const float4* send, float4* recv, uint64_t count, uint32_t root, hipStream_t stream,
                 std::string& err);

}  // namespace wpt
