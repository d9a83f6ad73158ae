// collective.h -- the one exchange step of the row-sharded decode (SURVEY.md
// §8(e)): an in-place all-gather of per-shard output rows.
//
// Each rank of a tensor-parallel group owns a contiguous slice of every
// projection's output rows (heads for q/k/v, rows for o/down, hidden units
// for gate/up, vocabulary rows for the logits) and writes it at
// buf + rank * bytes_per_rank of a full-size buffer; all_gather() fills in
// the other ranks' slices, stream-ordered on the session stream.
//
//  * RcclCollective: one process per GPU, ncclAllGather over xGMI; capturable
//    into the session's per-token hipGraph.
//  * LocalCollective: G sessions on ONE device driven from G host threads,
//    exchanging slices with device-to-device copies.  Not capturable (it
//    synchronises the host threads at every call); it exists so the sharding
//    itself is testable on a single GPU (RCCL refuses two ranks per device).
#pragma once

#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstddef>
#include <memory>
#include <mutex>
#include <vector>

namespace llmi {

class Collective {
 public:
  Collective(int rank, int size) : rank_(rank), size_(size) {}
  virtual ~Collective() = default;
  int rank() const { return rank_; }
  int size() const { return size_; }
  virtual bool graph_safe() const = 0;
  // in place: this rank's slice is already at buf + rank * bytes
  virtual void all_gather(void* buf, size_t bytes, hipStream_t s) = 0;

 protected:
  int rank_, size_;
};

// unique id for a new RCCL communicator (rank 0 makes it, the caller
// distributes it, every rank passes it to make_rccl)
void rccl_unique_id(void* out128);
std::unique_ptr<Collective> make_rccl(int rank, int size, const void* id128);

struct LocalGroup {
  explicit LocalGroup(int n);
  ~LocalGroup();
  // every rank reaches the same point; throws after a timeout (a rank that
  // failed leaves the others waiting otherwise)
  void barrier();

  const int n;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  unsigned long gen = 0;
  std::vector<bool> joined;
  std::vector<void*> bufs;
  std::vector<hipEvent_t> ready, done;
};

std::unique_ptr<Collective> make_local(LocalGroup* g, int rank);
// no exchange at all (diagnostics only: per-rank kernel time of a shard)
std::unique_ptr<Collective> make_null(int rank, int size);

}  // namespace llmi
