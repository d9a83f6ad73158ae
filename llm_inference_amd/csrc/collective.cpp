// collective.cpp -- RCCL and single-device implementations of collective.h.
#include "collective.h"

#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>

#include "common.h"

namespace llmi {

#define LLMI_NCCL(call)                                                                           \
  do {                                                                                            \
    ncclResult_t r_ = (call);                                                                     \
    if (r_ != ncclSuccess) throw hip_error(std::string(#call) + ": " + ncclGetErrorString(r_)); \
  } while (0)

void rccl_unique_id(void* out128) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId id;
  LLMI_NCCL(ncclGetUniqueId(&id));
  std::memcpy(out128, &id, sizeof(id));
}

namespace {

class RcclCollective : public Collective {
 public:
  RcclCollective(int rank, int size, const void* id128) : Collective(rank, size) {
    ncclUniqueId id;
    std::memcpy(&id, id128, sizeof(id));
    LLMI_NCCL(ncclCommInitRank(&comm_, size, id, rank));
  }
  ~RcclCollective() override {
    if (comm_) (void)ncclCommDestroy(comm_);
  }
  bool graph_safe() const override { return true; }
  void all_gather(void* buf, size_t bytes, hipStream_t s) override {
    char* b = static_cast<char*>(buf);
    LLMI_NCCL(ncclAllGather(b + (size_t)rank_ * bytes, b, bytes, ncclUint8, comm_, s));
  }

 private:
  ncclComm_t comm_ = nullptr;
};

class LocalCollective : public Collective {
 public:
  LocalCollective(LocalGroup* g, int rank) : Collective(rank, g->n), g_(g) {
    std::lock_guard<std::mutex> lk(g->mu);
    if (rank < 0 || rank >= g->n || g->joined[rank]) throw std::runtime_error("local group: bad or duplicate rank");
    g->joined[rank] = true;
    LLMI_HIP(hipEventCreateWithFlags(&g->ready[rank], hipEventDisableTiming));
    LLMI_HIP(hipEventCreateWithFlags(&g->done[rank], hipEventDisableTiming));
  }
  ~LocalCollective() override {
    std::lock_guard<std::mutex> lk(g_->mu);
    g_->joined[rank_] = false;
    (void)hipEventDestroy(g_->ready[rank_]);
    (void)hipEventDestroy(g_->done[rank_]);
    g_->ready[rank_] = g_->done[rank_] = nullptr;
  }
  bool graph_safe() const override { return false; }
  void all_gather(void* buf, size_t bytes, hipStream_t s) override {
    LocalGroup& g = *g_;
    char* b = static_cast<char*>(buf);
    // 1. publish this rank's buffer once its slice is written
    g.bufs[rank_] = buf;
    LLMI_HIP(hipEventRecord(g.ready[rank_], s));
    g.barrier();
    // 2. pull every other slice from its owner's buffer
    for (int q = 0; q < size_; q++) {
      if (q == rank_) continue;
      LLMI_HIP(hipStreamWaitEvent(s, g.ready[q], 0));
      LLMI_HIP(hipMemcpyAsync(b + (size_t)q * bytes, static_cast<char*>(g.bufs[q]) + (size_t)q * bytes, bytes,
                              hipMemcpyDeviceToDevice, s));
    }
    LLMI_HIP(hipEventRecord(g.done[rank_], s));
    g.barrier();
    // 3. nobody overwrites its slice before every peer has copied it
    for (int q = 0; q < size_; q++)
      if (q != rank_) LLMI_HIP(hipStreamWaitEvent(s, g.done[q], 0));
  }

 private:
  LocalGroup* g_;
};

// diagnostics (LLMI_TP_SOLO): one rank of a sharded group with the exchange
// left out, to time a rank's own kernels on a single GPU
class NullCollective : public Collective {
 public:
  using Collective::Collective;
  bool graph_safe() const override { return true; }
  void all_gather(void*, size_t, hipStream_t) override {}
};

}  // namespace

std::unique_ptr<Collective> make_null(int rank, int size) {
  return std::unique_ptr<Collective>(new NullCollective(rank, size));
}

LocalGroup::LocalGroup(int n_) : n(n_), joined(n_, false), bufs(n_, nullptr), ready(n_, nullptr), done(n_, nullptr) {
  if (n_ < 1) throw std::runtime_error("local group: size < 1");
}

LocalGroup::~LocalGroup() = default;

void LocalGroup::barrier() {
  std::unique_lock<std::mutex> lk(mu);
  const unsigned long my = gen;
  if (++arrived == n) {
    arrived = 0;
    gen++;
    cv.notify_all();
    return;
  }
  if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return gen != my; }))
    throw std::runtime_error("local group: barrier timeout (a rank stopped)");
}

std::unique_ptr<Collective> make_rccl(int rank, int size, const void* id128) {
  return std::unique_ptr<Collective>(new RcclCollective(rank, size, id128));
}

std::unique_ptr<Collective> make_local(LocalGroup* g, int rank) {
  return std::unique_ptr<Collective>(new LocalCollective(g, rank));
}

}  // namespace llmi
