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
//  * PeerCollective: one process per GPU, the one-shot push exchange of
//    k_exchange.hip (every rank writes its slice as data-tagged granules into
//    every peer's mailbox through xGMI peer mappings, then polls its own: one
//    kernel per all-gather, no RCCL call); the mailboxes' IPC handles are
//    swapped by the caller (llmi_session_peer_handle / _connect).  Capturable.
//  * LocalCollective: G sessions on ONE device driven from G host threads.
//    Default: the same push kernel, split into push and gather launches around
//    a host barrier (one process's ranks share its hardware queues, so a
//    waiting gather must not be able to block a peer's push); LLMI_TP_EXCHANGE=
//    copy: device-to-device slice copies.  Not capturable (it synchronises the
//    host threads at every call); it exists so the sharding and the exchange
//    are testable on a single GPU (RCCL refuses two ranks per device).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include <condition_variable>
#include <cstddef>
#include <memory>
#include <mutex>
#include <vector>

#include "px.h"

namespace llmi {

// exchange kinds (llmi_session_info.tp_exchange)
enum { EX_NONE = 0, EX_RCCL = 1, EX_COPY = 2, EX_PUSH = 3, EX_PUSH_FUSED = 4 };

class Collective {
 public:
  Collective(int rank, int size) : rank_(rank), size_(size) {}
  virtual ~Collective() = default;
  int rank() const { return rank_; }
  int size() const { return size_; }
  virtual bool graph_safe() const = 0;
  virtual int kind() const = 0;
  // in place: this rank's slice is already at buf + rank * bytes.  skip (push exchange): the fused exchanges
  // (px.h) recorded since the previous standalone one -- this exchange's tag follows theirs
  virtual void all_gather(void* buf, size_t bytes, hipStream_t s, int skip = 0) = 0;
  // column slices of `rows` rows in place (rank q's slice of row i at buf + i * pitch + q * slice bytes), read and
  // written by the exchange kernel itself; false: not supported (the caller packs, all_gathers and unpacks)
  virtual bool all_gather_cols(void*, size_t, size_t, int, hipStream_t, int skip = 0) {
    (void)skip;
    return false;
  }
  // fused exchanges (px.h), push-exchange collectives only: the mailboxes as the launches see them (every
  // message of ws <= fused_cap() words per rank); fused_point sits between a producing and a consuming launch (a
  // LocalCollective makes every rank's producer complete first -- its ranks share one process's hardware queues
  // -- others do nothing)
  virtual bool fused_capable() const { return false; }
  virtual void fused_link(PxLink& l);
  static constexpr int fused_cap() { return 1 << 18; }
  virtual void fused_point(hipStream_t) {}
  // the exchange failed on the device since the last call (a bounded wait timed out, or a received slice
  // failed its checksum); 0 = no.  The ranks' exchange counts may then differ: the session stops.
  virtual int failed() { return 0; }
  virtual std::string fail_detail() const { return std::string(); }  // after failed(): what the wait last saw
  // push exchange between processes: this rank's mailbox handle, then every rank's (rank order)
  virtual void peer_handle(void* out) const;
  virtual void peer_connect(const void* handles);

 protected:
  int rank_, size_;
};

// ---- the one-shot push all-gather (k_exchange.hip) ----
constexpr int PX_MAX_WG = 64;  // work-groups per exchange launch (= checksum granules per sender slot)
constexpr int PX_PUSH = 1, PX_GATHER = 2;
struct PushArgs {
  uint2* mail[PX_MAX_RANKS];  // every rank's mailbox [2][G][cap + PX_CS_RING * PX_MAX_CS] granules (this process's mapping)
  uint32_t* buf;              // word j of rank q's message at buf + q * stride + j (row_w == 0), or at
  size_t stride;              // buf + (j / row_w) * pitch + q * row_w + j % row_w (column slices of rows)
  size_t pitch;
  int row_w;
  size_t off;                 // this exchange's first word of the message (a chunk of a longer one)
  int words;                  // per rank, <= cap
  int rank, G, cap, phase;    // phase: PX_PUSH | PX_GATHER
  unsigned* epoch;            // seed - 1 + exchanges completed (tag = epoch + 1)
  unsigned* ticket;           // work-groups done with the gather (the last one advances epoch)
  int* err;                   // 1: a wait timed out; 2: a received slice failed its checksum
  uint64_t timeout;           // bound of every wait, in ticks of the 100 MHz wall clock
  int skip;                   // fused exchanges since the previous standalone one: tag = epoch + 1 + skip
};
void launch_push_exchange(const PushArgs& a, hipStream_t s);
constexpr int PEER_HANDLE_BYTES = 64;

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
  std::vector<uint2*> mail;  // push exchange: every rank's mailbox (same process, same device)
  uint32_t seed;             // push exchange: first tag of this group's lifetime (collective.cpp px_seed)
};

std::unique_ptr<Collective> make_local(LocalGroup* g, int rank, int size, hipStream_t s);
// one process per GPU, push exchange; all_gather throws until peer_connect
std::unique_ptr<Collective> make_peer(int rank, int size, hipStream_t s);
// no exchange at all (diagnostics only: per-rank kernel time of a shard)
std::unique_ptr<Collective> make_null(int rank, int size);

}  // namespace llmi
