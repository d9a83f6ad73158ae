// collective.cpp -- RCCL and single-device implementations of collective.h.
#include "collective.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <random>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "common.h"
#include "session_kernels.h"

namespace llmi {

#define LLMI_NCCL(call)                                                                           \
  do {                                                                                            \
    ncclResult_t r_ = (call);                                                                     \
    if (r_ != ncclSuccess) throw hip_error(std::string(#call) + ": " + ncclGetErrorString(r_)); \
  } while (0)

void Collective::fused_link(PxLink&) { throw std::runtime_error("fused exchange: not a push-exchange session"); }
void Collective::peer_handle(void*) const { throw std::runtime_error("peer handle: not a push-exchange (LLMI_TP_PEER) session"); }
void Collective::peer_connect(const void*) { throw std::runtime_error("peer connect: not a push-exchange (LLMI_TP_PEER) session"); }

void rccl_unique_id(void* out128) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId id;
  LLMI_NCCL(ncclGetUniqueId(&id));
  std::memcpy(out128, &id, sizeof(id));
}

namespace {

// The first tag of a push-exchange group's lifetime, in [1, 2^31): tags run seed, seed + 1, ... so a new group
// never matches granules an earlier group left at the same addresses (its memory may be a freed mailbox's, and
// round 3's one recorded wrong-logits failure of an 8-rank group on one GPU was consistent with exactly that: tags
// restarted at 1 for every group, so a stale line of the previous group's exchange n carried the new group's tag
// n).  Every rank of a group must use the same seed: a LocalGroup draws one; peer processes derive it from the
// exchanged handles (the same bytes on every rank).
uint32_t seed_from(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  return 1u + (uint32_t)(h % ((1ull << 31) - 1));
}

uint64_t px_timeout_ticks() {  // LLMI_PX_TIMEOUT_MS (default 10 s): the bound of every device-side wait
  double ms = 10000.0;
  if (const char* e = getenv("LLMI_PX_TIMEOUT_MS")) ms = std::max(1.0, atof(e));
  return (uint64_t)(ms * 1e5);  // 100 MHz wall clock
}

// One rank's side of the push exchange (k_exchange.hip): its mailbox of [2 halves][G slots][kCap + PX_MAX_WG]
// granules (words, then the per-work-group checksums), the peers' mailboxes as mapped into this process, and the
// exchange counter.  Messages longer than kCap words per rank go as consecutive exchanges of kCap-word chunks.
// The memory is uncached (fine-grained): the pushers' stores land in HBM and the gatherer's loads read HBM, whichever
// XCD (and so whichever L2) each work-group runs on -- the 8 XCDs' L2s are not coherent with each other, also
// inside one process on one device.
class Mailbox {
 public:
  static constexpr int kCap = (1 << 18) - PX_CS_RING * PX_MAX_CS;  // words per rank slot (~1 MB of payload): every decode exchange in one
  static constexpr size_t kSlot = (size_t)kCap + PX_CS_RING * PX_MAX_CS;  // words, then checksum granules (px.h)
  // zeroed on the owning session's stream and complete on return (a null-stream hipMemset is not ordered with the
  // session's non-blocking stream)
  Mailbox(int rank, int G, hipStream_t s) : rank_(rank), G_(G), timeout_(px_timeout_ticks()), s_(s) {
    if (G < 1 || G > PX_MAX_RANKS) throw std::runtime_error("push exchange: 1-16 ranks");
    if (rank < 0 || rank >= G) throw std::runtime_error("push exchange: rank out of range");
    // ONE uncached allocation, a whole number of 2 MiB: the exchange counter / error words in its first 4 KiB, the
    // mailbox after them.  (An uncached allocation of 16 MiB + 64 KiB held another buffer's bytes past its last 2 MiB
    // boundary -- sender 3's checksum granules of half 1, the mailbox's tail: 5 of 1,832 one-GPU 4-rank lifetimes,
    // 0 of 2,712 with the mailbox an exact 16 MiB; round 4's "foreign granule" sat at the same tail position of a
    // 16 MiB + 4 KiB mailbox.  DESIGN.md section 7.)
    const size_t bytes = (size_t)2 * G * kSlot * sizeof(uint2);
    constexpr size_t kHead = 4096, kAlign = (size_t)2 << 20;
    bytes_ = bytes;
    alloc_ = (kHead + bytes + kAlign - 1) / kAlign * kAlign;
    LLMI_HIP(hipExtMallocWithFlags(&base_, alloc_, hipDeviceMallocUncached));
    ctl_ = reinterpret_cast<unsigned*>(base_);
    mine_ = reinterpret_cast<uint2*>(reinterpret_cast<char*>(base_) + kHead);
    LLMI_HIP(hipMemsetAsync(base_, 0, kHead + bytes, s_));  // tag 0: nothing published (tags are >= 1)
    LLMI_HIP(hipStreamSynchronize(s_));
    peers_.assign(G, nullptr);
    peers_[rank] = mine_;
  }
  ~Mailbox() {
    for (int q = 0; q < G_; q++)
      if (q != rank_ && opened_ && opened_base_[q]) (void)hipIpcCloseMemHandle(opened_base_[q]);
    dev_free(base_);
  }
  // the group's first tag (before the first exchange: the counter is then at seed - 1)
  void seed(uint32_t first_tag) {
    const unsigned c = first_tag - 1u;
    LLMI_HIP(hipMemcpyAsync(ctl_, &c, sizeof(c), hipMemcpyHostToDevice, s_));
    LLMI_HIP(hipStreamSynchronize(s_));
    seeded_ = true;
  }
  uint2* mine() const { return mine_; }
  void set_peer(int q, uint2* p) { peers_[q] = p; }
  bool connected() const {
    if (!seeded_) return false;
    for (uint2* p : peers_)
      if (!p) return false;
    return true;
  }
  void handle(void* out) const {
    static_assert(sizeof(hipIpcMemHandle_t) <= PEER_HANDLE_BYTES, "IPC handle size");
    hipIpcMemHandle_t h;
    LLMI_HIP(hipIpcGetMemHandle(&h, base_));  // (the allocation's base; a peer adds the counter's 4 KiB)
    std::memset(out, 0, PEER_HANDLE_BYTES);
    std::memcpy(out, &h, sizeof(h));
  }
  void open(const void* handles) {
    for (int q = 0; q < G_; q++) {
      if (q == rank_) continue;
      hipIpcMemHandle_t h;
      std::memcpy(&h, static_cast<const char*>(handles) + (size_t)q * PEER_HANDLE_BYTES, sizeof(h));
      void* p = nullptr;
      LLMI_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      opened_base_[q] = p;
      peers_[q] = reinterpret_cast<uint2*>(static_cast<char*>(p) + 4096);
    }
    opened_ = true;
    // every rank hashes the same handle bytes: the same seed, unique to these allocations
    uint64_t h = 1469598103934665603ull;
    const unsigned char* b = static_cast<const unsigned char*>(handles);
    for (size_t i = 0; i < (size_t)G_ * PEER_HANDLE_BYTES; i++) h = (h ^ b[i]) * 1099511628211ull;
    seed(seed_from(h));
  }
  // the all-gather of `bytes` per rank at buf (rank q's slice at buf + q bytes), as `phase` launches
  void run(void* buf, size_t bytes, int phase, hipStream_t s, int skip) {
    for (size_t c = 0; c < chunks(bytes); c++) run_chunk(buf, bytes, c, phase, s, c == 0 ? skip : 0);
  }
  // column slices (Collective::all_gather_cols): `rows` rows of pitch bytes, rank q's slice of slice bytes each
  void run_cols(void* buf, size_t pitch, size_t slice, int rows, int phase, hipStream_t s, int skip) {
    for (size_t c = 0; c < chunks(slice * rows); c++)
      run_chunk(buf, slice * rows, c, phase, s, c == 0 ? skip : 0, pitch, slice);
  }
  // the mailboxes as the fused exchanges see them (px.h)
  void link(PxLink& l) const {
    if (!connected()) throw std::runtime_error("push exchange: peers not connected (llmi_session_peer_connect)");
    l = PxLink{};
    for (int q = 0; q < G_; q++) l.mail[q] = peers_[q];
    l.ctl = ctl_;
    l.err = reinterpret_cast<int*>(ctl_ + 2);
    l.timeout = timeout_;
    l.slot_w = (uint32_t)kSlot;
    l.cs0 = (uint32_t)kCap;
    l.rank = rank_;
    l.G = G_;
  }
  static constexpr int cap() { return kCap; }
  // a chunked message is a sequence of exchanges: the split (push / gather) caller needs them one at a time
  static size_t chunks(size_t bytes) { return (bytes / 4 + kCap - 1) / kCap; }
  // pitch / slice (bytes, column slices of rows) or 0 (the message contiguous per rank)
  void run_chunk(void* buf, size_t bytes, size_t c, int phase, hipStream_t s, int skip = 0, size_t pitch = 0,
                 size_t slice = 0) {
    if (!connected()) throw std::runtime_error("push exchange: peers not connected (llmi_session_peer_connect)");
    if (bytes % 4 || pitch % 4 || slice % 4) throw std::runtime_error("push exchange: bytes % 4 != 0");
    const size_t words = bytes / 4, off = c * kCap;
    PushArgs a{};
    for (int q = 0; q < G_; q++) a.mail[q] = peers_[q];
    a.buf = static_cast<uint32_t*>(buf);
    a.off = off;
    a.stride = words;
    a.pitch = pitch / 4;
    a.row_w = (int)(slice / 4);
    a.words = (int)std::min<size_t>(kCap, words - off);
    a.rank = rank_;
    a.G = G_;
    a.cap = kCap;
    a.phase = phase;
    a.epoch = ctl_;
    a.ticket = ctl_ + 1;
    a.err = reinterpret_cast<int*>(ctl_ + 2);
    a.timeout = timeout_;
    a.skip = skip;
    launch_push_exchange(a, s);
  }
  int failed() {  // reads and clears the device flag (callers have synchronised the stream)
    int e[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    LLMI_HIP(hipMemcpyAsync(e, ctl_ + 2, sizeof(e), hipMemcpyDeviceToHost, s_));
    LLMI_HIP(hipStreamSynchronize(s_));
    if (e[0]) {
      LLMI_HIP(hipMemsetAsync(ctl_ + 2, 0, sizeof(e), s_));
      LLMI_HIP(hipStreamSynchronize(s_));
      // a timed-out wait: the word it last saw (its tag relative to the expected one), kind and place
      detail_ = e[0] == 2 ? " [checksum mismatch, tag " + std::to_string((unsigned)e[3]) + " (consumer role " +
                                std::to_string(e[1] / 1000) + ", fused exchange " + std::to_string(e[1] % 1000) +
                                " of the step, work-group " + std::to_string(e[2]) + "): read " +
                                std::to_string((unsigned)e[4]) + ", pushed " + std::to_string((unsigned)e[5]) +
                                "; read again " + std::to_string((unsigned)e[6]) + ", granules of another tag: words " +
                                std::to_string(e[7] & 0xFFFF) + " checksums " + std::to_string(e[7] >> 16) +
                                "; first sender whose words and checksums differ " + std::to_string(e[10]) + "; " +
                                std::to_string(e[8]) + " checking work-groups failed, mask " + std::to_string(e[9]) +
                                "; a checksum granule of another tag: sender*10000+wg " + std::to_string(e[11]) +
                                " {tag " + std::to_string((unsigned)e[12]) + ", word " + std::to_string((unsigned)e[13]) +
                                "}]"
                          : std::string(e[0] == 3 ? " [fused" : " [standalone") + " exchange, tag " +
                                     std::to_string((unsigned)e[3]) + ", word " + std::to_string(e[2]) +
                                     " held tag " + (e[1] >= 0 ? "+" : "") + std::to_string(e[1]) + " word " +
                                     std::to_string((unsigned)e[4]) + " at " + std::to_string(e[5]) + "]";
    }
    return e[0];
  }
  const std::string& detail() const { return detail_; }
  // test hook (LLMI_PX_TEST_CORRUPT): in this rank's mailbox, word 0 of sender q's slot in the half holding the newer
  // exchange gets its low bit flipped, its tag kept (the consumer accepts it; the checksum must not)
  void corrupt_newest(int q) {
    uint64_t g[2];
    for (int h = 0; h < 2; h++)
      LLMI_HIP(hipMemcpyAsync(&g[h], mine_ + ((size_t)h * G_ + q) * kSlot, 8, hipMemcpyDeviceToHost, s_));
    LLMI_HIP(hipStreamSynchronize(s_));
    const int h = (uint32_t)(g[1] >> 32) > (uint32_t)(g[0] >> 32) ? 1 : 0;
    const uint64_t bad = g[h] ^ 1ull;
    fprintf(stderr, "[px test] rank %d: sender %d word 0, half 0 {tag %u, %08x}, half 1 {tag %u, %08x}: half %d altered\n",
            rank_, q, (unsigned)(g[0] >> 32), (unsigned)g[0], (unsigned)(g[1] >> 32), (unsigned)g[1], h);
    LLMI_HIP(hipMemcpyAsync(mine_ + ((size_t)h * G_ + q) * kSlot, &bad, 8, hipMemcpyHostToDevice, s_));
    LLMI_HIP(hipStreamSynchronize(s_));
  }

 private:
  int rank_, G_;
  uint64_t timeout_;
  hipStream_t s_;  // the owning session's stream
  size_t bytes_ = 0, alloc_ = 0;
  void* base_ = nullptr;  // the allocation: ctl_ at its start, then mine_
  void* opened_base_[PX_MAX_RANKS] = {};  // peers' allocations as IPC-mapped here
  bool seeded_ = false;
  uint2* mine_ = nullptr;
  unsigned* ctl_ = nullptr;  // [0] exchange count, [1] ticket, [2] error flag, [3..5] its diagnostics
  std::string detail_;
  std::vector<uint2*> peers_;
  bool opened_ = false;
};

// one process per GPU, the push exchange through IPC-mapped mailboxes
class PeerCollective : public Collective {
 public:
  PeerCollective(int rank, int size, hipStream_t s) : Collective(rank, size), mb_(rank, size, s) {}
  bool graph_safe() const override { return true; }
  int kind() const override { return EX_PUSH; }
  void all_gather(void* buf, size_t bytes, hipStream_t s, int skip) override {
    mb_.run(buf, bytes, PX_PUSH | PX_GATHER, s, skip);
  }
  bool all_gather_cols(void* buf, size_t pitch, size_t slice, int rows, hipStream_t s, int skip) override {
    mb_.run_cols(buf, pitch, slice, rows, PX_PUSH | PX_GATHER, s, skip);
    return true;
  }
  bool fused_capable() const override { return true; }
  void fused_link(PxLink& l) override { mb_.link(l); }
  int failed() override { return mb_.failed(); }
  std::string fail_detail() const override { return mb_.detail(); }
  void peer_handle(void* out) const override { mb_.handle(out); }
  void peer_connect(const void* handles) override { mb_.open(handles); }

 private:
  Mailbox mb_;
};

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
  int kind() const override { return EX_RCCL; }
  void all_gather(void* buf, size_t bytes, hipStream_t s, int) override {
    char* b = static_cast<char*>(buf);
    LLMI_NCCL(ncclAllGather(b + (size_t)rank_ * bytes, b, bytes, ncclUint8, comm_, s));
  }

 private:
  ncclComm_t comm_ = nullptr;
};

class LocalCollective : public Collective {
 public:
  LocalCollective(LocalGroup* g, int rank, hipStream_t s) : Collective(rank, g->n), g_(g) {
    const char* ex = getenv("LLMI_TP_EXCHANGE");
    push_ = !(ex && std::string(ex) == "copy");
    {
      std::lock_guard<std::mutex> lk(g->mu);
      if (rank < 0 || rank >= g->n || g->joined[rank])
        throw std::runtime_error("local group: bad rank, or the rank already joined this group (re-create the group)");
    }
    if (push_) {
      mb_.reset(new Mailbox(rank, g->n, s));
      mb_->seed(g->seed);
    }
    if (const char* d = getenv("LLMI_PX_TEST_DROP"))  // test hook: this rank skips its first push
      drop_ = atoi(d) == rank;
    if (const char* d = getenv("LLMI_PX_TEST_CORRUPT"))  // test hook: one received word altered, its tag kept
      corrupt_ = atoi(d) == rank;
    std::lock_guard<std::mutex> lk(g->mu);
    if (g->joined[rank]) throw std::runtime_error("local group: bad or duplicate rank");
    g->joined[rank] = true;
    if (push_) g->mail[rank] = mb_->mine();
    LLMI_HIP(hipEventCreateWithFlags(&g->ready[rank], hipEventDisableTiming));
    LLMI_HIP(hipEventCreateWithFlags(&g->done[rank], hipEventDisableTiming));
  }
  ~LocalCollective() override {
    std::lock_guard<std::mutex> lk(g_->mu);
    // joined[rank] stays set: a group's ranks join once (a rejoining rank's new mailbox would restart the group's
    // tags at its seed, so its tags would repeat within the group's lifetime: ADVICE r4)
    g_->mail[rank_] = nullptr;
    (void)hipEventDestroy(g_->ready[rank_]);
    (void)hipEventDestroy(g_->done[rank_]);
    g_->ready[rank_] = g_->done[rank_] = nullptr;
  }
  bool graph_safe() const override { return false; }
  int kind() const override { return push_ ? EX_PUSH : EX_COPY; }
  int failed() override { return push_ ? mb_->failed() : 0; }
  std::string fail_detail() const override { return push_ ? mb_->detail() : std::string(); }
  bool fused_capable() const override { return push_; }
  void fused_link(PxLink& l) override {
    if (!push_) Collective::fused_link(l);
    connect();
    mb_->link(l);
  }
  // every rank's producing launch has completed before any rank's consumer is enqueued (the ranks' streams share
  // the process's hardware queues: a consumer spinning ahead of a peer's producer could block it).  Host-side:
  // each rank drains its own stream, then the host barrier (with cross-stream event waits instead, the one-GPU
  // 4-rank repeat, scripts/dev/tp_repeat4.py, timed out about once in 15 runs)
  void fused_point(hipStream_t s) override {
    LLMI_HIP(hipStreamSynchronize(s));
    g_->barrier();
    if (corrupt_) {  // (test hook) the newest granule of the next peer's word 0: its word flipped, its tag kept
      corrupt_ = false;
      mb_->corrupt_newest((rank_ + 1) % size_);
    }
  }
  bool all_gather_cols(void* buf, size_t pitch, size_t slice, int rows, hipStream_t s, int skip) override {
    if (!push_) return false;
    push_gather(buf, slice * rows, s, skip, pitch, slice);
    return true;
  }
  void all_gather(void* buf, size_t bytes, hipStream_t s, int skip) override {
    if (push_) return push_gather(buf, bytes, s, skip);
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
  // push launch, host barrier, then the gather launch once every peer's push has run (the ranks' streams
  // share this process's hardware queues: a gather spinning ahead of a peer's push could block it)
  void connect() {  // first exchange: every rank has registered its mailbox
    if (mb_->connected()) return;
    g_->barrier();
    for (int q = 0; q < size_; q++) mb_->set_peer(q, g_->mail[q]);
  }
  void push_gather(void* buf, size_t bytes, hipStream_t s, int skip, size_t pitch = 0, size_t slice = 0) {
    LocalGroup& g = *g_;
    connect();
    for (size_t c = 0; c < Mailbox::chunks(bytes); c++) {
      const int sk = c == 0 ? skip : 0;
      if (drop_) drop_ = false;  // the test hook: the peers' gathers wait past their bound
      else mb_->run_chunk(buf, bytes, c, PX_PUSH, s, sk, pitch, slice);
      LLMI_HIP(hipStreamSynchronize(s));  // (as fused_point: every push done before any gather is enqueued)
      g.barrier();
      mb_->run_chunk(buf, bytes, c, PX_GATHER, s, sk, pitch, slice);
    }
  }

  LocalGroup* g_;
  bool push_ = true, drop_ = false, corrupt_ = false;
  std::unique_ptr<Mailbox> mb_;
};

// diagnostics (LLMI_TP_SOLO): one rank of a sharded group with the exchange
// left out, to time a rank's own kernels on a single GPU
class NullCollective : public Collective {
 public:
  using Collective::Collective;
  bool graph_safe() const override { return true; }
  int kind() const override { return EX_NONE; }
  void all_gather(void*, size_t, hipStream_t, int) override {}
};

}  // namespace

std::unique_ptr<Collective> make_null(int rank, int size) {
  return std::unique_ptr<Collective>(new NullCollective(rank, size));
}

LocalGroup::LocalGroup(int n_)
    : n(n_), joined(n_, false), bufs(n_, nullptr), ready(n_, nullptr), done(n_, nullptr), mail(n_, nullptr) {
  if (n_ < 1) throw std::runtime_error("local group: size < 1");
  static std::atomic<uint64_t> groups{0};
  std::random_device rd;
  seed = seed_from(((uint64_t)rd() << 32) ^ rd() ^ (++groups * 0x9E3779B97F4A7C15ull));
  if (const char* e = getenv("LLMI_PX_SEED")) {  // development: a fixed first tag, in [1, 2^31) (tag 0 = unwritten)
    const unsigned long v = strtoul(e, nullptr, 10);
    if (v < 1 || v >= (1ul << 31)) throw std::runtime_error("LLMI_PX_SEED must lie in [1, 2^31)");
    seed = (uint32_t)v;
  }
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
  static const int secs = getenv("LLMI_TP_BARRIER_S") ? std::max(1, atoi(getenv("LLMI_TP_BARRIER_S"))) : 120;
  if (!cv.wait_for(lk, std::chrono::seconds(secs), [&] { return gen != my; }))
    throw std::runtime_error("local group: barrier timeout (a rank stopped)");
}

std::unique_ptr<Collective> make_rccl(int rank, int size, const void* id128) {
  return std::unique_ptr<Collective>(new RcclCollective(rank, size, id128));
}

std::unique_ptr<Collective> make_local(LocalGroup* g, int rank, int size, hipStream_t s) {
  if (!g || size != g->n) throw std::runtime_error("local group: tp_size differs from the group's size");
  return std::unique_ptr<Collective>(new LocalCollective(g, rank, s));
}

std::unique_ptr<Collective> make_peer(int rank, int size, hipStream_t s) {
  return std::unique_ptr<Collective>(new PeerCollective(rank, size, s));
}

}  // namespace llmi
