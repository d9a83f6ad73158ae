// k_exchange.hip -- the one-shot push all-gather of the row-sharded decode
// ("a one-shot P2P push over xGMI (fully connected 8 GPUs)
// with flag signaling"), the exchange behind collective.h's push variants.
//
// Every rank owns a mailbox on its own device: [2 halves][G sender slots][cap]
// granules of 8 B = {32-bit word, 32-bit tag} (common.h's data-tagged
// granule, here across devices).  An all-gather of `words` per rank:
//   push   -- the rank writes each word of its slice, tagged, into slot
//             [half][rank] of EVERY rank's mailbox (peers' through xGMI peer
//             mappings), one 8-byte system-scope store per word and peer: the
//             word and its flag arrive together, no fence, no flag word;
//   gather -- the rank re-loads its own mailbox's other slots until every
//             granule carries this exchange's tag and writes the words into
//             the destination buffer.
// tag = seed + the rank's exchange count (a device counter the last gathering
// work-group advances, so it lives inside the token's hipGraph); every rank
// makes the same exchanges in the same order, so the counts agree.  The seed
// is drawn per group lifetime (collective.cpp) so a mailbox whose memory held
// an earlier group's granules can never match them.  Halves alternate with the
// tag's parity: a rank can push exchange n + 1 while a slower peer still reads
// exchange n (other half), but not n + 2 -- that needs the slow peer's own
// n + 1 push, which comes after its n gather.
// Self-check: work-group b of every pusher also stores a checksum granule of
// its words (slot index cap + b); the gatherer's work-group b sums what it
// received from each peer the same way and compares, so a stale or torn slice
// raises an error (*err = 2) instead of passing wrong words on.
// The waits are bounded by wall-clock time (*err = 1; the session reports it
// at the next sync and refuses further work: the ranks' counts may differ).
#include "collective.h"
#include "common.h"

namespace llmi {

namespace {

constexpr int PX_T = 256;                          // threads per work-group
constexpr int PX_B = 4;                            // granules per thread per gather batch

__device__ __forceinline__ void px_store(uint2* g, uint32_t v, uint32_t tag) {
  __hip_atomic_store(reinterpret_cast<uint64_t*>(g), ((uint64_t)tag << 32) | v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t px_load(const uint2* g) {
  return __hip_atomic_load(reinterpret_cast<const uint64_t*>(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint32_t px_mix(uint32_t v, uint32_t idx) {  // order-free checksum term
  return (v ^ (idx * 0x9E3779B9u)) * 0x85EBCA6Bu + idx;
}

// work-group b handles words [b per, (b + 1) per) of every rank's slice
__global__ __launch_bounds__(PX_T) void push_exchange_kernel(PushArgs a) {
  __shared__ uint32_t s_tag;
  __shared__ uint32_t s_sum[PX_MAX_RANKS];
  const int t = threadIdx.x;
  if (t == 0) s_tag = __hip_atomic_load(a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u + (uint32_t)a.skip;
  if (t < PX_MAX_RANKS) s_sum[t] = 0;
  __syncthreads();
  const uint32_t tag = s_tag;
  const size_t half = tag & 1u;
  const size_t slot_w = (size_t)a.cap + PX_CS_RING * PX_MAX_CS;  // granules per sender slot: words, then checksums
  const size_t cs = px_cs((uint32_t)a.cap, tag);                  // this exchange's checksum region (px.h)
  const int per = (a.words + gridDim.x - 1) / gridDim.x;
  const int w0 = blockIdx.x * per, n = max(0, min(a.words, w0 + per) - w0);
  auto word = [&](int q, int i) -> uint32_t* {  // word i of this exchange in rank q's part of the buffer
    const size_t j = a.off + (size_t)i;
    return a.row_w ? a.buf + (j / a.row_w) * a.pitch + (size_t)q * a.row_w + j % a.row_w
                   : a.buf + (size_t)q * a.stride + j;
  };
  if (a.phase & PX_PUSH) {
    const size_t slot = (half * a.G + a.rank) * slot_w;
    uint32_t sum = 0;
    for (int i = t; i < n; i += PX_T) {
      const uint32_t v = *word(a.rank, w0 + i);
      sum += px_mix(v, (uint32_t)(w0 + i));
#pragma unroll 4
      for (int q = 0; q < a.G; q++) px_store(a.mail[q] + slot + w0 + i, v, tag);
    }
    atomicAdd(&s_sum[0], sum);
    __syncthreads();
    if (t < a.G) px_store(a.mail[t] + slot + cs + blockIdx.x, s_sum[0], tag);
    __syncthreads();
    if (t == 0) s_sum[0] = 0;
    __syncthreads();
  }
  if (a.phase & PX_GATHER) {
    // items (peer q != rank, word i) in batches of PX_B per thread: every load of a batch is issued before any
    // tag is checked, and only the granules still missing are re-loaded
    const int nq = a.G - 1, items = nq * n;
    const uint2* mine = a.mail[a.rank];
    const uint64_t t0 = wall_clock64();
    bool late = false;
    for (int j0 = t; j0 < items; j0 += PX_T * PX_B) {
      uint32_t* dst[PX_B];
      int qk[PX_B], ik[PX_B];
      const uint2* src[PX_B];
      uint64_t g[PX_B];
      bool ok[PX_B];
#pragma unroll
      for (int k = 0; k < PX_B; k++) {
        const int j = min(j0 + k * PX_T, items - 1);  // clamped: the tail repeats the last item
        const int qi = j / n, i = j % n, q = qi + (qi >= a.rank ? 1 : 0);
        qk[k] = q;
        ik[k] = w0 + i;
        src[k] = mine + (half * a.G + q) * slot_w + w0 + i;
        dst[k] = word(q, w0 + i);
        g[k] = px_load(src[k]);
      }
      for (;;) {
        bool all = true;
#pragma unroll
        for (int k = 0; k < PX_B; k++) {
          ok[k] = (uint32_t)(g[k] >> 32) == tag;
          all = all && ok[k];
        }
        if (all || late) break;
        if (wall_clock64() - t0 > a.timeout) {
          late = true;
          for (int k = PX_B - 1; k >= 0; k--)
            if (!ok[k]) {
              __hip_atomic_store(a.err + 1, (int)((uint32_t)(g[k] >> 32) - tag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              __hip_atomic_store(a.err + 2, ik[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              __hip_atomic_store(a.err + 3, (int)tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int k = 0; k < PX_B; k++)
          if (!ok[k]) g[k] = px_load(src[k]);
      }
#pragma unroll
      for (int k = 0; k < PX_B; k++)
        if (j0 + k * PX_T < items) {
          *dst[k] = (uint32_t)g[k];
          atomicAdd(&s_sum[qk[k]], px_mix((uint32_t)g[k], (uint32_t)ik[k]));
        }
    }
    __syncthreads();
    // every peer's checksum granule for this work-group's words
    if (t < a.G && t != a.rank && n > 0) {
      const uint2* csg = mine + (half * a.G + t) * slot_w + cs + blockIdx.x;
      uint64_t g = px_load(csg);
      while ((uint32_t)(g >> 32) != tag && !late) {
        if (wall_clock64() - t0 > a.timeout) {
          late = true;  // (diagnostics: word -1 - peer = that peer's checksum granule)
          __hip_atomic_store(a.err + 1, (int)((uint32_t)(g >> 32) - tag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(a.err + 2, -1 - t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(a.err + 3, (int)tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(a.err + 4, (int)(uint32_t)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(a.err + 5, (int)(half * 100000 + blockIdx.x * 1000 + gridDim.x), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        g = px_load(csg);
      }
      if (!late && (uint32_t)g != s_sum[t]) __hip_atomic_store(a.err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the last work-group to finish advances the exchange count (the next exchange's tag)
    __syncthreads();
    if (t == 0) {
      if (gridDim.x == 1) {
        __hip_atomic_store(a.epoch, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        const unsigned k = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (k == gridDim.x - 1) {
          __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(a.epoch, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }
}

}  // namespace

void launch_push_exchange(const PushArgs& a, hipStream_t s) {
  if (a.G < 1 || a.G > PX_MAX_RANKS || a.rank < 0 || a.rank >= a.G || a.words < 0 || a.words > a.cap ||
      (!a.row_w && a.off + (size_t)a.words > a.stride) || a.skip < 0 || a.row_w < 0)
    throw std::runtime_error("push exchange: bad arguments");
  if (a.words == 0) return;
  // one work-group per 256 words up to 64 (a 1 MB prefill chunk: 4096 words each) -- a few CUs' worth of
  // spinning waves, whatever the peers are running
  const int nwg = std::max(1, std::min(PX_MAX_WG, (a.words + PX_T - 1) / PX_T));
  hipLaunchKernelGGL(push_exchange_kernel, dim3(nwg), dim3(PX_T), 0, s, a);
  LLMI_HIP(hipGetLastError());
}

}  // namespace llmi
