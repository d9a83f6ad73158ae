// px.h -- the push exchange fused into the decode launches ("a one-shot P2P push over xGMI
// ... with flag signaling, fused into the GEMV epilogue").
//
// The standalone exchange (k_exchange.hip) is one launch between a producer and its consumer.  Fused, the
// producing launch's epilogue stores each output word, tagged, straight into slot [half][rank] of every rank's
// mailbox (its own included), and the consuming launch's prologue reads the whole vector from its own mailbox,
// re-loading each granule until it carries this exchange's tag -- no exchange launch, no launch boundary.
//
// Tags: a step's fused exchanges are numbered k = 0, 1, ... in recording order and use tag = *ctl + 1 + k,
// where *ctl (the mailbox's exchange count) is constant during the step; the next standalone exchange (the
// step's argmax keys, always last) takes tag = *ctl + 1 + (fused count) and leaves *ctl there, so the tags of
// consecutive exchanges stay consecutive and never repeat within a group's lifetime (seeded per group).
// Halves alternate with the tag's parity.  Safe reuse of a half (exchange n + 2 lands where n was read): every
// launch that reads exchange n pushes its words of n + 1 only after reading, and every word of n + 1 is read by
// every consumer of n + 1 -- so a rank pushing n + 2 has consumed n + 1 from all its peers, each of which had
// finished reading n.
//
// Self-check (round 5): every producing work-group also pushes ONE checksum granule -- the sum of
// px_term(word, rank, index) over the words it pushed -- at granule px_cs(tag) + its index of the slot, and the first
// PX_CHECK_WG work-groups of every consuming launch (at least one per XCD when work-groups are dealt round-robin)
// sum the same terms over every word they read and compare with the sum of all producers' checksum granules
// (px_in_nwg per rank): a stale, torn or foreign word sets *err = 2 (the session raises LLMI_E_HIP and refuses
// further work) instead of reaching the logits.
// The checksum granules are read LATER than the words: a verifying work-group checks them when it retires, after
// its launch has pushed its own words of exchange n + 1 -- so a peer may already have read n + 1 and pushed n + 2
// (ADVICE r5).  n + 2 shares n's half, so the checksums take a second ring level on the tag's next bit: n + 2's
// land beside n's, and n + 4 (their next user) needs this rank's push of n + 3, which only a later launch makes.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace llmi {

constexpr int PX_MAX_RANKS = 16;
constexpr int PX_MAX_CS = 1024;  // checksum granules per sender slot: producing work-groups of one exchange
constexpr int PX_CHECK_WG = 8;   // consuming work-groups per launch that verify the checksums
constexpr int PX_CS_RING = 2;    // checksum regions per half (selected by tag bit 1; see above)

// a rank's mailboxes as its launches see them (device-resident, one per session); an exchange is (k, ws): its
// number within the step and its words per rank (word W of the whole vector is rank W / ws's word W % ws)
struct PxLink {
  uint2* mail[PX_MAX_RANKS];  // every rank's mailbox [2][G][slot_w] granules, as mapped in this process
  const unsigned* ctl;        // the rank's exchange count (constant during a step)
  int* err;                   // 3: a fused wait timed out; err[1..3]: that word's tag - the expected one, its
                              // number in the whole vector (-1 - producer work-group: a checksum granule), the
                              // expected tag; 2: a checksum mismatch (err[3]: the tag, err[4]/[5]: read/expected sum)
  uint64_t timeout;           // bound of every wait, ticks of the 100 MHz wall clock
  uint32_t slot_w;            // granules per sender slot
  uint32_t cs0;               // first checksum granule of a slot (words [0, cs0), checksums [cs0, slot_w):
                              // PX_CS_RING regions of PX_MAX_CS)
  int rank, G;
};

// the checksum region of exchange `tag` within its half's slots (granule offset from the slot start)
__host__ __device__ __forceinline__ uint32_t px_cs(uint32_t cs0, uint32_t tag) {
  return cs0 + ((tag >> 1) & 1u) * (uint32_t)PX_MAX_CS;
}

#ifdef __HIPCC__
__device__ __forceinline__ uint32_t px_link_tag(const PxLink& l, int k) {
  return __hip_atomic_load(l.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u + (uint32_t)k;
}

// word w of this rank's slice -> every rank's mailbox (one 8-byte system-scope store each: word and tag together)
__device__ __forceinline__ void px_push_word(const PxLink& l, uint32_t tag, int w, uint32_t v) {
  const size_t slot = ((size_t)(tag & 1u) * l.G + l.rank) * l.slot_w + (size_t)w;
  const uint64_t g = ((uint64_t)tag << 32) | v;
  for (int q = 0; q < l.G; q++)
    __hip_atomic_store(reinterpret_cast<uint64_t*>(l.mail[q] + slot), g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// order-free checksum term of word w of rank q's slice (w < 2^24)
__device__ __forceinline__ uint32_t px_term(uint32_t v, int q, int w) {
  const uint32_t idx = (uint32_t)w | ((uint32_t)q << 24);
  return (v ^ (idx * 0x9E3779B9u)) * 0x85EBCA6Bu + idx;
}

__device__ __forceinline__ void px_timeout(const PxLink& l, uint32_t seen, uint32_t tag, int where) {
  __hip_atomic_store(l.err + 1, (int)(seen - tag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(l.err + 2, where, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(l.err + 3, (int)tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(l.err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// N (1 or 4) consecutive words W.. of the whole vector from this rank's mailbox (W % N == 0 and ws % N == 0, so
// they lie in one sender's slot); bounded: on timeout *err = 3 and the words are garbage (the grid drains).  count:
// add the words' checksum terms to cs (false for a clamped duplicate read)
template <int N>
__device__ __forceinline__ void px_read_words(const PxLink& l, uint32_t tag, int ws, int W, uint32_t (&v)[N],
                                              uint32_t& cs, bool count) {
  const int q = W / ws, w = W - q * ws;
  const uint64_t* g = reinterpret_cast<const uint64_t*>(l.mail[l.rank] + ((size_t)(tag & 1u) * l.G + q) * l.slot_w + w);
  uint64_t x[N];
#pragma unroll
  for (int i = 0; i < N; i++) x[i] = __hip_atomic_load(g + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  uint64_t t0 = 0;
  for (int n = 0;; n++) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < N; i++) ok = ok && (uint32_t)(x[i] >> 32) == tag;
    if (ok) break;
    if (n == 0) t0 = wall_clock64();
    else if (wall_clock64() - t0 > l.timeout) {
      int bad = 0;
#pragma unroll
      for (int i = N - 1; i >= 0; i--)
        if ((uint32_t)(x[i] >> 32) != tag) bad = i;
      px_timeout(l, (uint32_t)(x[bad] >> 32), tag, W + bad);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int i = 0; i < N; i++)
      if ((uint32_t)(x[i] >> 32) != tag) x[i] = __hip_atomic_load(g + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
#pragma unroll
  for (int i = 0; i < N; i++) {
    v[i] = (uint32_t)x[i];
    if (count) cs += px_term(v[i], q, w + i);
  }
}

__device__ __forceinline__ uint32_t px_wave_add(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// a work-group's sum of one value per thread (every thread of the work-group calls it; s: a zeroed LDS word whose
// zeroing a barrier has ordered before this call)
__device__ __forceinline__ uint32_t px_wg_add(uint32_t v, uint32_t* s) {
  v = px_wave_add(v);
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(s, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __syncthreads();
  return *s;
}

// producer: work-group bid's checksum granule (cs: this thread's terms) to every rank's mailbox
__device__ __forceinline__ void px_push_checksum(const PxLink& l, uint32_t tag, int bid, uint32_t cs, uint32_t* s) {
  const uint32_t tot = px_wg_add(cs, s);
  if ((int)threadIdx.x < l.G) {
    const size_t slot = ((size_t)(tag & 1u) * l.G + l.rank) * l.slot_w + px_cs(l.cs0, tag) + (size_t)bid;
    __hip_atomic_store(reinterpret_cast<uint64_t*>(l.mail[threadIdx.x] + slot), ((uint64_t)tag << 32) | tot,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// consumer: the terms of every word this work-group read (cs) against the nwg checksum granules of every rank
// (s: zeroed LDS words, as px_wg_add: s[0], s[1] the sums, s[2] the timeout flag, s[3..] diagnostics)
// (where: the consumer's role * 1000 + the exchange's number in the step, and its work-group: err[1] / err[2])
__device__ __forceinline__ void px_verify(const PxLink& l, uint32_t tag, int nwg, uint32_t cs, uint32_t* s, int where,
                                          int bid, int ws, int nwords) {
  const uint32_t got = px_wg_add(cs, s);
  uint32_t want = 0;
  const uint64_t t0 = wall_clock64();
  for (int i = threadIdx.x; i < l.G * nwg; i += blockDim.x) {
    const int q = i / nwg, b = i - q * nwg;
    const uint64_t* g = reinterpret_cast<const uint64_t*>(l.mail[l.rank] + ((size_t)(tag & 1u) * l.G + q) * l.slot_w +
                                                          px_cs(l.cs0, tag) + b);
    uint64_t x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    while ((uint32_t)(x >> 32) != tag) {
      if (wall_clock64() - t0 > l.timeout) {
        px_timeout(l, (uint32_t)(x >> 32), tag, -1 - b);
        __hip_atomic_store(s + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    want += (uint32_t)x;
  }
  want = px_wg_add(want, s + 1);  // (its barrier also orders the timeout flag)
  const bool timed_out = *(volatile uint32_t*)(s + 2) != 0u;  // reported as a timeout (err 3), not as a mismatch
  if (!timed_out && want != got) {  // (uniform, rare) diagnostics: the whole vector and the checksums read once more, per sender
    uint32_t* sg = s + 4;                 // [G] words' terms read again, per sender
    uint32_t* sw = s + 4 + PX_MAX_RANKS;  // [G] checksum granules read again, per sender
    uint32_t other = 0;
    for (int W = threadIdx.x; W < nwords; W += blockDim.x) {
      const int q = W / ws, w = W - q * ws;
      const uint64_t x = __hip_atomic_load(
          reinterpret_cast<const uint64_t*>(l.mail[l.rank] + ((size_t)(tag & 1u) * l.G + q) * l.slot_w + w),
          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_fetch_add(sg + q, px_term((uint32_t)x, q, w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      other += (uint32_t)(x >> 32) != tag ? 1u : 0u;
    }
    for (int i = threadIdx.x; i < l.G * nwg; i += blockDim.x) {
      const int q = i / nwg, b = i - q * nwg;
      const uint64_t x = __hip_atomic_load(
          reinterpret_cast<const uint64_t*>(l.mail[l.rank] + ((size_t)(tag & 1u) * l.G + q) * l.slot_w +
                                            px_cs(l.cs0, tag) + b),
          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_fetch_add(sw + q, (uint32_t)x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if ((uint32_t)(x >> 32) != tag) {
        other += 0x10000u;
        __hip_atomic_store(l.err + 11, q * 10000 + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(l.err + 12, (int)(uint32_t)(x >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(l.err + 13, (int)(uint32_t)x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    other = px_wg_add(other, s + 3);  // (its barrier also orders the per-sender sums)
    if (threadIdx.x == 0) {
      uint32_t again = 0;
      int bad = -1;
      for (int q = 0; q < l.G; q++) {
        again += sg[q];
        if (bad < 0 && sg[q] != sw[q]) bad = q;
      }
      __hip_atomic_store(l.err + 6, (int)again, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(l.err + 7, (int)other, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(l.err + 10, bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(l.err + 8, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_or(l.err + 9, 1 << (bid & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (threadIdx.x == 0 && !timed_out && want != got) {
    __hip_atomic_store(l.err + 1, where, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(l.err + 2, bid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(l.err + 3, (int)tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(l.err + 4, (int)got, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(l.err + 5, (int)want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(l.err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__device__ __forceinline__ float4 px_read_f4(const PxLink& l, uint32_t tag, int ws, int W, uint32_t& cs, bool count) {
  uint32_t v[4];
  px_read_words<4>(l, tag, ws, W, v, cs, count);
  return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}
#endif

}  // namespace llmi
