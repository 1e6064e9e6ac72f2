// gfx950 (CDNA4, wave64) kernels for fugu's query hot path: conjunctive
// posting-list intersection + BM25 + top-k.
//
// Pipeline per planned batch:
//   k_conj   one workgroup per work item = (query, group of 2048-posting
//            chunks of the query's lead list, the lowest-cost term).  Each
//            lane holds 8 lead candidates.  The other lists are probed in
//            tantivy's intersection order (query/intersection.rs: children
//            sorted by cost): a dense list through its rank words (presence
//            bits + rank), any other through the per-term doc -> position bucket
//            directory (one directory load, then a branchless search inside
//            the ~4-posting bucket), all 8 items in lockstep so their loads
//            overlap.  Posting scores are formed at query time from the
//            posting's tf and fieldnorm id (DevIndex::tfn) with the query's
//            BM25 weights, in tantivy's Bm25Weight f32 arithmetic (the statistics
//            of the moment: a commit re-scores nothing); before each probe a MaxScore
//            bound (partial score + the remaining lists' maxima) drops
//            candidates that cannot reach the query's threshold.  Survivors
//            are summed in tantivy's order (Intersection::score), compacted
//            with ballot + popcount into LDS, and cut to the work item's exact
//            top-k by an LDS radix select over a 64-bit (score, ~doc) key.  The
//            k-th key raises a per-query threshold (atomicMax) that later
//            chunks use to prune.
//   k_final  one workgroup per query: gathers the chunk hits >= the query's
//            final threshold, exact top-k select + bitonic sort, writes
//            (score, doc) in (score desc, doc asc) order
//            (collector/top_collector.rs ComparableDoc).
//   k_merge  cross-shard merge of gathered per-GPU top-k lists.
// No MFMA: integer/indexing work bound by memory (roofline in DESIGN.md).
#include <hip/hip_runtime.h>

#include "fg_internal.h"

namespace fg {
namespace {

constexpr uint32_t kInvalid = 0xFFFFFFFFu;

// Diagnostic builds (-DFG_DIAG) stamp per-workgroup phase times (s_memrealtime,
// 100 MHz) into DevPlan::diag; the product build compiles them out.
#ifdef FG_DIAG
#define FG_STAMP(base, slot, val)                                     \
  do {                                                                \
    if (threadIdx.x == 0 && pl.diag) pl.diag[(base) * kDiagPerWg + (slot)] = (val); \
  } while (0)
#define FG_NOW() __builtin_amdgcn_s_memrealtime()
#else
#define FG_STAMP(base, slot, val) do { } while (0)
#define FG_NOW() 0ull
#endif

__device__ inline uint32_t lane_id() { return threadIdx.x & 63; }

// A multi-snapshot plan's DevIndex of slot v (DevPlan::segs), read through the
// constant address space: the plan's tables never change during a launch, so
// the compiler may keep the fields in SGPRs or reload them like kernel arguments
typedef const __attribute__((address_space(4))) DevIndex ConstDevIndex;
__device__ inline DevIndex seg_index(const DevPlan& pl, uint32_t s) {
#if defined(__HIP_DEVICE_COMPILE__)
  return ((ConstDevIndex*)pl.segs)[s];
#else
  return pl.segs[s];  // the host pass only parses device code
#endif
}
__device__ inline uint32_t wave_id() { return threadIdx.x >> 6; }

// Upper bounds are compared after inflating by 2^-17 relative: a bound sums at
// most 16 clauses plus the facet maximum (17 non-negative addends), whose f32
// summation-order error is below 2 * 17 * 2^-24 < 2^-18 relative, so
// bound-based pruning never drops a doc whose exactly-summed score reaches the
// threshold.
__device__ inline float inflate_bound(float x) { return x * 1.00000762939453125f; }  // 1 + 2^-17

// The rank word of doc d for rank-kind slot `slot`: plain, or sparse (block
// entry, then the word: the zero word when the term has none of the word's docs).
__device__ inline uint64_t rank_word_of(const DevIndex& ix, uint32_t slot, uint32_t d) {
  if (slot <= ix.n_prank) return ix.rank[(size_t)(slot - 1) * ix.rank_words + rank_word(d)];
  return ix.srank_w[srank_index(ix.srank[(size_t)(slot - 1 - ix.n_prank) * ix.srank_blocks + srank_block(d)], d)];
}
// A term's rank-kind structure as one array indexed by d >> shift: the plain
// rank words (shift 5) or the sparse block entries (shift 10, then srank_index)
__device__ inline const uint64_t* rank_base(const DevIndex& ix, uint32_t slot, uint32_t& shift) {
  if (slot <= ix.n_prank) {
    shift = 5u;
    return ix.rank + (size_t)(slot - 1) * ix.rank_words;
  }
  shift = 10u;
  return ix.srank + (size_t)(slot - 1 - ix.n_prank) * ix.srank_blocks;
}

// ---------------------------------------------------------------- query-time BM25

// A posting's tf / fieldnorm payload: tfn (text) in the low half, tfn_name
// (name, when the snapshot has name postings) in the high half.
// kF (the plan's DevPlan::feat, a template argument of the search kernels): 0
// every snapshot's statistics are its build's: the build-time posting scores
// (psc, one load); kFQt: scores formed at query time from the payloads, with
// kFName (some snapshot has `name` postings) and kFEsc (some posting's tf byte
// escaped) in the full variant.  Three instantiations (0, kFQt, kFQt | kFName |
// kFEsc): the common ones carry no name or escape code and fit the kernels'
// register budgets (k_conj 128 VGPRs at 4 waves, k_disj 96 at 5).
constexpr uint32_t kFName = 1, kFEsc = 2, kFQt = 4;
template <uint32_t kF>
__device__ inline uint32_t tfn_load(const DevIndex& ix, uint64_t p) {
  uint32_t v = ix.tfn[p];
  if ((kF & kFName) && ix.tfn_name) v |= (uint32_t)ix.tfn_name[p] << 16;
  return v;
}
// The posting's score for a clause of weights (wt, wn): Should(text:t, name:t)
// summed from 0.0 (SumCombiner), each field's part tantivy's Bm25Weight::score
// (field_score).  ct / cn: the text / name tf caches (LDS or the plan's copy).
// tfn_score_fast takes the tf bytes as they are; a payload with an escaped tf
// byte (tfn_escaped: tf >= 255, rare) is then scored again by tfn_score with
// the posting's position, in a fix-up pass outside the hot loops' registers.
template <uint32_t kF>
__device__ inline float tfn_score_fast(uint32_t v, float wt, float wn, const float* ct, const float* cn) {
  const uint32_t tt = v & 0xFFu, tn = (kF & kFName) ? (v >> 16) & 0xFFu : 0u;
  float s = 0.0f;
  if (tt) s += field_score(tt, (v >> 8) & 0xFFu, wt, ct);
  if (tn) s += field_score(tn, v >> 24, wn, cn);
  return s;
}
template <uint32_t kF>
__device__ inline bool tfn_escaped(uint32_t v) {
  return (kF & kFEsc) && ((v & 0xFFu) == kTfEsc || ((v >> 16) & 0xFFu) == kTfEsc);
}
__device__ inline float tfn_score(const DevIndex& ix, uint64_t p, uint32_t v, float wt, float wn, const float* ct,
                                  const float* cn) {
  uint32_t tt = v & 0xFFu, tn = (v >> 16) & 0xFFu;
  if (tt == kTfEsc || tn == kTfEsc) {
    const uint32_t e = tf_escaped(ix.esc_pos, ix.esc_tf, ix.n_esc, p);
    if (tt == kTfEsc) tt = e & 0xFFFFu;
    if (tn == kTfEsc) tn = e >> 16;
  }
  float s = 0.0f;
  if (tt) s += field_score(tt, (v >> 8) & 0xFFu, wt, ct);
  if (tn) s += field_score(tn, v >> 24, wn, cn);
  return s;
}

// Upper bound of term t's score in doc d: the tile maximum (4096-doc tiles)
// when the term has one, else the maximum of d's directory bucket.
__device__ inline float term_bound(const DevIndex& ix, uint32_t meta, uint32_t toff, uint32_t dir_off, uint32_t d) {
  return toff != 0xFFFFFFFFu ? ix.tmax[toff + (d >> kDisjTileShift)] : ix.bmax[dir_off + (d >> (meta & 0xFFu))];
}

// Does term (meta, postings at base, directory at dir_off) hold doc d?  (MustNot probes)
__device__ inline bool term_has_doc(const DevIndex& ix, uint32_t meta, uint64_t base, uint32_t dir_off, uint32_t d) {
  const uint32_t slot = meta_slot(meta);
  if (slot) return (rank_word_of(ix, slot, d) >> (d & 31u)) & 1ull;
  const uint32_t* __restrict__ dir = ix.dir + dir_off;
  const uint32_t b = d >> (meta & 0xFFu);
  uint32_t lo = dir[b], hi = dir[b + 1];
  const uint32_t* __restrict__ di = ix.doc + base;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (di[mid] < d) lo = mid + 1; else hi = mid;
  }
  return lo < dir[b + 1] && di[lo] == d;
}

// Position of doc d in term t's list (kInvalid: absent), through its rank words
// or its directory: the escaped-tf path recomputes it instead of keeping every
// probe's position live through the payload loads (registers)
__device__ inline uint32_t posting_pos(const DevIndex& ix, uint32_t t, uint32_t d) {
  const uint32_t meta = ix.tmeta[t], slot = meta_slot(meta);
  if (slot) return rank_pos(rank_word_of(ix, slot, d), d);
  const uint32_t* __restrict__ dir = ix.dir + ix.dir_off[t];
  const uint32_t b = d >> (meta & 0xFFu);
  uint32_t lo = dir[b], hi = dir[b + 1];
  const uint32_t* __restrict__ di = ix.doc + ix.off[t];
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (di[mid] < d) lo = mid + 1; else hi = mid;
  }
  return lo < dir[b + 1] && di[lo] == d ? lo : kInvalid;
}

// DevPlan::pub_mask: a linked group's shared thresholds are published
// score-only (the lowest key with the score), so a doc of another shard or
// namespace with an equal score is never pruned (the merge breaks ties by
// shard); an unlinked plan publishes exact keys.

// Histogram bin of a hit key for query bins (lo, sh), or kQBins (not counted:
// below bin 0's edge).
__device__ inline uint32_t qbin(uint64_t key, uint32_t lo, uint32_t sh) {
  const uint32_t bits = (uint32_t)(key >> 32);
  if (bits < lo) return kQBins;
  return min((bits - lo) >> sh, kQBins - 1);
}

// ---------------------------------------------------------------- workgroup helpers
// Exclusive prefix over the workgroup of one u32 per thread (256 threads).
__device__ inline uint32_t block_exclusive_scan(uint32_t v, uint32_t* scratch /*[4]*/) {
  const uint32_t lane = lane_id(), w = wave_id();
  uint32_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
    if (lane >= (uint32_t)o) incl += y;
  }
  if (lane == 63) scratch[w] = incl;
  __syncthreads();
  uint32_t base = 0;
#pragma unroll
  for (uint32_t i = 0; i < kThreads / 64; ++i) base += i < w ? scratch[i] : 0u;
  __syncthreads();
  return base + incl - v;
}

// The running threshold of query q from its score histogram: the lower edge of
// the highest bin b with >= K counted docs in bins >= b (score-only key), or 0.
// Relaxed agent-scope loads (sc1): the bins only grow, so a stale bin can only
// lower the threshold.  Workgroup-uniform result; scratch[0..6] used.
__device__ uint64_t hist_threshold(const uint32_t* gh, uint32_t K, uint32_t lo, uint32_t sh, uint32_t* scratch) {
  static_assert(kQBins == 2 * kThreads, "two bins per thread");
  const uint32_t tid = threadIdx.x;
  const uint32_t b0 = kQBins - 1 - 2 * tid, b1 = b0 - 1;  // descending
  const uint32_t v0 = __hip_atomic_load(gh + b0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t v1 = __hip_atomic_load(gh + b1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tid == 0) scratch[5] = kQBins;
  const uint32_t before = block_exclusive_scan(v0 + v1, scratch);
  if (before < K && before + v0 >= K) scratch[5] = b0;
  else if (before + v0 < K && before + v0 + v1 >= K) scratch[5] = b1;
  __syncthreads();
  const uint32_t b = scratch[5];
  __syncthreads();
  return b < kQBins ? (uint64_t)(lo + (b << sh)) << 32 : 0ull;
}

constexpr uint64_t kScoreOnly = 0xFFFFFFFF00000000ull;  // a key's score bits (thresholds shared across shards)

// A threshold published for batch query ql goes, score-only, to the peer plans
// too (DevPlan::peer_thr; their histograms: hist_add / hist_add16)
__device__ inline void peer_thr_max(const DevPlan& pl, uint32_t ql, uint64_t key) {
  for (uint32_t i = 0; i < pl.n_peers; ++i)
    atomicMax(reinterpret_cast<unsigned long long*>(pl.peer_thr[i] + ql), (unsigned long long)(key & kScoreOnly));
}

// Add the LDS bins to the query's global histogram (and the peers', a pass
// each over the bins: one loop holding every peer's address took k_conj past
// its register budget) and clear them.
__device__ inline void hist_add(uint32_t* lh, uint32_t* gh, const DevPlan& pl, uint32_t ql) {
  for (uint32_t i = 0; i < pl.n_peers; ++i)
    for (uint32_t b = threadIdx.x; b < kQBins; b += kThreads)
      if (const uint32_t c = lh[b]) atomicAdd(pl.peer_hist[i] + (size_t)ql * kQBins + b, c);
  for (uint32_t b = threadIdx.x; b < kQBins; b += kThreads) {
    const uint32_t c = lh[b];
    if (c) {
      atomicAdd(&gh[b], c);
      lh[b] = 0;
    }
  }
}

// Append `key` (when keep) to an LDS list through one LDS atomic per wave.
__device__ inline void wave_append(bool keep, uint64_t key, uint64_t* list, uint32_t* count, uint32_t cap) {
  const uint32_t lane = lane_id();
  const unsigned long long bal = __ballot(keep);
  const uint32_t nw = (uint32_t)__popcll(bal);
  if (!nw) return;
  uint32_t base = 0;
  if (lane == 0) base = atomicAdd(count, nw);
  base = (uint32_t)__shfl((int)base, 0, 64);
  const uint32_t at = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
  if (keep && at < cap) list[at] = key;
}

// Exact k-th largest over a set of unique 64-bit keys (visited by `each`,
// which calls its argument once per key): returns T with exactly K keys >= T.
// Bits-wide radix digits from the top; stops as soon as the digit holding the
// K-th key is taken whole.  Requires more than K keys.
template <uint32_t Bits = kHistBits, class Each>
__device__ uint64_t select_kth(uint32_t K, uint32_t* hist, uint32_t* scratch, Each each) {
  constexpr uint32_t kBins = 1u << Bits;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = wave_id();
  // Skip the bits every key shares (scores of one query cluster: the sign,
  // exponent and top mantissa bits are mostly equal).  Digits then start at
  // the highest differing bit, which keeps the first histogram spread out
  // instead of funnelling every LDS atomic into one or two bins.
  uint64_t kor = 0, kand = ~0ull;
  each([&](uint64_t k) { kor |= k; kand &= k; });
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    kor |= (uint64_t)__shfl_xor((long long)kor, o, 64);
    kand &= (uint64_t)__shfl_xor((long long)kand, o, 64);
  }
  uint64_t* red = reinterpret_cast<uint64_t*>(hist);
  if (lane == 0) { red[2 * wv] = kor; red[2 * wv + 1] = kand; }
  __syncthreads();
  kor = 0;
  kand = ~0ull;
#pragma unroll
  for (uint32_t i = 0; i < kThreads / 64; ++i) { kor |= red[2 * i]; kand &= red[2 * i + 1]; }
  __syncthreads();
  const uint64_t diff = kor ^ kand;
  int top = diff ? 64 - __clzll((long long)diff) : 0;  // bits >= top are common to all keys
  uint64_t prefix = top >= 64 ? 0 : (kand & (~0ull << top));
  uint32_t need = K;
  while (top > 0) {
    const int width = top < (int)Bits ? top : (int)Bits;
    const int sh = top - width;
    for (uint32_t i = tid; i < kBins; i += kThreads) hist[i] = 0;
    __syncthreads();
    each([&](uint64_t k) {
      if (top >= 64 || (k >> top) == (prefix >> top)) atomicAdd(&hist[(uint32_t)(k >> sh) & ((1u << width) - 1)], 1u);
    });
    __syncthreads();
    // thread t owns digits [bins-1-D*t-(D-1), bins-1-D*t] in descending order
    constexpr uint32_t D = kBins / kThreads;
    static_assert(D * kThreads == kBins, "whole digits per thread");
    uint32_t local[D], s = 0;
#pragma unroll
    for (uint32_t i = 0; i < D; ++i) {
      local[i] = hist[kBins - 1 - (tid * D + i)];
      s += local[i];
    }
    const uint32_t before = block_exclusive_scan(s, scratch);
    if (before < need && before + s >= need) {
      uint32_t c = before;
#pragma unroll
      for (uint32_t i = 0; i < D; ++i) {
        if (c < need && c + local[i] >= need) {
          scratch[4] = kBins - 1 - (tid * D + i);
          scratch[5] = need - c;
          scratch[6] = local[i];
        }
        c += local[i];
      }
    }
    __syncthreads();
    const uint32_t digit = scratch[4], nd = scratch[5], cnt = scratch[6];
    __syncthreads();
    prefix |= (uint64_t)digit << sh;
    need = nd;
    if (cnt == need) break;  // every key of this digit is in: threshold exact
    top = sh;
  }
  return prefix;
}

// Bitonic sort (descending) of P keys in LDS, P a power of two.
__device__ void bitonic_sort_desc(uint64_t* s, uint32_t P) {
  for (uint32_t k = 2; k <= P; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < P; i += kThreads) {
        const uint32_t ixj = i ^ j;
        if (ixj > i) {
          const uint64_t a = s[i], b = s[ixj];
          const bool desc = (i & k) == 0;
          if ((a < b) == desc) { s[i] = b; s[ixj] = a; }
        }
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------- k_conj
// A work item is a group of consecutive chunks of one query's lead list.  The
// workgroup keeps a local top-k buffer in LDS across its chunks (tantivy's
// TopNComputer: append, truncate to the exact k-th when the buffer passes
// 2048 keys) and, once per chunk, publishes its k-th key to the query's
// threshold and reads the best one any workgroup has published.
#ifndef FG_TRUNC
#define FG_TRUNC 1024
#endif
#ifndef FG_WAVES
#define FG_WAVES 4  // tools/ab_variants.py: 3 -> 4 waves/SIMD took k_conj 3.18 -> 2.58 ms
#endif
constexpr uint32_t kTrunc = FG_TRUNC;           // truncate the local buffer past this (>= kMaxK)
constexpr uint32_t kBuf = kTrunc + kChunk;       // kept keys (<= kTrunc) + one chunk of hits
// Deferred probes (queries of >= 3 unfiltered lists): the candidates that pass
// the second list wait in an LDS queue, and the remaining lists are probed for
// the whole queue at once (flush_deferred) instead of per chunk for the few
// lanes still alive.  The queue fills the LDS left at 4 workgroups per CU.
#ifndef FG_DEFER
#define FG_DEFER 896
#endif
constexpr uint32_t kDeferCap = FG_DEFER;                                // entries (doc << 32 | partial score)
#ifndef FG_DEFER_FLUSH
#define FG_DEFER_FLUSH (FG_DEFER / 2)
#endif
constexpr uint32_t kDeferFlush = FG_DEFER_FLUSH;                        // flush once this full at a chunk end
constexpr uint32_t kDeferR = kDeferCap ? (kDeferCap + kThreads - 1) / kThreads : 1;  // entries per thread in a flush
constexpr uint64_t kDeferNone = ~0ull;                                  // a reserved slot left empty
static_assert(kTrunc + kDeferCap <= kBuf, "a flush after truncation must fit the key buffer");

struct ConjShared {
  alignas(16) uint64_t buf[kBuf];
  float cache[512];  // the snapshot's tf caches (text, then name): DevIndex::cache
  uint32_t hist[1u << kConjHistBits];
  uint32_t scratch[8];
  uint32_t n_buf;
  uint64_t thr;
  uint64_t dq[kDeferCap > 0 ? kDeferCap : 1];  // deferred candidates
  uint32_t n_dq;                               // slots reserved (may pass kDeferCap: the rest went inline)
#ifdef FG_DIAG
  unsigned long long dgc[8];  // candidates alive at: load, after the first bound, after probe i (1..5)
#endif
};

#ifdef FG_DIAG
#define FG_COUNT(slot, mask)                                                            \
  do {                                                                                  \
    uint32_t c_ = 0;                                                                    \
    _Pragma("unroll") for (uint32_t j_ = 0; j_ < kItems; ++j_) c_ += (uint32_t)__popcll(__ballot(((mask) >> j_) & 1u)); \
    if (lane == 0 && (slot) < 8) atomicAdd(&sh.dgc[(slot)], (unsigned long long)c_);  \
  } while (0)
#else
#define FG_COUNT(slot, mask) do { } while (0)
#endif

// Keep exactly the K largest of buf[0, n) at the front (n <= Cap); returns the K-th key.
template <uint32_t Cap, uint32_t Bits = kHistBits>
__device__ uint64_t truncate_keys(uint64_t* buf, uint32_t* n_buf, uint32_t* hist, uint32_t* scratch, uint32_t n,
                                  uint32_t K) {
  const uint32_t tid = threadIdx.x;
  const uint64_t T = select_kth<Bits>(K, hist, scratch, [&](auto&& f) {
    for (uint32_t i = tid; i < n; i += kThreads) f(buf[i]);
  });
  constexpr uint32_t R = Cap / kThreads;
  uint64_t v[R];
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) {
    const uint32_t i = r * kThreads + tid;
    v[r] = i < n ? buf[i] : 0;
  }
  __syncthreads();
  if (tid == 0) *n_buf = 0;
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) wave_append(r * kThreads + tid < n && v[r] >= T, v[r], buf, n_buf, Cap);
  __syncthreads();
  return T;  // keys are unique: exactly K kept
}

__device__ inline uint64_t truncate_topk(ConjShared& sh, uint32_t n, uint32_t K) {
  return truncate_keys<kBuf, kConjHistBits>(sh.buf, &sh.n_buf, sh.hist, sh.scratch, n, K);
}

// Append the kept keys of buf[0, n) that clear `cur` to query q's candidate list.
__device__ uint32_t flush_candidates(const DevPlan& pl, uint32_t q, const uint64_t* buf, uint32_t n, uint64_t cur,
                                     uint32_t* scratch) {
  const uint32_t tid = threadIdx.x;
  uint32_t mine = 0;
  for (uint32_t i = tid; i < n; i += kThreads) mine += buf[i] >= cur ? 1u : 0u;
  const uint32_t before = block_exclusive_scan(mine, scratch);
  if (tid == kThreads - 1) scratch[6] = before + mine;
  __syncthreads();
  const uint32_t total = scratch[6];
  if (total) {
    if (tid == 0) scratch[7] = atomicAdd(&pl.cand_cnt[q], total);
    __syncthreads();
    uint64_t* out = pl.cand_keys + pl.cand_off[q] + scratch[7];
    uint32_t at = before;
    for (uint32_t i = tid; i < n; i += kThreads) {
      const uint64_t k = buf[i];
      if (k >= cur) out[at++] = k;
    }
  }
  return total;
}

// Term ti's score at the doc of each live item (-1: the term is absent from
// it), through the term's rank words or its bucket directory, then the hits'
// tf / fieldnorm payloads and their query-time scores (weights wt / wn, caches
// ct / cn); the N items' loads are in flight together.
template <uint32_t N, uint32_t kF>
__device__ inline void probe_list(const DevIndex& ix, uint32_t ti, const uint32_t (&doc)[N], uint32_t live,
                                  float wt, float wn, const float* ct, const float* cn, float (&sc)[N]) {
  const uint32_t meta = ix.tmeta[ti];
  const uint32_t dslot = meta_slot(meta);
  const uint64_t bi = ix.off[ti];
  uint32_t pos[N];
  if (dslot) {
    // rank words: presence + rank in one 8-B load per item (all items'
    // loads in flight together; sparse ones: the block entries, then the
    // words), then the score (or payload) of the hits
    uint32_t sh;
    const uint64_t* __restrict__ rw = rank_base(ix, dslot, sh);
    uint64_t x[N];
#pragma unroll
    for (uint32_t j = 0; j < N; ++j) x[j] = (live & (1u << j)) ? rw[doc[j] >> sh] : 0ull;
    if (sh != 5u) {
#pragma unroll
      for (uint32_t j = 0; j < N; ++j) {
        x[j] = ix.srank_w[srank_index(x[j], doc[j])];
      }
    }
    if constexpr (!(kF & kFQt)) {  // the build-time scores: one load per hit
      const float* __restrict__ ps = ix.psc + bi;
#pragma unroll
      for (uint32_t j = 0; j < N; ++j) {
        const uint32_t p = rank_pos(x[j], doc[j]);
        sc[j] = p != kInvalid ? ps[p] : -1.0f;
      }
      return;
    }
#pragma unroll
    for (uint32_t j = 0; j < N; ++j) pos[j] = rank_pos(x[j], doc[j]);
  } else {
    const uint32_t B = meta & 0xFFu, S = (meta >> 8) & 0xFFu;
    const uint32_t* __restrict__ di = ix.doc + bi;
    const uint32_t* __restrict__ dir = ix.dir + ix.dir_off[ti];
    // bucket of each live item, then a branchless power-of-two search in it
    uint32_t hi[N];
#pragma unroll
    for (uint32_t j = 0; j < N; ++j) {
      pos[j] = 0;
      hi[j] = 0;
      if (live & (1u << j)) {
        const uint32_t b = doc[j] >> B;
        pos[j] = dir[b];
        hi[j] = dir[b + 1];
      }
    }
    for (uint32_t st = S; st > 0; --st) {
      const uint32_t half = 1u << (st - 1);
#pragma unroll
      for (uint32_t j = 0; j < N; ++j) {
        const uint32_t idx = pos[j] + half - 1;
        if ((live & (1u << j)) && idx < hi[j] && di[idx] < doc[j]) pos[j] += half;
      }
    }
    if constexpr (!(kF & kFQt)) {
#pragma unroll
      for (uint32_t j = 0; j < N; ++j) {
        sc[j] = -1.0f;
        if ((live & (1u << j)) && pos[j] < hi[j] && di[pos[j]] == doc[j]) sc[j] = ix.psc[bi + pos[j]];
      }
      return;
    }
#pragma unroll
    for (uint32_t j = 0; j < N; ++j)
      if (!((live & (1u << j)) && pos[j] < hi[j] && di[pos[j]] == doc[j])) pos[j] = kInvalid;
  }
  // the hits' payloads (a posting's is never 0: tf >= 1 in some field), then their
  // scores; an escaped tf finds its position again (posting_pos)
  uint32_t v[N];
#pragma unroll
  for (uint32_t j = 0; j < N; ++j) v[j] = pos[j] != kInvalid ? tfn_load<kF>(ix, bi + pos[j]) : 0u;
  uint32_t esc = 0;
#pragma unroll
  for (uint32_t j = 0; j < N; ++j) {
    sc[j] = v[j] ? tfn_score_fast<kF>(v[j], wt, wn, ct, cn) : -1.0f;
    esc |= (tfn_escaped<kF>(v[j]) ? 1u : 0u) << j;
  }
  if constexpr ((kF & kFEsc) != 0) if (__builtin_expect(esc != 0, 0)) {
#pragma unroll
    for (uint32_t j = 0; j < N; ++j)
      if ((esc >> j) & 1u) {
        const uint64_t p = bi + posting_pos(ix, ti, doc[j]);
        sc[j] = tfn_score(ix, p, ix.tfn[p] | (ix.tfn_name ? (uint32_t)ix.tfn_name[p] << 16 : 0u), wt, wn, ct, cn);
      }
  }
}

// Probe lists 2.. of the queue's nd deferred candidates (doc, left + right
// score), in intersection order with the MaxScore bound after each, and append
// the survivors' keys.  The sums are the ones the inline path forms:
// (left + right) + (0.0 + s_2 + ...).  Unfiltered queries only (no facet term).
template <uint32_t kF>
__device__ void flush_deferred(const DevIndex& ix, ConjShared& sh, const uint32_t* terms, const float* qwt,
                               const float* qwn, uint32_t m, const float* qub, uint64_t thr, uint32_t nd) {
  const uint32_t tid = threadIdx.x;
  uint32_t doc[kDeferR], live = 0;
  float s01[kDeferR], acc[kDeferR];
#pragma unroll
  for (uint32_t r = 0; r < kDeferR; ++r) {
    const uint32_t i = r * kThreads + tid;
    const uint64_t e = i < nd ? sh.dq[i] : kDeferNone;
    doc[r] = (uint32_t)(e >> 32);
    s01[r] = __uint_as_float((uint32_t)e);
    acc[r] = 0.0f;
    live |= (doc[r] != kInvalid ? 1u : 0u) << r;
  }
  for (uint32_t i = 2; i < m; ++i) {
    if (!__any(live != 0)) break;
    float sc[kDeferR];
    probe_list<kDeferR, kF>(ix, terms[i], doc, live, qwt[i], qwn[i], sh.cache, sh.cache + 256, sc);
#pragma unroll
    for (uint32_t r = 0; r < kDeferR; ++r) {
      if (sc[r] < 0.0f) live &= ~(1u << r);
      else acc[r] += sc[r];
    }
    if (thr != 0 && i + 1 < m) {
      const float ub = qub[i + 1];
#pragma unroll
      for (uint32_t r = 0; r < kDeferR; ++r)
        if ((live & (1u << r)) && make_key(inflate_bound(s01[r] + acc[r] + ub), doc[r]) < thr) live &= ~(1u << r);
    }
  }
#pragma unroll
  for (uint32_t r = 0; r < kDeferR; ++r) {
    bool keep = (live >> r) & 1u;
    uint64_t key = 0;
    if (keep && ix.alive && !((ix.alive[doc[r] >> 5] >> (doc[r] & 31)) & 1u)) keep = false;
    if (keep) {
      key = make_key(s01[r] + acc[r], doc[r]);
      keep = key >= thr;
    }
    wave_append(keep, key, sh.buf, &sh.n_buf, kBuf);
  }
}

// FG_WAVES: minimum waves per SIMD the register allocation must allow (the
// kernel is bound by memory latency, so occupancy is its main lever)
// kSingle: the instantiation for single-list queries runs work items
// [0, n_single) (no probes; block-max chunk skipping), the general one
// [n_single, total_chunks); separate launches keep the general kernel's
// register allocation.
// k_conj's running thresholds from the query's score histogram: every item
// counts its final kept keys (its local top-k) into the query's bins when it
// ends, and k_final reads the bins' threshold once per query -- the k-th best
// among all the query's items, where the threshold word carries the best
// single item's k-th key (items reading the bins themselves cost more than
// they pruned: profiles/r03/ab/ab_conj_hist.log).
// kMulti: a multi-snapshot plan (DevPlan::segs): the item's snapshot from its query slot
template <bool kSingle, bool kMulti, uint32_t kF>
__global__ __launch_bounds__(kThreads, FG_WAVES) void k_conj(DevIndex ix0, DevPlan pl) {
  __shared__ ConjShared sh;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = wave_id();

  // XCD-aware remap (bijective): each XCD runs a contiguous stretch of the
  // doc sweep, so its L2 holds one doc window of the hot lists.
  const uint32_t nwg = gridDim.x, bid = blockIdx.x;
  const uint32_t xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const uint32_t w = (kSingle ? 0u : pl.n_single) +
                     (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);

  uint64_t t_start = FG_NOW(), t_probe = 0, t_keys = 0, t_sel = 0, n_app = 0;
  (void)t_start; (void)t_probe; (void)t_keys; (void)t_sel; (void)n_app;
  const uint32_t q = pl.work_q[w];
  const DevIndex ix = kMulti ? seg_index(pl, __builtin_amdgcn_readfirstlane(q / pl.seg_nq)) : ix0;
  // the batch query (threshold, histogram); uniform, and kept in SGPRs (the
  // division runs on the VALU: without readfirstlane its pointers took VGPRs)
  const uint32_t ql = kMulti ? __builtin_amdgcn_readfirstlane(q % pl.seg_nq) : q;
  const uint32_t c0 = pl.work_c[w], nc = pl.work_n[w];
  // terms: [Must (cost order)][MustNot][Should]; a query with Should clauses is
  // Must-driven (RequiredOptionalScorer): the Shoulds only add score
  const uint32_t qmv = kSingle ? qm_pack(1, 1, 0) : pl.q_m[q];
  const uint32_t m = qm_terms(qmv), nm = qm_must(qmv), nmx = nm + qm_not(qmv);
  const bool has_opt = m > nmx;
  const uint32_t* terms = pl.q_terms + (size_t)q * kMaxTerms;
  const float* qub = pl.q_ub + (size_t)q * kMaxTerms;
  // the clauses' query-time BM25 weights (uniform: scalar loads)
  const float* qwt = pl.q_wt + (size_t)q * kMaxTerms;
  const float* qwn = pl.q_wn + (size_t)q * kMaxTerms;
  const uint32_t K = pl.k;
  const uint32_t t0 = terms[0];
  const uint64_t lead_base = ix.off[t0];
  const uint32_t lead_df = pl.q_lead_df[q];
  unsigned long long* gthr = reinterpret_cast<unsigned long long*>(&pl.thresh[ql]);
  // facet filter (uniform per work item): Bool[Must(text), Must(facet union)]
  const uint32_t fslot = pl.f.q_filter[q];
  const uint32_t* fmask = nullptr;
  uint32_t fshift = 0;
  const float* ftab = nullptr;
  float fmax = 0.0f;
  if (fslot != kInvalid) {
    fmask = pl.f.fmask + pl.f.f_woff[fslot];
    fshift = pl.f.f_shift[fslot];
    ftab = pl.f.f_tab + (size_t)fslot * 256;
    fmax = pl.f.f_max[fslot];
  }
  // Threshold exchange without a blocking round trip: thread 0's returning
  // atomicMax (served at the memory side, so it sees every XCD's publications;
  // a plain or sc1 load could hit a stale L2 line) is issued at the end of a
  // chunk and its result folded in at the start of the next one, after that
  // chunk's lead loads are in flight.  A stale threshold is still a valid lower
  // bound of the query's k-th key (values only grow), so pruning stays exact.
  // the plan's starting threshold (single-list queries: the term's K'-th best score)
  const uint64_t thr0 = pl.q_thr0[q];
  uint64_t pend = 0;
  uint32_t* const gh = pl.hist + (size_t)ql * kQBins;
  const uint32_t h_lo = pl.q_hlo[q], h_sh = pl.q_hsh[q];
  if (tid == 0) {
    sh.n_buf = 0;
    sh.n_dq = 0;
    sh.thr = thr0;
    pend = atomicMax(gthr, (unsigned long long)(thr0 & pl.pub_mask));
    peer_thr_max(pl, ql, thr0);
  }
  // query-time scores: the tf caches into LDS (read after the first chunk's barrier)
  if constexpr (kF & kFQt)
    for (uint32_t i = tid; i < ((kF & kFName) && ix.tfn_name ? 512u : 256u); i += kThreads) sh.cache[i] = ix.cache[i];
#ifdef FG_DIAG
  if (tid < 8) sh.dgc[tid] = 0;
#endif
  uint64_t local_T = 0;
  // block-max skip (single lists): a chunk whose largest score (+ the facet
  // maximum) cannot reach the threshold is not loaded.  thr_k is the threshold
  // as every thread last saw it (uniform), so the skip is uniform too.  The
  // build-time chunk maxima scale by the lead's bound factor (DevPlan::q_rup).
  const float* __restrict__ cmax = ix.cmax + ix.coff[t0];
  const float rup0 = pl.q_rup[(size_t)q * kMaxTerms];
  uint64_t thr_k = thr0;
  // pure conjunctions (the multi-snapshot instantiation too: without deferred
  // probes it fits 128 VGPRs with no scratch, but C4 ran 1.44 -> 1.57 ms,
  // profiles/r04/ab/ab_multi_defer_c4.log)
  const bool defer = !kSingle && kDeferCap > 0 && m >= 3 && nm == m && !fmask;

  for (uint32_t cc = 0; cc < nc; ++cc) {
    const uint32_t c = c0 + cc;
    uint64_t tp0 = FG_NOW(), tp1 = tp0;
    (void)tp0; (void)tp1;
    if (!kSingle || make_key(inflate_bound(cmax[c] * rup0 + fmax), 0u) >= thr_k) {
    const uint64_t base0 = lead_base + (uint64_t)c * kChunk;
    const uint32_t cnt = min(kChunk, lead_df - c * kChunk);
    // lead candidates: item j of lane l = wv*512 + j*64 + l (coalesced per j)
    uint32_t doc[kItems];
    float s0[kItems];
    uint32_t live = 0;
    {
      uint32_t tv[kItems];
#pragma unroll
      for (uint32_t j = 0; j < kItems; ++j) {
        const uint32_t idx = wv * kWaveSpan + j * 64 + lane;
        const bool in = idx < cnt;
        // predicated loads: tools/ab_variants.py measured clamped unconditional
        // loads (every lane issuing) slower here, 1.57 -> 2.05 ms
        doc[j] = in ? ix.doc[base0 + idx] : kInvalid;
        if constexpr (kF & kFQt) tv[j] = in ? tfn_load<kF>(ix, base0 + idx) : 0u;
        else s0[j] = in ? ix.psc[base0 + idx] : 0.0f;
        live |= (in ? 1u : 0u) << j;
      }
      if (tid == 0 && pend > sh.thr) sh.thr = pend;
      __syncthreads();
      // the lead postings' query-time scores (the caches now in LDS)
      const float w0t = qwt[0], w0n = qwn[0];
      uint32_t esc = 0;
#pragma unroll
      for (uint32_t j = 0; j < kItems && (kF & kFQt); ++j) {
        s0[j] = tv[j] ? tfn_score_fast<kF>(tv[j], w0t, w0n, sh.cache, sh.cache + 256) : 0.0f;
        esc |= (tfn_escaped<kF>(tv[j]) ? 1u : 0u) << j;
      }
      if constexpr ((kF & kFEsc) != 0) if (__builtin_expect(esc != 0, 0)) {
#pragma unroll
        for (uint32_t j = 0; j < kItems; ++j)
          if ((esc >> j) & 1u) {
            const uint64_t p = base0 + wv * kWaveSpan + j * 64 + lane;
            s0[j] = tfn_score(ix, p, tfn_load<kF>(ix, p), w0t, w0n, sh.cache, sh.cache + 256);
          }
      }
    }
    const uint64_t thr = sh.thr;
    thr_k = thr;
    // MaxScore (uniform): once the query has a threshold, a candidate whose
    // partial score plus the remaining lists' maxima cannot reach it is dropped
    // before the next probe.  Bounds are inflated by 2^-17 (inflate_bound).
    const bool prune = thr != 0 && m > 1;
    if (fmask) {
      // the facet mask: one L2-resident bit probe drops a candidate before any list probe
#pragma unroll
      for (uint32_t j = 0; j < kItems; ++j)
        if ((live & (1u << j)) && !filter_bits(fmask, fshift, doc[j])) live &= ~(1u << j);
    }
    FG_COUNT(0, live);
    if (!prune) FG_COUNT(7, live);  // candidates of chunks that start with no threshold
    if (prune) {
      const float ub = qub[1] + fmax;
#pragma unroll
      for (uint32_t j = 0; j < kItems; ++j)
        if ((live & (1u << j)) && make_key(inflate_bound(s0[j] + ub), doc[j]) < thr) live &= ~(1u << j);
    }
    FG_COUNT(1, live);
#ifdef FG_DIAG
    {
      // tile-bound headroom (slot 6): candidates alive after the first bound
      // that the other lists' 4096-doc tile maxima, in place of their global
      // maxima, would drop; slots 4-6 then no longer count probes
      uint32_t extra = 0;
      if (prune) {
#pragma unroll
        for (uint32_t j = 0; j < kItems; ++j) {
          if (!((live >> j) & 1u)) continue;
          float ub = fmax;
          for (uint32_t i = 1; i < m; ++i) {
            const uint32_t t = terms[i], to = ix.toff[t];
            ub += to != kInvalid ? ix.tmax[to + (doc[j] >> kDisjTileShift)] : ix.tmaxs[t];
          }
          if (make_key(inflate_bound(s0[j] + ub), doc[j]) < thr) ++extra;
        }
      }
      for (int o = 32; o > 0; o >>= 1) extra += (uint32_t)__shfl_xor((int)extra, o, 64);
      if (lane == 0) atomicAdd(&sh.dgc[6], (unsigned long long)extra);
    }
#endif

    // every list probed in intersection order; a candidate whose partial score
    // plus the remaining lists' maxima cannot reach the threshold is dropped
    // before the next probe
    // after the first probe s0[j] holds left + right (the first two lists' sum);
    // then the MustNot lists drop the docs they hold; before the first Should
    // list s0[j] takes the whole required score and acc_o[j] restarts as the
    // optional union's sum (0.0 + s_a + ... in clause order)
    float acc_o[kItems];
#pragma unroll
    for (uint32_t j = 0; j < kItems; ++j) acc_o[j] = 0.0f;
    for (uint32_t i = 1; i < m; ++i) {
      if (!__any(live != 0)) break;  // wave-uniform early exit
      if (i == nmx && nm > 1) {
#pragma unroll
        for (uint32_t j = 0; j < kItems; ++j) {
          s0[j] = s0[j] + acc_o[j];
          acc_o[j] = 0.0f;
        }
      }
      const uint32_t ti = terms[i];
      float sc[kItems];
      probe_list<kItems, kF>(ix, ti, doc, live, qwt[i], qwn[i], sh.cache, sh.cache + 256, sc);
      // Intersection::score = left + right + (0.0 + others...)
      if (i < nm) {
#pragma unroll
        for (uint32_t j = 0; j < kItems; ++j) {
          if (sc[j] < 0.0f) { live &= ~(1u << j); continue; }
          if (i == 1) s0[j] = s0[j] + sc[j]; else acc_o[j] += sc[j];
        }
      } else if (i < nmx) {
#pragma unroll
        for (uint32_t j = 0; j < kItems; ++j)
          if (sc[j] >= 0.0f) live &= ~(1u << j);  // Exclude
      } else {
#pragma unroll
        for (uint32_t j = 0; j < kItems; ++j)
          if (sc[j] >= 0.0f) acc_o[j] += sc[j];  // RequiredOptionalScorer's optional union
      }
      if (prune && i + 1 < m) {
        const float ub = qub[i + 1] + fmax;
#pragma unroll
        for (uint32_t j = 0; j < kItems; ++j)
          if ((live & (1u << j)) && make_key(inflate_bound(s0[j] + acc_o[j] + ub), doc[j]) < thr)
            live &= ~(1u << j);
      }
      if (i == 1 && defer) {
        // park this wave's survivors in the queue when they fit (slots reserved
        // with one LDS atomic); a wave that does not fit probes on inline
        uint32_t nw = 0;
#pragma unroll
        for (uint32_t j = 0; j < kItems; ++j) nw += (uint32_t)__popcll(__ballot((live >> j) & 1u));
        if (nw) {
          uint32_t base = 0;
          if (lane == 0) base = atomicAdd(&sh.n_dq, nw);
          base = (uint32_t)__shfl((int)base, 0, 64);
          if (base + nw <= kDeferCap) {
            uint32_t at = base;
#pragma unroll
            for (uint32_t j = 0; j < kItems; ++j) {
              const bool b = (live >> j) & 1u;
              const unsigned long long bal = __ballot(b);
              if (b)
                sh.dq[at + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] =
                    ((uint64_t)doc[j] << 32) | __float_as_uint(s0[j]);
              at += (uint32_t)__popcll(bal);
            }
            live = 0;
          } else {
            for (uint32_t x = base + lane; x < kDeferCap; x += 64) sh.dq[x] = kDeferNone;  // the part that fit
          }
        }
      }
      if (i <= 2) FG_COUNT(1 + i, live);
    }
    tp1 = FG_NOW();

    // survivors: tantivy's summation order, alive bitset, pruning threshold,
    // append to the local top-k buffer
#pragma unroll
    for (uint32_t j = 0; j < kItems; ++j) {
      bool keep = (live >> j) & 1u;
      uint64_t key = 0;
      if (keep && ix.alive && !((ix.alive[doc[j] >> 5] >> (doc[j] & 31)) & 1u)) keep = false;
      if (keep) {
        // one Must term = the union itself; with Shoulds s0 = req, acc_o = opt:
        // (0.0 + req) + opt
        float s = (nm == 1 && !has_opt) ? s0[j] : s0[j] + acc_o[j];
        // with a filter: Intersection(text, facet union) = text + facet (two children)
        if (fmask) s = s + ftab[filter_bits(fmask, fshift, doc[j])];
        key = make_key(s, doc[j]);
        keep = key >= thr;
      }
      wave_append(keep, key, sh.buf, &sh.n_buf, kBuf);
    }
    }  // block-max skip
    __syncthreads();
    uint32_t n = sh.n_buf;
    uint64_t tp2 = FG_NOW();
    (void)tp2;
    if (defer) {
      const uint32_t nd = min(sh.n_dq, kDeferCap);
      if (nd >= kDeferFlush || (cc + 1 == nc && nd > 0)) {
        if (n > kTrunc) {  // room for the flush's keys
          local_T = truncate_topk(sh, n, K);
          if (local_T > thr_k) thr_k = local_T;
        }
        flush_deferred<kF>(ix, sh, terms, qwt, qwn, m, qub, thr_k, nd);
        __syncthreads();
        n = sh.n_buf;
        if (tid == 0) sh.n_dq = 0;
      }
    }
    if (n > kTrunc || (cc + 1 == nc && n > K)) {
      local_T = truncate_topk(sh, n, K);
      if (local_T > thr_k) thr_k = local_T;
    }
    uint64_t tp3 = FG_NOW();
    (void)tp3;
#ifdef FG_DIAG
    t_probe += tp1 - tp0; t_keys += tp2 - tp1; t_sel += tp3 - tp2; n_app += n;
#endif
    // publish the local k-th key; its reply (the best published one) is read next chunk
    if (tid == 0) {
      if (local_T > sh.thr) sh.thr = local_T;
      pend = atomicMax(gthr, (unsigned long long)(local_T & pl.pub_mask));
    }
  }
  if (tid == 0 && pend > sh.thr) sh.thr = pend;
  // the peers get the item's threshold once, when it ends (inside the chunk loop
  // the publication cost k_conj a spilled register)
  if (tid == 0) peer_thr_max(pl, ql, sh.thr);
  __syncthreads();

  // write the kept keys that still clear the freshest threshold
  const uint32_t total = flush_candidates(pl, q, sh.buf, sh.n_buf, sh.thr, sh.scratch);
  (void)total;
  // count the item's kept keys (distinct docs of its own lead chunks) into the
  // query's bins, through LDS bins (sh.hist is free once the last select ran)
  {
    static_assert((1u << kConjHistBits) >= kQBins, "LDS bins");
    const uint32_t n = min(sh.n_buf, kBuf);
    for (uint32_t b = tid; b < kQBins; b += kThreads) sh.hist[b] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < n; i += kThreads) {
      const uint32_t b = qbin(sh.buf[i], h_lo, h_sh);
      if (b < kQBins) atomicAdd(&sh.hist[b], 1u);
    }
    __syncthreads();
    hist_add(sh.hist, gh, pl, ql);
  }
  FG_STAMP(w, 0, t_start);
  FG_STAMP(w, 1, t_probe);
  FG_STAMP(w, 2, t_keys);
  FG_STAMP(w, 3, t_sel);
  FG_STAMP(w, 4, FG_NOW());
  FG_STAMP(w, 5, n_app);
  FG_STAMP(w, 6, ((uint64_t)nc << 40) | ((uint64_t)m << 32) | q);
  FG_STAMP(w, 7, total);
#ifdef FG_DIAG
  __syncthreads();
  for (uint32_t i = 0; i < 8; ++i) FG_STAMP(w, 8 + i, sh.dgc[i]);
#endif
}

// ---------------------------------------------------------------- k_disj
// Pure disjunction `t1 t2 ...` (Should clauses; query/union + SumCombiner,
// boolean_weight.rs): score = 0.0 + s_1 + s_2 + ... over the clauses a doc
// matches, in clause order.  A work item is a run of <= 32 consecutive
// 4096-doc tiles of one query.
//   R. all (tile, clause) posting ranges and bounds at once, one thread per
//      pair: [lo, hi) from the bucket directory, the bound from the per-term
//      tile maxima (DevIndex::tmax) or the bucket maximum (bmax);
//   S. MaxScore split per tile (one thread per tile) against the query's
//      threshold: sorted by bound, the longest prefix of clauses whose summed
//      bound cannot reach it is non-essential (a doc matching only those cannot
//      enter the top-k); all clauses non-essential: the tile is skipped;
//   P. the essential clauses' postings of the tiles left are streamed as one
//      flat list, two per thread per pass of 512 (the next pass's loads in
//      flight through this one).  Bound 1: a posting of clause c at doc d
//      plus the other clauses' tile bounds must reach the threshold; the
//      survivors wait in an LDS queue, and once it holds a full pass bound 2
//      runs over it with every lane busy: every other clause at d in clause
//      order (its rank word and posting score, or its bucket maximum).  When
//      every other clause is dense the bound-2 sum IS the exact score (a hit
//      right there); otherwise the candidate is rescored by probing every
//      clause ((candidate, clause) pairs in parallel), summed in clause
//      order.  A doc found through several essential clauses is kept only
//      from the first of them that it matches, so keys stay unique;
//   then hits go through the same local top-k buffer / threshold publication
//   as k_conj, and k_final selects the query's top-k.
// Bounds are compared after inflating by 2^-17 relative, which covers any f32
// summation-order difference of <= 16 clauses plus the facet maximum
// (inflate_bound), so the pruning never drops a true top-k doc: results equal
// the exhaustive union.
constexpr uint32_t kTileShift = kDisjTileShift;
constexpr uint32_t kTile = 1u << kTileShift;   // docs per tile (LDS score array: 16 KB)
// k_disj shape knobs: fg_internal.h (FG_DISJ_ROUND / HBITS / WAVES / G)
constexpr uint32_t kRound = FG_DISJ_ROUND;     // postings / docs per pass
constexpr uint32_t kBufD = kTrunc + kRound;    // kept keys + one pass of hits
constexpr uint32_t kPairs = kRound;            // (candidate, clause) rescoring pairs per pass
constexpr uint32_t kQCap = 2 * kRound;         // the bound-2 queue: < one pass queued + one pass appended
constexpr uint32_t kDisjHistBits = FG_DISJ_HBITS;
constexpr uint32_t kMaxTiles = kDisjMaxGroup;  // tiles per work item
constexpr uint32_t kMaxSeg = kDisjMaxPairs;    // (tile, clause) pairs per work item (the planner's cap)
static_assert(kMaxSeg <= 2 * kThreads, "k_disj segment list: two (tile, clause) pairs per thread");
static_assert(kMaxTiles <= 255 && kMaxTerms <= 16, "seg_info packs (tile << 4) | clause; cand (tile << 8) | clause");

// Query-time scoring's LDS (kFQt plans only: a build-time-score plan's k_disj
// keeps the LDS of round 5 -- past ~31.9 KB a CU holds 4 k_disj workgroups
// instead of 5, ab_rsub_lds_cliff.log)
template <bool kQt>
struct DisjQt {
  float c_wt[kMaxTerms], c_wn[kMaxTerms];  // query-time BM25 weights (text, name)
  float cache[256];                        // the text field's tf cache (DevIndex::cache; name: from the plan)
};
template <>
struct DisjQt<false> {};

template <bool kQt>
struct DisjShared : DisjQt<kQt> {
  alignas(16) uint64_t buf[kBufD];
  struct {
    // P: postings past bound 1 waiting for bound 2, (score bits << 32) | (clause
    // << kRelBits) | (doc - the item's first doc); a flushed chunk's slots then
    // hold its rescoring candidates, (maybe-mask << kRelBits + 4) | (clause <<
    // kRelBits) | doc offset (kRelBits: 17 for 32-tile items)
    uint64_t q[kQCap];
    union {                        // never live together: rescoring, then the truncation after it
      float cs[kPairs];            // P: per-(candidate, clause) term scores
      uint32_t hist[1u << kDisjHistBits];  // truncate_keys' select bins
    };
    uint32_t seg_start[kMaxSeg];   // P: prefix of the essential segments' lengths
  } p;
  uint32_t scratch[8];
  // R: per (tile, clause) ranges and bounds, index t * m + i
  uint32_t r_lo[kMaxSeg];            // R: first posting of the pair (within the term's list)
  uint16_t r_n[kMaxSeg];             // R: its postings in the tile (<= 4096)
  float r_ub[kMaxSeg];
  uint16_t b_ess[kMaxTiles * 8];     // S: essential-clause mask per 512-doc block
  uint64_t r_sub[kMaxSeg];           // R: the pair's sub-tile maxima (DevIndex::tsub; ~0: the tile bound)
  uint16_t t_ess[kMaxTiles];         // essential-clause mask per tile (the union of its blocks')
  uint32_t t_post;                   // bit t: tile t's essential postings are streamed (else skipped)
  uint16_t seg_info[kMaxSeg];        // P: (tile << 4) | clause of each segment
  // per-clause constants of the work item's query
  uint32_t c_meta[kMaxTerms], c_dir[kMaxTerms];
  uint64_t c_base[kMaxTerms];
  float c_rup[kMaxTerms];            // bound factors (DevPlan::q_rup)
  uint32_t max_s, n_seg, n_post;
  uint32_t n_buf, n_cand;
  uint32_t n_q;                      // P: queued postings
  uint32_t n_cnt;                    // buf[0, n_cnt) are counted in the query's histogram
  uint32_t n_lh;                     // keys counted into lh since its last flush (< 2^16: u16 halves)
  uint64_t thr;
  // hits per score bin not yet added to the global histogram: two u16 bins per
  // word (bin b in the half b & 1), flushed before any half could pass 65535
  uint32_t lh[kQBins / 2];
};
static_assert(kMaxTiles <= 32, "DisjShared::t_post: one bit per tile");

// Add the packed LDS bins (DisjShared::lh) to the query's global histogram
// (and the peers') and clear them.
__device__ inline void hist_add16(uint32_t* lh, uint32_t* gh, const DevPlan& pl, uint32_t ql) {
  for (uint32_t i = 0; i < pl.n_peers; ++i) {  // (a pass per peer, as hist_add)
    uint32_t* ph = pl.peer_hist[i] + (size_t)ql * kQBins;
    for (uint32_t b = threadIdx.x; b < kQBins / 2; b += kThreads)
      if (const uint32_t c = lh[b]) {
        if (c & 0xFFFFu) atomicAdd(&ph[2 * b], c & 0xFFFFu);
        if (c >> 16) atomicAdd(&ph[2 * b + 1], c >> 16);
      }
  }
  for (uint32_t b = threadIdx.x; b < kQBins / 2; b += kThreads) {
    const uint32_t c = lh[b];
    if (c) {
      if (c & 0xFFFFu) atomicAdd(&gh[2 * b], c & 0xFFFFu);
      if (c >> 16) atomicAdd(&gh[2 * b + 1], c >> 16);
      lh[b] = 0;
    }
  }
}

__device__ inline bool doc_alive(const DevIndex& ix, uint32_t d) {
  return !ix.alive || ((ix.alive[d >> 5] >> (d & 31)) & 1u);
}

// a clause's bound over 512-doc block z of a tile: its sub-tile byte against the
// tile bound M (-0.0, no posting in the tile: stays -0.0, adds nothing)
__device__ inline float sub_bound(uint64_t sub, uint32_t z, float M) {
  return q8_bound((uint32_t)(sub >> (8 * z)) & 0xFFu, M);
}

// The query's score histogram (DevPlan::hist) and its bin geometry.
struct QHist {
  uint32_t* gh;
  uint32_t lo, sh;
  uint64_t pub;      // DevPlan::pub_mask
  uint32_t m, mq;    // MustNot clauses: c_meta[m, mq)
  const DevPlan* pl;  // its peers (DevPlan::peer_*)
  uint32_t ql;        // the batch query
};

// Keep the threshold fresh: drop the keys appended since the last call whose
// doc a MustNot clause holds (Exclude: the hit loops never probe them), count
// the rest into the LDS bins, truncate the local buffer to K when it passes
// `limit`, and (publish) exchange the threshold with the query's (possibly
// shared) threshold word.  A query's work items run about one after another
// (the doc sweep keeps ~one per query in flight), so the LDS bins join the
// query's histogram once, when the item ends.
template <class Sh>
__device__ inline void disj_truncate(const DevIndex& ix, Sh& sh, uint32_t K, uint32_t limit, uint64_t* gthr,
                                     bool publish, const QHist& hq, uint64_t& pend) {
  uint32_t n = sh.n_buf;
  __syncthreads();  // every thread has read n before anyone appends again
  if (hq.mq > hq.m) {
    constexpr uint32_t R = kBufD / kThreads;
    uint64_t v[R];
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
      const uint32_t i = sh.n_cnt + r * kThreads + threadIdx.x;
      v[r] = i < n ? sh.buf[i] : 0ull;
      if (v[r]) {
        const uint32_t d = key_doc(v[r]);
        for (uint32_t c = hq.m; c < hq.mq; ++c)
          if (term_has_doc(ix, sh.c_meta[c], sh.c_base[c], sh.c_dir[c], d)) { v[r] = 0; break; }
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) sh.n_buf = sh.n_cnt;
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) wave_append(v[r] != 0, v[r], sh.buf, &sh.n_buf, kBufD);
    __syncthreads();
    n = sh.n_buf;
  }
  if (sh.n_lh + (n - sh.n_cnt) > 0xFFFFu) {  // uniform (LDS after a barrier): a u16 bin could overflow
    hist_add16(sh.lh, hq.gh, *hq.pl, hq.ql);
    __syncthreads();
    if (threadIdx.x == 0) sh.n_lh = 0;
  }
  for (uint32_t i = sh.n_cnt + threadIdx.x; i < n; i += kThreads) {
    const uint32_t b = qbin(sh.buf[i], hq.lo, hq.sh);
    if (b < kQBins) atomicAdd(&sh.lh[b >> 1], 1u << (16 * (b & 1u)));
  }
  __syncthreads();
  uint64_t T = 0;
  if (n > limit) T = truncate_keys<kBufD, kDisjHistBits>(sh.buf, &sh.n_buf, sh.p.hist, sh.scratch, n, K);
  if (threadIdx.x == 0) {
    const uint64_t mine = T > sh.thr ? T : sh.thr;
    // the exchange does not wait: the returned best is folded in when the
    // next pass starts (pend), after that pass's posting loads are in flight
    if (publish) {
      pend = atomicMax(reinterpret_cast<unsigned long long*>(gthr), (unsigned long long)(mine & hq.pub));
      peer_thr_max(*hq.pl, hq.ql, mine);
    }
    sh.thr = mine;
    sh.n_lh += n - sh.n_cnt;
    sh.n_cnt = sh.n_buf;
  }
  __syncthreads();
}


template <bool kMulti, uint32_t kF>
__global__ __launch_bounds__(kThreads, FG_DISJ_WAVES) void k_disj(DevIndex ix0, DevPlan pl) {
  __shared__ DisjShared<(kF & kFQt) != 0> sh;
  const uint32_t tid = threadIdx.x;
  const uint32_t nwg = gridDim.x, bid = blockIdx.x;
  const uint32_t xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const uint32_t w = pl.n_conj + (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);

  const uint32_t q = pl.work_q[w];
  const DevIndex ix = kMulti ? seg_index(pl, __builtin_amdgcn_readfirstlane(q / pl.seg_nq)) : ix0;
  // the batch query (threshold, histogram); uniform, and kept in SGPRs (the
  // division runs on the VALU: without readfirstlane its pointers took VGPRs)
  const uint32_t ql = kMulti ? __builtin_amdgcn_readfirstlane(q % pl.seg_nq) : q;
  const uint32_t tile0 = pl.work_c[w], ntile = pl.work_n[w];
  // terms: [Should clauses (clause order)][MustNot]; m = the Should clauses
  const uint32_t qmv = pl.q_m[q];
  const uint32_t mq = qm_terms(qmv), m = mq - qm_not(qmv);
  const uint32_t* terms = pl.q_terms + (size_t)q * kMaxTerms;
  const uint32_t K = pl.k;
  uint64_t* gthr = &pl.thresh[ql];
  const QHist hq{pl.hist + (size_t)ql * kQBins, pl.q_hlo[q], pl.q_hsh[q], pl.pub_mask, m, mq, &pl, ql};
  uint64_t pend = 0;  // thread 0: the last threshold exchange's reply, not yet folded in

  // facet filter: the union is intersected with the facet union, score = union + facet;
  // every bound below adds the facet score's maximum fmax
  const uint32_t fslot = pl.f.q_filter[q];
  const uint32_t* fmask = nullptr;
  uint32_t fshift = 0;
  const float* ftab = nullptr;
  float fmax = 0.0f;
  if (fslot != kInvalid) {
    fmask = pl.f.fmask + pl.f.f_woff[fslot];
    fshift = pl.f.f_shift[fslot];
    ftab = pl.f.f_tab + (size_t)fslot * 256;
    fmax = pl.f.f_max[fslot];
  }
#ifdef FG_DIAG
  const uint64_t dg_t0 = FG_NOW();
  uint64_t dg_mode[3] = {0, 0, 0}, dg_post = 0, dg_cand = 0, dg_trunc = 0, dg_ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t dg_b1 = 0;  // postings past bound 1 (this thread's)
  uint64_t ph = dg_t0;
#define FG_PHASE(slot) do { const uint64_t n_ = FG_NOW(); dg_ph[slot] += n_ - ph; ph = n_; } while (0)
#else
#define FG_PHASE(slot) do { } while (0)
#endif
  if (tid == 0) {
    sh.n_buf = 0;
    sh.n_cnt = 0;
    sh.n_lh = 0;
    sh.t_post = 0;
    const uint64_t t0 = pl.q_thr0[q];
    const uint64_t g = atomicMax(reinterpret_cast<unsigned long long*>(gthr), (unsigned long long)t0);
    peer_thr_max(pl, ql, t0);
    sh.thr = g > t0 ? g : t0;
  }
  for (uint32_t b = tid; b < kQBins / 2; b += kThreads) sh.lh[b] = 0;
  if constexpr (kF & kFQt)
    for (uint32_t i = tid; i < 256; i += kThreads) sh.cache[i] = ix.cache[i];
  // the name field's tf cache stays in the plan's copy (global, L1 / L2-resident): LDS
  // past ~32 KB drops k_disj from 5 to 4 workgroups per CU
  const float* const cn = ix.cache + 256;
  if (tid < mq) {
    const uint32_t t = terms[tid];
    sh.c_meta[tid] = ix.tmeta[t];
    sh.c_dir[tid] = ix.dir_off[t];
    sh.c_base[tid] = ix.off[t];
    sh.c_rup[tid] = pl.q_rup[(size_t)q * kMaxTerms + tid];
    if constexpr (kF & kFQt) {
      sh.c_wt[tid] = pl.q_wt[(size_t)q * kMaxTerms + tid];
      sh.c_wn[tid] = pl.q_wn[(size_t)q * kMaxTerms + tid];
    }
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t ms = 0;
    for (uint32_t i = 0; i < m; ++i) ms = max(ms, (sh.c_meta[i] >> 8) & 0xFFu);
    sh.max_s = ms;
  }

  // ---- R: ranges and bounds of every (tile, clause) pair, one thread per pair
  const uint32_t npair = ntile * m;
  for (uint32_t p = tid; p < npair; p += kThreads) {
    const uint32_t t = p / m, i = p - t * m;
    const uint32_t tile = tile0 + t;
    const uint32_t d0 = tile << kTileShift, d1 = min(d0 + kTile, ix.n_docs);
    const uint32_t meta = sh.c_meta[i], B = meta & 0xFFu;
    const uint32_t* __restrict__ dir = ix.dir + sh.c_dir[i];
    uint32_t lo, hi;
    float ub;
    const uint32_t toff = ix.toff[terms[i]];  // (L1-resident: the query's few terms)
    if (B <= kTileShift && toff != kInvalid) {
      // the tile directory: adjacent entries (32 tiles of a clause per line)
      const uint32_t to = toff + tile;
      lo = ix.tdir[to];
      hi = ix.tdir[to + 1];
      ub = ix.tmax[to];
      sh.r_sub[p] = ix.tsub[to];
    } else if (B <= kTileShift) {
      lo = dir[d0 >> B];
      hi = dir[((d1 - 1) >> B) + 1];
      ub = ix.tmaxs[terms[i]];
    } else {
      // one bucket holds the tile: branchless searches for d0 and d1 inside it
      const uint32_t b = d0 >> B;
      const uint32_t p0 = dir[b], p1 = dir[b + 1];
      const uint32_t* __restrict__ di = ix.doc + sh.c_base[i];
      const uint32_t S = (meta >> 8) & 0xFFu;
      uint32_t a = p0, c = p0;
      for (uint32_t st = S; st > 0; --st) {
        const uint32_t half = 1u << (st - 1);
        const uint32_t ia = a + half - 1, ic = c + half - 1;
        if (ia < p1 && di[ia] < d0) a += half;
        if (ic < p1 && di[ic] < d1) c += half;
      }
      if (a < p1 && di[a] < d0) ++a;
      if (c < p1 && di[c] < d1) ++c;
      lo = a;
      hi = c;
      ub = ix.bmax[sh.c_dir[i] + b];
    }
    sh.r_lo[p] = lo;
    sh.r_n[p] = (uint16_t)(hi > lo ? hi - lo : 0u);
    // the build-time bound scaled to the query's statistics (q8_bound of tsub then
    // scales with it: DevPlan::q_rup carries a margin for the rounding)
    sh.r_ub[p] = lo < hi ? ub * sh.c_rup[i] : -0.0f;  // -0.0: no posting in the tile (a posting score may be +0.0)
    if (!(B <= kTileShift && toff != kInvalid)) sh.r_sub[p] = ~0ull;
  }
  {
    // the query's running threshold (every work item's counted hits so far)
    const uint64_t H = hist_threshold(hq.gh, K, hq.lo, hq.sh, sh.scratch);
    if (tid == 0 && H > sh.thr) sh.thr = H;
  }
  __syncthreads();
  FG_PHASE(0);

  // ---- S: MaxScore split per tile (one thread per tile)
  if (tid < ntile) {
    const uint32_t t = tid;
    const uint32_t d0 = (tile0 + t) << kTileShift;
    const uint64_t thr = sh.thr;
    const float* ub = sh.r_ub + t * m;
    uint32_t ord[kMaxTerms];
    for (uint32_t i = 0; i < m; ++i) {
      uint32_t j = i;
      const float v = ub[i];
      while (j > 0 && ub[ord[j - 1]] > v) { ord[j] = ord[j - 1]; --j; }
      ord[j] = i;
    }
    float s = 0.0f;
    uint32_t P = 0;
    for (; P < m; ++P) {
      const float s2 = s + ub[ord[P]];
      if (make_key(inflate_bound(s2 + fmax), d0) >= thr) break;
      s = s2;
    }
    uint32_t ess = 0, any = 0;
    for (uint32_t j = 0; j < m; ++j) {
      const uint32_t n = sh.r_n[t * m + ord[j]];
      if (j < P) continue;
      ess |= 1u << ord[j];
      any |= n ? 1u : 0u;
    }
    sh.t_ess[t] = (uint16_t)ess;
    if (P < m && any) atomicOr(&sh.t_post, 1u << t);
  }
  __syncthreads();
  static_assert(kMaxTiles * 8 <= kThreads, "one thread per (tile, block)");
  // per 512-doc block (one thread per (tile, block)): the tile's non-essential
  // clauses plus more of its essential ones, smallest tile bound first, while
  // their block bounds (DevIndex::tsub) stay below the threshold together.  A
  // doc of the block scoring >= the threshold matches a clause left essential
  // there, whose tile segment is streamed; a posting of a clause not essential
  // in its block is dropped once loaded.
  if (tid < ntile * 8) {
    const uint32_t t = tid >> 3, z = tid & 7u, tile = tile0 + t;
    const uint32_t d0 = tile << kTileShift;
    const uint64_t thr = sh.thr;
    const float* ub = sh.r_ub + t * m;
    const uint32_t ess = sh.t_ess[t];
    auto bound = [&](uint32_t i) { return sub_bound(sh.r_sub[t * m + i], z, ub[i]); };
    float sz = 0.0f;
    for (uint32_t i = 0; i < m; ++i)
      if (!((ess >> i) & 1u)) sz += bound(i);
    uint32_t ez = ess, left = ess;
    while (left) {
      uint32_t c = __builtin_ctz(left);  // the remaining essential clause of the smallest tile bound
      for (uint32_t r = left & (left - 1); r; r &= r - 1) {
        const uint32_t i = __builtin_ctz(r);
        if (ub[i] < ub[c]) c = i;
      }
      left &= ~(1u << c);
      const float s2 = sz + bound(c);
      if (make_key(inflate_bound(s2 + fmax), d0) >= thr) break;
      sz = s2;
      ez &= ~(1u << c);
    }
    sh.b_ess[tid] = (uint16_t)ez;
  }
  __syncthreads();
  FG_PHASE(1);
#ifdef FG_DIAG
  if (tid == 0)
    for (uint32_t t = 0; t < ntile; ++t) {
      dg_mode[((sh.t_post >> t) & 1u) ? 2 : 0]++;
      for (uint32_t i = 0; i < m; ++i)
        if (((sh.t_post >> t) & 1u) && ((sh.t_ess[t] >> i) & 1u)) dg_post += sh.r_n[t * m + i];
    }
#endif

  FG_PHASE(2);

  // ---- P: flat list of the essential clauses' segments of the streamed tiles,
  // (tile, clause) pairs in order, compacted by two workgroup prefix sums
  {
    uint32_t len[2], cnt = 0, tot = 0;
#pragma unroll
    for (uint32_t r = 0; r < 2; ++r) {
      const uint32_t p = 2 * tid + r;
      len[r] = 0;
      if (p < npair) {
        const uint32_t t = p / m, i = p - t * m;
        if (((sh.t_post >> t) & 1u) && ((sh.t_ess[t] >> i) & 1u)) {
          // the segment trimmed to the blocks where the clause is essential
          // (first to last; the bucket directory's entries at those block
          // boundaries, or the enclosing buckets' when a bucket spans blocks)
          uint32_t bm = 0;
          for (uint32_t z = 0; z < 8; ++z) bm |= ((uint32_t)(sh.b_ess[t * 8 + z] >> i) & 1u) << z;
          const uint32_t B = sh.c_meta[i] & 0xFFu;
          if (bm != 0xFFu && B <= kTileShift && sh.r_n[p]) {
            const uint32_t hi0 = sh.r_lo[p] + sh.r_n[p];
            uint32_t lo = sh.r_lo[p], hi = sh.r_lo[p];
            if (bm) {
              const uint32_t z0 = __builtin_ctz(bm), z1 = 31u - __builtin_clz(bm);
              const uint32_t d0 = (tile0 + t) << kTileShift;
              const uint32_t da = d0 + (z0 << kSubShift), db = min(d0 + ((z1 + 1) << kSubShift), ix.n_docs);
              if (da < db) {
                const uint32_t* __restrict__ dir = ix.dir + sh.c_dir[i];
                lo = max(lo, dir[da >> B]);
                hi = max(lo, min(hi0, dir[((db - 1) >> B) + 1]));
              }
            }
            sh.r_lo[p] = lo;
            sh.r_n[p] = (uint16_t)(hi - lo);
          }
          len[r] = sh.r_n[p];
        }
      }
      cnt += len[r] ? 1u : 0u;
      tot += len[r];
    }
    uint32_t sb = block_exclusive_scan(cnt, sh.scratch);
    uint32_t pb = block_exclusive_scan(tot, sh.scratch);
#pragma unroll
    for (uint32_t r = 0; r < 2; ++r) {
      if (!len[r]) continue;
      const uint32_t p = 2 * tid + r, t = p / m, i = p - t * m;
      sh.p.seg_start[sb] = pb;
      sh.seg_info[sb] = (uint16_t)((t << 4) | i);
      ++sb;
      pb += len[r];
    }
    if (tid == kThreads - 1) {
      sh.n_seg = sb;
      sh.n_post = pb;
    }
  }
  __syncthreads();
  const uint32_t n_seg = sh.n_seg, n_post = sh.n_post;
  FG_PHASE(3);
  // the J postings of a thread go through every step in lockstep, so their
  // loads (the posting, then each clause's rank word and score) overlap
  constexpr uint32_t J = kRound / kThreads;
  // posting e of the flat list: its (tile, clause) segment (the last
  // seg_start <= e, binary search in LDS) and its position in the postings
  auto locate = [&](uint32_t e, uint32_t& t, uint32_t& c) -> uint64_t {
    uint32_t lo = 0, hi = n_seg;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (sh.p.seg_start[mid] <= e) lo = mid; else hi = mid;
    }
    const uint32_t info = sh.seg_info[lo];
    t = info >> 4;
    c = info & 15u;
    return sh.c_base[c] + sh.r_lo[t * m + c] + (e - sh.p.seg_start[lo]);
  };
  // Deferred bound 2.  A pass loads kRound postings and applies bound 1 (LDS
  // only); the survivors wait in an LDS queue, and bound 2 + the rescoring run
  // once the queue holds a full pass (or the item ends): their dependent gather
  // chains then run with every lane busy, once per kRound survivors, instead of
  // once per pass for the fraction of its postings that pass bound 1.
  // the doc within the item in kRelBits, the clause in the next 4 bits, a
  // candidate's maybe-mask above them
  constexpr uint32_t kRelBits = 32 - __builtin_clz(kDisjMaxGroup * kTile - 1);
  constexpr uint32_t kRelMask = (1u << kRelBits) - 1u;
  static_assert(kRelBits + 4 <= 32 && kMaxTerms <= 16, "a queue entry: doc offset + clause in 32 bits");
  const uint32_t dbase = tile0 << kTileShift;
  if (tid == 0) sh.n_q = 0;
  __syncthreads();
  // the next pass's postings are loaded before this pass's bound 1, so they are
  // in flight through its queue append and any flush (bound 2) that follows
  // (the tf / fieldnorm payloads; their scores are formed when the pass starts)
  uint32_t npd[J], npcl[J], npv[J];
  auto load_pass = [&](uint32_t e1) {
#pragma unroll
    for (uint32_t j = 0; j < J; ++j) {
      const uint32_t e = e1 + j * kThreads + tid;
      npd[j] = dbase;
      npcl[j] = 0;
      npv[j] = 0;
      if (e < n_post) {
        uint32_t t;
        const uint64_t at = locate(e, t, npcl[j]);
        npd[j] = ix.doc[at];
        if constexpr (kF & kFQt) npv[j] = tfn_load<kF>(ix, at);
        else npv[j] = __float_as_uint(ix.psc[at]);
      }
    }
  };
  load_pass(0);
  for (uint32_t e0 = 0; e0 < n_post; e0 += kRound) {
    uint32_t pd[J], pcl[J];
    float ps[J];
    bool pk[J];
    uint32_t esc = 0;
#pragma unroll
    for (uint32_t j = 0; j < J; ++j) {
      const uint32_t e = e0 + j * kThreads + tid;
      pk[j] = e < n_post;
      pd[j] = npd[j];
      pcl[j] = npcl[j];
      // the posting's score: the build's, or formed at query time
      if constexpr (kF & kFQt) ps[j] = pk[j] ? tfn_score_fast<kF>(npv[j], sh.c_wt[pcl[j]], sh.c_wn[pcl[j]], sh.cache, cn) : 0.0f;
      else ps[j] = pk[j] ? __uint_as_float(npv[j]) : 0.0f;
      esc |= (pk[j] && tfn_escaped<kF>(npv[j]) ? 1u : 0u) << j;
    }
    if constexpr ((kF & kFEsc) != 0) if (__builtin_expect(esc != 0, 0)) {  // an escaped tf: its position from the segment list again
#pragma unroll
      for (uint32_t j = 0; j < J; ++j)
        if ((esc >> j) & 1u) {
          uint32_t t_, c_;
          const uint64_t at = locate(e0 + j * kThreads + tid, t_, c_);
          ps[j] = tfn_score(ix, at, npv[j], sh.c_wt[pcl[j]], sh.c_wn[pcl[j]], sh.cache, cn);
        }
    }
    if (e0 + kRound < n_post) load_pass(e0 + kRound);
    // with this pass's posting loads in flight: the last exchange's reply
    if (tid == 0 && pend > sh.thr) sh.thr = pend;
    __syncthreads();
    {
      const uint64_t thr = sh.thr;
#pragma unroll
      for (uint32_t j = 0; j < J; ++j) {
        if (pk[j]) {
          // bound 1: the other clauses' tile bounds (LDS) and the facet maximum
          const uint32_t t = (pd[j] - dbase) >> kTileShift;
          float ub = ps[j] + fmax;
          const uint32_t zz = ((pd[j] - dbase) >> kSubShift) & 7u;
          for (uint32_t i = 0; i < m; ++i)
            if (i != pcl[j]) ub += sub_bound(sh.r_sub[t * m + i], zz, sh.r_ub[t * m + i]);
          pk[j] = make_key(inflate_bound(ub), pd[j]) >= thr;
          pk[j] = pk[j] && ((sh.b_ess[(pd[j] - dbase) >> kSubShift] >> pcl[j]) & 1u);
          if (pk[j] && fmask) pk[j] = filter_bits(fmask, fshift, pd[j]) != 0;
#ifdef FG_DIAG
          dg_b1 += pk[j] ? 1u : 0u;
#endif
        }
        wave_append(pk[j], ((uint64_t)__float_as_uint(ps[j]) << 32) | (pcl[j] << kRelBits) | (pd[j] - dbase), sh.p.q,
                    &sh.n_q, kQCap);
      }
    }
    __syncthreads();
    FG_PHASE(4);
    const uint32_t nqd = sh.n_q;  // uniform
    const bool last = e0 + kRound >= n_post;
    if (nqd < kRound && !(last && nqd)) continue;
    // flush: bound 2 and the rescoring over the queue, kRound entries at a time
    uint32_t done = 0;
    while (nqd - done >= kRound || (last && done < nqd)) {
      const uint32_t cnt = min(kRound, nqd - done);
      uint64_t ent[J];
#pragma unroll
      for (uint32_t j = 0; j < J; ++j) {
        const uint32_t i = j * kThreads + tid;
        pk[j] = i < cnt;
        ent[j] = pk[j] ? sh.p.q[done + i] : 0ull;
      }
      if (tid == 0) {
        sh.n_cand = 0;
        if (pend > sh.thr) sh.thr = pend;
      }
      __syncthreads();  // the chunk is in registers before its slots take the candidates
      const uint64_t thr = sh.thr;
      uint32_t pt[J], ess[J];
#pragma unroll
      for (uint32_t j = 0; j < J; ++j) {
        const uint32_t rel = (uint32_t)ent[j] & kRelMask;
        pd[j] = dbase + rel;
        pcl[j] = ((uint32_t)ent[j] >> kRelBits) & 15u;
        ps[j] = __uint_as_float((uint32_t)(ent[j] >> 32));
        pt[j] = rel >> kTileShift;
        ess[j] = 0;
        if (!pk[j]) continue;
        // bound 1 again: the threshold may have risen since the posting was queued
        float ub = ps[j] + fmax;
        const uint32_t zz = (rel >> kSubShift) & 7u;
        for (uint32_t i = 0; i < m; ++i)
          if (i != pcl[j]) ub += sub_bound(sh.r_sub[pt[j] * m + i], zz, sh.r_ub[pt[j] * m + i]);
        pk[j] = make_key(inflate_bound(ub), pd[j]) >= thr;
        ess[j] = sh.b_ess[rel >> kSubShift];
      }
      // bound 2: every other clause at d, one clause at a time in clause order:
      // its rank word (presence bits + rank) and then the posting's query-time
      // score, or its bucket maximum (scaled; -0.0: empty bucket).  When every
      // other clause has rank words (or no posting in the tile) the clause-order
      // sum IS the doc's exact SumCombiner score: a hit right here.
      float sum[J];
      uint32_t maybe[J];  // clauses whose structure at d says they may match (the rest cannot)
      bool exact[J];
#pragma unroll
      for (uint32_t j = 0; j < J; ++j) {
        sum[j] = 0.0f;
        maybe[j] = 0;
        exact[j] = true;
      }
      constexpr uint32_t kAbsent = 0xBF800000u;  // -1.0f: the clause is not on the doc
      // G clauses per step (FG_DISJ_G): their rank-word / table / bucket loads of
      // all J postings in flight together, then their posting-score loads
      constexpr uint32_t G = FG_DISJ_G;
      for (uint32_t i0 = 0; i0 < m; i0 += G) {
        uint32_t y[G][J];
        uint32_t need = 0;  // bit g * J + j
        {
          uint64_t x[G][J];
#pragma unroll
          for (uint32_t g = 0; g < G; ++g) {
            const uint32_t i = i0 + g;
            const uint32_t meta = i < m ? sh.c_meta[i] : 0u;
            const uint32_t slot = meta_slot(meta);
            const bool rank = slot && meta_rank(meta);
            uint32_t rsh = 5u;
            const uint64_t* __restrict__ rw = rank ? rank_base(ix, slot, rsh) : nullptr;
#pragma unroll
            for (uint32_t j = 0; j < J; ++j) {
              x[g][j] = kAbsent;
              if (i < m && pk[j] && i != pcl[j] && !signbit(sh.r_ub[pt[j] * m + i])) {
                need |= 1u << (g * J + j);
                if (rank) x[g][j] = rw[pd[j] >> rsh];
                else x[g][j] = __float_as_uint(ix.bmax[sh.c_dir[i] + (pd[j] >> (meta & 0xFFu))] * sh.c_rup[i]);
              }
            }
          }
          // sparse rank clauses: from the block entries to the words
#pragma unroll
          for (uint32_t g = 0; g < G; ++g) {
            const uint32_t meta = i0 + g < m ? sh.c_meta[i0 + g] : 0u;
            if (!(meta_rank(meta) && meta_slot(meta) > ix.n_prank)) continue;
#pragma unroll
            for (uint32_t j = 0; j < J; ++j)
              if ((need >> (g * J + j)) & 1u) x[g][j] = ix.srank_w[srank_index(x[g][j], pd[j])];
          }
#pragma unroll
          for (uint32_t g = 0; g < G; ++g) {
            const uint32_t meta = i0 + g < m ? sh.c_meta[i0 + g] : 0u;
            const bool rank = meta_slot(meta) && meta_rank(meta);
#pragma unroll
            for (uint32_t j = 0; j < J; ++j) {
              if (!rank || !((need >> (g * J + j)) & 1u)) {
                y[g][j] = (uint32_t)x[g][j];
              } else {
                const uint32_t p = rank_pos(x[g][j], pd[j]);
                y[g][j] = p != kInvalid ? p : kAbsent;
              }
            }
          }
        }
#pragma unroll
        for (uint32_t g = 0; g < G; ++g) {
          const uint32_t meta = i0 + g < m ? sh.c_meta[i0 + g] : 0u;
          if (!(meta_slot(meta) && meta_rank(meta))) continue;
          const uint64_t cb = sh.c_base[i0 + g];
          if constexpr (!(kF & kFQt)) {  // the build-time scores
#pragma unroll
            for (uint32_t j = 0; j < J; ++j)
              if (((need >> (g * J + j)) & 1u) && y[g][j] < 0x80000000u) y[g][j] = __float_as_uint(ix.psc[cb + y[g][j]]);
          } else {
          // the rank hits' payloads (all in flight), then their query-time scores
          const float wt = sh.c_wt[i0 + g], wn = sh.c_wn[i0 + g];
          uint32_t v[J];
#pragma unroll
          for (uint32_t j = 0; j < J; ++j)
            v[j] = (((need >> (g * J + j)) & 1u) && y[g][j] < 0x80000000u) ? tfn_load<kF>(ix, cb + y[g][j]) : 0u;
          uint32_t esc = 0;
#pragma unroll
          for (uint32_t j = 0; j < J; ++j) {
            if (v[j]) y[g][j] = __float_as_uint(tfn_score_fast<kF>(v[j], wt, wn, sh.cache, cn));  // a hit (payloads != 0)
            esc |= (tfn_escaped<kF>(v[j]) ? 1u : 0u) << j;
          }
          if constexpr ((kF & kFEsc) != 0) if (__builtin_expect(esc != 0, 0)) {  // an escaped tf finds its position again
            const uint32_t ti = terms[i0 + g];
#pragma unroll
            for (uint32_t j = 0; j < J; ++j)
              if ((esc >> j) & 1u) y[g][j] = __float_as_uint(tfn_score(ix, cb + posting_pos(ix, ti, pd[j]), v[j], wt, wn,
                                                                       sh.cache, cn));
          }
          }  // query-time scores
        }
        // the clause-order sum (the own clause: the streamed posting's score)
#pragma unroll
        for (uint32_t g = 0; g < G; ++g) {
          const uint32_t i = i0 + g;
          if (i >= m) break;
          const uint32_t slot = meta_slot(sh.c_meta[i]);
#pragma unroll
          for (uint32_t j = 0; j < J; ++j) {
            if (!pk[j]) continue;
            float b = ps[j];
            if (i != pcl[j]) {
              if (!((need >> (g * J + j)) & 1u)) continue;
              b = __uint_as_float(y[g][j]);
              exact[j] = exact[j] && slot != 0;
              if (signbit(b)) continue;  // clause i cannot match d
              maybe[j] |= 1u << i;
            }
            sum[j] += b;
          }
        }
      }
#pragma unroll
      for (uint32_t j = 0; j < J; ++j) {
        bool keep = false, direct = false;
        uint64_t dkey = 0;
        if (pk[j]) {
          if (exact[j]) {
            // unique keys: the doc is kept only from the first essential clause it matches
            const uint32_t first = (uint32_t)__builtin_ctz((maybe[j] | (1u << pcl[j])) & ess[j]);
            const float s2 = fmask ? sum[j] + ftab[filter_bits(fmask, fshift, pd[j])] : sum[j];
            dkey = make_key(s2, pd[j]);
            direct = first == pcl[j] && dkey >= thr && doc_alive(ix, pd[j]);
          } else {
            keep = make_key(inflate_bound(sum[j] + fmax), pd[j]) >= thr && doc_alive(ix, pd[j]);
          }
        }
        wave_append(direct, dkey, sh.buf, &sh.n_buf, kBufD);
        wave_append(keep, ((uint64_t)maybe[j] << (kRelBits + 4)) | (pcl[j] << kRelBits) | (pd[j] - dbase),
                    sh.p.q + done, &sh.n_cand, cnt);
      }
      __syncthreads();
      FG_PHASE(5);
      const uint32_t nc = sh.n_cand;
#ifdef FG_DIAG
      dg_cand += nc;
#endif
      // exact rescoring: every (candidate, clause) pair the doc may match -- its
      // own clause included -- probed in parallel, summed in clause order
      const uint64_t* cq = sh.p.q + done;
      const uint32_t Q = kPairs / m;
      for (uint32_t c0 = 0; c0 < nc; c0 += Q) {
        const uint32_t nq_ = min(Q, nc - c0), np = nq_ * m;
        constexpr uint32_t R = kPairs / kThreads;
        uint32_t rd[R], pc[R], pos[R], hi[R];
        float pv[R];  // the clause's score at the candidate, -1 = absent
#pragma unroll
        for (uint32_t j = 0; j < R; ++j) {
          const uint32_t p = j * kThreads + tid;
          pc[j] = kInvalid;
          rd[j] = 0;
          pv[j] = -1.0f;
          pos[j] = 0;
          hi[j] = 0;
          if (p < np) {
            const uint64_t cv = cq[c0 + p / m];
            const uint32_t i = p % m, src = ((uint32_t)cv >> kRelBits) & 15u;
            rd[j] = dbase + ((uint32_t)cv & kRelMask);
            pc[j] = (i == src || ((uint32_t)(cv >> (kRelBits + 4)) >> i) & 1u) ? i : (0x80000000u | i);
          }
          if (!(pc[j] & 0x80000000u)) {
            const uint32_t meta = sh.c_meta[pc[j]];
            if (meta_slot(meta)) {
              pos[j] = rank_pos(rank_word_of(ix, meta_slot(meta), rd[j]), rd[j]);  // kInvalid: absent
              pc[j] |= 0x40000000u;  // resolved by its rank word
            } else {
              const uint32_t* __restrict__ dir = ix.dir + sh.c_dir[pc[j]];
              const uint32_t b = rd[j] >> (meta & 0xFFu);
              pos[j] = dir[b];
              hi[j] = dir[b + 1];
            }
          }
        }
        for (uint32_t st = sh.max_s; st > 0; --st) {
#pragma unroll
          for (uint32_t j = 0; j < R; ++j) {
            if (pc[j] & 0xC0000000u) continue;  // invalid or resolved
            if (st > ((sh.c_meta[pc[j]] >> 8) & 0xFFu)) continue;
            const uint32_t half = 1u << (st - 1);
            const uint32_t idx = pos[j] + half - 1;
            if (idx < hi[j] && ix.doc[sh.c_base[pc[j]] + idx] < rd[j]) pos[j] += half;
          }
        }
        // the found postings' scores: the build's, or their payloads (all in flight)
        // and then their query-time scores
        uint32_t pvv[R];
#pragma unroll
        for (uint32_t j = 0; j < R; ++j) {
          const uint32_t ci = pc[j] & 15u;
          const uint64_t base = sh.c_base[ci];
          bool hit = false;
          if (!(pc[j] & 0x80000000u))
            hit = (pc[j] & 0x40000000u) ? pos[j] != kInvalid : pos[j] < hi[j] && ix.doc[base + pos[j]] == rd[j];
          if constexpr (kF & kFQt) pvv[j] = hit ? tfn_load<kF>(ix, base + pos[j]) : 0u;
          else if (hit) pv[j] = ix.psc[base + pos[j]];
        }
        uint32_t esc = 0;
        if constexpr ((kF & kFQt) != 0) {
#pragma unroll
          for (uint32_t j = 0; j < R; ++j) {
            const uint32_t ci = pc[j] & 15u;
            if (pvv[j]) pv[j] = tfn_score_fast<kF>(pvv[j], sh.c_wt[ci], sh.c_wn[ci], sh.cache, cn);  // a hit
            esc |= (tfn_escaped<kF>(pvv[j]) ? 1u : 0u) << j;
          }
        }
        if constexpr ((kF & kFEsc) != 0) if (__builtin_expect(esc != 0, 0)) {  // an escaped tf finds its position again
#pragma unroll
          for (uint32_t j = 0; j < R; ++j)
            if ((esc >> j) & 1u) {
              const uint32_t ci = pc[j] & 15u;
              pv[j] = tfn_score(ix, sh.c_base[ci] + posting_pos(ix, terms[ci], rd[j]), pvv[j], sh.c_wt[ci], sh.c_wn[ci],
                                sh.cache, cn);
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < R; ++j) {
          const uint32_t p = j * kThreads + tid;
          if (p < np) sh.p.cs[p] = pv[j];
        }
        __syncthreads();
        for (uint32_t cc0 = 0; cc0 < nq_; cc0 += kThreads) {
          const uint32_t cc = cc0 + tid;
          uint64_t key = 0;
          bool keep = cc < nq_;
          if (keep) {
            const uint64_t cv = cq[c0 + cc];
            const uint32_t rel = (uint32_t)cv & kRelMask, src = ((uint32_t)cv >> kRelBits) & 15u;
            const uint32_t d = dbase + rel;
            float sc = 0.0f;  // SumCombiner from 0.0 in clause order over the matching clauses
            uint32_t matched = 0;
            for (uint32_t i = 0; i < m; ++i) {
              const float v = sh.p.cs[cc * m + i];
              if (v >= 0.0f) {
                sc += v;
                matched |= 1u << i;
              }
            }
            // unique keys: keep the doc only from the first essential clause it matches
            const uint32_t first = (uint32_t)__builtin_ctz(matched & sh.b_ess[rel >> kSubShift]);
            if (fmask) sc = sc + ftab[filter_bits(fmask, fshift, d)];
            key = make_key(sc, d);
            keep = first == src && key >= thr;
          }
          wave_append(keep, key, sh.buf, &sh.n_buf, kBufD);
        }
        __syncthreads();
      }
      FG_PHASE(6);
#ifdef FG_DIAG
      if (sh.n_buf > K) dg_trunc++;
#endif
      disj_truncate(ix, sh, K, K, gthr, true, hq, pend);
      done += cnt;
    }
    // the rest of the queue (< kRound entries, behind the flushed chunks) moves to the front
    const uint32_t rem = nqd - done;
    for (uint32_t i = tid; i < rem; i += kThreads) sh.p.q[i] = sh.p.q[done + i];
    if (tid == 0) sh.n_q = rem;
    __syncthreads();
  }
  // the item's counted hits join the query's histogram (every key was counted
  // by the last disj_truncate)
  hist_add16(sh.lh, hq.gh, pl, ql);
  if (tid == 0 && pend > sh.thr) sh.thr = pend;
  __syncthreads();
  flush_candidates(pl, q, sh.buf, sh.n_buf, sh.thr, sh.scratch);
  FG_PHASE(7);
#ifdef FG_DIAG
  FG_STAMP(w, 0, dg_t0);
  FG_STAMP(w, 1, FG_NOW());
  FG_STAMP(w, 2, dg_mode[0]);
  FG_STAMP(w, 3, dg_mode[1]);
  FG_STAMP(w, 4, dg_mode[2]);
  FG_STAMP(w, 5, dg_post);
  {
    // postings past bound 1, summed over the workgroup (scratch is free after the flush)
    __syncthreads();
    if (tid == 0) sh.scratch[0] = 0;
    __syncthreads();
    atomicAdd(&sh.scratch[0], (uint32_t)dg_b1);
    __syncthreads();
    FG_STAMP(w, 6, ((uint64_t)sh.scratch[0] << 32) | (dg_cand & 0xFFFFFFFFull));
  }
  FG_STAMP(w, 7, (dg_trunc << 32) | q);
  for (uint32_t i = 0; i < 8; ++i) FG_STAMP(w, 8 + i, dg_ph[i]);
#endif
#undef FG_PHASE
}

// ---------------------------------------------------------------- k_fmask
// Facet masks of a batch's filters (DevFilters): one workgroup per 8192
// postings of one (filter, clause) facet list sets clause bit i of every doc
// in it.  Postings ascend, so the lanes of a wave mostly hit the same or
// neighbouring mask words: the atomics coalesce in L2.
template <bool kMulti>
__global__ __launch_bounds__(kThreads) void k_fmask(DevIndex ix0, DevPlan pl) {
  const uint32_t c = blockIdx.x;
  const uint32_t f = pl.f.ch_filter[c], i = pl.f.ch_clause[c], t = pl.f.ch_term[c], st = pl.f.ch_start[c];
  const DevIndex ix = kMulti ? seg_index(pl, pl.f.f_seg[f]) : ix0;
  const uint64_t b0 = ix.foff[t];
  const uint32_t n = (uint32_t)(ix.foff[t + 1] - b0);
  const uint32_t end = min(n, st + kFmaskChunk);
  const uint32_t sh = pl.f.f_shift[f];
  uint32_t* mask = pl.f.fmask + pl.f.f_woff[f];
  for (uint32_t p = st + threadIdx.x; p < end; p += kThreads) {
    const uint32_t bit = (ix.fdoc[b0 + p] << sh) + i;
    atomicOr(&mask[bit >> 5], 1u << (bit & 31));
  }
}

// ---------------------------------------------------------------- k_scan
// Queries without text terms (Dataset::search with an empty query,
// src/db/search.rs:115-116, 129-150): the facet union alone -- score =
// f_tab[bits] of the doc's matching clauses -- or AllQuery (every alive doc,
// score 1.0, query/all_query.rs).  A work item scans <= 32 consecutive
// 4096-doc tiles in doc order through the same local top-k buffer and
// threshold publication as k_disj.  Keys fall with the doc id at equal score,
// so once (max score, first doc of a tile) is below the threshold nothing
// later in the item can enter the top-k and the item stops.
struct ScanShared {
  alignas(16) uint64_t buf[kBufD];
  uint32_t hist[kHistBins];
  uint32_t scratch[8];
  uint32_t n_buf;
  uint64_t thr;
};

__device__ inline void scan_truncate(ScanShared& sh, uint32_t K, uint32_t limit, uint64_t* gthr, bool publish,
                                     uint64_t pub, const DevPlan& pl, uint32_t ql) {
  const uint32_t n = sh.n_buf;
  __syncthreads();
  uint64_t T = 0;
  if (n > limit) T = truncate_keys<kBufD>(sh.buf, &sh.n_buf, sh.hist, sh.scratch, n, K);
  if (threadIdx.x == 0) {
    uint64_t mine = T > sh.thr ? T : sh.thr;
    if (publish) {
      const uint64_t old = atomicMax(reinterpret_cast<unsigned long long*>(gthr), (unsigned long long)(mine & pub));
      peer_thr_max(pl, ql, mine);
      mine = old > mine ? old : mine;
    }
    sh.thr = mine;
  }
  __syncthreads();
}

template <bool kMulti>
__global__ __launch_bounds__(kThreads) void k_scan(DevIndex ix0, DevPlan pl) {
  __shared__ ScanShared sh;
  const uint32_t tid = threadIdx.x;
  const uint32_t w = pl.total_chunks + blockIdx.x;  // scan items follow the k_conj / k_disj items
  const uint32_t q = pl.work_q[w];
  const DevIndex ix = kMulti ? seg_index(pl, __builtin_amdgcn_readfirstlane(q / pl.seg_nq)) : ix0;
  const uint32_t ql = kMulti ? __builtin_amdgcn_readfirstlane(q % pl.seg_nq) : q;
  const uint32_t tile0 = pl.work_c[w], ntile = pl.work_n[w];
  const uint32_t K = pl.k;
  uint64_t* gthr = &pl.thresh[ql];
  const uint32_t fslot = pl.f.q_filter[q];
  const uint32_t* fmask = nullptr;
  uint32_t fshift = 0;
  const float* ftab = nullptr;
  float smax = 1.0f;  // AllScorer
  if (fslot != kInvalid) {
    fmask = pl.f.fmask + pl.f.f_woff[fslot];
    fshift = pl.f.f_shift[fslot];
    ftab = pl.f.f_tab + (size_t)fslot * 256;
    smax = pl.f.f_max[fslot];
  }
  if (tid == 0) {
    sh.n_buf = 0;
    sh.thr = atomicMax(reinterpret_cast<unsigned long long*>(gthr), 0ull);
  }
  __syncthreads();
  for (uint32_t t = 0; t < ntile; ++t) {
    const uint32_t d0 = (tile0 + t) << kTileShift;
    if (d0 >= ix.n_docs || make_key(smax, d0) < sh.thr) break;  // uniform: sh.thr read after a barrier
    const uint32_t d1 = min(d0 + kTile, ix.n_docs);
    for (uint32_t r0 = d0; r0 < d1; r0 += kRound) {
      const uint64_t thr = sh.thr;
#pragma unroll
      for (uint32_t j = 0; j < kRound / kThreads; ++j) {
        const uint32_t d = r0 + j * kThreads + tid;
        bool keep = d < d1 && doc_alive(ix, d);
        float sc = 1.0f;
        if (keep && fmask) {
          const uint32_t fb = filter_bits(fmask, fshift, d);
          keep = fb != 0;
          sc = ftab[fb];
        }
        const uint64_t key = keep ? make_key(sc, d) : 0;
        wave_append(keep && key >= thr, key, sh.buf, &sh.n_buf, kBufD);
      }
      __syncthreads();
      scan_truncate(sh, K, kTrunc, gthr, false, pl.pub_mask, pl, ql);
    }
    scan_truncate(sh, K, K, gthr, true, pl.pub_mask, pl, ql);
  }
  flush_candidates(pl, q, sh.buf, sh.n_buf, sh.thr, sh.scratch);
}

// ---------------------------------------------------------------- k_final
// Dynamic LDS (80 KB: 2 workgroups per CU): candidate keys, the k winners,
// the radix histogram.  Keeps 16-B alignment of the dynamic base (no static
// __shared__ in this kernel: cdna_hip_programming.md Guideline 17).
#ifndef FG_FINAL_HBITS
#define FG_FINAL_HBITS 11
#endif
constexpr uint32_t kFinalHistBits = FG_FINAL_HBITS;  // k_final's radix digits (its LDS sets its occupancy)
struct FinalShared {
  uint64_t keys[kFinalCap];
  uint64_t win[kMaxK];
  uint32_t hist[1u << kFinalHistBits];
  uint32_t scratch[8];
  uint32_t n_keys;
  uint32_t n_win;
};
constexpr size_t kFinalLds = sizeof(FinalShared);

// kMerged (a multi-snapshot plan with DevPlan::seg_base): one workgroup per
// batch query selects over the candidates of ALL its slots at once, each key's
// doc shifted by its snapshot's base (key - base: ~(base + doc)), so the order
// (score desc, snapshot base + doc asc) IS the merge by (score desc, shard asc,
// doc asc): the merged top-k without per-slot lists and k_merge_rank.  Slots
// past a query's count are written as score 0, doc 0, shard 0.
template <bool kMerged>
__global__ __launch_bounds__(kThreads) void k_final(DevPlan pl, float* __restrict__ out_score,
                                                     uint32_t* __restrict__ out_doc, uint32_t* __restrict__ out_n,
                                                     uint32_t* __restrict__ out_shard) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  FinalShared& sh = *reinterpret_cast<FinalShared*>(lds_raw);
  const uint32_t q = blockIdx.x, tid = threadIdx.x;
  const uint32_t dq = pl.total_chunks + pl.n_scan + q;
  (void)dq;
  FG_STAMP(dq, 0, FG_NOW());
  const uint32_t K = pl.k;
  // the threshold word, or the query's histogram threshold when higher (>= K
  // docs of the query -- or of its linked plans -- score at least that much)
  const uint32_t ql = kMerged ? q : slot_query(pl, q);  // a multi-snapshot plan: the slot's batch query
  const uint64_t T0 = max(pl.thresh[ql], hist_threshold(pl.hist + (size_t)ql * kQBins, K, pl.q_hlo[q], pl.q_hsh[q],
                                                        sh.scratch));
  const uint32_t n_lists = kMerged ? pl.n_segs : 1;
  uint32_t cnt = 0;  // candidates of all lists
  for (uint32_t s = 0; s < n_lists; ++s) cnt += pl.cand_cnt[kMerged ? s * pl.seg_nq + q : q];
  // every candidate of query q (of every slot of q), f(key >= lb, key) with the
  // whole workgroup converged; eight loads per thread in flight per round (the
  // lists are read once per pass and the passes are latency-bound).  Merged:
  // keys as (score, ~(snapshot base + doc)); thresholds are score-only there
  auto each_key = [&](uint64_t lb, auto&& f) {
    constexpr uint32_t U = 8;
    for (uint32_t s = 0; s < n_lists; ++s) {
      const uint32_t v = kMerged ? s * pl.seg_nq + q : q;
      const uint32_t c = kMerged ? pl.cand_cnt[v] : cnt;
      const uint64_t* src = pl.cand_keys + pl.cand_off[v];
      const uint64_t sub = kMerged ? pl.seg_base[s] : 0u;
      for (uint32_t i0 = 0; i0 < c; i0 += U * kThreads) {
        uint64_t key[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
          const uint32_t i = i0 + u * kThreads + tid;
          key[u] = i < c ? src[i] - sub : 0;
        }
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
          const uint32_t i = i0 + u * kThreads + tid;
          f(i < c && key[u] >= lb, key[u]);
        }
      }
    }
  };
  if (tid == 0) { sh.n_keys = 0; sh.n_win = 0; }
  __syncthreads();
  each_key(T0, [&](bool keep, uint64_t key) { wave_append(keep, key, sh.keys, &sh.n_keys, kFinalCap); });
  __syncthreads();
  const uint32_t nk = sh.n_keys;
  FG_STAMP(dq, 1, FG_NOW());
  FG_STAMP(dq, 5, cnt);
  FG_STAMP(dq, 6, nk);
  uint64_t* sorted = sh.keys;
  uint32_t nout = nk;
  if (nk > K) {
    // exact k-th key (in LDS, or straight from HBM when the list overflowed), then the K winners
    uint64_t T;
    if (nk > kFinalCap) {
      T = select_kth<kFinalHistBits>(K, sh.hist, sh.scratch, [&](auto&& f) {
        each_key(T0, [&](bool keep, uint64_t key) { if (keep) f(key); });
      });
      each_key(T, [&](bool keep, uint64_t key) { wave_append(keep, key, sh.win, &sh.n_win, kMaxK); });
    } else {
      T = select_kth<kFinalHistBits>(K, sh.hist, sh.scratch, [&](auto&& f) {
        for (uint32_t i = tid; i < nk; i += kThreads) f(sh.keys[i]);
      });
      for (uint32_t i0 = 0; i0 < nk; i0 += kThreads) {
        const uint32_t i = i0 + tid;
        const uint64_t key = i < nk ? sh.keys[i] : 0;
        wave_append(i < nk && key >= T, key, sh.win, &sh.n_win, kMaxK);
      }
    }
    __syncthreads();
    sorted = sh.win;
    nout = K;  // keys are unique: exactly K are >= T
  }
  FG_STAMP(dq, 2, FG_NOW());
  uint32_t P = 1;
  while (P < nout) P <<= 1;
  for (uint32_t i = nout + tid; i < P; i += kThreads) sorted[i] = 0;
  __syncthreads();
  bitonic_sort_desc(sorted, P);
  if (kMerged) {
    for (uint32_t i = tid; i < K; i += kThreads) {
      float sc = 0.0f;
      uint32_t d = 0, sd = 0;
      if (i < nout) {
        const uint64_t k = sorted[i];
        const uint32_t g = key_doc(k);  // snapshot base + doc
        uint32_t lo = 0, hi = pl.n_segs;  // the last snapshot whose base <= g
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (pl.seg_base[mid] <= g) lo = mid; else hi = mid;
        }
        sc = key_score(k);
        d = g - pl.seg_base[lo];
        sd = lo;
      }
      out_score[(size_t)q * K + i] = sc;
      out_doc[(size_t)q * K + i] = d;
      if (out_shard) out_shard[(size_t)q * K + i] = sd;
    }
  } else {
    for (uint32_t i = tid; i < nout; i += kThreads) {
      const uint64_t k = sorted[i];
      out_score[(size_t)q * K + i] = key_score(k);
      out_doc[(size_t)q * K + i] = key_doc(k);
    }
  }
  if (tid == 0) out_n[q] = nout;
  FG_STAMP(dq, 3, FG_NOW());
}

// ---------------------------------------------------------------- k_merge
// Cross-shard merge of per-shard top-k lists (each in key order) into the
// global top-k by (score desc, shard asc, doc asc).
//
// k_merge_rank: one workgroup per query.  The shards' scores go to LDS; every
// entry (s, i) then finds its output position directly,
//   pos = i + #{s' < s: score >= sc} + #{s' > s: score > sc},
// by one binary search per other shard (the lists are score-descending, and
// within a shard equal scores are already doc-ascending), and writes itself
// when pos < k.  No serial walk: every entry of every shard in parallel.
constexpr uint32_t kMergeCap = 12288;  // scores per query held in LDS (48 KB)

__device__ inline uint32_t count_ge(const float* l, uint32_t c, float x) {  // l descending
  uint32_t lo = 0, hi = c;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (l[mid] >= x) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ inline uint32_t count_gt(const float* l, uint32_t c, float x) {
  uint32_t lo = 0, hi = c;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (l[mid] > x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(kThreads) void k_merge_rank(uint32_t n_shards, uint32_t nq, uint32_t k,
                                                          const float* __restrict__ score,
                                                          const uint32_t* __restrict__ doc,
                                                          const uint32_t* __restrict__ n, float* __restrict__ out_score,
                                                          uint32_t* __restrict__ out_doc,
                                                          uint32_t* __restrict__ out_shard,
                                                          uint32_t* __restrict__ out_n) {
  __shared__ float ls[kMergeCap];
  __shared__ uint32_t cnt[65], off[65];
  const uint32_t q = blockIdx.x, tid = threadIdx.x;
  if (tid < n_shards) cnt[tid] = min(n[(size_t)tid * nq + q], k);
  __syncthreads();
  if (tid == 0) {
    uint32_t o = 0;
    for (uint32_t s = 0; s < n_shards; ++s) { off[s] = o; o += cnt[s]; }
    off[n_shards] = o;
  }
  __syncthreads();
  const uint32_t total = off[n_shards];
  for (uint32_t s = 0; s < n_shards; ++s) {
    const float* src = score + ((size_t)s * nq + q) * k;
    for (uint32_t i = tid; i < cnt[s]; i += kThreads) ls[off[s] + i] = src[i];
  }
  __syncthreads();
  for (uint32_t e = tid; e < total; e += kThreads) {
    uint32_t s = 0;
    while (off[s + 1] <= e) ++s;
    const uint32_t i = e - off[s];
    const float sc = ls[e];
    uint32_t pos = i;
    for (uint32_t t = 0; t < n_shards && pos < k; ++t) {
      if (t == s) continue;
      pos += t < s ? count_ge(ls + off[t], cnt[t], sc) : count_gt(ls + off[t], cnt[t], sc);
    }
    if (pos < k) {
      out_score[(size_t)q * k + pos] = sc;
      out_doc[(size_t)q * k + pos] = doc[((size_t)s * nq + q) * k + i];
      if (out_shard) out_shard[(size_t)q * k + pos] = s;
    }
  }
  // slots past the count: score 0, doc 0, shard 0 (defined, so a caller that
  // gathers by shard over all k slots stays in bounds)
  for (uint32_t e = min(total, k) + tid; e < k; e += kThreads) {
    out_score[(size_t)q * k + e] = 0.0f;
    out_doc[(size_t)q * k + e] = 0u;
    if (out_shard) out_shard[(size_t)q * k + e] = 0u;
  }
  if (tid == 0) out_n[q] = min(total, k);
}

// k_merge: the serial form (one lane per query walks the n_shards heads) for
// merges whose lists do not fit k_merge_rank's LDS (n_shards x k > kMergeCap).
__global__ __launch_bounds__(kThreads) void k_merge(uint32_t n_shards, uint32_t nq, uint32_t k,
                                                     const float* __restrict__ score, const uint32_t* __restrict__ doc,
                                                     const uint32_t* __restrict__ n, float* __restrict__ out_score,
                                                     uint32_t* __restrict__ out_doc, uint32_t* __restrict__ out_shard,
                                                     uint32_t* __restrict__ out_n) {
  const uint32_t q = blockIdx.x * kThreads + threadIdx.x;
  if (q >= nq) return;
  uint32_t head[64], cnt[64];
  for (uint32_t s = 0; s < n_shards; ++s) {
    head[s] = 0;
    cnt[s] = min(n[(size_t)s * nq + q], k);
  }
  uint32_t produced = 0;
  for (; produced < k; ++produced) {
    int best = -1;
    float bs = 0.0f;
    uint32_t bd = 0;
    for (uint32_t s = 0; s < n_shards; ++s) {
      if (head[s] >= cnt[s]) continue;
      const size_t at = ((size_t)s * nq + q) * k + head[s];
      const float sc = score[at];
      if (best < 0 || sc > bs) { best = (int)s; bs = sc; bd = doc[at]; }
    }
    if (best < 0) break;
    out_score[(size_t)q * k + produced] = bs;
    out_doc[(size_t)q * k + produced] = bd;
    if (out_shard) out_shard[(size_t)q * k + produced] = (uint32_t)best;
    head[best]++;
  }
  out_n[q] = produced;
  for (uint32_t e = produced; e < k; ++e) {  // slots past the count, as k_merge_rank
    out_score[(size_t)q * k + e] = 0.0f;
    out_doc[(size_t)q * k + e] = 0u;
    if (out_shard) out_shard[(size_t)q * k + e] = 0u;
  }
}

}  // namespace

template <bool kSingle, uint32_t kF>
static void conj_launch(const DevIndex& ix, const DevPlan& pl, uint32_t grid, hipStream_t s) {
  if (pl.segs) k_conj<kSingle, true, kF><<<grid, kThreads, 0, s>>>(ix, pl);
  else k_conj<kSingle, false, kF><<<grid, kThreads, 0, s>>>(ix, pl);
}
// the instantiation of a plan's features: 0 (build-time scores), kFQt, or kFQt with names / escapes
static inline uint32_t feat_of(const DevPlan& pl) {
  return !(pl.feat & kFQt) ? 0u : (pl.feat & (kFName | kFEsc)) ? (kFQt | kFName | kFEsc) : kFQt;
}
template <bool kSingle>
static void conj_launch_f(const DevIndex& ix, const DevPlan& pl, uint32_t grid, hipStream_t s) {
  switch (feat_of(pl)) {
    case 0: conj_launch<kSingle, 0>(ix, pl, grid, s); break;
    case kFQt: conj_launch<kSingle, kFQt>(ix, pl, grid, s); break;
    default: conj_launch<kSingle, kFQt | kFName | kFEsc>(ix, pl, grid, s); break;
  }
}

hipError_t launch_conj(const DevIndex& ix, const DevPlan& pl, hipStream_t s) {
  if (pl.n_single) {
    conj_launch_f<true>(ix, pl, pl.n_single, s);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (pl.n_conj > pl.n_single) conj_launch_f<false>(ix, pl, pl.n_conj - pl.n_single, s);
  return hipGetLastError();
}

template <uint32_t kF>
static void disj_launch(const DevIndex& ix, const DevPlan& pl, uint32_t grid, hipStream_t s) {
  if (pl.segs) k_disj<true, kF><<<grid, kThreads, 0, s>>>(ix, pl);
  else k_disj<false, kF><<<grid, kThreads, 0, s>>>(ix, pl);
}

hipError_t launch_disj(const DevIndex& ix, const DevPlan& pl, hipStream_t s, uint32_t first, uint32_t count) {
  const uint32_t n = pl.total_chunks > pl.n_conj ? pl.total_chunks - pl.n_conj : 0u;
  if (first >= n) return hipSuccess;
  count = min(count, n - first);
  if (!count) return hipSuccess;
  // a part of the sweep: the kernel's items start at pl.n_conj
  DevPlan part = pl;
  part.n_conj = pl.n_conj + first;
  switch (feat_of(pl)) {
    case 0: disj_launch<0>(ix, part, count, s); break;
    case kFQt: disj_launch<kFQt>(ix, part, count, s); break;
    default: disj_launch<kFQt | kFName | kFEsc>(ix, part, count, s); break;
  }
  return hipGetLastError();
}

hipError_t launch_fmask(const DevIndex& ix, const DevPlan& pl, hipStream_t s) {
  if (pl.f.n_chunks == 0) return hipSuccess;
  if (pl.segs) k_fmask<true><<<pl.f.n_chunks, kThreads, 0, s>>>(ix, pl);
  else k_fmask<false><<<pl.f.n_chunks, kThreads, 0, s>>>(ix, pl);
  return hipGetLastError();
}

hipError_t launch_scan(const DevIndex& ix, const DevPlan& pl, hipStream_t s) {
  if (pl.n_scan == 0) return hipSuccess;
  if (pl.segs) k_scan<true><<<pl.n_scan, kThreads, 0, s>>>(ix, pl);
  else k_scan<false><<<pl.n_scan, kThreads, 0, s>>>(ix, pl);
  return hipGetLastError();
}

hipError_t launch_final(const DevPlan& pl, float* out_score, uint32_t* out_doc, uint32_t* out_n, hipStream_t s,
                        uint32_t* out_shard) {
  const bool merged = out_shard != nullptr;
  if (merged && (!pl.seg_base || !pl.seg_nq)) return hipErrorInvalidValue;
  const uint32_t grid = merged ? pl.seg_nq : pl.n_queries;
  if (grid == 0) return hipSuccess;
  // opt in to > 64 KB of dynamic LDS once per device and instantiation
  static unsigned long long attr_set[2] = {0, 0};
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 64 && !((__atomic_load_n(&attr_set[merged], __ATOMIC_ACQUIRE) >> dev) & 1ull)) {
    const void* fn = merged ? reinterpret_cast<const void*>(&k_final<true>) : reinterpret_cast<const void*>(&k_final<false>);
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kFinalLds);
    if (e != hipSuccess) return e;
    __atomic_fetch_or(&attr_set[merged], 1ull << dev, __ATOMIC_RELEASE);
  }
  if (merged) k_final<true><<<grid, kThreads, kFinalLds, s>>>(pl, out_score, out_doc, out_n, out_shard);
  else k_final<false><<<grid, kThreads, kFinalLds, s>>>(pl, out_score, out_doc, out_n, nullptr);
  return hipGetLastError();
}

// Snapshot build: the rank words of every rank-kind term (fg_internal.h
// DevIndex::rank) in one launch.  One workgroup per (term slot, 2048 words =
// 65536 docs): two binary searches locate the chunk's postings, their presence
// bits are set in LDS, and a workgroup prefix sum of the words' popcounts gives
// each word's rank.
__global__ __launch_bounds__(kThreads) void k_rank(const uint32_t* __restrict__ doc_all,
                                                   const uint64_t* __restrict__ slot_base,
                                                   const uint32_t* __restrict__ slot_n, uint32_t chunks_per_slot,
                                                   uint32_t n_words, uint64_t* __restrict__ out_all) {
  __shared__ uint32_t bits[kRankChunkWords];
  __shared__ uint32_t scratch[8];
  __shared__ uint32_t range[2];
  const uint32_t tid = threadIdx.x;
  const uint32_t slot = blockIdx.x / chunks_per_slot, chunk = blockIdx.x - slot * chunks_per_slot;
  const uint32_t* __restrict__ doc = doc_all + slot_base[slot];
  const uint32_t n = slot_n[slot];
  uint64_t* __restrict__ out = out_all + (size_t)slot * n_words;
  const uint32_t w0 = chunk * kRankChunkWords;
  if (tid < 2) {
    const uint64_t target = ((uint64_t)w0 + (tid ? kRankChunkWords : 0u)) << 5;
    uint32_t lo = 0, hi = n;  // first posting with doc >= target
    while (lo < hi) {
      const uint32_t mid = lo + ((hi - lo) >> 1);
      if ((uint64_t)doc[mid] < target) lo = mid + 1; else hi = mid;
    }
    range[tid] = lo;
  }
  for (uint32_t i = tid; i < kRankChunkWords; i += kThreads) bits[i] = 0u;
  __syncthreads();
  for (uint32_t p = range[0] + tid; p < range[1]; p += kThreads) {
    const uint32_t d = doc[p];
    atomicOr(&bits[rank_word(d) - w0], 1u << (d & 31u));
  }
  __syncthreads();
  constexpr uint32_t R = kRankChunkWords / kThreads;
  uint32_t c[R], sum = 0;
#pragma unroll
  for (uint32_t i = 0; i < R; ++i) {
    c[i] = (uint32_t)__popc(bits[tid * R + i]);
    sum += c[i];
  }
  uint32_t r = range[0] + block_exclusive_scan(sum, scratch);
#pragma unroll
  for (uint32_t i = 0; i < R; ++i) {
    const uint32_t w = w0 + tid * R + i;
    if (w < n_words) out[w] = (uint64_t)bits[tid * R + i] | ((uint64_t)r << 32);
    r += c[i];
  }
}

hipError_t launch_rank(const uint32_t* doc, const uint64_t* slot_base, const uint32_t* slot_n, uint32_t n_slots,
                       uint32_t n_words, uint64_t* out, hipStream_t s) {
  if (n_words == 0 || n_slots == 0) return hipSuccess;
  const uint32_t cps = (n_words + kRankChunkWords - 1) / kRankChunkWords;
  if ((uint64_t)cps * n_slots > 0x7FFFFFFFull) return hipErrorInvalidValue;
  k_rank<<<cps * n_slots, kThreads, 0, s>>>(doc, slot_base, slot_n, cps, n_words, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------- build-time bounds
// The build's posting scores (ScoreJob::psc, a temporary) from the same
// payloads and arithmetic the search kernels use at query time (tfn_score):
// bounds computed from them hold bit for bit under the build's statistics.
__device__ inline float build_score(const ScoreJob& j, uint64_t p, uint32_t v, float wt, float wn, const float* cache) {
  uint32_t tt = v & 0xFFu, tn = (v >> 16) & 0xFFu;
  if (tt == kTfEsc || tn == kTfEsc) {
    const uint32_t e = tf_escaped(j.esc_pos, j.esc_tf, j.n_esc, p);
    if (tt == kTfEsc) tt = e & 0xFFFFu;
    if (tn == kTfEsc) tn = e >> 16;
  }
  float s = 0.0f;
  if (tt) s += field_score(tt, (v >> 8) & 0xFFu, wt, cache);
  if (tn) s += field_score(tn, v >> 24, wn, cache + 256);
  return s;
}

// Packed chunks (ScoreJob::sc_*): a long term's 2048-posting slice, or the
// postings of several whole short terms (a vocabulary's long tail would
// otherwise cost one workgroup per term).  A posting's term: the last of the
// chunk's term offsets (staged in LDS) at or below it.
template <class Off>
__device__ inline uint32_t slot_of(const Off* s_off, uint32_t nterm, uint64_t p) {
  uint32_t lo = 0, hi = nterm;  // s_off[lo] <= p < s_off[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if ((uint64_t)s_off[mid] <= p) lo = mid; else hi = mid;
  }
  return lo;
}

// The scoring kernels take their logical workgroup count n and loop over it in
// steps of gridDim.x: a background scoring (a commit's rescores) launches at most
// ScoreJob::grid_cap workgroups, so a search beside it finds wave slots free
// (launch_* below; tools/stall_probe.hip: a background kernel filling every slot
// held a search up for its whole span, one filling half of them did not).
__global__ __launch_bounds__(kThreads) void k_score(ScoreJob j, uint32_t n) {
  __shared__ float cache[512];
  __shared__ uint64_t s_off[kPackTerms + 1];
  __shared__ uint32_t s_max[kPackTerms];
  for (uint32_t i = threadIdx.x; i < 512; i += kThreads) cache[i] = j.cache[i];
  for (uint32_t c = blockIdx.x; c < n; c += gridDim.x) {
  __syncthreads();  // the previous chunk's LDS reads are done
  const uint32_t tf = j.sc_tf[c], nterm = j.sc_tl[c] - tf + 1;
  const uint64_t e0 = j.sc_e0[c], e1 = j.sc_e1[c];
  for (uint32_t i = threadIdx.x; i <= nterm; i += kThreads) s_off[i] = j.off[tf + i];
  for (uint32_t i = threadIdx.x; i < nterm; i += kThreads) s_max[i] = 0u;
  __syncthreads();
  // the chunk's payloads in one step per thread, in flight together (kScoreChunk / kThreads per thread)
  constexpr uint32_t R = kScoreChunk / kThreads;
  uint32_t tv[R];
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) {
    const uint64_t p = e0 + r * kThreads + threadIdx.x;
    tv[r] = p < e1 ? (uint32_t)j.tfn[p] | (j.tfn_name ? (uint32_t)j.tfn_name[p] << 16 : 0u) : 0u;
  }
  float mx = 0.0f;  // one term (uniform): reduced per wave, one LDS atomic
#pragma unroll
  for (uint32_t r = 0; r < R; ++r) {
    const uint64_t p = e0 + r * kThreads + threadIdx.x;
    if (p >= e1) continue;
    const uint32_t sl = nterm == 1 ? 0u : slot_of(s_off, nterm, p);
    const uint32_t t = tf + sl;
    const float v = build_score(j, p, tv[r], j.w_text[t], j.w_name[t], cache);
    j.psc[p] = v;
    if (nterm == 1) mx = fmaxf(mx, v);
    else atomicMax(&s_max[sl], __float_as_uint(v));
  }
  if (nterm == 1) {
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(&s_max[0], __float_as_uint(mx));
  }
  __syncthreads();
  // block-max of each term chunk (DevIndex::cmax: kChunk postings from the term's start)
  for (uint32_t i = threadIdx.x; i < nterm; i += kThreads) {
    const uint64_t b = s_off[i];
    if (s_off[i + 1] == b) continue;  // an empty term id
    const uint32_t t = tf + i;
    const uint64_t first = e0 > b ? e0 : b;
    j.cmax[j.coff[t] + (uint32_t)((first - b) / kChunk)] = __uint_as_float(s_max[i]);
  }
  }
}

// Bucket maxima (-0.0: empty bucket, a score may be +0.0), the term maxima and
// the 4096-doc tile maxima (terms whose buckets are no wider than a tile).
// Scores are >= 0, so their f32 bits order like the values (atomicMax on u32).
__global__ __launch_bounds__(kThreads) void k_bucket(ScoreJob j, uint32_t n_docs, uint32_t n) {
  __shared__ uint32_t s_doff[kPackTerms + 1];
  __shared__ uint32_t s_max[kPackTerms];
  for (uint32_t c = blockIdx.x; c < n; c += gridDim.x) {
  __syncthreads();  // the previous chunk's LDS reads are done
  const uint32_t tf = j.bk_tf[c], nterm = j.bk_tl[c] - tf + 1;
  const uint32_t e0 = j.bk_e0[c], e1 = j.bk_e1[c];
  for (uint32_t i = threadIdx.x; i <= nterm; i += kThreads)
    s_doff[i] = tf + i < j.n_terms ? j.dir_off[tf + i] : (uint32_t)j.n_dir;
  for (uint32_t i = threadIdx.x; i < nterm; i += kThreads) s_max[i] = 0u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t i0 = e0; i0 < e1; i0 += kThreads) {  // uniform trip count: every lane shuffles
    const uint32_t i = i0 + threadIdx.x;
    const uint32_t sl = nterm == 1 ? 0u : slot_of(s_doff, nterm, min(i, e1 - 1));
    const uint32_t t = tf + sl;
    const uint32_t meta = j.tmeta[t], B = meta & 0xFFu;
    const uint32_t nbk = (uint32_t)(((uint64_t)(n_docs - 1) >> B) + 1);
    const uint32_t bk = min(i, e1 - 1) - s_doff[sl];
    const bool in = i < e1 && bk < nbk;  // the term's last entry is its end, not a bucket
    const uint32_t lo = in ? j.dir[i] : 0u, hi = in ? j.dir[i + 1] : 0u;
    const float* ps = j.psc + j.off[t];
    float mx = -0.0f;
    uint32_t bits = 0;
    if (hi > lo) {
      mx = 0.0f;
      for (uint32_t p = lo; p < hi; ++p) mx = fmaxf(mx, ps[p]);
      bits = __float_as_uint(mx);
      atomicMax(&s_max[sl], bits);
    }
    if (in) j.bmax[i] = mx;
    // tile maxima: a segmented max over the wave's buckets (their (term, tile)
    // keys ascend with the lane), then one atomic per key the wave touches --
    // not one per bucket, which put up to 64 atomics on one address
    const uint32_t to = j.toff[t];
    const uint32_t key = (in && to != 0xFFFFFFFFu) ? to + (uint32_t)(((uint64_t)bk << B) >> kDisjTileShift) : 0xFFFFFFFFu;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
      const uint32_t b2 = (uint32_t)__shfl_down((int)bits, o, 64);
      const uint32_t k2 = (uint32_t)__shfl_down((int)key, o, 64);
      if (lane + o < 64 && k2 == key) bits = max(bits, b2);
    }
    const uint32_t prev = (uint32_t)__shfl_up((int)key, 1, 64);
    if (key != 0xFFFFFFFFu && bits && (lane == 0 || prev != key)) atomicMax(&j.tmax[key], bits);
  }
  __syncthreads();
  // the term maxima (a long term spans chunks: atomics)
  for (uint32_t i = threadIdx.x; i < nterm; i += kThreads)
    if (s_max[i]) atomicMax(&j.tmaxs[tf + i], s_max[i]);
  }
}

// Sub-tile maxima (DevIndex::tsub): one thread per tile entry walks
// the tile's buckets (bucket maxima from k_bucket, -0.0 = empty), takes the
// largest per 512-doc block -- a bucket wider than a block counts in each block
// it covers -- and quantizes them up against the tile maximum.  After k_bucket.
static_assert(kDisjTileShift - kSubShift == 3, "8 sub-tile blocks per tile: one byte each of a u64");
__global__ __launch_bounds__(kThreads) void k_tsub(ScoreJob j, uint32_t n_docs) {
  const uint32_t nt1 = j.n_tiles + 1;
  const uint64_t n_e = (uint64_t)j.n_tterm * nt1;
  for (uint64_t e = (uint64_t)blockIdx.x * kThreads + threadIdx.x; e < n_e; e += (uint64_t)gridDim.x * kThreads) {
  const uint32_t k = (uint32_t)(e / nt1), tile = (uint32_t)(e - (uint64_t)k * nt1);
  if (tile >= j.n_tiles) {  // the entry past a term's last tile (tdir's end): never read as a tile
    j.tsub[e] = ~0ull;
    continue;
  }
  const uint32_t t = j.tterm[k];
  const uint32_t B = j.tmeta[t] & 0xFFu;  // <= kDisjTileShift for a tile-table term
  const uint32_t nbk = (uint32_t)(((uint64_t)(n_docs - 1) >> B) + 1);
  const uint32_t b0 = tile << (kDisjTileShift - B), b1 = min(nbk, (tile + 1) << (kDisjTileShift - B));
  const float* bm = j.bmax + j.dir_off[t];
  float mx[8];
#pragma unroll
  for (uint32_t z = 0; z < 8; ++z) mx[z] = 0.0f;
  const uint32_t span = B > kSubShift ? 1u << (B - kSubShift) : 1u;  // blocks a bucket covers
  for (uint32_t b = b0; b < b1; ++b) {
    const float v = bm[b];
    if (signbit(v)) continue;  // empty bucket
    const uint32_t z0 = (((b - b0) << B) >> kSubShift);
#pragma unroll
    for (uint32_t z = 0; z < 8; ++z)
      if (z >= z0 && z < z0 + span) mx[z] = fmaxf(mx[z], v);
  }
  const float M = __uint_as_float(j.tmax[e]);
  uint64_t w = 0;
#pragma unroll
  for (uint32_t z = 0; z < 8; ++z) w |= (uint64_t)quant8(mx[z], M) << (8 * z);
  j.tsub[e] = w;
  }
}

// Per term the K-th best score over its ALIVE postings for K in kTopKs (0 when
// fewer): a doc among a term's top K scores at least that much in any
// disjunction containing the term, so the query's K-th best is >= it (k_disj's
// starting threshold).  Exact selects over unique (score, doc) keys.  A term of
// <= kKtopChunk postings: one workgroup (k_ktop).  A longer one is cut into
// kKtopChunk-posting chunks, one workgroup each (k_ktop_part: the chunk's
// alive count / extremes and its KM best keys), then one workgroup per such
// term selects over its chunks' keys (k_ktop_big): a 9M-posting term no longer
// streams its list through one workgroup several times.
constexpr uint32_t kKtopKM = kTopKs[kNumTopK - 1];  // the largest K: its keys are kept
constexpr uint32_t kKtopSort = 1024;                 // ... and sorted (a power of two >= KM)
static_assert(kKtopSort >= kKtopKM && (kKtopSort & (kKtopSort - 1)) == 0, "k_ktop sorts its KM keys in place");

struct KtopShared {
  uint32_t hist[kHistBins];
  uint32_t scratch[8];
  uint32_t red[3];  // alive postings, smallest alive score (bits), largest (bits)
  uint64_t top[kKtopSort];  // the KM best keys, then zero padding for the sort
  uint32_t n_top;
};

// term t's K-th best scores for K >= 10 from its na alive keys (each_key(f):
// f(ok, key) for every key, the workgroup converged): the KM best into LDS with
// one select over all keys, then one bitonic sort of them gives every K
template <class EachKey>
__device__ void ktop_finish(const ScoreJob& j, uint32_t t, uint32_t na, KtopShared& sh, EachKey each_key) {
  constexpr uint32_t KM = kKtopKM;
  if (na < (j.ladder ? kLadderExtra[0] : kTopKs[1])) return;  // uniform: only K = 1
  uint64_t T = 0;
  if (na > KM) {
    T = select_kth(KM, sh.hist, sh.scratch, [&](auto&& f) {
      each_key([&](bool ok, uint64_t key) { if (ok) f(key); });
    });
  }
  each_key([&](bool ok, uint64_t key) { wave_append(ok && key >= T, key, sh.top, &sh.n_top, KM); });
  __syncthreads();
  const uint32_t nt = min(na, KM);  // keys in top[] (unique: exactly KM are >= T)
  // one bitonic sort of the kept keys: the K-th key of every K is then top[K - 1]
  uint32_t P = 16;
  while (P < nt) P <<= 1;
  for (uint32_t i = nt + threadIdx.x; i < P; i += kThreads) sh.top[i] = 0;
  __syncthreads();
  bitonic_sort_desc(sh.top, P);
  if (threadIdx.x == 0)
    for (uint32_t kk = 1; kk < kNumTopK; ++kk)
      if (nt >= kTopKs[kk]) j.ktop[(size_t)t * kNumTopK + kk] = key_score(sh.top[kTopKs[kk] - 1]);
  if (j.ladder && threadIdx.x < kNumLadderExtra && nt >= kLadderExtra[threadIdx.x])
    j.ladder[(size_t)t * kNumLadderExtra + threadIdx.x] = key_score(sh.top[kLadderExtra[threadIdx.x] - 1]);
}

// postings [b + p0, b + p1) as f(valid && alive, score, doc), U loads per thread
// in flight, the workgroup converged (callers may use wave-wide operations)
template <class F>
__device__ inline void ktop_each_posting(const ScoreJob& j, uint64_t b, uint32_t p0, uint32_t p1, F&& f) {
  constexpr uint32_t U = 4;
  for (uint32_t q0 = p0; q0 < p1; q0 += U * kThreads) {
    uint32_t d[U];
    float s[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t p = q0 + u * kThreads + threadIdx.x;
      d[u] = p < p1 ? j.doc[b + p] : 0xFFFFFFFFu;
      s[u] = p < p1 ? j.psc[b + p] : 0.0f;
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const bool ok = d[u] != 0xFFFFFFFFu && (!j.alive || ((j.alive[d[u] >> 5] >> (d[u] & 31u)) & 1u));
      f(ok, s[u], d[u]);
    }
  }
}

// alive count, smallest and largest alive score bits of postings [p0, p1) into sh.red
__device__ inline void ktop_reduce(const ScoreJob& j, uint64_t b, uint32_t p0, uint32_t p1, KtopShared& sh) {
  if (threadIdx.x == 0) {
    sh.red[0] = 0;
    sh.red[1] = 0xFFFFFFFFu;
    sh.red[2] = 0;
    sh.n_top = 0;
  }
  __syncthreads();
  uint32_t c = 0, mx = 0, mn = 0xFFFFFFFFu;
  ktop_each_posting(j, b, p0, p1, [&](bool ok, float sv, uint32_t) {
    if (!ok) return;
    const uint32_t bits = __float_as_uint(sv);
    ++c;
    mx = max(mx, bits);
    mn = min(mn, bits);
  });
  for (int o = 32; o > 0; o >>= 1) {
    c += (uint32_t)__shfl_xor((int)c, o, 64);
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
    mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&sh.red[0], c);
    atomicMin(&sh.red[1], mn);
    atomicMax(&sh.red[2], mx);
  }
  __syncthreads();
}

// terms of <= kKtopTiny postings: one wave per term (four per workgroup), the
// alive keys sorted descending by a wave bitonic network (lane i: the i-th best)
__global__ __launch_bounds__(kThreads) void k_ktop_tiny(ScoreJob j) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t x = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6); x < j.n_tiny; x += gridDim.x * (kThreads / 64)) {
  const uint32_t t = j.kt_tiny[x];  // (a wave per term: the loop is wave-uniform)
  const uint64_t b = j.off[t];
  const uint32_t n = (uint32_t)(j.off[t + 1] - b);
  uint64_t key = 0;
  if (lane < n) {
    const uint32_t d = j.doc[b + lane];
    if (!j.alive || ((j.alive[d >> 5] >> (d & 31u)) & 1u)) key = make_key(j.psc[b + lane], d);
  }
  const uint32_t na = (uint32_t)__popcll(__ballot(key != 0));
  if (na == 0) continue;
  for (uint32_t k = 2; k <= 64; k <<= 1)
    for (uint32_t h = k >> 1; h > 0; h >>= 1) {
      const uint32_t lo32 = (uint32_t)__shfl_xor((int)(uint32_t)key, (int)h, 64);
      const uint32_t hi32 = (uint32_t)__shfl_xor((int)(uint32_t)(key >> 32), (int)h, 64);
      const uint64_t other = ((uint64_t)hi32 << 32) | lo32;
      const bool desc = (lane & k) == 0, lower = (lane & h) == 0;
      key = (lower == desc) ? (key > other ? key : other) : (key < other ? key : other);
    }
  // lane i holds the i-th best key (zeros -- dead or absent postings -- last)
  if (lane == 0) j.ktop[(size_t)t * kNumTopK] = key_score(key);
  for (uint32_t kk = 1; kk < kNumTopK; ++kk)
    if (kTopKs[kk] <= na && lane == kTopKs[kk] - 1) j.ktop[(size_t)t * kNumTopK + kk] = key_score(key);
  if (j.ladder)
    for (uint32_t kk = 0; kk < kNumLadderExtra; ++kk)
      if (kLadderExtra[kk] <= na && lane == kLadderExtra[kk] - 1)
        j.ladder[(size_t)t * kNumLadderExtra + kk] = key_score(key);
  }
}

// one workgroup per term of <= kKtopChunk postings
__global__ __launch_bounds__(kThreads) void k_ktop(ScoreJob j, uint32_t n) {
  __shared__ KtopShared sh;
  for (uint32_t w = blockIdx.x; w < n; w += gridDim.x) {
  __syncthreads();  // the previous term's LDS reads are done
  const uint32_t t = j.kt_terms[w];
  const uint64_t b = j.off[t];
  const uint32_t np = (uint32_t)(j.off[t + 1] - b);
  ktop_reduce(j, b, 0, np, sh);
  const uint32_t na = sh.red[0];
  if (threadIdx.x == 0 && na) j.ktop[(size_t)t * kNumTopK] = __uint_as_float(sh.red[2]);  // K = 1: the maximum
  ktop_finish(j, t, na, sh, [&](auto&& f) {
    ktop_each_posting(j, b, 0, np, [&](bool ok, float sv, uint32_t d) { f(ok, make_key(sv, d)); });
  });
  }
}

// one workgroup per kKtopChunk-posting chunk of a long term: the chunk's alive
// count and extremes (atomics into the term's slots) and its KM best keys
__global__ __launch_bounds__(kThreads) void k_ktop_part(ScoreJob j, uint32_t n_chunks) {
  __shared__ KtopShared sh;
  constexpr uint32_t KM = kKtopKM;
  for (uint32_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
  __syncthreads();  // the previous chunk's LDS reads are done
  const uint32_t bt = j.kc_big[c];
  const uint32_t t = j.kb_terms[bt];
  const uint64_t b = j.off[t];
  const uint32_t n = (uint32_t)(j.off[t + 1] - b);
  const uint32_t p0 = j.kc_start[c], p1 = min(n, p0 + kKtopChunk);
  ktop_reduce(j, b, p0, p1, sh);
  const uint32_t na = sh.red[0];
  if (threadIdx.x == 0 && na) {
    atomicAdd(&j.kb_stat[bt], na);
    atomicMin(&j.kb_stat[j.n_big + bt], sh.red[1]);
    atomicMax(&j.kb_stat[2 * j.n_big + bt], sh.red[2]);
  }
  uint64_t T = 0;
  if (na > KM) {
    T = select_kth(KM, sh.hist, sh.scratch, [&](auto&& f) {
      ktop_each_posting(j, b, p0, p1, [&](bool ok, float sv, uint32_t d) { if (ok) f(make_key(sv, d)); });
    });
  }
  ktop_each_posting(j, b, p0, p1, [&](bool ok, float sv, uint32_t d) {
    const uint64_t key = make_key(sv, d);
    wave_append(ok && key >= T, key, sh.top, &sh.n_top, KM);
  });
  __syncthreads();
  const uint32_t nt = min(na, KM);
  uint64_t* out = j.kc_keys + (size_t)c * KM;
  for (uint32_t i = threadIdx.x; i < nt; i += kThreads) out[i] = sh.top[i];
  if (threadIdx.x == 0) j.kc_cnt[c] = nt;
  }
}

// one workgroup per long term: its K-th best scores over its chunks' best keys
__global__ __launch_bounds__(kThreads) void k_ktop_big(ScoreJob j) {
  __shared__ KtopShared sh;
  constexpr uint32_t KM = kKtopKM;
  for (uint32_t bt = blockIdx.x; bt < j.n_big; bt += gridDim.x) {
  __syncthreads();  // the previous term's LDS reads are done
  const uint32_t t = j.kb_terms[bt];
  const uint32_t na = j.kb_stat[bt], mx = j.kb_stat[2 * j.n_big + bt];
  if (threadIdx.x == 0) {
    sh.n_top = 0;
    if (na) j.ktop[(size_t)t * kNumTopK] = __uint_as_float(mx);  // K = 1: the maximum
  }
  __syncthreads();
  const uint32_t c0 = j.kb_chunk0[bt], c1 = j.kb_chunk0[bt + 1];
  ktop_finish(j, t, na, sh, [&](auto&& f) {
    for (uint32_t c = c0; c < c1; ++c) {
      const uint32_t cn = j.kc_cnt[c];
      const uint64_t* keys = j.kc_keys + (size_t)c * KM;
      for (uint32_t i0 = 0; i0 < cn; i0 += kThreads) {
        const uint32_t i = i0 + threadIdx.x;
        f(i < cn, i < cn ? keys[i] : 0ull);
      }
    }
  });
  }
}

// a background scoring's grid: at most j.grid_cap workgroups (0: one per item)
static inline uint32_t capped(const ScoreJob& j, uint64_t n) {
  const uint64_t g = j.grid_cap && n > j.grid_cap ? j.grid_cap : n;
  return (uint32_t)(g < 0x7FFFFFFFull ? g : 0x7FFFFFFFull);
}

hipError_t launch_score(const ScoreJob& j, uint32_t n_chunks, hipStream_t s) {
  if (!n_chunks) return hipSuccess;
  k_score<<<capped(j, n_chunks), kThreads, 0, s>>>(j, n_chunks);
  return hipGetLastError();
}

hipError_t launch_bucket(const ScoreJob& j, uint32_t n_chunks, uint32_t n_docs, hipStream_t s) {
  if (!n_chunks) return hipSuccess;
  k_bucket<<<capped(j, n_chunks), kThreads, 0, s>>>(j, n_docs, n_chunks);
  return hipGetLastError();
}

hipError_t launch_tsub(const ScoreJob& j, uint32_t n_docs, hipStream_t s) {
  const uint64_t n = (uint64_t)j.n_tterm * (j.n_tiles + 1);
  if (!n || !j.tsub) return hipSuccess;
  if ((n + kThreads - 1) / kThreads > 0x7FFFFFFFull) return hipErrorInvalidValue;
  k_tsub<<<capped(j, (n + kThreads - 1) / kThreads), kThreads, 0, s>>>(j, n_docs);
  return hipGetLastError();
}

hipError_t launch_ktop(const ScoreJob& j, uint32_t n_terms, uint32_t n_chunks, uint32_t n_big, hipStream_t s) {
  if (j.n_tiny) {
    k_ktop_tiny<<<capped(j, (j.n_tiny + kThreads / 64 - 1) / (kThreads / 64)), kThreads, 0, s>>>(j);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (n_terms) {
    k_ktop<<<capped(j, n_terms), kThreads, 0, s>>>(j, n_terms);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (n_chunks) {
    k_ktop_part<<<capped(j, n_chunks), kThreads, 0, s>>>(j, n_chunks);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (n_big) k_ktop_big<<<capped(j, n_big), kThreads, 0, s>>>(j);
  return hipGetLastError();
}

// n u32 from src to dst in steps of the grid: a background scoring's read-back
// into pinned host memory as a capped kernel on its low-priority stream instead
// of a copy-engine transfer (the read-backs of a rescore held searches up:
// tools/rescore_stall.py)
__global__ __launch_bounds__(kThreads) void k_copy32(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src,
                                                    uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kThreads)
    dst[i] = src[i];
}

hipError_t launch_copy32(uint32_t* dst, const uint32_t* src, uint64_t n, uint32_t grid_cap, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint64_t want = (n + kThreads - 1) / kThreads;
  const uint64_t g = grid_cap && want > grid_cap ? grid_cap : want;
  k_copy32<<<(uint32_t)(g < 0x7FFFFFFFull ? g : 0x7FFFFFFFull), kThreads, 0, s>>>(dst, src, n);
  return hipGetLastError();
}

hipError_t launch_merge(uint32_t n_shards, uint32_t n_queries, uint32_t k, const float* score, const uint32_t* doc,
                        const uint32_t* n, float* out_score, uint32_t* out_doc, uint32_t* out_shard, uint32_t* out_n,
                        hipStream_t s) {
  if (n_queries == 0) return hipSuccess;
  if ((uint64_t)n_shards * k <= kMergeCap) {
    k_merge_rank<<<n_queries, kThreads, 0, s>>>(n_shards, n_queries, k, score, doc, n, out_score, out_doc, out_shard,
                                                 out_n);
    return hipGetLastError();
  }
  k_merge<<<(n_queries + kThreads - 1) / kThreads, kThreads, 0, s>>>(n_shards, n_queries, k, score, doc, n,
                                                                     out_score, out_doc, out_shard, out_n);
  return hipGetLastError();
}

}  // namespace fg
