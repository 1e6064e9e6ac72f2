// gfx950 (CDNA4, wave64) kernels for fugu's query hot path: conjunctive
// posting-list intersection + BM25 + top-k.
//
// Pipeline per planned batch:
//   k_conj    one workgroup per work item = (query, 2048-posting chunk of the
//             lead list).  Each wave owns 512 consecutive lead candidates and
//             probes the other lists in tantivy's intersection order
//             (query/intersection.rs: children sorted by cost).  A probe either
//             stages the covering segment of the probed list in the wave's LDS
//             slice (dense lists, merge-cost bytes) or binary-searches HBM
//             through the per-128-block skip array (sparse candidates).
//             Survivors are scored with tantivy's Bm25Weight arithmetic in f32
//             (query/bm25.rs), compacted with ballot + popcount into LDS, and
//             cut to the chunk's exact top-k by an LDS radix select on a 64-bit
//             (score, ~doc) key.  The chunk's k-th key raises a per-query
//             threshold (atomicMax) that later chunks use to drop hits early.
//   k_filter  drops every chunk hit below the final per-query threshold and
//             appends the rest to a per-query candidate list.
//   k_final   per query: exact top-k select + bitonic sort, writes (score, doc)
//             in (score desc, doc asc) order (collector/top_collector.rs).
// No MFMA: this is integer/indexing work bound by HBM (roofline in DESIGN.md).
#include <hip/hip_runtime.h>

#include "fg_internal.h"

namespace fg {
namespace {

constexpr uint32_t kInvalid = 0xFFFFFFFFu;

__device__ inline uint32_t lane_id() { return threadIdx.x & 63; }
__device__ inline uint32_t wave_id() { return threadIdx.x >> 6; }

__device__ inline uint32_t wave_min(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
__device__ inline uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
// Ordering point for LDS traffic between lanes of one wave (no workgroup barrier).
__device__ inline void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// lower_bound of x in d[lo, hi) using the skip array sk (last doc of each
// 128-entry block of the same list).  Entries before lo are < x.
__device__ inline uint32_t lower_bound_skip(const uint32_t* __restrict__ d, const uint32_t* __restrict__ sk,
                                            uint32_t lo, uint32_t hi, uint32_t x) {
  if (lo >= hi) return hi;
  uint32_t blo = lo >> 7, bhi = (hi - 1) >> 7;
  while (blo < bhi) {  // first block in [blo, bhi] whose last doc >= x (or bhi)
    uint32_t mid = (blo + bhi) >> 1;
    if (sk[mid] < x) blo = mid + 1; else bhi = mid;
  }
  uint32_t a = max(lo, blo << 7), b = min(hi, (blo << 7) + kBlock);
  while (a < b) {
    uint32_t mid = (a + b) >> 1;
    if (d[mid] < x) a = mid + 1; else b = mid;
  }
  return a;
}

// Branchless lower_bound of every live item over the SAME range [base,
// base+n) of arr: the step count depends only on n, so the kItems searches of
// a lane advance in lockstep and their loads overlap (ILP instead of a
// dependent chain per item).  Entries at index >= end read as +inf.
template <bool kGuard>
__device__ inline void lower_bound_lockstep(const uint32_t* __restrict__ arr, uint32_t base, uint32_t n, uint32_t end,
                                            const uint32_t (&x)[kItems], uint32_t live, uint32_t (&res)[kItems]) {
  uint32_t b[kItems];
#pragma unroll
  for (uint32_t j = 0; j < kItems; ++j) b[j] = base;
  while (n > 1) {
    const uint32_t half = n >> 1;
#pragma unroll
    for (uint32_t j = 0; j < kItems; ++j) {
      if (live & (1u << j)) {
        const uint32_t idx = b[j] + half - 1;
        const uint32_t v = (!kGuard || idx < end) ? arr[idx] : kInvalid;
        b[j] = v < x[j] ? b[j] + half : b[j];
      }
    }
    n -= half;
  }
#pragma unroll
  for (uint32_t j = 0; j < kItems; ++j) {
    uint32_t r = b[j];
    if (n == 1 && (live & (1u << j))) {
      const uint32_t v = (!kGuard || r < end) ? arr[r] : kInvalid;
      r += v < x[j] ? 1u : 0u;
    }
    res[j] = r;
  }
}

// One query term's score for one doc: Should(text:t, name:t) under a
// SumCombiner that starts at 0.0 (query/union, query/bm25.rs score()).
__device__ inline float term_score(uint32_t tfp, uint32_t fnp, float wt, float wn, const float* cache) {
  float s = 0.0f;
  uint32_t tt = tfp & 0xFFFFu, tn = tfp >> 16;
  if (tt) {
    float tf = (float)tt;
    s += wt * (tf / (tf + cache[fnp & 0xFFu]));
  }
  if (tn) {
    float tf = (float)tn;
    s += wn * (tf / (tf + cache[256 + (fnp >> 8)]));
  }
  return s;
}

// ---------------------------------------------------------------- block scan helpers
// Exclusive prefix over the workgroup of one u32 per thread (256 threads).
__device__ inline uint32_t block_exclusive_scan(uint32_t v, uint32_t* scratch /*[4]*/, uint32_t* total) {
  uint32_t lane = lane_id(), w = wave_id();
  uint32_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
    if (lane >= (uint32_t)o) incl += y;
  }
  if (lane == 63) scratch[w] = incl;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (uint32_t i = 0; i < kThreads / 64; ++i) {
    uint32_t x = scratch[i];
    if (i < w) base += x;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return base + incl - v;
}

// Exact select over n unique 64-bit keys in LDS: returns T such that exactly
// min(K, n) keys are >= T (T = 0 when n <= K).  11-bit radix digits from the
// top, stopping as soon as the digit holding the K-th key is fully taken.
__device__ uint64_t select_topk_threshold(const uint64_t* keys, uint32_t n, uint32_t K, uint32_t* hist,
                                          uint32_t* scratch) {
  if (n <= K) return 0;
  uint64_t prefix = 0;
  uint32_t need = K;
  const uint32_t tid = threadIdx.x;
  for (int r = 0; r < 6; ++r) {
    const int sh = r < 5 ? 53 - 11 * r : 0;
    const int width = r < 5 ? 11 : 9;
    const int top = sh + width;  // bits >= top must equal prefix
    for (uint32_t i = tid; i < kHistBins; i += kThreads) hist[i] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < n; i += kThreads) {
      uint64_t k = keys[i];
      bool match = top >= 64 ? true : ((k >> top) == (prefix >> top));
      if (match) atomicAdd(&hist[(uint32_t)(k >> sh) & ((1u << width) - 1)], 1u);
    }
    __syncthreads();
    // descending digit order: thread t owns digits [2047-8t-7, 2047-8t]
    uint32_t local[8];
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      local[i] = hist[kHistBins - 1 - (tid * 8 + i)];
      s += local[i];
    }
    uint32_t tot;
    uint32_t before = block_exclusive_scan(s, scratch, &tot);
    // the thread whose range contains the need-th key (counting from the top)
    if (before < need && before + s >= need) {
      uint32_t c = before;
      for (int i = 0; i < 8; ++i) {
        if (c + local[i] >= need) {
          uint32_t digit = kHistBins - 1 - (tid * 8 + i);
          scratch[4] = digit;
          scratch[5] = need - c;      // need within the digit
          scratch[6] = local[i];      // keys in the digit
          break;
        }
        c += local[i];
      }
    }
    __syncthreads();
    uint32_t digit = scratch[4], nd = scratch[5], cnt = scratch[6];
    __syncthreads();
    prefix |= (uint64_t)digit << sh;
    need = nd;
    if (cnt == need) break;  // every key of this digit is in: threshold exact
  }
  return prefix;
}

// Bitonic sort (descending) of P keys in LDS, P a power of two <= 4096.
__device__ void bitonic_sort_desc(uint64_t* s, uint32_t P) {
  for (uint32_t k = 2; k <= P; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < P; i += kThreads) {
        uint32_t ixj = i ^ j;
        if (ixj > i) {
          uint64_t a = s[i], b = s[ixj];
          bool desc = (i & k) == 0;
          if ((a < b) == desc) { s[i] = b; s[ixj] = a; }
        }
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------- k_conj
struct ConjShared {
  // wave staging slices; reused for keys + histogram after probing
  alignas(16) uint32_t seg[4][kSeg];
  uint32_t scratch[8];
  uint32_t n_keys;
  uint32_t work_q;
};
static_assert(sizeof(uint64_t) * kChunk + sizeof(uint32_t) * kHistBins <= sizeof(uint32_t) * 4 * kSeg,
              "keys + histogram must fit in the staging area");

__global__ __launch_bounds__(kThreads) void k_conj(DevIndex ix, DevPlan pl) {
  __shared__ ConjShared sh;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = wave_id();

  // XCD-aware remap: consecutive work items (adjacent regions of the same
  // lists) land on one XCD's L2.  Bijective for any grid size.
  const uint32_t nwg = gridDim.x, bid = blockIdx.x;
  const uint32_t xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const uint32_t w = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);

  const uint32_t q = pl.chunk_q[w];
  const uint32_t c = w - pl.chunk_start[q];
  const uint32_t m = pl.q_m[q];
  const uint32_t* terms = pl.q_terms + (size_t)q * kMaxTerms;
  const uint32_t K = pl.k;

  const uint32_t t0 = terms[0];
  const uint64_t base0 = ix.off[t0];
  const uint32_t df0 = pl.q_lead_df[q];
  const uint32_t cbeg = c * kChunk;
  const uint32_t cnt = min(kChunk, df0 - cbeg);
  const uint64_t thr = __hip_atomic_load(&pl.thresh[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

  // candidates of this wave: idx = wv*512 + j*64 + lane (coalesced per j)
  uint32_t doc[kItems];
  uint32_t fnp[kItems];
  float acc_r[kItems], acc_o[kItems];
  uint32_t live = 0;
#pragma unroll
  for (uint32_t j = 0; j < kItems; ++j) {
    uint32_t idx = wv * kWaveSpan + j * 64 + lane;
    doc[j] = idx < cnt ? ix.doc[base0 + cbeg + idx] : kInvalid;
    if (idx < cnt) live |= 1u << j;
    fnp[j] = kInvalid;
    acc_r[j] = 0.0f;
    acc_o[j] = 0.0f;
  }

  uint32_t* seg = sh.seg[wv];
  for (uint32_t i = 1; i < m; ++i) {
    // wave-uniform bounds of the live candidates
    uint32_t lmin = kInvalid, lmax = 0;
#pragma unroll
    for (uint32_t j = 0; j < kItems; ++j) {
      if (live & (1u << j)) { lmin = min(lmin, doc[j]); lmax = max(lmax, doc[j]); }
    }
    lmin = wave_min(lmin);
    lmax = wave_max(lmax);
    if (lmin == kInvalid) break;  // nothing left in this wave

    const uint32_t ti = terms[i];
    const uint64_t bi = ix.off[ti];
    const uint32_t ni = (uint32_t)(ix.off[ti + 1] - bi);
    const uint32_t* di = ix.doc + bi;
    const uint32_t* ski = ix.skip + ix.skip_off[ti];
    const float wt = ix.w_text[ti], wn = ix.w_name[ti];
    // range of list i that can hold the wave's candidates: lanes 0 and 1
    uint32_t bound = 0;
    if (lane < 2) bound = lower_bound_skip(di, ski, 0, ni, lane == 0 ? lmin : lmax + 1);
    const uint32_t LO = (uint32_t)__shfl((int)bound, 0, 64);
    const uint32_t HI = (uint32_t)__shfl((int)bound, 1, 64);
    const uint32_t len = HI - LO;

    uint32_t pos[kItems];
    if (len <= kSeg) {
      // dense: stage list i's covering segment in this wave's LDS slice
      // (8 loads in flight per lane), then search it
      for (uint32_t k0 = 0; k0 < len; k0 += 8 * 64) {
        uint32_t v[8];
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) {
          const uint32_t k = k0 + u * 64 + lane;
          v[u] = k < len ? di[LO + k] : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) {
          const uint32_t k = k0 + u * 64 + lane;
          if (k < len) seg[k] = v[u];
        }
      }
      wave_lds_sync();
      uint32_t p[kItems];
      lower_bound_lockstep<false>(seg, 0, len, len, doc, live, p);
#pragma unroll
      for (uint32_t j = 0; j < kItems; ++j)
        pos[j] = ((live >> j) & 1u) && p[j] < len && seg[p[j]] == doc[j] ? LO + p[j] : kInvalid;
      wave_lds_sync();
    } else {
      // sparse candidates: skip-array search over the wave's block range,
      // then a full-block search (guarded past the list end), all in HBM
      const uint32_t blo = LO >> 7, bhi = (HI - 1) >> 7;
      uint32_t blk[kItems];
      lower_bound_lockstep<false>(ski, blo, bhi - blo + 1, 0, doc, live, blk);
#pragma unroll
      for (uint32_t j = 0; j < kItems; ++j) blk[j] = min(blk[j], bhi) << 7;
      // per item block bases differ, so search each block in lockstep by offset
      uint32_t b[kItems];
#pragma unroll
      for (uint32_t j = 0; j < kItems; ++j) b[j] = blk[j];
      for (uint32_t n = kBlock; n > 1;) {
        const uint32_t half = n >> 1;
#pragma unroll
        for (uint32_t j = 0; j < kItems; ++j) {
          if (live & (1u << j)) {
            const uint32_t idx = b[j] + half - 1;
            const uint32_t v = idx < ni ? di[idx] : kInvalid;
            b[j] = v < doc[j] ? b[j] + half : b[j];
          }
        }
        n -= half;
      }
#pragma unroll
      for (uint32_t j = 0; j < kItems; ++j) {
        pos[j] = kInvalid;
        if (live & (1u << j)) {
          uint32_t r = b[j];
          uint32_t v = r < ni ? di[r] : kInvalid;
          if (v < doc[j]) { ++r; v = r < ni ? di[r] : kInvalid; }
          if (v == doc[j]) pos[j] = r;
        }
      }
    }
    // score the hits of list i; drop the misses
#pragma unroll
    for (uint32_t j = 0; j < kItems; ++j) {
      if (!(live & (1u << j))) continue;
      if (pos[j] == kInvalid) { live &= ~(1u << j); continue; }
      if (fnp[j] == kInvalid) {
        uint32_t f = ix.fn_text[doc[j]];
        if (ix.has_name) f |= (uint32_t)ix.fn_name[doc[j]] << 8;
        fnp[j] = f;
      }
      float s = term_score(ix.tf[bi + pos[j]], fnp[j], wt, wn, ix.cache);
      if (i == 1) acc_r[j] = s; else acc_o[j] += s;
    }
  }

  // survivors: lead-list score, final sum in tantivy's order, alive bitset,
  // threshold, and compaction into the LDS key buffer
  __syncthreads();  // staging slices become the key buffer
  uint64_t* keys = reinterpret_cast<uint64_t*>(&sh.seg[0][0]);
  uint32_t* hist = reinterpret_cast<uint32_t*>(keys + kChunk);
  if (tid == 0) { sh.n_keys = 0; }
  __syncthreads();
  const float wt0 = ix.w_text[t0], wn0 = ix.w_name[t0];
#pragma unroll
  for (uint32_t j = 0; j < kItems; ++j) {
    bool keep = (live >> j) & 1u;
    uint64_t key = 0;
    if (keep) {
      uint32_t d = doc[j];
      if (ix.alive && !((ix.alive[d >> 5] >> (d & 31)) & 1u)) keep = false;
      if (keep) {
        if (fnp[j] == kInvalid) {
          uint32_t f = ix.fn_text[d];
          if (ix.has_name) f |= (uint32_t)ix.fn_name[d] << 8;
          fnp[j] = f;
        }
        uint32_t idx = wv * kWaveSpan + j * 64 + lane;
        float s0 = term_score(ix.tf[base0 + cbeg + idx], fnp[j], wt0, wn0, ix.cache);
        // Intersection::score = left + right + (0.0 + others...); a single
        // term is the union itself.
        float s = m == 1 ? s0 : (s0 + acc_r[j]) + acc_o[j];
        key = make_key(s, d);
        keep = key >= thr;
      }
    }
    unsigned long long bal = __ballot(keep);
    uint32_t nw = (uint32_t)__popcll(bal);
    if (nw) {
      uint32_t wbase = 0;
      if (lane == 0) wbase = atomicAdd(&sh.n_keys, nw);
      wbase = (uint32_t)__shfl((int)wbase, 0, 64);
      if (keep) {
        uint32_t rank = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
        keys[wbase + rank] = key;
      }
    }
  }
  __syncthreads();
  const uint32_t n = sh.n_keys;
  uint64_t* slot = pl.slot_keys + (size_t)w * K;
  if (n <= K) {
    for (uint32_t i = tid; i < n; i += kThreads) slot[i] = keys[i];
    if (tid == 0) pl.slot_cnt[w] = n;
    return;
  }
  const uint64_t T = select_topk_threshold(keys, n, K, hist, sh.scratch);
  if (tid == 0) sh.n_keys = 0;
  __syncthreads();
  for (uint32_t i0 = 0; i0 < n; i0 += kThreads) {
    uint32_t i = i0 + tid;
    bool keep = i < n && keys[i] >= T;
    uint64_t key = keep ? keys[i] : 0;
    unsigned long long bal = __ballot(keep);
    uint32_t nw = (uint32_t)__popcll(bal);
    if (nw) {
      uint32_t wbase = 0;
      if (lane == 0) wbase = atomicAdd(&sh.n_keys, nw);
      wbase = (uint32_t)__shfl((int)wbase, 0, 64);
      if (keep) slot[wbase + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = key;
    }
  }
  __syncthreads();
  if (tid == 0) {
    pl.slot_cnt[w] = sh.n_keys;  // == K (keys are unique)
    atomicMax(reinterpret_cast<unsigned long long*>(&pl.thresh[q]), (unsigned long long)T);
  }
}

// ---------------------------------------------------------------- k_filter
// One wave per work item: keep the chunk's keys >= the query's final threshold.
__global__ __launch_bounds__(kThreads) void k_filter(DevPlan pl) {
  const uint32_t w = blockIdx.x * 4 + wave_id();
  if (w >= pl.total_chunks) return;
  const uint32_t lane = lane_id();
  const uint32_t q = pl.chunk_q[w];
  const uint64_t T = pl.thresh[q];
  const uint32_t n = pl.slot_cnt[w];
  const uint64_t* slot = pl.slot_keys + (size_t)w * pl.k;
  uint64_t* out = pl.cand_keys + pl.cand_off[q];
  for (uint32_t i0 = 0; i0 < n; i0 += 64) {
    uint32_t i = i0 + lane;
    uint64_t key = i < n ? slot[i] : 0;
    bool keep = i < n && key >= T;
    unsigned long long bal = __ballot(keep);
    uint32_t nw = (uint32_t)__popcll(bal);
    if (!nw) continue;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&pl.cand_cnt[q], nw);
    base = (uint32_t)__shfl((int)base, 0, 64);
    if (keep) out[base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = key;
  }
}

// ---------------------------------------------------------------- k_final
struct FinalShared {
  alignas(16) uint64_t keys[kFinalCap];
  uint32_t hist[kHistBins];
  uint32_t scratch[8];
  uint32_t n_keys;
};

__global__ __launch_bounds__(kThreads) void k_final(DevPlan pl, float* __restrict__ out_score,
                                                     uint32_t* __restrict__ out_doc, uint32_t* __restrict__ out_n) {
  __shared__ FinalShared sh;
  const uint32_t q = blockIdx.x, tid = threadIdx.x, lane = lane_id();
  const uint32_t K = pl.k;
  const uint64_t* src = pl.cand_keys + pl.cand_off[q];
  const uint32_t n = pl.cand_cnt[q];
  uint64_t T = 0;
  if (n > kFinalCap) {
    // rare: radix select straight from HBM, 11-bit digits
    uint64_t prefix = 0;
    uint32_t need = K;
    for (int r = 0; r < 6; ++r) {
      const int shf = r < 5 ? 53 - 11 * r : 0;
      const int width = r < 5 ? 11 : 9;
      const int top = shf + width;
      for (uint32_t i = tid; i < kHistBins; i += kThreads) sh.hist[i] = 0;
      __syncthreads();
      for (uint32_t i = tid; i < n; i += kThreads) {
        uint64_t k = src[i];
        bool match = top >= 64 ? true : ((k >> top) == (prefix >> top));
        if (match) atomicAdd(&sh.hist[(uint32_t)(k >> shf) & ((1u << width) - 1)], 1u);
      }
      __syncthreads();
      uint32_t local[8], s = 0;
      for (int i = 0; i < 8; ++i) { local[i] = sh.hist[kHistBins - 1 - (tid * 8 + i)]; s += local[i]; }
      uint32_t tot;
      uint32_t before = block_exclusive_scan(s, sh.scratch, &tot);
      if (before < need && before + s >= need) {
        uint32_t c = before;
        for (int i = 0; i < 8; ++i) {
          if (c + local[i] >= need) {
            sh.scratch[4] = kHistBins - 1 - (tid * 8 + i);
            sh.scratch[5] = need - c;
            sh.scratch[6] = local[i];
            break;
          }
          c += local[i];
        }
      }
      __syncthreads();
      uint32_t digit = sh.scratch[4], nd = sh.scratch[5], cnt = sh.scratch[6];
      __syncthreads();
      prefix |= (uint64_t)digit << shf;
      need = nd;
      if (cnt == need) break;
    }
    T = prefix;
  }
  // gather keys >= T into LDS (all of them when n <= cap)
  if (tid == 0) sh.n_keys = 0;
  __syncthreads();
  for (uint32_t i0 = 0; i0 < n; i0 += kThreads) {
    uint32_t i = i0 + tid;
    uint64_t key = i < n ? src[i] : 0;
    bool keep = i < n && key >= T;
    unsigned long long bal = __ballot(keep);
    uint32_t nw = (uint32_t)__popcll(bal);
    if (nw) {
      uint32_t wbase = 0;
      if (lane == 0) wbase = atomicAdd(&sh.n_keys, nw);
      wbase = (uint32_t)__shfl((int)wbase, 0, 64);
      if (keep) sh.keys[wbase + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = key;
    }
  }
  __syncthreads();
  uint32_t nk = sh.n_keys;
  if (nk > K) {
    const uint64_t T2 = select_topk_threshold(sh.keys, nk, K, sh.hist, sh.scratch);
    // compact keys >= T2 (exactly K) to the front; read everything first
    constexpr uint32_t R = kFinalCap / kThreads;
    uint64_t v[R];
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
      const uint32_t i = r * kThreads + tid;
      v[r] = i < nk ? sh.keys[i] : 0;
    }
    __syncthreads();
    if (tid == 0) sh.n_keys = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < R; ++r) {
      const bool keep = r * kThreads + tid < nk && v[r] >= T2;
      unsigned long long bal = __ballot(keep);
      uint32_t nw = (uint32_t)__popcll(bal);
      if (nw) {
        uint32_t wbase = 0;
        if (lane == 0) wbase = atomicAdd(&sh.n_keys, nw);
        wbase = (uint32_t)__shfl((int)wbase, 0, 64);
        if (keep) sh.keys[wbase + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = v[r];
      }
    }
    __syncthreads();
    nk = sh.n_keys;
  }
  uint32_t P = 1;
  while (P < nk) P <<= 1;
  for (uint32_t i = nk + tid; i < P; i += kThreads) sh.keys[i] = 0;
  __syncthreads();
  bitonic_sort_desc(sh.keys, P);
  for (uint32_t i = tid; i < nk; i += kThreads) {
    uint64_t k = sh.keys[i];
    out_score[(size_t)q * K + i] = key_score(k);
    out_doc[(size_t)q * K + i] = key_doc(k);
  }
  if (tid == 0) out_n[q] = nk;
}

// ---------------------------------------------------------------- k_merge
// Cross-shard merge of per-shard top-k lists (each in key order) into the
// global top-k by (score desc, shard asc, doc asc): one lane per query walks
// the n_shards heads (n_shards <= 64; k <= 1024).
__global__ __launch_bounds__(kThreads) void k_merge(uint32_t n_shards, uint32_t nq, uint32_t k,
                                                     const float* __restrict__ score, const uint32_t* __restrict__ doc,
                                                     const uint32_t* __restrict__ n, float* __restrict__ out_score,
                                                     uint32_t* __restrict__ out_doc, uint32_t* __restrict__ out_shard,
                                                     uint32_t* __restrict__ out_n) {
  const uint32_t q = blockIdx.x * kThreads + threadIdx.x;
  if (q >= nq) return;
  uint32_t head[64], cnt[64];
  for (uint32_t s = 0; s < n_shards; ++s) { head[s] = 0; cnt[s] = n[(size_t)s * nq + q]; }
  uint32_t produced = 0;
  for (; produced < k; ++produced) {
    int best = -1;
    float bs = 0.0f;
    uint32_t bd = 0;
    for (uint32_t s = 0; s < n_shards; ++s) {
      if (head[s] >= cnt[s]) continue;
      const size_t at = ((size_t)s * nq + q) * k + head[s];
      const float sc = score[at];
      const uint32_t d = doc[at];
      if (best < 0 || sc > bs) { best = (int)s; bs = sc; bd = d; }
    }
    if (best < 0) break;
    out_score[(size_t)q * k + produced] = bs;
    out_doc[(size_t)q * k + produced] = bd;
    if (out_shard) out_shard[(size_t)q * k + produced] = (uint32_t)best;
    head[best]++;
  }
  out_n[q] = produced;
}

}  // namespace

hipError_t launch_merge(uint32_t n_shards, uint32_t n_queries, uint32_t k, const float* score, const uint32_t* doc,
                        const uint32_t* n, float* out_score, uint32_t* out_doc, uint32_t* out_shard, uint32_t* out_n,
                        hipStream_t s) {
  if (n_queries == 0) return hipSuccess;
  k_merge<<<(n_queries + kThreads - 1) / kThreads, kThreads, 0, s>>>(n_shards, n_queries, k, score, doc, n,
                                                                     out_score, out_doc, out_shard, out_n);
  return hipGetLastError();
}

hipError_t launch_conj(const DevIndex& ix, const DevPlan& pl, hipStream_t s) {
  if (pl.total_chunks == 0) return hipSuccess;
  k_conj<<<pl.total_chunks, kThreads, 0, s>>>(ix, pl);
  return hipGetLastError();
}

hipError_t launch_filter(const DevPlan& pl, hipStream_t s) {
  if (pl.total_chunks == 0) return hipSuccess;
  k_filter<<<(pl.total_chunks + 3) / 4, kThreads, 0, s>>>(pl);
  return hipGetLastError();
}

hipError_t launch_final(const DevPlan& pl, float* out_score, uint32_t* out_doc, uint32_t* out_n, hipStream_t s) {
  if (pl.n_queries == 0) return hipSuccess;
  k_final<<<pl.n_queries, kThreads, 0, s>>>(pl, out_score, out_doc, out_n);
  return hipGetLastError();
}

}  // namespace fg
