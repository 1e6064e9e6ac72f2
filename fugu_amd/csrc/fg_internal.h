// Internal layout shared by the host side (fugu.cpp) and the gfx950 kernels
// (kernels.hip).  See DESIGN.md §HBM layout.
#pragma once
#include <cstdint>

#include <hip/hip_runtime.h>

namespace fg {

constexpr uint32_t kBlock = 128;          // tantivy block size (bytes model only)
#ifndef FG_BUCKET
#define FG_BUCKET 4  // tools/ab_variants.py: 32 -> 4 took k_conj 1.686 -> 1.591 ms, k_disj 22.8 -> 20.2 ms
#endif
constexpr uint32_t kBucketTarget = FG_BUCKET;  // directory: expected postings per bucket
constexpr uint32_t kThreads = 256;        // 4 waves of 64 per workgroup
#ifndef FG_ITEMS
#define FG_ITEMS 8
#endif
constexpr uint32_t kItems = FG_ITEMS;     // lead candidates per lane
constexpr uint32_t kChunk = kThreads * kItems;   // 2048 lead candidates per work item
constexpr uint32_t kWaveSpan = kChunk / 4;       // 512 consecutive candidates per wave
constexpr uint32_t kMaxTerms = 16;        // terms per query (FG_MAX_TERMS)
constexpr uint32_t kMaxK = 1024;          // largest top-k the device select supports
#ifndef FG_FINALCAP
#define FG_FINALCAP 4096  // tools/ab_variants.py: 8192 -> 4096 took k_final 0.132 -> 0.083 ms (5 WGs per CU), OR k=1000 0.99 -> 0.75
#endif
constexpr uint32_t kFinalCap = FG_FINALCAP;  // candidates kept in LDS by the final select (>= kMaxK)
static_assert(FG_FINALCAP >= 1024, "the final sort runs in place for up to kMaxK keys");
#ifndef FG_RANK_DIV
#define FG_RANK_DIV 16384
#endif
#ifndef FG_RANK_GIB
#define FG_RANK_GIB 64    // env FUGU_RANK_GIB
#endif
constexpr uint32_t kRankDiv = FG_RANK_DIV;    // terms in >= 1/kRankDiv of the docs may get rank words
constexpr uint64_t kRankBudget = (uint64_t)FG_RANK_GIB << 30;    // ... densest first, within this many bytes
#ifndef FG_RANK_FACTOR
#define FG_RANK_FACTOR 4.0  // tools/ab_rank_budget.py sweep (profiles/r03/ab_rank_sweep.log); env FUGU_RANK_FACTOR
#endif
constexpr double kRankFactor = FG_RANK_FACTOR;  // ... and within this many times the snapshot's posting bytes
#ifndef FG_RANK_PLAIN_DIV
#define FG_RANK_PLAIN_DIV 32  // env FUGU_RANK_PLAIN_DIV; profiles/r05/ab/ab_rank_layout.log
#endif
// ... a term in >= 1/kRankPlainDiv of the docs gets plain rank words, a sparser
// one sparse rank words (DevIndex::srank), unless plain ones cost it less
constexpr uint32_t kRankPlainDiv = FG_RANK_PLAIN_DIV;
constexpr uint32_t kMaxDense = 32767;     // slots per kind (tmeta bits 16-30)
constexpr uint32_t kRankChunkWords = 2048;  // k_rank: words (65536 docs) per workgroup
#ifndef FG_DISJ_GPQ
#define FG_DISJ_GPQ 64
#endif
constexpr uint32_t kGroupsPerQuery = FG_DISJ_GPQ;  // k_disj / k_scan: a query's doc tiles in ~this many work items
#ifndef FG_DISJ_SPREAD
#define FG_DISJ_SPREAD 16
#endif
constexpr uint32_t kDisjSmallSpread = FG_DISJ_SPREAD;  // ... times up to this for a small batch (batch of one: x16)
#ifndef FG_GPQ
// tools/ab_variants.py (ab_group*.log, round 2): 64 -> 16 with FG_MAXGROUP 16 -> 8: k_conj 1.08 -> 1.00 ms;
// round 5 (after the XCD split and the sparse rank words), 16 -> 8 with FG_MAXGROUP 8 -> 16: headline
// k_conj + k_final 1.043 -> 1.032 ms, C3 1.112 -> 1.075 ms, identical hits (profiles/r05/ab/conj_group_r05ab.log);
// round 6 (query-time-scoring build), 8 -> 4 items: headline k_conj + k_final 1.012 -> 0.984 ms, C3 1.049 ->
// 1.046 ms (2: 0.978 / 1.065; 1: 0.981 / 1.058; 3, 5, 6 and caps 12 / 20 / 24 / 32 between or worse),
// identical hits (profiles/r06/ab/conj_group_*.log)
#define FG_GPQ 4
#endif
constexpr uint32_t kConjGroupsPerQuery = FG_GPQ;  // k_conj: a query's lead chunks in ~this many work items
#ifndef FG_MAXGROUP
#define FG_MAXGROUP 16
#endif
constexpr uint32_t kMaxGroup = FG_MAXGROUP;  // ... of at most this many chunks each
#ifndef FG_HIST_BITS
#define FG_HIST_BITS 10  // tools/ab_variants.py: 11 -> 10 took k_conj 1.110 -> 1.082 ms (LDS 40.0 -> 35.9 KB, no spills)
#endif
constexpr uint32_t kHistBits = 11;                 // radix digit width of the LDS selects
constexpr uint32_t kHistBins = 1u << kHistBits;
constexpr uint32_t kConjHistBits = FG_HIST_BITS;   // ... k_conj's (its LDS sets its occupancy)
#ifndef FG_TILE_SHIFT
#define FG_TILE_SHIFT 12
#endif
constexpr uint32_t kDisjTileShift = FG_TILE_SHIFT;   // k_disj: 4096-doc tiles
// k_disj shape (A/B builds, profiles/r03/ab/ab_disj_occ*.log): postings per
// pass, the select's digit width, waves per SIMD (3 waves / 1024 / exhaustive
// LDS tiles / 11 bits -> 5 / 512 / none / 10: OR top-1000 7.97 -> 7.02 ms, top-20
// 5.28 -> 4.59 ms, identical outputs: more waves in flight beat more postings per
// wave and the exhaustive path's LDS; then the bound-2 LDS queue (9-bit digits):
// ab_disj_queue_k*.log, OR top-20 3.92 -> 3.23 ms, top-1000 6.13 -> 5.94 ms, and the
// next-pass prefetch: ab_disj_qpf_k*.log, 3.21 -> 3.15 / 5.94 -> 5.85 ms)
#ifndef FG_DISJ_ROUND
#define FG_DISJ_ROUND 512
#endif
#ifndef FG_DISJ_HBITS
#define FG_DISJ_HBITS 9  // the queue's LDS comes out of the select's digit width
#endif
#ifndef FG_DISJ_WAVES
#define FG_DISJ_WAVES 5
#endif
#ifndef FG_DISJ_G
#define FG_DISJ_G 1  // ab_disj_g_k*.log, ab_disj_gpq_k*.log: 4 / 2 / 1 -> OR top-1000 7.00 / 6.51 / 6.13 ms, top-20 4.60 / 4.27 / 3.94 ms
#endif
#ifndef FG_DISJ_MAXGROUP
#define FG_DISJ_MAXGROUP 32
#endif
constexpr uint32_t kDisjMaxGroup = FG_DISJ_MAXGROUP;  // ... at most this many tiles per work item
constexpr uint32_t kDisjMaxPairs = 256;  // ... and at most this many (tile, Should clause) pairs (k_disj LDS)
// per-term K-th best scores kept for these K (20: the /search default limit,
// ab_ktop20_k20.log: OR top-20 k_disj 4.27 -> 4.22 ms starting from it)
constexpr uint32_t kNumTopK = 5;
constexpr uint32_t kTopKs[kNumTopK] = {1, 10, 20, 100, 1000};
// fg_index_term_ladder: the same K-th scores at the ranks between them as well
// (ascending), from which the shards of a doc-sharded namespace bound the
// namespace-wide K-th score of a term (fg_kth_floor_combine: K = 1000 over 8
// shards needs each shard's 125th).  Computed on demand, never stored.
constexpr uint32_t kNumLadderExtra = 9;
constexpr uint32_t kLadderExtra[kNumLadderExtra] = {2, 3, 5, 13, 25, 50, 125, 250, 500};
constexpr uint32_t kNumLadder = kNumTopK + kNumLadderExtra;  // FG_LADDER_LEVELS
constexpr uint32_t kLadderKs[kNumLadder] = {1, 2, 3, 5, 10, 13, 20, 25, 50, 100, 125, 250, 500, 1000};

constexpr uint32_t kMaxFacetClauses = 8;  // facet clauses per query (FG_MAX_FACET_CLAUSES)
constexpr uint32_t kFmaskChunk = 8192;    // facet postings per k_fmask workgroup
constexpr uint32_t kScanMaxGroup = 32;    // k_scan: at most this many 4096-doc tiles per work item

constexpr uint32_t kModeAnd = 0;
constexpr uint32_t kModeOr = 1;

// Per-query running-threshold histograms (DevPlan::hist): every work item adds
// the exact scores of the hits it keeps; the largest bin edge with at least k
// counted docs at or above it is a lower bound of the query's k-th best score
// across ALL the query's work items (and across the shards of a linked group).
constexpr uint32_t kQBins = 512;

// DevPlan::q_m packing: bits 0-7 terms in q_terms, 8-15 Must clauses (k_conj
// queries; 0 for k_disj queries), 16-23 MustNot clauses.  q_terms holds, per
// query, k_conj: [Must (cost order)][MustNot][Should (clause order)];
// k_disj: [Should (clause order)][MustNot].
__host__ __device__ inline uint32_t qm_terms(uint32_t qm) { return qm & 0xFFu; }
__host__ __device__ inline uint32_t qm_must(uint32_t qm) { return (qm >> 8) & 0xFFu; }
__host__ __device__ inline uint32_t qm_not(uint32_t qm) { return (qm >> 16) & 0xFFu; }
__host__ __device__ inline uint32_t qm_pack(uint32_t m, uint32_t nm, uint32_t nx) { return m | (nm << 8) | (nx << 16); }

// Rank words (DevIndex::rank): one u64 per 32 docs, the low half the docs'
// presence bits, the high half the number of the term's postings before the
// word's first doc.  (40 presence bits + a 24-bit rank per word -- 1.25x the docs
// per 128-B line -- measured slower: profiles/r04/ab/ab_and.log.)
__host__ __device__ inline uint32_t rank_word(uint32_t d) { return d >> 5; }
// the term's posting position of doc d from its rank word, or 0xFFFFFFFF (absent)
__host__ __device__ inline uint32_t rank_pos(uint64_t x, uint32_t d) {
#if defined(__HIP_DEVICE_COMPILE__)
  // recompute the bit from d after the word's load instead of keeping it live
  // across the load (without this k_conj spills 14 VGPRs: 1.06 -> 1.41 ms,
  // profiles/r04/ab/spilled_ab_and.log)
  asm volatile("" : "+v"(d));
#endif
  const uint32_t b = d & 31u;
  if (!((x >> b) & 1ull)) return 0xFFFFFFFFu;
  const uint32_t below = (uint32_t)x & ((1u << b) - 1u);
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)(x >> 32) + (uint32_t)__popc(below);
#else
  return (uint32_t)(x >> 32) + (uint32_t)__builtin_popcount(below);
#endif
}

// Sparse rank words (DevIndex::srank, rank-kind slots above n_prank): per
// 1024-doc block one u64, the low half a bit per 32-doc word of the block that
// holds any of the term's docs, the high half the index in srank_w of the
// block's first such word; srank_w holds only those words, in the rank-word
// format above, after a zero word at index 0 (the word of every doc no sparse
// term holds: a probe loads it unconditionally, with no predicate kept live
// across the load).  A probe is the block's 8-B load, then the word's.  A term
// in 1/2000 of the docs takes ~1/25 of its plain rank words' bytes.
__host__ __device__ inline uint32_t srank_block(uint32_t d) { return d >> 10; }
// the srank_w index of doc d's word from its block entry (0: the zero word)
__host__ __device__ inline uint32_t srank_index(uint64_t e, uint32_t d) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(d));  // as rank_pos: nothing derived from d stays live across the word's load
#endif
  const uint32_t w = (d >> 5) & 31u;
  const uint32_t below = (uint32_t)e & ((1u << w) - 1u);
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t i = (uint32_t)(e >> 32) + (uint32_t)__popc(below);
#else
  const uint32_t i = (uint32_t)(e >> 32) + (uint32_t)__builtin_popcount(below);
#endif
  return ((e >> w) & 1ull) ? i : 0u;
}

// u8 bounds of a score range [0, M] (k_disj's sub-tile maxima): a score s as
// the least q with q8_bound(q, M) >= s; q8_bound(255, M) = M covers every
// rounding.  The kernels compute q8_bound with the same f32 operations
// (-ffp-contract=off), so the bound holds bit for bit.
__host__ __device__ inline float q8_step(float M) { return M * (1.0f / 255.0f); }
__host__ __device__ inline float q8_bound(uint32_t q, float M) { return q >= 255u ? M : (float)q * q8_step(M); }
__host__ __device__ inline uint32_t quant8(float s, float M) {
  const float st = q8_step(M);
  if (!(st > 0.0f) || !(s < M)) return 255u;
  uint32_t q = (uint32_t)fminf(254.0f, ceilf(s / st));
  while (q < 255u && q8_bound(q, M) < s) ++q;
  return q;
}
constexpr uint32_t kSubShift = 9;  // 512-doc blocks: 8 per k_disj tile

// tmeta of a term: bits 0-7 = B_t (bucket shift), 8-15 = S_t (search steps),
// 16-30 = rank slot + 1 (0: none), bit 31 = set with a slot (the round-1 f32 score tables, bit 31
// clear, went with the precomputed scores);
// rank-kind slots 1..n_prank are plain rank words, the ones above sparse (srank)
__host__ __device__ inline uint32_t meta_slot(uint32_t meta) { return (meta >> 16) & 0x7FFFu; }
__host__ __device__ inline bool meta_rank(uint32_t meta) { return (meta >> 31) != 0; }

// Device view of one namespace snapshot (all pointers device-resident).
//
// Per term t the postings are doc[off[t] .. off[t+1]) (ascending) with tfn[]
// (the posting's term frequency and its doc's fieldnorm id) alongside, and a
// doc -> position directory: bucket b covers docs [b << B_t, (b+1) << B_t) and
// dir[dir_off[t] + b] = first position in the list with doc >= b << B_t (the
// last entry is df_t).  B_t is chosen so a bucket holds ~kBucketTarget (4)
// postings; a probe is one directory load and a <= S_t step search inside one
// or two lines.  The densest terms (within a byte budget) additionally get
// RANK WORDS: one u64 per 32 docs, the low half the docs' presence bits, the
// high half the number of the term's postings before the word's first doc.  A
// probe is one 8-B load; on a hit the posting's position is rank + popcount(bits
// below the doc), and its tfn one 2-B load.  Scattered single-dword probes each
// move a 128-B line (profiles/r02_start: tools/calib_fetch gather_lines), and a
// line of rank words covers 512 docs, so the candidates of a long lead list
// share lines.
//
// Scores follow the statistics of the moment, as tantivy's TermScorer's do
// (src/db/search.rs:162 -> query/bm25.rs Bm25Weight::score).  While a
// snapshot's statistics are the ones it was built with, its postings' scores
// are the build's (psc: one 4-B load, k_score computed them once).  After a
// commit elsewhere in the namespace changed the statistics (fg_index_rescore),
// the kernels form them AT QUERY TIME instead: w_text * (tf / (tf + cache[fn]))
// (+ the name field's part) from the posting's payload (tfn), the query's
// per-clause weights (DevPlan::q_wt / q_wn) and the snapshot's tf cache
// (DevIndex::cache, set by the plan) -- so a commit only builds its new segment
// and the older ones keep every device array.  The MaxScore bounds (bmax, tmax,
// tsub, tmaxs, cmax) are the maxima under the build's statistics; a plan scales
// them by a per-clause factor q_rup >= the largest ratio of a posting's current
// score to its build-time one (1 exactly when the statistics are the build's).
constexpr uint32_t kTfEsc = 255;  // tfn's tf byte: >= this -> the exact tf is in esc_pos / esc_tf
__host__ __device__ inline uint32_t tfn_pack(uint32_t tf, uint32_t fn) { return (fn << 8) | (tf < kTfEsc ? tf : kTfEsc); }
struct DevIndex {
  const uint32_t* doc;       // [P] doc ids, CSR by term, ascending within a term
  const float* psc;          // [P] the posting's score under the statistics the snapshot was BUILT with
                             //     (k_score, tantivy's f32 order): what a plan over snapshots whose
                             //     statistics are still the build's reads (DevPlan::feat without kFQt)
  const uint16_t* tfn;       // [P] (fn_text[doc] << 8) | min(tf_text, 255): tf_text 0 = no text occurrence
  const uint16_t* tfn_name;  // [P] the same for the `name` field, or nullptr (no name postings)
  const uint64_t* esc_pos;   // [n_esc] postings whose tf byte is kTfEsc in either field, ascending
  const uint32_t* esc_tf;    // [n_esc] their exact tf_text | tf_name << 16
  const float* cache;        // [256 or 512] K1 * ((1 - B) + B * TABLE[id] / avgdl): text, then name (plan-set)
  const uint64_t* off;       // [V+1] posting offsets
  const uint32_t* dir;       // [D] bucket directory (positions within the list)
  const uint32_t* dir_off;   // [V] first directory entry of each term
  const uint32_t* tmeta;     // [V] meta_slot / meta_rank above
  const uint64_t* rank;      // [n_prank * rank_words] rank words, rank-kind slots 1..n_prank
  const uint64_t* srank;     // [n_srank * srank_blocks] sparse rank block entries, rank-kind slots above
  const uint64_t* srank_w;   // sparse rank words (srank_index)
  const float* tmaxs;        // [V] largest posting score of each term (build statistics)
  const uint32_t* alive;     // [ceil(N/32)] alive bitset, or nullptr (no deletes)
  const float* bmax;         // [D] parallel to dir: max term score of the postings in each bucket
  const float* tmax;         // tile maxima (k_disj tiles) of the terms with B_t <= kDisjTileShift
  const uint32_t* toff;      // [V] first tmax / tdir entry of each term (n_tiles + 1 per term), or
                             //     0xFFFFFFFF (bucket >= tile: use bmax)
  const uint32_t* tdir;      // tile directory: tdir[toff[t] + i] = first posting of t at doc >= i << kDisjTileShift
  const uint64_t* tsub;      // parallel to tmax: byte b = the largest posting score among the tile's docs
                             //     [b << kSubShift, (b + 1) << kSubShift) quantized up against the tile maximum
                             //     (q8_bound); a bucket wider than a block counts in every block it covers
  const float* cmax;         // [score chunks] largest posting score of each kChunk-posting chunk of a
                             //     list (block-max: k_conj skips a lead chunk that cannot reach the threshold)
  const uint32_t* coff;      // [V] index of each term's first chunk in cmax
  const uint32_t* fdoc;      // [PF] facet postings (doc ids, ascending), CSR by facet term
  const uint64_t* foff;      // [VF+1]
  uint64_t n_esc;
  uint32_t n_docs;
  uint32_t n_terms;
  uint32_t has_name;
  uint32_t n_fterms;
  uint32_t rank_words;       // words per plain rank-kind term: ceil(N / 32)
  uint32_t n_prank;          // plain rank-kind slots
  uint32_t srank_blocks;     // block entries per sparse rank-kind term: ceil(N / 1024)
};

// The exact tf_text | tf_name << 16 of posting p whose tf byte escaped (binary
// search of the snapshot's escape list; rare: tf >= 255)
__host__ __device__ inline uint32_t tf_escaped(const uint64_t* esc_pos, const uint32_t* esc_tf, uint64_t n, uint64_t p) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (esc_pos[mid] < p) lo = mid + 1; else hi = mid;
  }
  return lo < n ? esc_tf[lo] : 0u;
}

// Bm25Weight::score in tantivy's f32 operation order (query/bm25.rs: weight *
// (tf / (tf + cache[fieldnorm_id]))) for one field.  -ffp-contract=off and IEEE
// f32 division: bit-identical to the host arithmetic (fugu.cpp, the oracle).
__host__ __device__ inline float field_score(uint32_t tf, uint32_t fn, float w, const float* cache) {
  const float f = (float)tf;
  return w * (f / (f + cache[fn]));
}

// Facet filters of a planned batch (DevPlan).  Every distinct clause list
// (filter) gets a doc-indexed mask in HBM built by k_fmask from the facet
// postings: 2^shift bits per doc (shift 0..3, >= the filter's clause count),
// bit i set when the doc holds clause i's facet term.  f_tab[f*256 + bits] is
// the facet union's score for that set of matching clauses, summed on the
// host in clause order from 0.0 (SumCombiner), so the kernels add one f32.
struct DevFilters {
  uint32_t n_filters;
  uint32_t n_chunks;            // k_fmask workgroups
  const uint32_t* q_filter;     // [nq] filter of each query, 0xFFFFFFFF = none
  const uint32_t* f_shift;      // [n_filters] log2(bits per doc)
  const uint64_t* f_woff;       // [n_filters] first mask word
  const float* f_tab;           // [n_filters * 256]
  const float* f_max;           // [n_filters] largest f_tab entry (upper bound of the facet score)
  const uint32_t* ch_filter;    // [n_chunks] k_fmask chunk -> filter
  const uint32_t* ch_clause;    // [n_chunks] clause index in the filter
  const uint32_t* ch_term;      // [n_chunks] facet term
  const uint32_t* ch_start;     // [n_chunks] first posting of the chunk within the term's list
  const uint32_t* f_seg;        // [n_filters] the snapshot of each filter (multi-snapshot plans), or nullptr
  uint32_t* fmask;              // workspace, zeroed per run
};

__host__ __device__ inline uint32_t filter_bits(const uint32_t* mask, uint32_t shift, uint32_t d) {
  const uint32_t bit = d << shift;  // fits: the plan rejects n_docs << shift > 2^32
  return (mask[bit >> 5] >> (bit & 31)) & ((1u << (1u << shift)) - 1u);
}

// Device view of one planned batch.  Work items (query, 2048-candidate chunk
// of the query's lead list) are ordered as a doc sweep across the batch:
// items covering similar doc ranges of different queries run together, so the
// segments of hot posting lists they probe are shared through L2 / MALL.
constexpr uint32_t kMaxPeers = 15;  // peers of one plan (fugu.h FG_MAX_PEERS, fg_plan_set_peers)

struct DevPlan {
  uint32_t n_queries;
  uint32_t total_chunks;        // k_conj items [0, n_conj) then k_disj items [n_conj, total_chunks)
  uint32_t k;
  uint32_t n_conj;
  const uint32_t* q_m;          // [nq] packed term counts (qm_terms / qm_must / qm_not)
  const uint32_t* q_terms;      // [nq * kMaxTerms] term ids (layout: qm_pack above)
  const uint32_t* q_lead_df;    // [nq] length of the lead list (0 => empty result)
  const uint32_t* work_q;       // [total_chunks] query of each work item (sweep order)
  const uint32_t* work_c;       // [total_chunks] first chunk of the item's group (k_disj: first tile)
  const uint32_t* work_n;       // [total_chunks] chunks in the item's group (k_disj: tiles)
  const uint64_t* cand_off;     // [nq+1] candidate-list capacity offsets (work items of q * k)
  const uint64_t* q_thr0;       // [nq] starting threshold key (k_disj: per-term top-K bound), 0 = none
  const float* q_ub;            // [nq * kMaxTerms] k_conj MaxScore bounds: q_ub[i] = sum over the query's
                                //     terms j >= i (intersection order) of their scaled tmaxs, i >= 1
  const float* q_wt;            // [nq * kMaxTerms] each clause's BM25 weight, text field (query time)
  const float* q_wn;            // [nq * kMaxTerms] ... and name field
  const float* q_rup;           // [nq * kMaxTerms] factor on the clause's build-time bounds (tmax, bmax,
                                //     cmax, tsub's tile maxima): >= current score / build score of any posting
  const uint32_t* q_hlo;        // [nq] f32 bits of the histogram's bin 0 lower edge
  const uint32_t* q_hsh;        // [nq] bin width: 2^q_hsh f32 ulps
  // workspace, zeroed per run (thresh and hist may be a linked group's shared ones)
  uint64_t* thresh;             // [nq] monotone lower bound on the k-th best key (published score-only)
  uint32_t* hist;               // [nq * kQBins] counted hits per score bin
  uint64_t pub_mask;            // thresholds published as key & pub_mask: ~0 exact, or score-only (linked)
  uint32_t* cand_cnt;           // [nq] keys appended to each query's candidate list
  uint64_t* cand_keys;          // [cand_off[nq]] per-query candidate lists
  uint64_t* diag;               // diagnostic builds only (-DFG_DIAG): per-workgroup stamps
  uint32_t feat;                // kernel features the plan's snapshots need: bit 2 query-time scores (a snapshot
                                // whose statistics changed since its build), with bit 0 `name` postings
                                // (tfn_name) and bit 1 escaped tf bytes (esc_pos); the kernels are instantiated
                                // per value (0, 4 = query-time, 7 = query-time with names / escapes)
  uint32_t n_single;            // k_conj: the first n_single work items belong to single-list queries
  uint32_t n_scan;              // k_scan work items (queries with no text terms), after the total_chunks
                                // k_conj / k_disj items in work_q / work_c / work_n
  // Multi-snapshot plans (several segments / doc shards / namespaces of one
  // device in ONE launch per kernel): query slot v = s * seg_nq + q is query q
  // of the batch on snapshot segs[s]; every per-query array above is indexed by
  // the slot, except thresh and hist, which are the batch query's own (shared
  // score-only by the slots of q: pub_mask).  seg_nq = 0: one snapshot (the
  // kernel's DevIndex argument).
  const DevIndex* segs;         // [n_segs] or nullptr
  uint32_t seg_nq;              // queries of the batch (slots per snapshot), 0 = one snapshot
  uint32_t n_segs;
  const uint32_t* seg_base;     // [n_segs] first doc of each snapshot in the concatenation (k_final's merged
                                // select), or nullptr when the snapshots hold >= 2^32 docs together
  DevFilters f;
  // Peer plans (fg_plan_set_peers: the other doc shards of one namespace, on
  // other devices or in other processes): every threshold this plan publishes
  // and every count it adds to its histogram also go, score-only, into the
  // peers' thresh / hist of the same batch query, so each shard prunes with the
  // hits of all of them as they are found (the cross-device form of
  // fg_plan_link's shared words)
  uint32_t n_peers;
  uint32_t* peer_hist[kMaxPeers];
  uint64_t* peer_thr[kMaxPeers];
};

// The batch query of a query slot (thresh / hist index)
__host__ __device__ inline uint32_t slot_query(const DevPlan& pl, uint32_t v) {
  return pl.seg_nq ? v % pl.seg_nq : v;
}

constexpr uint32_t kDiagPerWg = 16;  // u64 stamps per workgroup in diagnostic builds

// Key of a hit: larger is better.  (score bits << 32) | ~doc orders by
// score descending, then doc ascending (tantivy ComparableDoc order); scores
// are finite and >= 0 so the f32 bit pattern is order preserving.
__host__ __device__ inline uint64_t make_key(float score, uint32_t doc) {
  union { float f; uint32_t u; } c;
  c.f = score;
  return ((uint64_t)c.u << 32) | (uint64_t)(0xFFFFFFFFu - doc);
}
__host__ __device__ inline float key_score(uint64_t k) {
  union { float f; uint32_t u; } c;
  c.u = (uint32_t)(k >> 32);
  return c.f;
}
__host__ __device__ inline uint32_t key_doc(uint64_t k) { return 0xFFFFFFFFu - (uint32_t)k; }

// Bound tables of a snapshot build (k_score / k_bucket / k_tsub / k_ktop), run
// ONCE per segment build or merge: every posting's BM25 term score under the
// build's statistics (into a temporary), then the bounds the kernels prune with
// and the per-term K-th best scores.  A commit never runs them on an older
// segment (fg_index_rescore only scales them at query time: DevPlan::q_rup).
// Work is split into chunks of one term: k_score over postings, k_bucket over
// directory buckets; ch_* arrays are the chunk tables.
constexpr uint32_t kScoreChunk = kChunk;  // postings per k_score workgroup (= a k_conj lead chunk: cmax)
constexpr uint32_t kBucketChunk = 2048;  // buckets per k_bucket workgroup
static_assert(kScoreChunk == kChunk, "DevIndex::cmax: a k_score chunk is a k_conj lead chunk");
struct ScoreJob {
  const uint32_t* doc;
  const uint16_t* tfn;        // [P] DevIndex::tfn
  const uint16_t* tfn_name;   // [P] or nullptr
  const uint64_t* esc_pos;    // DevIndex::esc_pos / esc_tf
  const uint32_t* esc_tf;
  uint64_t n_esc;
  const uint64_t* off;        // [V+1]
  const uint32_t* dir;
  const uint32_t* dir_off;
  const uint32_t* tmeta;
  const uint32_t* toff;       // [V] tile-maxima offset or 0xFFFFFFFF
  const uint32_t* alive;      // bitset or nullptr
  const float* w_text;        // [V] idf * (1 + K1)
  const float* w_name;        // [V]
  const float* cache;         // [512] K1 * ((1 - B) + B * TABLE[id] / avgdl), text then name
  float* psc;                 // [P] out: the build's posting scores (a temporary, freed after the build)
  float* bmax;                // [D] out
  uint32_t* tmaxs;            // [V] out (f32 bits, zeroed first)
  uint32_t* tmax;             // [tiles] out (f32 bits, zeroed first)
  uint64_t* tsub;             // [tiles] out (k_tsub)
  const uint32_t* tterm;      // [tile-table terms] the term of each n_tiles + 1 tile entries, in toff order
  uint32_t n_tterm;           // tile-table terms
  uint32_t n_tiles;           // tiles per term (4096-doc k_disj tiles)
  float* ktop;                // [V * kNumTopK] out (zeroed first)
  float* ladder;              // [V * kNumLadderExtra] out (zeroed first) or nullptr: fg_index_term_ladder only
  float* cmax;               // [cmax entries] out: the largest score of each kChunk postings of a term
  const uint32_t* coff;       // [V] first cmax entry of each term
  // packed chunk tables (a chunk: terms [tf, tl], postings / directory entries
  // [e0, e1) of them; one long term's slice, or several whole short terms)
  const uint32_t* sc_tf;      // k_score chunks
  const uint32_t* sc_tl;
  const uint64_t* sc_e0;
  const uint64_t* sc_e1;
  const uint32_t* bk_tf;      // k_bucket chunks (global directory entries)
  const uint32_t* bk_tl;
  const uint32_t* bk_e0;
  const uint32_t* bk_e1;
  uint32_t n_terms;
  uint32_t grid_cap;          // at most this many workgroups per scoring launch (0: one per item)
  uint64_t n_dir;             // directory entries (dir_off of term n_terms)
  const uint32_t* kt_tiny;    // k_ktop_tiny: terms with 1..kKtopTiny postings (one wave each)
  uint32_t n_tiny;
  const uint32_t* kt_terms;   // k_ktop: terms with kKtopTiny+1..kKtopChunk postings
  // terms with more postings: k_ktop_part per chunk, then k_ktop_big per term
  const uint32_t* kb_terms;   // [n_big] the long terms
  const uint32_t* kb_chunk0;  // [n_big + 1] first chunk of each
  const uint32_t* kc_big;     // [n_chunks] long-term index of each chunk
  const uint32_t* kc_start;   // [n_chunks] first posting of each chunk within its term's list
  uint64_t* kc_keys;          // [n_chunks * kTopKs[last]] each chunk's best keys
  uint32_t* kc_cnt;           // [n_chunks]
  uint32_t* kb_stat;          // [3][n_big] alive postings, min / max alive score bits (0, ~0, 0 first)
  uint32_t n_big;
};
#ifndef FG_KTOP_CHUNK
#define FG_KTOP_CHUNK 32768
#endif
constexpr uint32_t kKtopChunk = FG_KTOP_CHUNK;  // postings per k_ktop_part workgroup (and k_ktop's largest term)
constexpr uint32_t kKtopTiny = 64;              // k_ktop_tiny: terms of at most this many postings, one wave each
constexpr uint32_t kPackTerms = 256;            // k_score / k_bucket: term ids per packed chunk

// kernels.hip entry points (host-callable launchers)
hipError_t launch_conj(const DevIndex& ix, const DevPlan& pl, hipStream_t s);
// k_disj over the items [first, first + count) of the plan's k_disj range (in
// sweep order: the first part of every query's doc range first)
hipError_t launch_disj(const DevIndex& ix, const DevPlan& pl, hipStream_t s, uint32_t first = 0,
                       uint32_t count = 0xFFFFFFFFu);
hipError_t launch_fmask(const DevIndex& ix, const DevPlan& pl, hipStream_t s);
hipError_t launch_scan(const DevIndex& ix, const DevPlan& pl, hipStream_t s);
// out_shard != nullptr: the merged select of a multi-snapshot plan (one list per batch query)
hipError_t launch_final(const DevPlan& pl, float* out_score, uint32_t* out_doc, uint32_t* out_n, hipStream_t s,
                        uint32_t* out_shard = nullptr);
hipError_t launch_rank(const uint32_t* doc, const uint64_t* slot_base, const uint32_t* slot_n, uint32_t n_slots,
                       uint32_t n_words, uint64_t* out, hipStream_t s);
hipError_t launch_score(const ScoreJob& j, uint32_t n_chunks, hipStream_t s);
hipError_t launch_bucket(const ScoreJob& j, uint32_t n_chunks, uint32_t n_docs, hipStream_t s);  // packed chunks
hipError_t launch_tsub(const ScoreJob& j, uint32_t n_docs, hipStream_t s);                        // after k_bucket
hipError_t launch_ktop(const ScoreJob& j, uint32_t n_terms, uint32_t n_chunks, uint32_t n_big, hipStream_t s);
hipError_t launch_copy32(uint32_t* dst, const uint32_t* src, uint64_t n, uint32_t grid_cap, hipStream_t s);
hipError_t launch_merge(uint32_t n_shards, uint32_t n_queries, uint32_t k, const float* score, const uint32_t* doc,
                        const uint32_t* n, float* out_score, uint32_t* out_doc, uint32_t* out_shard, uint32_t* out_n,
                        hipStream_t s);

}  // namespace fg
