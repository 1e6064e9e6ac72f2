// Internal layout shared by the host side (index.cpp, plan.cpp, api.cpp) and
// the gfx950 kernels (kernels.hip).  See DESIGN.md §HBM layout.
#pragma once
#include <cstdint>

#include <hip/hip_runtime.h>

namespace fg {

constexpr uint32_t kBlock = 128;          // postings per skip block (tantivy: 128-doc blocks)
constexpr uint32_t kThreads = 256;        // 4 waves of 64 per workgroup
constexpr uint32_t kItems = 8;            // candidates per lane
constexpr uint32_t kChunk = kThreads * kItems;   // 2048 candidates of the lead list per workgroup
constexpr uint32_t kWaveSpan = kChunk / 4;       // 512 consecutive candidates per wave
constexpr uint32_t kSeg = 2048;           // LDS staging budget per wave (u32 doc ids)
constexpr uint32_t kMaxTerms = 16;        // terms per query (FG_MAX_TERMS)
constexpr uint32_t kMaxK = 1024;          // largest top-k the device select supports
constexpr uint32_t kFinalCap = 4096;      // candidates kept in LDS by the final select
constexpr uint32_t kHistBins = 2048;      // 11-bit radix digits

constexpr uint32_t kModeAnd = 0;
constexpr uint32_t kModeOr = 1;

// Device view of one namespace snapshot (all pointers device-resident).
struct DevIndex {
  const uint32_t* doc;       // [P] doc ids, CSR by term, ascending within a term
  const uint32_t* tf;        // [P] packed: lo16 = tf in `text`, hi16 = tf in `name`
  const uint64_t* off;       // [V+1] posting offsets
  const uint32_t* skip;      // [S] last doc id of each 128-posting block
  const uint32_t* skip_off;  // [V+1] skip offsets
  const float* w_text;       // [V] idf(df_text)*(1+K1)
  const float* w_name;       // [V] idf(df_name)*(1+K1)
  const uint8_t* fn_text;    // [N] fieldnorm ids
  const uint8_t* fn_name;    // [N] fieldnorm ids (all 0 when no `name` values)
  const uint32_t* alive;     // [ceil(N/32)] alive bitset, or nullptr (no deletes)
  const float* cache;        // [512] bm25 tf cache: [0,256) text, [256,512) name
  uint32_t n_docs;
  uint32_t n_terms;
  uint32_t has_name;
};

// Device view of one planned batch.
struct DevPlan {
  uint32_t n_queries;
  uint32_t total_chunks;
  uint32_t k;
  uint32_t mode;
  const uint32_t* q_m;          // [nq] terms per query
  const uint32_t* q_terms;      // [nq * kMaxTerms] term ids, intersection (cost) order
  const uint32_t* q_lead_df;    // [nq] length of the lead list (0 => empty result)
  const uint32_t* chunk_start;  // [nq+1] first work item of each query
  const uint32_t* chunk_q;      // [total_chunks] query of each work item
  const uint64_t* cand_off;     // [nq+1] capacity offsets of the per-query candidate lists
  // workspace (zeroed per execution where noted)
  uint64_t* thresh;             // [nq] monotone lower bound on the k-th best key (zeroed)
  uint32_t* slot_cnt;           // [total_chunks] keys written by each work item
  uint64_t* slot_keys;          // [total_chunks * k]
  uint32_t* cand_cnt;           // [nq] (zeroed)
  uint64_t* cand_keys;          // [cand_off[nq]]
};

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

// kernels.hip entry points (host-callable launchers)
hipError_t launch_conj(const DevIndex& ix, const DevPlan& pl, hipStream_t s);
hipError_t launch_filter(const DevPlan& pl, hipStream_t s);
hipError_t launch_final(const DevPlan& pl, float* out_score, uint32_t* out_doc, uint32_t* out_n, hipStream_t s);
hipError_t launch_merge(uint32_t n_shards, uint32_t n_queries, uint32_t k, const float* score, const uint32_t* doc,
                        const uint32_t* n, float* out_score, uint32_t* out_doc, uint32_t* out_shard, uint32_t* out_n,
                        hipStream_t s);

}  // namespace fg
