// Host-side internals of libfugu shared by fugu.cpp (snapshot build, plans,
// execution, the C ABI) and model.cpp (the byte / line models of the roofline):
// the opaque handles of include/fugu.h and their memory pools.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/fugu.h"
#include "fg_internal.h"
#include "fg_pool.h"
#include "fg_trace.h"

namespace fgh {

// set the thread-local message of fg_last_error() and return `code`
int fail(int code, const char* fmt, ...);
// host threads for builds, planning and models (FUGU_THREADS, the CPU share)
int hw_threads(int req);

// parallel_ranges / parallel_dynamic / run_helped: fg_pool.h

// Device memory some structure keeps cached for reuse (released scoring
// blocks, plan workspaces).  Every cache registers itself; an allocation that
// fails drops ALL of them and retries once (dev_malloc), so a build or a plan
// never fails with FG_EOOM while idle cached blocks sit on the device.
struct DevCache {
  DevCache();
  virtual ~DevCache() { unregister_cache(); }
  // first thing in a derived destructor: no drop_all_cached reaches a cache
  // whose own destructor has started
  void unregister_cache();
  DevCache(const DevCache&) = delete;
  DevCache& operator=(const DevCache&) = delete;
  virtual void drop_cached() = 0;  // free what is cached (not what is handed out)
};
void drop_all_cached();
// hipMalloc, after dropping every registered cache if the first try fails
hipError_t dev_malloc(void** p, size_t bytes);
// hipMallocAsync on `s`, likewise
hipError_t dev_malloc_async(void** p, size_t bytes, hipStream_t s);

struct DevAllocs {
  std::vector<void*> ptrs;
  int dev = 0;
  ~DevAllocs() {
    if (ptrs.empty()) return;
    const uint64_t t0 = commit_trace_on() ? now_ns() : 0;
    (void)hipSetDevice(dev);
    for (void* p : ptrs) (void)hipFree(p);
    if (t0) trace_span("free", "snapshot arrays (hipFree)", t0);
  }
};

// The scoring tables of the snapshots of ONE structure (a segment and its
// rescores) come in one block of one size; a released snapshot's block is kept
// for the structure's next rescore instead of freed (a commit rescores every
// older segment: fresh hipMallocs of those blocks from several threads
// serialised in the runtime, 10s of ms per commit).  The release waits for the
// device to drain, as hipFree would, so no kernel still reads a block handed out
// again.
struct ScorePool : DevCache {
  static constexpr size_t kKeep = 2;  // blocks cached per structure
  std::mutex mu;
  std::vector<std::pair<size_t, void*>> free_blocks;
  // pinned host blocks of the per-term maxima read back after every scoring
  // (tmaxs, ktop: 24 B per vocabulary term): the device writes them in place and
  // a rescore reuses a released snapshot's block (a fresh pageable array per
  // rescore cost page faults on every page and a staging copy)
  std::vector<std::pair<size_t, void*>> free_host;
  int dev = 0;
  void* get_host(size_t bytes) {
    {
      std::lock_guard<std::mutex> l(mu);
      for (size_t i = 0; i < free_host.size(); ++i)
        if (free_host[i].first == bytes) {
          void* p = free_host[i].second;
          free_host.erase(free_host.begin() + i);
          return p;
        }
    }
    void* p = nullptr;
    if (hipHostMalloc(&p, std::max<size_t>(bytes, 16), hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    return p;
  }
  void put_host(void* p, size_t bytes) {
    {
      std::lock_guard<std::mutex> l(mu);
      if (free_host.size() < kKeep) {
        free_host.emplace_back(bytes, p);
        return;
      }
    }
    (void)hipHostFree(p);
  }
  void* get(size_t bytes) {
    {
      std::lock_guard<std::mutex> l(mu);
      for (size_t i = 0; i < free_blocks.size(); ++i)
        if (free_blocks[i].first == bytes) {
          void* p = free_blocks[i].second;
          free_blocks.erase(free_blocks.begin() + i);
          return p;
        }
    }
    void* p = nullptr;
    if (dev_malloc(&p, bytes) != hipSuccess) return nullptr;
    return p;
  }
  // (the caller runs where waiting for the device is harmless: a snapshot's
  // last release happens on the db's reaper thread, or a build / test thread)
  void put(void* p, size_t bytes) {
    const uint64_t t0 = commit_trace_on() ? now_ns() : 0;
    (void)hipSetDevice(dev);
    (void)hipDeviceSynchronize();
    if (t0) trace_span("free", "scoring block: device drain", t0);
    {
      std::lock_guard<std::mutex> l(mu);
      if (free_blocks.size() < kKeep) {
        free_blocks.emplace_back(bytes, p);
        return;
      }
    }
    const uint64_t t1 = commit_trace_on() ? now_ns() : 0;
    (void)hipFree(p);
    if (t1) trace_span("free", "scoring block (hipFree)", t1);
  }
  void release_all() {
    std::lock_guard<std::mutex> l(mu);
    for (auto& b : free_blocks) (void)hipFree(b.second);
    free_blocks.clear();
  }
  void drop_cached() override { release_all(); }
  ~ScorePool() override {
    unregister_cache();
    for (auto& b : free_host) (void)hipHostFree(b.second);
    if (free_blocks.empty()) return;
    (void)hipSetDevice(dev);
    for (auto& b : free_blocks) (void)hipFree(b.second);
  }
};
struct ScoreBlock {
  void* p = nullptr;  // device scoring tables
  size_t bytes = 0;
  void* hp = nullptr;  // pinned host block (tmaxs, ktop) or nullptr
  size_t hbytes = 0;
  std::vector<float> hown;  // tmaxs / ktop when no pinned block was had
  std::shared_ptr<ScorePool> pool;
  ~ScoreBlock() {
    if (hp && pool) pool->put_host(hp, hbytes);
    if (p && pool) pool->put(p, bytes);
  }
};

// A host array of a snapshot's structure (or of one scoring's weights), shared
// by the snapshot and its rescores: copying one copies the pointer.  Written
// only while a single owner holds it (the build); mut() copies it first
// otherwise.  A rescore used to copy ~28 MB of such arrays per segment.
template <class T>
class SharedVec {
  std::shared_ptr<std::vector<T>> p_ = std::make_shared<std::vector<T>>();

 public:
  SharedVec() = default;
  SharedVec(std::vector<T>&& v) : p_(std::make_shared<std::vector<T>>(std::move(v))) {}
  SharedVec& operator=(std::vector<T>&& v) {
    p_ = std::make_shared<std::vector<T>>(std::move(v));
    return *this;
  }
  SharedVec& operator=(const std::vector<T>& v) {
    p_ = std::make_shared<std::vector<T>>(v);
    return *this;
  }
  const T& operator[](size_t i) const { return (*p_)[i]; }
  size_t size() const { return p_->size(); }
  bool empty() const { return p_->empty(); }
  const T* data() const { return p_->data(); }
  typename std::vector<T>::const_iterator begin() const { return p_->begin(); }
  typename std::vector<T>::const_iterator end() const { return p_->end(); }
  const std::vector<T>& vec() const { return *p_; }
  std::vector<T>& mut() {
    if (p_.use_count() > 1) p_ = std::make_shared<std::vector<T>>(*p_);
    return *p_;
  }
};

// BM25 weights of one set of statistics, shared by the snapshots scored with
// them (fg_index_rescore_many)
struct Weights {
  SharedVec<float> wt, wn;
};


}  // namespace fgh

#define HIPCHK(x)                                                                  \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) return fgh::fail(FG_EHIP, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)

using fgh::DevAllocs;

struct fg_ctx {
  std::vector<int> devs;
  std::vector<std::pair<int, int>> peers;  // (a, b): a reaches b's memory directly
};

// Plan workspaces of one index, recycled across batches (a server plans a new
// batch every few ms; a hipMalloc/hipFree pair per batch would serialise the
// device).  Buffers are reused when they fit a request within 2x; at most
// kPoolKeep bytes stay cached.
namespace fgh {
// the size a pooled buffer of `bytes` is allocated at: the next power of two
// (>= 4 KiB; past 256 MiB the next 1/16 of one), so a cached buffer serves the
// requests a little smaller than it
inline size_t size_class(size_t bytes) {
  size_t n = 4096;
  while (n < bytes) n <<= 1;
  if (n <= (256ull << 20)) return n;
  const size_t step = n / 16;
  return (bytes + step - 1) / step * step;
}
struct WsPool : DevCache {
  static constexpr size_t kPoolKeep = 1ull << 30;
  std::mutex mu;
  std::multimap<size_t, void*> free_bufs;
  size_t cached = 0;
  int dev = 0;
  void* get(size_t bytes, size_t* got) {
    {
      std::lock_guard<std::mutex> l(mu);
      auto it = free_bufs.lower_bound(bytes);
      if (it != free_bufs.end() && it->first <= 2 * bytes) {
        void* p = it->second;
        *got = it->first;
        cached -= it->first;
        free_bufs.erase(it);
        return p;
      }
    }
    void* p = nullptr;
    // sized up to a power of two: a plan a little larger than the last (one
    // more segment after a commit) reuses its buffer instead of a hipMalloc in
    // the search's path.  The cached workspaces and scoring blocks (of every
    // index) may be what the device lacks: dev_malloc frees them and retries once
    const size_t n = size_class(bytes);
    if (dev_malloc(&p, n) != hipSuccess) return nullptr;
    *got = n;
    return p;
  }
  void drop_cached() override {
    std::lock_guard<std::mutex> l(mu);
    (void)hipSetDevice(dev);
    for (auto& kv : free_bufs) (void)hipFree(kv.second);
    free_bufs.clear();
    cached = 0;
  }
  void put(void* p, size_t bytes) {
    {
      std::lock_guard<std::mutex> l(mu);
      if (cached + bytes <= kPoolKeep) {
        free_bufs.emplace(bytes, p);
        cached += bytes;
        return;
      }
    }
    (void)hipSetDevice(dev);
    (void)hipFree(p);
  }
  ~WsPool() override {
    unregister_cache();
    if (free_bufs.empty()) return;
    (void)hipSetDevice(dev);
    for (auto& kv : free_bufs) (void)hipFree(kv.second);
  }
};

// Pinned host buffers of a device's snapshots: plan uploads and result copies
// go through them (a pageable copy is staged by the runtime and synchronises on
// the way), which takes ~tens of us off a batch-of-one search.
struct PinnedPool {
  const size_t kKeep;  // bytes kept cached
  std::mutex mu;
  std::multimap<size_t, void*> free_bufs;
  size_t cached = 0;
  explicit PinnedPool(size_t keep = 16ull << 20) : kKeep(keep) {}
  void* get(size_t bytes, size_t* got) {
    {
      std::lock_guard<std::mutex> l(mu);
      auto it = free_bufs.lower_bound(bytes);
      if (it != free_bufs.end() && it->first <= 4 * bytes + 65536) {
        void* p = it->second;
        *got = it->first;
        cached -= it->first;
        free_bufs.erase(it);
        return p;
      }
    }
    void* p = nullptr;
    const size_t n = size_class(bytes);  // (as WsPool::get)
    if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) return nullptr;
    *got = n;
    return p;
  }
  void put(void* p, size_t bytes) {
    {
      std::lock_guard<std::mutex> l(mu);
      if (cached + bytes <= kKeep) {
        free_bufs.emplace(bytes, p);
        cached += bytes;
        return;
      }
    }
    (void)hipHostFree(p);
  }
  ~PinnedPool() {
    for (auto& kv : free_bufs) (void)hipHostFree(kv.second);
  }
};
// a pinned buffer of the pool for one scope
struct PinnedLease {
  PinnedPool& pool;
  void* p = nullptr;
  size_t n = 0;
  PinnedLease(PinnedPool& pl, size_t bytes) : pool(pl) {
    if (bytes) p = pool.get(bytes, &n);
  }
  ~PinnedLease() { if (p) pool.put(p, n); }
};
}  // namespace fgh
using fgh::PinnedLease;
using fgh::PinnedPool;
using fgh::WsPool;
namespace fgh {
// The plan-workspace and pinned pools of device `dev`, shared by every live
// snapshot on it: a commit's rescored snapshots (new fg_index objects) reuse
// the buffers of the ones they replace, so the first search after a commit does
// not hipMalloc / hipHostMalloc (those sat in the slowest 1% of the searches
// beside commits: tools/stall_trace.py).  Freed with the device's last snapshot.
void device_pools(int dev, std::shared_ptr<WsPool>* ws, std::shared_ptr<PinnedPool>* pin);
}  // namespace fgh

struct fg_index {
  std::atomic<int> refs{1};
  int dev = 0;
  uint32_t n_docs = 0, n_terms = 0;
  bool has_name = false;
  uint64_t n_postings = 0, device_bytes = 0, dir_entries = 0, tile_entries = 0;
  uint32_t n_dense = 0, n_rank = 0;  // n_rank: rank-kind slots, plain (d.n_prank) and sparse
  uint64_t n_srank_words = 0;        // sparse rank words (d.srank_w)
  // ---- statistics (this snapshot's own: the Searcher-wide ones of its commit).
  // Scores are formed at query time from them (DevIndex::tfn, DevPlan::q_wt /
  // q_wn, the plan's copy of `cache`), as tantivy's TermScorer does.
  uint64_t tot[2] = {0, 0};
  uint64_t n_stats = 0;  // N the BM25 statistics use (global N of a doc-sharded namespace)
  float avgdl[2] = {0, 0};
  float cache[512];
  fgh::SharedVec<float> w_text, w_name;
  fgh::SharedVec<uint32_t> h_alive;  // the alive bitset of this snapshot (empty: every doc)
  // ---- bounds: computed ONCE when the structure is built (k_score / k_bucket /
  // k_tsub / k_ktop under the build's statistics) and shared by every rescore of
  // it; a plan scales them by the ratio of the current to the build statistics
  // (term_ratio).  sblock holds the device tables and the host tmaxs / ktop.
  std::shared_ptr<fgh::ScoreBlock> sblock;
  const float* ktop = nullptr;   // [V * kNumTopK] K-th best score per term at the build (alive docs then)
  const float* tmaxs = nullptr;  // [V] largest posting score per term at the build
  fgh::SharedVec<float> wb_text, wb_name;  // the build's BM25 weights
  float cache_b[512];                      // the build's tf caches
  fgh::SharedVec<uint32_t> h_alive_b;      // the alive bitset ktop was selected over (empty: every doc)
  uint32_t n_dead = 0;     // docs dead now that were alive in h_alive_b (ktop's K-th then needs K + n_dead)
  bool same_stats = true;  // the current statistics are the build's (every ratio exactly 1)
  double cup[2] = {1, 1}, cdn[2] = {1, 1};  // per field: max / min over fieldnorms of the tf-factor ratio
  std::shared_ptr<void> alive_hold;         // the device alive bitset when it is this snapshot's own
  // [V * kNumTopK] namespace-wide floor of the current K-th scores (fg_index_set_kth_floor) or
  // null; read and replaced with std::atomic_load / atomic_store
  std::shared_ptr<const std::vector<float>> kth_floor;
  // ---- structure (independent of the statistics; shared with rescored snapshots)
  // The snapshot's own term dictionary (tantivy keeps one per segment): a build
  // over far fewer distinct terms than the vocabulary it was given (a commit's
  // new docs) numbers its terms locally, tmap[l] = the vocabulary id of local
  // term l (ascending); empty: local ids ARE vocabulary ids.  Every per-term
  // array here and on the device is indexed by local id; the C ABI takes
  // vocabulary ids (fgh::local_term).  n_terms counts local terms, n_vocab the
  // vocabulary (fg_index_stats::n_terms).
  fgh::SharedVec<uint32_t> tmap;
  uint32_t n_vocab = 0;
  fgh::SharedVec<uint64_t> off;
  fgh::SharedVec<uint32_t> df_text, df_name;  // this snapshot's own postings (tantivy's per-segment cost order)
  fgh::SharedVec<uint32_t> first_doc, last_doc;
  std::shared_ptr<const std::vector<uint32_t>> h_doc;  // optional host copy for fg_bytes_model(_gpu)
  fgh::SharedVec<uint32_t> tmeta;  // host copy of DevIndex::tmeta (probe kind of each term)
  uint64_t tot_local[2] = {0, 0};
  // facet field (FG_FIELD_FACET)
  uint32_t n_fterms = 0;
  uint64_t tot_f = 0, tot_f_local = 0;
  float avgdl_f = 0.0f, cache_f1 = 0.0f;
  fgh::SharedVec<uint64_t> foff;
  std::vector<uint32_t> df_facet;
  fgh::SharedVec<uint32_t> df_facet_local, ffirst, flast;
  std::vector<float> fscore;    // a facet clause's score in a doc holding the term (tf 1, fieldnorm id 1)
  // device: structure arrays (smem, shared), the scoring tables (sblock, from the
  // structure's spool) and other snapshot-own arrays (mem)
  std::shared_ptr<DevAllocs> smem;
  std::shared_ptr<fgh::ScorePool> spool;
  uint64_t struct_bytes = 0;
  // packed chunk tables of k_score / k_bucket (fg_internal.h ScoreJob::sc_* / bk_*)
  const uint32_t *d_sc_tf = nullptr, *d_sc_tl = nullptr, *d_bk_tf = nullptr, *d_bk_tl = nullptr, *d_bk_e0 = nullptr,
                 *d_bk_e1 = nullptr, *d_kt_terms = nullptr, *d_kt_tiny = nullptr;
  const uint64_t *d_sc_e0 = nullptr, *d_sc_e1 = nullptr;
  uint32_t n_scb = 0, n_ktiny = 0;  // k_score chunks; k_ktop_tiny terms
  const uint32_t* d_tterm = nullptr;  // tile-table terms in toff order (k_tsub)
  uint32_t n_tterm = 0, n_tiles = 0;
  // k_ktop's tables (structure): long terms, their first chunk, each chunk's term and first posting
  const uint32_t *d_kb_terms = nullptr, *d_kb_chunk0 = nullptr, *d_kc_big = nullptr, *d_kc_start = nullptr;
  uint32_t n_sc = 0, n_bk = 0, n_kt = 0, n_kbig = 0, n_kchunks = 0;
  fg::DevIndex d{};
  DevAllocs mem;
  // plan workspaces and the pinned host staging of plan uploads and result
  // copies: the device's pools, shared by every snapshot on it (fgh::device_pools)
  std::shared_ptr<WsPool> pool;
  std::shared_ptr<PinnedPool> pinned;
};

struct fg_plan {
  fg_index* ix = nullptr;
  // nq: query slots = n_segs x nq_batch (one snapshot: the batch's queries)
  uint32_t nq = 0, k = 0, total_chunks = 0, n_scan = 0, nq_batch = 0, n_segs = 1;
  std::vector<fg_index*> segs;  // a multi-snapshot plan's snapshots after ix (retained)
  int mode = FG_MODE_AND;
  fg::DevPlan d{};
  fg::DevIndex d0{};  // the first snapshot's view with the plan's copy of its tf caches (DevIndex::cache)
  void* ws = nullptr;  // workspace from ix->pool
  size_t ws_got = 0;
  float* own_score = nullptr;
  uint32_t* own_doc = nullptr;
  uint32_t* own_n = nullptr;
  void* zero_region = nullptr;
  size_t zero_bytes = 0;
  size_t diag_words = 0;
  uint64_t ws_bytes = 0;
  DevAllocs mem;
  hipStream_t last_stream = nullptr;
  bool profile = false;
  std::vector<hipEvent_t> pending;  // 3 per profiled execute
  double ms[2] = {0, 0};
  uint32_t n_prof = 0;
  ~fg_plan() {
    for (hipEvent_t e : pending) (void)hipEventDestroy(e);
    if (pin) {  // an upload nothing waited for yet (created without sync, never executed)
      (void)hipSetDevice(ix->dev);
      (void)hipStreamSynchronize(up_stream);
    }
    if (ws) {
      // the workspace may still be read by this plan's last launch (a per-thread
      // stream handle resolves on the current device: select the plan's first)
      if (last_stream_used) {
        (void)hipSetDevice(ix->dev);
        (void)hipStreamSynchronize(last_stream);
      }
      if (pin) ix->pinned->put(pin, pin_n);
      ix->pool->put(ws, ws_got);
    }
    if (!ipc_maps.empty()) {
      (void)hipSetDevice(ix->dev);
      for (void* m : ipc_maps) (void)hipIpcCloseMemHandle(m);
    }
    if (ix) fg_index_release(ix);
    for (fg_index* x : segs) fg_index_release(x);
  }
  bool last_stream_used = false;
  std::vector<uint32_t> h_lo, h_hi;  // per query slot: f32 bits spanned by its score histogram (fg_plan_link)
  std::vector<uint8_t> h_any;        // per batch query: some slot has work items (fg_plan_hist_span)
  double part_next = 0.0;            // where the next fg_plan_execute_part must start (0: a new round)
  bool zeroed = false;        // the zero region arrived zeroed with the upload: the first execute skips its memset
  void* pin = nullptr;        // pinned upload staging still in flight (create without sync), returned at destroy
  size_t pin_n = 0;
  std::vector<void*> ipc_maps;  // peers' workspaces mapped through HIP IPC (fg_plan_set_ipc_peers), closed at destroy
  hipStream_t up_stream = hipStreamPerThread;  // the stream the plan was uploaded on
};


namespace fgh {
// the local id of vocabulary term t in snapshot ix (fg_index::tmap), or
// 0xFFFFFFFF (>= n_terms: absent) when the snapshot holds no posting of it
inline uint32_t local_term(const fg_index* ix, uint32_t t) {
  if (ix->tmap.empty()) return t;
  const auto it = std::lower_bound(ix->tmap.begin(), ix->tmap.end(), t);
  return it != ix->tmap.end() && *it == t ? (uint32_t)(it - ix->tmap.begin()) : 0xFFFFFFFFu;
}
// Per-term bounds under a snapshot's current statistics from its build-time
// tables (fugu.cpp): the score ratio factors, the largest score, and a lower
// bound of the K-th best alive score (K the smallest stored level >= k; with_floor:
// or the namespace-wide floor of a doc-sharded namespace's shard when higher)
void term_ratio(const fg_index* ix, uint32_t t, float* rdn, float* rup);
float term_max_now(const fg_index* ix, uint32_t t);
float term_max_scaled(const fg_index* ix, uint32_t t, float rup);  // tmaxs[t] x rup, rounded up
float term_kth_now(const fg_index* ix, uint32_t t, uint32_t k, bool with_floor);
}  // namespace fgh
