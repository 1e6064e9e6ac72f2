// libfugu host side: index snapshot build + HBM upload, batch planning,
// execution and the C ABI of include/fugu.h.
//
// The BM25 statistics follow tantivy 0.24.1 as fugu uses it (SURVEY.md
// Appendix A): N = max_doc (deleted docs included), avgdl = total tokens / N,
// idf = ln(1 + (N - df + 0.5) / (df + 0.5)), weight = idf * (1 + K1), tf cache
// K1 * ((1 - B) + B * FIELD_NORMS_TABLE[id] / avgdl).  They are computed here,
// on the host, in that operation order with the host libm, so the device only
// multiplies/divides precomputed f32 values (bit-identical to the CPU path).
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <functional>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/fugu.h"
#include "fg_host.h"
#include "fg_internal.h"

namespace {
thread_local std::string g_err;
}  // namespace

int fgh::fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

// shared with host.cpp so fg_last_error() reports host-side failures too
void fg_set_last_error(const std::string& msg) { g_err = msg; }
int fg_host_threads();  // below (hw_threads(0)), shared with host.cpp

namespace {

using fgh::fail;
using fgh::hw_threads;
using fgh::parallel_dynamic;
using fgh::parallel_ranges;

// ---------------------------------------------------------------- tantivy constants
constexpr float kK1 = 1.2f;
constexpr float kB = 0.75f;

struct FieldNormTable {
  uint32_t v[256];
  FieldNormTable() {
    uint32_t i = 0;
    for (; i <= 40; ++i) v[i] = i;
    uint64_t x = 40, step = 2;
    while (i < 256) {
      for (int j = 0; j < 8 && i < 256; ++j) { x += step; v[i++] = (uint32_t)x; }
      step <<= 1;
    }
  }
};
const FieldNormTable& fn_table() {
  static const FieldNormTable t;
  return t;
}
// FIELD_NORMS_TABLE.binary_search(n).unwrap_or_else(|i| i - 1)
uint8_t fieldnorm_id(uint64_t n) {
  const uint32_t* t = fn_table().v;
  uint32_t x = n > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)n;
  return (uint8_t)(std::upper_bound(t, t + 256, x) - t - 1);
}
float bm25_weight(uint64_t df, uint64_t n_docs) {
  float x = ((float)(n_docs - df) + 0.5f) / ((float)df + 0.5f);
  return logf(1.0f + x) * (1.0f + kK1);
}
void bm25_cache(float avgdl, float* out) {
  const uint32_t* t = fn_table().v;
  for (int i = 0; i < 256; ++i) out[i] = kK1 * ((1.0f - kB) + (kB * (float)t[i]) / avgdl);
}
// kernels.hip term_score on the host (same f32 operations; -ffp-contract=off)
float term_score_host(uint32_t tfp, uint32_t fn_t, uint32_t fn_n, float wt, float wn, const float* cache) {
  float s = 0.0f;
  const uint32_t tt = tfp & 0xFFFFu, tn = tfp >> 16;
  if (tt) {
    const float tf = (float)tt;
    s += wt * (tf / (tf + cache[fn_t]));
  }
  if (tn) {
    const float tf = (float)tn;
    s += wn * (tf / (tf + cache[256 + fn_n]));
  }
  return s;
}

// Bin width (2^shift f32 ulps) of a query score histogram spanning the f32
// bit patterns [lo, hi] in fewer than kQBins bins (DevPlan::hist).
uint32_t bin_shift(uint32_t lo, uint32_t hi) {
  uint32_t sh = 0;
  while (sh < 31 && ((uint64_t)(hi - lo) >> sh) >= fg::kQBins - 1) ++sh;
  return sh;
}

// FUGU_BUILD_TRACE=1: per-phase wall time of a snapshot build on stderr
struct BuildTrace {
  bool on = false;
  std::chrono::steady_clock::time_point t;
  void start() {
    on = getenv("FUGU_BUILD_TRACE") != nullptr;
    t = std::chrono::steady_clock::now();
  }
  void mark(const char* what) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    // @: the phase's end on the steady clock (ms; Python's time.monotonic), to line
    // phases up with other threads' events (tools/stall_trace.py)
    fprintf(stderr, "[fg build] %-24s %9.1f ms @%.3f\n", what, std::chrono::duration<double, std::milli>(n - t).count(),
            std::chrono::duration<double, std::milli>(n.time_since_epoch()).count());
    t = n;
  }
};
thread_local BuildTrace g_bt;

}  // namespace
// Host threads for snapshot builds and planning: FUGU_THREADS when set; else
// OMP_NUM_THREADS when it states a share above one (16 per GPU on the box; a
// launcher's default of 1 -- torchrun sets it for every rank -- is not a CPU
// share and is ignored); else the CPUs this process may run on (affinity,
// capped by the cgroup quota), at most 64.
int fgh::hw_threads(int req) {
  if (req > 0) return std::min(req, 256);
  static const int n = [] {
    int t = 0;
    if (const char* e = getenv("FUGU_THREADS")) t = atoi(e);
    if (t <= 0)
      if (const char* e = getenv("OMP_NUM_THREADS"))
        if (atoi(e) > 1) t = atoi(e);
    if (t <= 0) {
      cpu_set_t cs;
      t = sched_getaffinity(0, sizeof cs, &cs) == 0 ? CPU_COUNT(&cs) : (int)std::thread::hardware_concurrency();
      if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        long long per = 0;
        if (fscanf(f, "%31s %lld", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0)
          t = std::min<long long>(t, std::max<long long>(1, atoll(q) / per));
        fclose(f);
      }
      t = std::min(t, 64);
    }
    t = std::max(1, std::min(t, 256));
    if (getenv("FUGU_BUILD_TRACE")) fprintf(stderr, "[fg build] host threads: %d\n", t);
    return t;
  }();
  return n;
}
int fg_host_threads() { return hw_threads(0); }

// fgh::pool_post's threads: as many as the host threads builds use, started on
// first use, never destroyed (idle ones end with the process)
void fgh::pool_post(std::function<void()> job) {
  struct Pool {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void()>> q;
  };
  static Pool* pool = [] {
    auto* p = new Pool;
    for (int i = 0, n = std::max(1, hw_threads(0) - 1); i < n; ++i)
      std::thread([p] {
        for (;;) {
          std::function<void()> j;
          {
            std::unique_lock<std::mutex> l(p->mu);
            p->cv.wait(l, [&] { return !p->q.empty(); });
            j = std::move(p->q.front());
            p->q.pop_front();
          }
          j();
        }
      }).detach();
    return p;
  }();
  {
    std::lock_guard<std::mutex> l(pool->mu);
    pool->q.push_back(std::move(job));
  }
  pool->cv.notify_one();
}

namespace fgh {
namespace {
std::mutex& cache_mu() {
  static std::mutex m;
  return m;
}
std::vector<DevCache*>& caches() {
  static std::vector<DevCache*> v;
  return v;
}
}  // namespace
DevCache::DevCache() {
  std::lock_guard<std::mutex> l(cache_mu());
  caches().push_back(this);
}
void DevCache::unregister_cache() {
  std::lock_guard<std::mutex> l(cache_mu());
  auto& v = caches();
  v.erase(std::remove(v.begin(), v.end(), this), v.end());
}
// Stream-ordered allocations (hipMallocAsync: scoring scratch, rescore
// weights) keep their memory in the device's default pool instead of returning
// it at every synchronisation (release threshold: no limit).  A hipMallocAsync
// that maps fresh memory held up a search kernel on another stream for ~1 ms
// (4 MiB) to ~8.6 ms (256 MiB); with the pool kept, 0.04 ms
// (tools/stall_probe.hip, profiles/r05/stall/probe_r05q.json).  The pools are
// trimmed with the other caches when an allocation fails.
std::mutex& pool_mu() {
  static std::mutex m;
  return m;
}
std::vector<int>& kept_pools() {
  static std::vector<int> v;
  return v;
}
void keep_async_pool(int dev) {
  std::lock_guard<std::mutex> l(pool_mu());
  auto& v = kept_pools();
  if (std::find(v.begin(), v.end(), dev) != v.end()) return;
  hipMemPool_t pool = nullptr;
  if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess && pool) {
    uint64_t thr = ~0ull;
    if (hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr) != hipSuccess) (void)hipGetLastError();
  } else {
    (void)hipGetLastError();
  }
  v.push_back(dev);
}
void drop_all_cached() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  {
    std::lock_guard<std::mutex> l(cache_mu());
    for (DevCache* c : caches()) c->drop_cached();
  }
  {
    std::lock_guard<std::mutex> l(pool_mu());
    for (int d : kept_pools()) {
      hipMemPool_t pool = nullptr;
      if (hipDeviceGetDefaultMemPool(&pool, d) == hipSuccess && pool) (void)hipMemPoolTrimTo(pool, 0);
      (void)hipGetLastError();
    }
  }
  (void)hipSetDevice(dev);
}
void device_pools(int dev, std::shared_ptr<WsPool>* ws, std::shared_ptr<PinnedPool>* pin) {
  static std::mutex mu;
  static std::map<int, std::pair<std::weak_ptr<WsPool>, std::weak_ptr<PinnedPool>>> reg;
  std::lock_guard<std::mutex> l(mu);
  auto& e = reg[dev];
  *ws = e.first.lock();
  if (!*ws) {
    *ws = std::make_shared<WsPool>();
    (*ws)->dev = dev;
    e.first = *ws;
  }
  *pin = e.second.lock();
  if (!*pin) {
    *pin = std::make_shared<PinnedPool>(64ull << 20);
    e.second = *pin;
  }
}
hipError_t dev_malloc(void** p, size_t bytes) {
  const uint64_t t0 = commit_trace_on() ? now_ns() : 0;
  if (hipMalloc(p, bytes) == hipSuccess) {
    if (t0 && now_ns() - t0 > 200000) trace_span("alloc", "hipMalloc (> 0.2 ms)", t0);
    return hipSuccess;
  }
  (void)hipGetLastError();
  drop_all_cached();
  const hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) (void)hipGetLastError();
  return e;
}
hipError_t dev_malloc_async(void** p, size_t bytes, hipStream_t s) {
  int dev = 0;
  if (hipGetDevice(&dev) == hipSuccess) keep_async_pool(dev);
  if (hipMallocAsync(p, bytes, s) == hipSuccess) return hipSuccess;
  (void)hipGetLastError();
  drop_all_cached();
  const hipError_t e = hipMallocAsync(p, bytes, s);
  if (e != hipSuccess) (void)hipGetLastError();
  return e;
}
}  // namespace fgh
namespace {

// Host-side postings before upload (merged text U name per term).
struct HostPostings {
  uint32_t n_docs = 0, n_terms = 0;
  std::vector<uint64_t> off;      // [V+1]
  std::vector<uint32_t> doc, tf;  // tf packed lo16 text / hi16 name
  std::vector<uint32_t> df_text, df_name;
  std::vector<uint8_t> fn_text, fn_name;
  std::vector<uint32_t> alive;    // bitset, empty when no deletes
  uint64_t tot[2] = {0, 0};
  bool has_name = false;
  // facet field: postings (docs only: IndexRecordOption::Basic) per facet term
  uint32_t n_fterms = 0;
  std::vector<uint64_t> foff{0};  // [VF+1]
  std::vector<uint32_t> fdoc;
  std::vector<uint32_t> df_facet;
  uint64_t tot_f = 0;             // total_num_tokens(facet), duplicates included
};

}  // namespace

namespace {

// Snapshot builds and rescores run on the calling thread's own stream (never
// the legacy null stream, which serialises with every other stream): a
// commit's rescores of the older segments, its new segment's build and the
// background merger's build run side by side.  Uploads are synchronous with
// the host (the sources may be freed right after).
// (a thread may point it at another stream: fg_index_rescore_many's workers
// use the device's background streams; a thread under fg_thread_background
// uses one of them for everything it builds)
thread_local hipStream_t tl_build_stream = nullptr;
thread_local int tl_background = 0;
hipStream_t background_stream(int dev, uint32_t i);
hipStream_t build_stream() {
  if (tl_build_stream) return tl_build_stream;
  if (tl_background) {
    thread_local const uint32_t mine = [] {
      static std::atomic<uint32_t> next{0};
      return next.fetch_add(1);
    }();
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess)
      if (hipStream_t st = background_stream(dev, mine)) return st;
  }
  return hipStreamPerThread;
}
#define kBuildStream build_stream()

// Does the calling thread work in the background (fg_thread_background, or a
// rescore worker on a background stream)?
bool on_background() { return tl_background || tl_build_stream; }
// The workgroup cap of a background scoring's launches (fg::ScoreJob::grid_cap):
// FUGU_BG_GRID workgroups per CU (default kBgGridPerCu; 0: no cap).  With the
// K-th reuse (kth_reuse_bound) and one background stream, GET /search during
// commits p99 0.37 -> 0.25 ms, 1.5x its idle p99 (profiles/r05/stall/bg_j2/);
// before the reuse the cap had raised p99 (the capped k_ktop held its slots)
constexpr uint32_t kBgGridPerCu = 2;
uint32_t bg_grid_cap(int dev) {
  if (!on_background()) return 0;
  static const uint32_t per_cu = [] {
    const char* e = getenv("FUGU_BG_GRID");
    return e && *e ? (uint32_t)std::max(0, atoi(e)) : kBgGridPerCu;
  }();
  if (!per_cu) return 0;
  int n_cu = 0;
  if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0) {
    (void)hipGetLastError();
    return 0;
  }
  return per_cu * (uint32_t)n_cu;
}

// A high-priority stream on device `dev` for the calling thread's searches (the
// search path's own: its kernels are dispatched ahead of a commit's builds on
// the same GPU).  Streams come from a fixed per-device pool (kSearchStreams),
// handed out round-robin at a thread's first search and kept in a thread_local
// -- a server whose worker threads come and go (tokio's spawn_blocking pool
// retires idle threads) reuses the pool's streams instead of creating one per
// thread without bound.  Work on one stream is ordered, so threads sharing a
// stream serialise only their own launches; 16 streams >> the hardware queues.
static constexpr uint32_t kSearchStreams = 16;
// alt: the thread's second stream (the pool's stream half way round from its
// own), for a batch whose second half overlaps the first (fg_search_sharded)
static hipStream_t search_stream(int dev, bool alt = false) {
  thread_local std::map<int, std::pair<hipStream_t, hipStream_t>> mine;
  auto it = mine.find(dev);
  if (it != mine.end()) return alt ? it->second.second : it->second.first;
  static std::mutex mu;
  static std::map<int, std::pair<std::vector<hipStream_t>, uint32_t>> pools;
  hipStream_t s = hipStreamPerThread, s2 = hipStreamPerThread;
  {
    std::lock_guard<std::mutex> l(mu);
    auto& pool = pools[dev];
    if (pool.first.empty()) {
      int cur = 0, least = 0, greatest = 0;
      (void)hipGetDevice(&cur);
      (void)hipSetDevice(dev);
      if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = 0;
      for (uint32_t i = 0; i < kSearchStreams; ++i) {
        hipStream_t x = nullptr;
        if (hipStreamCreateWithPriority(&x, hipStreamNonBlocking, greatest) != hipSuccess) {
          (void)hipGetLastError();
          x = hipStreamPerThread;
        }
        pool.first.push_back(x);
      }
      (void)hipSetDevice(cur);
    }
    const uint32_t i = pool.second++ % kSearchStreams;
    s = pool.first[i];
    s2 = pool.first[(i + kSearchStreams / 2) % kSearchStreams];
  }
  mine[dev] = {s, s2};
  return alt ? s2 : s;
}

// The background stream of a device (a db's segment builds and merges),
// created once at low priority (the searches' own are high priority).  ONE
// stream: a commit's device work queues behind itself instead of all hitting the
// GPU together (GET /search during commits p99 0.62 -> 0.37 ms at the same
// commit latency, profiles/r05/stall/bg_j2/).  (A CU-masked stream measured no
// better: the mask is not honoured on this platform, tools/stall_probe.hip,
// profiles/r05/stall/probe_r05p.json.)
hipStream_t background_stream(int dev, uint32_t) {
  static std::mutex mu;
  static std::map<int, hipStream_t> streams;
  std::lock_guard<std::mutex> l(mu);
  auto it = streams.find(dev);
  if (it != streams.end()) return it->second;
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(dev);
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) least = 0;
  hipStream_t st = nullptr;
  if (hipStreamCreateWithPriority(&st, hipStreamNonBlocking, least) != hipSuccess) {
    (void)hipGetLastError();
    st = nullptr;
  }
  (void)hipSetDevice(cur);
  streams[dev] = st;
  return st;
}

template <class T>
int dev_upload(DevAllocs& m, const T* src, size_t n, T** out, uint64_t* bytes) {
  size_t b = std::max<size_t>(n * sizeof(T), 16);
  void* p = nullptr;
  if (fgh::dev_malloc(&p, b) != hipSuccess) return fail(FG_EOOM, "hipMalloc(%zu) failed", b);
  m.ptrs.push_back(p);
  if (n) {
    HIPCHK(hipMemcpyAsync(p, src, n * sizeof(T), hipMemcpyHostToDevice, kBuildStream));
    HIPCHK(hipStreamSynchronize(kBuildStream));
  }
  *out = static_cast<T*>(p);
  *bytes += b;
  return FG_OK;
}

// Several host arrays into ONE device allocation (one hipMalloc instead of one
// per array: a small segment's build is otherwise dominated by allocation).
struct UploadBatch {
  struct E { const void* src; size_t bytes; void** out; };
  std::vector<E> es;
  size_t total = 0;
  template <class T>
  void add(const T* src, size_t n, T** out) {
    es.push_back(E{src, n * sizeof(T), reinterpret_cast<void**>(out)});
    total += (std::max<size_t>(n * sizeof(T), 16) + 16 + 255) & ~size_t(255);  // >= 16 B of slack after each array
  }
  int commit(DevAllocs& m, uint64_t* bytes) {
    void* p = nullptr;
    if (fgh::dev_malloc(&p, std::max<size_t>(total, 256)) != hipSuccess) return fail(FG_EOOM, "hipMalloc(%zu) failed", total);
    m.ptrs.push_back(p);
    // the arrays laid out in a pooled pinned staging buffer by all host threads,
    // then ONE copy: a small segment's arrays are sized by the vocabulary (~40 MB
    // for 2^20 terms), and pageable copies of them -- staged by the runtime,
    // beside a commit's rescores -- took ~16 ms of a 1000-doc segment's build
    // (a bulk build's arrays are larger than the pool keeps: pageable copies)
    PinnedLease pin(stage_pool(), total <= kStageMax ? total : 0);
    if (pin.p && total <= kStageMax) {
      struct Piece { char* dst; const char* src; size_t n; };
      std::vector<Piece> pieces;
      size_t o = 0;
      for (const E& e : es) {
        for (size_t b = 0; b < e.bytes; b += kStagePiece)
          pieces.push_back(Piece{static_cast<char*>(pin.p) + o + b, static_cast<const char*>(e.src) + b,
                                 std::min(kStagePiece, e.bytes - b)});
        o += (std::max<size_t>(e.bytes, 16) + 16 + 255) & ~size_t(255);
      }
      parallel_dynamic((uint32_t)pieces.size(), std::min<int>(hw_threads(0), (int)pieces.size()), 1,
                       [&](int, uint32_t b, uint32_t e) {
        for (uint32_t i = b; i < e; ++i) std::memcpy(pieces[i].dst, pieces[i].src, pieces[i].n);
      });
      HIPCHK(hipMemcpyAsync(p, pin.p, total, hipMemcpyHostToDevice, kBuildStream));
    }
    size_t o = 0;
    for (const E& e : es) {
      char* d = static_cast<char*>(p) + o;
      if (!(pin.p && total <= kStageMax) && e.bytes) HIPCHK(hipMemcpyAsync(d, e.src, e.bytes, hipMemcpyHostToDevice, kBuildStream));
      *e.out = d;
      o += (std::max<size_t>(e.bytes, 16) + 16 + 255) & ~size_t(255);
    }
    HIPCHK(hipStreamSynchronize(kBuildStream));
    *bytes += total;
    return FG_OK;
  }
  static constexpr size_t kStagePiece = 1u << 20;
  static constexpr size_t kStageMax = 128ull << 20;
  // process-wide: builds run on many threads (a commit's builder, the merger)
  static PinnedPool& stage_pool() {
    static PinnedPool pool(256ull << 20);
    return pool;
  }
};

int check_device(int dev) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(FG_ENODEV, "no HIP device visible");
  if (dev < 0 || dev >= n) return fail(FG_ENODEV, "device %d out of range (%d visible)", dev, n);
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, dev));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(FG_ENODEV, "device %d is %s; libfugu is built for gfx950 only", dev, prop.gcnArchName);
  return FG_OK;
}

// ---------------------------------------------------------------- statistics and bounds
// The statistics-dependent state of a snapshot is host-only: BM25 weights and
// tf caches (tantivy's f32 order with the host libm), read by the plans; the
// device forms the scores at query time.  The bound tables (maxima and K-th
// best scores the kernels prune with) are computed on the device once per
// structure under its build statistics.  `df_t`/`df_n`/`df_f`: the statistics'
// doc frequencies (global for a doc-sharded namespace).

// BM25 weights of terms [0, V) for statistics (Ns, df_t, df_n) (tantivy's f32 order)
void bm25_weights(uint64_t Ns, const uint32_t* df_t, const uint32_t* df_n, uint32_t V, std::vector<float>& wt,
                  std::vector<float>& wn) {
  wt.resize(V);
  wn.resize(V);
  parallel_ranges(V, hw_threads(0), [&](int, uint32_t b, uint32_t e) {
    for (uint32_t t = b; t < e; ++t) {
      wt[t] = bm25_weight(df_t[t], Ns);
      wn[t] = bm25_weight(df_n ? df_n[t] : 0u, Ns);
    }
  });
}

// The statistics of a snapshot (host only, tantivy's f32 order with the host
// libm): N, token totals, avgdl and the tf caches, the BM25 weights (`wts`:
// shared precomputed ones of the same statistics, or nullptr: computed here),
// the facet clause scores.  The device sees them only through plans (query-time
// scoring: DevPlan::q_wt / q_wn and the plan's copy of the caches).
void set_stats(fg_index* ix, uint64_t Ns, const uint64_t tot2[2], const uint32_t* df_t, const uint32_t* df_n,
               uint64_t tot_f, const uint32_t* df_f, const fgh::Weights* wts) {
  const uint32_t V = ix->n_terms;
  ix->n_stats = Ns;
  ix->tot[0] = tot2[0];
  ix->tot[1] = tot2[1];
  for (int f = 0; f < 2; ++f) {
    ix->avgdl[f] = (float)ix->tot[f] / (float)Ns;  // total_num_tokens as f32 / N as f32
    bm25_cache(ix->avgdl[f], ix->cache + 256 * f);
  }
  if (wts) {  // shared: at least V terms
    ix->w_text = wts->wt;
    ix->w_name = wts->wn;
  } else {
    std::vector<float> wt, wn;
    bm25_weights(Ns, df_t, df_n, V, wt, wn);
    ix->w_text = std::move(wt);
    ix->w_name = std::move(wn);
  }
  // facet field: Bm25Weight of a facet TermQuery (tf 1, no fieldnorms ->
  // FieldNormReader::constant(max_doc, 1) -> id 1, avg = total_num_tokens / N)
  const uint32_t VF = ix->n_fterms;
  ix->tot_f = tot_f;
  ix->df_facet.assign(df_f, df_f + VF);
  ix->fscore.assign(VF, 0.0f);
  if (ix->tot_f > 0) {
    float cf[256];
    ix->avgdl_f = (float)ix->tot_f / (float)Ns;
    bm25_cache(ix->avgdl_f, cf);
    ix->cache_f1 = cf[1];
    for (uint32_t t = 0; t < VF; ++t) ix->fscore[t] = bm25_weight(ix->df_facet[t], Ns) * (1.0f / (1.0f + ix->cache_f1));
  }
}

// How the current statistics relate to the build's (fg_index::same_stats,
// cup / cdn): a posting's score w * tf / (tf + c[fn]) changes by (w' / w) *
// (tf + c[fn]) / (tf + c'[fn]); over tf >= 1 the second factor lies between 1
// and its value at tf = 1, so per field it is bounded by the extremes over the
// fieldnorm ids of (1 + c) / (1 + c').
void relate_stats(fg_index* ix) {
  ix->same_stats = std::memcmp(ix->cache, ix->cache_b, sizeof ix->cache) == 0 &&
                   (ix->w_text.data() == ix->wb_text.data() || ix->w_text.vec() == ix->wb_text.vec()) &&
                   (ix->w_name.data() == ix->wb_name.data() || ix->w_name.vec() == ix->wb_name.vec());
  for (int f = 0; f < 2; ++f) {
    double up = 1.0, dn = 1.0;
    for (int fn = 0; fn < 256; ++fn) {
      const double q = (1.0 + (double)ix->cache_b[256 * f + fn]) / (1.0 + (double)ix->cache[256 * f + fn]);
      if (!std::isfinite(q)) continue;  // (a field without tokens: no posting scores in it)
      up = std::max(up, q);
      dn = std::min(dn, q);
    }
    ix->cup[f] = up;
    ix->cdn[f] = dn;
  }
}

}  // namespace

// Per-term bounds under the CURRENT statistics from the build-time tables
// (shared by the planner, fg_index_term_kth and the byte models).
namespace fgh {
// f32 factors with rdn * s_build <= s_now <= rup * s_build for every posting of
// term t (relate_stats' extremes times the weight ratio, over the fields the term
// has postings in, with a 2^-19 margin for the f32 roundings of both scores);
// exactly 1 when the statistics are the build's
void term_ratio(const fg_index* ix, uint32_t t, float* rdn, float* rup) {
  *rdn = *rup = 1.0f;
  if (ix->same_stats || t >= ix->n_terms) return;
  double lo = HUGE_VAL, hi = 0.0;
  for (int f = 0; f < (ix->has_name ? 2 : 1); ++f) {
    if ((f == 0 ? ix->df_text[t] : ix->df_name[t]) == 0) continue;  // no posting scores in the field
    const double wb = f == 0 ? ix->wb_text[t] : ix->wb_name[t], wn = f == 0 ? ix->w_text[t] : ix->w_name[t];
    if (!(wb > 0.0)) continue;
    const double r = wn / wb;
    hi = std::max(hi, r * ix->cup[f]);
    lo = std::min(lo, r * ix->cdn[f]);
  }
  if (!(hi > 0.0) || !std::isfinite(lo)) return;
  const double m = std::ldexp(1.0, -19);
  const double u = hi * (1.0 + m), d = lo * (1.0 - m);
  float fu = (float)u, fd = (float)d;
  if ((double)fu < u) fu = std::nextafter(fu, HUGE_VALF);
  if ((double)fd > d) fd = std::nextafter(fd, 0.0f);
  *rup = fu;
  *rdn = std::max(fd, 0.0f);
}
// the largest current score of term t (an upper bound; exact without a statistics change)
float term_max_scaled(const fg_index* ix, uint32_t t, float rup) {
  if (t >= ix->n_terms) return 0.0f;
  if (rup == 1.0f) return ix->tmaxs[t];
  const double v = (double)ix->tmaxs[t] * rup;
  float f = (float)v;
  if ((double)f < v) f = std::nextafter(f, HUGE_VALF);
  return f;
}
float term_max_now(const fg_index* ix, uint32_t t) {
  if (t >= ix->n_terms) return 0.0f;
  float rdn, rup;
  term_ratio(ix, t, &rdn, &rup);
  return term_max_scaled(ix, t, rup);
}
// a lower bound of term t's K-th best current score over the alive docs, K the
// smallest stored level >= k (0: none): the build's K'-th best for the smallest
// stored K' >= K + n_dead (at most n_dead of those docs died since), times rdn;
// or the namespace-wide floor of a doc-sharded namespace's shard when higher
float term_kth_now(const fg_index* ix, uint32_t t, uint32_t k, bool with_floor) {
  if (t >= ix->n_terms) return 0.0f;
  float v = 0.0f;
  const uint64_t need = (uint64_t)k + ix->n_dead;
  for (uint32_t j = 0; j < fg::kNumTopK; ++j) {
    if (fg::kTopKs[j] < need) continue;
    float rdn, rup;
    term_ratio(ix, t, &rdn, &rup);
    const double x = (double)ix->ktop[(size_t)t * fg::kNumTopK + j] * rdn;
    v = (float)x;
    if ((double)v > x) v = std::nextafter(v, 0.0f);
    break;
  }
  if (!with_floor) return v;
  if (const std::shared_ptr<const std::vector<float>> floor = std::atomic_load(&ix->kth_floor))
    for (uint32_t j = 0; j < fg::kNumTopK; ++j) {
      if (fg::kTopKs[j] < k) continue;
      v = std::max(v, (*floor)[(size_t)t * fg::kNumTopK + j]);
      break;
    }
  return v;
}
}  // namespace fgh
namespace {

// k_ktop over the build's scores (j.psc, j.alive -> j.ktop, and j.ladder when
// set): terms of <= kKtopChunk postings one workgroup each; longer terms in
// kKtopChunk-posting chunks (k_ktop_part), then one select per term over its
// chunks' best keys (k_ktop_big).  The chunk tables are the structure's; the key
// scratch is one stream-ordered temporary (freeing it does not synchronize the
// device: searches on other streams keep running).
static int ktop_pass(const fg_index* ix, fg::ScoreJob& j) {
  const size_t n_small = ix->n_kt, n_big = ix->n_kbig, n_chunks = ix->n_kchunks;
  const size_t kck_b = (8ull * n_chunks * fg::kTopKs[fg::kNumTopK - 1] + 255) & ~size_t(255);
  const size_t kcc_b = (4ull * n_chunks + 255) & ~size_t(255), kbs_b = 4ull * 3 * n_big;
  void* ktmp = nullptr;
  if (fgh::dev_malloc_async(&ktmp, kck_b + kcc_b + kbs_b + 16, kBuildStream) != hipSuccess)
    return fail(FG_EOOM, "hipMallocAsync(%zu) failed", kck_b + kcc_b + kbs_b);
  struct KtmpBack {
    void* p;
    ~KtmpBack() { (void)hipFreeAsync(p, kBuildStream); }
  } ktmp_back{ktmp};
  char* kb = static_cast<char*>(ktmp);
  uint32_t* d_kbs = reinterpret_cast<uint32_t*>(kb + kck_b + kcc_b);
  // per long term: alive postings 0, min alive score bits ~0, max 0 ([3][n_big])
  if (n_big) {
    HIPCHK(hipMemsetAsync(d_kbs, 0, 4ull * 3 * n_big, kBuildStream));
    HIPCHK(hipMemsetD32Async(d_kbs + n_big, (int)0xFFFFFFFFu, n_big, kBuildStream));
  }
  j.kt_tiny = ix->d_kt_tiny;
  j.n_tiny = ix->n_ktiny;
  j.kt_terms = ix->d_kt_terms;
  j.kb_terms = ix->d_kb_terms;
  j.kb_chunk0 = ix->d_kb_chunk0;
  j.kc_big = ix->d_kc_big;
  j.kc_start = ix->d_kc_start;
  j.kc_keys = reinterpret_cast<uint64_t*>(kb);
  j.kc_cnt = reinterpret_cast<uint32_t*>(kb + kck_b);
  j.kb_stat = d_kbs;
  j.n_big = (uint32_t)n_big;
  HIPCHK(fg::launch_ktop(j, (uint32_t)n_small, (uint32_t)n_chunks, (uint32_t)n_big, kBuildStream));
  return FG_OK;
}

// Every posting's score under the snapshot's CURRENT statistics (k_score) into
// `psc` (a build's bound block) or a stream-ordered temporary, for the bound
// kernels of a build and for fg_index_term_ladder.  `tmp` returns the temporary
// (freed stream-ordered by the caller); j gets the postings inputs, the weights
// and caches (inside tmp) and j.psc / j.cmax (cmax: the caller's, or a scratch
// part of tmp).
static int score_postings(const fg_index* ix, fg::ScoreJob& j, float* cmax, float* psc, void** tmp) {
  const uint32_t V = ix->n_terms;
  auto al = [](size_t x) { return (std::max<size_t>(x, 16) + 255) & ~size_t(255); };
  const size_t b_psc = psc ? 0 : al(4ull * ix->n_postings + 16), b_w = al(4ull * V), b_c = al(4ull * 512),
               b_cm = cmax ? 0 : al(4ull * ix->n_sc);
  if (fgh::dev_malloc_async(tmp, b_psc + 2 * b_w + b_c + b_cm, kBuildStream) != hipSuccess)
    return fail(FG_EOOM, "hipMallocAsync(%zu) failed", b_psc + 2 * b_w + b_c + b_cm);
  char* t = static_cast<char*>(*tmp);
  float* d_psc = psc ? psc : reinterpret_cast<float*>(t);
  float* d_wt = reinterpret_cast<float*>(t + b_psc);
  float* d_wn = reinterpret_cast<float*>(t + b_psc + b_w);
  float* d_cache = reinterpret_cast<float*>(t + b_psc + 2 * b_w);
  HIPCHK(hipMemcpyAsync(d_wt, ix->w_text.data(), 4ull * V, hipMemcpyHostToDevice, kBuildStream));
  HIPCHK(hipMemcpyAsync(d_wn, ix->w_name.data(), 4ull * V, hipMemcpyHostToDevice, kBuildStream));
  HIPCHK(hipMemcpyAsync(d_cache, ix->cache, 4ull * 512, hipMemcpyHostToDevice, kBuildStream));
  j.doc = ix->d.doc;
  j.tfn = ix->d.tfn;
  j.tfn_name = ix->d.tfn_name;
  j.esc_pos = ix->d.esc_pos;
  j.esc_tf = ix->d.esc_tf;
  j.n_esc = ix->d.n_esc;
  j.off = ix->d.off;
  j.dir = ix->d.dir;
  j.dir_off = ix->d.dir_off;
  j.tmeta = ix->d.tmeta;
  j.toff = ix->d.toff;
  j.w_text = d_wt;
  j.w_name = d_wn;
  j.cache = d_cache;
  j.psc = d_psc;
  j.cmax = cmax ? cmax : reinterpret_cast<float*>(t + b_psc + 2 * b_w + b_c);
  j.coff = ix->d.coff;
  j.sc_tf = ix->d_sc_tf;
  j.sc_tl = ix->d_sc_tl;
  j.sc_e0 = ix->d_sc_e0;
  j.sc_e1 = ix->d_sc_e1;
  j.n_terms = V;
  j.grid_cap = bg_grid_cap(ix->dev);
  HIPCHK(fg::launch_score(j, ix->n_scb, kBuildStream));
  return FG_OK;
}

// The bounds of a freshly built structure under its build statistics (which
// are its current ones): the posting scores into a temporary (k_score, with the
// block-max per 2048 postings), bucket / term / tile maxima (k_bucket), sub-tile
// maxima (k_tsub), per-term K-th best alive scores (k_ktop), and the read-back
// of tmaxs / ktop for the planner.  Once per build or merge: a commit's
// rescores of older segments share them (rescore_one).
int build_bounds(fg_index* ix, const std::vector<uint32_t>& alive) {
  const uint32_t V = ix->n_terms;
  HIPCHK(hipSetDevice(ix->dev));
  struct Part { size_t bytes; void** out; };
  float *d_psc, *d_bmax, *d_ktop, *d_cmax;
  uint64_t* d_tsub = nullptr;
  uint32_t *d_alive = nullptr, *d_tmaxs, *d_tmax;
  const Part parts[] = {
      {4ull * ix->n_postings + 16, reinterpret_cast<void**>(&d_psc)},  // 16 B of slack after the scores
      {alive.empty() ? 0 : 4ull * alive.size(), reinterpret_cast<void**>(&d_alive)},
      {4ull * ix->dir_entries, reinterpret_cast<void**>(&d_bmax)},
      {4ull * V, reinterpret_cast<void**>(&d_tmaxs)},
      {4ull * ix->tile_entries, reinterpret_cast<void**>(&d_tmax)},
      {4ull * V * fg::kNumTopK, reinterpret_cast<void**>(&d_ktop)},
      {4ull * ix->n_sc, reinterpret_cast<void**>(&d_cmax)},
      {8ull * ix->tile_entries, reinterpret_cast<void**>(&d_tsub)},
  };
  size_t total = 0;
  for (const Part& pt : parts) total += (std::max<size_t>(pt.bytes, 16) + 255) & ~size_t(255);
  if (!ix->spool) {
    ix->spool = std::make_shared<fgh::ScorePool>();
    ix->spool->dev = ix->dev;
  }
  auto sb = std::make_shared<fgh::ScoreBlock>();
  char* blk = static_cast<char*>(ix->spool->get(total));
  if (!blk) return fail(FG_EOOM, "bound tables: hipMalloc(%zu) failed", total);
  sb->p = blk;
  sb->bytes = total;
  sb->pool = ix->spool;
  ix->sblock = sb;
  {
    size_t o = 0;
    for (const Part& pt : parts) {
      *pt.out = pt.bytes ? blk + o : nullptr;
      o += (std::max<size_t>(pt.bytes, 16) + 255) & ~size_t(255);
    }
  }
  if (d_alive) HIPCHK(hipMemcpyAsync(d_alive, alive.data(), 4ull * alive.size(), hipMemcpyHostToDevice, kBuildStream));
  HIPCHK(hipMemsetAsync(d_tmaxs, 0, 4ull * V, kBuildStream));
  HIPCHK(hipMemsetAsync(d_tmax, 0, std::max<size_t>(4ull * ix->tile_entries, 16), kBuildStream));
  HIPCHK(hipMemsetAsync(d_ktop, 0, 4ull * V * fg::kNumTopK, kBuildStream));
  g_bt.mark("bound tables + uploads");
  fg::ScoreJob j{};
  void* tmp = nullptr;
  if (int rc = score_postings(ix, j, d_cmax, d_psc, &tmp)) return rc;
  struct TmpBack {
    void* p;
    ~TmpBack() { (void)hipFreeAsync(p, kBuildStream); }
  } tmp_back{tmp};
  j.alive = d_alive;
  j.bmax = d_bmax;
  j.tmaxs = d_tmaxs;
  j.tmax = d_tmax;
  j.ktop = d_ktop;
  j.bk_tf = ix->d_bk_tf;
  j.bk_tl = ix->d_bk_tl;
  j.bk_e0 = ix->d_bk_e0;
  j.bk_e1 = ix->d_bk_e1;
  j.n_dir = ix->dir_entries;
  HIPCHK(fg::launch_bucket(j, ix->n_bk, ix->n_docs, kBuildStream));
  j.tsub = d_tsub;
  j.tterm = ix->d_tterm;
  j.n_tterm = ix->n_tterm;
  j.n_tiles = ix->n_tiles;
  HIPCHK(fg::launch_tsub(j, ix->n_docs, kBuildStream));
  if (int rc = ktop_pass(ix, j)) return rc;
  g_bt.mark("bound launches");
  // tmaxs [V] then ktop [V * kNumTopK], read straight into a pooled pinned block
  {
    const size_t hb = 4ull * V * (1 + fg::kNumTopK);
    float* h = static_cast<float*>(ix->spool->get_host(hb));
    if (h) {
      sb->hp = h;
      sb->hbytes = hb;
    } else {
      sb->hown.resize((size_t)V * (1 + fg::kNumTopK));
      h = sb->hown.data();
    }
    if (on_background() && sb->hp) {
      // a background build: the read-back as a copy kernel of short workgroups
      // on its low-priority stream (pinned host memory is device-visible), not a
      // copy-engine transfer (those held searches up: tools/rescore_stall.py)
      HIPCHK(fg::launch_copy32(reinterpret_cast<uint32_t*>(h), d_tmaxs, V, j.grid_cap, kBuildStream));
      HIPCHK(fg::launch_copy32(reinterpret_cast<uint32_t*>(h + V), reinterpret_cast<const uint32_t*>(d_ktop),
                               (uint64_t)V * fg::kNumTopK, j.grid_cap, kBuildStream));
    } else {
      HIPCHK(hipMemcpyAsync(h, d_tmaxs, 4ull * V, hipMemcpyDeviceToHost, kBuildStream));
      HIPCHK(hipMemcpyAsync(h + V, d_ktop, 4ull * V * fg::kNumTopK, hipMemcpyDeviceToHost, kBuildStream));
    }
    HIPCHK(hipStreamSynchronize(kBuildStream));
    ix->tmaxs = h;
    ix->ktop = h + V;
  }
  g_bt.mark("device bounds");
  // the build's statistics are the bounds' reference
  ix->wb_text = ix->w_text;
  ix->wb_name = ix->w_name;
  std::memcpy(ix->cache_b, ix->cache, sizeof ix->cache);
  ix->h_alive = alive;
  ix->h_alive_b = ix->h_alive;
  ix->n_dead = 0;
  relate_stats(ix);
  ix->d.psc = d_psc;
  ix->d.bmax = d_bmax;
  ix->d.tmaxs = reinterpret_cast<const float*>(d_tmaxs);
  ix->d.tmax = reinterpret_cast<const float*>(d_tmax);
  ix->d.tsub = d_tsub;
  ix->d.cmax = d_cmax;
  ix->d.alive = d_alive;
  ix->device_bytes = ix->struct_bytes + total;
  return FG_OK;
}

// The statistics-independent half of a snapshot (postings, tf, fieldnorm ids,
// bucket directory, rank words, facet postings, chunk tables) is uploaded into
// ix->smem, then score_index computes the rest.  Consumes hp.  g: global
// statistics of a doc-sharded namespace (NULL: the shard's own).
int finish_index(int dev, HostPostings& hp, bool keep_host, fg_index** out, const fg_global_stats* g = nullptr) {
  auto ix = std::make_unique<fg_index>();
  ix->dev = dev;
  ix->mem.dev = dev;
  fgh::device_pools(dev, &ix->pool, &ix->pinned);
  ix->smem = std::make_shared<DevAllocs>();
  ix->smem->dev = dev;
  ix->n_docs = hp.n_docs;
  ix->n_terms = hp.n_terms;
  ix->n_vocab = hp.n_terms;
  ix->has_name = hp.has_name;
  ix->n_postings = hp.off[hp.n_terms];
  ix->tot_local[0] = hp.tot[0];
  ix->tot_local[1] = hp.tot[1];
  const uint64_t N = hp.n_docs;  // docs of this shard (array sizes)
  const uint32_t V = hp.n_terms;
  if (g && g->df_name == nullptr && hp.has_name) return fail(FG_EINVAL, "global statistics lack df_name for a shard with names");
  // doc -> position bucket directory (fg_internal.h DevIndex): bucket width
  // 2^B_t docs with B_t the largest shift keeping ~kBucketTarget postings per bucket
  std::vector<uint32_t> dir_off(V), tmeta(V);
  uint64_t nd = 0;
  for (uint32_t t = 0; t < V; ++t) {
    const uint64_t n = hp.off[t + 1] - hp.off[t];
    uint32_t B = 0;
    if (n == 0) B = 31;
    else while (B < 31 && (n << (B + 1)) <= (uint64_t)fg::kBucketTarget * N) ++B;
    const uint64_t nbk = ((N - 1) >> B) + 1;
    if (nd > 0xFFFFFFFFull) return fail(FG_EINVAL, "directory too large");
    dir_off[t] = (uint32_t)nd;
    tmeta[t] = B;
    nd += nbk + 1;
  }
  std::vector<uint32_t> dir(nd);
  // term ranges of about equal work (postings + a per-term constant): a million
  // mostly empty terms of a small segment cost one range grab per range, not
  // one per term, and the densest terms still spread over the threads
  std::vector<uint32_t> cuts{0};
  {
    const int nth = hw_threads(0);
    const uint64_t tot = hp.off[V] + 64ull * V, step = std::max<uint64_t>(1, tot / (uint64_t)(nth * 16));
    uint64_t acc = 0;
    for (uint32_t t = 0; t < V; ++t) {
      acc += (hp.off[t + 1] - hp.off[t]) + 64;
      if (acc >= step) { cuts.push_back(t + 1); acc = 0; }
    }
    if (cuts.back() != V) cuts.push_back(V);
  }
  parallel_dynamic((uint32_t)cuts.size() - 1, hw_threads(0), 1, [&](int, uint32_t rb, uint32_t re) {
    for (uint32_t t = cuts[rb]; t < cuts[re]; ++t) {
      const uint64_t b0 = hp.off[t], n = hp.off[t + 1] - b0;
      const uint32_t B = tmeta[t];
      const uint64_t nbk = ((N - 1) >> B) + 1;
      uint32_t* dt = dir.data() + dir_off[t];
      uint64_t p = 0;
      uint32_t maxocc = 0;
      for (uint64_t b = 0; b <= nbk; ++b) {
        const uint64_t lo = b << B;
        const uint64_t p0 = p;
        while (p < n && hp.doc[b0 + p] < lo) ++p;
        dt[b] = (uint32_t)p;
        if (b) maxocc = std::max<uint32_t>(maxocc, (uint32_t)(p - p0));
      }
      uint32_t S = 0;
      while ((1ull << S) <= maxocc) ++S;  // 2^S > largest bucket
      tmeta[t] = B | (S << 8);
    }
  });
  g_bt.mark("directory");
  // per-term tile maxima (4096-doc tiles of k_disj) for terms whose buckets are
  // no wider than a tile: one load gives a clause's bound over a tile; and the
  // tile directory beside them: tdir[toff + i] = the first posting of tile i
  // (n_tiles + 1 entries per term, the last = df), so a tile's posting range
  // is two adjacent loads -- 32 tiles per line, where the bucket directory puts
  // a dense term's consecutive tile boundaries 4096 >> B_t entries apart
  std::vector<uint32_t> toff(V, 0xFFFFFFFFu);
  const uint64_t n_tiles = ((uint64_t)N + (1u << fg::kDisjTileShift) - 1) >> fg::kDisjTileShift;
  uint64_t ntm = 0;
  for (uint32_t t = 0; t < V; ++t)
    if ((tmeta[t] & 0xFFu) <= fg::kDisjTileShift && hp.off[t + 1] > hp.off[t]) {
      if (ntm + n_tiles + 1 > 0xFFFFFFFFull) break;
      toff[t] = (uint32_t)ntm;
      ntm += n_tiles + 1;
    }
  std::vector<uint32_t> tdir(ntm);
  std::vector<uint32_t> tterm;  // the tile-table terms in toff order (k_tsub)
  tterm.reserve(ntm / (n_tiles + 1));
  for (uint32_t t = 0; t < V; ++t)
    if (toff[t] != 0xFFFFFFFFu) tterm.push_back(t);
  parallel_dynamic(V, hw_threads(0), 64, [&](int, uint32_t tb, uint32_t te) {
    for (uint32_t t = tb; t < te; ++t) {
      if (toff[t] == 0xFFFFFFFFu) continue;
      const uint32_t B = tmeta[t] & 0xFFu;
      const uint64_t nbk = ((N - 1) >> B) + 1;
      const uint32_t* dt = dir.data() + dir_off[t];
      for (uint64_t i = 0; i <= n_tiles; ++i)
        tdir[toff[t] + i] = dt[std::min<uint64_t>(i << (fg::kDisjTileShift - B), nbk)];
    }
  });
  ix->dir_entries = nd;
  ix->tile_entries = ntm;
  // chunk tables of the scoring kernels: (term, first posting) per <= kScoreChunk
  // postings, (term, first bucket) per <= kBucketChunk buckets, terms with postings
  // and of k_ktop (they depend on the postings only, so every rescore reuses
  // them): terms of <= kKtopChunk postings one workgroup each (kt); longer terms
  // (kb_terms) in kKtopChunk-posting chunks (kc_big / kc_start, the chunks of
  // long term x from kb_chunk0[x])
  // k_score / k_bucket chunks are PACKED: a long term's slice of kScoreChunk
  // postings (kBucketChunk directory entries), or several whole short terms
  // (<= kPackTerms term ids, <= a slice's postings / entries together) -- the
  // long tail of a vocabulary in a workgroup per term was most of a small
  // segment's scoring time
  std::vector<uint32_t> kt, kt_tiny, coff(V), kb_terms, kb_chunk0, kc_big, kc_start;
  std::vector<uint32_t> sc_tf, sc_tl, bk_tf, bk_tl, bk_e0, bk_e1;
  std::vector<uint64_t> sc_e0, sc_e1;
  uint32_t n_cmax = 0;
  {
    // postings: pack [pt0, t) open while short terms fit
    uint32_t pt0 = 0;
    uint64_t pe0 = 0;
    bool open = false;
    auto flush_sc = [&](uint32_t t_end) {  // terms [pt0, t_end)
      if (!open) return;
      sc_tf.push_back(pt0);
      sc_tl.push_back(t_end - 1);
      sc_e0.push_back(pe0);
      sc_e1.push_back(hp.off[t_end]);
      open = false;
    };
    for (uint32_t t = 0; t < V; ++t) {
      const uint64_t n = hp.off[t + 1] - hp.off[t];
      coff[t] = n_cmax;  // the term's first block-max entry (DevIndex::cmax: kChunk postings each)
      n_cmax += (uint32_t)((n + fg::kChunk - 1) / fg::kChunk);
      if (n >= fg::kScoreChunk) {
        flush_sc(t);
        for (uint64_t f = 0; f < n; f += fg::kScoreChunk) {
          sc_tf.push_back(t);
          sc_tl.push_back(t);
          sc_e0.push_back(hp.off[t] + f);
          sc_e1.push_back(hp.off[t] + std::min<uint64_t>(n, f + fg::kScoreChunk));
        }
        continue;
      }
      if (open && (hp.off[t + 1] - pe0 > fg::kScoreChunk || t - pt0 >= fg::kPackTerms)) flush_sc(t);
      if (!open) {
        pt0 = t;
        pe0 = hp.off[t];
        open = true;
      }
    }
    flush_sc(V);
  }
  {
    // directory entries (each term: its nbk buckets + the end entry)
    uint32_t pt0 = 0, pe0 = 0;
    bool open = false;
    auto flush_bk = [&](uint32_t t_end) {
      if (!open) return;
      bk_tf.push_back(pt0);
      bk_tl.push_back(t_end - 1);
      bk_e0.push_back(pe0);
      bk_e1.push_back(t_end < V ? dir_off[t_end] : (uint32_t)nd);
      open = false;
    };
    for (uint32_t t = 0; t < V; ++t) {
      const uint32_t ne = (t + 1 < V ? dir_off[t + 1] : (uint32_t)nd) - dir_off[t];  // nbk + 1
      if (ne > fg::kBucketChunk) {
        flush_bk(t);
        for (uint32_t f = 0; f < ne; f += fg::kBucketChunk) {
          bk_tf.push_back(t);
          bk_tl.push_back(t);
          bk_e0.push_back(dir_off[t] + f);
          bk_e1.push_back(dir_off[t] + std::min<uint32_t>(ne, f + fg::kBucketChunk));
        }
        continue;
      }
      if (open && (dir_off[t] + ne - pe0 > fg::kBucketChunk || t - pt0 >= fg::kPackTerms)) flush_bk(t);
      if (!open) {
        pt0 = t;
        pe0 = dir_off[t];
        open = true;
      }
    }
    flush_bk(V);
  }
  for (uint32_t t = 0; t < V; ++t) {
    const uint64_t n = hp.off[t + 1] - hp.off[t];
    if (!n) continue;
    if (n <= fg::kKtopTiny) {
      kt_tiny.push_back(t);
      continue;
    }
    if (n <= fg::kKtopChunk) {
      kt.push_back(t);
      continue;
    }
    kb_chunk0.push_back((uint32_t)kc_big.size());
    for (uint64_t st = 0; st < n; st += fg::kKtopChunk) {
      kc_big.push_back((uint32_t)kb_terms.size());
      kc_start.push_back((uint32_t)st);
    }
    kb_terms.push_back(t);
  }
  kb_chunk0.push_back((uint32_t)kc_big.size());
  if (sc_tf.size() > 0x7FFFFFFFull || bk_tf.size() > 0x7FFFFFFFull) return fail(FG_EUNSUPPORTED, "index too large");
  HIPCHK(hipSetDevice(dev));
  DevAllocs& sm = *ix->smem;
  uint64_t& bytes = ix->struct_bytes;
  int rc;
  uint32_t *d_doc, *d_dir, *d_dir_off, *d_tmeta, *d_toff, *d_tdir, *d_fdoc, *d_tterm, *d_esc_tf = nullptr;
  uint16_t *d_tfn = nullptr, *d_tfn_name = nullptr;
  uint64_t* d_esc_pos = nullptr;
  uint64_t *d_off, *d_foff;
  uint32_t *d_sctf, *d_sctl, *d_bktf, *d_bktl, *d_bke0, *d_bke1, *d_kt, *d_ktt, *d_coff, *d_kbt, *d_kb0, *d_kcb, *d_kcs;
  uint64_t *d_sce0, *d_sce1;
  // the postings' payloads (DevIndex::tfn): per field (fieldnorm id of the doc
  // << 8) | tf, 2 B per posting -- what a query-time score needs besides the
  // clause's weight, beside the doc id -- and the postings whose tf does not fit
  // the byte (>= 255) in a sorted escape list
  std::vector<uint16_t> tfn(hp.tf.size()), tfn_name(hp.has_name ? hp.tf.size() : 0);
  std::vector<uint64_t> esc_pos;
  std::vector<uint32_t> esc_tf;
  {
    const size_t np = hp.tf.size(), piece = (np + 1023) / 1024;  // > 2^32 postings: 64-bit pieces
    std::vector<std::vector<uint64_t>> ep(1024);
    parallel_dynamic(1024, hw_threads(0), 8, [&](int, uint32_t b, uint32_t e) {
      for (uint32_t pc = b; pc < e; ++pc)
        for (size_t i = (size_t)pc * piece; i < std::min(np, (size_t)(pc + 1) * piece); ++i) {
          const uint32_t d = hp.doc[i], tt = hp.tf[i] & 0xFFFFu, tn = hp.tf[i] >> 16;
          tfn[i] = (uint16_t)fg::tfn_pack(tt, hp.fn_text[d]);
          if (hp.has_name) tfn_name[i] = (uint16_t)(tn ? fg::tfn_pack(tn, hp.fn_name[d]) : 0u);
          if (tt >= fg::kTfEsc || (hp.has_name && tn >= fg::kTfEsc)) ep[pc].push_back(i);
        }
    });
    for (auto& v : ep)
      for (uint64_t i : v) {
        esc_pos.push_back(i);
        esc_tf.push_back(hp.tf[i]);
      }
  }
  {
    UploadBatch ub;
    ub.add(hp.doc.data(), hp.doc.size(), &d_doc);
    ub.add(tfn.data(), tfn.size(), &d_tfn);
    if (hp.has_name) ub.add(tfn_name.data(), tfn_name.size(), &d_tfn_name);
    if (!esc_pos.empty()) {
      ub.add(esc_pos.data(), esc_pos.size(), &d_esc_pos);
      ub.add(esc_tf.data(), esc_tf.size(), &d_esc_tf);
    }
    ub.add(hp.off.data(), hp.off.size(), &d_off);
    ub.add(dir.data(), dir.size(), &d_dir);
    ub.add(dir_off.data(), dir_off.size(), &d_dir_off);
    ub.add(toff.data(), toff.size(), &d_toff);
    ub.add(tdir.data(), tdir.size(), &d_tdir);
    ub.add(tterm.data(), tterm.size(), &d_tterm);
    ub.add(hp.fdoc.data(), hp.fdoc.size(), &d_fdoc);
    ub.add(hp.foff.data(), hp.foff.size(), &d_foff);
    ub.add(sc_tf.data(), sc_tf.size(), &d_sctf);
    ub.add(sc_tl.data(), sc_tl.size(), &d_sctl);
    ub.add(sc_e0.data(), sc_e0.size(), &d_sce0);
    ub.add(sc_e1.data(), sc_e1.size(), &d_sce1);
    ub.add(bk_tf.data(), bk_tf.size(), &d_bktf);
    ub.add(bk_tl.data(), bk_tl.size(), &d_bktl);
    ub.add(bk_e0.data(), bk_e0.size(), &d_bke0);
    ub.add(bk_e1.data(), bk_e1.size(), &d_bke1);
    ub.add(kt.data(), kt.size(), &d_kt);
    ub.add(kt_tiny.data(), kt_tiny.size(), &d_ktt);
    ub.add(kb_terms.data(), kb_terms.size(), &d_kbt);
    ub.add(kb_chunk0.data(), kb_chunk0.size(), &d_kb0);
    ub.add(kc_big.data(), kc_big.size(), &d_kcb);
    ub.add(kc_start.data(), kc_start.size(), &d_kcs);
    ub.add(coff.data(), coff.size(), &d_coff);
    if ((rc = ub.commit(sm, &bytes))) return rc;
  }
  std::vector<uint16_t>().swap(tfn);
  std::vector<uint16_t>().swap(tfn_name);
  std::vector<uint32_t>().swap(hp.tf);
  std::vector<uint32_t>().swap(dir);
  std::vector<uint32_t>().swap(tdir);
  g_bt.mark("upload");
  // rank words (fg_internal.h DevIndex) for the terms with df >= N / kRankDiv,
  // densest first (ties by term id), within a budget of the snapshot's own:
  // FUGU_RANK_FACTOR (default kRankFactor) times its postings' bytes (doc id +
  // tf + score, 12 B each), at most FUGU_RANK_GIB -- so a namespace's share
  // depends on its size, not on how many namespaces were built on the device
  // before it.  A term with df >= N / kRankPlainDiv (FUGU_RANK_PLAIN_DIV) gets
  // plain rank words (8 B per 32 docs), a sparser one sparse rank words (8 B per
  // 1024-doc block + 8 B per word holding any of its docs) unless plain ones
  // cost it less (small snapshots).  A quarter of the free memory caps them
  // only when HBM is short, and a failed allocation is retried with half the
  // terms (down to none), so a build never fails for want of them.  They hang
  // on doc ids only, so rescored snapshots share them.
  std::vector<uint32_t> by_df;
  for (uint32_t t = 0; t < V; ++t)
    if (hp.off[t + 1] > hp.off[t] && (hp.off[t + 1] - hp.off[t]) * fg::kRankDiv >= N) by_df.push_back(t);
  std::stable_sort(by_df.begin(), by_df.end(), [&](uint32_t a, uint32_t b) {
    return hp.off[a + 1] - hp.off[a] > hp.off[b + 1] - hp.off[b];
  });
  const uint32_t rank_words = (uint32_t)((N + 31) / 32), sblocks = (N + 1023) / 1024;
  const uint32_t pdiv = [] {
    const char* e = getenv("FUGU_RANK_PLAIN_DIV");
    return e && *e ? (uint32_t)std::max(1l, atol(e)) : fg::kRankPlainDiv;
  }();
  auto plain_df = [&](uint32_t t) { return (hp.off[t + 1] - hp.off[t]) * pdiv >= N; };
  // the words of each sparse candidate that hold any of its docs
  std::vector<uint32_t> nwords(by_df.size(), 0);
  parallel_dynamic((uint32_t)by_df.size(), hw_threads(0), 16, [&](int, uint32_t b, uint32_t e) {
    for (uint32_t i = b; i < e; ++i) {
      const uint32_t t = by_df[i];
      if (plain_df(t)) continue;
      uint32_t n = 0, last = 0xFFFFFFFFu;
      for (uint64_t p = hp.off[t]; p < hp.off[t + 1]; ++p) {
        const uint32_t w = hp.doc[p] >> 5;
        n += w != last;
        last = w;
      }
      nwords[i] = n;
    }
  });
  std::vector<uint32_t> rank_terms, sparse_terms, sparse_nw;
  uint64_t* d_rank = nullptr;
  uint64_t* d_srank = nullptr;
  uint64_t n_swords = 0;
  {
    const char* v = getenv("FUGU_RANK_GIB");
    const uint64_t cap = v && *v ? (uint64_t)(atof(v) * (double)(1ull << 30)) : fg::kRankBudget;
    const char* f = getenv("FUGU_RANK_FACTOR");
    const double factor = f && *f ? atof(f) : fg::kRankFactor;
    const uint64_t want = std::min<uint64_t>(cap, (uint64_t)(factor * 12.0 * (double)hp.off[V]));
    size_t free_b = ~size_t(0), total_b = 0;
    if (want > (256ull << 20)) HIPCHK(hipMemGetInfo(&free_b, &total_b));  // (~1 ms: not for a small segment's)
    const uint64_t brk = std::min<uint64_t>(want, free_b / 4);
    uint64_t used = 0;
    for (size_t i = 0; i < by_df.size(); ++i) {
      const uint64_t cp = rank_words * 8ull, cs = (sblocks + (uint64_t)nwords[i]) * 8ull;
      const bool plain = plain_df(by_df[i]) || cp <= cs;
      const uint64_t c = plain ? cp : cs;
      if (used + c > brk || rank_terms.size() + sparse_terms.size() >= fg::kMaxDense) break;
      if (!plain && n_swords + nwords[i] >= 0xFFFFFFFFull) break;  // srank_w indices are u32
      used += c;
      if (plain) {
        rank_terms.push_back(by_df[i]);
      } else {
        sparse_terms.push_back(by_df[i]);
        sparse_nw.push_back(nwords[i]);
        n_swords += nwords[i];
      }
    }
    while (!rank_terms.empty()) {
      void* q = nullptr;
      if (fgh::dev_malloc(&q, rank_words * 8ull * rank_terms.size()) == hipSuccess) {
        sm.ptrs.push_back(q);
        bytes += rank_words * 8ull * rank_terms.size();
        d_rank = static_cast<uint64_t*>(q);
        break;
      }
      (void)hipGetLastError();
      rank_terms.resize(rank_terms.size() / 2);
    }
    while (!sparse_terms.empty()) {
      const uint64_t sb = (sblocks * (uint64_t)sparse_terms.size() + 1 + n_swords) * 8ull;
      void* q = nullptr;
      if (fgh::dev_malloc(&q, sb) == hipSuccess) {
        sm.ptrs.push_back(q);
        bytes += sb;
        d_srank = static_cast<uint64_t*>(q);
        break;
      }
      (void)hipGetLastError();
      sparse_terms.resize(sparse_terms.size() / 2);
      sparse_nw.resize(sparse_terms.size());
      n_swords = 0;
      for (uint32_t n : sparse_nw) n_swords += n;
    }
  }
  g_bt.mark("rank words: budget");
  if (!sparse_terms.empty()) {
    // built on the host from the postings: per term its block entries, then
    // the zero word and all terms' words (term by term), one upload
    const uint32_t ns = (uint32_t)sparse_terms.size();
    const uint32_t first_slot = (uint32_t)rank_terms.size() + 1;
    std::vector<uint64_t> wbase(ns + 1, 1);
    for (uint32_t s2 = 0; s2 < ns; ++s2) wbase[s2 + 1] = wbase[s2] + sparse_nw[s2];
    std::vector<uint64_t> hs(sblocks * (uint64_t)ns + 1 + n_swords);
    hs[sblocks * (uint64_t)ns] = 0;
    parallel_dynamic(ns, hw_threads(0), 16, [&](int, uint32_t b, uint32_t e) {
      for (uint32_t s2 = b; s2 < e; ++s2) {
        const uint32_t t = sparse_terms[s2];
        uint64_t* blk = hs.data() + (uint64_t)s2 * sblocks;
        uint64_t* wd = hs.data() + (uint64_t)ns * sblocks;
        std::fill(blk, blk + sblocks, 0ull);
        uint64_t cur = wbase[s2];
        uint32_t last = 0xFFFFFFFFu;
        for (uint64_t p = hp.off[t]; p < hp.off[t + 1]; ++p) {
          const uint32_t d = hp.doc[p], w = d >> 5;
          if (w != last) {
            if (last != 0xFFFFFFFFu) ++cur;
            last = w;
            wd[cur] = (uint64_t)(p - hp.off[t]) << 32;  // postings before the word's first doc
            uint64_t& be = blk[fg::srank_block(d)];
            if (!(uint32_t)be) be = cur << 32;  // the block's first word
            be |= 1ull << (w & 31u);
          }
          wd[cur] |= 1ull << (d & 31u);
        }
      }
    });
    HIPCHK(hipMemcpyAsync(d_srank, hs.data(), hs.size() * 8, hipMemcpyHostToDevice, kBuildStream));
    HIPCHK(hipStreamSynchronize(kBuildStream));
    for (uint32_t s2 = 0; s2 < ns; ++s2) tmeta[sparse_terms[s2]] |= ((first_slot + s2) << 16) | 0x80000000u;
  }
  g_bt.mark("rank words: sparse");
  if (!rank_terms.empty()) {
    // one k_rank launch for every rank term: per slot the term's posting range
    std::vector<uint64_t> sb(rank_terms.size());
    std::vector<uint32_t> sn(rank_terms.size());
    for (uint32_t s2 = 0; s2 < rank_terms.size(); ++s2) {
      const uint32_t t = rank_terms[s2];
      sb[s2] = hp.off[t];
      sn[s2] = (uint32_t)(hp.off[t + 1] - hp.off[t]);
      tmeta[t] |= ((s2 + 1) << 16) | 0x80000000u;
    }
    // the slot tables are stream-ordered temporaries: freeing them does not
    // synchronise the device (hipFree would wait for every stream's work)
    void* d_tab = nullptr;
    const size_t nb = sb.size() * 8, nn = sn.size() * 4;
    if (fgh::dev_malloc_async(&d_tab, nb + nn + 16, kBuildStream) != hipSuccess) return fail(FG_EOOM, "hipMallocAsync failed");
    uint64_t* d_sb = static_cast<uint64_t*>(d_tab);
    uint32_t* d_sn = reinterpret_cast<uint32_t*>(static_cast<char*>(d_tab) + nb);
    HIPCHK(hipMemcpyAsync(d_sb, sb.data(), nb, hipMemcpyHostToDevice, kBuildStream));
    HIPCHK(hipMemcpyAsync(d_sn, sn.data(), nn, hipMemcpyHostToDevice, kBuildStream));
    HIPCHK(fg::launch_rank(d_doc, d_sb, d_sn, (uint32_t)rank_terms.size(), rank_words, d_rank, kBuildStream));
    HIPCHK(hipFreeAsync(d_tab, kBuildStream));
    HIPCHK(hipStreamSynchronize(kBuildStream));
  }
  ix->n_rank = (uint32_t)(rank_terms.size() + sparse_terms.size());
  ix->n_srank_words = sparse_terms.empty() ? 0 : 1 + n_swords;
  if ((rc = dev_upload(sm, tmeta.data(), tmeta.size(), &d_tmeta, &bytes))) return rc;
  ix->tmeta = tmeta;
  g_bt.mark("rank words");
  ix->d.tfn = d_tfn;
  ix->d.tfn_name = d_tfn_name;
  ix->d.esc_pos = d_esc_pos;
  ix->d.esc_tf = d_esc_tf;
  ix->d.n_esc = esc_pos.size();
  ix->d_sc_tf = d_sctf;
  ix->d_sc_tl = d_sctl;
  ix->d_sc_e0 = d_sce0;
  ix->d_sc_e1 = d_sce1;
  ix->d_bk_tf = d_bktf;
  ix->d_bk_tl = d_bktl;
  ix->d_bk_e0 = d_bke0;
  ix->d_bk_e1 = d_bke1;
  ix->d_kt_tiny = d_ktt;
  ix->n_ktiny = (uint32_t)kt_tiny.size();
  ix->d_tterm = d_tterm;
  ix->n_tterm = (uint32_t)tterm.size();
  ix->n_tiles = (uint32_t)n_tiles;
  ix->d_kt_terms = d_kt;
  ix->d_kb_terms = d_kbt;
  ix->d_kb_chunk0 = d_kb0;
  ix->d_kc_big = d_kcb;
  ix->d_kc_start = d_kcs;
  ix->n_kbig = (uint32_t)kb_terms.size();
  ix->n_kchunks = (uint32_t)kc_big.size();
  ix->n_sc = n_cmax;
  ix->n_scb = (uint32_t)sc_tf.size();
  ix->n_bk = (uint32_t)bk_tf.size();
  ix->n_kt = (uint32_t)kt.size();
  ix->d.doc = d_doc;
  ix->d.off = d_off;
  ix->d.dir = d_dir;
  ix->d.dir_off = d_dir_off;
  ix->d.tmeta = d_tmeta;
  ix->d.rank = d_rank;
  ix->d.srank = d_srank;
  ix->d.srank_w = d_srank ? d_srank + (uint64_t)sblocks * sparse_terms.size() : nullptr;
  ix->d.n_prank = (uint32_t)rank_terms.size();
  ix->d.srank_blocks = sblocks;
  ix->d.toff = d_toff;
  ix->d.tdir = d_tdir;
  ix->d.coff = d_coff;
  ix->d.fdoc = d_fdoc;
  ix->d.foff = d_foff;
  ix->d.n_docs = hp.n_docs;
  ix->d.n_terms = hp.n_terms;
  ix->d.has_name = hp.has_name ? 1u : 0u;
  ix->d.n_fterms = hp.n_fterms;
  ix->d.rank_words = rank_words;
  // host bookkeeping of the structure
  ix->off = std::move(hp.off);
  ix->df_text = std::move(hp.df_text);
  ix->df_name = std::move(hp.df_name);
  {
    std::vector<uint32_t> fd(V, 0), ld(V, 0);
    for (uint32_t t = 0; t < V; ++t)
      if (ix->off[t + 1] > ix->off[t]) {
        fd[t] = hp.doc[ix->off[t]];
        ld[t] = hp.doc[ix->off[t + 1] - 1];
      }
    ix->first_doc = std::move(fd);
    ix->last_doc = std::move(ld);
  }
  if (keep_host) ix->h_doc = std::make_shared<const std::vector<uint32_t>>(std::move(hp.doc));
  const uint32_t VF = hp.n_fterms;
  ix->n_fterms = VF;
  ix->df_facet_local = hp.df_facet;
  ix->tot_f_local = hp.tot_f;
  {
    std::vector<uint32_t> ff(VF, 0), fl(VF, 0);
    for (uint32_t t = 0; t < VF; ++t)
      if (hp.foff[t + 1] > hp.foff[t]) {
        ff[t] = hp.fdoc[hp.foff[t]];
        fl[t] = hp.fdoc[hp.foff[t + 1] - 1];
      }
    ix->ffirst = std::move(ff);
    ix->flast = std::move(fl);
  }
  ix->foff = std::move(hp.foff);
  // statistics: the shard's own, or the namespace's global ones
  if (g && VF && !g->df_facet) return fail(FG_EINVAL, "global statistics lack df_facet for a faceted shard");
  if (g && VF)
    for (uint32_t t = 0; t < VF; ++t)
      if (g->df_facet[t] < ix->df_facet_local[t]) return fail(FG_EINVAL, "global facet df of term %u is below this shard's", t);
  const uint64_t tot_local[2] = {ix->tot_local[0], ix->tot_local[1]};
  set_stats(ix.get(), g ? g->n_docs : N, g ? g->tot_tokens : tot_local, g ? g->df_text : ix->df_text.data(),
            g ? g->df_name : ix->df_name.data(), g ? g->tot_facet_tokens : ix->tot_f_local,
            g && VF ? g->df_facet : ix->df_facet_local.data(), nullptr);
  g_bt.mark("weights");
  if ((rc = build_bounds(ix.get(), hp.alive))) return rc;
  g_bt.mark("tail");
  *out = ix.release();
  return FG_OK;
}

// Sorted (term, tf) runs of one field of one doc into `runs` (term << 0, tf).
inline void doc_runs(const uint32_t* tok, uint64_t len, std::vector<uint32_t>& scratch,
                     std::vector<std::pair<uint32_t, uint32_t>>& runs) {
  runs.clear();
  if (!len) return;
  scratch.assign(tok, tok + len);
  std::sort(scratch.begin(), scratch.end());
  for (size_t i = 0; i < scratch.size();) {
    size_t j = i;
    while (j < scratch.size() && scratch[j] == scratch[i]) ++j;
    runs.emplace_back(scratch[i], (uint32_t)(j - i));
    i = j;
  }
}

// Facet postings from per-doc FacetTokenizer tokens (fg_docs_input): each doc
// once per distinct token (df), every token counted in total_num_tokens.
int build_facets(const fg_docs_input* in, HostPostings& hp, int T) {
  hp.n_fterms = 0;
  hp.foff.assign(1, 0);
  hp.fdoc.clear();
  hp.df_facet.clear();
  hp.tot_f = 0;
  if (!in->facet_off) return FG_OK;
  const uint32_t N = in->n_docs, VF = in->n_facet_terms;
  if (in->facet_off[0] != 0 || (!in->facet_tok && in->facet_off[N] > 0))
    return fail(FG_EINVAL, "bad facet token arrays");
  for (uint32_t d = 0; d < N; ++d)
    if (in->facet_off[d + 1] < in->facet_off[d]) return fail(FG_EINVAL, "facet_off not monotone at doc %u", d);
  hp.n_fterms = VF;
  hp.tot_f = in->facet_off[N];
  std::vector<std::vector<uint32_t>> cnt(T);
  std::atomic<bool> bad{false};
  auto runs = [&](uint32_t d, std::vector<uint32_t>& sc) {
    sc.assign(in->facet_tok + in->facet_off[d], in->facet_tok + in->facet_off[d + 1]);
    std::sort(sc.begin(), sc.end());
    sc.erase(std::unique(sc.begin(), sc.end()), sc.end());
  };
  parallel_ranges(N, T, [&](int t, uint32_t b, uint32_t e) {
    cnt[t].assign(VF, 0);
    std::vector<uint32_t> sc;
    for (uint32_t d = b; d < e; ++d) {
      runs(d, sc);
      for (uint32_t x : sc) {
        if (x >= VF) { bad = true; return; }
        cnt[t][x]++;
      }
    }
  });
  if (bad) return fail(FG_EINVAL, "facet token id >= n_facet_terms");
  std::vector<std::vector<uint64_t>> cur(T);
  hp.foff.assign(VF + 1, 0);
  hp.df_facet.assign(VF, 0);
  uint64_t acc = 0;
  for (int t = 0; t < T; ++t) cur[t].assign(VF, 0);
  for (uint32_t x = 0; x < VF; ++x) {
    hp.foff[x] = acc;
    for (int t = 0; t < T; ++t) {
      if (cnt[t].empty()) continue;
      cur[t][x] = acc;
      acc += cnt[t][x];
      hp.df_facet[x] += cnt[t][x];
    }
  }
  hp.foff[VF] = acc;
  hp.fdoc.resize(acc);
  parallel_ranges(N, T, [&](int t, uint32_t b, uint32_t e) {
    std::vector<uint32_t> sc;
    for (uint32_t d = b; d < e; ++d) {
      runs(d, sc);
      for (uint32_t x : sc) hp.fdoc[cur[t][x]++] = d;
    }
  });
  return FG_OK;
}

}  // namespace

// ================================================================ C ABI
extern "C" {

const char* fg_last_error(void) { return g_err.c_str(); }
const char* fg_version(void) { return "libfugu 0.4 (gfx950)"; }
int fg_abi_version(void) { return FG_ABI_VERSION; }

int fg_device_count(int* out) {
  if (!out) return fail(FG_EINVAL, "out is NULL");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *out = n;
  return FG_OK;
}

int fg_ctx_create(int ndev, const int* devs, fg_ctx** out) {
  if (!out || ndev < 0 || (ndev > 0 && !devs)) return fail(FG_EINVAL, "bad arguments");
  auto c = std::make_unique<fg_ctx>();
  if (ndev == 0) {
    int n = 0;
    fg_device_count(&n);
    if (n == 0) return fail(FG_ENODEV, "no HIP device visible");
    c->devs.push_back(0);
  } else {
    c->devs.assign(devs, devs + ndev);
  }
  for (int d : c->devs) {
    int rc = check_device(d);
    if (rc) return rc;
  }
  // fg_search_sharded moves each shard's top-k to the first shard's device
  // with hipMemcpyPeerAsync: direct xGMI transfers need peer access, so it is
  // enabled on every pair that supports it (already-enabled is fine).  A pair
  // without it still works (the runtime stages the copy through the host);
  // fg_ctx_peer_access reports which pairs are direct.  The caller's current
  // device is restored.
  int prev = 0;
  HIPCHK(hipGetDevice(&prev));
  for (int a : c->devs)
    for (int b : c->devs) {
      if (a == b) continue;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) {
        (void)hipGetLastError();
        continue;
      }
      if (hipSetDevice(a) != hipSuccess) break;
      const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
      (void)hipGetLastError();
      if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) c->peers.emplace_back(a, b);
    }
  (void)hipSetDevice(prev);
  *out = c.release();
  return FG_OK;
}

int fg_ctx_destroy(fg_ctx* ctx) {
  delete ctx;
  return FG_OK;
}

int fg_ctx_peer_access(const fg_ctx* ctx, int a, int b, int* enabled) {
  if (!ctx || !enabled) return fail(FG_EINVAL, "bad arguments");
  *enabled = std::find(ctx->peers.begin(), ctx->peers.end(), std::make_pair(a, b)) != ctx->peers.end() ? 1 : 0;
  return FG_OK;
}

int fg_index_build_from_docs(fg_ctx* ctx, int dev, const fg_docs_input* in, fg_index** out) {
  return fg_index_build_from_docs_global(ctx, dev, in, nullptr, out);
}

int fg_docs_stats(const fg_docs_input* in, uint32_t* df_text, uint32_t* df_name, uint64_t* tot_tokens2) {
  if (!in || !df_text || !df_name || !tot_tokens2 || !in->text_off || (!in->text_tok && in->text_off[in->n_docs] > 0))
    return fail(FG_EINVAL, "bad arguments");
  const uint32_t N = in->n_docs, V = in->n_terms;
  const bool has_name_in = in->name_off && in->name_tok;
  const int T = hw_threads(in->threads);
  std::vector<std::vector<uint32_t>> dft(T), dfn(T);
  std::vector<uint64_t> tt(T, 0), tn(T, 0);
  std::atomic<bool> bad{false};
  parallel_ranges(N, T, [&](int t, uint32_t b, uint32_t e) {
    dft[t].assign(V, 0);
    dfn[t].assign(V, 0);
    std::vector<uint32_t> scratch;
    std::vector<std::pair<uint32_t, uint32_t>> runs;
    for (uint32_t d = b; d < e; ++d) {
      const uint64_t lt = in->text_off[d + 1] - in->text_off[d];
      tt[t] += lt;
      doc_runs(in->text_tok + in->text_off[d], lt, scratch, runs);
      for (auto& r : runs) {
        if (r.first >= V) { bad = true; return; }
        dft[t][r.first]++;
      }
      if (has_name_in) {
        const uint64_t ln = in->name_off[d + 1] - in->name_off[d];
        tn[t] += ln;
        doc_runs(in->name_tok + in->name_off[d], ln, scratch, runs);
        for (auto& r : runs) {
          if (r.first >= V) { bad = true; return; }
          dfn[t][r.first]++;
        }
      }
    }
  });
  if (bad) return fail(FG_EINVAL, "token id >= n_terms");
  std::fill(df_text, df_text + V, 0u);
  std::fill(df_name, df_name + V, 0u);
  tot_tokens2[0] = tot_tokens2[1] = 0;
  for (int t = 0; t < T; ++t) {
    if (dft[t].empty()) continue;
    for (uint32_t v = 0; v < V; ++v) {
      df_text[v] += dft[t][v];
      df_name[v] += dfn[t][v];
    }
    tot_tokens2[0] += tt[t];
    tot_tokens2[1] += tn[t];
  }
  return FG_OK;
}

int fg_docs_facet_stats(const fg_docs_input* in, uint32_t* df_facet, uint64_t* tot_facet) {
  if (!in || !tot_facet || (in->facet_off && in->n_facet_terms && !df_facet)) return fail(FG_EINVAL, "bad arguments");
  HostPostings hp;
  if (int rc = build_facets(in, hp, hw_threads(in->threads))) return rc;
  if (hp.n_fterms) std::copy(hp.df_facet.begin(), hp.df_facet.end(), df_facet);
  *tot_facet = hp.tot_f;
  return FG_OK;
}

}  // extern "C"

// A build's own term dictionary (fg_index::tmap).  Its docs' distinct terms are
// marked in a vocabulary bitset; when they are fewer than 1/kLocalDiv of the
// vocabulary (a commit's 1000 new docs hold ~2% of a 10M-doc namespace's), the
// build runs on local ids: the tokens renumbered in vocabulary order (a rank in
// the bitset) and the statistics gathered to them, so its work and its device
// arrays scale with its own terms, not the vocabulary's.  The marking stops as
// soon as the count passes the limit (a large build decides within its first
// docs).  L.tmap stays empty: vocabulary ids.
namespace {
constexpr uint32_t kLocalDiv = 4;
struct LocalDict {
  std::vector<uint32_t> tmap, ttok, ntok, df_t, df_n;
  fg_docs_input in{};
  fg_global_stats g{};
};
int local_dict(const fg_docs_input* in, const fg_global_stats* g, LocalDict& L) {
  const uint32_t N = in->n_docs, V = in->n_terms;
  const bool has_name = in->name_off && in->name_tok;
  const uint64_t limit = V / kLocalDiv;
  std::vector<uint64_t> bits(((uint64_t)V + 63) / 64, 0);
  uint64_t n = 0;
  auto mark = [&](const uint32_t* tok, uint64_t b, uint64_t e) {
    for (uint64_t i = b; i < e; ++i) {
      const uint32_t t = tok[i];
      if (t >= V) return false;
      uint64_t& w = bits[t >> 6];
      const uint64_t m = 1ull << (t & 63);
      n += (w & m) == 0;
      w |= m;
    }
    return true;
  };
  for (uint32_t d = 0; d < N && n <= limit; ++d) {
    if (!mark(in->text_tok, in->text_off[d], in->text_off[d + 1])) return fail(FG_EINVAL, "token id >= n_terms");
    if (has_name && !mark(in->name_tok, in->name_off[d], in->name_off[d + 1]))
      return fail(FG_EINVAL, "token id >= n_terms");
  }
  if (n > limit || n == 0) return FG_OK;
  const uint32_t v = (uint32_t)n;
  std::vector<uint32_t> rank(bits.size());
  L.tmap.reserve(v);
  for (size_t w = 0; w < bits.size(); ++w) {
    rank[w] = (uint32_t)L.tmap.size();
    for (uint64_t x = bits[w]; x; x &= x - 1) L.tmap.push_back((uint32_t)(w * 64 + __builtin_ctzll(x)));
  }
  auto local = [&](uint32_t t) {
    return rank[t >> 6] + (uint32_t)__builtin_popcountll(bits[t >> 6] & ((1ull << (t & 63)) - 1));
  };
  const uint64_t nt = in->text_off[N], nn = has_name ? in->name_off[N] : 0;
  L.ttok.resize(nt);
  for (uint64_t i = in->text_off[0]; i < nt; ++i) L.ttok[i] = local(in->text_tok[i]);
  if (has_name) {
    L.ntok.resize(nn);
    for (uint64_t i = in->name_off[0]; i < nn; ++i) L.ntok[i] = local(in->name_tok[i]);
  }
  L.in = *in;
  L.in.n_terms = v;
  L.in.text_tok = L.ttok.data();
  if (has_name) L.in.name_tok = L.ntok.data();
  if (g) {
    L.df_t.resize(v);
    L.df_n.resize(v);
    for (uint32_t l = 0; l < v; ++l) {
      L.df_t[l] = g->df_text[L.tmap[l]];
      L.df_n[l] = g->df_name ? g->df_name[L.tmap[l]] : 0u;
    }
    L.g = *g;
    L.g.df_text = L.df_t.data();
    L.g.df_name = g->df_name ? L.df_n.data() : nullptr;
  }
  return FG_OK;
}
}  // namespace

extern "C" {

static int build_from_docs(fg_ctx* ctx, int dev, const fg_docs_input* in, const fg_global_stats* g, fg_index** out);

int fg_index_build_from_docs_global(fg_ctx* ctx, int dev, const fg_docs_input* in, const fg_global_stats* g,
                                    fg_index** out) {
  if (!ctx || !in || !out || !in->text_off || (!in->text_tok && in->text_off[in->n_docs] > 0))
    return fail(FG_EINVAL, "bad arguments");
  if (g && (!g->df_text || g->n_docs < in->n_docs || g->n_docs >= 0x7FFFFFFFull))
    return fail(FG_EINVAL, "bad global statistics");
  if (in->n_docs == 0) return fail(FG_EINVAL, "empty index (n_docs == 0)");
  if (in->n_docs >= 0x7FFFFFFFu) return fail(FG_EINVAL, "n_docs must be < 2^31 (tantivy DocId)");
  g_bt.start();
  LocalDict L;
  if (int rc = local_dict(in, g, L)) return rc;
  if (L.tmap.empty()) return build_from_docs(ctx, dev, in, g, out);
  g_bt.mark("local dictionary");
  const uint32_t V = in->n_terms;
  fg_index* ix = nullptr;
  if (int rc = build_from_docs(ctx, dev, &L.in, g ? &L.g : nullptr, &ix)) return rc;
  ix->tmap = std::move(L.tmap);
  ix->n_vocab = V;
  *out = ix;
  return FG_OK;
}

static int build_from_docs(fg_ctx* ctx, int dev, const fg_docs_input* in, const fg_global_stats* g, fg_index** out) {
  if (!ctx || !in || !out || !in->text_off || (!in->text_tok && in->text_off[in->n_docs] > 0))
    return fail(FG_EINVAL, "bad arguments");
  if (g && (!g->df_text || g->n_docs < in->n_docs || g->n_docs >= 0x7FFFFFFFull))
    return fail(FG_EINVAL, "bad global statistics");
  if (in->n_docs == 0) return fail(FG_EINVAL, "empty index (n_docs == 0)");
  if (in->n_docs >= 0x7FFFFFFFu) return fail(FG_EINVAL, "n_docs must be < 2^31 (tantivy DocId)");
  if (std::find(ctx->devs.begin(), ctx->devs.end(), dev) == ctx->devs.end())
    return fail(FG_EINVAL, "device %d not in context", dev);
  const uint32_t N = in->n_docs, V = in->n_terms;
  const bool has_name_in = in->name_off && in->name_tok;
  // every thread of pass 1 zeroes and merges three vocabulary-sized count
  // arrays: a small build (a commit's new docs) uses few threads
  const int T = std::max(1, std::min(hw_threads(in->threads), (int)(N / 4096)));
  HostPostings hp;
  hp.n_docs = N;
  hp.n_terms = V;
  hp.fn_text.resize(N);
  hp.fn_name.assign(N, 0);
  // pass 1: per-thread counts (merged df, df_text, df_name), fieldnorms
  std::vector<std::vector<uint32_t>> cnt(T), dft(T), dfn(T);
  std::vector<uint64_t> tot_t(T, 0), tot_n(T, 0);
  std::atomic<bool> bad{false};
  parallel_ranges(N, T, [&](int t, uint32_t b, uint32_t e) {
    cnt[t].assign(V, 0);
    dft[t].assign(V, 0);
    dfn[t].assign(V, 0);
    std::vector<uint32_t> scratch;
    std::vector<std::pair<uint32_t, uint32_t>> rt, rn;
    for (uint32_t d = b; d < e; ++d) {
      uint64_t lt = in->text_off[d + 1] - in->text_off[d];
      uint64_t ln = has_name_in ? in->name_off[d + 1] - in->name_off[d] : 0;
      tot_t[t] += lt;
      tot_n[t] += ln;
      hp.fn_text[d] = fieldnorm_id(lt);
      if (has_name_in) hp.fn_name[d] = fieldnorm_id(ln);
      doc_runs(in->text_tok + in->text_off[d], lt, scratch, rt);
      if (has_name_in) doc_runs(in->name_tok + in->name_off[d], ln, scratch, rn); else rn.clear();
      size_t i = 0, j = 0;
      while (i < rt.size() || j < rn.size()) {
        uint32_t a = i < rt.size() ? rt[i].first : 0xFFFFFFFFu;
        uint32_t c = j < rn.size() ? rn[j].first : 0xFFFFFFFFu;
        uint32_t term = std::min(a, c);
        if (term >= V) { bad = true; return; }
        cnt[t][term]++;
        if (a == term) { dft[t][term]++; ++i; }
        if (c == term) { dfn[t][term]++; ++j; }
      }
    }
  });
  if (bad) return fail(FG_EINVAL, "token id >= n_terms");
  const int used = (int)std::count_if(cnt.begin(), cnt.end(), [](auto& v) { return !v.empty(); });
  hp.off.assign(V + 1, 0);
  hp.df_text.assign(V, 0);
  hp.df_name.assign(V, 0);
  // per-thread write cursors (reuse cnt as u64 cursors via a separate array)
  std::vector<std::vector<uint64_t>> cur(used);
  for (int t = 0; t < used; ++t) cur[t].resize(V);
  uint64_t acc = 0;
  for (uint32_t term = 0; term < V; ++term) {
    hp.off[term] = acc;
    for (int t = 0; t < used; ++t) {
      cur[t][term] = acc;
      acc += cnt[t][term];
      hp.df_text[term] += dft[t][term];
      hp.df_name[term] += dfn[t][term];
    }
  }
  hp.off[V] = acc;
  cnt.clear();
  dft.clear();
  dfn.clear();
  for (int t = 0; t < used; ++t) { hp.tot[0] += tot_t[t]; hp.tot[1] += tot_n[t]; }
  hp.has_name = hp.tot[1] > 0;
  try {
    hp.doc.resize(acc);
    hp.tf.resize(acc);
  } catch (...) {
    return fail(FG_EOOM, "host postings (%llu) allocation failed", (unsigned long long)acc);
  }
  g_bt.mark("pass 1 counts + offsets");
  // pass 2: fill (thread t's docs land after threads < t within each term)
  parallel_ranges(N, T, [&](int t, uint32_t b, uint32_t e) {
    std::vector<uint32_t> scratch;
    std::vector<std::pair<uint32_t, uint32_t>> rt, rn;
    std::vector<uint64_t>& c = cur[t];
    for (uint32_t d = b; d < e; ++d) {
      uint64_t lt = in->text_off[d + 1] - in->text_off[d];
      uint64_t ln = has_name_in ? in->name_off[d + 1] - in->name_off[d] : 0;
      doc_runs(in->text_tok + in->text_off[d], lt, scratch, rt);
      if (has_name_in) doc_runs(in->name_tok + in->name_off[d], ln, scratch, rn); else rn.clear();
      size_t i = 0, j = 0;
      while (i < rt.size() || j < rn.size()) {
        uint32_t a = i < rt.size() ? rt[i].first : 0xFFFFFFFFu;
        uint32_t cc = j < rn.size() ? rn[j].first : 0xFFFFFFFFu;
        uint32_t term = std::min(a, cc);
        uint32_t tt = 0, tn = 0;
        if (a == term) { tt = std::min<uint32_t>(rt[i].second, 0xFFFF); ++i; }
        if (cc == term) { tn = std::min<uint32_t>(rn[j].second, 0xFFFF); ++j; }
        uint64_t p = c[term]++;
        hp.doc[p] = d;
        hp.tf[p] = tt | (tn << 16);
      }
    }
  });
  if (in->deleted) {
    hp.alive.assign((N + 31) / 32, 0);
    for (uint32_t d = 0; d < N; ++d)
      if (!in->deleted[d]) hp.alive[d >> 5] |= 1u << (d & 31);
  }
  if (g)
    for (uint32_t t = 0; t < V; ++t)
      if (g->df_text[t] < hp.df_text[t] || (g->df_name ? g->df_name[t] : 0u) < hp.df_name[t])
        return fail(FG_EINVAL, "global df of term %u is below this shard's", t);
  g_bt.mark("pass 2 fill");
  if (int rc = build_facets(in, hp, T)) return rc;
  g_bt.mark("facets");
  return finish_index(dev, hp, in->keep_host_postings != 0, out, g);
}

int fg_index_build(fg_ctx* ctx, int dev, const fg_index_input* in, fg_index** out) {
  return fg_index_build_global(ctx, dev, in, nullptr, out);
}

int fg_index_build_global(fg_ctx* ctx, int dev, const fg_index_input* in, const fg_global_stats* g, fg_index** out) {
  if (!ctx || !in || !out || !in->term_off || !in->fn_text) return fail(FG_EINVAL, "bad arguments");
  if (g && (!g->df_text || g->n_docs < in->n_docs || g->n_docs >= 0x7FFFFFFFull))
    return fail(FG_EINVAL, "bad global statistics");
  g_bt.start();
  if (in->n_docs == 0 || in->n_docs >= 0x7FFFFFFFu) return fail(FG_EINVAL, "n_docs out of range");
  if (in->term_off[0] != 0) return fail(FG_EINVAL, "term_off[0] must be 0");
  if (in->term_off[in->n_terms] > 0 && (!in->doc || (!in->tf_text && !in->tf_name)))
    return fail(FG_EINVAL, "postings without doc ids or term frequencies");
  if (std::find(ctx->devs.begin(), ctx->devs.end(), dev) == ctx->devs.end())
    return fail(FG_EINVAL, "device %d not in context", dev);
  HostPostings hp;
  const uint32_t N = in->n_docs, V = in->n_terms;
  hp.n_docs = N;
  hp.n_terms = V;
  for (uint32_t t = 0; t < V; ++t)
    if (in->term_off[t + 1] < in->term_off[t]) return fail(FG_EINVAL, "term_off not monotone at %u", t);
  hp.off.assign(in->term_off, in->term_off + V + 1);
  const uint64_t P = hp.off[V];
  hp.doc.assign(in->doc, in->doc + P);
  hp.tf.resize(P);
  hp.df_text.assign(V, 0);
  hp.df_name.assign(V, 0);
  for (uint32_t t = 0; t < V; ++t) {
    for (uint64_t p = hp.off[t]; p < hp.off[t + 1]; ++p) {
      uint32_t tt = in->tf_text ? in->tf_text[p] : 0, tn = in->tf_name ? in->tf_name[p] : 0;
      if (!tt && !tn) return fail(FG_EINVAL, "posting %llu has tf 0 in both fields", (unsigned long long)p);
      if (hp.doc[p] >= N || (p > hp.off[t] && hp.doc[p] <= hp.doc[p - 1]))
        return fail(FG_EINVAL, "postings of term %u not strictly ascending / in range", t);
      hp.tf[p] = tt | (tn << 16);
      hp.df_text[t] += tt ? 1 : 0;
      hp.df_name[t] += tn ? 1 : 0;
    }
  }
  hp.fn_text.assign(in->fn_text, in->fn_text + N);
  if (in->fn_name) hp.fn_name.assign(in->fn_name, in->fn_name + N); else hp.fn_name.assign(N, 0);
  hp.tot[0] = in->tot_tokens[0];
  hp.tot[1] = in->tot_tokens[1];
  hp.has_name = hp.tot[1] > 0;
  if (in->deleted) {
    hp.alive.assign((N + 31) / 32, 0);
    for (uint32_t d = 0; d < N; ++d)
      if (!in->deleted[d]) hp.alive[d >> 5] |= 1u << (d & 31);
  }
  if (in->facet_term_off) {
    const uint32_t VF = in->n_facet_terms;
    hp.n_fterms = VF;
    hp.foff.assign(in->facet_term_off, in->facet_term_off + VF + 1);
    if (hp.foff[0] != 0 || (!in->facet_doc && hp.foff[VF] > 0)) return fail(FG_EINVAL, "bad facet postings");
    hp.fdoc.assign(in->facet_doc, in->facet_doc + hp.foff[VF]);
    hp.df_facet.assign(VF, 0);
    for (uint32_t t = 0; t < VF; ++t) {
      if (hp.foff[t + 1] < hp.foff[t]) return fail(FG_EINVAL, "facet_term_off not monotone at %u", t);
      for (uint64_t p = hp.foff[t]; p < hp.foff[t + 1]; ++p)
        if (hp.fdoc[p] >= N || (p > hp.foff[t] && hp.fdoc[p] <= hp.fdoc[p - 1]))
          return fail(FG_EINVAL, "facet postings of term %u not strictly ascending / in range", t);
      hp.df_facet[t] = (uint32_t)(hp.foff[t + 1] - hp.foff[t]);
    }
    hp.tot_f = in->tot_facet_tokens;
  }
  if (g)
    for (uint32_t t = 0; t < V; ++t)
      if (g->df_text[t] < hp.df_text[t] || (g->df_name ? g->df_name[t] : 0u) < hp.df_name[t])
        return fail(FG_EINVAL, "global df of term %u is below this segment's", t);
  return finish_index(dev, hp, true, out, g);
}

}  // extern "C"

// one snapshot rescored (fg_index_rescore); wts: shared precomputed weights or
// nullptr.  Host only: tantivy scores at query time (src/db/search.rs:162), so
// a new Searcher's statistics need no device work -- the snapshot shares every
// device array of its base (structure and bound tables) and gets the new
// statistics (plans read them), a new alive bitset when docs were deleted, and
// the ratios that scale the build-time bounds (relate_stats).
static int rescore_one(const fg_index* base, const fg_global_stats* g, const uint8_t* deleted, fg_index** out,
                       const fgh::Weights* wts) {
  if (!base || !g || !out || !g->df_text) return fail(FG_EINVAL, "bad arguments");
  const uint32_t N = base->n_docs, V = base->n_terms, VF = base->n_fterms;
  if (g->n_docs < N || g->n_docs >= 0x7FFFFFFFull) return fail(FG_EINVAL, "bad global statistics");
  if (base->has_name && !g->df_name) return fail(FG_EINVAL, "global statistics lack df_name for a snapshot with names");
  if (VF && !g->df_facet) return fail(FG_EINVAL, "global statistics lack df_facet for a faceted snapshot");
  // the statistics' doc frequencies of the snapshot's terms (gathered to local
  // ids when it has its own dictionary: a commit's rescores then cost its terms)
  const uint32_t* gt = g->df_text;
  const uint32_t* gn = g->df_name;
  std::vector<uint32_t> lt, ln;
  if (!base->tmap.empty()) {
    const uint32_t* tm = base->tmap.data();
    lt.resize(V);
    for (uint32_t t = 0; t < V; ++t) lt[t] = g->df_text[tm[t]];
    gt = lt.data();
    if (g->df_name) {
      ln.resize(V);
      for (uint32_t t = 0; t < V; ++t) ln[t] = g->df_name[tm[t]];
      gn = ln.data();
    }
    wts = nullptr;  // (shared weights are vocabulary-indexed)
  }
  {  // (branch-free scans: every older segment of every commit runs them over its terms)
    const uint32_t* bt = base->df_text.data();
    bool bad = false;
    for (uint32_t t = 0; t < V; ++t) bad |= gt[t] < bt[t];
    if (gn) {
      const uint32_t* bn = base->df_name.data();
      for (uint32_t t = 0; t < V; ++t) bad |= gn[t] < bn[t];
    } else if (base->has_name) {
      bad = true;
    }
    for (uint32_t t = 0; t < VF; ++t) bad |= g->df_facet[t] < base->df_facet_local[t];
    if (bad) return fail(FG_EINVAL, "global doc frequencies below this snapshot's own");
  }
  auto ix = std::make_unique<fg_index>();
  ix->dev = base->dev;
  ix->mem.dev = base->dev;
  fgh::device_pools(base->dev, &ix->pool, &ix->pinned);
  // the structure: shared device arrays and host bookkeeping (SharedVec)
  ix->smem = base->smem;
  ix->spool = base->spool;
  ix->struct_bytes = base->struct_bytes;
  ix->n_docs = N;
  ix->n_terms = V;
  ix->n_vocab = base->n_vocab;
  ix->tmap = base->tmap;
  ix->has_name = base->has_name;
  ix->n_postings = base->n_postings;
  ix->dir_entries = base->dir_entries;
  ix->tile_entries = base->tile_entries;
  ix->n_rank = base->n_rank;
  ix->n_srank_words = base->n_srank_words;
  ix->off = base->off;
  ix->df_text = base->df_text;
  ix->df_name = base->df_name;
  ix->first_doc = base->first_doc;
  ix->last_doc = base->last_doc;
  ix->h_doc = base->h_doc;
  ix->tot_local[0] = base->tot_local[0];
  ix->tot_local[1] = base->tot_local[1];
  ix->tmeta = base->tmeta;
  ix->n_fterms = VF;
  ix->tot_f_local = base->tot_f_local;
  ix->foff = base->foff;
  ix->df_facet_local = base->df_facet_local;
  ix->ffirst = base->ffirst;
  ix->flast = base->flast;
  ix->d_sc_tf = base->d_sc_tf;
  ix->d_sc_tl = base->d_sc_tl;
  ix->d_sc_e0 = base->d_sc_e0;
  ix->d_sc_e1 = base->d_sc_e1;
  ix->d_bk_tf = base->d_bk_tf;
  ix->d_bk_tl = base->d_bk_tl;
  ix->d_bk_e0 = base->d_bk_e0;
  ix->d_bk_e1 = base->d_bk_e1;
  ix->d_kt_tiny = base->d_kt_tiny;
  ix->n_ktiny = base->n_ktiny;
  ix->d_tterm = base->d_tterm;
  ix->n_tterm = base->n_tterm;
  ix->n_tiles = base->n_tiles;
  ix->d_kt_terms = base->d_kt_terms;
  ix->d_kb_terms = base->d_kb_terms;
  ix->d_kb_chunk0 = base->d_kb_chunk0;
  ix->d_kc_big = base->d_kc_big;
  ix->d_kc_start = base->d_kc_start;
  ix->n_kbig = base->n_kbig;
  ix->n_kchunks = base->n_kchunks;
  ix->n_sc = base->n_sc;
  ix->n_scb = base->n_scb;
  ix->n_bk = base->n_bk;
  ix->n_kt = base->n_kt;
  ix->d = base->d;
  // the bounds and the build statistics they are under
  ix->sblock = base->sblock;
  ix->ktop = base->ktop;
  ix->tmaxs = base->tmaxs;
  ix->wb_text = base->wb_text;
  ix->wb_name = base->wb_name;
  std::memcpy(ix->cache_b, base->cache_b, sizeof ix->cache_b);
  ix->h_alive_b = base->h_alive_b;
  ix->device_bytes = base->device_bytes;
  set_stats(ix.get(), g->n_docs, g->tot_tokens, gt, gn, g->tot_facet_tokens, VF ? g->df_facet : nullptr, wts);
  relate_stats(ix.get());
  // deletions: the alive bitset (the base's device copy when unchanged), and
  // the docs dead now that ktop's selection counted alive (term_kth)
  std::vector<uint32_t> alive;
  if (deleted) {
    alive.assign((N + 31) / 32, 0);
    for (uint32_t d = 0; d < N; ++d)
      if (!deleted[d]) alive[d >> 5] |= 1u << (d & 31);
  }
  if (alive == base->h_alive.vec()) {
    ix->h_alive = base->h_alive;
    ix->alive_hold = base->alive_hold;
  } else if (alive.empty()) {
    ix->d.alive = nullptr;
  } else {
    HIPCHK(hipSetDevice(ix->dev));
    auto m = std::make_shared<DevAllocs>();
    m->dev = ix->dev;
    uint32_t* d_alive = nullptr;
    uint64_t b = 0;
    if (int rc = dev_upload(*m, alive.data(), alive.size(), &d_alive, &b)) return rc;
    ix->d.alive = d_alive;
    ix->alive_hold = m;
    ix->h_alive = std::move(alive);
  }
  {
    uint64_t dead = 0;
    const auto& now = ix->h_alive.vec();
    const auto& then = ix->h_alive_b.vec();
    for (uint32_t w = 0; w < (N + 31) / 32; ++w) {
      const uint32_t valid = (w + 1) * 32 <= N ? 0xFFFFFFFFu : (1u << (N & 31)) - 1u;
      const uint32_t a0 = then.empty() ? valid : then[w], a1 = now.empty() ? valid : now[w];
      dead += (uint32_t)__builtin_popcount(a0 & ~a1 & valid);
    }
    ix->n_dead = (uint32_t)std::min<uint64_t>(dead, 0xFFFFFFFFu);
  }
  *out = ix.release();
  return FG_OK;
}

extern "C" {

int fg_index_rescore(const fg_index* base, const fg_global_stats* g, const uint8_t* deleted, fg_index** out) {
  g_bt.start();
  return rescore_one(base, g, deleted, out, nullptr);
}

int fg_index_rescore_many(const fg_index* const* bases, uint32_t n, const fg_global_stats* g,
                          const uint8_t* const* deleted, fg_index** outs) {
  if ((n && (!bases || !outs)) || !g || !g->df_text) return fail(FG_EINVAL, "bad arguments");
  uint32_t V = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (!bases[i]) return fail(FG_EINVAL, "NULL snapshot %u", i);
    if (bases[i]->tmap.empty()) V = std::max(V, bases[i]->n_terms);
    outs[i] = nullptr;
  }
  if (n == 0) return FG_OK;
  // the weights once for every snapshot on vocabulary ids (they depend on the
  // statistics only; a snapshot with its own dictionary gathers its own)
  fgh::Weights wts;
  g_bt.start();
  if (V) {
    std::vector<float> wt, wn;
    bm25_weights(g->n_docs, g->df_text, g->df_name, V, wt, wn);
    wts.wt = std::move(wt);
    wts.wn = std::move(wn);
  }
  g_bt.mark("rescore: shared weights");
  for (uint32_t i = 0; i < n; ++i) {
    const int rc = rescore_one(bases[i], g, deleted ? deleted[i] : nullptr, &outs[i], &wts);
    g_bt.mark(bases[i]->tmap.empty() ? "rescore: a snapshot" : "rescore: a snapshot (own dictionary)");
    if (rc) {
      const std::string e = fg_last_error();
      for (uint32_t j2 = 0; j2 < n; ++j2)
        if (outs[j2]) {
          fg_index_release(outs[j2]);
          outs[j2] = nullptr;
        }
      return fail(rc, "snapshot %u: %s", i, e.c_str());
    }
  }
  return FG_OK;
}

int fg_thread_background(int on) {
  const int prev = tl_background;
  tl_background = on ? 1 : 0;
  return prev;
}

int fg_index_retain(fg_index* ix) {
  if (!ix) return fail(FG_EINVAL, "NULL index");
  ix->refs.fetch_add(1);
  return FG_OK;
}

int fg_index_release(fg_index* ix) {
  if (!ix) return FG_OK;
  if (ix->refs.fetch_sub(1) == 1) delete ix;
  return FG_OK;
}

int fg_index_stats_get(const fg_index* ix, fg_index_stats* o) {
  if (!ix || !o) return fail(FG_EINVAL, "bad arguments");
  o->n_docs = ix->n_docs;
  o->n_terms = ix->n_vocab;
  o->n_postings = ix->n_postings;
  o->device_bytes = ix->device_bytes;
  o->tot_tokens[0] = ix->tot[0];
  o->tot_tokens[1] = ix->tot[1];
  o->avgdl[0] = ix->avgdl[0];
  o->avgdl[1] = ix->avgdl[1];
  o->has_name = ix->has_name;
  o->device = ix->dev;
  o->n_facet_terms = ix->n_fterms;
  o->tot_facet_tokens = ix->tot_f;
  o->n_dense_f32 = ix->n_dense;
  o->n_rank_terms = ix->n_rank;
  o->n_sparse_rank_terms = ix->n_rank - ix->d.n_prank;
  o->reserved0 = 0;
  o->rank_bytes = 8ull * ix->d.n_prank * ix->d.rank_words +
                  8ull * (ix->n_rank - ix->d.n_prank) * ix->d.srank_blocks + 8ull * ix->n_srank_words;
  return FG_OK;
}

uint64_t fg_index_df(const fg_index* ix, int field, uint32_t term) {
  if (ix && field == FG_FIELD_FACET) return term < ix->n_fterms ? ix->df_facet[term] : 0;
  if (!ix) return 0;
  term = fgh::local_term(ix, term);
  if (term >= ix->n_terms) return 0;
  if (field == FG_FIELD_TEXT) return ix->df_text[term];
  if (field == FG_FIELD_NAME) return ix->df_name[term];
  return ix->off[term + 1] - ix->off[term];
}

int fg_index_term_kth(const fg_index* ix, uint32_t term, float* out) {
  if (!ix || !out) return fail(FG_EINVAL, "bad arguments");
  static_assert(fg::kNumTopK == 5, "fugu.h documents five K");
  term = fgh::local_term(ix, term);
  for (uint32_t k = 0; k < fg::kNumTopK; ++k) out[k] = fgh::term_kth_now(ix, term, fg::kTopKs[k], false);
  return FG_OK;
}

int fg_index_term_ladder(const fg_index* ix, float* out) {
  if (!ix || !out) return fail(FG_EINVAL, "bad arguments");
  static_assert(fg::kNumLadder == FG_LADDER_LEVELS, "fugu.h FG_LADDER_LEVELS");
  const uint32_t V = ix->n_terms;
  if (V == 0) return FG_OK;
  HIPCHK(hipSetDevice(ix->dev));
  // one temporary: the main K-th scores [V * kNumTopK], then the extra levels
  const size_t nm = (size_t)V * fg::kNumTopK, nx = (size_t)V * fg::kNumLadderExtra;
  void* tmp = nullptr;
  if (fgh::dev_malloc_async(&tmp, 4 * (nm + nx) + 16, kBuildStream) != hipSuccess)
    return fail(FG_EOOM, "hipMallocAsync(%zu) failed", 4 * (nm + nx));
  struct Back {
    void* p;
    ~Back() { (void)hipFreeAsync(p, kBuildStream); }
  } back{tmp};
  float* d = static_cast<float*>(tmp);
  HIPCHK(hipMemsetAsync(d, 0, 4 * (nm + nx), kBuildStream));
  // the posting scores under the snapshot's statistics (a temporary), then k_ktop with the extra levels
  fg::ScoreJob j{};
  void* ptmp = nullptr;
  if (int rc = score_postings(ix, j, nullptr, nullptr, &ptmp)) return rc;
  struct PBack {
    void* p;
    ~PBack() { (void)hipFreeAsync(p, kBuildStream); }
  } pback{ptmp};
  j.alive = ix->d.alive;
  j.ktop = d;
  j.ladder = d + nm;
  if (int rc = ktop_pass(ix, j)) return rc;
  std::vector<float> h(nm + nx);
  HIPCHK(hipMemcpyAsync(h.data(), d, 4 * (nm + nx), hipMemcpyDeviceToHost, kBuildStream));
  HIPCHK(hipStreamSynchronize(kBuildStream));
  // interleave into ascending K per term
  uint32_t src[fg::kNumLadder];  // level l: (main?, index)
  for (uint32_t l = 0; l < fg::kNumLadder; ++l) {
    src[l] = 0xFFFFFFFFu;
    for (uint32_t i = 0; i < fg::kNumTopK; ++i)
      if (fg::kTopKs[i] == fg::kLadderKs[l]) src[l] = i;
    for (uint32_t i = 0; i < fg::kNumLadderExtra; ++i)
      if (fg::kLadderExtra[i] == fg::kLadderKs[l]) src[l] = 0x10000u | i;
    if (src[l] == 0xFFFFFFFFu) return fail(FG_EINVAL, "ladder level %u unmapped", l);
  }
  // (vocabulary ids: a snapshot with its own dictionary scatters its terms, zeros elsewhere)
  const uint32_t* tm = ix->tmap.empty() ? nullptr : ix->tmap.data();
  if (tm) std::fill(out, out + (size_t)ix->n_vocab * fg::kNumLadder, 0.0f);
  for (uint32_t t = 0; t < V; ++t)
    for (uint32_t l = 0; l < fg::kNumLadder; ++l) {
      const uint32_t s = src[l];
      out[(size_t)(tm ? tm[t] : t) * fg::kNumLadder + l] = (s & 0x10000u) ? h[nm + (size_t)t * fg::kNumLadderExtra + (s & 0xFFFFu)]
                                                            : h[(size_t)t * fg::kNumTopK + s];
    }
  return FG_OK;
}

int fg_kth_floor_combine(uint32_t n_shards, uint32_t n_terms, const float* const* ladders, float* out) {
  if (!out || (n_shards && !ladders) || (n_terms && n_shards == 0)) return fail(FG_EINVAL, "bad arguments");
  for (uint32_t s = 0; s < n_shards; ++s)
    if (!ladders[s]) return fail(FG_EINVAL, "NULL ladder of shard %u", s);
  constexpr uint32_t L = fg::kNumLadder;
  fgh::parallel_dynamic(n_terms, fgh::hw_threads(0), 8192, [&](int, uint32_t b, uint32_t e) {
    std::vector<std::pair<float, uint32_t>> c;  // (score, shard * L + level)
    std::vector<uint32_t> cur(n_shards);        // the largest K of each shard at or above the sweep
    for (uint32_t t = b; t < e; ++t) {
      c.clear();
      for (uint32_t s = 0; s < n_shards; ++s)
        for (uint32_t l = 0; l < L; ++l) {
          const float v = ladders[s][(size_t)t * L + l];
          if (v > 0.0f) c.emplace_back(v, s * L + l);
        }
      std::sort(c.begin(), c.end(), [](const auto& x, const auto& y) { return x.first > y.first; });
      std::fill(cur.begin(), cur.end(), 0u);
      uint64_t total = 0;  // docs known to score >= the sweep's score
      float res[fg::kNumTopK] = {0, 0, 0, 0, 0};
      uint32_t next = 0;
      for (size_t i = 0; i < c.size() && next < fg::kNumTopK;) {
        const float x = c[i].first;
        for (; i < c.size() && c[i].first == x; ++i) {  // every level scoring exactly x counts at x
          const uint32_t s = c[i].second / L, K = fg::kLadderKs[c[i].second % L];
          if (K > cur[s]) {
            total += K - cur[s];
            cur[s] = K;
          }
        }
        for (; next < fg::kNumTopK && total >= fg::kTopKs[next]; ++next) res[next] = x;
      }
      for (uint32_t k = 0; k < fg::kNumTopK; ++k) out[(size_t)t * fg::kNumTopK + k] = res[k];
    }
  });
  return FG_OK;
}

int fg_index_set_kth_floor(fg_index* ix, const float* floor, uint32_t n_terms) {
  if (!ix) return fail(FG_EINVAL, "NULL index");
  std::shared_ptr<const std::vector<float>> f;
  if (floor) {
    if (n_terms != ix->n_vocab) return fail(FG_EINVAL, "floor of %u terms for a snapshot of %u", n_terms, ix->n_vocab);
    if (ix->tmap.empty()) {
      f = std::make_shared<const std::vector<float>>(floor, floor + (size_t)n_terms * fg::kNumTopK);
    } else {  // gathered to local ids
      std::vector<float> v((size_t)ix->n_terms * fg::kNumTopK);
      for (uint32_t t = 0; t < ix->n_terms; ++t)
        std::copy(floor + (size_t)ix->tmap[t] * fg::kNumTopK, floor + (size_t)(ix->tmap[t] + 1) * fg::kNumTopK,
                  v.begin() + (size_t)t * fg::kNumTopK);
      f = std::make_shared<const std::vector<float>>(std::move(v));
    }
  }
  std::atomic_store(&ix->kth_floor, f);
  return FG_OK;
}

int fg_index_bm25(const fg_index* ix, uint32_t term, float* w_text, float* w_name, float* cache512) {
  if (!ix) return fail(FG_EINVAL, "NULL index");
  term = fgh::local_term(ix, term);
  if (term < ix->n_terms) {
    if (w_text) *w_text = ix->w_text[term];
    if (w_name) *w_name = ix->w_name[term];
  } else {
    if (w_text) *w_text = bm25_weight(0, ix->n_stats);
    if (w_name) *w_name = bm25_weight(0, ix->n_stats);
  }
  if (cache512) std::memcpy(cache512, ix->cache, sizeof ix->cache);
  return FG_OK;
}

// ---------------------------------------------------------------- planning
static int plan_create(fg_index* ix, const fg_query_batch* q, uint32_t k, fg_plan** out, bool sync,
                       hipStream_t up = hipStreamPerThread);
static int plan_create_multi(fg_index* const* ixs, uint32_t n_segs, const fg_query_batch* q, uint32_t k,
                             fg_plan** out, bool sync, hipStream_t up);

int fg_plan_create(fg_index* ix, const fg_query_batch* q, uint32_t k, fg_plan** out) {
  return plan_create(ix, q, k, out, true);
}

int fg_plan_create_multi(fg_index* const* ixs, uint32_t n_segs, const fg_query_batch* q, uint32_t k, fg_plan** out) {
  return plan_create_multi(ixs, n_segs, q, k, out, true, hipStreamPerThread);
}

// sync = false (fg_search_batch): the upload stays in flight on the calling
// thread's per-thread stream, where the plan's execute is queued behind it;
// the pinned staging is returned when the plan is destroyed
static int plan_create(fg_index* ix, const fg_query_batch* q, uint32_t k, fg_plan** out, bool sync,
                       hipStream_t up) {
  return plan_create_multi(&ix, 1, q, k, out, sync, up);
}

namespace {

struct WItem { double key; uint32_t q, c, n; };

// One snapshot's side of a planned batch, built on the host alone (no HIP
// call): per-query tables, facet filters (ids local to the snapshot) and the
// unsorted work items.  plan_create_multi joins one per snapshot.
struct HostPlan {
  std::vector<uint32_t> q_m, q_terms, lead, nchunk, q_filter;
  std::vector<uint64_t> thr0;
  std::vector<float> q_ub, q_wt, q_wn, q_rup;
  uint32_t nf = 0;
  std::vector<uint32_t> f_shift;
  std::vector<uint64_t> f_woff;
  std::vector<float> f_tab, f_max;
  std::vector<uint32_t> ch_f, ch_c, ch_t, ch_s;
  std::vector<WItem> citems, ditems, scan;
  std::vector<uint32_t> ngroup, q_hlo, q_hhi, q_hsh;
  // (a thread's plans reuse one set: assign / push_back into kept capacity, no
  // page faults on fresh arrays -- ~0.2 ms of an 8-snapshot batch's planning)
  void clear_lists() {
    ch_f.clear(); ch_c.clear(); ch_t.clear(); ch_s.clear();
    citems.clear(); ditems.clear(); scan.clear();
  }
};

// n_segs: the snapshots the plan spans; a query's work items are spread over
// all of them, so each snapshot gets its share of the per-query item counts.
// nq_size: the batch size the item counts are sized for (q may be a slice of
// that batch: plan_create_multi plans a snapshot's queries in pieces)
int plan_host(const fg_index* ix, const fg_query_batch* q, uint32_t k, uint32_t n_segs, HostPlan& h,
              uint32_t nq_size) {
  if (!ix || !q || (q->n_queries && !q->q_off)) return fail(FG_EINVAL, "bad arguments");
  if (q->n_queries && q->q_off[q->n_queries] > q->q_off[0] && !q->terms) return fail(FG_EINVAL, "q_off without terms");
  if (q->f_off && q->n_queries && q->f_off[q->n_queries] > q->f_off[0] && !q->f_terms)
    return fail(FG_EINVAL, "f_off without f_terms");
  if (k < 1) return fail(FG_EINVAL, "k must be >= 1 (TopDocs::with_limit asserts limit >= 1)");
  if (k > FG_MAX_K) return fail(FG_EUNSUPPORTED, "k=%u > FG_MAX_K=%d", k, FG_MAX_K);
  if (q->mode != FG_MODE_AND && q->mode != FG_MODE_OR) return fail(FG_EINVAL, "bad mode %d", q->mode);
  const uint32_t nq = q->n_queries;
  const uint64_t N = ix->n_docs;
  const bool disj = q->mode == FG_MODE_OR;
  h.clear_lists();
  auto &q_m = h.q_m, &q_terms = h.q_terms, &lead = h.lead, &nchunk = h.nchunk;
  auto& thr0 = h.thr0;
  auto& q_ub = h.q_ub;
  q_m.assign(nq, 0);
  q_terms.assign((size_t)nq * fg::kMaxTerms, 0);
  lead.assign(nq, 0);
  nchunk.assign(nq, 0);
  thr0.assign(nq, 0);
  q_ub.assign((size_t)nq * fg::kMaxTerms, 0.0f);
  h.q_wt.assign((size_t)nq * fg::kMaxTerms, 0.0f);
  h.q_wn.assign((size_t)nq * fg::kMaxTerms, 0.0f);
  h.q_rup.assign((size_t)nq * fg::kMaxTerms, 1.0f);

  // ---- facet filters: one mask per distinct clause list (fg_internal.h DevFilters)
  auto& q_filter = h.q_filter;
  q_filter.assign(nq, 0xFFFFFFFFu);
  std::vector<std::vector<uint32_t>> flist;
  std::vector<uint8_t> q_nomatch(nq, 0);  // the filter matches no doc: no work items
  if (q->f_off) {
    std::map<std::vector<uint32_t>, uint32_t> fid;
    for (uint32_t i = 0; i < nq; ++i) {
      const uint32_t b = q->f_off[i], e = q->f_off[i + 1];
      if (e < b) return fail(FG_EINVAL, "f_off not monotone at query %u", i);
      if (e == b) continue;
      if (e - b > fg::kMaxFacetClauses)
        return fail(FG_EUNSUPPORTED, "query %u has %u facet clauses (> %u)", i, e - b, fg::kMaxFacetClauses);
      std::vector<uint32_t> c(q->f_terms + b, q->f_terms + e);
      bool any = false;
      for (uint32_t t : c) any |= t < ix->n_fterms && ix->df_facet[t] > 0;
      if (!any) { q_nomatch[i] = 1; continue; }
      auto it = fid.find(c);
      if (it == fid.end()) {
        it = fid.emplace(c, (uint32_t)flist.size()).first;
        flist.push_back(std::move(c));
      }
      q_filter[i] = it->second;
    }
  }
  const uint32_t nf = h.nf = (uint32_t)flist.size();
  auto& f_shift = h.f_shift;
  auto& f_woff = h.f_woff;
  auto& f_tab = h.f_tab;
  auto& f_max = h.f_max;
  auto &ch_f = h.ch_f, &ch_c = h.ch_c, &ch_t = h.ch_t, &ch_s = h.ch_s;
  f_shift.assign(nf, 0);
  f_woff.assign(nf + 1, 0);
  f_tab.assign((size_t)nf * 256, 0.0f);
  f_max.assign(nf, 0.0f);
  std::vector<uint32_t> f_lo(nf, 0xFFFFFFFFu), f_hi(nf, 0);  // doc span of the filter's postings
  for (uint32_t f = 0; f < nf; ++f) {
    const std::vector<uint32_t>& c = flist[f];
    const uint32_t n = (uint32_t)c.size();
    const uint32_t sh = n <= 1 ? 0 : n <= 2 ? 1 : n <= 4 ? 2 : 3;
    if ((N << sh) > (1ull << 32)) return fail(FG_EUNSUPPORTED, "facet mask of %u clauses too large for %llu docs", n,
                                              (unsigned long long)N);
    f_shift[f] = sh;
    f_woff[f + 1] = f_woff[f] + ((((N << sh) + 31) / 32 + 63) & ~63ull);  // 256-B aligned masks
    // union score of each set of matching clauses: 0.0 + s_i in clause order (SumCombiner)
    for (uint32_t v = 0; v < (1u << n); ++v) {
      float sc = 0.0f;
      for (uint32_t i = 0; i < n; ++i)
        if ((v >> i) & 1u) sc += c[i] < ix->n_fterms ? ix->fscore[c[i]] : 0.0f;
      f_tab[(size_t)f * 256 + v] = sc;
      f_max[f] = std::max(f_max[f], sc);
    }
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t t = c[i];
      if (t >= ix->n_fterms || ix->df_facet[t] == 0) continue;
      f_lo[f] = std::min(f_lo[f], ix->ffirst[t]);
      f_hi[f] = std::max(f_hi[f], ix->flast[t]);
      const uint64_t df = ix->foff[t + 1] - ix->foff[t];
      for (uint64_t st = 0; st < df; st += fg::kFmaskChunk) {
        ch_f.push_back(f);
        ch_c.push_back(i);
        ch_t.push_back(t);
        ch_s.push_back((uint32_t)st);
      }
    }
  }

  // work items: each query's chunks (Must-driven: k_conj) or doc tiles (Should
  // only: k_disj) in ~kGroupsPerQuery groups, ordered as a doc sweep across the
  // batch (a group centred at doc fraction x runs with the other queries'
  // groups near x), ties by query.  Queries without text terms (facet-only /
  // AllQuery) scan doc tiles (k_scan).  Per-term occurs (q->occur) make a
  // query Must-driven when it has a Must clause (RequiredOptionalScorer over
  // its Shoulds), a union of its Shoulds otherwise; MustNot clauses exclude.
  using W = WItem;
  // k_disj / k_scan groups per query, spread over the plan's snapshots; a small
  // batch (the batch-of-one latency: the GPU holds nothing else) splits each
  // query over up to 16x more, shorter items that run side by side
  const uint32_t gpq_batch =
      fg::kGroupsPerQuery * std::min<uint32_t>(fg::kDisjSmallSpread, std::max<uint32_t>(1, 256 / std::max(nq_size, 1u)));
  const uint32_t gpq = std::max<uint32_t>(1, gpq_batch / n_segs);
  // k_conj items per query per snapshot of a multi-snapshot plan: the single-
  // snapshot count / n_segs, so a query keeps ~the single-snapshot item count
  // over all its slots (C4, 8 x 1.25M namespaces: k_conj 1.300 -> 1.085 ms, /16
  // 1.065 ms, identical hits: profiles/r05/ab/c4_ab_r05q.json; round 4 measured
  // the opposite before the sparse rank words and the XCD split);
  const uint32_t conj_gpq = fg::kConjGroupsPerQuery, conj_maxg = fg::kMaxGroup;
  const uint32_t cdiv = n_segs <= 1 ? 1u : n_segs;
  auto &citems = h.citems, &ditems = h.ditems, &scan = h.scan;
  auto &ngroup = h.ngroup, &q_hlo = h.q_hlo, &q_hhi = h.q_hhi, &q_hsh = h.q_hsh;
  ngroup.assign(nq, 0);
  q_hlo.assign(nq, 0x3F800000u);
  q_hhi.assign(nq, 0x3F800000u);
  q_hsh.assign(nq, 31);
  auto present = [&](uint32_t t) { return t < ix->n_terms && ix->off[t + 1] > ix->off[t]; };
  // a clause's query-time weights and bound factor (DevPlan::q_wt / q_wn / q_rup),
  // and its largest current score into cm[j] (the ratio computed once per clause)
  float cm[fg::kMaxTerms];
  auto set_clause = [&](uint32_t i, uint32_t j, uint32_t t) {
    const size_t x = (size_t)i * fg::kMaxTerms + j;
    h.q_wt[x] = ix->w_text[t];
    h.q_wn[x] = ix->w_name[t];
    float rdn, rup;
    fgh::term_ratio(ix, t, &rdn, &rup);
    h.q_rup[x] = rup;
    cm[j] = fgh::term_max_scaled(ix, t, rup);
  };
  // histogram bins of query i: bin 0 at the starting threshold (or ub / 256), the
  // top bin at the query's largest possible score ub; ~kQBins bins between
  auto set_bins = [&](uint32_t i, float ub) {
    const float lo = thr0[i] ? fg::key_score(thr0[i]) : ub / 256.0f;
    uint32_t lb, hb;
    std::memcpy(&lb, &lo, 4);
    std::memcpy(&hb, &ub, 4);
    lb = std::max<uint32_t>(lb, 1);
    hb = std::max(hb, lb);
    q_hlo[i] = lb;
    q_hhi[i] = hb;
    q_hsh[i] = bin_shift(lb, hb);
  };
  for (uint32_t i = 0; i < nq; ++i) {
    const uint32_t b = q->q_off[i], e = q->q_off[i + 1];
    if (e < b) return fail(FG_EINVAL, "q_off not monotone at query %u", i);
    const uint32_t m = e - b;
    if (m > fg::kMaxTerms) return fail(FG_EUNSUPPORTED, "query %u has %u terms (> %u)", i, m, fg::kMaxTerms);
    if (q_nomatch[i]) continue;  // the facet clauses match nothing: no hits
    const float fmx = q_filter[i] == 0xFFFFFFFFu ? 0.0f : f_max[q_filter[i]];
    if (m == 0) {
      // empty text query: the facet union alone, or AllQuery (src/db/search.rs:115-116, 131-137)
      q_m[i] = 0;
      const uint32_t f = q_filter[i];
      const uint64_t dlo = f == 0xFFFFFFFFu ? 0 : f_lo[f], dhi = f == 0xFFFFFFFFu ? N - 1 : f_hi[f];
      const uint32_t tlo = (uint32_t)(dlo >> fg::kDisjTileShift), thi = (uint32_t)(dhi >> fg::kDisjTileShift);
      const uint32_t nt = thi - tlo + 1;
      const uint32_t G = std::min<uint32_t>(fg::kScanMaxGroup,
                                            std::max<uint32_t>(1, (nt + gpq - 1) / gpq));
      const uint32_t ng = (nt + G - 1) / G;
      ngroup[i] = ng;
      // the groups of all queries in doc order: the first groups publish the
      // thresholds that let the later ones stop early
      for (uint32_t g = 0; g < ng; ++g) scan.push_back(W{(double)g, i, tlo + g * G, std::min(G, nt - g * G)});
      continue;
    }
    // the query's clauses by occur; a Should or MustNot clause on a term the
    // snapshot lacks matches nothing and is dropped; a missing Must empties it
    uint32_t tm[fg::kMaxTerms], ts_[fg::kMaxTerms], tx[fg::kMaxTerms];
    uint32_t nm = 0, ns = 0, nx = 0;
    bool must_missing = false;
    for (uint32_t j = 0; j < m; ++j) {
      const uint32_t t = fgh::local_term(ix, q->terms[b + j]);  // (the snapshot's own ids from here on)
      const uint8_t oc = q->occur ? q->occur[b + j] : (disj ? FG_OCCUR_SHOULD : FG_OCCUR_MUST);
      if (oc > FG_OCCUR_MUST_NOT) return fail(FG_EINVAL, "query %u: bad occur %u", i, (unsigned)oc);
      if (oc == FG_OCCUR_MUST) {
        tm[nm++] = t;
        must_missing |= !present(t);
      } else if (present(t)) {
        (oc == FG_OCCUR_SHOULD ? ts_[ns++] : tx[nx++]) = t;
      }
    }
    // one positive clause: the union of one Should IS that clause, so it runs
    // Must-driven (k_conj's single-list and exclusion paths); same docs, same score
    if (nm == 0 && ns == 1) {
      tm[nm++] = ts_[0];
      ns = 0;
    }
    uint32_t* qt = q_terms.data() + (size_t)i * fg::kMaxTerms;
    if (nm == 0) {
      if (ns == 0) continue;  // no positive clause: EmptyScorer, no hits
      // Should clauses in clause order (SumCombiner order), then the MustNots
      uint32_t dlo = 0xFFFFFFFFu, dhi = 0;
      for (uint32_t j = 0; j < ns; ++j) {
        qt[j] = ts_[j];
        dlo = std::min(dlo, ix->first_doc[ts_[j]]);
        dhi = std::max(dhi, ix->last_doc[ts_[j]]);
      }
      for (uint32_t j = 0; j < nx; ++j) qt[ns + j] = tx[j];
      for (uint32_t j = 0; j < ns + nx; ++j) set_clause(i, j, qt[j]);
      q_m[i] = fg::qm_pack(ns + nx, 0, nx);
      if (q_filter[i] != 0xFFFFFFFFu) {
        dlo = std::max(dlo, f_lo[q_filter[i]]);
        dhi = std::min(dhi, f_hi[q_filter[i]]);
        if (dlo > dhi) continue;  // the text and facet doc spans do not meet
      }
      // starting threshold: the best per-clause K'-th score for the smallest stored
      // K' >= k (unfiltered and unexcluded only: a filter or an exclusion may
      // remove a term's best docs)
      if (q_filter[i] == 0xFFFFFFFFu && nx == 0) {
        float v = 0.0f;
        for (uint32_t c = 0; c < ns; ++c) v = std::max(v, fgh::term_kth_now(ix, qt[c], k, true));
        if (v > 0.0f) thr0[i] = fg::make_key(v, 0xFFFFFFFFu);  // lowest key with score v
      }
      float ub = fmx;
      for (uint32_t c = 0; c < ns; ++c) ub += cm[c];
      set_bins(i, ub);

      const uint32_t tlo = dlo >> fg::kDisjTileShift, thi = dhi >> fg::kDisjTileShift;
      const uint32_t nt = thi - tlo + 1;
      // tiles per item: ~gpq items per query (capping an item's postings, or the
      // items of heavy queries first, measured slower: ab_disj_itemcap_k*.log,
      // ab_disj_heavy_k*.log)
      const uint32_t G = std::min<uint32_t>(std::min(fg::kDisjMaxGroup, fg::kDisjMaxPairs / ns),
                                            std::max<uint32_t>(1, (nt + gpq - 1) / gpq));
      // (shorter first items -- G >> r, G >> (r-1), ... tiles -- so the items that
      // start with no threshold publish one early: r = 2 / 3 / 5 / 8 slower at
      // k = 1000 and 20, +0.4% to +7%: profiles/r05/ab/disj_ramp_r05t.log)
      // (shorter items at the end of each query's range -- half-size in its last
      // 1/8, 1/4, 1/2 -- measured +8.6 / +18 / +34% at top-20, +9 / +18 / +33% at
      // top-1000; 64-tile items -0.5% / +1.8%: profiles/r06/ab/)
      const uint32_t ng = (nt + G - 1) / G;
      for (uint32_t g = 0; g < ng; ++g) {
        const uint32_t t0 = tlo + g * G, n = std::min(G, nt - g * G);
        const double mid = ((double)t0 + 0.5 * n) * (double)(1u << fg::kDisjTileShift) / (double)ix->n_docs;
        ditems.push_back(W{mid, i, t0, n});
      }
      ngroup[i] = ng;
      if (ditems.size() > 0x7FFFFFFFull) return fail(FG_EUNSUPPORTED, "batch too large (%zu work items)", ditems.size());
      continue;
    }
    if (must_missing) continue;  // a Must clause matches nothing: no hits
    // tantivy intersect_scorers: the Must children sorted by cost (union cost =
    // df_text + df_name), stable; then the MustNots, then the Shoulds in clause order
    struct T { uint64_t cost; uint32_t pos, term; };
    T tc[fg::kMaxTerms];
    for (uint32_t j = 0; j < nm; ++j) tc[j] = T{(uint64_t)ix->df_text[tm[j]] + ix->df_name[tm[j]], j, tm[j]};
    std::stable_sort(tc, tc + nm, [](const T& x, const T& y) { return x.cost < y.cost; });
    for (uint32_t j = 0; j < nm; ++j) qt[j] = tc[j].term;
    for (uint32_t j = 0; j < nx; ++j) qt[nm + j] = tx[j];
    for (uint32_t j = 0; j < ns; ++j) qt[nm + nx + j] = ts_[j];
    const uint32_t mt = nm + nx + ns;
    for (uint32_t j = 0; j < mt; ++j) set_clause(i, j, qt[j]);
    q_m[i] = fg::qm_pack(mt, nm, nx);
    // MaxScore suffix bounds of the probed lists (k_conj prunes a candidate once its
    // partial score plus these cannot reach the query's threshold): the Must and
    // Should maxima from position j on (MustNots add nothing)
    {
      float acc = 0.0f;
      for (uint32_t j = mt; j-- > 1;) {
        if (j < nm || j >= nm + nx) acc += cm[j];
        q_ub[(size_t)i * fg::kMaxTerms + j] = acc;
      }
    }
    // one list: its K'-th best alive score (the smallest stored K' >= k) bounds
    // the query's k-th best from below, so k_conj starts from that threshold and
    // skips the lead chunks whose block-max cannot reach it (the block-max
    // pruning tantivy's TopDocs runs on a single TermScorer: block_wand_single_scorer)
    if (mt == 1 && q_filter[i] == 0xFFFFFFFFu) {
      const float v = fgh::term_kth_now(ix, qt[0], k, true);
      if (v > 0.0f) thr0[i] = fg::make_key(v, 0xFFFFFFFFu);  // lowest key with score v
    }
    {
      float ub = fmx + cm[0];
      for (uint32_t j = 1; j < mt; ++j)
        if (j < nm || j >= nm + nx) ub += cm[j];
      set_bins(i, ub);
    }
    const uint64_t df0 = ix->off[qt[0] + 1] - ix->off[qt[0]];
    lead[i] = (uint32_t)df0;
    nchunk[i] = (uint32_t)((df0 + fg::kChunk - 1) / fg::kChunk);
    if (citems.size() + nchunk[i] > 0x7FFFFFFFull)
      return fail(FG_EUNSUPPORTED, "batch too large (%zu work items)", citems.size());
    const uint32_t nch = nchunk[i];
    // items per query: ~kConjGroupsPerQuery in a full batch; a small batch (a
    // batch of one: the p50 latency) spreads a query over up to 64 items so its
    // chunks run side by side instead of up to kMaxGroup in a row, while its
    // k_final still reads at most 64 x k candidates
    // (a multi-snapshot plan: divided by cdiv, above)
    const uint32_t per_q =
        std::max<uint32_t>(1, std::min<uint32_t>(64, std::max<uint32_t>(conj_gpq, 1024 / std::max(nq_size, 1u))) / cdiv);
    const uint32_t G = std::min<uint32_t>(conj_maxg, std::max<uint32_t>(1, (nch + per_q - 1) / per_q));
    const uint32_t ng = (nch + G - 1) / G;
    ngroup[i] = ng;
    for (uint32_t g = 0; g < ng; ++g)
      citems.push_back(W{(g + 0.5) / ng, i, g * G, std::min(G, nch - g * G)});
  }
  return FG_OK;
}

}  // namespace

// Plans of one batch on one or several snapshots of one device (a multi-
// snapshot plan: DevPlan::segs, query slot v = s * nq + q): every snapshot is
// planned on the host (in parallel for a large batch), then the slots are
// joined into ONE set of work items, uploaded once and run by one launch per
// kernel.  Several snapshots share each batch query's threshold and histogram
// (score-only), and their bins span the union of the snapshots' score ranges.
static void run_parallel(uint32_t n, const std::function<void(uint32_t)>& f);  // ShardWorkers, below

static int plan_create_multi(fg_index* const* ixs, uint32_t S, const fg_query_batch* q, uint32_t k,
                             fg_plan** out, bool sync, hipStream_t up) {
  if (!ixs || !q || !out || S == 0 || S > FG_MAX_SEGMENTS) return fail(FG_EINVAL, "bad arguments");
  for (uint32_t s = 0; s < S; ++s) {
    if (!ixs[s]) return fail(FG_EINVAL, "NULL snapshot");
    if (ixs[s]->dev != ixs[0]->dev) return fail(FG_EINVAL, "the snapshots of one plan live on different devices");
  }
  fg_index* ix = ixs[0];
  // FUGU_SHARD_TRACE: the planning phases of a multi-snapshot batch on stderr
  static const bool ptrace = getenv("FUGU_SHARD_TRACE") != nullptr;
  auto pnow = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  double pt[5] = {ptrace ? pnow() : 0.0, 0, 0, 0, 0};
  // (reused: HostPlan::clear_lists; a plain reference, so the planning workers'
  // lambdas see THIS thread's copy, not their own thread_local one)
  static thread_local std::vector<HostPlan> hs_tl;
  std::vector<HostPlan>& hs = hs_tl;
  const uint32_t nq1 = q->n_queries;  // batch queries
  if ((uint64_t)S * nq1 > 0x7FFFFFFFull) return fail(FG_EUNSUPPORTED, "batch too large (%u x %u query slots)", S, nq1);
  const uint32_t nq = S * nq1;  // query slots
  // pieces: each snapshot's queries planned in P slices of >= 128 queries so
  // the host's threads all plan (8 snapshots on 16 threads: 2 pieces each);
  // piece p = s * P + r holds snapshot s's queries [pa(r), pa(r + 1)), and the
  // pieces joined in order give the same tables and item lists as one plan per
  // snapshot (plan_host sizes items by the whole batch)
  const bool par = S > 1 && nq1 >= 64;
  const uint32_t P =
      par ? std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)fgh::hw_threads(0) / S, nq1 / 128)) : 1u;
  auto pa = [&](uint32_t r) { return (uint32_t)((uint64_t)nq1 * r / P); };
  if (hs.size() < (size_t)S * P) hs.resize((size_t)S * P);
  // ---- the joined tables (this thread's buffers, reused like hs): several
  // snapshots' per-query tables are copied into their slots by the planning
  // workers themselves, the lists joined after
  struct Join {
    std::vector<uint32_t> q_m, q_terms, lead, q_filter, ngroup, q_hlo, q_hhi, q_hsh, f_shift, f_seg, ch_f, ch_c, ch_t, ch_s;
    std::vector<uint64_t> thr0, f_woff;
    std::vector<float> q_ub, q_wt, q_wn, q_rup, f_tab, f_max;
    std::vector<WItem> citems, ditems, scan, items;
  };
  static thread_local Join J_tl;
  Join& J = J_tl;
  for (auto* v : {&J.q_m, &J.q_terms, &J.lead, &J.q_filter, &J.ngroup, &J.q_hlo, &J.q_hhi, &J.q_hsh, &J.f_shift, &J.f_seg,
                  &J.ch_f, &J.ch_c, &J.ch_t, &J.ch_s})
    v->clear();
  for (auto* v : {&J.thr0, &J.f_woff}) v->clear();
  for (auto* v : {&J.q_ub, &J.q_wt, &J.q_wn, &J.q_rup, &J.f_tab, &J.f_max}) v->clear();
  for (auto* v : {&J.citems, &J.ditems, &J.scan, &J.items}) v->clear();
  auto &q_m = J.q_m, &q_terms = J.q_terms, &lead = J.lead, &q_filter = J.q_filter, &ngroup = J.ngroup, &q_hlo = J.q_hlo,
       &q_hhi = J.q_hhi, &q_hsh = J.q_hsh, &f_shift = J.f_shift, &f_seg = J.f_seg, &ch_f = J.ch_f, &ch_c = J.ch_c,
       &ch_t = J.ch_t, &ch_s = J.ch_s;
  auto &thr0 = J.thr0, &f_woff = J.f_woff;
  auto &q_ub = J.q_ub, &q_wt = J.q_wt, &q_wn = J.q_wn, &q_rup = J.q_rup, &f_tab = J.f_tab, &f_max = J.f_max;
  auto &citems = J.citems, &ditems = J.ditems, &scan = J.scan;
  const size_t nqt = (size_t)nq1 * fg::kMaxTerms;
  if (S > 1) {
    q_m.resize(nq);
    lead.resize(nq);
    ngroup.resize(nq);
    thr0.resize(nq);
    q_terms.resize(nqt * S);
    q_ub.resize(nqt * S);
    q_wt.resize(nqt * S);
    q_wn.resize(nqt * S);
    q_rup.resize(nqt * S);
  }
  auto put_slot = [&](uint32_t pc) {  // piece pc's per-query tables into its slots
    const HostPlan& h = hs[pc];
    const size_t v0 = (size_t)(pc / P) * nq1 + pa(pc % P), t0 = v0 * fg::kMaxTerms;
    auto cp = [](auto& dst, const auto& src, size_t at) { std::copy(src.begin(), src.end(), dst.begin() + at); };
    cp(q_m, h.q_m, v0);
    cp(lead, h.lead, v0);
    cp(ngroup, h.ngroup, v0);
    cp(thr0, h.thr0, v0);
    cp(q_terms, h.q_terms, t0);
    cp(q_ub, h.q_ub, t0);
    cp(q_wt, h.q_wt, t0);
    cp(q_wn, h.q_wn, t0);
    cp(q_rup, h.q_rup, t0);
  };
  if (par) {
    std::vector<int> rcs((size_t)S * P, FG_OK);
    std::vector<std::string> errs((size_t)S * P);
    run_parallel(S * P, [&](uint32_t pc) {
      const uint32_t a = pa(pc % P), b = pa(pc % P + 1);
      fg_query_batch qp = *q;  // the slice: q_off / f_off hold absolute offsets
      qp.n_queries = b - a;
      qp.q_off = q->q_off + a;
      if (q->f_off) qp.f_off = q->f_off + a;
      if ((rcs[pc] = plan_host(ixs[pc / P], &qp, k, S, hs[pc], nq1))) errs[pc] = fg_last_error();
      else put_slot(pc);
    });
    for (uint32_t pc = 0; pc < S * P; ++pc)
      if (rcs[pc]) return fail(rcs[pc], "snapshot %u: %s", pc / P, errs[pc].c_str());
  } else {
    for (uint32_t s = 0; s < S; ++s) {
      if (int rc = plan_host(ixs[s], q, k, S, hs[s], nq1)) {
        if (S == 1) return rc;
        const std::string e = fg_last_error();
        return fail(rc, "snapshot %u: %s", s, e.c_str());
      }
      if (S > 1) put_slot(s);
    }
  }
  if (ptrace) pt[1] = pnow();
  uint32_t nf = 0;
  if (S == 1) {
    HostPlan& h = hs[0];
    q_m.swap(h.q_m); q_terms.swap(h.q_terms); lead.swap(h.lead); q_filter.swap(h.q_filter); ngroup.swap(h.ngroup);
    q_hlo.swap(h.q_hlo); q_hhi.swap(h.q_hhi); q_hsh.swap(h.q_hsh); thr0.swap(h.thr0); q_ub.swap(h.q_ub);
    q_wt.swap(h.q_wt); q_wn.swap(h.q_wn); q_rup.swap(h.q_rup);
    f_shift.swap(h.f_shift); f_woff.swap(h.f_woff); f_tab.swap(h.f_tab); f_max.swap(h.f_max);
    ch_f.swap(h.ch_f); ch_c.swap(h.ch_c); ch_t.swap(h.ch_t); ch_s.swap(h.ch_s);
    citems.swap(h.citems); ditems.swap(h.ditems); scan.swap(h.scan);
    nf = h.nf;
  } else {
    auto cat = [](auto& dst, const auto& src) { dst.insert(dst.end(), src.begin(), src.end()); };
    f_woff.push_back(0);
    for (uint32_t pc = 0; pc < S * P; ++pc) {
      HostPlan& h = hs[pc];
      const uint32_t s = pc / P, fb = nf, vb = s * nq1 + pa(pc % P);
      for (uint32_t f : h.q_filter) q_filter.push_back(f == 0xFFFFFFFFu ? f : fb + f);
      cat(f_shift, h.f_shift); cat(f_tab, h.f_tab); cat(f_max, h.f_max);
      const uint64_t wb = f_woff.back();
      for (uint32_t f = 0; f < h.nf; ++f) {
        f_woff.push_back(wb + h.f_woff[f + 1]);
        f_seg.push_back(s);
      }
      for (uint32_t f : h.ch_f) ch_f.push_back(fb + f);
      cat(ch_c, h.ch_c); cat(ch_t, h.ch_t); cat(ch_s, h.ch_s);
      for (WItem x : h.citems) { x.q += vb; citems.push_back(x); }
      for (WItem x : h.ditems) { x.q += vb; ditems.push_back(x); }
      for (WItem x : h.scan) { x.q += vb; scan.push_back(x); }
      nf += h.nf;
    }
    // one bin geometry per batch query over the snapshots where it has work
    // items (fg_plan_link's rule): a bin counts the same scores in every slot
    q_hlo.assign(nq, 0x3F800000u);
    q_hhi.assign(nq, 0x3F800000u);
    q_hsh.assign(nq, 31);
    for (uint32_t i = 0, r = 0; i < nq1; ++i) {
      while (i >= pa(r + 1)) ++r;  // the piece of query i
      const uint32_t li = i - pa(r);
      uint32_t l = 0, hh = 0;
      bool any = false;
      for (uint32_t s = 0; s < S; ++s) {
        const HostPlan& h = hs[s * P + r];
        if (!h.ngroup[li]) continue;
        l = std::max(l, h.q_hlo[li]);
        hh = std::max(hh, h.q_hhi[li]);
        any = true;
      }
      if (!any) continue;
      hh = std::max(hh, l);
      for (uint32_t s = 0; s < S; ++s) {
        q_hlo[s * nq1 + i] = l;
        q_hhi[s * nq1 + i] = hh;
        q_hsh[s * nq1 + i] = bin_shift(l, hh);
      }
    }
  }
  if (ptrace) pt[2] = pnow();
  if (f_woff[nf] * 4 > (8ull << 30)) return fail(FG_EUNSUPPORTED, "facet masks of this batch exceed 8 GiB");
  if (ch_f.size() > 0x7FFFFFFFull) return fail(FG_EUNSUPPORTED, "facet postings of this batch too large");
  if (citems.size() + ditems.size() + scan.size() > 0x7FFFFFFFull)
    return fail(FG_EUNSUPPORTED, "batch too large (%zu work items)", citems.size() + ditems.size() + scan.size());
  using W = WItem;
  // k_conj: single-list queries' items first (their own k_conj launch), each part
  // in sweep order; k_disj: sweep order.  A stable LSD radix sort on (not single,
  // key quantized to 31 bits): the order is a scheduling choice only (every
  // order gives the same hits), and it takes a fraction of a comparison sort's
  // host time on a 20K-item batch.
  auto single = [&](const W& x) { return q_m[x.q] == fg::qm_pack(1, 1, 0); };
  // k_conj: the sweep split into 8 query groups, one per XCD (the kernel hands
  // XCD x the x-th eighth of its items), the queries whose lead list is the
  // same term in one group, groups balanced by items: headline k_conj 1.049 ->
  // 1.001 ms, identical hits (profiles/r05/ab/ab_xcd_key_balanced.log; by the
  // second list, ab_xcd_part.json: L2 hit rate 0.32 -> 0.23, DRAM 4.09 -> 4.57
  // GB, each XCD walks the whole doc range for fewer queries).  The same split of k_disj by
  // densest clause: OR top-20 2.78 -> 3.30 ms, top-1000 5.26 -> 6.86 ms -- its
  // sweep stays doc-ordered.
  constexpr bool xcd_part = true;
  std::vector<uint8_t> q_grp;
  auto groups = [&](const std::vector<W>& items) {
    q_grp.assign(nq, 0);
    // grouped by the lead list (ab_xcd_key_balanced.log: and3 1.001 ms, against 1.009
    // by the second list; the last list, the query alone and the slot's snapshot
    // measured no better)
    auto probe_term = [&](uint32_t qv) { return q_terms[(size_t)qv * fg::kMaxTerms]; };
    // the multi-list items only (single-list ones keep the sweep and run as a
    // launch of their own, k_conj<true> over the first n_single items), counted
    // per query slot (all of a slot's items share its lead term): the slots
    // radix-sorted by term, the (term, items) counts, the terms by items
    // (a comparison sort over every item's term cost ~0.4 ms of an 8-snapshot batch)
    static thread_local std::vector<uint64_t> ka, kb;
    ka.clear();
    for (uint32_t v = 0; v < nq; ++v)
      if (ngroup[v] && fg::qm_must(q_m[v]) && q_m[v] != fg::qm_pack(1, 1, 0))  // (k_conj slots only)
        ka.push_back(((uint64_t)probe_term(v) << 32) | v);
    kb.resize(ka.size());
    for (int sh = 32; sh < 64; sh += 11) {
      uint32_t cnt[2049] = {0};
      for (uint64_t x : ka) cnt[((x >> sh) & 2047u) + 1]++;
      for (int d = 0; d < 2048; ++d) cnt[d + 1] += cnt[d];
      for (uint64_t x : ka) kb[cnt[(x >> sh) & 2047u]++] = x;
      ka.swap(kb);
    }
    std::vector<std::pair<uint64_t, uint32_t>> by;  // (items, first index in ka)
    for (size_t i = 0; i < ka.size();) {
      size_t j = i;
      uint64_t c = 0;
      for (; j < ka.size() && (ka[j] >> 32) == (ka[i] >> 32); ++j) c += ngroup[(uint32_t)ka[j]];
      by.emplace_back(c, (uint32_t)i);
      i = j;
    }
    std::sort(by.begin(), by.end(), [&](auto& a, auto& b) {
      return a.first > b.first || (a.first == b.first && (ka[a.second] >> 32) < (ka[b.second] >> 32));
    });
    uint64_t gl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (auto& [c, i0] : by) {
      const uint32_t g = (uint32_t)(std::min_element(gl, gl + 8) - gl);
      gl[g] += c;
      for (size_t j = i0; j < ka.size() && (ka[j] >> 32) == (ka[i0] >> 32); ++j) q_grp[(uint32_t)ka[j]] = (uint8_t)g;
    }
    (void)items;
  };
  auto radix = [&](std::vector<W>& items, bool conj) {
    const size_t n = items.size();
    static thread_local std::vector<uint64_t> a, bb;  // (sort key << 32) | item index
    a.resize(n);
    bb.resize(n);
    // (items of queries probing the same list next to each other within each
    // 1/2048 of the sweep, so one XCD's L2 serves that list to all of them:
    // measured slower, profiles/r04/ab/ab_sweep_*.log)
    const bool part = conj && xcd_part;
    if (part) groups(items);
    for (size_t x = 0; x < n; ++x) {
      const double kk = std::min(std::max(items[x].key, 0.0), 1.0);
      // single-list items keep the plain sweep (grouped: C3's mix 1.07 -> 1.11 ms)
      // (within a group, the sweep alone: also keying the items of one second / third /
      // lead list together inside each 1/16 or 1/64 of the sweep ran 0.971 -> 1.004 /
      // 0.999 / 0.982 ms, identical hits: profiles/r06/ab/conj_order.log)
      const uint32_t sw = part && !single(items[x]) ? ((uint32_t)q_grp[items[x].q] << 28) | (uint32_t)(kk * 268435455.0)
                                                    : (uint32_t)(kk * 2147483647.0);
      const uint32_t rk = (conj && single(items[x]) ? 0u : 0x80000000u) | sw;
      a[x] = ((uint64_t)rk << 32) | (uint64_t)x;
    }
    for (int sh = 32; sh < 64; sh += 11) {
      uint32_t cnt[2049] = {0};
      for (size_t x = 0; x < n; ++x) cnt[((a[x] >> sh) & 2047u) + 1]++;
      for (int d = 0; d < 2048; ++d) cnt[d + 1] += cnt[d];
      for (size_t x = 0; x < n; ++x) bb[cnt[(a[x] >> sh) & 2047u]++] = a[x];
      a.swap(bb);
    }
    static thread_local std::vector<W> sorted;
    sorted.resize(n);
    for (size_t x = 0; x < n; ++x) sorted[x] = items[(uint32_t)a[x]];
    items.swap(sorted);
  };
  radix(citems, true);
  radix(ditems, false);
  auto& items = J.items;
  items.reserve(citems.size() + ditems.size() + scan.size());
  items.insert(items.end(), citems.begin(), citems.end());
  const uint64_t n_conj = citems.size();
  items.insert(items.end(), ditems.begin(), ditems.end());
  uint64_t n_single = 0;
  for (const W& x : citems) n_single += single(x) ? 1 : 0;
  std::stable_sort(scan.begin(), scan.end(), [](const W& a, const W& b) { return a.key < b.key; });
  const uint64_t n_main = items.size(), n_scan = scan.size();
  const uint64_t chunks = n_main + n_scan;  // from here on: work items (k_conj / k_disj, then k_scan)
  if (chunks > 0x7FFFFFFFull) return fail(FG_EUNSUPPORTED, "batch too large (%llu work items)", (unsigned long long)chunks);
  items.insert(items.end(), scan.begin(), scan.end());
  static thread_local std::vector<uint32_t> work_q, work_c, work_n;
  static thread_local std::vector<uint64_t> cand_off;
  work_q.resize(chunks);
  work_c.resize(chunks);
  work_n.resize(chunks);
  cand_off.assign(nq + 1, 0);
  for (uint64_t w = 0; w < chunks; ++w) {
    work_q[w] = items[w].q;
    work_c[w] = items[w].c;
    work_n[w] = items[w].n;
  }
  // each work item appends at most k keys to its query's candidate list
  for (uint32_t i = 0; i < nq; ++i) cand_off[i + 1] = cand_off[i] + (uint64_t)ngroup[i] * k;

  if (ptrace) pt[3] = pnow();
  auto p = std::make_unique<fg_plan>();
  p->nq = nq;
  p->nq_batch = nq1;
  p->n_segs = S;
  p->k = k;
  p->mode = q->mode;
  p->total_chunks = (uint32_t)chunks;
  p->n_scan = (uint32_t)n_scan;
  p->mem.dev = ix->dev;
  // one allocation: [inputs | zeroed (thresh, cand_cnt, facet masks) | candidates | outputs]
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t nch = ch_f.size();
  const size_t s_qm = al(4ull * nq), s_qt = al(4ull * nq * fg::kMaxTerms), s_lead = al(4ull * nq),
               s_wq = al(4ull * chunks), s_wc = al(4ull * chunks), s_wn = al(4ull * chunks),
               s_co = al(8ull * (nq + 1)), s_t0 = al(8ull * nq), s_ub = al(4ull * nq * fg::kMaxTerms),
               s_cache = al(4ull * 512 * S),
               s_qf = al(4ull * nq), s_fs = al(4ull * nf),
               s_fw = al(8ull * nf), s_ft = al(4ull * nf * 256), s_fm = al(4ull * nf), s_ch = al(4ull * nch),
               s_hb = al(4ull * nq), s_fg = S > 1 ? al(4ull * nf) : 0,
               s_sg = S > 1 ? al(sizeof(fg::DevIndex) * S) : 0, s_sb = S > 1 ? al(4ull * S) : 0;
  // the snapshots' first docs in their concatenation (k_final's merged select)
  std::vector<uint32_t> seg_base;
  if (S > 1) {
    uint64_t b = 0;
    for (uint32_t x = 0; x < S; ++x) {
      seg_base.push_back((uint32_t)std::min<uint64_t>(b, 0xFFFFFFFFull));
      b += ixs[x]->n_docs;
    }
    if (b > 0xFFFFFFFFull) seg_base.clear();  // no merged select past 2^32 docs
  }
  // the snapshots' tf caches (query-time scoring, DevIndex::cache): one copy per
  // distinct set of statistics (a namespace's segments share one)
  std::vector<uint32_t> cache_of(S, 0);
  for (uint32_t x = 0; x < S; ++x) {
    uint32_t c = 0;
    while (c < x && std::memcmp(ixs[cache_of[c]]->cache, ixs[x]->cache, sizeof ixs[x]->cache) != 0) ++c;
    cache_of[x] = c < x ? cache_of[c] : x;  // x: the first snapshot with these statistics
  }
  const size_t s_in = s_qm + s_qt + s_lead + s_wq + s_wc + s_wn + s_co + s_t0 + 4 * s_ub + s_cache + s_qf + s_fs + s_fw +
                      s_ft + s_fm + 4 * s_ch + 2 * s_hb + s_fg + s_sg + s_sb;
  // one score histogram per query (DevPlan::hist: k_conj's and k_disj's running thresholds)
  // (thresholds and histograms: one per batch query, shared by its slots)
  const size_t s_thr = al(8ull * nq1), s_cc = al(4ull * nq), s_mask = al(4ull * f_woff[nf]),
               s_hist = al(4ull * nq1 * fg::kQBins);
  const size_t s_ck = al(8ull * cand_off[nq]);
  const size_t s_os = al(4ull * nq * k), s_od = al(4ull * nq * k), s_on = al(4ull * nq);
#ifdef FG_DIAG
  const size_t s_dg = al(8ull * fg::kDiagPerWg * (chunks + nq));
#else
  const size_t s_dg = 0;
#endif
  const size_t total = s_in + s_thr + s_cc + s_mask + s_hist + s_ck + s_os + s_od + s_on + s_dg;
  HIPCHK(hipSetDevice(ix->dev));
  char* base = static_cast<char*>(ix->pool->get(std::max<size_t>(total, 256), &p->ws_got));
  if (!base) return fail(FG_EOOM, "plan workspace hipMalloc(%zu) failed", total);
  p->ws = base;
  p->ix = ix;  // owns the workspace from here on (returned to ix->pool); retained below
  fg_index_retain(ix);
  for (uint32_t s = 1; s < S; ++s) {
    fg_index_retain(ixs[s]);
    p->segs.push_back(ixs[s]);
  }
  p->ws_bytes = total;
  // a small zero region (thresholds, candidate counts, facet masks) travels
  // zeroed with the upload, so the first execute needs no memset
  const size_t s_zero = s_thr + s_cc + s_mask + s_hist;
  const size_t s_up = s_in + (s_zero <= (64u << 10) ? s_zero : 0);
  PinnedLease pin(*ix->pinned, s_up);
  std::vector<char> staging_pageable;  // only if the pinned allocation failed
  char* staging = static_cast<char*>(pin.p);
  if (!staging) {
    staging_pageable.assign(s_up, 0);
    staging = staging_pageable.data();
  } else if (s_up > s_in) {
    std::memset(staging + s_in, 0, s_up - s_in);
  }
  size_t o = 0;
  auto put = [&](const void* src, size_t bytes, size_t slot) {
    if (bytes) std::memcpy(staging + o, src, bytes);
    void* dptr = base + o;
    o += slot;
    return dptr;
  };
  p->d.q_m = (const uint32_t*)put(q_m.data(), 4ull * nq, s_qm);
  p->d.q_terms = (const uint32_t*)put(q_terms.data(), 4ull * nq * fg::kMaxTerms, s_qt);
  p->d.q_lead_df = (const uint32_t*)put(lead.data(), 4ull * nq, s_lead);
  p->d.work_q = (const uint32_t*)put(work_q.data(), 4ull * chunks, s_wq);
  p->d.work_c = (const uint32_t*)put(work_c.data(), 4ull * chunks, s_wc);
  p->d.work_n = (const uint32_t*)put(work_n.data(), 4ull * chunks, s_wn);
  p->d.cand_off = (const uint64_t*)put(cand_off.data(), 8ull * (nq + 1), s_co);
  p->d.q_thr0 = (const uint64_t*)put(thr0.data(), 8ull * nq, s_t0);
  p->d.q_ub = (const float*)put(q_ub.data(), 4ull * nq * fg::kMaxTerms, s_ub);
  p->d.q_wt = (const float*)put(q_wt.data(), 4ull * nq * fg::kMaxTerms, s_ub);
  p->d.q_wn = (const float*)put(q_wn.data(), 4ull * nq * fg::kMaxTerms, s_ub);
  p->d.q_rup = (const float*)put(q_rup.data(), 4ull * nq * fg::kMaxTerms, s_ub);
  std::vector<const float*> d_cache(S, nullptr);
  {
    const size_t o0 = o;
    for (uint32_t x = 0; x < S; ++x) {
      if (cache_of[x] != x) continue;
      std::memcpy(staging + o, ixs[x]->cache, 4ull * 512);
      d_cache[x] = (const float*)(base + o);
      o += 4ull * 512;
    }
    for (uint32_t x = 0; x < S; ++x) d_cache[x] = d_cache[cache_of[x]];
    o = o0 + s_cache;
  }
  p->d0 = ix->d;
  p->d0.cache = d_cache[0];
  p->d.f.q_filter = (const uint32_t*)put(q_filter.data(), 4ull * nq, s_qf);
  p->d.f.f_shift = (const uint32_t*)put(f_shift.data(), 4ull * nf, s_fs);
  p->d.f.f_woff = (const uint64_t*)put(f_woff.data(), 8ull * nf, s_fw);
  p->d.f.f_tab = (const float*)put(f_tab.data(), 4ull * nf * 256, s_ft);
  p->d.f.f_max = (const float*)put(f_max.data(), 4ull * nf, s_fm);
  p->d.f.ch_filter = (const uint32_t*)put(ch_f.data(), 4ull * nch, s_ch);
  p->d.f.ch_clause = (const uint32_t*)put(ch_c.data(), 4ull * nch, s_ch);
  p->d.f.ch_term = (const uint32_t*)put(ch_t.data(), 4ull * nch, s_ch);
  p->d.f.ch_start = (const uint32_t*)put(ch_s.data(), 4ull * nch, s_ch);
  p->d.q_hlo = (const uint32_t*)put(q_hlo.data(), 4ull * nq, s_hb);
  p->d.q_hsh = (const uint32_t*)put(q_hsh.data(), 4ull * nq, s_hb);
  if (S > 1) {
    std::vector<fg::DevIndex> segs(S);
    for (uint32_t s = 0; s < S; ++s) {
      segs[s] = ixs[s]->d;
      segs[s].cache = d_cache[s];
    }
    p->d.f.f_seg = (const uint32_t*)put(f_seg.data(), 4ull * nf, s_fg);
    p->d.segs = (const fg::DevIndex*)put(segs.data(), sizeof(fg::DevIndex) * S, s_sg);
    const uint32_t* sb = (const uint32_t*)put(seg_base.data(), 4ull * seg_base.size(), s_sb);
    p->d.seg_base = seg_base.empty() ? nullptr : sb;
  }
  // on the planning thread's own stream (or the caller's `up`): a plan built
  // while another thread's batch runs does not serialise against it through the
  // legacy null stream
  HIPCHK(hipMemcpyAsync(base, staging, s_up, hipMemcpyHostToDevice, up));
  p->up_stream = up;
  p->zeroed = s_up > s_in;
  if (sync || !pin.p) {
    HIPCHK(hipStreamSynchronize(up));
  } else {
    p->pin = pin.p;  // the plan returns it (after a sync) when destroyed
    p->pin_n = pin.n;
    pin.p = nullptr;
  }
  char* cur = base + s_in;
  p->zero_region = cur;
  p->zero_bytes = s_zero;
  p->d.thresh = (uint64_t*)cur;
  cur += s_thr;
  p->d.cand_cnt = (uint32_t*)cur;
  cur += s_cc;
  p->d.f.fmask = (uint32_t*)cur;
  cur += s_mask;
  p->d.hist = (uint32_t*)cur;
  cur += s_hist;
  p->d.cand_keys = (uint64_t*)cur;
  cur += s_ck;
  p->own_score = (float*)cur;
  cur += s_os;
  p->own_doc = (uint32_t*)cur;
  cur += s_od;
  p->own_n = (uint32_t*)cur;
  cur += s_on;
  p->d.diag = s_dg ? (uint64_t*)cur : nullptr;
  p->diag_words = s_dg / 8;
  p->d.n_queries = nq;
  p->d.total_chunks = (uint32_t)n_main;
  p->d.n_conj = (uint32_t)n_conj;
  p->d.n_scan = (uint32_t)n_scan;
  p->d.n_single = (uint32_t)n_single;
  p->d.k = k;
  p->d.seg_nq = S > 1 ? nq1 : 0;
  p->d.n_segs = S;
  // query-time scores when some snapshot's statistics changed since its build
  // (a commit elsewhere in the namespace); else the build-time scores
  p->d.feat = 0;
  for (uint32_t x = 0; x < S; ++x)
    if (!ixs[x]->same_stats) p->d.feat = 4u;
  for (uint32_t x = 0; x < S && p->d.feat; ++x)
    p->d.feat |= (ixs[x]->d.tfn_name ? 1u : 0u) | (ixs[x]->d.n_esc ? 2u : 0u);
  // several snapshots: a batch query's slots share its threshold score-only, so a
  // doc of another snapshot tied with the k-th score is never pruned (the merge
  // breaks such ties by snapshot)
  p->d.pub_mask = S > 1 ? 0xFFFFFFFF00000000ull : ~0ull;
  p->h_any.assign(nq1, 0);
  for (uint32_t v = 0; v < nq; ++v)
    if (ngroup[v]) p->h_any[v % nq1] = 1;
  p->h_lo.swap(q_hlo);
  p->h_hi.swap(q_hhi);
  p->d.f.n_filters = nf;
  p->d.f.n_chunks = (uint32_t)nch;
  if (ptrace && S > 1) {
    pt[4] = pnow();
    fprintf(stderr, "[fg plan] %u snapshots x %u queries: plan_host %.3f join %.3f items %.3f stage+upload %.3f ms\n", S,
            nq1, pt[1] - pt[0], pt[2] - pt[1], pt[3] - pt[2], pt[4] - pt[3]);
  }
  *out = p.release();
  return FG_OK;
}

// the kernels of a planned batch on stream s, or of one part of it: the k_disj
// items [from, to) of its sweep (fractions of the k_disj range, in sweep order:
// every query's first docs first).  The first part (from = 0) zeroes the plan's
// state and runs k_fmask + k_conj, the last (to = 1) k_scan + k_final;
// out_shard != nullptr: a multi-snapshot plan's merged select
static int execute_impl(fg_plan* p, hipStream_t s, float* os, uint32_t* od, uint32_t* on, uint32_t* oshard,
                        double from = 0.0, double to = 1.0) {
  HIPCHK(hipSetDevice(p->ix->dev));
  const bool first = from <= 0.0, last = to >= 1.0;
  if (first && !p->d.n_peers) {  // (with peers: fg_plan_reset, ordered before every peer's execute)
    if (p->zeroed) p->zeroed = false;  // the first execute after the upload
    else HIPCHK(hipMemsetAsync(p->zero_region, 0, p->zero_bytes, s));
  }
  hipEvent_t ev[3] = {};
  if (p->profile) {
    for (auto& e : ev) HIPCHK(hipEventCreate(&e));
    HIPCHK(hipEventRecord(ev[0], s));
  }
  if (first && p->d.f.n_chunks) HIPCHK(fg::launch_fmask(p->d0, p->d, s));
  if (first && p->d.n_conj) HIPCHK(fg::launch_conj(p->d0, p->d, s));
  const uint32_t nd = p->d.total_chunks - p->d.n_conj;
  const uint32_t a = first ? 0u : (uint32_t)std::min<double>(nd, std::llround(from * nd));
  const uint32_t b = last ? nd : (uint32_t)std::min<double>(nd, std::llround(to * nd));
  if (b > a) HIPCHK(fg::launch_disj(p->d0, p->d, s, a, b - a));
  if (last && p->d.n_scan) HIPCHK(fg::launch_scan(p->d0, p->d, s));
  if (p->profile) HIPCHK(hipEventRecord(ev[1], s));
  if (last) HIPCHK(fg::launch_final(p->d, os, od, on, s, oshard));
  if (p->profile) {
    HIPCHK(hipEventRecord(ev[2], s));
    p->pending.insert(p->pending.end(), ev, ev + 3);
  }
  p->last_stream = s;
  p->last_stream_used = true;
  return FG_OK;
}

int fg_plan_execute(fg_plan* p, void* stream, float* d_out_score, uint32_t* d_out_doc, uint32_t* d_out_n) {
  if (!p) return fail(FG_EINVAL, "NULL plan");
  return execute_impl(p, static_cast<hipStream_t>(stream), d_out_score ? d_out_score : p->own_score,
                      d_out_doc ? d_out_doc : p->own_doc, d_out_n ? d_out_n : p->own_n, nullptr);
}

// A multi-snapshot plan straight to the merged top-k of every batch query: the
// kernels of fg_plan_execute, then ONE k_final over all slots of each query
// (keys shifted by the snapshots' bases) in place of per-slot lists + merge
int fg_plan_execute_merged(fg_plan* p, void* stream, float* d_out_score, uint32_t* d_out_doc, uint32_t* d_out_shard,
                           uint32_t* d_out_n) {
  if (!p || !d_out_score || !d_out_doc || !d_out_shard || !d_out_n) return fail(FG_EINVAL, "bad arguments");
  if (p->n_segs < 2 || !p->d.seg_base)
    return fail(FG_EUNSUPPORTED, "not a multi-snapshot plan over < 2^32 docs (use fg_plan_execute + fg_merge_shards)");
  return execute_impl(p, static_cast<hipStream_t>(stream), d_out_score, d_out_doc, d_out_n, d_out_shard);
}

// One part of a plan's k_disj sweep (fugu.h): doc-sharded namespaces over
// several devices or processes exchange their per-query score histograms
// between the parts, so every shard's later items prune with the counts of all
// shards' earlier ones (what linked plans share through memory on one device)
int fg_plan_execute_part(fg_plan* p, void* stream, double from, double to, float* d_out_score, uint32_t* d_out_doc,
                         uint32_t* d_out_shard, uint32_t* d_out_n) {
  if (!p) return fail(FG_EINVAL, "NULL plan");
  if (!(from >= 0.0 && from < to && to <= 1.0)) return fail(FG_EINVAL, "part [%g, %g) not inside [0, 1)", from, to);
  // parts in sweep order, each starting where the last one ended (the first
  // zeroes the plan's state, the last runs the final select)
  if (from > 0.0 && from != p->part_next)
    return fail(FG_EINVAL, "part [%g, %g) does not continue the plan's sweep (next part starts at %g)", from, to,
                p->part_next);
  if (d_out_shard && (p->n_segs < 2 || !p->d.seg_base))
    return fail(FG_EUNSUPPORTED, "merged select: not a multi-snapshot plan over < 2^32 docs");
  if (d_out_shard && (!d_out_score || !d_out_doc || !d_out_n)) return fail(FG_EINVAL, "merged select needs every output");
  const int rc = execute_impl(p, static_cast<hipStream_t>(stream), d_out_score ? d_out_score : p->own_score,
                              d_out_doc ? d_out_doc : p->own_doc, d_out_n ? d_out_n : p->own_n, d_out_shard, from, to);
  if (rc == FG_OK) p->part_next = to >= 1.0 ? 0.0 : to;
  return rc;
}

int fg_plan_set_peers(fg_plan* p, fg_plan* const* peers, uint32_t n) {
  if (!p || (n && !peers)) return fail(FG_EINVAL, "bad arguments");
  if (n > FG_MAX_PEERS) return fail(FG_EUNSUPPORTED, "%u peers (> FG_MAX_PEERS = %d)", n, FG_MAX_PEERS);
  for (uint32_t i = 0; i < n; ++i) {
    const fg_plan* o = peers[i];
    if (!o || o == p) return fail(FG_EINVAL, "peer %u: NULL or the plan itself", i);
    if (o->nq_batch != p->nq_batch || o->k != p->k) return fail(FG_EINVAL, "peer %u plans another batch or k", i);
    if (o->h_lo.size() != p->h_lo.size()) return fail(FG_EINVAL, "peer %u: another number of query slots", i);
    if (o->ix->dev != p->ix->dev) {
      int ok = 0;
      HIPCHK(hipDeviceCanAccessPeer(&ok, p->ix->dev, o->ix->dev));
      if (!ok) return fail(FG_EUNSUPPORTED, "device %d cannot reach peer %u's device %d", p->ix->dev, i, o->ix->dev);
    }
  }
  p->d.n_peers = n;
  for (uint32_t i = 0; i < n; ++i) {
    p->d.peer_hist[i] = peers[i]->d.hist;
    p->d.peer_thr[i] = peers[i]->d.thresh;
  }
  if (n) p->d.pub_mask = 0xFFFFFFFF00000000ull;  // score-only: the peers' docs are other docs
  return FG_OK;
}

int fg_plan_ipc_export(const fg_plan* p, fg_plan_ipc* out) {
  if (!p || !out) return fail(FG_EINVAL, "bad arguments");
  const char* ws = static_cast<const char*>(p->ws);
  const char* th = reinterpret_cast<const char*>(p->d.thresh);
  const char* hi = reinterpret_cast<const char*>(p->d.hist);
  if (th < ws || th >= ws + p->ws_got || hi < ws || hi >= ws + p->ws_got)
    return fail(FG_EUNSUPPORTED, "the plan's thresholds are another plan's (linked): export that plan");
  std::memset(out, 0, sizeof *out);
  hipIpcMemHandle_t h;
  HIPCHK(hipSetDevice(p->ix->dev));
  HIPCHK(hipIpcGetMemHandle(&h, p->ws));
  static_assert(sizeof h <= sizeof out->handle, "fg_plan_ipc::handle");
  std::memcpy(out->handle, &h, sizeof h);
  out->thresh_off = (uint64_t)(th - ws);
  out->hist_off = (uint64_t)(hi - ws);
  out->n_queries = p->nq_batch;
  out->k = p->k;
  out->device = p->ix->dev;
  return FG_OK;
}

int fg_plan_set_ipc_peers(fg_plan* p, const fg_plan_ipc* peers, uint32_t n) {
  if (!p || (n && !peers)) return fail(FG_EINVAL, "bad arguments");
  if (n > FG_MAX_PEERS) return fail(FG_EUNSUPPORTED, "%u peers (> FG_MAX_PEERS = %d)", n, FG_MAX_PEERS);
  for (uint32_t i = 0; i < n; ++i)
    if (peers[i].n_queries != p->nq_batch || peers[i].k != p->k) return fail(FG_EINVAL, "peer %u plans another batch or k", i);
  HIPCHK(hipSetDevice(p->ix->dev));
  std::vector<void*> maps;
  for (uint32_t i = 0; i < n; ++i) {
    hipIpcMemHandle_t h;
    std::memcpy(&h, peers[i].handle, sizeof h);
    void* base = nullptr;
    if (hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      (void)hipGetLastError();
      for (void* m : maps) (void)hipIpcCloseMemHandle(m);
      return fail(FG_EHIP, "peer %u: hipIpcOpenMemHandle failed", i);
    }
    maps.push_back(base);
  }
  for (void* m : p->ipc_maps) (void)hipIpcCloseMemHandle(m);
  p->ipc_maps = maps;
  p->d.n_peers = n;
  for (uint32_t i = 0; i < n; ++i) {
    p->d.peer_thr[i] = reinterpret_cast<uint64_t*>(static_cast<char*>(maps[i]) + peers[i].thresh_off);
    p->d.peer_hist[i] = reinterpret_cast<uint32_t*>(static_cast<char*>(maps[i]) + peers[i].hist_off);
  }
  if (n) p->d.pub_mask = 0xFFFFFFFF00000000ull;
  return FG_OK;
}

int fg_plan_reset(fg_plan* p, void* stream) {
  if (!p) return fail(FG_EINVAL, "NULL plan");
  HIPCHK(hipSetDevice(p->ix->dev));
  HIPCHK(hipMemsetAsync(p->zero_region, 0, p->zero_bytes, static_cast<hipStream_t>(stream)));
  p->zeroed = false;
  return FG_OK;
}

static_assert(fg::kQBins == FG_HIST_BINS, "fugu.h's histogram size");
static_assert(fg::kMaxPeers == FG_MAX_PEERS, "fugu.h's peer count");

int fg_plan_hist_span(const fg_plan* p, uint32_t* lo, uint32_t* hi) {
  if (!p || !lo || !hi) return fail(FG_EINVAL, "bad arguments");
  const uint32_t nb = p->nq_batch;
  for (uint32_t i = 0; i < nb; ++i) {
    const bool any = i < p->h_any.size() && p->h_any[i];
    lo[i] = any ? p->h_lo[i] : 0u;
    hi[i] = any ? p->h_hi[i] : 0u;
  }
  return FG_OK;
}

int fg_plan_set_hist_span(fg_plan* p, const uint32_t* lo, const uint32_t* hi) {
  if (!p || !lo || !hi) return fail(FG_EINVAL, "bad arguments");
  const uint32_t nb = p->nq_batch, S = p->n_segs;
  if (p->h_lo.size() < (size_t)nb * S || p->h_hi.size() < (size_t)nb * S)
    return fail(FG_EUNSUPPORTED, "a linked plan's bins are redrawn by fg_plan_link");
  std::vector<uint32_t> L(p->nq), SH(p->nq);
  for (uint32_t s = 0; s < S; ++s)
    for (uint32_t i = 0; i < nb; ++i) {
      const size_t v = (size_t)s * nb + i;
      uint32_t l = lo[i], h = std::max(hi[i], lo[i]);
      if (l == 0 && h == 0) {  // no shard has work for the query: keep the plan's own bins
        l = p->h_lo[v];
        h = p->h_hi[v];
      }
      p->h_lo[v] = l;
      p->h_hi[v] = h;
      L[v] = l;
      SH[v] = bin_shift(l, h);
    }
  HIPCHK(hipSetDevice(p->ix->dev));
  if (p->pin) HIPCHK(hipStreamSynchronize(p->up_stream));  // an upload still in flight would overwrite them
  if (p->nq) {
    HIPCHK(hipMemcpy(const_cast<uint32_t*>(p->d.q_hlo), L.data(), 4ull * p->nq, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(const_cast<uint32_t*>(p->d.q_hsh), SH.data(), 4ull * p->nq, hipMemcpyHostToDevice));
  }
  return FG_OK;
}

int fg_plan_hist_copy(fg_plan* p, void* stream, uint32_t* d_buf, int into_plan) {
  if (!p || !d_buf) return fail(FG_EINVAL, "bad arguments");
  HIPCHK(hipSetDevice(p->ix->dev));
  const size_t bytes = 4ull * p->nq_batch * fg::kQBins;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (into_plan) HIPCHK(hipMemcpyAsync(p->d.hist, d_buf, bytes, hipMemcpyDeviceToDevice, s));
  else HIPCHK(hipMemcpyAsync(d_buf, p->d.hist, bytes, hipMemcpyDeviceToDevice, s));
  return FG_OK;
}

int fg_plan_results(fg_plan* p, float* out_score, uint32_t* out_doc, uint32_t* out_n) {
  if (!p) return fail(FG_EINVAL, "NULL plan");
  HIPCHK(hipSetDevice(p->ix->dev));
  // copies on the plan's stream (a per-thread stream under fg_search_batch), then wait for it
  const size_t nk = (size_t)p->nq * p->k;
  hipStream_t s = p->last_stream;
  // own_score, own_doc, own_n are consecutive in the workspace: one D2H into a
  // pinned buffer, then host copies (small batches: the batch-of-one latency)
  const char* first = reinterpret_cast<const char*>(p->own_score);
  const size_t span = reinterpret_cast<const char*>(p->own_n) + 4ull * p->nq - first;
  if (span <= (4ull << 20)) {
    PinnedLease pin(*p->ix->pinned, span);
    if (pin.p) {
      HIPCHK(hipMemcpyAsync(pin.p, first, span, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      const char* h = static_cast<const char*>(pin.p);
      if (out_score) std::memcpy(out_score, h, 4 * nk);
      if (out_doc) std::memcpy(out_doc, h + (reinterpret_cast<const char*>(p->own_doc) - first), 4 * nk);
      if (out_n) std::memcpy(out_n, h + (reinterpret_cast<const char*>(p->own_n) - first), 4ull * p->nq);
      return FG_OK;
    }
  }
  if (out_score) HIPCHK(hipMemcpyAsync(out_score, p->own_score, 4 * nk, hipMemcpyDeviceToHost, s));
  if (out_doc) HIPCHK(hipMemcpyAsync(out_doc, p->own_doc, 4 * nk, hipMemcpyDeviceToHost, s));
  if (out_n) HIPCHK(hipMemcpyAsync(out_n, p->own_n, 4ull * p->nq, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return FG_OK;
}

int fg_plan_info_get(const fg_plan* p, fg_plan_info* o) {
  if (!p || !o) return fail(FG_EINVAL, "bad arguments");
  o->n_queries = p->nq;
  o->k = p->k;
  o->total_chunks = p->total_chunks;
  o->workspace_bytes = p->ws_bytes;
  return FG_OK;
}

int fg_plan_profile(fg_plan* p, int enable) {
  if (!p) return fail(FG_EINVAL, "NULL plan");
  p->profile = enable != 0;
  return FG_OK;
}

int fg_plan_kernel_ms(fg_plan* p, double* ms_out, uint32_t* n_out) {
  if (!p) return fail(FG_EINVAL, "NULL plan");
  HIPCHK(hipSetDevice(p->ix->dev));
  for (size_t i = 0; i + 2 < p->pending.size(); i += 3) {
    HIPCHK(hipEventSynchronize(p->pending[i + 2]));
    for (int kx = 0; kx < 2; ++kx) {
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, p->pending[i + kx], p->pending[i + kx + 1]));
      p->ms[kx] += ms;
    }
    p->n_prof++;
  }
  for (hipEvent_t e : p->pending) (void)hipEventDestroy(e);
  p->pending.clear();
  if (ms_out) for (int kx = 0; kx < 2; ++kx) ms_out[kx] = p->ms[kx];
  if (n_out) *n_out = p->n_prof;
  p->ms[0] = p->ms[1] = 0;
  p->n_prof = 0;
  return FG_OK;
}

int fg_plan_diag(fg_plan* p, uint64_t* out, size_t n_words, uint32_t* cand_cnt) {
  if (!p) return fail(FG_EINVAL, "NULL plan");
  HIPCHK(hipSetDevice(p->ix->dev));
  HIPCHK(hipStreamSynchronize(p->last_stream));
  if (cand_cnt) HIPCHK(hipMemcpy(cand_cnt, p->d.cand_cnt, 4ull * p->nq, hipMemcpyDeviceToHost));
  if (out && n_words) {
    if (!p->d.diag) return fail(FG_EUNSUPPORTED, "not a diagnostic build (-DFG_DIAG)");
    HIPCHK(hipMemcpy(out, p->d.diag, 8 * std::min(n_words, p->diag_words), hipMemcpyDeviceToHost));
  }
  return FG_OK;
}

int fg_plan_destroy(fg_plan* p) {
  delete p;
  return FG_OK;
}

// One per-query threshold word and score histogram for plans of one batch on
// one device (fugu.h).  Every plan's bins are re-drawn over the union of the
// plans' score spans, so a bin means the same scores in every plan.
int fg_plan_link(fg_plan* const* plans, uint32_t n) {
  if (!plans || n == 0) return fail(FG_EINVAL, "bad arguments");
  fg_plan* o = plans[0];
  for (uint32_t i = 0; i < n; ++i) {
    if (!plans[i]) return fail(FG_EINVAL, "NULL plan");
    if (plans[i]->nq != o->nq || plans[i]->k != o->k) return fail(FG_EINVAL, "linked plans differ in batch or k");
    if (plans[i]->ix->dev != o->ix->dev) return fail(FG_EINVAL, "linked plans live on different devices");
    if (plans[i]->n_segs > 1) return fail(FG_EUNSUPPORTED, "a multi-snapshot plan already shares its thresholds");
  }
  const uint32_t nq = o->nq;
  std::vector<uint32_t> lo(nq, 0), sh(nq, 0);
  for (uint32_t q = 0; q < nq; ++q) {
    uint32_t l = 0, h = 0;
    for (uint32_t i = 0; i < n; ++i) {
      l = std::max(l, plans[i]->h_lo[q]);
      h = std::max(h, plans[i]->h_hi[q]);
    }
    h = std::max(h, l);
    lo[q] = l;
    sh[q] = bin_shift(l, h);
  }
  HIPCHK(hipSetDevice(o->ix->dev));
  for (uint32_t i = 0; i < n; ++i) {
    fg_plan* p = plans[i];
    if (nq) {
      HIPCHK(hipMemcpy(const_cast<uint32_t*>(p->d.q_hlo), lo.data(), 4ull * nq, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(const_cast<uint32_t*>(p->d.q_hsh), sh.data(), 4ull * nq, hipMemcpyHostToDevice));
    }
    p->h_lo = lo;
    for (uint32_t q = 0; q < nq; ++q) p->h_hi[q] = std::max(p->h_hi[q], lo[q]);
    p->d.thresh = o->d.thresh;
    p->d.hist = o->d.hist;
    p->d.pub_mask = 0xFFFFFFFF00000000ull;  // score-only
  }
  return FG_OK;
}

int fg_search_batch(fg_index* ix, const fg_query_batch* q, uint32_t k, float* out_score, uint32_t* out_doc,
                    uint32_t* out_n) {
  fg_plan* p = nullptr;
  int rc = plan_create(ix, q, k, &p, false);  // execute is queued behind the upload on the same stream
  if (rc) return rc;
  std::unique_ptr<fg_plan> guard(p);
  // the calling thread's own stream: concurrent callers (tokio workers sharing
  // one Arc<Dataset>, src/db/config.rs:93) run their batches side by side
  if ((rc = fg_plan_execute(p, hipStreamPerThread, nullptr, nullptr, nullptr))) return rc;
  return fg_plan_results(p, out_score, out_doc, out_n);
}

int fg_merge_shards(uint32_t n_shards, uint32_t n_queries, uint32_t k, const float* d_score, const uint32_t* d_doc,
                    const uint32_t* d_n, float* d_out_score, uint32_t* d_out_doc, uint32_t* d_out_shard,
                    uint32_t* d_out_n, void* stream) {
  if (n_shards == 0 || n_shards > 64 || k == 0 || !d_score || !d_doc || !d_n || !d_out_score || !d_out_doc || !d_out_n)
    return fail(FG_EINVAL, "bad arguments");
  HIPCHK(fg::launch_merge(n_shards, n_queries, k, d_score, d_doc, d_n, d_out_score, d_out_doc, d_out_shard, d_out_n,
                          static_cast<hipStream_t>(stream)));
  return FG_OK;
}

// Persistent worker threads of fg_search_sharded's batch mode: a thread's
// first HIP call sets up per-thread runtime state, so threads made per call
// cost more than the planning they run.  Jobs never wait on other jobs, so a
// fixed pool serves any number of concurrent callers.  Never destroyed (idle
// workers end with the process).
class ShardWorkers {
 public:
  static ShardWorkers& get() {
    static ShardWorkers* w = new ShardWorkers(std::max(8, std::min(64, hw_threads(0))));
    return *w;
  }
  // f(0..n-1) on the workers; returns when all have run
  void run(uint32_t n, const std::function<void(uint32_t)>& f) {
    struct Batch { std::mutex m; std::condition_variable c; uint32_t left; } b;
    b.left = n;
    {
      std::lock_guard<std::mutex> l(mu_);
      for (uint32_t i = 0; i < n; ++i)
        q_.push_back([&b, &f, i] {
          f(i);
          std::lock_guard<std::mutex> lb(b.m);
          if (--b.left == 0) b.c.notify_all();
        });
    }
    cv_.notify_all();
    std::unique_lock<std::mutex> lb(b.m);
    b.c.wait(lb, [&] { return b.left == 0; });
  }

 private:
  explicit ShardWorkers(int n) {
    for (int i = 0; i < n; ++i)
      std::thread([this] {
        for (;;) {
          std::function<void()> job;
          {
            std::unique_lock<std::mutex> l(mu_);
            cv_.wait(l, [&] { return !q_.empty(); });
            job = std::move(q_.front());
            q_.pop_front();
          }
          job();
        }
      }).detach();
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
};

static void run_parallel(uint32_t n, const std::function<void(uint32_t)>& f) { ShardWorkers::get().run(n, f); }

// One batch over several shards / segments / namespaces of one logical index
// (SURVEY.md §8b fg_search_sharded, §8e).  The shards of each device run as ONE
// multi-snapshot plan (fg_plan_create_multi: one upload, one launch per kernel,
// one shared score-only threshold per query); every shard's top-k lists land in
// gathered buffers on the first shard's device -- directly, or over xGMI
// (hipMemcpyPeerAsync) from another device -- and k_merge_rank merges them
// there into (score desc, shard asc, doc asc): tantivy's merge_fruits over
// DocAddress (segment_ord, doc).  Everything runs on the calling thread's
// per-thread streams.
}  // extern "C"
namespace fgh {
SearchTrace& search_trace() {
  static SearchTrace t;
  return t;
}
}  // namespace fgh
extern "C" {

int fg_search_trace(int enable, double* out_ms, uint32_t n, uint64_t* calls) {
  fgh::SearchTrace& t = fgh::search_trace();
  if (out_ms)
    for (uint32_t i = 0; i < n; ++i) out_ms[i] = i < fgh::kNumPhases ? (double)t.ns[i].exchange(0) * 1e-6 : 0.0;
  if (calls) *calls = t.calls.exchange(0);
  if (enable >= 0) t.on.store(enable ? 1 : 0);
  return FG_OK;
}

int fg_search_sharded(fg_ctx* ctx, fg_index* const* shards, uint32_t n_shards, const fg_query_batch* q, uint32_t k,
                      float* out_score, uint32_t* out_doc, uint32_t* out_shard, uint32_t* out_n) {
  if (!shards || n_shards == 0 || n_shards > FG_MAX_SEGMENTS || !q || k == 0 || !out_score || !out_doc || !out_n)
    return fail(FG_EINVAL, "bad arguments");
  for (uint32_t s = 0; s < n_shards; ++s) {
    if (!shards[s]) return fail(FG_EINVAL, "NULL shard");
    if (ctx && std::find(ctx->devs.begin(), ctx->devs.end(), shards[s]->dev) == ctx->devs.end())
      return fail(FG_EINVAL, "a shard lives on a device outside the context");
  }
  const uint32_t nq = q->n_queries;
  if (nq == 0) return FG_OK;
  if (k > FG_MAX_K) return fail(FG_EUNSUPPORTED, "k > FG_MAX_K");
  // ---- gathered lists + merged output on the first shard's device (its pool)
  const int dev0 = shards[0]->dev;
  const size_t nk = (size_t)nq * k;
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t g_s = al(4 * nk * n_shards), g_n = al(4ull * nq * n_shards), o_k = al(4 * nk), o_n = al(4ull * nq);
  const size_t total = 2 * g_s + g_n + 3 * o_k + o_n;
  size_t got = 0;
  HIPCHK(hipSetDevice(dev0));
  char* base = static_cast<char*>(shards[0]->pool->get(total, &got));
  if (!base) return fail(FG_EOOM, "hipMalloc of the shard merge buffers failed");
  float* gs = reinterpret_cast<float*>(base);
  uint32_t* gd = reinterpret_cast<uint32_t*>(base + g_s);
  uint32_t* gn = reinterpret_cast<uint32_t*>(base + 2 * g_s);
  float* ms = reinterpret_cast<float*>(base + 2 * g_s + g_n);
  uint32_t* md = reinterpret_cast<uint32_t*>(base + 2 * g_s + g_n + o_k);
  uint32_t* msh = reinterpret_cast<uint32_t*>(base + 2 * g_s + g_n + 2 * o_k);
  uint32_t* mn = reinterpret_cast<uint32_t*>(base + 2 * g_s + g_n + 3 * o_k);
  // the shards of each device, in shard order
  std::vector<int> gdev;
  std::vector<std::vector<uint32_t>> groups;
  for (uint32_t s = 0; s < n_shards; ++s) {
    const auto it = std::find(gdev.begin(), gdev.end(), shards[s]->dev);
    if (it == gdev.end()) {
      gdev.push_back(shards[s]->dev);
      groups.push_back({s});
    } else {
      groups[it - gdev.begin()].push_back(s);
    }
  }
  const size_t ng = groups.size();
  // every shard on the first device: the calling thread's high-priority stream
  // there, so a search's kernels are dispatched ahead of a commit's segment
  // build and the merger's; else per-thread streams
  const hipStream_t hs = ng == 1 && gdev[0] == dev0 ? search_stream(dev0) : hipStreamPerThread;
  // a batch run in two halves: the second half on the thread's second stream
  // there, so its kernels start while the first half's drain
  const hipStream_t hs2 = ng == 1 && gdev[0] == dev0 ? search_stream(dev0, true) : hs;
  uint32_t split = 0;  // the second half's first query (0: one part)
  bool merged = false;  // the plan's merged select already wrote ms / md / msh / mn
  std::vector<std::unique_ptr<fg_plan>> plans(ng), parts;
  std::vector<hipEvent_t> evs(ng, nullptr);
  // teardown (also on error returns): every device's stream drained, then the
  // events, the plans and the buffers
  struct Back {
    const std::vector<int>& dv; int d0; fg_index* ix0; void* p; size_t n; std::vector<hipEvent_t>& ev; hipStream_t s0,
        s1;
    ~Back() {
      for (size_t g = 0; g < dv.size(); ++g) {
        (void)hipSetDevice(dv[g]);
        (void)hipStreamSynchronize(hipStreamPerThread);
        if (ev[g]) (void)hipEventDestroy(ev[g]);
      }
      (void)hipSetDevice(d0);
      (void)hipStreamSynchronize(s0);
      if (s1 != s0) (void)hipStreamSynchronize(s1);
      ix0->pool->put(p, n);
    }
  } back{gdev, dev0, shards[0], base, got, evs, hs, hs2};
  static const bool trace_env = getenv("FUGU_SHARD_TRACE") != nullptr;
  fgh::SearchTrace& st = fgh::search_trace();
  const bool trace = trace_env || st.enabled();
  auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double t_0 = trace ? now() : 0.0;
  double t_plan = 0.0;
  for (size_t g = 0; g < ng; ++g) {
    const std::vector<uint32_t>& gi = groups[g];
    const uint32_t S = (uint32_t)gi.size();
    std::vector<fg_index*> ixs(S);
    for (uint32_t j = 0; j < S; ++j) ixs[j] = shards[gi[j]];
    fg_plan* p = nullptr;
    // every shard on dev0 in one plan, a batch: its merged select writes the
    // merged lists directly (no per-shard lists, no k_merge_rank); a small batch
    // keeps one final select per shard (more workgroups in parallel: a single
    // query over 8 segments 0.070 vs 0.077 ms p50): the merged select from
    // batches of merged_min queries (tools/multi_ab.py, round 3).  A batch of
    // 2 x kPipeMin queries or more runs as two halves, the second planned on the
    // host while the first one's kernels run (C4, 1024 queries: one plan 478K
    // q/s, two halves 560K, four quarters 487K, 256 + 768 queries 513K)
    constexpr uint32_t merged_min = 256u, kPipeMin = 256u;
    uint64_t docs = 0;
    for (fg_index* x : ixs) docs += x->n_docs;
    if (ng == 1 && gdev[0] == dev0 && S > 1 && docs <= 0xFFFFFFFFull && nq >= merged_min) {
      const uint32_t np = nq >= 2 * kPipeMin ? 2u : 1u;
      for (uint32_t i = 0; i < np; ++i) {
        const uint32_t b = (uint32_t)((uint64_t)nq * i / np), e = (uint32_t)((uint64_t)nq * (i + 1) / np);
        fg_query_batch qi = *q;  // queries [b, e): the same term arrays, offsets from q_off[b]
        qi.n_queries = e - b;
        qi.q_off = q->q_off + b;
        if (q->f_off) qi.f_off = q->f_off + b;
        const double t_p = trace ? now() : 0.0;
        fg_plan* pi = nullptr;
        const hipStream_t si = i == 0 ? hs : hs2;
        if (i > 0) split = b;
        if (int rc = plan_create_multi(ixs.data(), S, &qi, k, &pi, false, si)) return rc;
        parts.emplace_back(pi);
        if (trace) t_plan += now() - t_p;
        if (int rc = execute_impl(pi, si, ms + (size_t)b * k, md + (size_t)b * k, mn + b, msh + (size_t)b * k)) return rc;
      }
      merged = true;
      break;
    }
    // the upload is queued on this thread's stream of the device, ahead of the
    // execute on the same stream: no host round trip
    const double t_p = trace ? now() : 0.0;
    if (int rc = plan_create_multi(ixs.data(), S, q, k, &p, false, hs)) {
      if (n_shards == 1) return rc;
      const std::string e = fg_last_error();
      return fail(rc, "device %d: %s", gdev[g], e.c_str());
    }
    plans[g].reset(p);
    if (trace) t_plan += now() - t_p;
    // lists straight into the gathered buffers when the group's shards are
    // consecutive and on dev0 ([S][nq][k] is the gathered layout)
    const bool direct = gdev[g] == dev0 && gi.back() - gi.front() + 1 == S;
    const size_t s0 = gi.front();
    if (int rc = direct ? fg_plan_execute(p, hs, gs + s0 * nk, gd + s0 * nk, gn + s0 * nq)
                        : fg_plan_execute(p, hs, nullptr, nullptr, nullptr))
      return rc;
    if (!direct) {
      for (uint32_t j = 0; j < S; ++j) {
        const size_t s = gi[j];
        if (gdev[g] == dev0) {
          HIPCHK(hipMemcpyAsync(gs + s * nk, p->own_score + j * nk, 4 * nk, hipMemcpyDeviceToDevice, hs));
          HIPCHK(hipMemcpyAsync(gd + s * nk, p->own_doc + j * nk, 4 * nk, hipMemcpyDeviceToDevice, hs));
          HIPCHK(hipMemcpyAsync(gn + s * nq, p->own_n + (size_t)j * nq, 4ull * nq, hipMemcpyDeviceToDevice,
                                hs));
        } else {
          HIPCHK(hipMemcpyPeerAsync(gs + s * nk, dev0, p->own_score + j * nk, gdev[g], 4 * nk, hs));
          HIPCHK(hipMemcpyPeerAsync(gd + s * nk, dev0, p->own_doc + j * nk, gdev[g], 4 * nk, hs));
          HIPCHK(hipMemcpyPeerAsync(gn + s * nq, dev0, p->own_n + (size_t)j * nq, gdev[g], 4ull * nq,
                                    hs));
        }
      }
    }
    if (gdev[g] != dev0) {
      HIPCHK(hipEventCreateWithFlags(&evs[g], hipEventDisableTiming));
      HIPCHK(hipEventRecord(evs[g], hs));
    }
  }
  const double t_run = trace ? now() : 0.0;
  HIPCHK(hipSetDevice(dev0));
  for (hipEvent_t e : evs)
    if (e) HIPCHK(hipStreamWaitEvent(hs, e, 0));
  if (!merged) HIPCHK(fg::launch_merge(n_shards, nq, k, gs, gd, gn, ms, md, msh, mn, hs));
  const bool two = split && hs2 != hs;
  if (trace_env) {
    HIPCHK(hipStreamSynchronize(hs));
    if (two) HIPCHK(hipStreamSynchronize(hs2));
    fprintf(stderr, "[fg_search_sharded] nq %u shards %u devices %zu merged %d: plan %.3f launch %.3f kernels+merge %.3f ms\n",
            nq, n_shards, ng, (int)merged, t_plan, t_run - t_0 - t_plan, now() - t_run);
  }
  // the search trace's phases: planning, launches, then the wait for the hits
  struct PhaseOut {
    fgh::SearchTrace& st; bool on; double t0, tp, tr; double (*clk)();
    ~PhaseOut() {
      if (!on) return;
      st.add(fgh::kPhPlan, (uint64_t)(tp * 1e6));
      st.add(fgh::kPhLaunch, (uint64_t)((tr - t0 - tp) * 1e6));
      st.add(fgh::kPhWait, (uint64_t)((clk() - tr) * 1e6));
    }
  } phase_out{st, st.enabled(), t_0, t_plan, t_run, +now};
  // the merged lists are consecutive: one D2H into a pinned buffer (small batches)
  const size_t span = 3 * o_k + 4ull * nq;
  if (span <= (4ull << 20)) {
    PinnedLease pin(*shards[0]->pinned, span);
    if (pin.p && two) {
      // each half's hits copied back on its own stream, the first half's copied
      // out of the pinned buffer while the second half's kernels run
      char* h = static_cast<char*>(pin.p);
      const char* d = reinterpret_cast<const char*>(ms);
      for (int half = 0; half < 2; ++half) {
        const hipStream_t sh = half ? hs2 : hs;
        const size_t q0 = half ? split : 0, q1 = half ? nq : split;
        for (size_t a = 0; a < 3; ++a)
          HIPCHK(hipMemcpyAsync(h + a * o_k + 4 * q0 * k, d + a * o_k + 4 * q0 * k, 4 * (q1 - q0) * k,
                                hipMemcpyDeviceToHost, sh));
        HIPCHK(hipMemcpyAsync(h + 3 * o_k + 4 * q0, d + 3 * o_k + 4 * q0, 4 * (q1 - q0), hipMemcpyDeviceToHost, sh));
      }
      for (int half = 0; half < 2; ++half) {
        HIPCHK(hipStreamSynchronize(half ? hs2 : hs));
        const size_t q0 = half ? split : 0, q1 = half ? nq : split;
        std::memcpy(out_score + q0 * k, h + 4 * q0 * k, 4 * (q1 - q0) * k);
        std::memcpy(out_doc + q0 * k, h + o_k + 4 * q0 * k, 4 * (q1 - q0) * k);
        if (out_shard) std::memcpy(out_shard + q0 * k, h + 2 * o_k + 4 * q0 * k, 4 * (q1 - q0) * k);
        std::memcpy(out_n + q0, h + 3 * o_k + 4 * q0, 4 * (q1 - q0));
      }
      return FG_OK;
    }
    if (two) HIPCHK(hipStreamSynchronize(hs2));  // (no pinned buffer: one copy on hs)
    if (pin.p) {
      HIPCHK(hipMemcpyAsync(pin.p, ms, span, hipMemcpyDeviceToHost, hs));
      HIPCHK(hipStreamSynchronize(hs));
      const char* h = static_cast<const char*>(pin.p);
      std::memcpy(out_score, h, 4 * nk);
      std::memcpy(out_doc, h + o_k, 4 * nk);
      if (out_shard) std::memcpy(out_shard, h + 2 * o_k, 4 * nk);
      std::memcpy(out_n, h + 3 * o_k, 4ull * nq);
      return FG_OK;
    }
  }
  if (two) HIPCHK(hipStreamSynchronize(hs2));
  HIPCHK(hipMemcpyAsync(out_score, ms, 4 * nk, hipMemcpyDeviceToHost, hs));
  HIPCHK(hipMemcpyAsync(out_doc, md, 4 * nk, hipMemcpyDeviceToHost, hs));
  if (out_shard) HIPCHK(hipMemcpyAsync(out_shard, msh, 4 * nk, hipMemcpyDeviceToHost, hs));
  HIPCHK(hipMemcpyAsync(out_n, mn, 4ull * nq, hipMemcpyDeviceToHost, hs));
  HIPCHK(hipStreamSynchronize(hs));
  return FG_OK;
}

}  // extern "C"
