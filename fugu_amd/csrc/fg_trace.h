// Search phase trace shared by the device library (fugu.cpp) and the host
// mirror (host.cpp, plain C++: no HIP headers here).
#pragma once
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

namespace fgh {

// Phase times of searches while enabled (fg_search_trace): cumulative ns per
// phase over every call of the process, read and reset together.  Off: one
// relaxed load per phase boundary.
enum SearchPhase : uint32_t {
  kPhParse = 0,  // fg_db_search*: parse + facet clauses + dictionary lookups
  kPhPlan,       // fg_search_sharded: host planning of the snapshots + the upload queued
  kPhLaunch,     // fg_search_sharded: kernel launches queued
  kPhWait,       // fg_search_sharded: kernels + merge + D2H until the hits are on the host
  kPhFetch,      // GET /search JSON: stored fields of the hits + serialization
  kPhTotal,      // fg_db_search*: the whole call (without the JSON phase)
  kNumPhases
};
struct SearchTrace {
  std::atomic<int> on{0};
  std::atomic<uint64_t> ns[kNumPhases] = {};
  std::atomic<uint64_t> calls{0};
  bool enabled() const { return on.load(std::memory_order_relaxed) != 0; }
  void add(SearchPhase p, uint64_t v) { ns[p].fetch_add(v, std::memory_order_relaxed); }
};
SearchTrace& search_trace();
inline uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

// FUGU_COMMIT_TRACE: device memory releases (the reaper's frees) on stderr as
// "[fg free] <what> <ms> ms @<end on the steady clock, ms>", like the commit phases
inline bool commit_trace_on() {
  static const bool on = getenv("FUGU_COMMIT_TRACE") != nullptr;
  return on;
}
inline void trace_span(const char* tag, const char* what, uint64_t t0_ns) {
  const uint64_t t1 = now_ns();
  fprintf(stderr, "[fg %s] %-28s %9.2f ms @%.3f\n", tag, what, (double)(t1 - t0_ns) * 1e-6, (double)t1 * 1e-6);
}

}  // namespace fgh
