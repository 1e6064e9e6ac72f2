// Host parallel loops over a persistent helper pool (the pool: fugu.cpp).
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>

namespace fgh {

// A persistent pool of helper threads (fugu.cpp): starting threads per call
// cost a small build (a commit's 1000 docs) several ms over its parallel loops.
void pool_post(std::function<void()> job);

// work(t) on the calling thread (t = 0) and on up to `helpers` pool threads
// (t = 1, 2, ...) that start before the caller's own work(0) returns; then
// waits for the helpers that did start.  A helper queued behind others never
// holds the caller up (nor can nested calls deadlock): the caller does all the
// work alone when the pool is busy.
struct HelpJoin {
  std::mutex m;
  std::condition_variable c;
  int active = 0;
  bool closed = false;
  std::atomic<int> ids{1};
};
template <class W>
void run_helped(int helpers, W&& work) {
  auto j = std::make_shared<HelpJoin>();
  for (int h = 0; h < helpers; ++h)
    pool_post([j, &work] {
      {
        std::lock_guard<std::mutex> l(j->m);
        if (j->closed) return;
        ++j->active;
      }
      work(j->ids.fetch_add(1));
      {
        std::lock_guard<std::mutex> l(j->m);
        --j->active;
      }
      j->c.notify_all();
    });
  work(0);
  std::unique_lock<std::mutex> l(j->m);
  j->closed = true;
  j->c.wait(l, [&] { return j->active == 0; });
}

// f(r, begin, end) over `threads` equal ranges r of [0, n), each run once by
// the caller or a pool helper
template <class F>
void parallel_ranges(uint32_t n, int threads, F&& f) {
  if (threads <= 1 || n < 1024) { f(0, 0u, n); return; }
  const uint32_t step = (n + threads - 1) / threads;
  std::atomic<int> next{0};
  run_helped(threads - 1, [&](int) {
    for (int r; (r = next.fetch_add(1)) < threads;) {
      const uint32_t b = std::min<uint64_t>((uint64_t)r * step, n), e = std::min<uint64_t>((uint64_t)(r + 1) * step, n);
      f(r, b, e);
    }
  });
}

// Dynamic schedule over [0, n) in chunks of `grain` (per-term loops: Zipf term
// ids put most postings in the first terms, so a static split leaves one
// thread with nearly all the work).  f(thread, begin, end), thread < threads.
template <class F>
void parallel_dynamic(uint32_t n, int threads, uint32_t grain, F&& f) {
  if (threads <= 1 || n <= grain) { f(0, 0u, n); return; }
  threads = (int)std::min<uint64_t>((uint64_t)threads, ((uint64_t)n + grain - 1) / grain);  // no more than chunks
  std::atomic<uint64_t> next{0};
  run_helped(threads - 1, [&](int t) {
    for (;;) {
      const uint64_t b = next.fetch_add(grain);
      if (b >= n) break;
      f(t, (uint32_t)b, (uint32_t)std::min<uint64_t>(n, b + grain));
    }
  });
}

}  // namespace fgh
