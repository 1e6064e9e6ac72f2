// Stall probe: what makes a small, latency-bound search on its own
// high-priority stream wait while other work shares the GPU?
//
// A "search" thread runs back to back: one small streaming kernel (a
// k_disj-sized batch of one: 512 workgroups over 32 MiB) on a high-priority
// stream, a 4 KiB D2H into pinned memory, hipStreamSynchronize -- and records
// host-in to host-out latency.  A "background" thread meanwhile runs ONE kind
// of work per phase, each the shape of something a commit does
// (fg_db_commit: scoring kernels, allocations, uploads, read-backs, device
// drains).  Per phase: p50 / p99 / max of the search latency, as one JSON line.
//
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -o tools/stall_probe tools/stall_probe.hip -lpthread
//   tools/stall_probe [seconds per phase] [phase names...]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// the search: a grid-stride sum over n u32, one u32 per workgroup out
__global__ __launch_bounds__(256) void k_search(const uint32_t* __restrict__ a, size_t n, uint32_t* out) {
  uint32_t s = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i];
  __shared__ uint32_t red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

// background: every workgroup streams its share of n u32 `reps` times
__global__ __launch_bounds__(256) void k_stream(const uint32_t* __restrict__ a, size_t n, int reps, uint32_t* out) {
  uint32_t s = 0;
  for (int r = 0; r < reps; ++r)
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i] ^ r;
  if (s == 0x12345678u) out[blockIdx.x] = s;
}

// background: short workgroups, each one u32 per thread of one 1024-u32 slice per rep
__global__ __launch_bounds__(256) void k_short(const uint32_t* __restrict__ a, size_t n, int reps, uint32_t* out) {
  uint32_t s = 0;
  const size_t base = (size_t)blockIdx.x * 1024;
  for (int r = 0; r < reps; ++r)
    for (int j = 0; j < 4; ++j) {
      const size_t i = base + j * 256 + threadIdx.x;
      if (i < n) s += a[i] ^ r;
    }
  if (s == 0x12345678u) out[blockIdx.x & 1023] = s;
}

// background: few long-lived workgroups (one per "term", like k_ktop on a
// long list), each spinning `us` microseconds on the 100 MHz clock with
// `lds` bytes of LDS held
template <int LDS>
__global__ __launch_bounds__(256) void k_long(uint64_t ticks, uint32_t* out) {
  __shared__ uint32_t buf[LDS / 4 > 0 ? LDS / 4 : 1];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = threadIdx.x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    x = x * 1664525u + 1013904223u;
    if (LDS) buf[(x >> 8) % (LDS / 4)] = x;
  }
  __syncthreads();
  if (x == 0x12345678u) out[blockIdx.x] = x + (LDS ? buf[0] : 0);
}

struct Lat {
  std::vector<double> v;
  void add(double x) { v.push_back(x); }
  double q(double p) {
    if (v.empty()) return 0;
    std::vector<double> s = v;
    std::sort(s.begin(), s.end());
    return s[std::min(s.size() - 1, (size_t)(p * s.size()))];
  }
};

int main(int argc, char** argv) {
  const double phase_s = argc > 1 ? atof(argv[1]) : 2.0;
  std::vector<std::string> phases;
  for (int i = 2; i < argc; ++i) phases.push_back(argv[i]);
  if (phases.empty())
    phases = {"idle",        "stream",         "stream_masked", "stream_lowprio", "long",          "long_lds",
              "long_masked", "long_lds_masked", "malloc_free",  "host_malloc",    "h2d_pinned",    "h2d_pageable",
              "d2h_pinned",  "devsync",        "memset",        "malloc_async",   "stream_create", "idle"};
  CK(hipSetDevice(0));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int n_cu = prop.multiProcessorCount;
  int least = 0, greatest = 0;
  CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  hipStream_t ss, bs, bs_lo, bs_mask;
  CK(hipStreamCreateWithPriority(&ss, hipStreamNonBlocking, greatest));
  CK(hipStreamCreateWithFlags(&bs, hipStreamNonBlocking));
  CK(hipStreamCreateWithPriority(&bs_lo, hipStreamNonBlocking, least));
  std::vector<uint32_t> mask((n_cu + 31) / 32, 0u);
  const int off = n_cu / 4;  // 3/4 of the CUs, the left-out ones spread evenly
  for (int c = 0; c < n_cu; ++c)
    if ((uint64_t)(c + 1) * off / n_cu == (uint64_t)c * off / n_cu) mask[c / 32] |= 1u << (c % 32);
  CK(hipExtStreamCreateWithCUMask(&bs_mask, (uint32_t)mask.size(), mask.data()));
  // several background streams at once (a commit rescores 8 segments side by side)
  hipStream_t bs8[8], bs8_lo[8];
  for (int i = 0; i < 8; ++i) {
    CK(hipStreamCreateWithFlags(&bs8[i], hipStreamNonBlocking));
    CK(hipStreamCreateWithPriority(&bs8_lo[i], hipStreamNonBlocking, least));
  }

  const size_t n_search = 8u << 20;  // 32 MiB
  const size_t n_bg = 1u << 30;      // 4 GiB
  uint32_t *d_s, *d_out, *d_bg, *d_bg_out;
  CK(hipMalloc(&d_s, n_search * 4));
  CK(hipMalloc(&d_out, 1 << 20));
  CK(hipMalloc(&d_bg, n_bg * 4));
  CK(hipMalloc(&d_bg_out, 1 << 20));
  CK(hipMemset(d_s, 1, n_search * 4));
  CK(hipMemset(d_bg, 2, n_bg * 4));
  uint32_t* h_res;
  CK(hipHostMalloc(&h_res, 4096, hipHostMallocDefault));
  const size_t cp_bytes = 256u << 20;
  void *h_pin, *d_cp;
  CK(hipHostMalloc(&h_pin, cp_bytes, hipHostMallocDefault));
  void* h_page = malloc(cp_bytes);
  memset(h_page, 3, cp_bytes);
  CK(hipMalloc(&d_cp, cp_bytes));
  CK(hipDeviceSynchronize());

  for (const std::string& ph : phases) {
    std::atomic<bool> stop{false};
    std::atomic<long> bg_ops{0};
    std::thread bg([&] {
      CK(hipSetDevice(0));
      const uint64_t ticks_5ms = 500000;  // 100 MHz
      while (!stop.load()) {
        if (ph == "idle") {
          std::this_thread::sleep_for(std::chrono::milliseconds(1));
          continue;
        } else if (ph == "stream" || ph == "stream_masked" || ph == "stream_lowprio") {
          hipStream_t s = ph == "stream" ? bs : ph == "stream_masked" ? bs_mask : bs_lo;
          // ~5 ms of HBM streaming per launch, 4 launches queued
          for (int i = 0; i < 4; ++i) k_stream<<<4096, 256, 0, s>>>(d_bg, n_bg, 5, d_bg_out);
          CK(hipStreamSynchronize(s));
        } else if (ph == "short" || ph == "short_lowprio") {
          hipStream_t s = ph == "short" ? bs : bs_lo;
          // the same ~5 ms of streaming per launch as "stream", in 1M short workgroups
          for (int i = 0; i < 4; ++i) k_short<<<(unsigned)(n_bg / 1024), 256, 0, s>>>(d_bg, n_bg, 5, d_bg_out);
          CK(hipStreamSynchronize(s));
        } else if (ph == "short8" || ph == "short8_lowprio" || ph == "short2_lowprio" || ph == "short4_lowprio") {
          // short-workgroup kernels on several streams at once, 1/N of the work each
          const int N = ph == "short2_lowprio" ? 2 : ph == "short4_lowprio" ? 4 : 8;
          hipStream_t* v = ph == "short8" ? bs8 : bs8_lo;
          for (int i = 0; i < 4; ++i)
            for (int j = 0; j < N; ++j)
              k_short<<<(unsigned)(n_bg / 1024 / N), 256, 0, v[j]>>>(d_bg + j * (n_bg / N), n_bg / N, 5, d_bg_out);
          for (int j = 0; j < N; ++j) CK(hipStreamSynchronize(v[j]));
        } else if (ph == "long_half" || ph == "long_half_lowprio") {
          hipStream_t s = ph == "long_half" ? bs : bs_lo;
          // 4 workgroups per CU (half the wave slots), each 5 ms
          k_long<0><<<4 * n_cu, 256, 0, s>>>(ticks_5ms, d_bg_out);
          CK(hipStreamSynchronize(s));
        } else if (ph == "spin_short_lowprio") {
          // 100 us workgroups, 16 per CU queued per launch round, low priority
          k_long<0><<<64 * n_cu, 256, 0, bs_lo>>>(10000, d_bg_out);
          CK(hipStreamSynchronize(bs_lo));
        } else if (ph == "malloc_async_keep" || ph == "malloc_async_small") {
          static bool once = false;
          if (!once && ph == "malloc_async_keep") {
            hipMemPool_t pool;
            CK(hipDeviceGetDefaultMemPool(&pool, 0));
            uint64_t thr = ~0ull;
            CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr));
            once = true;
          }
          const size_t b = ph == "malloc_async_small" ? (4u << 20) : (256u << 20);
          void* p;
          CK(hipMallocAsync(&p, b, bs));
          k_stream<<<64, 256, 0, bs>>>((const uint32_t*)p, b / 4 < (1u << 20) ? b / 4 : (1u << 20), 1, d_bg_out);
          CK(hipFreeAsync(p, bs));
          CK(hipStreamSynchronize(bs));
        } else if (ph == "long" || ph == "long_masked") {
          hipStream_t s = ph == "long" ? bs : bs_mask;
          // 8 workgroups per CU, each 5 ms
          k_long<0><<<8 * n_cu, 256, 0, s>>>(ticks_5ms, d_bg_out);
          CK(hipStreamSynchronize(s));
        } else if (ph == "long_lds" || ph == "long_lds_masked") {
          hipStream_t s = ph == "long_lds" ? bs : bs_mask;
          // 2 workgroups per CU holding 64 KiB of LDS each (the CU's LDS full)
          k_long<65536><<<2 * n_cu, 256, 0, s>>>(ticks_5ms, d_bg_out);
          CK(hipStreamSynchronize(s));
        } else if (ph == "malloc_free") {
          void* p;
          CK(hipMalloc(&p, 256u << 20));
          k_stream<<<64, 256, 0, bs>>>((const uint32_t*)p, 1 << 20, 1, d_bg_out);
          CK(hipFree(p));
        } else if (ph == "host_malloc") {
          void* p;
          CK(hipHostMalloc(&p, 24u << 20, hipHostMallocDefault));
          memset(p, 0, 24u << 20);
          CK(hipHostFree(p));
        } else if (ph == "h2d_pinned") {
          CK(hipMemcpyAsync(d_cp, h_pin, cp_bytes, hipMemcpyHostToDevice, bs));
          CK(hipStreamSynchronize(bs));
        } else if (ph == "h2d_pageable") {
          CK(hipMemcpyAsync(d_cp, h_page, cp_bytes, hipMemcpyHostToDevice, bs));
          CK(hipStreamSynchronize(bs));
        } else if (ph == "d2h_pinned") {
          CK(hipMemcpyAsync(h_pin, d_cp, cp_bytes, hipMemcpyDeviceToHost, bs));
          CK(hipStreamSynchronize(bs));
        } else if (ph == "devsync") {
          k_stream<<<4096, 256, 0, bs>>>(d_bg, n_bg / 8, 1, d_bg_out);
          CK(hipDeviceSynchronize());
        } else if (ph == "memset") {
          CK(hipMemsetAsync(d_bg, 0, n_bg, bs));
          CK(hipStreamSynchronize(bs));
        } else if (ph == "malloc_async") {
          void* p;
          CK(hipMallocAsync(&p, 256u << 20, bs));
          k_stream<<<64, 256, 0, bs>>>((const uint32_t*)p, 1 << 20, 1, d_bg_out);
          CK(hipFreeAsync(p, bs));
          CK(hipStreamSynchronize(bs));
        } else if (ph == "stream_create") {
          hipStream_t s;
          CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
          k_stream<<<64, 256, 0, s>>>(d_bg, 1 << 20, 1, d_bg_out);
          CK(hipStreamSynchronize(s));
          CK(hipStreamDestroy(s));
        } else {
          fprintf(stderr, "unknown phase %s\n", ph.c_str());
          exit(2);
        }
        bg_ops.fetch_add(1);
      }
    });
    Lat lat;
    const double t_end = now_ms() + phase_s * 1000.0;
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    while (now_ms() < t_end) {
      const double t0 = now_ms();
      k_search<<<512, 256, 0, ss>>>(d_s, n_search, d_out);
      CK(hipMemcpyAsync(h_res, d_out, 4096, hipMemcpyDeviceToHost, ss));
      CK(hipStreamSynchronize(ss));
      lat.add(now_ms() - t0);
    }
    stop.store(true);
    bg.join();
    CK(hipDeviceSynchronize());
    printf("{\"phase\": \"%s\", \"searches\": %zu, \"p50_ms\": %.4f, \"p90_ms\": %.4f, \"p99_ms\": %.4f, "
           "\"max_ms\": %.3f, \"bg_ops\": %ld}\n",
           ph.c_str(), lat.v.size(), lat.q(0.5), lat.q(0.9), lat.q(0.99), lat.q(1.0), bg_ops.load());
    fflush(stdout);
  }
  return 0;
}
