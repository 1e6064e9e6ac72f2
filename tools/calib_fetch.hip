// HBM counter calibration for gfx950 (MI355X_MICROARCH.md §HBM: "other access
// widths are uncalibrated: calibrate on a known byte count in your own access
// pattern").  Under rocprofv3 --pmc each launch below is compared with its known
// byte count / request count:
//   stream4 / stream16   1 GiB read once, coalesced, 4 B and 16 B per lane
//   gather_lines         one 4-B load in each 128-B line of a 4 GiB table, every line
//                        exactly once, in a scattered (bijective hash) order: the
//                        access shape of k_conj's dense-table / directory probes
//                        (single dwords far apart), with a known line count
//   gather_random        uniformly random 4-B loads over the 4 GiB table (k_conj-like)
// k_conj's traffic is dominated by such scattered single-dword gathers, so the
// counter read on them -- not only on streams -- decides how FETCH_SIZE and the
// size-aware TCC_EA0_RDREQ_DRAM_32B translate into HBM bytes (tools/pmc_traffic.py).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void stream4(const uint32_t* __restrict__ a, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc ^= a[i];
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void stream16(const uint4* __restrict__ a, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// line index i -> (i * odd) mod 2^k: a bijection over the 2^k lines
__global__ void gather_lines(const uint32_t* __restrict__ a, uint64_t n_lines, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n_lines; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t line = (i * 0x9E3779B97F4A7C15ull) & (n_lines - 1);
    acc ^= a[line * 32 + (i & 31)];  // one dword of the 128-B line
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void gather_random(const uint32_t* __restrict__ a, uint64_t n_words, uint64_t n_loads, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n_loads; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = i + 0x9E3779B97F4A7C15ull;  // SplitMix64 finaliser
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    acc ^= a[z & (n_words - 1)];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const size_t stream_bytes = 1ull << 30, table_bytes = 4ull << 30;
  const uint64_t n_lines = table_bytes / 128, n_rand = 1ull << 25;
  uint32_t *a, *out;
  if (hipMalloc(&a, table_bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  if (hipMemset(a, 1, table_bytes) != hipSuccess) return 1;
  for (int r = 0; r < 3; ++r) {
    stream4<<<4096, 256>>>(a, stream_bytes / 4, out);
    stream16<<<4096, 256>>>(reinterpret_cast<const uint4*>(a), stream_bytes / 16, out);
    gather_lines<<<8192, 256>>>(a, n_lines, out);
    gather_random<<<8192, 256>>>(a, table_bytes / 4, n_rand, out);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("calib: stream4/stream16 read exactly %zu bytes; gather_lines reads one dword in each of %llu 128-B lines "
         "(4 GiB table); gather_random makes %llu random dword loads\n",
         stream_bytes, (unsigned long long)n_lines, (unsigned long long)n_rand);
  (void)hipFree(a);
  (void)hipFree(out);
  return 0;
}
