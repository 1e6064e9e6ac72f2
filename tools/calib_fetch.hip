// FETCH_SIZE calibration for gfx950 (MI355X_MICROARCH.md §HBM: "other access
// widths are uncalibrated: calibrate on a known byte count in your own access
// pattern").  Streams a 1 GiB buffer once per kernel with the load widths the
// search kernels use (4 B and 16 B per lane, coalesced), so rocprofv3
// --pmc FETCH_SIZE can be compared against the exact byte count.
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

int main() {
  const size_t bytes = 1ull << 30;
  uint32_t *a, *out;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  if (hipMemset(a, 1, bytes) != hipSuccess) return 1;
  for (int r = 0; r < 3; ++r) {
    stream4<<<4096, 256>>>(a, bytes / 4, out);
    stream16<<<4096, 256>>>(reinterpret_cast<const uint4*>(a), bytes / 16, out);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("calib: each launch reads exactly %zu bytes\n", bytes);
  (void)hipFree(a);
  (void)hipFree(out);
  return 0;
}
