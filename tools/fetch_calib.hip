// FETCH_SIZE calibration on gfx950 for the access widths the scheduler's kernels use
// (MI355X_MICROARCH.md: only 16-B-per-lane streaming reads are calibrated, at 1/2).
// Each kernel reads a 256 MiB buffer once with one pattern; run under
//   rocprofv3 --pmc FETCH_SIZE -- tools/bin/fetch_calib
// and divide FETCH_SIZE x 1024 by the bytes of the 64-B lines the pattern touches
// (printed here per kernel). build: hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/bin/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHK(x)                                                                     \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

// contiguous, 16 B per lane
__global__ void calib_wide16(const uint4* p, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}
// contiguous, 8 B per lane (the SoA int64 totals, one node per lane)
__global__ void calib_cont8(const uint64_t* p, size_t n, uint32_t* out) {
  uint64_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if ((uint32_t)acc == 0x9e3779b9u) out[0] = (uint32_t)acc;
}
// contiguous, 4 B per lane
__global__ void calib_cont4(const uint32_t* p, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if (acc == 0x9e3779b9u) out[0] = acc;
}
// one 8-B load per 64-B line (a gather: a bitmap word, a node's total)
__global__ void calib_gather8_64(const uint64_t* p, size_t lines, uint32_t* out) {
  uint64_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < lines; i += (size_t)gridDim.x * blockDim.x)
    acc ^= p[i * 8];
  if ((uint32_t)acc == 0x9e3779b9u) out[0] = (uint32_t)acc;
}
// one 8-B load per 128-B pair of lines
__global__ void calib_gather8_128(const uint64_t* p, size_t pairs, uint32_t* out) {
  uint64_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < pairs; i += (size_t)gridDim.x * blockDim.x)
    acc ^= p[i * 16];
  if ((uint32_t)acc == 0x9e3779b9u) out[0] = (uint32_t)acc;
}
// agent-scope (sc1) 8-B loads, one per 64-B line (ld_mut in the kernels)
__global__ void calib_gather8_64_sc1(const uint64_t* p, size_t lines, uint32_t* out) {
  uint64_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < lines; i += (size_t)gridDim.x * blockDim.x)
    acc ^= __hip_atomic_load(const_cast<uint64_t*>(p + i * 8), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((uint32_t)acc == 0x9e3779b9u) out[0] = (uint32_t)acc;
}

int main() {
  const size_t bytes = (size_t)256 << 20;
  void* buf = nullptr;
  uint32_t* out = nullptr;
  CHK(hipMalloc(&buf, bytes));
  CHK(hipMalloc((void**)&out, 64));
  CHK(hipMemset(buf, 1, bytes));
  CHK(hipDeviceSynchronize());
  const dim3 g(4096), b(256);
  // (a different 256 MiB region between kernels would be needed to defeat the 256 MiB MALL;
  // FETCH_SIZE counts MALL hits as well, so one buffer serves)
  calib_wide16<<<g, b>>>((const uint4*)buf, bytes / 16, out);
  calib_cont8<<<g, b>>>((const uint64_t*)buf, bytes / 8, out);
  calib_cont4<<<g, b>>>((const uint32_t*)buf, bytes / 4, out);
  calib_gather8_64<<<g, b>>>((const uint64_t*)buf, bytes / 64, out);
  calib_gather8_128<<<g, b>>>((const uint64_t*)buf, bytes / 128, out);
  calib_gather8_64_sc1<<<g, b>>>((const uint64_t*)buf, bytes / 64, out);
  CHK(hipGetLastError());
  CHK(hipDeviceSynchronize());
  // bytes of 64-B lines each pattern touches
  printf("{\"calib_wide16\": %zu, \"calib_cont8\": %zu, \"calib_cont4\": %zu, \"calib_gather8_64\": %zu, "
         "\"calib_gather8_128\": %zu, \"calib_gather8_64_sc1\": %zu}\n",
         bytes, bytes, bytes, bytes, bytes / 2, bytes);
  CHK(hipFree(buf));
  CHK(hipFree(out));
  return 0;
}
