// FETCH_SIZE calibration: a known number of bytes read from HBM with
// 4-byte-per-lane loads (the eval_check tap loads), 16-byte-per-lane loads (what the guide's
// x2 correction was measured on) and the 4-byte pattern with a second load of the same column
// 16 bytes back (a `back 1` tap in the 4x domain). Each kernel streams a 2 GiB buffer once
// (well past the 256 MiB Infinity Cache) and writes one word per lane.
//   hipcc --offload-arch=gfx950 -O3 fetch_calib.hip -o fetch_calib
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT -o run -- ./fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void read4(const uint32_t* __restrict__ in, uint32_t* out, size_t n) {
  uint32_t acc = 0;
  const size_t stride = size_t(gridDim.x) * 256;
  for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride) acc += in[i];
  out[size_t(blockIdx.x) * 256 + threadIdx.x] = acc;
}
__global__ __launch_bounds__(256) void read16(const uint4* __restrict__ in, uint32_t* out, size_t n4) {
  uint32_t acc = 0;
  const size_t stride = size_t(gridDim.x) * 256;
  for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n4; i += stride) {
    const uint4 v = in[i];
    acc += v.x + v.y + v.z + v.w;
  }
  out[size_t(blockIdx.x) * 256 + threadIdx.x] = acc;
}
// one lane per point, reading point i and point i - 4 of the same column (eval_check's back 1)
__global__ __launch_bounds__(256) void read4_back(const uint32_t* __restrict__ in, uint32_t* out, size_t n) {
  uint32_t acc = 0;
  const size_t stride = size_t(gridDim.x) * 256;
  for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride) acc += in[i] ^ in[(i - 4) & (n - 1)];
  out[size_t(blockIdx.x) * 256 + threadIdx.x] = acc;
}

int main() {
  const size_t bytes = size_t(2) << 30, n = bytes / 4;
  uint32_t *in, *out;
  if (hipMalloc(&in, bytes) != hipSuccess || hipMalloc(&out, size_t(8) << 20) != hipSuccess) return 1;
  (void)hipMemset(in, 1, bytes);
  const int blocks = 256 * 8;  // 8 workgroups per CU, grid-stride
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int rep = 0; rep < 2; rep++) {
    float ms[3];
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(read4, dim3(blocks), dim3(256), 0, 0, in, out, n);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms[0], a, b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(read16, dim3(blocks), dim3(256), 0, 0, reinterpret_cast<const uint4*>(in), out, n / 4);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms[1], a, b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(read4_back, dim3(blocks), dim3(256), 0, 0, in, out, n);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms[2], a, b);
    printf("bytes %zu: read4 %.3f ms (%.0f GB/s)  read16 %.3f ms (%.0f GB/s)  read4_back %.3f ms\n", bytes, ms[0],
           bytes / ms[0] / 1e6, ms[1], bytes / ms[1] / 1e6, ms[2]);
  }
  return 0;
}
