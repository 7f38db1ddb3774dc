// Small device-to-host copies and per-call costs, the per-op path's query phase (one 32-byte
// get_at per Merkle node, as the reference's MerkleTreeProver::prove does over a HAL without
// unified memory). Prints microseconds per operation.
//   hipcc --offload-arch=gfx950 -O2 small_d2h.hip -o small_d2h && ./small_d2h
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void touch(uint32_t* p) { if (threadIdx.x == 0) p[0] += 1; }

int main() {
  const int N = 2000;
  uint32_t* d;
  CK(hipMalloc(&d, 1 << 20));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<uint32_t> pageable(1 << 16);
  uint32_t* pinned;
  CK(hipHostMalloc((void**)&pinned, 1 << 20, hipHostMallocDefault));
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto us = [&](auto t0) { return std::chrono::duration<double, std::micro>(now() - t0).count() / N; };
  for (int bytes : {32, 256, 4096}) {
    for (int rep = 0; rep < 2; rep++) {
      auto t0 = now();
      for (int i = 0; i < N; i++) { CK(hipMemcpyAsync(pageable.data(), d + (i % 64) * 8, bytes, hipMemcpyDeviceToHost, s)); CK(hipStreamSynchronize(s)); }
      double a = us(t0);
      t0 = now();
      for (int i = 0; i < N; i++) { CK(hipMemcpyAsync(pinned, d + (i % 64) * 8, bytes, hipMemcpyDeviceToHost, s)); CK(hipStreamSynchronize(s)); memcpy(pageable.data(), pinned, bytes); }
      double b = us(t0);
      t0 = now();
      for (int i = 0; i < N; i++) CK(hipMemcpy(pageable.data(), d + (i % 64) * 8, bytes, hipMemcpyDeviceToHost));
      double c = us(t0);
      t0 = now();
      for (int i = 0; i < N; i++) CK(hipMemcpyDtoH(pageable.data(), (hipDeviceptr_t)(d + (i % 64) * 8), bytes));
      double e = us(t0);
      if (rep) printf("%5d B: async pageable+sync %.2f  async pinned+sync+memcpy %.2f  hipMemcpy %.2f  hipMemcpyDtoH %.2f us\n", bytes, a, b, c, e);
    }
  }
  auto t0 = now();
  for (int i = 0; i < N; i++) { hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, s, d); CK(hipStreamSynchronize(s)); }
  printf("launch+sync %.2f us\n", us(t0));
  t0 = now();
  for (int i = 0; i < N; i++) CK(hipStreamSynchronize(s));
  printf("idle stream sync %.2f us\n", us(t0));
  return 0;
}
