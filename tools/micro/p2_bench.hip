// Poseidon2 permutation throughput on gfx950, state in registers (no memory traffic):
// each lane runs ITERS chained permutations. Compare with hash_rows' perms/s to split
// permutation cost from load/occupancy effects.
//   hipcc --offload-arch=gfx950 -O3 -I../../risc0_amd/csrc p2_bench.hip -o p2_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "poseidon2.h"

constexpr int ITERS = 64;

template <int LB>
__global__ __launch_bounds__(256, LB) void k(uint32_t* out, uint32_t seed) {
  uint32_t c[24];
#pragma unroll
  for (int i = 0; i < 24; i++) c[i] = (seed * 2654435761u + i * 40503u + threadIdx.x) % r0::kP;
  for (int it = 0; it < ITERS; it++) r0::poseidon2_mix(c);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) acc ^= c[i];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int LB>
void run(uint32_t* out, int blocks_per_cu) {
  int nblk = 256 * blocks_per_cu;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k<LB>, dim3(nblk), dim3(256), 0, 0, out, 1u);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k<LB>, dim3(nblk), dim3(256), 0, 0, out, uint32_t(r + 2));
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  double perms = 3.0 * nblk * 256.0 * ITERS;
  printf("launch_bounds min-waves %d, %2d blocks/CU: %8.3f ms  %6.2f G perm/s\n", LB, blocks_per_cu, ms,
         perms / (ms * 1e-3) / 1e9);
}

int main() {
  uint32_t* out;
  (void)hipMalloc(&out, 256 * 64 * 256 * 4);
  for (int b : {4, 8, 16, 32}) run<1>(out, b);
  for (int b : {8, 16, 32}) run<2>(out, b);
  for (int b : {16, 32}) run<4>(out, b);
  return 0;
}
