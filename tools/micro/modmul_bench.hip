// Throughput of the integer primitives a BabyBear modmul is built from, on gfx950.
// Each thread runs 8 independent chains for ITERS iterations; grid fills the chip.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)
constexpr uint32_t P = 0x78000001u, NPINV = 0x77ffffffu, PINV = 0x88000001u;
constexpr int ITERS = 4096, CH = 8;

__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint32_t mont_v1(uint32_t a, uint32_t b) {
  uint64_t t = uint64_t(a) * b;
  uint32_t m = uint32_t(t) * NPINV;
  uint32_t r = uint32_t((t + uint64_t(m) * P) >> 32);
  return umin(r, r - P);
}
__device__ __forceinline__ uint32_t mont_v2(uint32_t a, uint32_t b) {
  // signed-difference Montgomery: r = hi(ab) - hi(q p), q = lo(ab) * p^-1
  uint32_t lo = a * b, hi = __umulhi(a, b);
  uint32_t q = lo * PINV;
  uint32_t qp = __umulhi(q, P);
  uint32_t r = hi - qp;
  return umin(r, r + P);
}
__device__ __forceinline__ uint32_t shoup(uint32_t a, uint32_t b, uint32_t bs) {
  uint32_t q = __umulhi(a, bs);
  uint32_t r = a * b - q * P;
  return umin(r, r - P);
}

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
  uint32_t v[CH];
  uint32_t tid = blockIdx.x * 256 + threadIdx.x;
#pragma unroll
  for (int c = 0; c < CH; c++) v[c] = (tid * 2654435761u + c * 40503u + seed) % P;
  uint32_t b = (seed * 7 + 1) % P, bs = uint32_t((uint64_t(b) << 32) / P);
  double dv[CH];
  float fv[CH];
#pragma unroll
  for (int c = 0; c < CH; c++) { dv[c] = v[c]; fv[c] = float(v[c]); }
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CH; c++) {
      if (OP == 0) v[c] = v[c] * v[c] + b;                       // mul_lo (+add)
      if (OP == 1) v[c] = __umulhi(v[c], b) ^ v[c];              // mul_hi
      if (OP == 2) { uint64_t t = uint64_t(v[c]) * b + v[c]; v[c] = uint32_t(t >> 32) ^ uint32_t(t); } // mad_u64
      if (OP == 3) v[c] = mont_v1(v[c], v[c ^ 1]);
      if (OP == 4) v[c] = mont_v2(v[c], v[c ^ 1]);
      if (OP == 5) v[c] = shoup(v[c], b, bs);
      if (OP == 6) dv[c] = fma(dv[c], 1.0000001, 0.5);
      if (OP == 7) fv[c] = fmaf(fv[c], 1.0000001f, 0.5f);
      if (OP == 8) v[c] = __umul24(v[c], b) + v[c];              // mul_u32_u24
      if (OP == 9) v[c] = (v[c] + b) ^ (v[c] >> 3);              // add + xor/shift (2 simple ops)
      if (OP == 10) { uint32_t s = v[c] + b; v[c] = umin(s, s - P); } // fp_add: 3 ops
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) acc ^= v[c] ^ uint32_t(dv[c]) ^ uint32_t(fv[c]);
  out[tid] = acc;
}

template <int OP>
int run(const char* name, uint32_t* out, int nblk) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k<OP>, dim3(nblk), dim3(256), 0, 0, out, 1u);
  CHECK(hipDeviceSynchronize());
  hipEventRecord(e0);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k<OP>, dim3(nblk), dim3(256), 0, 0, out, uint32_t(r + 2));
  hipEventRecord(e1);
  CHECK(hipEventSynchronize(e1));
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  double ops = 5.0 * nblk * 256.0 * ITERS * CH;
  printf("%-28s %8.3f ms  %8.2f Gop/s (lane-ops)\n", name, ms, ops / (ms * 1e-3) / 1e9);
  return 0;
}

int main() {
  int nblk = 256 * 8 * 4;
  uint32_t* out;
  CHECK(hipMalloc(&out, size_t(nblk) * 256 * 4));
  run<0>("mul_lo+add", out, nblk);
  run<1>("mul_hi+xor", out, nblk);
  run<2>("mad_u64_u32+xor", out, nblk);
  run<3>("mont_v1 (mad64)", out, nblk);
  run<4>("mont_v2 (mulhi signed)", out, nblk);
  run<5>("shoup const", out, nblk);
  run<6>("fma_f64", out, nblk);
  run<7>("fma_f32", out, nblk);
  run<8>("mul_u24+add", out, nblk);
  run<9>("add+xor+shift", out, nblk);
  run<10>("fp_add (add,sub,min)", out, nblk);
  return 0;
}
