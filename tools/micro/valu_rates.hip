// Issue rate of single gfx950 VALU instructions (inline asm, 8 independent chains per
// lane, 8 waves per SIMD): lane-instructions per second over the whole chip.
//   hipcc --offload-arch=gfx950 -O3 valu_rates.hip -o valu_rates && ./valu_rates
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int ITERS = 2048;

#define R8(S) S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7)
template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
  uint32_t x0 = seed ^ threadIdx.x, x1 = x0 * 3, x2 = x0 * 5, x3 = x0 * 7, x4 = x0 * 9, x5 = x0 * 11, x6 = x0 * 13,
           x7 = x0 * 15;
  uint64_t y0 = x0, y1 = x1, y2 = x2, y3 = x3, y4 = x4, y5 = x5, y6 = x6, y7 = x7;
  const uint32_t b = seed * 7 + 1;
  uint64_t sd;
  for (int i = 0; i < ITERS; i++) {
#define ADD(n) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x##n) : "v"(b));
#define MIN(n) asm volatile("v_min_u32 %0, %0, %1" : "+v"(x##n) : "v"(b));
#define MULLO(n) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x##n) : "v"(b));
#define MULHI(n) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x##n) : "v"(b));
#define MAD64(n) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(y##n), "=s"(sd) : "v"(x##n), "v"(b));
#define LSHLADD64(n) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(y##n) : "v"(y0));
#define ADDCO(n) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x##n) : "v"(b) : "vcc");
#define SUB(n) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x##n) : "v"(b));
#define ADD3(n) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x##n) : "v"(b));
    if (OP == 0) { R8(ADD) }
    if (OP == 1) { R8(MIN) }
    if (OP == 2) { R8(MULLO) }
    if (OP == 3) { R8(MULHI) }
    if (OP == 4) { R8(MAD64) }
    if (OP == 5) { R8(LSHLADD64) }
    if (OP == 6) { R8(ADDCO) }
    if (OP == 7) { R8(SUB) }
    if (OP == 8) { R8(ADD3) }
  }
  out[blockIdx.x * 256 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ uint32_t(y0 ^ y1 ^ y2 ^ y3 ^ y4 ^ y5 ^ y6 ^ y7);
}

template <int OP>
void run(const char* name, uint32_t* out, int nblk) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k<OP>, dim3(nblk), dim3(256), 0, 0, out, 1u);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k<OP>, dim3(nblk), dim3(256), 0, 0, out, uint32_t(r + 2));
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  double ops = 5.0 * nblk * 256.0 * ITERS * 8;
  printf("%-16s %8.3f ms  %8.2f T lane-instr/s\n", name, ms, ops / (ms * 1e-3) / 1e12);
}

int main(int argc, char** argv) {
  uint32_t* out;
  // waves per SIMD = blocks per CU (256 threads = one wave on each of the 4 SIMDs)
  int wps = argc > 1 ? atoi(argv[1]) : 8;
  int nblk = 256 * wps;
  printf("waves per SIMD: %d\n", wps);
  hipMalloc(&out, nblk * 256 * 4);
  run<0>("v_add_u32", out, nblk);
  run<1>("v_min_u32", out, nblk);
  run<2>("v_mul_lo_u32", out, nblk);
  run<3>("v_mul_hi_u32", out, nblk);
  run<4>("v_mad_u64_u32", out, nblk);
  run<5>("v_lshl_add_u64", out, nblk);
  run<6>("v_add_co_u32", out, nblk);
  run<7>("v_sub_u32", out, nblk);
  run<8>("v_add3_u32", out, nblk);
  return 0;
}
