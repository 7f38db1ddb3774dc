// Recursion circuit accumulation on the GPU: risc0_circuit_recursion_cuda_accum's role
// (recursion-sys/kernels/cuda/ffi.cu; CPU driver recursion-sys/kernels/cxx/ffi.cpp:160-217):
//   1. compute : per cycle, the accumulator factor (generated kernels, gen/accum/)
//   2. prefix  : inclusive product of the factors over the work cycles (FpExt, in order;
//                the product is commutative, so a tree scan gives the sequential words)
//   3. verify  : per cycle, the accum-group registers from the prefix products
// The per-cycle value starts at FpExt 1 (AccumContext's accum(steps, FpExt(1))).
//
// The scan is three passes over 16 B per cycle: tile products (256 lanes x 4 cycles per
// tile), one workgroup scanning the tile products, then the in-tile scan times its tile's
// prefix. HBM traffic is negligible next to steps 1 and 3.
#include "accum_gen.h"
#include "devmem.h"

namespace r0 {
namespace {

constexpr int kT = 256;
constexpr int kPer = 4;
constexpr uint32_t kTile = kT * kPer;

__device__ __forceinline__ FpExt ld4(const uint4* p) {
  const uint4 v = *p;
  return FpExt{{v.x, v.y, v.z, v.w}};
}
__device__ __forceinline__ void st4(uint4* p, const FpExt& a) { *p = make_uint4(a.c[0], a.c[1], a.c[2], a.c[3]); }

__device__ __forceinline__ FpExt shfl_up4(const FpExt& a, int d) {
  FpExt r;
#pragma unroll
  for (int i = 0; i < 4; i++) r.c[i] = __shfl_up(a.c[i], d, 64);
  return r;
}

// workgroup inclusive product scan of one FpExt per lane
__device__ FpExt wg_scan_mul(FpExt v, FpExt* lds) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const FpExt o = shfl_up4(v, d);
    if (lane >= d) v = fe_mul(v, o);
  }
  if (lane == 63) lds[wave] = v;
  __syncthreads();
  FpExt off = fe_one();
  for (int w = 0; w < wave; w++) off = fe_mul(off, lds[w]);
  __syncthreads();
  return fe_mul(v, off);
}

__global__ __launch_bounds__(kT) void tile_products_kernel(const uint4* vals, uint32_t steps, uint4* prods) {
  __shared__ FpExt lds[kT / 64];
  const uint64_t base = uint64_t(blockIdx.x) * kTile + uint64_t(threadIdx.x) * kPer;
  FpExt p = fe_one();
#pragma unroll
  for (int i = 0; i < kPer; i++)
    if (base + i < steps) p = fe_mul(p, ld4(vals + base + i));
  p = wg_scan_mul(p, lds);
  if (threadIdx.x == kT - 1) st4(prods + blockIdx.x, p);
}

// exclusive prefix of this lane within the workgroup, from wg_scan_mul's inclusive value
// (lds still holds the per-wave totals)
__device__ __forceinline__ FpExt wg_exclusive(const FpExt& inc, const FpExt* lds) {
  FpExt prev = shfl_up4(inc, 1);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    prev = fe_one();
    for (int w = 0; w < wave; w++) prev = fe_mul(prev, lds[w]);
  }
  return prev;
}

// one workgroup: exclusive product scan of the tile products, in place
__global__ __launch_bounds__(kT) void scan_products_kernel(uint4* prods, uint32_t ntiles) {
  __shared__ FpExt lds[kT / 64];
  __shared__ FpExt total;
  FpExt carry = fe_one();
  for (uint32_t b = 0; b < ntiles; b += kT) {
    const uint32_t i = b + threadIdx.x;
    const FpExt v = i < ntiles ? ld4(prods + i) : fe_one();
    const FpExt inc = wg_scan_mul(v, lds);
    const FpExt ex = wg_exclusive(inc, lds);
    if (i < ntiles) st4(prods + i, fe_mul(carry, ex));
    if (threadIdx.x == kT - 1) total = inc;
    __syncthreads();
    carry = fe_mul(carry, total);
    __syncthreads();
  }
}

__global__ __launch_bounds__(kT) void apply_products_kernel(uint4* vals, uint32_t steps, const uint4* prods) {
  __shared__ FpExt lds[kT / 64];
  const uint64_t base = uint64_t(blockIdx.x) * kTile + uint64_t(threadIdx.x) * kPer;
  FpExt x[kPer];
  FpExt p = fe_one();
#pragma unroll
  for (int i = 0; i < kPer; i++) {
    x[i] = base + i < steps ? ld4(vals + base + i) : fe_one();
    p = fe_mul(p, x[i]);
  }
  const FpExt inc = wg_scan_mul(p, lds);
  FpExt run = fe_mul(ld4(prods + blockIdx.x), wg_exclusive(inc, lds));
#pragma unroll
  for (int i = 0; i < kPer; i++) {
    run = fe_mul(run, x[i]);
    if (base + i < steps) st4(vals + base + i, run);
  }
}

__global__ void fill_one_kernel(uint4* vals, uint64_t n) {
  const uint64_t i = uint64_t(blockIdx.x) * kT + threadIdx.x;
  if (i < n) vals[i] = make_uint4(kOne, 0u, 0u, 0u);
}

}  // namespace

void recursion_accum(hipStream_t s, const uint32_t* ctrl, const uint32_t* global, const uint32_t* data,
                     const uint32_t* mix, uint32_t* accum, size_t steps, size_t cycles) {
  R0_REQUIRE(cycles >= 4 && (cycles & (cycles - 1)) == 0 && cycles <= (size_t(1) << 26),
             "recursion_accum: cycles must be a power of two in [4, 2^26]");
  R0_REQUIRE(steps >= 1 && steps <= cycles, "recursion_accum: need 1 <= steps <= cycles");
  KScope ks("recursion_accum", double(steps) * (23 + 128 + 12 + 8) * 4);
  uint4* vals = static_cast<uint4*>(scratch(steps * 16, kSlotRecAccVals));
  const uint32_t ntiles = uint32_t((steps + kTile - 1) / kTile);
  uint4* prods = static_cast<uint4*>(scratch(size_t(ntiles) * 16, kSlotRecAccProds));
  hipLaunchKernelGGL(fill_one_kernel, dim3(div_up(steps, kT)), dim3(kT), 0, s, vals, uint64_t(steps));
  HIP_OK(hipGetLastError());
  AccArgs A;
  A.a[0] = const_cast<uint32_t*>(ctrl);
  A.a[1] = const_cast<uint32_t*>(global);
  A.a[2] = const_cast<uint32_t*>(data);
  A.a[3] = const_cast<uint32_t*>(mix);
  A.a[4] = accum;
  A.vals = vals;
  A.steps = uint32_t(steps);
  A.cycles = uint32_t(cycles);
  recursion_accum_compute(s, A);
  hipLaunchKernelGGL(tile_products_kernel, dim3(ntiles), dim3(kT), 0, s, vals, uint32_t(steps), prods);
  HIP_OK(hipGetLastError());
  hipLaunchKernelGGL(scan_products_kernel, dim3(1), dim3(kT), 0, s, prods, ntiles);
  HIP_OK(hipGetLastError());
  hipLaunchKernelGGL(apply_products_kernel, dim3(ntiles), dim3(kT), 0, s, vals, uint32_t(steps), prods);
  HIP_OK(hipGetLastError());
  recursion_accum_verify(s, A);
}

}  // namespace r0
