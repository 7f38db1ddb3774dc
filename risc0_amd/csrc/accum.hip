// rv32im accumulation, phases 2 and 3 (risc0/circuit/rv32im-sys/kernels/cuda/ffi.cu:465-514,
// CPU: kernels/cxx/ffi.cpp:326-360) on the GPU: after the per-cycle accum step has filled the
// accum group, the last 4 columns become inclusive prefix sums over rows [0, last_cycle)
// (the reference uses thrust::inclusive_scan per column), then each row adds the previous
// row's (cyclically) prefix values to the machine columns [split, cols - 4).
//
// The scan is mod-p addition of Montgomery words (addition is representation-independent),
// in three HBM passes over the 4 columns: per-tile sums, one workgroup per column scanning
// the tile sums, and the in-tile scan with the tile's offset. A tile is 256 lanes x 16
// consecutive rows; every load and store is a coalesced 64-byte-per-lane run.
#include "bb31.h"
#include "devmem.h"
#include "accum_gen.h"
#include "runtime.h"

namespace r0 {
namespace {

constexpr int kT = 256;      // lanes per workgroup
constexpr int kPer = 16;     // rows per lane
constexpr uint32_t kTile = kT * kPer;

// workgroup inclusive scan of one value per lane (mod p), wave64 shuffles + LDS
__device__ __forceinline__ uint32_t wg_scan(uint32_t v, uint32_t* lds) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t o = __shfl_up(v, d, 64);
    if (lane >= d) v = fp_add(v, o);
  }
  if (lane == 63) lds[wave] = v;
  __syncthreads();
  uint32_t off = 0;
  for (int w = 0; w < wave; w++) off = fp_add(off, lds[w]);
  __syncthreads();
  return fp_add(v, off);
}

__global__ __launch_bounds__(kT) void tile_sums_kernel(const uint32_t* accum, uint64_t rows, uint32_t cols,
                                                       uint64_t last, uint32_t* sums, uint32_t ntiles) {
  __shared__ uint32_t lds[kT / 64];
  const uint32_t col = cols - 4 + blockIdx.y, tile = blockIdx.x;
  const uint32_t* c = accum + uint64_t(col) * rows;
  const uint64_t base = uint64_t(tile) * kTile + uint64_t(threadIdx.x) * kPer;
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kPer; i++)
    if (base + i < last) s = fp_add(s, c[base + i]);
  s = wg_scan(s, lds);
  if (threadIdx.x == kT - 1) sums[blockIdx.y * ntiles + tile] = s;
}

// one workgroup per column: exclusive scan of the tile sums in place
__global__ __launch_bounds__(kT) void scan_sums_kernel(uint32_t* sums, uint32_t ntiles) {
  __shared__ uint32_t lds[kT / 64];
  uint32_t* s = sums + blockIdx.x * ntiles;
  uint32_t carry = 0;
  for (uint32_t b = 0; b < ntiles; b += kT) {
    const uint32_t i = b + threadIdx.x;
    const uint32_t v = i < ntiles ? s[i] : 0u;
    const uint32_t inc = wg_scan(v, lds);
    if (i < ntiles) s[i] = fp_add(carry, fp_sub(inc, v));  // exclusive
    __shared__ uint32_t last_inc;
    if (threadIdx.x == kT - 1) last_inc = inc;
    __syncthreads();
    carry = fp_add(carry, last_inc);
    __syncthreads();
  }
}

__global__ __launch_bounds__(kT) void tile_scan_kernel(uint32_t* accum, uint64_t rows, uint32_t cols, uint64_t last,
                                                       const uint32_t* sums, uint32_t ntiles) {
  __shared__ uint32_t lds[kT / 64];
  const uint32_t col = cols - 4 + blockIdx.y, tile = blockIdx.x;
  uint32_t* c = accum + uint64_t(col) * rows;
  const uint64_t base = uint64_t(tile) * kTile + uint64_t(threadIdx.x) * kPer;
  uint32_t v[kPer];
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kPer; i++) {
    v[i] = base + i < last ? c[base + i] : 0u;
    s = fp_add(s, v[i]);
    v[i] = s;  // in-lane inclusive prefix
  }
  const uint32_t inc = wg_scan(s, lds);
  const uint32_t off = fp_add(sums[blockIdx.y * ntiles + tile], fp_sub(inc, s));
#pragma unroll
  for (int i = 0; i < kPer; i++)
    if (base + i < last) c[base + i] = fp_add(v[i], off);
}

// phase 3: row r adds prefix[(r - 1) mod last] to every machine column but the last group
__global__ __launch_bounds__(kT) void finalize_kernel(uint32_t* accum, uint64_t rows, uint32_t cols, uint32_t split,
                                                      uint64_t last) {
  const uint64_t row = uint64_t(blockIdx.x) * kT + threadIdx.x;
  if (row >= last) return;
  const uint64_t back1 = row == 0 ? last - 1 : row - 1;
  uint32_t prev[4];
#pragma unroll
  for (int k = 0; k < 4; k++) prev[k] = accum[uint64_t(cols - 4 + k) * rows + back1];
  const uint32_t groups = (cols - split) / 4;
  for (uint32_t j = 0; j + 1 < groups; j++) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uint32_t* p = accum + uint64_t(split + j * 4 + k) * rows + row;
      *p = fp_add(*p, prev[k]);
    }
  }
}

// BigInt accumulator states (bigint.cpp): record k's 12 words into accum columns 0..11 of its
// row (BigIntAccumState::offsets, rv32im witgen/byte_poly.rs:362-377)
__global__ __launch_bounds__(kT) void bigint_scatter_kernel(uint32_t* accum, uint64_t rows, const uint32_t* row_of,
                                                            const uint32_t* states, uint64_t n) {
  const uint64_t k = uint64_t(blockIdx.x) * kT + threadIdx.x;
  if (k >= n) return;
  const uint64_t row = row_of[k];
#pragma unroll
  for (int c = 0; c < 12; c++) accum[uint64_t(c) * rows + row] = states[k * 12 + c];
}

}  // namespace

void bigint_scatter(hipStream_t s, uint32_t* accum, size_t rows, const uint32_t* d_rows, const uint32_t* d_states,
                    size_t n) {
  if (n == 0) return;
  hipLaunchKernelGGL(bigint_scatter_kernel, dim3(div_up(n, kT)), dim3(kT), 0, s, accum, uint64_t(rows), d_rows,
                     d_states, uint64_t(n));
  HIP_OK(hipGetLastError());
}

// The whole accumulation (risc0_circuit_rv32im_cuda_accum, rv32im-sys/kernels/cuda/ffi.cu:
// 362-514; CPU ffi.cpp:313-368): phase 1 runs the per-cycle step generated from
// risc0_amd/circuits/rv32im.accum.ir (tools/gen_rv32im_accum_ir.py -> tools/gen_accum.py;
// one lane per cycle, its stores guarded by the instruction arm the cycle selects), then
// phases 2-3 above. `accum` arrives as the prover allocates it (INVALID words).
void rv32im_accum(hipStream_t s, const uint32_t* data, uint32_t* accum, const uint32_t* global,
                  const uint32_t* mix, size_t rows, size_t cols, size_t last) {
  R0_REQUIRE(rows >= 4 && (rows & (rows - 1)) == 0 && rows <= (size_t(1) << 26),
             "rv32im_accum: rows must be a power of two in [4, 2^26]");
  R0_REQUIRE(last <= rows, "rv32im_accum: last_cycle > rows");
  R0_REQUIRE(cols == 103, "rv32im_accum: the rv32im accum group has 103 columns");
  if (last == 0) return;
  {
    KScope ks("accum_step", double(last) * 4 * (211 + 2 * 103));
    AccArgs A{};
    A.a[0] = const_cast<uint32_t*>(data);
    A.a[1] = accum;
    A.a[2] = const_cast<uint32_t*>(global);
    A.a[3] = const_cast<uint32_t*>(mix);
    A.steps = uint32_t(last);
    A.cycles = uint32_t(rows);
    rv32im_accum_compute(s, A);
  }
  rv32im_accum_finalize(s, accum, rows, cols, 23, last);
}

void rv32im_accum_finalize(hipStream_t s, uint32_t* accum, size_t rows, size_t cols, size_t split, size_t last) {
  R0_REQUIRE(cols >= 4 && split <= cols - 4 && last <= rows, "accum_finalize: bad shape");
  if (last == 0) return;
  const uint32_t ntiles = uint32_t((last + kTile - 1) / kTile);
  const size_t groups = (cols - split) / 4;
  KScope ks("accum_finalize", double(last) * 4 * (4 * 2 + 4 + 8 * 4 * (groups ? groups - 1 : 0)));
  // per-thread scratch, reused only on this thread's stream: no host sync before returning
  uint32_t* sums = static_cast<uint32_t*>(scratch(size_t(4) * ntiles * 4, kSlotAccTileSums));
  hipLaunchKernelGGL(tile_sums_kernel, dim3(ntiles, 4), dim3(kT), 0, s, accum, uint64_t(rows), uint32_t(cols),
                     uint64_t(last), sums, ntiles);
  hipLaunchKernelGGL(scan_sums_kernel, dim3(4), dim3(kT), 0, s, sums, ntiles);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(ntiles, 4), dim3(kT), 0, s, accum, uint64_t(rows), uint32_t(cols),
                     uint64_t(last), sums, ntiles);
  hipLaunchKernelGGL(finalize_kernel, dim3(div_up(last, kT)), dim3(kT), 0, s, accum, uint64_t(rows), uint32_t(cols),
                     uint32_t(split), uint64_t(last));
  HIP_OK(hipGetLastError());
}

}  // namespace r0
