// Recursion circuit witness generation on the GPU: the role of
// risc0_circuit_recursion_{cpu,cuda}_witgen (recursion-sys/kernels/cxx/ffi.cpp:57-205,
// called from circuit/recursion/src/prove/witgen.rs:91-100 with StepMode::Parallel).
//
//   1. exec: step_exec over the work cycles (generated, gen/rwitgen/witgen_exec.hip), one
//      lane per run of cycles — a run starts at cycle 0 or at a parallel-safe cycle and takes
//      the following cycles that are not (MachineContext::parStepExec). Each cycle appends
//      its WOM argument rows (addr, value) to its own slots. Runs are independent, so they
//      are bucketed by major (the one-hot selector among control columns 1..7 shared by all
//      of a run's cycles; bucket 8 for runs of several majors without the MACRO block; else
//      bucket 0) and each bucket runs a step specialised to it: one register allocation per
//      bucket instead of the union of all majors.
//   2. verifyWom (ffi.cpp:118-135): the rows sorted as WomArgumentRow::operator< orders them
//      (address, then the value's elements as field integers) — five stable LSD radix passes
//      over 32-bit keys carrying a permutation; the per-cycle row counts exclusive-scanned
//      into each cycle's first sorted row.
//   3. injectWomBacks (ffi.cpp:137-158): data columns 0..4 of row c - 1 get the sorted row
//      just before cycle c's first (or zeros).
//   4. verify: step_verify_mem per cycle (generated, gen/rwitgen/witgen_verify.hip).
//
// The preflight trace (WOM, per-cycle {iopIdx, isParSafe}, IOP values) comes from the host,
// as RawPreflightTrace does. Checks that throw in the reference record an error here, which
// the launcher raises after the kernels drain.
#include <hipcub/hipcub.hpp>

#include <string>
#include <vector>

#include "devmem.h"
#include "witgen_gen.h"

namespace r0 {
namespace {

using rwg::kMaxWomRows;
using rwg::kRowWords;
constexpr uint32_t kT = 256;

// key pass k of the lexicographic sort: 0..3 the value's elements 3..0 as Fp integers, 4 the
// address (WomArgumentRow::operator<: std::tie(addr, value.elems[0..3]), Fp::operator<
// compares decode(val))
__global__ __launch_bounds__(kT) void row_key_kernel(const uint32_t* rows, const uint32_t* perm, uint32_t* key,
                                                    uint32_t n, uint32_t pass) {
  const uint32_t i = blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const uint32_t* r = rows + uint64_t(perm[i]) * kRowWords;
  key[i] = pass == 4 ? r[0] : mont_reduce(r[4 - pass]);
}

// bucket of each run: the major m in 1..7 when every cycle of the run has control column m
// equal to one and the other selectors zero; 8 when the cycles have different majors of that
// form, none of them column 2 (the MACRO block, which alone needs 512 VGPRs and scratch); else
// 0 (the generic step). Counts per bucket.
constexpr uint32_t kBuckets = 9;
__global__ __launch_bounds__(kT) void run_key_kernel(const uint32_t* ctrl, uint32_t steps, const uint32_t* run_start,
                                                    uint32_t nruns, uint32_t* key, uint32_t* idx, uint32_t* counts) {
  __shared__ uint32_t h[kBuckets];
  if (threadIdx.x < kBuckets) h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t r = blockIdx.x * kT + threadIdx.x;
  if (r < nruns) {
    uint32_t k = 0xFFu;
    bool valid = true, macro = false;
    for (uint32_t c = run_start[r]; c < run_start[r + 1]; c++) {
      uint32_t m = 0, n = 0;
      for (uint32_t j = 1; j <= 7; j++) {
        const uint32_t v = ctrl[uint64_t(j) * steps + c];
        if (v != 0u) {
          n++;
          m = v == kOne ? j : 0u;
        }
      }
      const uint32_t cm = n == 1 ? m : 0u;
      valid = valid && cm != 0u;
      macro = macro || cm == 2u;
      k = k == 0xFFu ? cm : (k == cm ? k : 8u);
    }
    if (!valid) k = 0u;
    else if (k == 8u && macro) k = 0u;
    key[r] = k;
    idx[r] = r;
    atomicAdd(&h[k], 1u);
  }
  __syncthreads();
  if (threadIdx.x < kBuckets && h[threadIdx.x]) atomicAdd(&counts[threadIdx.x], h[threadIdx.x]);
}

__global__ __launch_bounds__(kT) void iota_kernel(uint32_t* p, uint32_t n) {
  const uint32_t i = blockIdx.x * kT + threadIdx.x;
  if (i < n) p[i] = i;
}

__global__ __launch_bounds__(kT) void gather_rows_kernel(const uint32_t* rows, const uint32_t* perm, uint32_t* out,
                                                        uint32_t n) {
  const uint32_t i = blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const uint32_t* r = rows + uint64_t(perm[i]) * kRowWords;
  uint32_t* o = out + uint64_t(i) * kRowWords;
#pragma unroll
  for (uint32_t k = 0; k < kRowWords; k++) o[k] = r[k];
}

// injectWomBacks: cycle c >= 1 writes data columns 0..4 of row c - 1
__global__ __launch_bounds__(kT) void inject_backs_kernel(uint32_t* data, uint32_t steps, const uint32_t* sorted,
                                                         const uint32_t* index, uint32_t ncycles) {
  const uint32_t c = blockIdx.x * kT + threadIdx.x + 1;
  if (c >= ncycles) return;
  const uint32_t idx = index[c];
  uint32_t v[5] = {0u, 0u, 0u, 0u, 0u};
  if (idx) {
    const uint32_t* r = sorted + uint64_t(idx - 1) * kRowWords;
    v[0] = rwg::fp_from_u32(r[0]);
#pragma unroll
    for (int k = 1; k < 5; k++) v[k] = r[k];
  }
#pragma unroll
  for (int k = 0; k < 5; k++) data[uint64_t(k) * steps + c - 1] = v[k];
}

std::string witgen_error(uint32_t code, uint32_t cycle) {
  using namespace rwg;
  const std::string at = " (cycle " + std::to_string(cycle) + ")";
  if (code >= kErrEqz && code < kErrCoefficients)
    return "eqz failed at: zirgen/circuit/recursion/wom.cpp:" + std::to_string(code - kErrEqz) + at;
  if (code == kErrCoefficients) return "extern_readCoefficients not implemented" + at;
  if (code == kErrWomAddr) return "WOM read past the preflight's memory" + at;
  if (code == kErrWomRows) return "more than 9 WOM argument rows in one cycle" + at;
  if (code == kErrIop) return "IOP read past the preflight's values" + at;
  return "witness generation error " + std::to_string(code) + at;
}

}  // namespace

void recursion_witgen(hipStream_t s, const uint32_t* ctrl, uint32_t* data, uint32_t* global, size_t total_cycles,
                      const uint32_t* h_wom, size_t n_wom, const uint32_t* h_cycles, size_t ncycles,
                      const uint32_t* h_iops, size_t n_iops) {
  R0_REQUIRE(total_cycles >= 4 && (total_cycles & (total_cycles - 1)) == 0 && total_cycles <= (size_t(1) << 24),
             "recursion_witgen: total_cycles must be a power of two in [4, 2^24]");
  R0_REQUIRE(ncycles <= total_cycles, "recursion_witgen: more work cycles than rows");
  R0_REQUIRE((n_wom == 0 || h_wom) && (ncycles == 0 || h_cycles) && (n_iops == 0 || h_iops),
             "recursion_witgen: null trace array with a nonzero count");
  if (ncycles == 0) return;
  // the runs of MachineContext::parStepExec and each cycle's first IOP value
  std::vector<uint32_t> run_start, iop_idx(ncycles);
  for (size_t c = 0; c < ncycles; c++) {
    iop_idx[c] = h_cycles[2 * c];
    if (c == 0 || h_cycles[2 * c + 1] != 0) run_start.push_back(uint32_t(c));
  }
  const uint32_t nruns = uint32_t(run_start.size());
  run_start.push_back(uint32_t(ncycles));
  const size_t nrows = ncycles * kMaxWomRows;
  R0_REQUIRE(nrows < (size_t(1) << 31), "recursion_witgen: too many cycles");

  uint32_t* d_wom = static_cast<uint32_t*>(scratch(n_wom * 16 + 16, kSlotWitgenWom));
  uint32_t* d_iops = static_cast<uint32_t*>(scratch(n_iops * 16 + 16, kSlotWitgenIops));
  uint32_t* d_runs = static_cast<uint32_t*>(scratch(run_start.size() * 4, kSlotWitgenRuns));
  uint32_t* d_iop_idx = static_cast<uint32_t*>(scratch(ncycles * 4, kSlotWitgenIopIdx));
  upload_async(d_wom, h_wom, n_wom * 16);
  upload_async(d_iops, h_iops, n_iops * 16);
  upload_async(d_runs, run_start.data(), run_start.size() * 4);
  upload_async(d_iop_idx, iop_idx.data(), ncycles * 4);
  DevBuf rows(nrows * kRowWords), sorted(nrows * kRowWords), count(ncycles), index(ncycles), err(2);
  DevBuf perm_a(nrows), perm_b(nrows), key_a(nrows), key_b(nrows);
  HIP_OK(hipMemsetD32Async(rows.p, rwg::kInvalidWord, nrows * kRowWords, s));  // {kInvalidPattern, FpExt::invalid()}
  HIP_OK(hipMemsetD32Async(count.p, 0, ncycles, s));
  HIP_OK(hipMemsetD32Async(err.p, 0, 2, s));

  rwg::WitgenArgs A{};
  A.ctrl = ctrl;
  A.global = global;
  A.data = data;
  A.steps = uint32_t(total_cycles);
  A.ncycles = uint32_t(ncycles);
  A.run_start = d_runs;
  A.nruns = nruns;
  A.wom = d_wom;
  A.n_wom = uint32_t(n_wom);
  A.iops = d_iops;
  A.n_iops = uint32_t(n_iops);
  A.iop_idx = d_iop_idx;
  A.rows = rows.p;
  A.wom_count = count.p;
  A.wom_index = index.p;
  A.sorted = sorted.p;
  A.err = err.p;
  {
    KScope ks("recursion_witgen_exec", double(ncycles) * 4 * (23 + 2 * 128));
    // runs bucketed by major (radix sort on the 4-bit key), one specialised launch per bucket
    uint32_t* key = static_cast<uint32_t*>(scratch(size_t(nruns) * 4, kSlotWitgenRunKey));
    uint32_t* idx = static_cast<uint32_t*>(scratch(size_t(nruns) * 4, kSlotWitgenRunKey + 1));
    uint32_t* key2 = static_cast<uint32_t*>(scratch(size_t(nruns) * 4, kSlotWitgenRunKey + 2));
    uint32_t* idx2 = static_cast<uint32_t*>(scratch(size_t(nruns) * 4, kSlotWitgenRunKey + 3));
    DevBuf counts(kBuckets);
    HIP_OK(hipMemsetD32Async(counts.p, 0, kBuckets, s));
    hipLaunchKernelGGL(run_key_kernel, dim3((nruns + kT - 1) / kT), dim3(kT), 0, s, ctrl, uint32_t(total_cycles),
                       d_runs, nruns, key, idx, counts.p);
    size_t sort_bytes = 0;
    HIP_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, key, key2, idx, idx2, int(nruns), 0, 4, s));
    void* sort_temp = scratch(sort_bytes + 256, kSlotWitgenRunTemp);
    HIP_OK(hipcub::DeviceRadixSort::SortPairs(sort_temp, sort_bytes, key, key2, idx, idx2, int(nruns), 0, 4, s));
    uint32_t h_counts[kBuckets];
    HIP_OK(hipMemcpyAsync(h_counts, counts.p, sizeof(h_counts), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    uint32_t off = 0;
    for (int k = 0; k < int(kBuckets); k++) {
      recursion_witgen_exec(s, A, k, idx2 + off, h_counts[k]);
      off += h_counts[k];
    }
    R0_REQUIRE(off == nruns, "recursion_witgen: run buckets do not cover the runs");
  }
  {
    // verifyWom: lexicographic sort of the argument rows (five stable radix passes)
    KScope ks("recursion_witgen_sort", double(nrows) * 4 * (kRowWords * 2 + 5 * 6));
    const uint32_t n = uint32_t(nrows), g = (n + kT - 1) / kT;
    hipLaunchKernelGGL(iota_kernel, dim3(g), dim3(kT), 0, s, perm_a.p, n);
    size_t temp_bytes = 0;
    HIP_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, key_a.p, key_b.p, perm_a.p, perm_b.p, int(n), 0,
                                              32, s));
    size_t scan_bytes = 0;
    HIP_OK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, count.p, index.p, int(ncycles), s));
    void* temp = scratch(std::max(temp_bytes, scan_bytes) + 256, kSlotWitgenTemp);
    uint32_t* perm = perm_a.p;
    uint32_t* perm_out = perm_b.p;
    for (uint32_t pass = 0; pass < 5; pass++) {
      hipLaunchKernelGGL(row_key_kernel, dim3(g), dim3(kT), 0, s, rows.p, perm, key_a.p, n, pass);
      HIP_OK(hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, key_a.p, key_b.p, perm, perm_out, int(n), 0, 32, s));
      std::swap(perm, perm_out);
    }
    hipLaunchKernelGGL(gather_rows_kernel, dim3(g), dim3(kT), 0, s, rows.p, perm, sorted.p, n);
    HIP_OK(hipcub::DeviceScan::ExclusiveSum(temp, scan_bytes, count.p, index.p, int(ncycles), s));
    if (ncycles > 1)
      hipLaunchKernelGGL(inject_backs_kernel, dim3(uint32_t((ncycles - 1 + kT - 1) / kT)), dim3(kT), 0, s, data,
                         uint32_t(total_cycles), sorted.p, index.p, uint32_t(ncycles));
    HIP_OK(hipGetLastError());
  }
  {
    KScope ks("recursion_witgen_verify", double(ncycles) * 4 * (23 + 2 * 128));
    recursion_witgen_verify(s, A);
  }
  uint32_t h_err[2] = {0, 0};
  HIP_OK(hipMemcpyAsync(h_err, err.p, 8, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  R0_REQUIRE(h_err[0] == 0, "recursion witgen: " + witgen_error(h_err[0], h_err[1]));
}

}  // namespace r0
