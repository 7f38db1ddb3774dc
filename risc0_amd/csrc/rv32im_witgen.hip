// rv32im witness generation on the GPU: the role of risc0_circuit_rv32im_{cpu,cuda}_witgen
// (rv32im-sys/kernels/cxx/ffi.cpp:230-308, kernels/cuda/ffi.cu:362-470), called from
// WitnessGenerator::hal_generate_witness (circuit/rv32im/src/prove/witgen/mod.rs:135-176)
// after the injector's scatter into the all-INVALID data group.
//
// stepExec runs step_Top (generated from steps.cpp, gen/rvwitgen/witgen_k*.hip) once per
// cycle in two phases, as par_stepExec does: cycles [0, tableSplitCycle) first — their
// lookupDelta calls count the u8/u16 lookup tables (summed per workgroup in LDS, flushed once
// with device atomics) — then the table and done rows [tableSplitCycle, lastCycle), whose
// lookupCurrent reads those counts. Within a phase the cycles are bucketed by their preflight
// major (then minor), and one kernel per instruction arm runs step_Top specialised to that arm
// over its bucket: a wavefront's lanes share the arm. The arms store into compact per-bin
// buffers; merge_kernel writes the data group from them.
// Every phase is a set of independent cycles: the rows a step reads at back > 0 are the
// injected ones (cycle, next pc/state/mode, the Poseidon2/SHA/BigInt states), exactly what
// makes the reference's parallel mode well defined. The reference's forward and reverse
// modes give the same words on a trace it accepts (tests/test_rv32im_witgen_ir.py), so every
// mode runs this schedule.
//
// The preflight trace comes from the host, as RawPreflightTrace does (host pointers), or is
// already resident (rv32im_witgen_dev). The cycles are bucketed on the device (counts, one
// 27-word read-back for the launch sizes, a radix sort). Checks that throw in the reference
// record the lane's first failure, raised after the kernels drain.
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "devmem.h"
#include "rv32im_witgen.h"

namespace r0 {
namespace {

std::string witgen_error(const uint32_t* e) {
  using namespace rvwg;
  const uint32_t code = e[0], cycle = e[1], detail = e[2];
  const std::string at = " (cycle " + std::to_string(cycle) + ")";
  auto where = [&] {
    return detail >= 0x10000u ? " global " + std::to_string(detail - 0x10000u) : " col " + std::to_string(detail);
  };
  if (code >= kErrEqz && code < kErrUnset)
    return "[" + std::to_string(cycle) + "]: eqz failure at: " + rv32im_witgen_message(code - kErrEqz);
  switch (code) {
    case kErrUnset: return "Read of unset value:" + where() + at;
    case kErrInconsistent: return "Inconsistent set:" + where() + at;
    case kErrUnreachable: return "Reached unreachable mux arm" + at;
    case kErrTxnCycle: return "txn cycle mismatch" + at;
    case kErrTxnAddr: return "memory peek not in preflight" + at;
    case kErrTxnRange: return "memory transaction past the preflight's" + at;
    case kErrLookupTable: return "Invalid lookup table" + at;
    case kErrLookupIndex: return "u8/16 table error (index " + std::to_string(detail) + ")" + at;
    case kErrBigint: return "bigint bytes past the preflight's" + at;
    case kErrDiffCount: return "getDiffCount past the preflight's cycles" + at;
    case kErrMajor: return "cycle major " + std::to_string(detail) + " selects no instruction arm" + at;
    case kErrInjectorRow:
      return "injector entry of row " + std::to_string(cycle) + " sets word " + std::to_string(detail) +
             " of another row (Injector::set writes its own row)";
    default: return "witness generation error " + std::to_string(code) + at;
  }
}

}  // namespace

namespace {

constexpr uint32_t kBins = 2 * rvwg::kMajors;  // (phase, major)
constexpr uint32_t kBucketThreads = 256;
constexpr uint32_t kMergeThreads = 256;

// per (phase, instruction arm) cycle counts; a major outside the 13 arms is an error (the
// reference's OneHot EQZ on majorOnehot fails for it). keys/vals: each cycle's bin and index,
// for the stable sort into cycle order within each bin.
__global__ __launch_bounds__(kBucketThreads) void bucket_count_kernel(rvwg::Args A, uint32_t split, uint32_t* counts,
                                                                     uint8_t* keys, uint32_t* vals, uint32_t minor_bits) {
  __shared__ uint32_t h[kBins];
  if (threadIdx.x < kBins) h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t c = blockIdx.x * kBucketThreads + threadIdx.x;
  if (c < A.ncycles) {
    const uint32_t m = A.cycles[c].major;
    const uint32_t b = (c >= split) * rvwg::kMajors + m;
    if (m >= rvwg::kMajors)
      rvwg::fail(A, rvwg::kErrMajor, c, m);
    else
      atomicAdd(&h[b], 1u);
    // the sort key: the bin, and with minor_bits = 3 the minor below it (a bin's cycles then
    // run minor by minor: fewer divergent minor arms per wavefront, rows further apart)
    keys[c] = uint8_t(((m >= rvwg::kMajors ? kBins : b) << minor_bits) | (A.cycles[c].minor & ((1u << minor_bits) - 1u)));
    vals[c] = c;
  }
  __syncthreads();
  if (threadIdx.x < kBins && h[threadIdx.x]) atomicAdd(&counts[threadIdx.x], h[threadIdx.x]);
}

struct BinTable {
  uint32_t minor_bits;      // sort keys are bin << minor_bits | minor
  uint32_t nslots[rvwg::kMajors];  // each arm's slots; its mask words follow them
  uint32_t off[kBins + 1];  // first list index of each bin
  uint32_t cnt[kBins];
  uint64_t cbase[kBins];    // each bin's compact values in the compact buffer (words)
};

// each cycle's place in its bin's list (the lane that ran it, its compact column index)
__global__ __launch_bounds__(kBucketThreads) void bin_pos_kernel(const uint32_t* list, const uint8_t* sorted_keys,
                                                                uint32_t n, BinTable T, uint32_t* pos) {
  const uint32_t j = blockIdx.x * kBucketThreads + threadIdx.x;
  if (j < n) pos[list[j]] = j - T.off[sorted_keys[j] >> T.minor_bits];
}

// the data group from the arms' compact values, a column line at a time: word (col, row) is the
// row's stored value if its arm stored one, else the data word as the injector left it (an
// injected value or INVALID). Every word of rows [0, rows) is written, so each line of a column
// goes out whole. prover: the data group is the prover's own, INVALID in the injected columns but
// where the injector wrote, so only those are read back, and INVALID becomes 0 (the zeroize).
// full (the public witgen, or a prover whose injector sets words outside its rows' injected
// columns, re-initialised for it): every column is read back.
__global__ __launch_bounds__(kMergeThreads) void merge_kernel(uint32_t* data, uint32_t rows, uint32_t ncycles,
                                                             const uint32_t* cbuf, const uint8_t* keys,
                                                             const uint32_t* pos, const int16_t* slot_of, BinTable T,
                                                             bool prover, bool full, bool xcd_tiles, uint32_t* err) {
  constexpr uint32_t kMaskWords = (rvwg::kDataCols + 31) / 32;
  __shared__ int16_t slot[(rvwg::kMajors + 1) * rvwg::kDataCols];
  __shared__ uint32_t msk[kMaskWords][kMergeThreads];  // this thread's row: its arm's stored-slot bits
  for (uint32_t t = threadIdx.x; t < rvwg::kMajors * rvwg::kDataCols; t += kMergeThreads) slot[t] = slot_of[t];
  // rows past the stepped cycles keep their data words: in the prover's group only the injected
  // columns hold them (the others were never written, and become 0)
  for (uint32_t t = threadIdx.x; t < rvwg::kDataCols; t += kMergeThreads) {
    uint32_t inj = prover ? 0u : uint32_t(rvwg::kInjectedCol);
    for (uint32_t k = 0; prover && k < rvwg::kMajors; k++) inj |= uint32_t(slot_of[k * rvwg::kDataCols + t]) & rvwg::kInjectedCol;
    slot[rvwg::kMajors * rvwg::kDataCols + t] = int16_t(rvwg::kNoSlot | inj);
  }
  // xcd_tiles: consecutive workgroups go to the 8 XCDs in turn; renumbered, each XCD takes one
  // contiguous run of rows, so the compact lines that neighbouring row tiles share stay in its L2
  // (po2 20 loop guest: 0.71 -> 0.68 ms, profiles/r4v_witgen_merge_ab.txt)
  uint32_t tile = blockIdx.x;
  if (xcd_tiles) {
    const uint32_t per = gridDim.x / 8, rem = gridDim.x % 8, x = blockIdx.x % 8, q = blockIdx.x / 8;
    tile = x < rem ? x * (per + 1) + q : rem * (per + 1) + (x - rem) * per + q;
  }
  const uint32_t r = tile * kMergeThreads + threadIdx.x;
  const bool stepped = r < ncycles;
  const uint32_t b = stepped ? uint32_t(keys[r]) >> T.minor_bits : 0u;
  const uint32_t arm = b % rvwg::kMajors;
  const uint32_t n = stepped ? T.cnt[b] : 0u, i = stepped ? pos[r] : 0u;
  const uint32_t* cb = cbuf + (stepped ? T.cbase[b] : 0u);
  const uint32_t ns = T.nslots[arm];
  for (uint32_t w = 0; w < kMaskWords; w++)
    msk[w][threadIdx.x] = stepped && 32 * w < ns ? cb[size_t(ns + w) * n + i] : 0u;
  __syncthreads();
  if (r >= rows) return;
  const int16_t* sl = slot + (stepped ? arm : rvwg::kMajors) * rvwg::kDataCols;
#pragma unroll 8
  for (uint32_t col = 0; col < rvwg::kDataCols; col++) {
    const uint32_t e = uint32_t(sl[col]);
    const uint32_t slot = e & rvwg::kNoSlot;
    uint32_t* p = data + uint64_t(col) * rows + r;
    const bool stored = slot != rvwg::kNoSlot && ((msk[slot >> 5][threadIdx.x] >> (slot & 31)) & 1u);
    // the stored value and the data word the row keeps otherwise, loaded side by side (the
    // read-back no longer waits on the compact load's result)
    const uint32_t c = stored ? cb[size_t(slot) * n + i] : rvwg::kInvalid;
    const uint32_t d = full || (e & rvwg::kInjectedCol) ? *p : rvwg::kInvalid;
    // a word set before the arm ran in a column the arm stores but does not take from the
    // injector (so never compared in the arm): Buffer::set's check (buffers.h:30-42) fails only
    // on another value; a word in a column the arm does not store is kept, as there
    if (full && stepped && stored && !(e & rvwg::kInjectedCol) && d != rvwg::kInvalid && d != c &&
        atomicCAS(err, 0u, rvwg::kErrInconsistent) == 0u) {
      err[1] = r;
      err[2] = col;
    }
    uint32_t v = c != rvwg::kInvalid ? c : d;
    if (prover && v == rvwg::kInvalid) v = 0u;
    *p = v;
  }
}

// one lane per row: the injected columns INVALID, code 0, accum INVALID in [acc_inv_begin,
// acc_inv_end) and 0 elsewhere (needs no input: queued before the trace has landed)
struct InjectedCols {
  uint32_t n;
  uint8_t col[rvwg::kDataCols];
  uint32_t arm_mask[rvwg::kMajors][(rvwg::kDataCols + 31) / 32];  // kInjectedCol per arm, as bits
};
__global__ __launch_bounds__(kMergeThreads) void prover_groups_fill_kernel(uint32_t* data, uint32_t* code,
                                                                          uint32_t* accum, uint32_t rows,
                                                                          uint32_t accum_cols, InjectedCols U,
                                                                          uint32_t acc_inv_begin,
                                                                          uint32_t acc_inv_end) {
  const uint32_t r = blockIdx.x * kMergeThreads + threadIdx.x;
  if (r >= rows) return;
  for (uint32_t k = 0; k < U.n; k++) data[uint64_t(U.col[k]) * rows + r] = rvwg::kInvalid;
  code[r] = 0u;
  for (uint32_t c = 0; c < accum_cols; c++)
    accum[uint64_t(c) * rows + r] = c >= acc_inv_begin && c < acc_inv_end ? rvwg::kInvalid : 0u;
}

// one lane per injector row: its entries (Injector::set writes only its own row, witgen/mod.rs:
// 352-377; an entry of another row is refused). err[3] != 0 marks an entry in a column the row's
// arm does not take from the injector: the prover then re-initialises the group whole
// (rv32im_witgen_dev's reinit) so the merge can read every column back.
__global__ __launch_bounds__(kMergeThreads) void prover_inject_kernel(uint32_t* data, uint32_t rows,
                                                                     InjectedCols U, const uint32_t* index,
                                                                     const uint32_t* offsets, const uint32_t* values,
                                                                     uint32_t inj_rows, uint64_t limit,
                                                                     const rvwg::PreflightCycle* cycles,
                                                                     uint32_t row_shift, uint32_t* err) {
  const uint32_t r = blockIdx.x * kMergeThreads + threadIdx.x;
  if (r >= inj_rows) return;
  const uint32_t end = min(index[r + 1], index[inj_rows]);
  const uint32_t arm = cycles[r].major;  // a major past the arms fails in the bucket kernel
  for (uint32_t i = index[r]; i < end; i++) {
    const uint32_t off = offsets[i];
    if (off >= limit) continue;
    if ((off & (rows - 1)) != r) {
      if (atomicCAS(err, 0u, rvwg::kErrInjectorRow) == 0u) {
        err[1] = r;
        err[2] = off;
      }
      continue;
    }
    data[off] = values[i];
    const uint32_t col = off >> row_shift;
    if (arm < rvwg::kMajors && !((U.arm_mask[arm][col >> 5] >> (col & 31)) & 1u)) atomicOr(err + 3, 1u);
  }
}

}  // namespace

namespace {
// the data columns any arm takes from the injector, and each arm's (the slot table's kInjectedCol)
const InjectedCols& injected_cols() {
  using namespace rvwg;
  static const InjectedCols U = [] {
    InjectedCols u{};
    const int16_t* t = rv32im_witgen_slot_table();
    for (uint32_t c = 0; c < kDataCols; c++) {
      bool inj = false;
      for (uint32_t k = 0; k < kMajors; k++)
        if (uint32_t(t[k * kDataCols + c]) & kInjectedCol) {
          inj = true;
          u.arm_mask[k][c >> 5] |= 1u << (c & 31);
        }
      if (inj) u.col[u.n++] = uint8_t(c);
    }
    return u;
  }();
  return U;
}
}  // namespace

void rv32im_prover_groups_fill(hipStream_t s, uint32_t* data, uint32_t* code, uint32_t* accum, size_t rows,
                               size_t accum_cols) {
  using namespace rvwg;
  R0_REQUIRE(rows >= 4 && rows <= (size_t(1) << 24) && (rows & (rows - 1)) == 0,
             "rv32im_prover_groups_fill: bad shape");
  // accum: the machine columns phase 3 adds the previous row's totals to (kUserAccumSplit = 23 up
  // to the last group, rv32im-sys/kernels/cxx/ffi.cpp:341-356) stay INVALID as the reference
  // leaves the cells stepAccum does not write (INVALID + total is what it stores there); every
  // other accum cell is written by the step or is INVALID only to be zeroized, so it starts 0
  R0_REQUIRE(accum_cols == 103, "rv32im_prover_groups_fill: the rv32im accum group has 103 columns");
  const uint32_t acc_inv_begin = 23, acc_inv_end = 23 + 4 * ((103 - 23) / 4 - 1);
  const InjectedCols& U = injected_cols();
  KScope ks("rv32im_groups_init", double(rows) * 4.0 * (U.n + 1 + accum_cols));
  hipLaunchKernelGGL(prover_groups_fill_kernel, dim3(uint32_t((rows + kMergeThreads - 1) / kMergeThreads)),
                     dim3(kMergeThreads), 0, s, data, code, accum, uint32_t(rows), uint32_t(accum_cols), U,
                     acc_inv_begin, acc_inv_end);
  HIP_OK(hipGetLastError());
}

void rv32im_prover_inject(hipStream_t s, uint32_t* data, size_t rows, const uint32_t* index, const uint32_t* offsets,
                          const uint32_t* values, size_t inj_rows, uint64_t limit, const rvwg::PreflightCycle* d_cycles,
                          uint32_t* err) {
  R0_REQUIRE(rows >= 4 && rows <= (size_t(1) << 24) && (rows & (rows - 1)) == 0 && inj_rows <= rows,
             "rv32im_prover_inject: bad shape");
  if (inj_rows == 0) return;
  KScope ks("rv32im_groups_init", double(inj_rows) * 8.0);
  hipLaunchKernelGGL(prover_inject_kernel, dim3(uint32_t((inj_rows + kMergeThreads - 1) / kMergeThreads)),
                     dim3(kMergeThreads), 0, s, data, uint32_t(rows), injected_cols(), index, offsets, values,
                     uint32_t(inj_rows), limit, d_cycles, uint32_t(__builtin_ctzll(rows)), err);
  HIP_OK(hipGetLastError());
}

void rv32im_witgen_dev(hipStream_t s, uint32_t mode, uint32_t* data, uint32_t* global, size_t rows,
                       const rvwg::PreflightCycle* d_cycles, const rvwg::MemoryTxn* d_txns, size_t n_txns,
                       const uint8_t* d_bigint, size_t n_bigint, uint32_t table_split, uint32_t last_cycle,
                       bool zeroize, const uint32_t* extra_err, const std::function<void()>& reinit) {
  using namespace rvwg;
  R0_REQUIRE(mode <= 2, "rv32im_witgen: mode must be 0 (parallel), 1 (forward) or 2 (reverse)");
  R0_REQUIRE(rows >= 4 && (rows & (rows - 1)) == 0 && rows <= (size_t(1) << 24),
             "rv32im_witgen: rows must be a power of two in [4, 2^24]");
  R0_REQUIRE(last_cycle <= rows && table_split <= last_cycle, "rv32im_witgen: need tableSplitCycle <= lastCycle <= rows");
  R0_REQUIRE((last_cycle == 0 || d_cycles) && (n_txns == 0 || d_txns) && (n_bigint == 0 || d_bigint),
             "rv32im_witgen: null trace array with a nonzero count");
  R0_REQUIRE(n_txns < (size_t(1) << 32) && n_bigint < (size_t(1) << 32), "rv32im_witgen: trace too long");
  if (last_cycle == 0) {
    if (zeroize) eltwise_zeroize(s, data, rows * kDataCols);
    return;
  }
  // lookup tables, error record, bucket counts and a zero transaction record / bigint byte (what
  // an empty trace's pointers show the kernels) in one scratch block
  constexpr size_t kTabWords = 256 + 65536 + 4 + kBins + 8;
  auto* tab = static_cast<uint32_t*>(scratch(kTabWords * 4, kSlotRvwgTables));
  auto* d_list = static_cast<uint32_t*>(scratch(size_t(last_cycle) * 4, kSlotRvwgLists));
  HIP_OK(hipMemsetD32Async(tab, 0, kTabWords, s));
  const uint32_t* zero_rec = tab + 256 + 65536 + 4 + kBins;
  Args A{};
  A.data = data;
  A.global = global;
  A.rows = uint32_t(rows);
  A.ncycles = last_cycle;
  A.cycles = d_cycles;
  A.txns = n_txns ? d_txns : reinterpret_cast<const MemoryTxn*>(zero_rec);
  A.n_txns = uint32_t(n_txns);
  A.bigint = n_bigint ? d_bigint : reinterpret_cast<const uint8_t*>(zero_rec);
  A.n_bigint = uint32_t(n_bigint);
  A.u8 = tab;
  A.u16 = tab + 256;
  A.err = tab + 256 + 65536;
  uint32_t* counts = A.err + 4;
  const uint32_t g = (last_cycle + kBucketThreads - 1) / kBucketThreads;
  // the two phases' cycles bucketed by instruction arm: counts (one read-back for the launch
  // sizes), then a stable radix sort of (bin, cycle): each bucket in cycle order, so a wave's
  // lanes read nearby transactions and injected rows
  const size_t kb_bytes = (size_t(last_cycle) * 2 + 15) & ~size_t(15);
  auto* kb = static_cast<uint8_t*>(scratch(kb_bytes + size_t(last_cycle) * 8 + 64, kSlotRvwgKeys));
  uint8_t* keys = kb;
  uint8_t* keys_out = kb + last_cycle;
  uint32_t* vals = reinterpret_cast<uint32_t*>(kb + kb_bytes);
  uint32_t* pos = vals + last_cycle;
  // each bin's cycles ordered by minor, then cycle: a wavefront's lanes mostly share the arm's
  // minor mux branch (phase 1 at po2=20: 1.27 -> 0.85 ms, the merge's gathers 0.57 -> 0.73 ms;
  // `profiles/r4l_*`). R0_RVWG_MINOR=0 keeps plain cycle order.
  static const uint32_t minor_bits = [] {
    const char* e = std::getenv("R0_RVWG_MINOR");
    return e && e[0] == '0' ? 0u : 3u;
  }();
  static const bool merge_xcd = [] {
    const char* e = std::getenv("R0_RVWG_MERGE_XCD");
    return !(e && e[0] == '0');
  }();
  uint32_t h[4 + kBins], h_init[4] = {0, 0, 0, 0};
  {
    KScope ks("rv32im_witgen_bucket", double(last_cycle) * 2 * sizeof(PreflightCycle));
    hipLaunchKernelGGL(bucket_count_kernel, dim3(g), dim3(kBucketThreads), 0, s, A, table_split, counts, keys, vals,
                       minor_bits);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(h, A.err, sizeof(h), hipMemcpyDeviceToHost, s));  // err[0..2], pad, counts
    if (extra_err) HIP_OK(hipMemcpyAsync(h_init, extra_err, sizeof(h_init), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
  }
  R0_REQUIRE(h_init[0] == 0, "rv32im witgen: " + witgen_error(h_init));
  R0_REQUIRE(h[0] == 0, "rv32im witgen: " + witgen_error(h));
  // the prover's injector set a word in a column its row's arm does not take from the injector:
  // the group is re-initialised whole (INVALID, the injector scattered in, as the reference
  // prepares it) and the merge reads every column back and checks it as Buffer::set does
  bool full = !zeroize;
  if (zeroize && h_init[3]) {
    R0_REQUIRE(static_cast<bool>(reinit), "rv32im witgen: injector outside the arms' columns and no re-initialisation");
    reinit();
    full = true;
  }
  const uint32_t* cnt = h + 4;  // counts start at A.err + 4
  BinTable T{};
  T.minor_bits = minor_bits;
  T.off[0] = 0;
  size_t cwords = 0;
  for (uint32_t k = 0; k < kMajors; k++) T.nslots[k] = rv32im_witgen_nslots(k);
  for (uint32_t b = 0; b < kBins; b++) {
    T.off[b + 1] = T.off[b] + cnt[b];
    T.cnt[b] = cnt[b];
    T.cbase[b] = cwords;
    const uint32_t ns = T.nslots[b % kMajors];
    cwords += size_t(ns + (ns + 31) / 32) * cnt[b];  // the slots, then the lanes' mask words
  }
  R0_REQUIRE(T.off[kBins] == last_cycle, "rv32im witgen: bucket counts do not add up");
  size_t temp_bytes = 0;
  const int end_bit = 5 + int(minor_bits);
  HIP_OK(hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, keys, keys_out, vals, d_list, int(last_cycle), 0,
                                            end_bit, s));
  void* temp = scratch(temp_bytes + 256, kSlotRvwgSortTemp);
  HIP_OK(hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys, keys_out, vals, d_list, int(last_cycle), 0,
                                            end_bit, s));
  hipLaunchKernelGGL(bin_pos_kernel, dim3(g), dim3(kBucketThreads), 0, s, d_list, keys_out, last_cycle, T, pos);
  HIP_OK(hipGetLastError());
  // the arms' compact values (read only where a lane's mask says stored: no fill)
  auto* cbuf = static_cast<uint32_t*>(scratch(cwords * 4 + 16, kSlotRvwgCompact));
  for (int p = 0; p < 2; p++) {
    KScope ks(p ? "rv32im_witgen_tables" : "rv32im_witgen_exec",
              double(T.off[(p + 1) * kMajors] - T.off[p * kMajors]) * (4.0 * 211 + sizeof(PreflightCycle)));
    for (uint32_t k = 0; k < kMajors; k++) {
      const uint32_t b = p * kMajors + k;
      rv32im_witgen_major(k, s, A, d_list + T.off[b], T.cnt[b], cbuf + T.cbase[b]);
    }
  }
  {
    // the slot table (constant, 5.5 KB) into this thread's scratch
    const size_t slot_bytes = size_t(kMajors) * kDataCols * sizeof(int16_t);
    auto* d_slot = static_cast<int16_t*>(scratch(slot_bytes, kSlotRvwgSlotTable));
    upload_async(d_slot, rv32im_witgen_slot_table(), slot_bytes);
    KScope ks("rv32im_witgen_merge", double(rows) * kDataCols * 8.0 + double(cwords) * 4.0);
    hipLaunchKernelGGL(merge_kernel, dim3(uint32_t((rows + kMergeThreads - 1) / kMergeThreads)), dim3(kMergeThreads), 0,
                       s, data, uint32_t(rows), last_cycle, cbuf, keys, pos, d_slot, T, zeroize, full, merge_xcd,
                       A.err);
    HIP_OK(hipGetLastError());
  }
  uint32_t h_err[3] = {0, 0, 0};
  HIP_OK(hipMemcpyAsync(h_err, A.err, 12, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  R0_REQUIRE(h_err[0] == 0, "rv32im witgen: " + witgen_error(h_err));
}

const rvwg::PreflightCycle* rv32im_upload_cycles(const rvwg::PreflightCycle* h_cycles, size_t n) {
  auto* d = static_cast<rvwg::PreflightCycle*>(scratch(n * sizeof(rvwg::PreflightCycle) + 16, kSlotRvwgCycles));
  upload_async(d, h_cycles, n * sizeof(rvwg::PreflightCycle));
  return d;
}

void rv32im_witgen(hipStream_t s, uint32_t mode, uint32_t* data, uint32_t* global, size_t rows,
                   const rvwg::PreflightCycle* h_cycles, const rvwg::MemoryTxn* h_txns, size_t n_txns,
                   const uint8_t* h_bigint, size_t n_bigint, uint32_t table_split, uint32_t last_cycle, bool zeroize,
                   const uint32_t* extra_err, const std::function<void()>& reinit) {
  using namespace rvwg;
  R0_REQUIRE(last_cycle <= rows && last_cycle <= (size_t(1) << 24), "rv32im_witgen: more cycles than rows");
  R0_REQUIRE((last_cycle == 0 || h_cycles) && (n_txns == 0 || h_txns) && (n_bigint == 0 || h_bigint),
             "rv32im_witgen: null trace array with a nonzero count");
  auto* d_cycles = static_cast<PreflightCycle*>(scratch(size_t(last_cycle) * sizeof(PreflightCycle) + 16, kSlotRvwgCycles));
  auto* d_txns = static_cast<MemoryTxn*>(scratch(n_txns * sizeof(MemoryTxn) + 16, kSlotRvwgTxns));
  auto* d_bigint = static_cast<uint8_t*>(scratch(n_bigint + 16, kSlotRvwgBigint));
  upload_async(d_cycles, h_cycles, size_t(last_cycle) * sizeof(PreflightCycle));
  upload_async(d_txns, h_txns, n_txns * sizeof(MemoryTxn));
  upload_async(d_bigint, h_bigint, n_bigint);
  rv32im_witgen_dev(s, mode, data, global, rows, d_cycles, n_txns ? d_txns : nullptr, n_txns,
                    n_bigint ? d_bigint : nullptr, n_bigint, table_split, last_cycle, zeroize, extra_err, reinit);
}

}  // namespace r0
