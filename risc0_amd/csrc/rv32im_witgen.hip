// rv32im witness generation on the GPU: the role of risc0_circuit_rv32im_{cpu,cuda}_witgen
// (rv32im-sys/kernels/cxx/ffi.cpp:230-308, kernels/cuda/ffi.cu:362-470), called from
// WitnessGenerator::hal_generate_witness (circuit/rv32im/src/prove/witgen/mod.rs:135-176)
// after the injector's scatter into the all-INVALID data group.
//
// stepExec runs step_Top (generated from steps.cpp, gen/rvwitgen/witgen_k*.hip) once per
// cycle in two phases, as par_stepExec does: cycles [0, tableSplitCycle) first — their
// lookupDelta calls count the u8/u16 lookup tables with device atomics — then the table and
// done rows [tableSplitCycle, lastCycle), whose lookupCurrent reads those counts. Within a
// phase the cycles are bucketed by their preflight major, and one kernel per instruction arm
// runs step_Top specialised to that arm over its bucket: a wavefront's lanes share the arm.
// Every phase is a set of independent cycles: the rows a step reads at back > 0 are the
// injected ones (cycle, next pc/state/mode, the Poseidon2/SHA/BigInt states), exactly what
// makes the reference's parallel mode well defined. The reference's forward and reverse
// modes give the same words on a trace it accepts (tests/test_rv32im_witgen_ir.py), so every
// mode runs this schedule.
//
// The preflight trace comes from the host, as RawPreflightTrace does (host pointers). Checks
// that throw in the reference record an error code and the cycle, raised after the kernels
// drain.
#include <string>
#include <vector>

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
    default: return "witness generation error " + std::to_string(code) + at;
  }
}

}  // namespace

void rv32im_witgen(hipStream_t s, uint32_t mode, uint32_t* data, uint32_t* global, size_t rows,
                   const rvwg::PreflightCycle* h_cycles, const rvwg::MemoryTxn* h_txns, size_t n_txns,
                   const uint8_t* h_bigint, size_t n_bigint, uint32_t table_split, uint32_t last_cycle) {
  using namespace rvwg;
  R0_REQUIRE(mode <= 2, "rv32im_witgen: mode must be 0 (parallel), 1 (forward) or 2 (reverse)");
  R0_REQUIRE(rows >= 4 && (rows & (rows - 1)) == 0 && rows <= (size_t(1) << 24),
             "rv32im_witgen: rows must be a power of two in [4, 2^24]");
  R0_REQUIRE(last_cycle <= rows && table_split <= last_cycle, "rv32im_witgen: need tableSplitCycle <= lastCycle <= rows");
  R0_REQUIRE((last_cycle == 0 || h_cycles) && (n_txns == 0 || h_txns) && (n_bigint == 0 || h_bigint),
             "rv32im_witgen: null trace array with a nonzero count");
  R0_REQUIRE(n_txns < (size_t(1) << 32) && n_bigint < (size_t(1) << 32), "rv32im_witgen: trace too long");
  if (last_cycle == 0) return;
  // the two phases' cycles bucketed by instruction arm (counting sort on the preflight major)
  std::vector<uint32_t> list(last_cycle);
  uint32_t off[2][kMajors + 1] = {};
  for (uint32_t c = 0; c < last_cycle; c++) {
    const uint32_t m = h_cycles[c].major;
    if (m >= kMajors) {
      const uint32_t e[3] = {kErrMajor, c, m};
      R0_REQUIRE(false, "rv32im witgen: " + witgen_error(e));
    }
    off[c >= table_split][m + 1]++;
  }
  for (int p = 0; p < 2; p++) {
    off[p][0] = p ? table_split : 0;
    for (uint32_t k = 0; k < kMajors; k++) off[p][k + 1] += off[p][k];
  }
  {
    uint32_t pos[2][kMajors];
    for (int p = 0; p < 2; p++)
      for (uint32_t k = 0; k < kMajors; k++) pos[p][k] = off[p][k];
    for (uint32_t c = 0; c < last_cycle; c++) list[pos[c >= table_split][h_cycles[c].major]++] = c;
  }
  auto* d_cycles = static_cast<PreflightCycle*>(scratch(size_t(last_cycle) * sizeof(PreflightCycle), kSlotRvwgCycles));
  auto* d_txns = static_cast<MemoryTxn*>(scratch(n_txns * sizeof(MemoryTxn) + 16, kSlotRvwgTxns));
  auto* d_bigint = static_cast<uint8_t*>(scratch(n_bigint + 16, kSlotRvwgBigint));
  auto* d_list = static_cast<uint32_t*>(scratch(size_t(last_cycle) * 4, kSlotRvwgLists));
  auto* d_tables = static_cast<uint32_t*>(scratch((256 + 65536 + 4) * 4, kSlotRvwgTables));
  upload_async(d_cycles, h_cycles, size_t(last_cycle) * sizeof(PreflightCycle));
  upload_async(d_txns, h_txns, n_txns * sizeof(MemoryTxn));
  upload_async(d_bigint, h_bigint, n_bigint);
  upload_async(d_list, list.data(), size_t(last_cycle) * 4);
  HIP_OK(hipMemsetD32Async(d_tables, 0, 256 + 65536 + 4, s));

  Args A{};
  A.data = data;
  A.global = global;
  A.rows = uint32_t(rows);
  A.ncycles = last_cycle;
  A.cycles = d_cycles;
  A.txns = d_txns;
  A.n_txns = uint32_t(n_txns);
  A.bigint = d_bigint;
  A.n_bigint = uint32_t(n_bigint);
  A.u8 = d_tables;
  A.u16 = d_tables + 256;
  A.err = d_tables + 256 + 65536;
  for (int p = 0; p < 2; p++) {
    KScope ks(p ? "rv32im_witgen_tables" : "rv32im_witgen_exec",
              double(off[p][kMajors] - off[p][0]) * (4.0 * 211 + sizeof(PreflightCycle)));
    for (uint32_t k = 0; k < kMajors; k++)
      rv32im_witgen_major(k, s, A, d_list + off[p][k], off[p][k + 1] - off[p][k]);
  }
  uint32_t h_err[3] = {0, 0, 0};
  HIP_OK(hipMemcpyAsync(h_err, A.err, 12, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  R0_REQUIRE(h_err[0] == 0, "rv32im witgen: " + witgen_error(h_err));
}

}  // namespace r0
