// Shared by the generated recursion witness-generation kernels (tools/gen_witgen.py ->
// gen/rwitgen/*.hip) and their driver (recursion_witgen.hip): the argument block and the
// device side of the reference's externs (recursion-sys/kernels/cxx/extern.cpp).
#pragma once
#include "bb31.h"
#include "runtime.h"

namespace r0 {
namespace rwg {

constexpr uint32_t kWitgenThreads = 128;
constexpr uint32_t kMaxWomRows = 9;             // kMaxWomRowsPerCycle (context.h)
constexpr uint32_t kInvalidWord = 0xFFFFFFFFu;  // Fp::invalid()
constexpr uint32_t kRowWords = 5;               // WomArgumentRow: addr (plain), value (4 words)
// error codes (A.err[0]); A.err[1] is the cycle
constexpr uint32_t kErrEqz = 0x10000u;           // + the wom.cpp line of the failed EQZ
constexpr uint32_t kErrCoefficients = 0x20001u;  // extern_readCoefficients (checked bytes)
constexpr uint32_t kErrWomAddr = 0x20002u;       // extern_womRead past the preflight WOM
constexpr uint32_t kErrWomRows = 0x20003u;       // more than kMaxWomRows argument rows in a cycle
constexpr uint32_t kErrIop = 0x20004u;           // extern_readIOPBody past the preflight IOP values

struct WitgenArgs {
  const uint32_t* ctrl;  // args[0]
  uint32_t* global;      // args[1]
  uint32_t* data;        // args[2]
  uint32_t steps;        // rows of every group (total cycles, a power of two)
  uint32_t ncycles;      // work cycles (the program's rows)
  const uint32_t* run_start;  // nruns + 1 entries: runs of cycles for exec
  uint32_t nruns;
  const uint32_t* wom;  // preflight WOM, 4 words per address
  uint32_t n_wom;
  const uint32_t* iops;  // preflight IOP values, 4 words each
  uint32_t n_iops;
  const uint32_t* iop_idx;  // per cycle: its first IOP value (PreflightCycle::iopIdx)
  uint32_t* rows;           // ncycles x kMaxWomRows argument rows (exec), kRowWords each
  uint32_t* wom_count;      // per cycle: rows written (exec)
  const uint32_t* wom_index;  // per cycle: its first sorted row (exclusive scan of wom_count)
  const uint32_t* sorted;     // the rows sorted (verify)
  uint32_t* err;              // [code, cycle]; 0 = none
};

// Fp::asUInt32 / Fp(uint32_t)
__device__ __forceinline__ uint32_t fp_to_u32(uint32_t x) { return mont_reduce(x); }
__device__ __forceinline__ uint32_t fp_from_u32(uint32_t v) { return fp_mul(v % kP, kR2); }

__device__ __forceinline__ void fail(const WitgenArgs& A, uint32_t code, uint32_t cycle) {
  if (atomicCAS(A.err, 0u, code) == 0u) A.err[1] = cycle;
}

// extern_womRead: the preflight's write-once memory at addr.asUInt32()
__device__ __forceinline__ void wom_read(const WitgenArgs& A, uint32_t cycle, uint32_t addr_word, uint32_t& d0,
                                         uint32_t& d1, uint32_t& d2, uint32_t& d3) {
  const uint32_t addr = fp_to_u32(addr_word);
  if (addr >= A.n_wom) {
    fail(A, kErrWomAddr, cycle);
    d0 = d1 = d2 = d3 = 0u;
    return;
  }
  const uint4 v = *reinterpret_cast<const uint4*>(A.wom + uint64_t(addr) * 4);
  d0 = v.x;
  d1 = v.y;
  d2 = v.z;
  d3 = v.w;
}

// extern_plonkWrite_wom: the cycle's next WOM argument row (addr stored as a plain integer)
__device__ __forceinline__ void plonk_write(const WitgenArgs& A, uint32_t cycle, uint32_t& nrow, uint32_t addr_word,
                                            uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3) {
  if (nrow >= kMaxWomRows) {
    fail(A, kErrWomRows, cycle);
    return;
  }
  uint32_t* r = A.rows + (uint64_t(cycle) * kMaxWomRows + nrow) * kRowWords;
  r[0] = fp_to_u32(addr_word);
  r[1] = v0;
  r[2] = v1;
  r[3] = v2;
  r[4] = v3;
  nrow++;
}

// extern_plonkRead_wom: the next sorted row, its address as an Fp
__device__ __forceinline__ void plonk_read(const WitgenArgs& A, uint32_t& rd, uint32_t& d0, uint32_t& d1,
                                           uint32_t& d2, uint32_t& d3, uint32_t& d4) {
  const uint32_t* r = A.sorted + uint64_t(rd) * kRowWords;
  d0 = fp_from_u32(r[0]);
  d1 = r[1];
  d2 = r[2];
  d3 = r[3];
  d4 = r[4];
  rd++;
}

// extern_readIOPBody: trace->iops[cycles[cycle].iopIdx++]
__device__ __forceinline__ void iop_body(const WitgenArgs& A, uint32_t cycle, uint32_t& iop, uint32_t& d0,
                                         uint32_t& d1, uint32_t& d2, uint32_t& d3) {
  if (iop >= A.n_iops) {
    fail(A, kErrIop, cycle);
    d0 = d1 = d2 = d3 = 0u;
    return;
  }
  const uint4 v = *reinterpret_cast<const uint4*>(A.iops + uint64_t(iop) * 4);
  d0 = v.x;
  d1 = v.y;
  d2 = v.z;
  d3 = v.w;
  iop++;
}

}  // namespace rwg

// step_exec over runs[0, n) (indices into A.run_start); maj 1..7: every cycle of those runs has
// major selector column maj (rwg::exec_kernel<maj>), 8: majors other than column 2, 0: any runs
void recursion_witgen_exec(hipStream_t s, const rwg::WitgenArgs& A, int maj, const uint32_t* runs, uint32_t n);
void recursion_witgen_verify(hipStream_t s, const rwg::WitgenArgs& A);

}  // namespace r0
