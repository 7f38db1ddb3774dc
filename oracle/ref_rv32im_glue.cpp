// ORACLE (test infrastructure only). C-ABI glue over the reference's rv32im witness /
// accumulation C++ (risc0/circuit/rv32im-sys/kernels/cxx/ffi.cpp + steps.cpp), compiled
// from the sources where they lie under /root/reference by oracle/Makefile into
// oracle/_ref/libref_rv32im_accum.so (never copied, never shipped).
//   risc0_circuit_rv32im_cpu_accum (ffi.cpp:313-368) is exported by ffi.cpp itself: phase 1
//   (stepAccum per cycle), phase 2 (inclusive scan of the last 4 accum columns), phase 3
//   (the previous row's totals added to every machine accum column).
//   ref_rv32im_accum_phase1 below runs phase 1 alone (the same stepAccum, ffi.cpp:238-247,
//   sequentially), so a test can feed its output to an implementation of phases 2-3 and
//   compare with the reference's whole function.
#include "preflight.h"
#include "tables.h"
#include "witgen.h"

#include <cstdint>
#include <cstring>
#include <exception>

namespace risc0::circuit::rv32im_v2::cpu {
void stepAccum(AccumBuffers& buffers, PreflightTrace& preflight, LookupTables& tables, size_t cycle);
}

using namespace risc0::circuit::rv32im_v2::cpu;

extern "C" const char* ref_rv32im_accum_phase1(AccumBuffers* buffers, uint32_t last_cycle) {
  try {
    PreflightTrace preflight{};
    LookupTables tables;
    for (uint32_t cycle = 0; cycle < last_cycle; cycle++) stepAccum(*buffers, preflight, tables, cycle);
  } catch (const std::exception& e) {
    return strdup(e.what());
  } catch (...) {
    return strdup("unknown exception");
  }
  return nullptr;
}
