// ORACLE (test infrastructure only). Thin C-ABI glue over the reference's own
// generated C++ constraint code, compiled from the sources where they lie under
// /root/reference by oracle/Makefile into oracle/_ref/ (never copied, never shipped).
//   rv32im   : risc0/circuit/rv32im-sys/kernels/cxx/rust_poly_fp_{0..3}.cpp
//   recursion: risc0/circuit/recursion-sys/kernels/cxx/poly_fp.cpp
#include "fp.h"
#include "fpext.h"

#include <cstdint>
#include <cstring>
#include <exception>

using namespace risc0;

namespace risc0::circuit::rv32im_v2 {
FpExt poly_fp(size_t cycle, size_t steps, FpExt* poly_mix, Fp** args);
}
namespace risc0::circuit::recursion {
FpExt poly_fp(size_t cycle, size_t steps, FpExt* poly_mix, Fp** args);
}

template <FpExt (*F)(size_t, size_t, FpExt*, Fp**)>
static const char* wrap(size_t cycle, size_t steps, const uint32_t* poly_mix, const uint32_t** args,
                        uint32_t* result) {
  try {
    FpExt r = F(cycle, steps, (FpExt*)poly_mix, (Fp**)args);
    memcpy(result, &r, 16);
  } catch (const std::exception& e) {
    return strdup(e.what());
  }
  return nullptr;
}

extern "C" const char* ref_rv32im_poly_fp(size_t c, size_t s, const uint32_t* pm, const uint32_t** a,
                                          uint32_t* r) {
  return wrap<risc0::circuit::rv32im_v2::poly_fp>(c, s, pm, a, r);
}
extern "C" const char* ref_recursion_poly_fp(size_t c, size_t s, const uint32_t* pm,
                                             const uint32_t** a, uint32_t* r) {
  return wrap<risc0::circuit::recursion::poly_fp>(c, s, pm, a, r);
}
