// rv32im BigInt accumulation states: the host half of the witness generator's accum step.
//
// Before the per-cycle accumulation runs, the reference computes, on the host and with the
// final mix drawn from the transcript, the running BigInt accumulator state (poly, term,
// total: three FpExt) after every Back::BigInt cycle of the preflight trace, and scatters
// those 12 words into accum columns 0..11 of the cycle's row
// (circuit/rv32im/src/prove/witgen/mod.rs:178-205; BigIntAccum::{new,step},
// witgen/byte_poly.rs:381-470; offsets :362-377). The generated step code then reads the
// previous cycle's state at back 1 (rv32im.accum.ir), which is why it must be in place before
// the step kernels run on all cycles at once.
//
// The recurrence is sequential and tiny (a few FpExt products per BigInt cycle), so it stays
// on the host as in the reference; only the scatter of the states is a kernel (accum.hip).
#include <string>
#include <vector>

#include "../../include/r0hip.h"
#include "bb31.h"
#include "runtime.h"

namespace r0 {

namespace {
constexpr int kWidthBytes = 16;  // BIGINT_WIDTH_BYTES (risc0_circuit_rv32im::execute::bigint)
constexpr size_t kMixWords = 36; // REGCOUNT_MIX

FpExt fe_u32(uint32_t v) { return fe_from_fp(fp_encode(v)); }  // ExtVal::from_u32
}  // namespace

// byte_poly.rs:381-470, restated over this library's field code; one state per record
std::vector<uint32_t> rv32im_bigint_accum_states(const uint32_t* mix, const r0hip_bigint_back* backs, size_t n,
                                                 size_t rows) {
  // the final mix (witgen/mod.rs:184: mix[mix.len() - 4..])
  const FpExt last_mix{{mix[kMixWords - 4], mix[kMixWords - 3], mix[kMixWords - 2], mix[kMixWords - 1]}};
  FpExt powers[kWidthBytes + 1];  // MAX_POWERS = BIGINT_WIDTH_BYTES + 1
  FpExt cur = fe_one();
  for (auto& p : powers) {
    p = cur;
    cur = fe_mul(cur, last_mix);
  }
  FpExt neg_poly = fe_zero();
  for (int i = 0; i < kWidthBytes; i++) neg_poly = fe_add(neg_poly, fe_mul(powers[i], fe_u32(128)));
  FpExt poly = fe_zero(), term = fe_one(), total = fe_zero();  // BigIntAccumState::new
  auto reset = [&] {
    poly = fe_zero();
    term = fe_one();
    total = fe_zero();
  };
  std::vector<uint32_t> out(n * 12);
  for (size_t k = 0; k < n; k++) {
    const r0hip_bigint_back& b = backs[k];
    R0_REQUIRE(b.row < rows, "bigint back: row " + std::to_string(b.row) + " outside the segment");
    R0_REQUIRE(k == 0 || b.row > backs[k - 1].row, "bigint backs must be in increasing row order (trace order)");
    FpExt delta = fe_zero();
    for (int i = 0; i < kWidthBytes; i++) delta = fe_add(delta, fe_mul(powers[i], fe_u32(b.bytes[i])));
    const FpExt new_poly = fe_add(poly, delta);
    switch (b.poly_op) {
      case 0:  // Reset
        reset();
        break;
      case 1:  // Shift
        poly = fe_mul(new_poly, powers[kWidthBytes]);
        break;
      case 2:  // SetTerm
        poly = fe_zero();
        term = new_poly;
        break;
      case 3: {  // AddTotal
        const FpExt coeff = fe_sub(fe_u32(b.coeff), fe_u32(4));
        total = fe_add(total, fe_mul(fe_mul(coeff, term), new_poly));
        poly = fe_zero();
        term = fe_one();
        break;
      }
      case 4:  // Carry1
        poly = fe_add(poly, fe_mul(fe_sub(delta, neg_poly), fe_u32(64 * 256)));
        break;
      case 5:  // Carry2
        poly = fe_add(poly, fe_mul(delta, fe_u32(256)));
        break;
      case 6: {  // EqZero
        const FpExt carry = fe_sub(powers[1], fe_u32(256));
        const FpExt goal = fe_add(total, fe_mul(new_poly, carry));
        R0_REQUIRE(fe_eq(goal, fe_zero()), "Invalid eqz in bigint accum (row " + std::to_string(b.row) + ")");
        reset();
        break;
      }
      default:
        R0_REQUIRE(false, "bigint back: invalid poly_op " + std::to_string(b.poly_op));
    }
    // BigIntAccumState::as_array order: poly, term, total (offsets 0..11)
    for (int i = 0; i < 4; i++) {
      out[k * 12 + i] = poly.c[i];
      out[k * 12 + 4 + i] = term.c[i];
      out[k * 12 + 8 + i] = total.c[i];
    }
  }
  return out;
}

// the injection itself: states computed above, then one lane per record writes its 12 words
void rv32im_bigint_inject(hipStream_t s, uint32_t* accum, size_t rows, const uint32_t* mix,
                          const r0hip_bigint_back* backs, size_t n) {
  if (n == 0) return;
  R0_REQUIRE(backs, "bigint backs: null pointer with a nonzero count");
  std::vector<uint32_t> states = rv32im_bigint_accum_states(mix, backs, n, rows);
  std::vector<uint32_t> row_of(n);
  for (size_t k = 0; k < n; k++) row_of[k] = backs[k].row;
  uint32_t* d_rows = static_cast<uint32_t*>(scratch(n * 4, kSlotBigIntRows));
  uint32_t* d_states = static_cast<uint32_t*>(scratch(n * 48, kSlotBigIntStates));
  upload_async(d_rows, row_of.data(), n * 4);
  upload_async(d_states, states.data(), n * 48);
  bigint_scatter(s, accum, rows, d_rows, d_states, n);
}

}  // namespace r0
