// Host-side seal verifier: the STARK verifier of risc0-zkp, natively, so a host can check
// a seal from r0hip_prove_segment(s) before it leaves the process (the reference prover
// verifies its own receipts, zkvm/src/host/server/prove/prover_impl.rs:165-170).
//   verify            risc0/zkp/src/verify/mod.rs:500-560 (+ rv32im version word, circuit/rv32im/src/lib.rs:78-92)
//   groups            mod.rs:201-244
//   the rest          verify_core.h (read IOP, Merkle, verify_validity, FRI)
// Everything the reference checks is checked: transcript replay, the validity equation
// (mod.rs:340-394, with poly_ext run from the circuit's constraint program), every Merkle
// path, every FRI fold, the final polynomial and the seal length, plus the check_code hook
// (mod.rs:531): the code (control) root is returned, and when the caller passes an allow-list
// the root must be in it. Field words in the seal must be canonical (read_field_elem_slice).
// r0hip_testing_verify_seal_structure skips the validity equation for seals of synthetic
// witnesses, which do not satisfy the constraints; it is for tests, never for receipts.
// Host code only — no HIP call, so it runs without a GPU.
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/r0hip.h"
#include "circuit.h"
#include "runtime.h"
#include "verify_core.h"

namespace r0 {

// PolyExt::poly_ext (the circuits' generated poly_ext.rs, e.g. circuit/recursion/src/poly_ext.rs,
// as called by verify_validity, zkp/src/verify/mod.rs:356-386): the constraint polynomial at
// the out-of-domain point from the tap evaluations, by running the circuit's flattened program
// (CircuitDef::ir, from <c>.poly.ir) over FpExt. mix/global are Montgomery words; eval_u holds
// one value per tap in tap order.
FpExt poly_ext(const CircuitDef& c, const uint32_t* mix, const uint32_t* global, const FpExt* eval_u,
               FpExt poly_mix) {
  std::vector<FpExt> pows(c.n_poly_mix);
  for (size_t k = 0; k < c.n_poly_mix; k++) pows[k] = fe_pow(poly_mix, c.poly_mix_powers[k]);
  std::vector<FpExt> val(c.n_ir);
  for (size_t k = 0; k < c.n_ir; k++) {
    const uint32_t* r = c.ir + 6 * k;
    FpExt& v = val[r[1]];
    switch (r[0]) {
      case 0: v = fe_from_fp(r[2]); break;                              // c: constant
      case 1: v = FpExt{{r[2], r[3], r[4], r[5]}}; break;               // e: extension constant
      case 2: v = eval_u[r[2]]; break;                                   // l: tap
      case 3: v = fe_from_fp((r[2] ? global : mix)[r[3]]); break;        // g: mix / global word
      case 4: v = fe_add(val[r[2]], val[r[3]]); break;
      case 5: v = fe_sub(val[r[2]], val[r[3]]); break;
      case 6: v = fe_mul(val[r[2]], val[r[3]]); break;
      case 7: v = fe_add(val[r[2]], fe_mul(val[r[3]], pows[r[4]])); break;  // a: acc + x * mix^k
      case 8: v = fe_add(val[r[2]], fe_mul(fe_mul(val[r[3]], val[r[4]]), pows[r[5]])); break;
      case 9: return v;  // r: result (the record names the value in its dst slot)
      default: throw std::runtime_error("r0hip: bad constraint program record");
    }
  }
  throw std::runtime_error("r0hip: constraint program has no result");
}

namespace {
using namespace vfy;

uint32_t verify_seal(const CircuitDef& c, int suite, const uint32_t* seal, size_t len, bool check_validity,
                     const uint32_t* code_roots, size_t n_code_roots, uint32_t* code_root_out) {
  if (c.name == std::string("rv32im")) {  // rv32im/src/lib.rs:78-92: a version word leads the seal
    if (len < 1 || seal[0] != 2) throw VerifyError("bad rv32im seal version");
    seal++;
    len--;
  }
  ReadIOP iop(seal, len, suite);
  iop.defer = true;  // openings hashed after the transcript, on several threads (check_pending)
  uint32_t psi[16], ci[16];
  for (int i = 0; i < 16; i++) {
    psi[i] = fp_encode(uint8_t(PROOF_SYSTEM_INFO[i]));
    ci[i] = fp_encode(uint8_t(c.circuit_info[i]));
  }
  iop.commit(hash_elems(suite, psi, 16));
  iop.commit(hash_elems(suite, ci, 16));
  const uint32_t* header = iop.read_elems(c.output_size + 1);
  iop.commit(hash_elems(suite, header, c.output_size + 1));
  const uint32_t po2 = header[c.output_size];
  if (po2 < 2 || po2 > 24) throw VerifyError("po2 out of range");
  const size_t domain = INV_RATE * (size_t(1) << po2);
  // groups in commit order: code, data, then (after the mix draw) accum (mod.rs:215-244)
  MerkleVerifier code(iop, domain, c.group_sizes[1]);
  // check_code(po2, code_root) (mod.rs:531): e.g. the recursion control-id inclusion check
  // (zkvm/src/receipt/succinct.rs:143-157) is made against the allow-list the caller passes
  if (code_root_out) memcpy(code_root_out, code.root.w, 32);
  if (n_code_roots) {
    bool found = false;
    for (size_t i = 0; i < n_code_roots && !found; i++) found = same(digest_of(code_roots + 8 * i), code.root);
    if (!found) throw VerifyError("code root is not in the allowed set");
  }
  MerkleVerifier data(iop, domain, c.group_sizes[2]);
  std::vector<uint32_t> mix(c.mix_size);
  for (auto& m : mix) m = iop.rng->random_elem();
  MerkleVerifier accum(iop, domain, c.group_sizes[0]);
  const MerkleVerifier* groups[3] = {&accum, &code, &data};
  const TapView taps{c.taps, c.n_taps, c.combo_taps, c.combo_begin, c.combos_count};
  verify_validity_and_fri(iop, taps, po2, groups, check_validity, [&](FpExt poly_mix, const FpExt* eval_u) {
    return poly_ext(c, mix.data(), header, eval_u, poly_mix);
  });
  return po2;
}

}  // namespace
}  // namespace r0

using namespace r0;

static const char* verify_entry(const char* circuit, int suite, const uint32_t* seal, size_t seal_len,
                                bool check_validity, const uint32_t* code_roots, size_t n_code_roots,
                                uint32_t* code_root_out, uint32_t* po2_out) {
  try {
    const CircuitDef* c = find_circuit(circuit ? circuit : "");
    R0_REQUIRE(c, std::string("unknown circuit ") + (circuit ? circuit : "(null)"));
    R0_REQUIRE(suite >= 0 && suite <= 2, "unknown hash suite");
    R0_REQUIRE(seal || seal_len == 0, "seal is NULL");
    R0_REQUIRE(code_roots || n_code_roots == 0, "code_roots is NULL");
    uint32_t po2 = verify_seal(*c, suite, seal, seal_len, check_validity, code_roots, n_code_roots, code_root_out);
    if (po2_out) *po2_out = po2;
    return nullptr;
  } catch (const std::exception& e) {
    return strdup(e.what());
  } catch (...) {
    return strdup("r0hip: unknown error");
  }
}

extern "C" const char* r0hip_verify_seal(const char* circuit, int suite, const uint32_t* seal, size_t seal_len,
                                         const uint32_t* h_code_roots, size_t n_code_roots,
                                         uint32_t* h_code_root_out, uint32_t* po2_out) {
  return verify_entry(circuit, suite, seal, seal_len, true, h_code_roots, n_code_roots, h_code_root_out, po2_out);
}

extern "C" const char* r0hip_testing_verify_seal_structure(const char* circuit, int suite, const uint32_t* seal,
                                                           size_t seal_len, uint32_t* po2_out) {
  return verify_entry(circuit, suite, seal, seal_len, false, nullptr, 0, nullptr, po2_out);
}

extern "C" const char* r0hip_poly_ext(const char* circuit, const uint32_t* h_mix, const uint32_t* h_global,
                                      const uint32_t* h_eval_u, const uint32_t* h_poly_mix, uint32_t* h_out) {
  try {
    const CircuitDef* c = find_circuit(circuit ? circuit : "");
    R0_REQUIRE(c, std::string("unknown circuit ") + (circuit ? circuit : "(null)"));
    R0_REQUIRE(h_mix && h_global && h_eval_u && h_poly_mix && h_out, "poly_ext: null argument");
    std::vector<FpExt> eval_u(c->n_taps);
    for (size_t i = 0; i < c->n_taps; i++) eval_u[i] = vfy::load_ext(h_eval_u + 4 * i);
    FpExt r = poly_ext(*c, h_mix, h_global, eval_u.data(), vfy::load_ext(h_poly_mix));
    memcpy(h_out, r.c, 16);
    return nullptr;
  } catch (const std::exception& e) {
    return strdup(e.what());
  } catch (...) {
    return strdup("r0hip: unknown error");
  }
}
