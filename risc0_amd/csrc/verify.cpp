// Host-side seal verifier: the STARK verifier of risc0-zkp, natively, so a host can check
// a seal from r0hip_prove_segment(s) before it leaves the process (the reference prover
// verifies its own receipts, zkvm/src/host/server/prove/prover_impl.rs:165-170).
//   transcript        risc0/zkp/src/verify/read_iop.rs:20-84
//   verify            risc0/zkp/src/verify/mod.rs:500-560 (+ rv32im version word, circuit/rv32im/src/lib.rs:78-92)
//   groups / checks   mod.rs:201-244, 292-474
//   DEEP-ALI taps     mod.rs:246-290 (fri_eval_taps)
//   Merkle openings   risc0/zkp/src/verify/merkle.rs:79-186 with zkp/src/merkle.rs:36-66 params
//   FRI               risc0/zkp/src/verify/fri.rs:36-155
// Everything the reference checks is checked: transcript replay, the validity equation
// (mod.rs:340-394, with poly_ext run from the circuit's constraint program), every Merkle
// path, every FRI fold, the final polynomial and the seal length. The validity check can be
// switched off for seals of synthetic witnesses, which do not satisfy the constraints.
// Host code only — no HIP call, so it runs without a GPU.
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/r0hip.h"
#include "circuit.h"
#include "runtime.h"
#include "transcript.h"

namespace r0 {
namespace {

constexpr size_t INV_RATE = 4, QUERIES = 50, FRI_FOLD = 16, FRI_MIN_DEGREE = 256, CHECK_SIZE = 16;
const char PROOF_SYSTEM_INFO[] = "RISC0_STARK:v1__";  // adapter.rs:120

struct VerifyError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

size_t lg2(size_t v) {
  size_t r = 0;
  while ((size_t(1) << r) < v) r++;
  return r;
}

Digest digest_of(const uint32_t* w) {
  Digest d;
  memcpy(d.w, w, 32);
  return d;
}

bool same(const Digest& a, const Digest& b) { return memcmp(a.w, b.w, 32) == 0; }

Digest hash_pair(int suite, const Digest& a, const Digest& b) {
  if (suite == 1) return sha::hash_pair(a, b);
  if (suite == 2) {
    Digest d;
    p254_hash_pair(a.w, b.w, d.w);
    return d;
  }
  uint32_t both[16];  // poseidon2: the unpadded hash of a || b (poseidon2/mod.rs:247-255)
  memcpy(both, a.w, 32);
  memcpy(both + 8, b.w, 32);
  return p2_hash_words(both, 16);
}

// read_iop.rs: a cursor over the seal plus the Fiat-Shamir RNG
struct ReadIOP {
  const uint32_t* words;
  size_t size, pos = 0;
  int suite;
  std::unique_ptr<Rng> rng;
  ReadIOP(const uint32_t* w, size_t n, int s) : words(w), size(n), suite(s), rng(make_rng(s)) {}
  const uint32_t* read(size_t n) {
    if (n > size - pos) throw VerifyError("seal too short");
    const uint32_t* p = words + pos;
    pos += n;
    return p;
  }
  void commit(const Digest& d) { rng->mix(d); }
};

// verify/merkle.rs:79-186: reads the top layer, recomputes the nodes above it, commits the root
struct MerkleVerifier {
  size_t rows, cols, top_size = 1;
  std::vector<Digest> top, rest;  // rest[i], 1 <= i < top_size
  Digest root;

  MerkleVerifier(ReadIOP& iop, size_t row_size, size_t col_size) : rows(row_size), cols(col_size) {
    const size_t layers = lg2(rows);
    size_t top_layer = 0;
    for (size_t i = 1; i < layers; i++) {
      if ((size_t(1) << i) > QUERIES) break;
      top_layer = i;
    }
    top_size = size_t(1) << top_layer;
    const uint32_t* t = iop.read(top_size * 8);
    for (size_t i = 0; i < top_size; i++) top.push_back(digest_of(t + 8 * i));
    rest.resize(top_size);
    for (size_t i = top_size; i-- > top_size / 2;)
      rest[i] = hash_pair(iop.suite, top[2 * i - top_size], top[2 * i + 1 - top_size]);
    for (size_t i = top_size / 2; i-- > 1;) rest[i] = hash_pair(iop.suite, rest[2 * i], rest[2 * i + 1]);
    root = top_size > 1 ? rest[1] : top[0];
    iop.commit(root);
  }

  // opens row `idx`: the column values, checked against the committed tree
  const uint32_t* verify(ReadIOP& iop, size_t idx) const {
    if (idx >= rows) throw VerifyError("merkle query out of range");
    const uint32_t* out = iop.read(cols);
    Digest cur = hash_elems(iop.suite, out, cols);
    idx += rows;
    while (idx >= 2 * top_size) {
      const bool low = idx & 1;
      Digest other = digest_of(iop.read(8));
      idx >>= 1;
      cur = low ? hash_pair(iop.suite, other, cur) : hash_pair(iop.suite, cur, other);
    }
    const Digest& present = idx >= top_size ? top[idx - top_size] : rest[idx];
    if (!same(present, cur)) throw VerifyError("merkle path mismatch");
    return out;
  }
};

FpExt load_ext(const uint32_t* w) { return FpExt{{w[0], w[1], w[2], w[3]}}; }

}  // namespace

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

FpExt poly_eval(const FpExt* coeffs, size_t n, FpExt x) {
  FpExt tot = fe_zero();
  for (size_t i = n; i-- > 0;) tot = fe_add(fe_mul(tot, x), coeffs[i]);
  return tot;
}

// fri.rs:36-155; `inner(pos)` is the DEEP-ALI value of the query at `pos`
template <typename Inner>
void fri_verify(ReadIOP& iop, size_t degree, Inner inner) {
  const size_t orig_domain = INV_RATE * degree;
  size_t domain = orig_domain;
  struct Round {
    size_t domain;
    MerkleVerifier merkle;
    FpExt mix;
  };
  std::vector<Round> rounds;
  while (degree > FRI_MIN_DEGREE) {
    const size_t d = domain / FRI_FOLD;
    MerkleVerifier m(iop, d, FRI_FOLD * 4);
    FpExt mix = iop.rng->random_ext_elem();
    rounds.push_back(Round{d, std::move(m), mix});
    domain = d;
    degree /= FRI_FOLD;
  }
  const uint32_t* final_words = iop.read(4 * degree);
  iop.commit(hash_elems(iop.suite, final_words, 4 * degree));
  std::vector<FpExt> final_poly(degree);
  for (size_t i = 0; i < degree; i++)
    for (int j = 0; j < 4; j++) final_poly[i].c[j] = final_words[j * degree + i];
  const uint32_t gen = fp_encode(kRouFwd[lg2(domain)]);
  const uint32_t inv16 = fp_inv(fp_encode(FRI_FOLD));
  const uint32_t w16 = fp_encode(kRouRev[4]);
  uint32_t w16_pow[FRI_FOLD];
  for (size_t k = 0; k < FRI_FOLD; k++) w16_pow[k] = fp_pow(w16, k);
  for (size_t q = 0; q < QUERIES; q++) {
    size_t pos = iop.rng->random_bits(lg2(orig_domain));
    FpExt goal = inner(pos);
    for (const Round& r : rounds) {  // verify_query, fri.rs:61-95
      const size_t quot = pos / r.domain, group = pos % r.domain;
      const uint32_t* data = r.merkle.verify(iop, group);
      FpExt data_ext[FRI_FOLD];
      for (size_t i = 0; i < FRI_FOLD; i++)
        for (int j = 0; j < 4; j++) data_ext[i].c[j] = data[j * FRI_FOLD + i];
      if (!fe_eq(data_ext[quot], goal)) throw VerifyError("FRI fold mismatch");
      const uint32_t inv_wk = fp_pow(fp_encode(kRouRev[lg2(FRI_FOLD * r.domain)]), group);
      // interpolate_ntt + bit_reverse: the natural-order coefficients of the fold
      FpExt coeffs[FRI_FOLD];
      for (size_t k = 0; k < FRI_FOLD; k++) {
        FpExt acc = fe_zero();
        for (size_t jj = 0; jj < FRI_FOLD; jj++) acc = fe_add(acc, fe_mul_fp(data_ext[jj], w16_pow[(jj * k) % FRI_FOLD]));
        coeffs[k] = fe_mul_fp(acc, inv16);
      }
      goal = poly_eval(coeffs, FRI_FOLD, fe_mul_fp(r.mix, inv_wk));
      pos = group;
    }
    FpExt x = fe_from_fp(fp_pow(gen, pos));
    if (!fe_eq(poly_eval(final_poly.data(), degree, x), goal)) throw VerifyError("FRI final polynomial mismatch");
  }
}

uint32_t verify_seal(const CircuitDef& c, int suite, const uint32_t* seal, size_t len, bool check_validity) {
  if (c.name == std::string("rv32im")) {  // rv32im/src/lib.rs:78-92: a version word leads the seal
    if (len < 1 || seal[0] != 2) throw VerifyError("bad rv32im seal version");
    seal++;
    len--;
  }
  ReadIOP iop(seal, len, suite);
  uint32_t psi[16], ci[16];
  for (int i = 0; i < 16; i++) {
    psi[i] = fp_encode(uint8_t(PROOF_SYSTEM_INFO[i]));
    ci[i] = fp_encode(uint8_t(c.circuit_info[i]));
  }
  iop.commit(hash_elems(suite, psi, 16));
  iop.commit(hash_elems(suite, ci, 16));
  const uint32_t* header = iop.read(c.output_size + 1);
  iop.commit(hash_elems(suite, header, c.output_size + 1));
  const uint32_t po2 = header[c.output_size];
  if (po2 < 2 || po2 > 24) throw VerifyError("po2 out of range");
  const size_t n = size_t(1) << po2, domain = INV_RATE * n;
  // groups in commit order: code, data, then (after the mix draw) accum (mod.rs:215-244)
  MerkleVerifier code(iop, domain, c.group_sizes[1]);
  MerkleVerifier data(iop, domain, c.group_sizes[2]);
  std::vector<uint32_t> mix(c.mix_size);
  for (auto& m : mix) m = iop.rng->random_elem();
  MerkleVerifier accum(iop, domain, c.group_sizes[0]);
  const MerkleVerifier* groups[3] = {&accum, &code, &data};
  // verify_validity (mod.rs:292-474)
  const FpExt poly_mix = iop.rng->random_ext_elem();
  MerkleVerifier check(iop, domain, CHECK_SIZE);
  const FpExt z = iop.rng->random_ext_elem();
  const uint32_t back_one = fp_encode(kRouRev[po2]);
  const size_t nt = c.n_taps;
  const uint32_t* coeff_words = iop.read((nt + CHECK_SIZE) * 4);
  iop.commit(hash_elems(suite, coeff_words, (nt + CHECK_SIZE) * 4));
  std::vector<FpExt> coeff_u(nt + CHECK_SIZE);
  for (size_t i = 0; i < coeff_u.size(); i++) coeff_u[i] = load_ext(coeff_words + 4 * i);
  if (check_validity) {  // mod.rs:340-394: poly_ext(z) == check(z) * ((3z)^N - 1)
    std::vector<FpExt> eval_u;
    size_t pos = 0;
    c.regs(0, nt, [&](size_t cur) {
      const size_t size = c.tap(cur).skip;
      for (size_t i = 0; i < size; i++) {
        const FpExt x = fe_mul_fp(z, fp_pow(back_one, c.tap(cur + i).back));
        eval_u.push_back(poly_eval(&coeff_u[pos], size, x));
      }
      pos += size;
    });
    FpExt check = fe_zero();
    const size_t remap[4] = {0, 2, 1, 3};
    for (size_t i = 0; i < 4; i++) {
      const FpExt zi = fe_pow(z, i);
      for (size_t k = 0; k < 4; k++) {
        FpExt unit = fe_zero();
        unit.c[k] = kOne;
        check = fe_add(check, fe_mul(fe_mul(coeff_u[nt + remap[i] + 4 * k], zi), unit));
      }
    }
    check = fe_mul(check, fe_sub(fe_pow(fe_mul_fp(z, fp_encode(3)), n), fe_one()));
    if (!fe_eq(check, poly_ext(c, mix.data(), header, eval_u.data(), poly_mix)))
      throw VerifyError("verification indicates proof is invalid");
  }

  // DEEP-ALI mixing (mod.rs:396-440)
  const FpExt fri_mix = iop.rng->random_ext_elem();
  const size_t tot_backs = c.combo_begin[c.combos_count];
  std::vector<FpExt> combo_u(tot_backs + 1, fe_zero());
  struct Reg {
    size_t group, offset, combo;
    FpExt mix_pow;
  };
  std::vector<Reg> regs;
  FpExt cur_mix = fe_one();
  size_t pos = 0;
  c.regs(0, nt, [&](size_t cur) {
    const auto& t = c.tap(cur);
    for (size_t i = 0; i < t.skip; i++) {
      const size_t k = c.combo_begin[t.combo] + i;
      combo_u[k] = fe_add(combo_u[k], fe_mul(cur_mix, coeff_u[pos + i]));
    }
    regs.push_back(Reg{t.group, t.offset, t.combo, cur_mix});
    cur_mix = fe_mul(cur_mix, fri_mix);
    pos += t.skip;
  });
  std::vector<FpExt> check_mix_pows;
  for (size_t i = 0; i < CHECK_SIZE; i++) {
    combo_u[tot_backs] = fe_add(combo_u[tot_backs], fe_mul(cur_mix, coeff_u[pos++]));
    check_mix_pows.push_back(cur_mix);
    cur_mix = fe_mul(cur_mix, fri_mix);
  }
  // the per-combo divisors' roots z * back_one^back, and z^INV_RATE for the check combo
  std::vector<FpExt> roots(tot_backs);
  for (size_t k = 0; k < tot_backs; k++) roots[k] = fe_mul_fp(z, fp_pow(back_one, c.combo_taps[k]));
  const FpExt z_rate = fe_pow(z, INV_RATE);
  const uint32_t gen = fp_encode(kRouFwd[lg2(domain)]);

  auto inner = [&](size_t idx) {  // fri_eval_taps, mod.rs:246-290
    const FpExt x = fe_from_fp(fp_pow(gen, idx));
    const uint32_t* rows[3];
    for (int g = 0; g < 3; g++) rows[g] = groups[g]->verify(iop, idx);
    const uint32_t* check_row = check.verify(iop, idx);
    std::vector<FpExt> tot(c.combos_count + 1, fe_zero());
    for (const Reg& r : regs) tot[r.combo] = fe_add(tot[r.combo], fe_mul_fp(r.mix_pow, rows[r.group][r.offset]));
    for (size_t i = 0; i < CHECK_SIZE; i++)
      tot[c.combos_count] = fe_add(tot[c.combos_count], fe_mul_fp(check_mix_pows[i], check_row[i]));
    FpExt ret = fe_zero();
    for (size_t i = 0; i < c.combos_count; i++) {
      const size_t b = c.combo_begin[i], e = c.combo_begin[i + 1];
      FpExt num = fe_sub(tot[i], poly_eval(&combo_u[b], e - b, x));
      FpExt div = fe_one();
      for (size_t k = b; k < e; k++) div = fe_mul(div, fe_sub(x, roots[k]));
      ret = fe_add(ret, fe_mul(num, fe_inv(div)));
    }
    FpExt check_num = fe_sub(tot[c.combos_count], combo_u[tot_backs]);
    return fe_add(ret, fe_mul(check_num, fe_inv(fe_sub(x, z_rate))));
  };
  fri_verify(iop, n, inner);
  if (iop.pos != iop.size) throw VerifyError("trailing words in seal");  // read_iop.rs:66-71
  return po2;
}

}  // namespace
}  // namespace r0

using namespace r0;

extern "C" const char* r0hip_verify_seal(const char* circuit, int suite, const uint32_t* seal, size_t seal_len,
                                         int check_validity, uint32_t* po2_out) {
  try {
    const CircuitDef* c = find_circuit(circuit ? circuit : "");
    R0_REQUIRE(c, std::string("unknown circuit ") + (circuit ? circuit : "(null)"));
    R0_REQUIRE(suite >= 0 && suite <= 2, "unknown hash suite");
    R0_REQUIRE(seal || seal_len == 0, "seal is NULL");
    uint32_t po2 = verify_seal(*c, suite, seal, seal_len, check_validity != 0);
    if (po2_out) *po2_out = po2;
    return nullptr;
  } catch (const std::exception& e) {
    return strdup(e.what());
  } catch (...) {
    return strdup("r0hip: unknown error");
  }
}

extern "C" const char* r0hip_poly_ext(const char* circuit, const uint32_t* h_mix, const uint32_t* h_global,
                                      const uint32_t* h_eval_u, const uint32_t* h_poly_mix, uint32_t* h_out) {
  try {
    const CircuitDef* c = find_circuit(circuit ? circuit : "");
    R0_REQUIRE(c, std::string("unknown circuit ") + (circuit ? circuit : "(null)"));
    R0_REQUIRE(h_mix && h_global && h_eval_u && h_poly_mix && h_out, "poly_ext: null argument");
    std::vector<FpExt> eval_u(c->n_taps);
    for (size_t i = 0; i < c->n_taps; i++) eval_u[i] = load_ext(h_eval_u + 4 * i);
    FpExt r = poly_ext(*c, h_mix, h_global, eval_u.data(), load_ext(h_poly_mix));
    memcpy(h_out, r.c, 16);
    return nullptr;
  } catch (const std::exception& e) {
    return strdup(e.what());
  } catch (...) {
    return strdup("r0hip: unknown error");
  }
}
