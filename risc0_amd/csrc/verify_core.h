// Host-only core of the STARK verifier (risc0/zkp/src/verify/): the read IOP, Merkle
// openings, verify_validity and FRI, parameterised by the tap set and the circuit's
// poly_ext so the segment seals (verify.cpp) and other tap sets share one implementation.
//   transcript        risc0/zkp/src/verify/read_iop.rs:20-84
//   Merkle openings   risc0/zkp/src/verify/merkle.rs:79-186 with zkp/src/merkle.rs:36-66 params
//   verify_validity   risc0/zkp/src/verify/mod.rs:292-474 (DEEP-ALI taps: fri_eval_taps, :246-290)
//   FRI               risc0/zkp/src/verify/fri.rs:36-155
// No HIP: compiles with g++ as well as hipcc.
#pragma once
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "transcript.h"

namespace r0 {
namespace vfy {


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
  // the reference asserts every word is reduced (poseidon2/mod.rs:47-59): a seal whose
  // digests carry words >= p is rejected there, so it is rejected here
  for (uint32_t w : both)
    if (w >= kP) throw VerifyError("non-canonical Poseidon2 digest word in seal");
  return p2_hash_words(both, 16);
}

struct MerkleVerifier;
// A Merkle opening read from the seal whose hashes are checked later (ReadIOP::defer): the
// transcript never depends on a hash of an opening, so the query loop reads and checks the
// arithmetic in order, and the openings' hash paths run afterwards on several threads.
struct PendingOpening {
  const MerkleVerifier* tree;
  const uint32_t* row;   // cols field words
  const uint32_t* path;  // 8 words per level above the top layer
  size_t idx;
};

// read_iop.rs: a cursor over the seal plus the Fiat-Shamir RNG
struct ReadIOP {
  const uint32_t* words;
  size_t size, pos = 0;
  int suite;
  std::unique_ptr<Rng> rng;
  bool defer = false;  // Merkle openings go to `pending` instead of being hashed at once
  std::vector<PendingOpening> pending;
  ReadIOP(const uint32_t* w, size_t n, int s) : words(w), size(n), suite(s), rng(make_rng(s)) {}
  const uint32_t* read(size_t n) {
    if (n > size - pos) throw VerifyError("seal too short");
    const uint32_t* p = words + pos;
    pos += n;
    return p;
  }
  // read_field_elem_slice (read_iop.rs:45-48): field words must be canonical (< p), as the
  // reference's checked cast of the seal words into BabyBearElem enforces
  const uint32_t* read_elems(size_t n) {
    const uint32_t* p = read(n);
    for (size_t i = 0; i < n; i++)
      if (p[i] >= kP) throw VerifyError("non-canonical field element in seal");
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

  // opens row `idx`: the column values, checked against the committed tree (now, or with
  // iop.defer in check_pending)
  const uint32_t* verify(ReadIOP& iop, size_t idx) const {
    if (idx >= rows) throw VerifyError("merkle query out of range");
    const uint32_t* out = iop.read_elems(cols);
    size_t levels = 0;
    for (size_t i = idx + rows; i >= 2 * top_size; i >>= 1) levels++;
    const uint32_t* path = iop.read(8 * levels);
    if (iop.defer)
      iop.pending.push_back(PendingOpening{this, out, path, idx});
    else
      check(iop.suite, out, path, idx);
    return out;
  }
  void check(int suite, const uint32_t* out, const uint32_t* path, size_t idx) const {
    Digest cur = hash_elems(suite, out, cols);
    idx += rows;
    while (idx >= 2 * top_size) {
      const bool low = idx & 1;
      Digest other = digest_of(path);
      path += 8;
      idx >>= 1;
      cur = low ? hash_pair(suite, other, cur) : hash_pair(suite, cur, other);
    }
    const Digest& present = idx >= top_size ? top[idx - top_size] : rest[idx];
    if (!same(present, cur)) throw VerifyError("merkle path mismatch");
  }
};

// the deferred openings' hash paths on up to `threads` host threads; the first failure (in
// opening order) is thrown
inline void check_pending(ReadIOP& iop, unsigned threads) {
  const size_t n = iop.pending.size();
  if (n == 0) return;
  threads = unsigned(std::max<size_t>(1, std::min<size_t>(threads, n)));
  std::vector<std::string> err(threads);
  std::vector<size_t> err_at(threads, SIZE_MAX);
  auto work = [&](unsigned t) {
    for (size_t i = t; i < n; i += threads) {
      const PendingOpening& p = iop.pending[i];
      try {
        p.tree->check(iop.suite, p.row, p.path, p.idx);
      } catch (const std::exception& e) {
        err[t] = e.what();
        err_at[t] = i;
        return;
      }
    }
  };
  std::vector<std::thread> pool;
  for (unsigned t = 1; t < threads; t++) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  size_t first = SIZE_MAX;
  unsigned which = 0;
  for (unsigned t = 0; t < threads; t++)
    if (err_at[t] < first) first = err_at[t], which = t;
  if (first != SIZE_MAX) throw VerifyError(err[which]);
}

FpExt load_ext(const uint32_t* w) { return FpExt{{w[0], w[1], w[2], w[3]}}; }

// host threads for the deferred Merkle openings: R0HIP_VERIFY_THREADS, else up to 8 of the cores
inline unsigned verify_threads() {
  static const unsigned n = [] {
    const char* e = std::getenv("R0HIP_VERIFY_THREADS");
    if (e) return unsigned(std::max(1L, std::strtol(e, nullptr, 10)));
    return std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  }();
  return n;
}

// The tap-set view (taps.rs) the verifier needs: taps as {offset, back, group, combo, skip}
struct TapView {
  const uint32_t* taps;
  size_t n_taps;
  const uint32_t* combo_taps;
  const uint32_t* combo_begin;  // combos_count + 1
  size_t combos_count;
  struct Tap {
    uint32_t offset, back, group, combo, skip;
  };
  const Tap& tap(size_t i) const { return reinterpret_cast<const Tap*>(taps)[i]; }
  template <typename F>
  void regs(F f) const {  // RegisterIter, taps.rs:202-227
    for (size_t cur = 0; cur < n_taps; cur += tap(cur).skip) f(cur);
  }
};


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
  const uint32_t* final_words = iop.read_elems(4 * degree);
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
  check_pending(iop, verify_threads());  // while the rounds' verifiers are alive
}

// verify_validity (mod.rs:292-474) then fri_verify and verify_complete (read_iop.rs:66-71),
// once the caller has replayed the group commitments. groups[g] is the Merkle verifier of
// register group g (accum 0, code 1, data 2); poly_ext(poly_mix, eval_u) is the circuit's
// constraint polynomial at z (checked only when check_validity).
template <typename PolyExt>
void verify_validity_and_fri(ReadIOP& iop, const TapView& t, uint32_t po2, const MerkleVerifier* const* groups,
                             bool check_validity, PolyExt poly_ext) {
  const size_t n = size_t(1) << po2, domain = INV_RATE * n;
  const FpExt poly_mix = iop.rng->random_ext_elem();
  MerkleVerifier check(iop, domain, CHECK_SIZE);
  const FpExt z = iop.rng->random_ext_elem();
  const uint32_t back_one = fp_encode(kRouRev[po2]);
  const size_t nt = t.n_taps;
  const uint32_t* coeff_words = iop.read_elems((nt + CHECK_SIZE) * 4);
  iop.commit(hash_elems(iop.suite, coeff_words, (nt + CHECK_SIZE) * 4));
  std::vector<FpExt> coeff_u(nt + CHECK_SIZE);
  for (size_t i = 0; i < coeff_u.size(); i++) coeff_u[i] = load_ext(coeff_words + 4 * i);
  if (check_validity) {  // mod.rs:340-394: poly_ext(z) == check(z) * ((3z)^N - 1)
    std::vector<FpExt> eval_u;
    size_t pos = 0;
    t.regs([&](size_t cur) {
      const size_t size = t.tap(cur).skip;
      for (size_t i = 0; i < size; i++) {
        const FpExt x = fe_mul_fp(z, fp_pow(back_one, t.tap(cur + i).back));
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
    if (!fe_eq(check, poly_ext(poly_mix, eval_u.data())))
      throw VerifyError("verification indicates proof is invalid");
  }

  // DEEP-ALI mixing (mod.rs:396-440)
  const FpExt fri_mix = iop.rng->random_ext_elem();
  const size_t tot_backs = t.combo_begin[t.combos_count];
  std::vector<FpExt> combo_u(tot_backs + 1, fe_zero());
  struct Reg {
    size_t group, offset, combo;
    FpExt mix_pow;
  };
  std::vector<Reg> regs;
  FpExt cur_mix = fe_one();
  size_t pos = 0;
  t.regs([&](size_t cur) {
    const auto& tap = t.tap(cur);
    for (size_t i = 0; i < tap.skip; i++) {
      const size_t k = t.combo_begin[tap.combo] + i;
      combo_u[k] = fe_add(combo_u[k], fe_mul(cur_mix, coeff_u[pos + i]));
    }
    regs.push_back(Reg{tap.group, tap.offset, tap.combo, cur_mix});
    cur_mix = fe_mul(cur_mix, fri_mix);
    pos += tap.skip;
  });
  std::vector<FpExt> check_mix_pows;
  for (size_t i = 0; i < CHECK_SIZE; i++) {
    combo_u[tot_backs] = fe_add(combo_u[tot_backs], fe_mul(cur_mix, coeff_u[pos++]));
    check_mix_pows.push_back(cur_mix);
    cur_mix = fe_mul(cur_mix, fri_mix);
  }
  // the per-combo divisors' roots z * back_one^back, and z^INV_RATE for the check combo
  std::vector<FpExt> roots(tot_backs);
  for (size_t k = 0; k < tot_backs; k++) roots[k] = fe_mul_fp(z, fp_pow(back_one, t.combo_taps[k]));
  const FpExt z_rate = fe_pow(z, INV_RATE);
  const uint32_t gen = fp_encode(kRouFwd[lg2(domain)]);

  auto inner = [&](size_t idx) {  // fri_eval_taps, mod.rs:246-290
    const FpExt x = fe_from_fp(fp_pow(gen, idx));
    const uint32_t* rows[3];
    for (int g = 0; g < 3; g++) rows[g] = groups[g]->verify(iop, idx);
    const uint32_t* check_row = check.verify(iop, idx);
    std::vector<FpExt> tot(t.combos_count + 1, fe_zero());
    for (const Reg& r : regs) tot[r.combo] = fe_add(tot[r.combo], fe_mul_fp(r.mix_pow, rows[r.group][r.offset]));
    for (size_t i = 0; i < CHECK_SIZE; i++)
      tot[t.combos_count] = fe_add(tot[t.combos_count], fe_mul_fp(check_mix_pows[i], check_row[i]));
    FpExt ret = fe_zero();
    for (size_t i = 0; i < t.combos_count; i++) {
      const size_t b = t.combo_begin[i], e = t.combo_begin[i + 1];
      FpExt num = fe_sub(tot[i], poly_eval(&combo_u[b], e - b, x));
      FpExt div = fe_one();
      for (size_t k = b; k < e; k++) div = fe_mul(div, fe_sub(x, roots[k]));
      ret = fe_add(ret, fe_mul(num, fe_inv(div)));
    }
    FpExt check_num = fe_sub(tot[t.combos_count], combo_u[tot_backs]);
    return fe_add(ret, fe_mul(check_num, fe_inv(fe_sub(x, z_rate))));
  };
  fri_verify(iop, n, inner);
  if (iop.pos != iop.size) throw VerifyError("trailing words in seal");
}

}  // namespace vfy
}  // namespace r0
