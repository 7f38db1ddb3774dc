// ORACLE (test infrastructure only — never linked into the product path).
//
// CPU restatement of the reference STARK prover on top of the oracle CpuHal:
//   risc0/zkp/src/prove/prover.rs:38-393   (make_coeffs, commit_group, finalize)
//   risc0/zkp/src/prove/poly_group.rs:55-83
//   risc0/zkp/src/prove/merkle.rs:54-140 + risc0/zkp/src/merkle.rs:39-67
//   risc0/zkp/src/prove/fri.rs:39-126
//   risc0/zkp/src/prove/write_iop.rs:24-76
//   risc0/zkp/src/core/poly.rs:23-89
//   risc0/circuit/rv32im/src/prove/hal/mod.rs:143-224 (segment header / group order)
#include <algorithm>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "core.h"
#include "oracle.h"

using namespace oracle;

extern "C" {
void oracle_batch_expand_into_evaluate_ntt(uint32_t*, size_t, const uint32_t*, size_t, size_t, size_t);
void oracle_batch_interpolate_ntt(uint32_t*, size_t, size_t);
void oracle_batch_bit_reverse(uint32_t*, size_t, size_t);
void oracle_batch_evaluate_any(const uint32_t*, size_t, size_t, const uint32_t*, const uint32_t*,
                               uint32_t*, size_t);
void oracle_zk_shift(uint32_t*, size_t, size_t);
void oracle_mix_poly_coeffs(uint32_t*, size_t, const uint32_t*, const uint32_t*, const uint32_t*,
                            const uint32_t*, size_t, size_t);
void oracle_eltwise_sum_extelem(uint32_t*, size_t, const uint32_t*, size_t);
void oracle_fri_fold(uint32_t*, size_t, const uint32_t*, const uint32_t*);
void oracle_hash_rows(int, uint32_t*, size_t, const uint32_t*, size_t);
void oracle_hash_fold(int, uint32_t*, size_t, size_t);
void oracle_combos_prepare(uint32_t*, const uint32_t*, size_t, size_t, const uint32_t*,
                           const uint32_t*, size_t, const uint32_t*);
long oracle_combos_divide(uint32_t*, size_t, const uint32_t*, const uint32_t*, size_t);
}

namespace {

// Wall time per Hal op of the proofs run so far (the CPU baseline's per-op breakdown,
// BASELINE.md §2). Keys follow the reference Hal method names.
std::mutex g_op_mu;
std::map<std::string, std::pair<double, long>> g_op_time;
struct OpTime {
  const char* name;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  explicit OpTime(const char* n) : name(n) {}
  ~OpTime() {
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::lock_guard<std::mutex> lk(g_op_mu);
    auto& e = g_op_time[name];
    e.first += s;
    e.second += 1;
  }
};
#define OP_CAT2(a, b) a##b
#define OP_CAT(a, b) OP_CAT2(a, b)
#define OP_TIME(n) OpTime OP_CAT(op_time_, __LINE__)(n)

constexpr size_t INV_RATE = 4, QUERIES = 50, FRI_FOLD = 16, FRI_MIN_DEGREE = 256, EXT = 4,
                 CHECK_SIZE = INV_RATE * EXT;
const char PROOF_SYSTEM_INFO[17] = "RISC0_STARK:v1__";  // adapter.rs:120

typedef std::vector<uint32_t> Buf;

struct Tap {
  uint32_t offset, back, group, combo, skip;
};

// taps.rs:57-140
struct TapSet {
  const oracle_circuit_t* c;
  const Tap* tap(size_t i) const { return reinterpret_cast<const Tap*>(c->taps) + i; }
  size_t group_size(size_t g) const { return tap(c->group_begin[g + 1] - 1)->offset + 1; }
  // RegisterIter over [begin, end): cursor advances by skip
  template <typename F>
  void regs(size_t begin, size_t end, F f) const {
    size_t cur = begin;
    while (cur < c->n_taps) {
      size_t next = cur + tap(cur)->skip;
      if (next > end) break;
      f(cur);
      cur = next;
    }
  }
};

// write_iop.rs
struct WriteIOP {
  std::vector<uint32_t> proof;
  std::unique_ptr<Rng> rng;
  int suite;
  explicit WriteIOP(int s) : rng(new_rng(s)), suite(s) {}
  void write_u32(const uint32_t* p, size_t n) { proof.insert(proof.end(), p, p + n); }
  void commit(const Digest& d) { rng->mix(d); }
};

// merkle.rs:39-67
struct MerkleTreeParams {
  size_t row_size, col_size, layers, top_size;
  MerkleTreeParams(size_t rows, size_t cols, size_t queries) : row_size(rows), col_size(cols) {
    layers = log2_ceil(rows);
    if ((size_t(1) << layers) != rows) throw std::runtime_error("rows not po2");
    size_t top_layer = 0;
    for (size_t i = 1; i < layers; i++) {
      if ((size_t(1) << i) > queries) break;
      top_layer = i;
    }
    top_size = size_t(1) << top_layer;
  }
};

// prove/merkle.rs:26-140
struct MerkleTreeProver {
  MerkleTreeParams params;
  const Buf* matrix;
  Buf nodes;  // 2*rows digests
  Digest root;
  MerkleTreeProver(int suite, const Buf& m, size_t rows, size_t cols, size_t queries)
      : params(rows, cols, queries), matrix(&m), nodes(rows * 2 * 8, 0) {
    {
      OP_TIME("hash_rows");
      oracle_hash_rows(suite, nodes.data() + rows * 8, rows, m.data(), rows * cols);
    }
    OP_TIME("hash_fold");
    for (size_t i = params.layers; i-- > 0;) {
      size_t layer = size_t(1) << i;
      oracle_hash_fold(suite, nodes.data(), layer * 2, layer);
    }
    memcpy(root.w, nodes.data() + 8, 32);
  }
  void commit(WriteIOP& iop) const {
    iop.write_u32(nodes.data() + params.top_size * 8, params.top_size * 8);
    iop.commit(root);
  }
  void prove(WriteIOP& iop, size_t idx) const {
    if (idx >= params.row_size) throw std::runtime_error("merkle idx");
    for (size_t i = 0; i < params.col_size; i++) iop.proof.push_back((*matrix)[idx + i * params.row_size]);
    idx += params.row_size;
    while (idx >= 2 * params.top_size) {
      size_t low = idx % 2;
      idx /= 2;
      size_t other = 2 * idx + (1 - low);
      iop.write_u32(nodes.data() + other * 8, 8);
    }
  }
};

// poly_group.rs:55-83
struct PolyGroup {
  Buf coeffs;
  size_t count;
  Buf evaluated;
  std::unique_ptr<MerkleTreeProver> merkle;
  PolyGroup(int suite, Buf c, size_t cnt, size_t size) : coeffs(std::move(c)), count(cnt) {
    size_t domain = size * INV_RATE;
    evaluated.assign(count * domain, 0);
    {
      OP_TIME("batch_expand_into_evaluate_ntt");
      oracle_batch_expand_into_evaluate_ntt(evaluated.data(), evaluated.size(), coeffs.data(),
                                            coeffs.size(), count, log2_ceil(INV_RATE));
    }
    {
      OP_TIME("batch_bit_reverse");
      oracle_batch_bit_reverse(coeffs.data(), coeffs.size(), count);
    }
    merkle.reset(new MerkleTreeProver(suite, evaluated, domain, count, QUERIES));
  }
};

// core/poly.rs
ExtElem poly_eval(const ExtElem* c, size_t n, ExtElem x) {
  ExtElem mul = ExtElem::one(), tot = ExtElem::zero();
  for (size_t i = 0; i < n; i++) {
    tot += c[i] * mul;
    mul *= x;
  }
  return tot;
}
ExtElem poly_divide(ExtElem* p, size_t n, ExtElem z) {
  ExtElem cur = ExtElem::zero();
  for (size_t i = n; i-- > 0;) {
    ExtElem next = z * cur + p[i];
    p[i] = cur;
    cur = next;
  }
  return cur;
}
// poly.rs:41-78. NOTE: like the reference, clears the whole tail of `out`.
void poly_interpolate(ExtElem* out, size_t out_len, const ExtElem* x, const ExtElem* fx, size_t size) {
  if (size == 1) {
    out[0] = fx[0];
    return;
  }
  if (size == 2) {
    out[1] = (fx[1] - fx[0]) * (x[1] - x[0]).inv();
    out[0] = fx[0] - out[1] * x[0];
    return;
  }
  std::vector<ExtElem> ft(size + 1, ExtElem::zero());
  ft[0] = ExtElem::one();
  for (size_t i = 0; i < size; i++) {
    for (size_t j = i + 1; j-- > 0;) {
      ExtElem value = ft[j];
      ft[j + 1] += value;
      ft[j] *= -x[i];
    }
  }
  for (size_t i = 0; i < out_len; i++) out[i] = ExtElem::zero();
  for (size_t i = 0; i < size; i++) {
    std::vector<ExtElem> fr = ft;
    poly_divide(fr.data(), fr.size(), x[i]);
    ExtElem fr_xi = poly_eval(fr.data(), fr.size(), x[i]);
    ExtElem mul = fx[i] * fr_xi.inv();
    for (size_t j = 0; j < size; j++) out[j] += mul * fr[j];
  }
}

// field/mod.rs:243-270
std::vector<ExtElem> map_pow(ExtElem base, const uint32_t* exps, size_t n) {
  std::vector<ExtElem> r;
  if (!n) return r;
  r.push_back(base.pow(exps[0]));
  for (size_t i = 1; i < n; i++) {
    if (exps[i] == exps[i - 1] + 1)
      r.push_back(r.back() * base);
    else
      r.push_back(r.back() * base.pow(exps[i] - exps[i - 1]));
  }
  return r;
}

void eval_check(const oracle_circuit_t* c, uint32_t* check, const uint32_t** groups,
                const uint32_t* mix, const uint32_t* global, ExtElem poly_mix, uint32_t po2) {
  if (!c->poly_fp) throw std::runtime_error("circuit has no poly_fp (oracle/_ref not built?)");
  size_t steps = size_t(1) << po2, domain = steps * INV_RATE;
  std::vector<ExtElem> pows = map_pow(poly_mix, c->poly_mix_powers, c->n_poly_mix);
  std::vector<const uint32_t*> args(c->n_eval_args);
  for (size_t i = 0; i < c->n_eval_args; i++) {
    int a = c->eval_args[i];
    args[i] = a >= 0 ? groups[a] : (a == -1 ? mix : global);
  }
  Elem rou = rou_fwd(po2 + 2);
  parallel_for(domain, [&](size_t b, size_t e) {
    for (size_t cycle = b; cycle < e; cycle++) {
      uint32_t tot_w[4];
      const char* err = c->poly_fp(cycle, domain, &pows[0].e[0].v, args.data(), tot_w);
      if (err) abort();
      ExtElem tot = ExtElem::raw(tot_w);
      Elem x = rou.pow(cycle);
      Elem y = (Elem::from(3) * x).pow(steps);
      ExtElem ret = tot * (y - Elem::one()).inv();
      for (size_t i = 0; i < 4; i++) check[i * domain + cycle] = ret.e[i].v;
    }
  });
}

// Full-size eval_check at sampled cycles (test infrastructure). The evaluated groups are
// the device's synthetic words (r0hip_fill_uniform: splitmix64 of (seed, index) mod p), so
// any tap value is recomputed here from its index instead of copying GB-sized buffers to
// the host. The reference poly_fp reads a tap only as args[col*steps + ((cycle - 4*back) &
// (steps-1))] (rv32im-sys/kernels/cxx/rust_poly_fp_*.cpp), so each sampled cycle is
// evaluated on a small window domain holding, for every column, the values at
// cycle - 4*back of the full domain; the result is multiplied by the full-size
// ((3*w^cycle)^N - 1)^-1 exactly as eval_check above (cpu.rs:145-207).
static uint32_t splitmix_word(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  z ^= z >> 31;
  return uint32_t(z % P);
}

void eval_check_sampled(const oracle_circuit_t* c, const uint64_t* group_seeds, const uint32_t* mix,
                        const uint32_t* global, ExtElem poly_mix, uint32_t po2, const uint64_t* cycles,
                        size_t n, uint32_t* out) {
  if (!c->poly_fp) throw std::runtime_error("circuit has no poly_fp (oracle/_ref not built?)");
  TapSet taps{c};
  uint32_t max_back = 0;
  for (size_t i = 0; i < c->n_taps; i++) max_back = std::max(max_back, taps.tap(i)->back);
  size_t win = 1;
  while (win < INV_RATE * (max_back + 2)) win <<= 1;
  const size_t steps = size_t(1) << po2, domain = steps * INV_RATE;
  std::vector<ExtElem> pows = map_pow(poly_mix, c->poly_mix_powers, c->n_poly_mix);
  Elem rou = rou_fwd(po2 + 2);
  for (size_t s = 0; s < n; s++)
    if (cycles[s] >= domain) throw std::runtime_error("sampled cycle out of range");
  parallel_for(n, [&](size_t b, size_t e) {
    std::vector<Buf> w(c->n_groups);
    for (size_t g = 0; g < c->n_groups; g++) w[g].assign(taps.group_size(g) * win, 0);
    std::vector<const uint32_t*> args(c->n_eval_args);
    for (size_t s = b; s < e; s++) {
      uint64_t cyc = cycles[s];
      size_t local = INV_RATE * (max_back + 1) + (cyc & 3);  // same coset, every back in range
      for (size_t g = 0; g < c->n_groups; g++) {
        size_t gs = taps.group_size(g);
        for (size_t col = 0; col < gs; col++)
          for (uint32_t bk = 0; bk <= max_back; bk++) {
            uint64_t full = (cyc - INV_RATE * bk) & (domain - 1);
            w[g][col * win + ((local - INV_RATE * bk) & (win - 1))] =
                splitmix_word(group_seeds[g], col * domain + full);
          }
      }
      for (size_t i = 0; i < c->n_eval_args; i++) {
        int a = c->eval_args[i];
        args[i] = a >= 0 ? w[a].data() : (a == -1 ? mix : global);
      }
      uint32_t tot_w[4];
      const char* err = c->poly_fp(local, win, &pows[0].e[0].v, args.data(), tot_w);
      if (err) abort();
      ExtElem tot = ExtElem::raw(tot_w);
      Elem y = (Elem::from(3) * rou.pow(cyc)).pow(steps);
      ExtElem ret = tot * (y - Elem::one()).inv();
      for (size_t i = 0; i < 4; i++) out[s * 4 + i] = ret.e[i].v;
    }
  });
}

struct Prover {
  const oracle_circuit_t* c;
  TapSet taps;
  int suite;
  WriteIOP iop;
  std::vector<std::unique_ptr<PolyGroup>> groups;
  size_t cycles = 0, po2 = 0;

  Prover(const oracle_circuit_t* circ, int s) : c(circ), suite(s), iop(s) {
    taps.c = circ;
    groups.resize(circ->n_groups);
  }

  // prover.rs:38-48 + 81-108
  void commit_group(size_t g, const uint32_t* witness) {
    size_t gs = taps.group_size(g);
    Buf coeffs(witness, witness + gs * cycles);
    {
      OP_TIME("batch_interpolate_ntt");
      oracle_batch_interpolate_ntt(coeffs.data(), coeffs.size(), gs);
    }
    {
      OP_TIME("zk_shift");
      oracle_zk_shift(coeffs.data(), coeffs.size(), gs);
    }
    groups[g].reset(new PolyGroup(suite, std::move(coeffs), gs, cycles));
    groups[g]->merkle->commit(iop);
  }

  // prover.rs:111-393
  void finalize(const uint32_t* mix, const uint32_t* global) {
    ExtElem poly_mix = iop.rng->random_ext_elem();
    size_t domain = cycles * INV_RATE;
    Buf check(EXT * domain, 0);
    std::vector<const uint32_t*> gptrs;
    for (auto& g : groups) gptrs.push_back(g->evaluated.data());
    {
      OP_TIME("eval_check");
      eval_check(c, check.data(), gptrs.data(), mix, global, poly_mix, (uint32_t)po2);
    }
    {
      OP_TIME("batch_interpolate_ntt");
      oracle_batch_interpolate_ntt(check.data(), check.size(), EXT);
    }
    PolyGroup check_group(suite, std::move(check), CHECK_SIZE, cycles);
    check_group.merkle->commit(iop);

    ExtElem z = iop.rng->random_ext_elem();
    ExtElem back_one = ExtElem::from_fp(rou_rev(po2));
    std::vector<ExtElem> all_xs, eval_u;
    for (size_t id = 0; id < groups.size(); id++) {
      std::vector<uint32_t> which;
      std::vector<ExtElem> xs;
      for (size_t t = c->group_begin[id]; t < c->group_begin[id + 1]; t++) {
        which.push_back(taps.tap(t)->offset);
        ExtElem x = back_one.pow(taps.tap(t)->back) * z;
        xs.push_back(x);
        all_xs.push_back(x);
      }
      std::vector<ExtElem> out(which.size());
      OP_TIME("batch_evaluate_any");
      oracle_batch_evaluate_any(groups[id]->coeffs.data(), groups[id]->coeffs.size(),
                                groups[id]->count, which.data(), &xs[0].e[0].v, &out[0].e[0].v,
                                which.size());
      eval_u.insert(eval_u.end(), out.begin(), out.end());
    }
    std::vector<ExtElem> coeff_u(eval_u.size(), ExtElem::zero());
    {
      size_t pos = 0;
      taps.regs(0, c->n_taps, [&](size_t cur) {
        size_t sz = taps.tap(cur)->skip;
        poly_interpolate(&coeff_u[pos], coeff_u.size() - pos, &all_xs[pos], &eval_u[pos], sz);
        pos += sz;
      });
    }
    ExtElem z_pow = z.pow(EXT);
    {
      std::vector<uint32_t> which(CHECK_SIZE);
      for (size_t i = 0; i < CHECK_SIZE; i++) which[i] = (uint32_t)i;
      std::vector<ExtElem> xs(CHECK_SIZE, z_pow), out(CHECK_SIZE);
      OP_TIME("batch_evaluate_any");
      oracle_batch_evaluate_any(check_group.coeffs.data(), check_group.coeffs.size(), CHECK_SIZE,
                                which.data(), &xs[0].e[0].v, &out[0].e[0].v, CHECK_SIZE);
      coeff_u.insert(coeff_u.end(), out.begin(), out.end());
      iop.write_u32(&coeff_u[0].e[0].v, coeff_u.size() * 4);
      iop.commit(hash_ext_elem_slice(suite, coeff_u.data(), coeff_u.size()));
    }
    ExtElem mix_fri = iop.rng->random_ext_elem();
    size_t combo_count = c->combos_count;
    Buf combos(cycles * (combo_count + 1) * 4, 0);
    {
      OP_TIME("mix_poly_coeffs");
      ExtElem cur_mix = ExtElem::one();
      for (size_t id = 0; id < groups.size(); id++) {
        size_t gs = taps.group_size(id);
        std::vector<uint32_t> which;
        taps.regs(c->group_begin[id], c->group_begin[id + 1],
                  [&](size_t cur) { which.push_back(taps.tap(cur)->combo); });
        uint32_t cm[4], mm[4];
        cur_mix.store(cm);
        mix_fri.store(mm);
        oracle_mix_poly_coeffs(combos.data(), combos.size() / 4, cm, mm, groups[id]->coeffs.data(),
                               which.data(), gs, cycles);
        cur_mix *= mix_fri.pow(gs);
      }
      std::vector<uint32_t> which(CHECK_SIZE, (uint32_t)combo_count);
      uint32_t cm[4], mm[4];
      cur_mix.store(cm);
      mix_fri.store(mm);
      oracle_mix_poly_coeffs(combos.data(), combos.size() / 4, cm, mm, check_group.coeffs.data(),
                             which.data(), CHECK_SIZE, cycles);
    }
    {
      std::vector<uint32_t> reg_sizes, reg_combo_ids;
      taps.regs(0, c->n_taps, [&](size_t cur) {
        reg_sizes.push_back(taps.tap(cur)->skip);
        reg_combo_ids.push_back(taps.tap(cur)->combo);
      });
      uint32_t mm[4];
      mix_fri.store(mm);
      OP_TIME("combos_prepare+combos_divide");
      oracle_combos_prepare(combos.data(), &coeff_u[0].e[0].v, combo_count, cycles, reg_sizes.data(),
                            reg_combo_ids.data(), reg_sizes.size(), mm);
      std::vector<ExtElem> pows;
      std::vector<uint32_t> begin{0};
      for (size_t i = 0; i < combo_count; i++) {
        for (uint32_t k = c->combo_begin[i]; k < c->combo_begin[i + 1]; k++)
          pows.push_back(z * back_one.pow(c->combo_taps[k]));
        begin.push_back((uint32_t)pows.size());
      }
      pows.push_back(z_pow);
      begin.push_back((uint32_t)pows.size());
      long bad = oracle_combos_divide(combos.data(), combo_count + 1, &pows[0].e[0].v, begin.data(), cycles);
      if (bad >= 0) throw std::runtime_error("combos_divide: nonzero remainder in chunk " + std::to_string(bad));
    }
    Buf final_poly(cycles * EXT, 0);
    {
      OP_TIME("eltwise_sum_extelem");
      oracle_eltwise_sum_extelem(final_poly.data(), final_poly.size(), combos.data(), combos.size() / 4);
    }
    {
      OP_TIME("batch_bit_reverse");
      oracle_batch_bit_reverse(final_poly.data(), final_poly.size(), EXT);
    }
    fri_prove(final_poly, check_group);
  }

  // fri.rs:86-126
  struct Round {
    size_t domain;
    Buf coeffs;
    Buf evaluated;
    std::unique_ptr<MerkleTreeProver> merkle;
  };
  void fri_prove(const Buf& coeffs0, const PolyGroup& check_group) {
    size_t orig_domain = coeffs0.size() / EXT * INV_RATE;
    std::vector<std::unique_ptr<Round>> rounds;
    const Buf* coeffs = &coeffs0;
    while (coeffs->size() / EXT > FRI_MIN_DEGREE) {
      // fri.rs:39-74 ProveRoundInfo::new
      std::unique_ptr<Round> r(new Round);
      size_t size = coeffs->size() / EXT;
      r->domain = size * INV_RATE;
      r->evaluated.assign(r->domain * EXT, 0);
      {
        OP_TIME("batch_expand_into_evaluate_ntt");
        oracle_batch_expand_into_evaluate_ntt(r->evaluated.data(), r->evaluated.size(), coeffs->data(),
                                              coeffs->size(), EXT, log2_ceil(INV_RATE));
      }
      r->merkle.reset(new MerkleTreeProver(suite, r->evaluated, r->domain / FRI_FOLD, FRI_FOLD * EXT, QUERIES));
      r->merkle->commit(iop);
      ExtElem fold_mix = iop.rng->random_ext_elem();
      r->coeffs.assign(size / FRI_FOLD * EXT, 0);
      uint32_t fm[4];
      fold_mix.store(fm);
      OP_TIME("fri_fold");
      oracle_fri_fold(r->coeffs.data(), r->coeffs.size(), coeffs->data(), fm);
      rounds.push_back(std::move(r));
      coeffs = &rounds.back()->coeffs;
    }
    Buf final_coeffs = *coeffs;
    oracle_batch_bit_reverse(final_coeffs.data(), final_coeffs.size(), EXT);
    iop.write_u32(final_coeffs.data(), final_coeffs.size());
    iop.commit(hash_elem_slice(suite, reinterpret_cast<const Elem*>(final_coeffs.data()), final_coeffs.size()));
    for (size_t q = 0; q < QUERIES; q++) {
      size_t pos = iop.rng->random_bits(log2_ceil(orig_domain));
      for (auto& g : groups) g->merkle->prove(iop, pos);
      check_group.merkle->prove(iop, pos);
      for (auto& r : rounds) {
        size_t group = pos % (r->domain / FRI_FOLD);
        r->merkle->prove(iop, group);
        pos = group;
      }
    }
  }
};

}  // namespace

// "name=seconds:calls;..." for every Hal op timed since the last reset (reset = nonzero)
extern "C" size_t oracle_op_times(char* buf, size_t cap, int reset) {
  std::lock_guard<std::mutex> lk(g_op_mu);
  std::string s;
  for (auto& kv : g_op_time)
    s += kv.first + "=" + std::to_string(kv.second.first) + ":" + std::to_string(kv.second.second) + ";";
  if (reset) g_op_time.clear();
  if (buf && cap) {
    const size_t n = std::min(cap - 1, s.size());
    memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return s.size();
}

extern "C" const char* oracle_eval_check(const oracle_circuit_t* c, uint32_t* check,
                                         const uint32_t** groups, const uint32_t* mix,
                                         const uint32_t* global, const uint32_t* poly_mix,
                                         uint32_t po2) {
  try {
    eval_check(c, check, groups, mix, global, ExtElem::raw(poly_mix), po2);
  } catch (const std::exception& e) {
    return strdup(e.what());
  }
  return nullptr;
}

extern "C" const char* oracle_eval_check_sampled(const oracle_circuit_t* c, const uint64_t* group_seeds,
                                                 const uint32_t* mix, const uint32_t* global,
                                                 const uint32_t* poly_mix, uint32_t po2, const uint64_t* cycles,
                                                 size_t n, uint32_t* out) {
  try {
    eval_check_sampled(c, group_seeds, mix, global, ExtElem::raw(poly_mix), po2, cycles, n, out);
  } catch (const std::exception& e) {
    return strdup(e.what());
  }
  return nullptr;
}

// The reference's compiled poly_fp at one cycle whose taps read given base-field values
// (test infrastructure: pins the verifier's poly_ext to the reference's constraint code).
// poly_fp reads a tap only as args[col*steps + ((cycle - 4*back) & (steps-1))], so a small
// window domain per group holds tap i's value at its (col, back) position.
extern "C" const char* oracle_poly_fp_at_taps(const oracle_circuit_t* c, const uint32_t* tap_values,
                                              const uint32_t* mix, const uint32_t* global,
                                              const uint32_t* poly_mix, uint32_t* out) {
  try {
    if (!c->poly_fp) throw std::runtime_error("circuit has no poly_fp (oracle/_ref not built?)");
    TapSet taps{c};
    uint32_t max_back = 0;
    for (size_t i = 0; i < c->n_taps; i++) max_back = std::max(max_back, taps.tap(i)->back);
    size_t win = 1;
    while (win < INV_RATE * (max_back + 2)) win <<= 1;
    const size_t local = INV_RATE * (max_back + 1);
    std::vector<Buf> w(c->n_groups);
    for (size_t g = 0; g < c->n_groups; g++) w[g].assign(taps.group_size(g) * win, 0);
    for (size_t i = 0; i < c->n_taps; i++) {
      const Tap* t = taps.tap(i);
      w[t->group][t->offset * win + ((local - INV_RATE * t->back) & (win - 1))] = tap_values[i];
    }
    std::vector<const uint32_t*> args(c->n_eval_args);
    for (size_t i = 0; i < c->n_eval_args; i++) {
      int a = c->eval_args[i];
      args[i] = a >= 0 ? w[a].data() : (a == -1 ? mix : global);
    }
    std::vector<ExtElem> pows = map_pow(ExtElem::raw(poly_mix), c->poly_mix_powers, c->n_poly_mix);
    if (const char* err = c->poly_fp(local, win, &pows[0].e[0].v, args.data(), out)) return err;
  } catch (const std::exception& e) {
    return strdup(e.what());
  }
  return nullptr;
}

// The witness generator's accumulation between the mix draw and the accum commit
// (WitnessGenerator::accum, circuit/rv32im/src/prove/witgen/mod.rs:178-223): fills `accum`
// from the drawn mix; returns NULL or a message.
typedef const char* (*oracle_accum_cb)(const uint32_t* mix, uint32_t* accum, void* ctx);

static const char* prove_segment_impl(const oracle_circuit_t* c, int suite, uint32_t po2, const uint32_t* code,
                                      const uint32_t* data, uint32_t* accum, oracle_accum_cb cb, void* cb_ctx,
                                      uint32_t* global, int write_version, uint32_t version, uint32_t* seal,
                                      size_t seal_cap, size_t* seal_len, uint32_t* mix_out) {
  try {
    Prover p(c, suite);
    if (write_version) p.iop.proof.push_back(version);
    Elem psi[16], ci[16];
    for (int i = 0; i < 16; i++) {
      psi[i] = Elem::from((uint8_t)PROOF_SYSTEM_INFO[i]);
      ci[i] = Elem::from(c->circuit_info[i]);
    }
    p.iop.commit(hash_elem_slice(suite, psi, 16));
    p.iop.commit(hash_elem_slice(suite, ci, 16));
    std::vector<Elem> header(c->output_size + 1);
    for (size_t i = 0; i < c->output_size; i++) {
      Elem v = Elem::raw(global[i]).valid_or_zero();
      global[i] = v.v;
      header[i] = v;
    }
    header[c->output_size] = Elem::raw(po2);
    p.iop.commit(hash_elem_slice(suite, header.data(), header.size()));
    p.iop.write_u32(&header[0].v, header.size());
    p.po2 = po2;
    p.cycles = size_t(1) << po2;
    // group ids: accum 0, code/ctrl 1, data 2 (rv32im defs.rs.inc, recursion lib.rs:46-49)
    p.commit_group(1, code);
    p.commit_group(2, data);
    std::vector<uint32_t> mix(c->mix_size);
    for (size_t i = 0; i < c->mix_size; i++) mix[i] = p.iop.rng->random_elem().v;
    if (mix_out) memcpy(mix_out, mix.data(), mix.size() * 4);
    if (cb) {
      if (const char* e = cb(mix.data(), accum, cb_ctx)) throw std::runtime_error(std::string("accumulation: ") + e);
    }
    p.commit_group(0, accum);
    p.finalize(mix.data(), global);
    if (seal_len) *seal_len = p.iop.proof.size();
    if (seal && p.iop.proof.size() <= seal_cap) memcpy(seal, p.iop.proof.data(), p.iop.proof.size() * 4);
    else if (seal) return strdup("seal buffer too small");
  } catch (const std::exception& e) {
    return strdup(e.what());
  }
  return nullptr;
}

extern "C" const char* oracle_prove_segment(const oracle_circuit_t* c, int suite, uint32_t po2,
                                            const uint32_t* code, const uint32_t* data,
                                            const uint32_t* accum, uint32_t* global,
                                            int write_version, uint32_t version, uint32_t* seal,
                                            size_t seal_cap, size_t* seal_len, uint32_t* mix_out) {
  return prove_segment_impl(c, suite, po2, code, data, const_cast<uint32_t*>(accum), nullptr, nullptr, global,
                            write_version, version, seal, seal_cap, seal_len, mix_out);
}

// the same with the accum group filled by `cb` once the mix is drawn (prove_core's order)
extern "C" const char* oracle_prove_segment_cb(const oracle_circuit_t* c, int suite, uint32_t po2,
                                               const uint32_t* code, const uint32_t* data, uint32_t* accum,
                                               oracle_accum_cb cb, void* cb_ctx, uint32_t* global,
                                               int write_version, uint32_t version, uint32_t* seal,
                                               size_t seal_cap, size_t* seal_len, uint32_t* mix_out) {
  return prove_segment_impl(c, suite, po2, code, data, accum, cb, cb_ctx, global, write_version, version, seal,
                            seal_cap, seal_len, mix_out);
}
