// The reference prover over the per-op C ABI (integration/hal_prover.h): every device step is
// one r0hip_* Hal call, in the order and with the arguments of
//   risc0/zkp/src/prove/prover.rs:38-393      (make_coeffs, commit_group, finalize)
//   risc0/zkp/src/prove/poly_group.rs:55-83   (PolyGroup::new)
//   risc0/zkp/src/prove/merkle.rs:54-140      (MerkleTreeProver::{new, commit, prove})
//   risc0/zkp/src/prove/fri.rs:39-126         (fri_prove)
//   risc0/circuit/rv32im/src/prove/hal/mod.rs:143-224, witgen/mod.rs:106-223 (prove_core)
// as integration/rust/hal_hip.rs forwards them (tests/hal_prover.py is the same sequence in
// Python). The host holds what the reference host holds: the transcript, the out-of-domain
// evaluations and the register polynomials.
#include "hal_prover.h"

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../risc0_amd/csrc/bb31.h"
#include "../risc0_amd/csrc/transcript.h"

namespace {
using namespace r0;

constexpr size_t INV_RATE = 4, QUERIES = 50, FRI_FOLD = 16, FRI_MIN_DEGREE = 256, EXT = 4, CHECK_SIZE = 16;
const char PROOF_SYSTEM_INFO[] = "RISC0_STARK:v1__";  // adapter.rs:120

// ffi_wrap (risc0/sys/src/lib.rs:53-75): a non-NULL result is the error message
void ok(const char* err) {
  if (err) {
    std::string m(err);
    free(const_cast<char*>(err));
    throw std::runtime_error(m);
  }
}

size_t lg(size_t n) {
  size_t r = 0;
  while ((size_t(1) << r) < n) r++;
  if ((size_t(1) << r) != n) throw std::runtime_error("halp: size is not a power of two");
  return r;
}

// a device buffer of u32 words (BufferImpl over cust's DeviceBuffer; freed on drop)
struct Buf {
  uint32_t* p = nullptr;
  size_t words = 0;
  // get_at through a page-locked host mirror of the whole buffer (hal_hip.rs BufferImpl::
  // get_at on a Merkle node heap). hash_fold's root layer starts one device-to-host copy of the
  // heap beside the Prover's next calls (mirror_start: r0hip_memcpy_d2h_start); get_at reads the
  // mirror once it has landed and reads the one node synchronously until then (the root and top
  // layer right after the build). The Prover writes a node heap only while it builds the tree
  // (hash_rows, hash_fold), so a tree's ~50 x 17 openings cost one overlapped bulk copy (268 MB
  // at po2=20, ~5 ms of PCIe) instead of one synchronous 13 us copy per node.
  mutable uint32_t* host = nullptr;
  mutable bool host_ok = false;
  mutable void* pending = nullptr;  // the mirror's copy in flight
  // gather_sample into a buffer with no device memory yet (hal_hip.rs DeviceAlloc::gathered):
  // the words are gathered straight to the host (r0hip_gather_sample_host) and read from there;
  // MerkleTreeProver::prove's sample is only viewed, so it never gets device memory
  std::vector<uint32_t> gathered;
  Buf() = default;
  explicit Buf(size_t n) : words(n) {
    void* d = nullptr;
    ok(r0hip_alloc(&d, (n ? n : 1) * 4));
    p = static_cast<uint32_t*>(d);
  }
  Buf(Buf&& o) noexcept
      : p(o.p), words(o.words), host(o.host), host_ok(o.host_ok), pending(o.pending), gathered(std::move(o.gathered)) {
    o.p = nullptr;
    o.host = nullptr;
    o.pending = nullptr;
  }
  Buf& operator=(Buf&& o) noexcept {
    std::swap(p, o.p);
    std::swap(words, o.words);
    std::swap(host, o.host);
    std::swap(host_ok, o.host_ok);
    std::swap(pending, o.pending);
    std::swap(gathered, o.gathered);
    return *this;
  }
  // alloc_elem as the HAL does it: the device allocation waits for the first device use
  static Buf unallocated(size_t n) {
    Buf b;
    b.words = n;
    return b;
  }
  // Hal::gather_sample(this, src, idx, size, stride) (cuda.rs:589-603)
  void gather_sample(const Buf& src, size_t idx, size_t size, size_t stride) {
    if (!p && size == words) {
      gathered.resize(size);
      ok(r0hip_gather_sample_host(gathered.data(), src.p, idx, size, stride));
      return;
    }
    if (!p) *this = Buf(words);
    ok(r0hip_gather_sample(p, src.p, idx, size, stride));
  }
  ~Buf() {
    settle();
    if (p) free(const_cast<char*>(r0hip_free(p)));  // a drop never fails the proof
    if (host) free(const_cast<char*>(r0hip_host_free(host)));
  }
  // wait out a mirror copy in flight (before the buffer is written or freed)
  void settle() const noexcept {
    if (!pending) return;
    int done = 0;
    free(const_cast<char*>(r0hip_copy_finish(pending, 1, &done)));
    pending = nullptr;
  }
  void written() {
    settle();
    host_ok = false;
  }
  void mirror_start() {
    written();
    if (!host) {
      void* h = nullptr;
      ok(r0hip_host_alloc(&h, words * 4));
      host = static_cast<uint32_t*>(h);
    }
    void* c = nullptr;
    ok(r0hip_memcpy_d2h_start(host, p, words * 4, &c));
    pending = c;
    host_ok = true;  // valid once `pending` has finished
  }
  // n words at off: from the landed mirror, else one synchronous copy
  const uint32_t* at(size_t off, size_t n, uint32_t* one) const {
    if (host_ok && pending) {
      int done = 0;
      void* c = pending;
      pending = nullptr;  // finish releases the handle when done; keep it otherwise
      ok(r0hip_copy_finish(c, 0, &done));
      if (!done) pending = c;
    }
    if (host_ok && !pending) return host + off;
    ok(r0hip_memcpy_d2h(one, p + off, n * 4));
    return one;
  }
  static Buf from(const uint32_t* h, size_t n) {
    Buf b(n);
    if (n) ok(r0hip_memcpy_h2d(b.p, h, n * 4));
    return b;
  }
  std::vector<uint32_t> to_host(size_t off = 0, size_t n = SIZE_MAX) const {
    if (n == SIZE_MAX) n = words - off;
    if (!p && gathered.size() == words)
      return std::vector<uint32_t>(gathered.begin() + off, gathered.begin() + off + n);
    std::vector<uint32_t> h(n);
    if (n) ok(r0hip_memcpy_d2h(h.data(), p + off, n * 4));
    return h;
  }
};

struct Profile {
  std::ostringstream os;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void mark(const char* name) {
    auto now = std::chrono::steady_clock::now();
    os << name << "=" << std::chrono::duration<double, std::milli>(now - t).count() << ";";
    t = now;
  }
};
thread_local std::string g_profile;

FpExt fe_words(const uint32_t* w) { return FpExt{{w[0], w[1], w[2], w[3]}}; }

// MerkleTreeProver (prove/merkle.rs:26-140, MerkleTreeParams merkle.rs:39-67)
struct Merkle {
  const Buf* matrix;
  size_t rows, cols, top_size = 1;
  Buf nodes;
  Digest root;
  int suite;
  Merkle(int s, const Buf& m, size_t r, size_t c) : matrix(&m), rows(r), cols(c), nodes(r * 2 * 8), suite(s) {
    const size_t layers = lg(rows);
    size_t top_layer = 0;
    for (size_t i = 1; i < layers; i++) {
      if ((size_t(1) << i) > QUERIES) break;
      top_layer = i;
    }
    top_size = size_t(1) << top_layer;
    ok(r0hip_hash_rows(suite, nodes.p + rows * 8, matrix->p, rows, cols));
    for (size_t i = layers; i-- > 0;) ok(r0hip_hash_fold(suite, nodes.p, (size_t(1) << i) * 2, size_t(1) << i));
    nodes.mirror_start();
    uint32_t one[8];
    memcpy(root.w, nodes.at(8, 8, one), 32);  // get_at(1)
  }
  void commit(WriteIOP& iop) const {
    std::vector<uint32_t> top(top_size * 8);  // nodes.slice(top_size, top_size).view
    iop.write(nodes.at(top_size * 8, top.size(), top.data()), top.size());
    iop.commit(root);
  }
  // prove/merkle.rs:108-140: gather_sample, then one get_at per node up the tree
  void prove(WriteIOP& iop, size_t idx) const {
    Buf sample = Buf::unallocated(cols);  // hal.alloc_elem("sample", cols)
    sample.gather_sample(*matrix, idx, cols, rows);
    auto s = sample.to_host();  // sample.view
    iop.write(s.data(), s.size());
    idx += rows;
    while (idx >= 2 * top_size) {
      const size_t low = idx % 2;
      idx /= 2;
      uint32_t one[8];
      iop.write(nodes.at((2 * idx + (1 - low)) * 8, 8, one), 8);
    }
  }
};

// PolyGroup::new (poly_group.rs:55-83): coeffs already interpolated and zk-shifted
struct PolyGroup {
  Buf coeffs, evaluated;
  size_t count;
  Merkle* merkle = nullptr;
  PolyGroup(int suite, Buf c, size_t cnt, size_t size) : coeffs(std::move(c)), count(cnt) {
    const size_t domain = size * INV_RATE;
    evaluated = Buf(count * domain);
    ok(r0hip_batch_expand_into_evaluate_ntt(evaluated.p, coeffs.p, count, uint32_t(lg(domain)), uint32_t(lg(INV_RATE))));
    ok(r0hip_batch_bit_reverse(coeffs.p, count, uint32_t(lg(size))));
    merkle = new Merkle(suite, evaluated, domain, count);
  }
  ~PolyGroup() { delete merkle; }
};

FpExt poly_eval(const std::vector<FpExt>& c, FpExt x) {
  FpExt mul = fe_one(), tot = fe_zero();
  for (auto& v : c) {
    tot = fe_add(tot, fe_mul(v, mul));
    mul = fe_mul(mul, x);
  }
  return tot;
}
FpExt poly_divide(std::vector<FpExt>& p, FpExt z) {  // core/poly.rs:81-89
  FpExt cur = fe_zero();
  for (size_t i = p.size(); i-- > 0;) {
    FpExt next = fe_add(fe_mul(z, cur), p[i]);
    p[i] = cur;
    cur = next;
  }
  return cur;
}
void poly_interpolate(FpExt* out, size_t out_len, const FpExt* x, const FpExt* fx, size_t size) {  // core/poly.rs:41-78
  if (size == 1) {
    out[0] = fx[0];
    return;
  }
  if (size == 2) {
    out[1] = fe_mul(fe_sub(fx[1], fx[0]), fe_inv(fe_sub(x[1], x[0])));
    out[0] = fe_sub(fx[0], fe_mul(out[1], x[0]));
    return;
  }
  std::vector<FpExt> ft(size + 1, fe_zero());
  ft[0] = fe_one();
  for (size_t i = 0; i < size; i++)
    for (size_t j = i + 1; j-- > 0;) {
      FpExt v = ft[j];
      ft[j + 1] = fe_add(ft[j + 1], v);
      ft[j] = fe_mul(ft[j], fe_neg(x[i]));
    }
  for (size_t i = 0; i < out_len; i++) out[i] = fe_zero();
  for (size_t i = 0; i < size; i++) {
    std::vector<FpExt> fr = ft;
    poly_divide(fr, x[i]);
    FpExt mul = fe_mul(fx[i], fe_inv(poly_eval(fr, x[i])));
    for (size_t j = 0; j < size; j++) out[j] = fe_add(out[j], fe_mul(mul, fr[j]));
  }
}

struct Tap {
  uint32_t offset, back, group, combo, skip;
};

struct Prover {
  const char* circuit;
  const halp_taps& t;
  int suite;
  WriteIOP iop;
  size_t po2 = 0, cycles = 0;
  PolyGroup* groups[3] = {nullptr, nullptr, nullptr};
  Profile prof;
  Prover(const char* c, const halp_taps& taps, int s) : circuit(c), t(taps), suite(s), iop(s) {}
  ~Prover() {
    for (auto* g : groups) delete g;
  }
  const Tap& tap(size_t i) const { return reinterpret_cast<const Tap*>(t.taps)[i]; }
  template <typename F>
  void regs(size_t begin, size_t end, F f) const {  // RegisterIter (taps.rs:202-227)
    size_t cur = begin;
    while (cur < t.n_taps) {
      const size_t next = cur + tap(cur).skip;
      if (next > end) break;
      f(cur);
      cur = next;
    }
  }

  // prover.rs:38-48 make_coeffs + 81-108 commit_group
  void commit_group(size_t g, const uint32_t* witness) {
    const size_t gs = t.group_sizes[g];
    Buf coeffs(gs * cycles);
    ok(r0hip_eltwise_copy_elem(coeffs.p, witness, coeffs.words));
    ok(r0hip_batch_interpolate_ntt(coeffs.p, gs, uint32_t(po2)));
    ok(r0hip_zk_shift(coeffs.p, gs, uint32_t(po2)));
    groups[g] = new PolyGroup(suite, std::move(coeffs), gs, cycles);
    groups[g]->merkle->commit(iop);
  }

  // prover.rs:111-393
  void finalize(const Buf& mix, uint32_t* global) {
    const FpExt poly_mix = iop.rng->random_ext_elem();
    const size_t domain = cycles * INV_RATE;
    Buf check(EXT * domain);
    const uint32_t* gptr[3] = {groups[0]->evaluated.p, groups[1]->evaluated.p, groups[2]->evaluated.p};
    ok(r0hip_eval_check(circuit, check.p, gptr, mix.p, global, poly_mix.c, uint32_t(po2)));
    ok(r0hip_batch_interpolate_ntt(check.p, EXT, uint32_t(lg(domain))));
    prof.mark("eval_check");
    PolyGroup check_group(suite, std::move(check), CHECK_SIZE, cycles);
    check_group.merkle->commit(iop);
    prof.mark("check_group");
    const FpExt z = iop.rng->random_ext_elem();
    const FpExt back_one = fe_from_fp(fp_encode(kRouRev[po2]));
    std::vector<FpExt> all_xs, eval_u;
    for (size_t gid = 0; gid < 3; gid++) {
      std::vector<uint32_t> which;
      std::vector<FpExt> xs;
      for (size_t i = t.group_begin[gid]; i < t.group_begin[gid + 1]; i++) {
        which.push_back(tap(i).offset);
        const FpExt x = fe_mul(fe_pow(back_one, tap(i).back), z);
        xs.push_back(x);
        all_xs.push_back(x);
      }
      Buf dw = Buf::from(which.data(), which.size());
      Buf dx = Buf::from(&xs[0].c[0], xs.size() * 4);
      Buf out(which.size() * 4);
      ok(r0hip_batch_evaluate_any(out.p, groups[gid]->coeffs.p, groups[gid]->count, uint32_t(po2), dw.p, dx.p,
                                  which.size()));
      auto h = out.to_host();
      for (size_t i = 0; i < which.size(); i++) eval_u.push_back(fe_words(&h[4 * i]));
    }
    std::vector<FpExt> coeff_u(eval_u.size(), fe_zero());
    {
      size_t pos = 0;
      regs(0, t.n_taps, [&](size_t cur) {
        const size_t sz = tap(cur).skip;
        poly_interpolate(&coeff_u[pos], coeff_u.size() - pos, &all_xs[pos], &eval_u[pos], sz);
        pos += sz;
      });
    }
    const FpExt z_pow = fe_pow(z, EXT);
    {
      std::vector<uint32_t> which(CHECK_SIZE);
      for (size_t i = 0; i < CHECK_SIZE; i++) which[i] = uint32_t(i);
      std::vector<FpExt> xs(CHECK_SIZE, z_pow);
      Buf dw = Buf::from(which.data(), which.size()), dx = Buf::from(&xs[0].c[0], xs.size() * 4), out(CHECK_SIZE * 4);
      ok(r0hip_batch_evaluate_any(out.p, check_group.coeffs.p, CHECK_SIZE, uint32_t(po2), dw.p, dx.p, CHECK_SIZE));
      auto h = out.to_host();
      for (size_t i = 0; i < CHECK_SIZE; i++) coeff_u.push_back(fe_words(&h[4 * i]));
    }
    iop.write(&coeff_u[0].c[0], coeff_u.size() * 4);
    iop.commit(hash_elems(suite, &coeff_u[0].c[0], coeff_u.size() * 4));
    prof.mark("eval_u");
    const FpExt mix_fri = iop.rng->random_ext_elem();
    const size_t combo_count = t.combos_count;
    Buf combos(cycles * (combo_count + 1) * 4);
    ok(r0hip_memset32(combos.p, 0, combos.words));
    FpExt cur_mix = fe_one();
    for (size_t gid = 0; gid < 3; gid++) {
      std::vector<uint32_t> which;
      regs(t.group_begin[gid], t.group_begin[gid + 1], [&](size_t cur) { which.push_back(tap(cur).combo); });
      if (which.size() != t.group_sizes[gid]) throw std::runtime_error("halp: group registers != group size");
      ok(r0hip_mix_poly_coeffs(combos.p, groups[gid]->coeffs.p, which.data(), cur_mix.c, mix_fri.c, which.size(),
                               cycles));
      cur_mix = fe_mul(cur_mix, fe_pow(mix_fri, uint32_t(which.size())));
    }
    {
      std::vector<uint32_t> which(CHECK_SIZE, uint32_t(combo_count));
      ok(r0hip_mix_poly_coeffs(combos.p, check_group.coeffs.p, which.data(), cur_mix.c, mix_fri.c, CHECK_SIZE, cycles));
    }
    prof.mark("mix");
    std::vector<uint32_t> reg_sizes, reg_combo_ids;
    regs(0, t.n_taps, [&](size_t cur) {
      reg_sizes.push_back(tap(cur).skip);
      reg_combo_ids.push_back(tap(cur).combo);
    });
    ok(r0hip_combos_prepare(combos.p, &coeff_u[0].c[0], combo_count, cycles, reg_sizes.data(), reg_combo_ids.data(),
                            reg_sizes.size(), mix_fri.c));
    std::vector<FpExt> pows;
    std::vector<uint32_t> begin{0};
    for (size_t i = 0; i < combo_count; i++) {
      for (uint32_t k = t.combo_begin[i]; k < t.combo_begin[i + 1]; k++)
        pows.push_back(fe_mul(z, fe_pow(back_one, t.combo_taps[k])));
      begin.push_back(uint32_t(pows.size()));
    }
    pows.push_back(z_pow);
    begin.push_back(uint32_t(pows.size()));
    int64_t bad = -1;
    ok(r0hip_combos_divide(combos.p, combo_count + 1, &pows[0].c[0], begin.data(), cycles, &bad));
    if (bad >= 0) throw std::runtime_error("halp: combos_divide: nonzero remainder in chunk " + std::to_string(bad));
    Buf final_coeffs(cycles * EXT);
    ok(r0hip_eltwise_sum_extelem(final_coeffs.p, combos.p, combo_count + 1, cycles));
    ok(r0hip_batch_bit_reverse(final_coeffs.p, EXT, uint32_t(po2)));
    combos = Buf();
    prof.mark("divide");
    fri_prove(std::move(final_coeffs), check_group);
  }

  // fri.rs:86-126
  void fri_prove(Buf coeffs, const PolyGroup& check_group) {
    size_t size = coeffs.words / EXT;
    const size_t orig_domain = size * INV_RATE;
    struct Round {
      size_t domain;
      Buf evaluated;
      Merkle* merkle;
      ~Round() { delete merkle; }
    };
    std::vector<std::unique_ptr<Round>> rounds;
    while (size > FRI_MIN_DEGREE) {
      const size_t domain = size * INV_RATE;
      Buf evaluated(domain * EXT);
      ok(r0hip_batch_expand_into_evaluate_ntt(evaluated.p, coeffs.p, EXT, uint32_t(lg(domain)), uint32_t(lg(INV_RATE))));
      rounds.emplace_back(new Round{domain, std::move(evaluated), nullptr});
      Round& r = *rounds.back();
      r.merkle = new Merkle(suite, r.evaluated, domain / FRI_FOLD, FRI_FOLD * EXT);
      r.merkle->commit(iop);
      const FpExt fold_mix = iop.rng->random_ext_elem();
      Buf out(size / FRI_FOLD * EXT);
      ok(r0hip_fri_fold(out.p, coeffs.p, fold_mix.c, size / FRI_FOLD));
      coeffs = std::move(out);
      size /= FRI_FOLD;
    }
    Buf fin(coeffs.words);
    ok(r0hip_eltwise_copy_elem(fin.p, coeffs.p, coeffs.words));
    ok(r0hip_batch_bit_reverse(fin.p, EXT, uint32_t(lg(size))));
    auto h = fin.to_host();
    iop.write(h.data(), h.size());
    iop.commit(hash_elems(suite, h.data(), h.size()));
    prof.mark("fri_fold");
    for (size_t q = 0; q < QUERIES; q++) {
      size_t pos = iop.rng->random_bits(lg(orig_domain));
      for (auto* g : groups) g->merkle->prove(iop, pos);
      check_group.merkle->prove(iop, pos);
      for (auto& r : rounds) {
        const size_t group = pos % (r->domain / FRI_FOLD);
        r->merkle->prove(iop, group);
        pos = group;
      }
    }
    prof.mark("queries");
  }
};

std::vector<uint32_t> prove(const char* circuit, const halp_taps& t, int suite, uint32_t po2, const uint32_t* code,
                            const uint32_t* data, uint32_t* accum, uint32_t* global, int accum_mode, size_t work_cycles,
                            const r0hip_bigint_back* bigint, size_t n_bigint, bool write_version, uint32_t version,
                            std::vector<uint32_t>* mix_out, Profile* outer) {
  Prover p(circuit, t, suite);
  if (write_version) p.iop.proof.push_back(version);
  uint32_t psi[16], ci[16];
  for (int i = 0; i < 16; i++) {
    psi[i] = fp_encode(uint8_t(PROOF_SYSTEM_INFO[i]));
    ci[i] = fp_encode(uint8_t(t.circuit_info[i]));
  }
  p.iop.commit(hash_elems(suite, psi, 16));
  p.iop.commit(hash_elems(suite, ci, 16));
  // global.view_mut (prove/hal/mod.rs:189-196): INVALID -> 0, then header = globals || po2
  std::vector<uint32_t> header(t.output_size + 1);
  ok(r0hip_memcpy_d2h(header.data(), global, t.output_size * 4));
  for (size_t i = 0; i < t.output_size; i++)
    if (header[i] >= kP) header[i] = 0;
  ok(r0hip_memcpy_h2d(global, header.data(), t.output_size * 4));
  header[t.output_size] = po2;
  p.iop.commit(hash_elems(suite, header.data(), header.size()));
  p.iop.write(header.data(), header.size());
  p.po2 = po2;
  p.cycles = size_t(1) << po2;
  p.prof.mark("start");
  p.commit_group(1, code);
  p.prof.mark("commit_code");
  p.commit_group(2, data);
  p.prof.mark("commit_data");
  std::vector<uint32_t> mix(t.mix_size);
  for (auto& m : mix) m = p.iop.rng->random_elem();
  if (mix_out) *mix_out = mix;
  Buf dmix = Buf::from(mix.data(), mix.size());
  const size_t acc_words = t.group_sizes[0] * p.cycles;
  if (accum_mode == 1) {  // rv32im WitnessGenerator::accum (witgen/mod.rs:178-221)
    ok(r0hip_memset32(accum, 0xFFFFFFFFu, acc_words));
    ok(r0hip_rv32im_bigint_accum_inject(accum, p.cycles, mix.data(), bigint, n_bigint));
    ok(r0hip_rv32im_accum(data, accum, global, dmix.p, p.cycles, t.group_sizes[0], work_cycles));
    ok(r0hip_eltwise_zeroize_elem(accum, acc_words));
  } else if (accum_mode == 2) {  // recursion (prove/witgen.rs:162-177)
    ok(r0hip_recursion_accum(code, global, data, dmix.p, accum, work_cycles, p.cycles));
    ok(r0hip_eltwise_zeroize_elem(accum, acc_words));
  }
  p.prof.mark("accumulate");
  p.commit_group(0, accum);
  p.prof.mark("commit_accum");
  p.finalize(dmix, global);
  if (outer) outer->os << p.prof.os.str();
  return std::move(p.iop.proof);
}

template <typename F>
const char* wrap(F f) {
  try {
    f();
  } catch (const std::exception& e) {
    return strdup(e.what());
  }
  return nullptr;
}

void seal_out(const std::vector<uint32_t>& seal, const std::vector<uint32_t>& mix, uint32_t* h_seal, size_t seal_cap,
              size_t* seal_len, uint32_t* h_mix_out) {
  if (seal_len) *seal_len = seal.size();
  if (h_mix_out) memcpy(h_mix_out, mix.data(), mix.size() * 4);
  if (h_seal) {
    if (seal.size() > seal_cap) throw std::runtime_error("halp: seal buffer too small");
    memcpy(h_seal, seal.data(), seal.size() * 4);
  }
}

}  // namespace

extern "C" {

const char* halp_last_profile(char* buf, size_t cap) {
  if (buf && cap) {
    strncpy(buf, g_profile.c_str(), cap - 1);
    buf[cap - 1] = 0;
  }
  return nullptr;
}

const char* halp_prove_segment(const char* circuit, const halp_taps* taps, int suite, uint32_t po2,
                               const uint32_t* d_code, const uint32_t* d_data, uint32_t* d_accum, uint32_t* d_global,
                               int accum_mode, size_t work_cycles, const r0hip_bigint_back* h_bigint, size_t n_bigint,
                               int write_version, uint32_t version, uint32_t* h_seal, size_t seal_cap, size_t* seal_len,
                               uint32_t* h_mix_out) {
  return wrap([&] {
    if (!circuit || !taps || !d_code || !d_data || !d_accum || !d_global) throw std::runtime_error("halp: null argument");
    Profile prof;
    std::vector<uint32_t> mix;
    auto seal = prove(circuit, *taps, suite, po2, d_code, d_data, d_accum, d_global, accum_mode, work_cycles, h_bigint,
                      n_bigint, write_version != 0, version, &mix, &prof);
    g_profile = prof.os.str();
    seal_out(seal, mix, h_seal, seal_cap, seal_len, h_mix_out);
  });
}

const char* halp_prove_trace(const halp_taps* taps, int suite, uint32_t po2, uint32_t mode, const uint32_t* h_global,
                             const uint32_t* h_inj_index, size_t inj_rows, const uint32_t* h_inj_offsets,
                             const uint32_t* h_inj_values, const r0hip_raw_preflight_trace* preflight,
                             const r0hip_bigint_back* h_bigint, size_t n_bigint, uint32_t* h_seal, size_t seal_cap,
                             size_t* seal_len, uint32_t* h_mix_out) {
  return wrap([&] {
    if (!taps || !h_global || !h_inj_index || !preflight) throw std::runtime_error("halp: null argument");
    Profile prof;
    const size_t n = size_t(1) << po2;
    // WitnessGenerator::new (witgen/mod.rs:106-176): the groups INVALID, the injector scattered
    // into data, stepExec over the preflight (the circuit HAL's generate_witness), zeroize
    Buf code(taps->group_sizes[1] * n), data(taps->group_sizes[2] * n), accum(taps->group_sizes[0] * n);
    Buf global = Buf::from(h_global, taps->output_size);
    ok(r0hip_memset32(code.p, 0, code.words));
    ok(r0hip_memset32(data.p, 0xFFFFFFFFu, data.words));
    const size_t n_inj = h_inj_index[inj_rows];
    {
      Buf idx = Buf::from(h_inj_index, inj_rows + 1), off = Buf::from(h_inj_offsets, n_inj),
          val = Buf::from(h_inj_values, n_inj);
      ok(r0hip_scatter(data.p, idx.p, off.p, val.p, inj_rows));
    }
    r0hip_raw_exec_buffers bufs{{global.p, 1, taps->output_size, true}, {data.p, n, taps->group_sizes[2], true}};
    ok(r0hip_rv32im_witgen(mode, &bufs, preflight, uint32_t(n)));
    ok(r0hip_eltwise_zeroize_elem(data.p, data.words));
    ok(r0hip_eltwise_zeroize_elem(global.p, global.words));
    prof.mark("witgen");
    std::vector<uint32_t> mix;
    auto seal = prove("rv32im", *taps, suite, po2, code.p, data.p, accum.p, global.p, 1, n, h_bigint, n_bigint, true, 2,
                      &mix, &prof);
    g_profile = prof.os.str();
    seal_out(seal, mix, h_seal, seal_cap, seal_len, h_mix_out);
  });
}

}  // extern "C"
