// Segment prover driving the HIP HAL: the STARK protocol of risc0-zkp
//   risc0/zkp/src/prove/prover.rs:38-393   (make_coeffs, commit_group, finalize)
//   risc0/zkp/src/prove/poly_group.rs:55-83, merkle.rs:54-140, fri.rs:39-126
//   risc0/zkp/src/merkle.rs:39-67, core/poly.rs:23-89
// as driven by the circuit segment provers
//   risc0/circuit/rv32im/src/prove/hal/mod.rs:143-224 (rv32im)
//   risc0/circuit/recursion/src/prove/mod.rs:164-230  (recursion)
//
// Every polynomial, evaluation domain and Merkle tree stays resident in HBM; the
// host only holds the transcript. Kernels are queued on one stream and the host
// synchronises only where the protocol needs a value back: each Merkle root
// (Fiat-Shamir), the out-of-domain evaluations, the division remainders, the
// final FRI coefficients and one batched gather of every query opening.
#include <chrono>
#include <cstring>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "circuit.h"
#include "devmem.h"
#include "runtime.h"
#include "transcript.h"

namespace r0 {

// launchers implemented in eltwise.hip (declared here to keep runtime.h small)
void combos_sub(hipStream_t s, uint32_t* combos, const uint32_t* deltas, size_t rows, size_t width,
                size_t cycles);
void gather_words(hipStream_t s, uint32_t* dst, const uint32_t* const* bases, const uint32_t* base_id,
                  const uint64_t* offsets, size_t n);

namespace {

constexpr size_t INV_RATE = 4, QUERIES = 50, FRI_FOLD = 16, FRI_MIN_DEGREE = 256, EXT = 4,
                 CHECK_SIZE = INV_RATE * EXT;
const char PROOF_SYSTEM_INFO[] = "RISC0_STARK:v1__";  // adapter.rs:120

size_t log2_exact(size_t v) {
  size_t r = 0;
  while ((size_t(1) << r) < v) r++;
  R0_REQUIRE((size_t(1) << r) == v, "size is not a power of two");
  return r;
}

// host copies through a stream-ordered D2H followed by a sync
void d2h(void* h, const void* d, size_t bytes) { download(h, d, bytes); }
template <typename T>
uint32_t* upload(const std::vector<T>& v, int slot) {
  size_t bytes = v.size() * sizeof(T);
  uint32_t* d = static_cast<uint32_t*>(scratch(bytes ? bytes : 16, slot));
  upload_async(d, v.data(), bytes);
  return d;
}

struct Profile {
  std::vector<std::pair<std::string, hipEvent_t>> marks;
  void mark(const std::string& name) {
    hipEvent_t e;
    HIP_OK(hipEventCreate(&e));
    HIP_OK(hipEventRecord(e, stream()));
    marks.push_back({name, e});
  }
  std::string finish() {
    HIP_OK(hipStreamSynchronize(stream()));
    std::ostringstream os;
    for (size_t i = 1; i < marks.size(); i++) {
      float ms = 0;
      HIP_OK(hipEventElapsedTime(&ms, marks[i - 1].second, marks[i].second));
      os << marks[i].first << "=" << ms << ";";
    }
    for (auto& m : marks) (void)hipEventDestroy(m.second);
    marks.clear();
    return os.str();
  }
};

// merkle.rs:39-67 + prove/merkle.rs:26-140
struct MerkleTree {
  size_t rows = 0, cols = 0, layers = 0, top_size = 1;
  const uint32_t* matrix = nullptr;  // device, owned by the PolyGroup / FRI round
  DevBuf nodes;                      // heap of 2*rows digests, root at 1
  Digest root;
  std::vector<uint32_t> top;  // nodes[top_size .. 2*top_size)

  void build(int suite, const uint32_t* m, size_t r, size_t c) {
    DevBuf n(r * 2 * 8);
    {
      Span sp("commit");  // prove/merkle.rs:85
      merkle_tree(stream(), suite, n.p, m, r, c);
    }
    finish(std::move(n), m, r, c);
  }
  // the leaves are already in leaf_nodes[r .. 2r) (hash_rows_range as the matrix arrived)
  void build_from_leaves(int suite, DevBuf leaf_nodes, const uint32_t* m, size_t r, size_t c) {
    {
      Span sp("commit");
      merkle_layers(stream(), suite, leaf_nodes.p, r, c);
    }
    finish(std::move(leaf_nodes), m, r, c);
  }
  void finish(DevBuf n, const uint32_t* m, size_t r, size_t c) {
    rows = r;
    cols = c;
    matrix = m;
    nodes = std::move(n);
    layers = log2_exact(rows);
    size_t top_layer = 0;
    for (size_t i = 1; i < layers; i++) {
      if ((size_t(1) << i) > QUERIES) break;
      top_layer = i;
    }
    top_size = size_t(1) << top_layer;
    // root (node 1) .. end of the top layer in one copy
    std::vector<uint32_t> h((2 * top_size - 1) * 8);
    d2h(h.data(), nodes.p + 8, h.size() * 4);
    memcpy(root.w, h.data(), 32);
    top.assign(h.begin() + (top_size - 1) * 8, h.end());
  }
  void commit(WriteIOP& iop) const {
    iop.write(top.data(), top.size());
    iop.commit(root);
  }
};

// From po2 = 12 the coefficient rows stay in the bit-reversed order the inverse NTT leaves
// (the order the forward NTT takes): evaluate_any reads them with bit-reversed power tables
// and mix_poly_coeffs is elementwise, so the only natural-order consumer is combos_divide,
// which gets the (combo_count + 1) mixed rows reversed instead of every trace column.
bool coeffs_stay_bitrev(size_t po2) { return po2 >= kEvalBitrevMinLog; }

struct PolyGroup {
  DevBuf coeffs;
  size_t count = 0;
  bool bitrev = false;  // coeffs rows in bit-reversed order
  DevBuf evaluated;
  MerkleTree tree;
  // poly_group.rs:63-83 (coeffs already interpolated + zk-shifted)
  PolyGroup(int suite, DevBuf c, size_t cnt, size_t po2)
      : coeffs(std::move(c)), count(cnt), bitrev(coeffs_stay_bitrev(po2)) {
    size_t size = size_t(1) << po2, domain = size * INV_RATE;
    evaluated = DevBuf(count * domain);
    ntt_evaluate(stream(), evaluated.p, coeffs.p, count, uint32_t(po2 + 2), 2);
    if (!bitrev) bit_reverse(stream(), coeffs.p, count, uint32_t(po2));
    tree.build(suite, evaluated.p, domain, count);
  }
  // coefficients (natural order below po2 12), evaluations and leaf digests already made
  // chunk by chunk
  PolyGroup(int suite, DevBuf c, DevBuf ev, DevBuf leaf_nodes, size_t cnt, size_t po2)
      : coeffs(std::move(c)), count(cnt), bitrev(coeffs_stay_bitrev(po2)), evaluated(std::move(ev)) {
    tree.build_from_leaves(suite, std::move(leaf_nodes), evaluated.p, (size_t(1) << po2) * INV_RATE, count);
  }
};

FpExt fe_from_words(const uint32_t* w) { return FpExt{{w[0], w[1], w[2], w[3]}}; }

// core/poly.rs (host, tiny)
FpExt poly_eval(const std::vector<FpExt>& c, FpExt x) {
  FpExt mul = fe_one(), tot = fe_zero();
  for (auto& v : c) {
    tot = fe_add(tot, fe_mul(v, mul));
    mul = fe_mul(mul, x);
  }
  return tot;
}
FpExt poly_divide_host(std::vector<FpExt>& p, FpExt z) {
  FpExt cur = fe_zero();
  for (size_t i = p.size(); i-- > 0;) {
    FpExt next = fe_add(fe_mul(z, cur), p[i]);
    p[i] = cur;
    cur = next;
  }
  return cur;
}
// poly.rs:41-78 (the reference clears the whole tail of `out`; later registers overwrite it)
void poly_interpolate(FpExt* out, size_t out_len, const FpExt* x, const FpExt* fx, size_t size) {
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
    poly_divide_host(fr, x[i]);
    FpExt mul = fe_mul(fx[i], fe_inv(poly_eval(fr, x[i])));
    for (size_t j = 0; j < size; j++) out[j] = fe_add(out[j], fe_mul(mul, fr[j]));
  }
}

std::vector<FpExt> map_pow(FpExt base, const uint32_t* exps, size_t n) {  // field/mod.rs:243-270
  std::vector<FpExt> r;
  if (!n) return r;
  r.push_back(fe_pow(base, exps[0]));
  for (size_t i = 1; i < n; i++)
    r.push_back(exps[i] == exps[i - 1] + 1 ? fe_mul(r.back(), base)
                                           : fe_mul(r.back(), fe_pow(base, exps[i] - exps[i - 1])));
  return r;
}

}  // namespace

// eval_check for one circuit (rv32im/src/prove/hal/cpu.rs:145-207 semantics)
void run_eval_check(const CircuitDef& c, uint32_t* check, const uint32_t* const* groups, const uint32_t* mix,
                    const uint32_t* global, FpExt poly_mix, size_t po2, const uint32_t* h_mix,
                    const uint32_t* h_global) {
  hipStream_t s = stream();
  EvalCheckInfo info;
  c.info(&info);
  size_t steps = size_t(1) << po2, domain = steps * INV_RATE;
  std::vector<FpExt> pm = map_pow(poly_mix, c.poly_mix_powers, c.n_poly_mix);
  R0_REQUIRE(pm.size() >= size_t(info.npm), "poly_mix table shorter than the kernels expect");
  pm.resize(info.npm);
  for (int j = 0, k = 0; j < info.ncombos; j++) {
    int n = info.combos[k++];
    FpExt prod = fe_one();
    for (int q = 0; q < n; q++) prod = fe_mul(prod, pm[info.combos[k++]]);
    pm.push_back(prod);
  }
  // inv((3 * w_D^c)^N - 1) depends only on c mod 4 (w_D^(cN) = w_4^c)
  std::vector<uint32_t> vinv(4);
  uint32_t w = fp_encode(kRouFwd[po2 + 2]);
  for (uint32_t q = 0; q < 4; q++) {
    uint32_t x = fp_pow(w, q);
    uint32_t y = fp_pow(fp_mul(fp_encode(3), x), steps);
    vinv[q] = fp_inv(fp_sub(y, kOne));
  }
  std::vector<const uint32_t*> args(c.n_eval_args);
  for (size_t i = 0; i < c.n_eval_args; i++) {
    int a = c.eval_args[i];
    args[i] = a >= 0 ? groups[a] : (a == -1 ? mix : global);
  }
  EvalCheckArgs e;
  e.args = args.data();
  e.nargs = args.size();
  // one base pointer per column the generated program reads (saddr-form tap loads)
  std::vector<const uint32_t*> colptr(info.ncols);
  for (int i = 0; i < info.ncols; i++) colptr[i] = args[info.col_arg[i]] + size_t(info.col_idx[i]) * domain;
  e.colptr = reinterpret_cast<const uint32_t* const*>(upload(colptr, kSlotEcColPtr));
  e.poly_mix = upload(pm, kSlotEcPolyMix);
  std::vector<FpExt> pmn(pm.size());
  for (size_t i = 0; i < pm.size(); i++) pmn[i] = fe_mul_fp(pm[i], kNBeta);
  e.poly_mix_nb = upload(pmn, kSlotEcPolyMixNb);
  e.vinv = upload(vinv, kSlotEcVinv);
  // the lane-independent values (functions of mix, global and poly_mix only), from host
  // copies of mix and global (read back here when the caller has none)
  std::vector<uint32_t> uv(4 * size_t(info.n_uniform > 0 ? info.n_uniform : 1), 0);
  if (info.n_uniform > 0) {
    std::vector<uint32_t> hm, hg;
    if (!h_mix && c.mix_size) {
      hm.resize(c.mix_size);
      d2h(hm.data(), mix, c.mix_size * 4);
      h_mix = hm.data();
    }
    if (!h_global && c.output_size) {
      hg.resize(c.output_size);
      d2h(hg.data(), global, c.output_size * 4);
      h_global = hg.data();
    }
    std::vector<const uint32_t*> hargs(c.n_eval_args, nullptr);
    for (size_t i = 0; i < c.n_eval_args; i++) {
      if (c.eval_args[i] == -1) hargs[i] = h_mix;
      if (c.eval_args[i] == -2) hargs[i] = h_global;
    }
    info.uniform(hargs.data(), reinterpret_cast<const uint32_t*>(pm.data()), uv.data());
  }
  e.uniform = upload(uv, kSlotEcUniform);
  e.acc = static_cast<uint32_t*>(scratch(domain * 16, kSlotEcAcc));
  e.mat_fp = static_cast<uint32_t*>(scratch(size_t(info.mat_fp) * domain * 4 + 16, kSlotEcMatFp));
  e.mat_ext = static_cast<uint32_t*>(scratch(size_t(info.mat_ext) * domain * 16 + 16, kSlotEcMatExt));
  e.check = check;
  e.domain = uint32_t(domain);
  {
    static const uint32_t tile_env = [] {
      const char* t = getenv("R0_EC_TILE");
      return t ? uint32_t(strtoul(t, nullptr, 0)) : 0u;
    }();
    e.tile = tile_env;
    // R0_EC_WIDE (experiments, tests): mask of the kernels that take the column-base tap form,
    // read on every call
    const char* wide_env = getenv("R0_EC_WIDE");
    e.wide = wide_env ? int64_t(strtoull(wide_env, nullptr, 0)) : int64_t(-1);
  }
  double bytes = 16.0 * domain;
  for (int g = 0; g < 3; g++) bytes += 4.0 * domain * c.group_sizes[g];
  Span span("eval_check");
  KScope ks("eval_check", bytes, double(domain) * info.modmuls_per_point);
  c.eval_check(s, e);
}

namespace {

struct Prover {
  const CircuitDef& c;
  int suite;
  WriteIOP iop;
  size_t po2 = 0, cycles = 0;
  std::unique_ptr<PolyGroup> groups[3];
  Profile* prof;

  Prover(const CircuitDef& circ, int s, Profile* p) : c(circ), suite(s), iop(s), prof(p) {}

  // prover.rs:38-48 + 81-108; zk_shift fused into the interpolation's last pass
  // A group still uploading in column chunks (the segment pipeline): each chunk's
  // interpolate, evaluate, bit-reverse and leaf-hash range run as soon as it lands, so the
  // group's NTTs and row hashes overlap its own upload. Same words as commit_group.
  void commit_group_streamed(size_t g, int up_group, const uint32_t* witness, const UploadGate& up) {
    Span span("commit_group");
    hipStream_t s = stream();
    const size_t gs = c.group_size(g), n = cycles, domain = n * INV_RATE, ch = up.chunk_cols(up_group);
    DevBuf coeffs(gs * n), evaluated(gs * domain), nodes(domain * 2 * 8), state(domain * 8);
    for (size_t c0 = 0; c0 < gs; c0 += ch) {
      const size_t cc = std::min(ch, gs - c0);
      up.wait(up_group, c0 + cc, s);
      {
        Span sp("make_coeffs");
        ntt_interpolate_from(s, coeffs.p + c0 * n, witness + c0 * n, cc, uint32_t(po2), true);
      }
      ntt_evaluate(s, evaluated.p + c0 * domain, coeffs.p + c0 * n, cc, uint32_t(po2 + 2), 2);
      if (!coeffs_stay_bitrev(po2)) bit_reverse(s, coeffs.p + c0 * n, cc, uint32_t(po2));
      hash_rows_range(s, suite, nodes.p + domain * 8, state.p, evaluated.p + c0 * domain, domain, cc, c0 == 0,
                      c0 + cc == gs);
    }
    groups[g].reset(new PolyGroup(suite, std::move(coeffs), std::move(evaluated), std::move(nodes), gs, po2));
    groups[g]->tree.commit(iop);
  }

  void commit_group(size_t g, const uint32_t* witness) {
    Span span("commit_group");
    size_t gs = c.group_size(g);
    DevBuf coeffs(gs * cycles);
    {
      Span sp("make_coeffs");
      ntt_interpolate_from(stream(), coeffs.p, witness, gs, uint32_t(po2), true);
    }
    groups[g].reset(new PolyGroup(suite, std::move(coeffs), gs, po2));
    groups[g]->tree.commit(iop);
  }

  // prover.rs:111-393
  void finalize(const uint32_t* mix, const uint32_t* global, const uint32_t* h_mix, const uint32_t* h_global) {
    Span span("finalize");
    hipStream_t s = stream();
    FpExt poly_mix = iop.rng->random_ext_elem();
    size_t domain = cycles * INV_RATE;
    DevBuf check(EXT * domain);
    const uint32_t* gptr[3] = {groups[0]->evaluated.p, groups[1]->evaluated.p, groups[2]->evaluated.p};
    run_eval_check(c, check.p, gptr, mix, global, poly_mix, po2, h_mix, h_global);
    if (prof) prof->mark("eval_check");
    ntt_interpolate(s, check.p, EXT, uint32_t(po2 + 2), false);
    PolyGroup check_group(suite, std::move(check), CHECK_SIZE, po2);
    check_group.tree.commit(iop);
    if (prof) prof->mark("check_group");

    FpExt z = iop.rng->random_ext_elem();
    FpExt back_one = fe_from_fp(fp_encode(kRouRev[po2]));
    std::vector<FpExt> all_xs, eval_u;
    Span span_u("eval_u");
    {
      // one batched launch per group; a single host sync for all of them
      std::vector<std::vector<uint32_t>> whichs(3);
      std::vector<std::vector<FpExt>> xss(3);
      size_t total = 0;
      for (size_t id = 0; id < 3; id++) {
        for (size_t t = c.group_begin[id]; t < c.group_begin[id + 1]; t++) {
          whichs[id].push_back(c.tap(t).offset);
          FpExt x = fe_mul(fe_pow(back_one, c.tap(t).back), z);
          xss[id].push_back(x);
          all_xs.push_back(x);
        }
        total += whichs[id].size();
      }
      DevBuf out((total + CHECK_SIZE) * 4);
      size_t off = 0;
      for (size_t id = 0; id < 3; id++) {
        uint32_t* dx = upload(xss[id], kSlotTapXs + int(id));
        batch_evaluate_any_host(s, groups[id]->coeffs.p, groups[id]->count, uint32_t(po2), whichs[id], dx,
                                out.p + off * 4, groups[id]->bitrev);
        off += whichs[id].size();
      }
      std::vector<uint32_t> h(total * 4);
      d2h(h.data(), out.p, h.size() * 4);
      for (size_t i = 0; i < total; i++) eval_u.push_back(fe_from_words(&h[4 * i]));
    }
    std::vector<FpExt> coeff_u(eval_u.size(), fe_zero());
    {
      size_t pos = 0;
      c.regs(0, c.n_taps, [&](size_t cur) {
        size_t sz = c.tap(cur).skip;
        poly_interpolate(&coeff_u[pos], coeff_u.size() - pos, &all_xs[pos], &eval_u[pos], sz);
        pos += sz;
      });
    }
    FpExt z_pow = fe_pow(z, EXT);
    {
      std::vector<uint32_t> which(CHECK_SIZE);
      for (size_t i = 0; i < CHECK_SIZE; i++) which[i] = uint32_t(i);
      std::vector<FpExt> xs(CHECK_SIZE, z_pow);
      DevBuf out(CHECK_SIZE * 4);
      batch_evaluate_any_host(s, check_group.coeffs.p, CHECK_SIZE, uint32_t(po2), which, upload(xs, kSlotCheckXs), out.p,
                              check_group.bitrev);
      std::vector<uint32_t> h(CHECK_SIZE * 4);
      d2h(h.data(), out.p, h.size() * 4);
      for (size_t i = 0; i < CHECK_SIZE; i++) coeff_u.push_back(fe_from_words(&h[4 * i]));
      iop.write(&coeff_u[0].c[0], coeff_u.size() * 4);
      iop.commit(hash_elems(suite, &coeff_u[0].c[0], coeff_u.size() * 4));
    }
    if (prof) prof->mark("eval_u");
    FpExt mix_fri = iop.rng->random_ext_elem();
    Span span_mix("mix_poly_coeffs");

    size_t combo_count = c.combos_count;
    DevBuf combos(cycles * (combo_count + 1) * 4);
    HIP_OK(hipMemsetAsync(combos.p, 0, combos.words * 4, s));
    {
      FpExt cur_mix = fe_one();
      for (size_t id = 0; id < 3; id++) {
        size_t gs = c.group_size(id);
        std::vector<uint32_t> which;
        c.regs(c.group_begin[id], c.group_begin[id + 1], [&](size_t cur) { which.push_back(c.tap(cur).combo); });
        R0_REQUIRE(which.size() == gs, "group registers != group size");
        mix_poly_coeffs(s, combos.p, groups[id]->coeffs.p, upload(which, kSlotMixWhich), which, cur_mix, mix_fri, gs, cycles);
        cur_mix = fe_mul(cur_mix, fe_pow(mix_fri, gs));
      }
      std::vector<uint32_t> which(CHECK_SIZE, uint32_t(combo_count));
      mix_poly_coeffs(s, combos.p, check_group.coeffs.p, upload(which, kSlotMixWhichCheck), which, cur_mix, mix_fri, CHECK_SIZE,
                      cycles);
      R0_REQUIRE(check_group.bitrev == groups[0]->bitrev && groups[1]->bitrev == groups[0]->bitrev &&
                     groups[2]->bitrev == groups[0]->bitrev,
                 "coefficient groups in mixed orders");
      if (check_group.bitrev) bit_reverse_ext(s, combos.p, combo_count + 1, uint32_t(po2));
    }
    if (prof) prof->mark("mix");
    {
      Span sp("divide");
      // combos_prepare (hal/mod.rs:202-234) as per-row deltas on the low coefficients
      size_t width = 1;
      c.regs(0, c.n_taps, [&](size_t cur) { width = std::max<size_t>(width, c.tap(cur).skip); });
      std::vector<FpExt> deltas((combo_count + 1) * width, fe_zero());
      size_t cur_pos = 0;
      FpExt cur = fe_one();
      c.regs(0, c.n_taps, [&](size_t t) {
        size_t sz = c.tap(t).skip, id = c.tap(t).combo;
        for (size_t i = 0; i < sz; i++)
          deltas[id * width + i] = fe_add(deltas[id * width + i], fe_mul(cur, coeff_u[cur_pos + i]));
        cur = fe_mul(cur, mix_fri);
        cur_pos += sz;
      });
      for (size_t i = 0; i < CHECK_SIZE; i++) {
        deltas[combo_count * width] = fe_add(deltas[combo_count * width], fe_mul(cur, coeff_u[cur_pos]));
        cur_pos++;
        cur = fe_mul(cur, mix_fri);
      }
      combos_sub(s, combos.p, upload(deltas, kSlotCombosDeltas), combo_count + 1, width, cycles);
      // combos_divide (hal/mod.rs:236-257; cuda.rs:1034-1048)
      std::vector<std::vector<FpExt>> zs(combo_count + 1);
      for (size_t i = 0; i < combo_count; i++)
        for (uint32_t k = c.combo_begin[i]; k < c.combo_begin[i + 1]; k++)
          zs[i].push_back(fe_mul(z, fe_pow(back_one, c.combo_taps[k])));
      zs[combo_count].push_back(z_pow);
      size_t maxz = 0;
      for (auto& v : zs) maxz = std::max(maxz, v.size());
      DevBuf rem((combo_count + 1) * maxz * 4);
      HIP_OK(hipMemsetAsync(rem.p, 0, rem.words * 4, s));
      poly_divide_rows(s, combos.p, cycles, zs, rem.p);
      std::vector<uint32_t> h(rem.words);
      d2h(h.data(), rem.p, h.size() * 4);
      for (size_t i = 0; i < h.size(); i++)
        R0_REQUIRE(h[i] == 0, "combos_divide: nonzero remainder in chunk " + std::to_string(i / (4 * maxz)));
    }
    if (prof) prof->mark("divide");
    DevBuf final_poly(cycles * EXT);
    Span span_sum("sum");
    eltwise_sum_extelem(s, final_poly.p, combos.p, cycles, combo_count + 1);
    bit_reverse(s, final_poly.p, EXT, uint32_t(po2));
    combos = DevBuf();
    fri_prove(std::move(final_poly), check_group);
  }

  struct Round {
    size_t domain;
    DevBuf evaluated;
    MerkleTree tree;
  };

  // fri.rs:86-126 with all query openings gathered in one device pass
  void fri_prove(DevBuf coeffs, const PolyGroup& check_group) {
    Span span("fri_prove");
    hipStream_t s = stream();
    size_t size = coeffs.words / EXT;
    size_t orig_domain = size * INV_RATE;
    std::vector<std::unique_ptr<Round>> rounds;
    while (size > FRI_MIN_DEGREE) {
      std::unique_ptr<Round> r(new Round);
      r->domain = size * INV_RATE;
      r->evaluated = DevBuf(r->domain * EXT);
      ntt_evaluate(s, r->evaluated.p, coeffs.p, EXT, uint32_t(log2_exact(r->domain)), 2);
      r->tree.build(suite, r->evaluated.p, r->domain / FRI_FOLD, FRI_FOLD * EXT);
      r->tree.commit(iop);
      FpExt fold_mix = iop.rng->random_ext_elem();
      DevBuf out(size / FRI_FOLD * EXT);
      fri_fold(s, out.p, coeffs.p, fold_mix, size / FRI_FOLD);
      coeffs = std::move(out);
      size /= FRI_FOLD;
      rounds.push_back(std::move(r));
    }
    if (prof) prof->mark("fri_fold");
    {
      DevBuf fin(coeffs.words);
      HIP_OK(hipMemcpyAsync(fin.p, coeffs.p, coeffs.words * 4, hipMemcpyDeviceToDevice, s));
      bit_reverse(s, fin.p, EXT, uint32_t(log2_exact(size)));
      std::vector<uint32_t> h(fin.words);
      d2h(h.data(), fin.p, h.size() * 4);
      iop.write(h.data(), h.size());
      iop.commit(hash_elems(suite, h.data(), h.size()));
    }
    // The query loop only writes to the proof, so the positions can all be drawn first.
    std::vector<size_t> positions(QUERIES);
    for (auto& p : positions) p = iop.rng->random_bits(log2_exact(orig_domain));
    std::vector<const uint32_t*> bases;
    std::vector<uint32_t> base_id;
    std::vector<uint64_t> offs;
    auto add_base = [&](const uint32_t* p) {
      bases.push_back(p);
      return uint32_t(bases.size() - 1);
    };
    struct T {
      const MerkleTree* t;
      uint32_t mat, nodes;
    };
    std::vector<T> trees;
    for (auto& g : groups) trees.push_back({&g->tree, add_base(g->tree.matrix), add_base(g->tree.nodes.p)});
    trees.push_back({&check_group.tree, add_base(check_group.tree.matrix), add_base(check_group.tree.nodes.p)});
    std::vector<T> rtrees;
    for (auto& r : rounds) rtrees.push_back({&r->tree, add_base(r->tree.matrix), add_base(r->tree.nodes.p)});
    auto prove = [&](const T& t, size_t idx) {  // prove/merkle.rs:108-140
      const MerkleTree& m = *t.t;
      for (size_t i = 0; i < m.cols; i++) {
        base_id.push_back(t.mat);
        offs.push_back(idx + i * m.rows);
      }
      idx += m.rows;
      while (idx >= 2 * m.top_size) {
        size_t low = idx % 2;
        idx /= 2;
        size_t other = 2 * idx + (1 - low);
        for (size_t k = 0; k < 8; k++) {
          base_id.push_back(t.nodes);
          offs.push_back(other * 8 + k);
        }
      }
    };
    for (size_t pos : positions) {
      for (auto& t : trees) prove(t, pos);
      for (size_t ri = 0; ri < rounds.size(); ri++) {
        size_t group = pos % (rounds[ri]->domain / FRI_FOLD);
        prove(rtrees[ri], group);
        pos = group;
      }
    }
    DevBuf words(offs.size());
    const uint32_t* const* dbases = reinterpret_cast<const uint32_t* const*>(upload(bases, kSlotQueryBases));
    gather_words(s, words.p, dbases, upload(base_id, kSlotQueryIds), reinterpret_cast<const uint64_t*>(upload(offs, kSlotQueryOffs)),
                 offs.size());
    std::vector<uint32_t> h(offs.size());
    d2h(h.data(), words.p, h.size() * 4);
    iop.write(h.data(), h.size());
    if (prof) prof->mark("queries");
  }
};

thread_local std::string g_last_profile;  // per host thread (segments in flight)

}  // namespace

std::string last_profile() { return g_last_profile; }

// circuit/rv32im/src/prove/hal/mod.rs:181-224 (recursion: prove/mod.rs:176-226, no version word)
// `uploads` (optional): the groups may still be uploading; each is waited for just before
// its first use, so a segment's early phases overlap the upload of its later groups
std::vector<uint32_t> prove_segment(const CircuitDef& c, int suite, uint32_t po2, const uint32_t* code,
                                    const uint32_t* data, const uint32_t* accum, uint32_t* global,
                                    bool write_version, uint32_t version, std::vector<uint32_t>* mix_out,
                                    const UploadGate* uploads, const AccumStep* acc) {
  R0_REQUIRE(suite >= 0 && suite <= 2, "unknown hash suite");
  R0_REQUIRE(!acc || (acc->accum && !accum), "prove_segment: give the accum group or an accumulation, not both");
  R0_REQUIRE(po2 >= 2 && po2 <= 24, "po2 out of range");
  Span span("prove_core");
  hipStream_t s = stream();
  auto gate = [&](int g) {
    if (uploads) uploads->wait(g, SIZE_MAX, s);
  };
  stage_reset();
  Profile prof;
  prof.mark("start");
  Prover p(c, suite, &prof);
  if (write_version) p.iop.proof.push_back(version);
  uint32_t psi[16], ci[16];
  for (int i = 0; i < 16; i++) {
    psi[i] = fp_encode(uint8_t(PROOF_SYSTEM_INFO[i]));
    ci[i] = fp_encode(uint8_t(c.circuit_info[i]));
  }
  p.iop.commit(hash_elems(suite, psi, 16));
  p.iop.commit(hash_elems(suite, ci, 16));
  // header = globals (INVALID -> 0, in place) || po2 as a raw word
  gate(3);
  eltwise_zeroize(s, global, c.output_size);
  std::vector<uint32_t> header(c.output_size + 1);
  d2h(header.data(), global, c.output_size * 4);
  header[c.output_size] = po2;
  p.iop.commit(hash_elems(suite, header.data(), header.size()));
  p.iop.write(header.data(), header.size());
  p.po2 = po2;
  p.cycles = size_t(1) << po2;
  // reference group index, pipeline buffer index (0 code, 1 data, 2 accum)
  auto commit = [&](size_t g, int up_group, const uint32_t* w) {
    const size_t gs = c.group_size(g);
    if (uploads && suite != 2 && gs > uploads->chunk_cols(up_group) && uploads->chunk_cols(up_group) % 16 == 0) {
      p.commit_group_streamed(g, up_group, w, *uploads);
    } else {
      gate(up_group);
      p.commit_group(g, w);
    }
  };
  commit(1, 0, code);
  prof.mark("commit_code");
  commit(2, 1, data);
  prof.mark("commit_data");
  std::vector<uint32_t> mix(c.mix_size);
  for (auto& m : mix) m = p.iop.rng->random_elem();
  if (mix_out) *mix_out = mix;
  DevBuf dmix(mix.size() ? mix.size() : 1);
  upload_async(dmix.p, mix.data(), mix.size() * 4);
  if (acc) {
    Span acc_span("accumulate");
    const size_t rows = p.cycles, cols = c.group_size(0);
    const std::string name = c.name;
    if (acc->fill_invalid) HIP_OK(hipMemsetD32Async(acc->accum, 0xFFFFFFFFu, rows * cols, s));
    if (name == "rv32im") {
      // witgen/mod.rs:182-205: the BigInt states with the final mix, then the step
      rv32im_bigint_inject(s, acc->accum, rows, mix.data(), acc->bigint, acc->n_bigint);
      rv32im_accum(s, data, acc->accum, global, dmix.p, rows, cols, acc->work_cycles);
    } else if (name == "recursion") {
      R0_REQUIRE(acc->n_bigint == 0, "prove_segment: BigInt backs are an rv32im trace record");
      recursion_accum(s, code, global, data, dmix.p, acc->accum, acc->work_cycles, rows);
    } else {
      R0_REQUIRE(false, "prove_segment: no device accumulation for circuit " + name);
    }
    if (!acc->zeroed) eltwise_zeroize(s, acc->accum, rows * cols);
    prof.mark("accumulate");
    p.commit_group(0, acc->accum);  // nothing to wait for: the group never uploads
  } else {
    commit(0, 2, accum);
  }
  prof.mark("commit_accum");
  p.finalize(dmix.p, global, mix.data(), header.data());
  HIP_OK(hipStreamSynchronize(s));
  g_last_profile = prof.finish();
  return std::move(p.iop.proof);
}

}  // namespace r0
