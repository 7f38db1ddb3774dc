#!/usr/bin/env python3
"""Emit the gfx950 eval_check kernels for a circuit from its constraint program
(risc0_amd/circuits/<circuit>.poly.ir, see tools/gen_poly_ir.py).

  check[k*D + cycle] = (poly_fp(cycle) * inv((3*w_D^cycle)^N - 1))[k]
  — risc0/circuit/rv32im/src/prove/hal/cpu.rs:145-207 (rv32im),
    risc0/circuit/recursion-sys/kernels/cxx/ffi.cpp:220-247 (recursion).

MI355X design. One lane per evaluation point, all values in VGPRs. The ~20k-op
program is too large for one kernel (register spills, and LLVM compile time grows
super-linearly: 2.6k ops ~ 100 s with spills, 1.4k ops ~ 3 s without), so it is
scheduled as a short sequence of kernels, each below a cost budget:
  1. linear split: poly_fp = sum_i expr_i * prod(factors_i); accumulate nodes
     (ACC + T*pm[k], ACC + T*U*pm[k]) are split into their summands until every
     term's dependency cone fits the budget or is not an accumulation;
  2. materialisation: for terms still over budget, the largest sub-expression that
     fits is computed by an earlier kernel and stored per point in HBM (4 B per
     Fp, 16 B per FpExt), becoming a leaf for its consumers;
  3. packing: items are packed into kernels in dependency order; each kernel adds
     its terms into an FpExt accumulator; the last one applies the vanishing-
     polynomial inverse (4 distinct values on the 4N domain, from the host) and
     writes the 4 SoA planes.
Trace taps are reloaded by every kernel that needs them (coalesced per column).
Products of several poly_mix powers are folded into host-computed constants.

Usage: gen_eval_check.py CIRCUIT OUTDIR [BUDGET]
Writes OUTDIR/eval_check_<circuit>_k<i>.hip (one per kernel, compiled in parallel)
and OUTDIR/eval_check_<circuit>.hip (launcher).
"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
P = 15 * 2**27 + 1


def load(circuit):
    prog = []
    with open(os.path.join(ROOT, "risc0_amd", "circuits", circuit + ".poly.ir")) as f:
        for line in f:
            if line.startswith("#") or not line.strip():
                continue
            t = line.split()
            prog.append((t[0],) + tuple(int(x) for x in t[1:]))
    return prog


def deps(ins):
    op = ins[0]
    if op in "+-*a":
        return [ins[2], ins[3]]
    if op == "b":
        return [ins[2], ins[3], ins[4]]
    return []


def enc(x):
    return (x % P) * 2**32 % P


class Program:
    def __init__(self, circuit):
        self.circuit = circuit
        self.prog = load(circuit)
        self.byid = {ins[1]: ins for ins in self.prog if ins[0] != "r"}
        self.order = {ins[1]: n for n, ins in enumerate(self.prog) if ins[0] != "r"}
        self.res = [ins for ins in self.prog if ins[0] == "r"][0][1]
        t = {}
        for ins in self.prog:
            op = ins[0]
            if op in ("c", "l", "g"):
                t[ins[1]] = "f"
            elif op in ("e", "a", "b"):
                t[ins[1]] = "e"
            elif op in "+-*":
                t[ins[1]] = "e" if "e" in (t[ins[2]], t[ins[3]]) else "f"
        self.types = t
        self.mat = set()

    def cost(self, v):
        ins = self.byid[v]
        op = ins[0]
        ty = self.types
        if op in "clge":
            return 0
        if op in "+-":
            return 4 if ty[v] == "e" else 1
        if op == "*":
            a, b = ty[ins[2]], ty[ins[3]]
            return 16 if (a, b) == ("e", "e") else (4 if "e" in (a, b) else 1)
        if op == "a":
            return 8 if ty[ins[3]] == "f" else 20
        return 9 if ty[ins[3]] == "f" and ty[ins[4]] == "f" else 24

    def cone(self, roots):
        seen = set()
        rs = set(roots)
        stack = list(roots)
        while stack:
            v = stack.pop()
            if v in seen:
                continue
            seen.add(v)
            if v in self.mat and v not in rs:
                continue
            stack.extend(deps(self.byid[v]))
        return seen

    def cone_cost(self, roots):
        rs = set(roots)
        return sum(self.cost(v) for v in self.cone(roots) if not (v in self.mat and v not in rs))


def modmuls(pg):
    """Field multiplications of the program as written (Fp x Fp = 1, FpExt x Fp = 4,
    FpExt x FpExt = 16; accumulate ops count their products) — the algorithmic op count
    the VALU roofline is quoted in."""
    ty = pg.types
    n = 0
    for ins in pg.prog:
        op = ins[0]
        if op == "*":
            a, b = ty[ins[2]], ty[ins[3]]
            n += 16 if (a, b) == ("e", "e") else (4 if "e" in (a, b) else 1)
        elif op == "a":
            n += 16 if ty[ins[3]] == "e" else 4
        elif op == "b":
            fe = "e" in (ty[ins[3]], ty[ins[4]])
            n += (4 if fe else 1) + (16 if fe else 4)
    return n


def dfs_order(pg, need, roots, leaves):
    """Post-order over `need` from `roots`: an accumulate op visits its running sum
    first, so each term value is computed just before it is added. `leaves` (loads,
    constants, materialised values) are placed separately by the caller."""
    out, seen = [], set()
    for r in roots:
        if r in seen or r not in need:
            continue
        stack = [(r, False)]
        while stack:
            v, done = stack.pop()
            if done:
                out.append(v)
                continue
            if v in seen:
                continue
            seen.add(v)
            stack.append((v, True))
            if v in leaves:
                continue
            ds = [d for d in deps(pg.byid[v]) if d in need and d not in seen]
            for d in reversed(ds):  # first dep (the running sum) is visited first
                stack.append((d, False))
    return out


def term_roots(t):
    return [t[0]] + [x[1] for x in t[1] if x[0] == "v"]


def schedule(pg, budget):
    byid = pg.byid
    # 1. linear split
    terms = [(pg.res, [])]
    while True:
        best, bestc = None, -1
        for i, t in enumerate(terms):
            if byid[t[0]][0] in "ab":
                c = pg.cone_cost(term_roots(t))
                if c > bestc:
                    best, bestc = i, c
        if best is None or bestc <= budget:
            break
        e, f = terms[best]
        ins = byid[e]
        if ins[0] == "a":
            new = [(ins[2], f), (ins[3], f + [("pm", ins[4])])]
        else:
            T, U = ins[3], ins[4]
            if byid[U][0] in "ab" and byid[T][0] not in "ab":
                T, U = U, T
            new = [(ins[2], f), (T, f + [("v", U), ("pm", ins[5])])]
        terms[best:best + 1] = new

    # 2. materialise sub-expressions of over-budget items
    def fix(roots):
        while pg.cone_cost(roots) > budget:
            best, bestc = None, -1
            for v in pg.cone(roots):
                if v in roots or v in pg.mat or byid[v][0] in "clge":
                    continue
                c = pg.cone_cost([v])
                if bestc < c <= budget:
                    best, bestc = v, c
            if best is None:
                raise RuntimeError("cannot materialise below budget")
            pg.mat.add(best)

    for t in terms:
        fix(term_roots(t))

    level = {}

    def lev(v):
        if v not in level:
            level[v] = 1 + max([lev(u) for u in pg.cone([v]) if u != v and u in pg.mat] + [-1])
        return level[v]

    items = []
    for v in pg.mat:
        items.append((lev(v), pg.order[v], "mat", v))
    for n, t in enumerate(terms):
        rs = term_roots(t)
        l = 1 + max([lev(u) for u in pg.cone(rs) if u in pg.mat and u not in rs] + [-1])
        items.append((l, 10**9 + n, "term", t))
    items.sort(key=lambda x: (x[0], x[1]))
    # 3. pack in order; a kernel only reads values produced by earlier kernels
    kernels = []
    cur, cur_roots = [], []
    done = set()
    for it in items:
        roots = [it[3]] if it[2] == "mat" else term_roots(it[3])
        need = [u for u in pg.cone(roots) if u in pg.mat and u not in roots]
        ok = all(u in done for u in need)
        if cur and (not ok or pg.cone_cost(cur_roots + roots) > budget):
            kernels.append(cur)
            done.update(x[3] for x in cur if x[2] == "mat")
            cur, cur_roots = [], []
        cur.append(it)
        cur_roots += roots
    if cur:
        kernels.append(cur)
    return terms, kernels


CHUNK = int(os.environ.get("EC_CHUNK", "0"))
# emission order: "ir" (the reference program's order) or "dfs" (each value computed
# right before its first use, accumulation chains first; loads hoisted EC_PF ops ahead)
ORDER = os.environ.get("EC_ORDER", "dfs")
PF = int(os.environ.get("EC_PF", "512"))
# minimum waves per SIMD requested from the register allocator (1 = no limit)
WAVES = int(os.environ.get("EC_WAVES", "2"))


def kernel_config(circuit, budget):
    """Per-kernel (waves, prefetch) chosen by tools/tune_eval_check.py on an MI355X and
    committed as risc0_amd/circuits/<circuit>.ectune.json; EC_WAVES/EC_PF (if set) or
    the defaults apply to kernels it does not list (or when EC_NOTUNE is set)."""
    path = os.path.join(ROOT, "risc0_amd", "circuits", circuit + ".ectune.json")
    if os.environ.get("EC_NOTUNE") or "EC_WAVES" in os.environ or "EC_PF" in os.environ or not os.path.exists(path):
        return {}
    import json
    with open(path) as f:
        t = json.load(f)
    if t.get("budget") != budget or t.get("order") != ORDER:
        return {}
    return {int(k): v for k, v in t["kernels"].items()}


def emit(circuit, outdir, budget):
    pg = Program(circuit)
    terms, kernels = schedule(pg, budget)
    tune = kernel_config(circuit, budget)
    prog, types = pg.prog, pg.types
    nargs = 1 + max(ins[2] for ins in prog if ins[0] in ("l", "g"))
    npm = max([ins[4] for ins in prog if ins[0] == "a"] + [ins[5] for ins in prog if ins[0] == "b"]) + 1
    mat = sorted(pg.mat, key=lambda v: pg.order[v])
    slot = {}
    nf = ne = 0
    for v in mat:
        if types[v] == "f":
            slot[v] = ("f", nf)
            nf += 1
        else:
            slot[v] = ("e", ne)
            ne += 1
    combo_index = {}
    os.makedirs(outdir, exist_ok=True)

    common = [
        '#include "bb31.h"',
        '#include "evalcheck.h"',
        "namespace r0 {",
        f"namespace ec_{circuit} {{",
        "struct Args {",
        f"  const uint32_t* a[{nargs}];",
        "  const uint32_t* pm;   // poly_mix powers then folded products, FpExt AoS",
        "  const uint32_t* pmn;  // the same times NBETA",
        "  uint32_t* acc;        // FpExt AoS accumulator per point",
        "  uint32_t* check;      // 4 SoA planes",
        "  const uint32_t* vinv; // inv((3x)^N - 1) for cycle & 3",
        "  uint32_t* mf;         // materialised Fp values, [slot][domain]",
        "  uint32_t* me;         // materialised FpExt values, [slot][domain] AoS",
        "  uint32_t domain;",
        "  uint32_t base, count;  // this launch covers points [base, base + count)",
        "};",
        f"constexpr int NPM = {npm};",
        "__device__ __forceinline__ FpExt eadd(FpExt a, FpExt b) { return fe_add(a, b); }",
        "__device__ __forceinline__ FpExt eadd(FpExt a, uint32_t b) { a.c[0] = fp_add(a.c[0], b); return a; }",
        "__device__ __forceinline__ FpExt eadd(uint32_t a, FpExt b) { b.c[0] = fp_add(a, b.c[0]); return b; }",
        "__device__ __forceinline__ FpExt esub(FpExt a, FpExt b) { return fe_sub(a, b); }",
        "__device__ __forceinline__ FpExt esub(FpExt a, uint32_t b) { a.c[0] = fp_sub(a.c[0], b); return a; }",
        "__device__ __forceinline__ FpExt esub(uint32_t a, FpExt b) { return fe_sub(fe_from_fp(a), b); }",
        "__device__ __forceinline__ FpExt emul(FpExt a, FpExt b) { return fe_mul(a, b); }",
        "__device__ __forceinline__ FpExt emul(FpExt a, uint32_t b) { return fe_mul_fp(a, b); }",
        "__device__ __forceinline__ FpExt emul(uint32_t a, FpExt b) { return fe_mul_fp(b, a); }",
        "__device__ __forceinline__ uint32_t emul(uint32_t a, uint32_t b) { return fp_mul(a, b); }",
        "// Lazy FpExt accumulator: four unreduced 64-bit sums of Montgomery products",
        "// (each < p^2); the generator tracks an upper bound per value and folds",
        "// (hi * (2^32 mod p) + lo, < 2^60) before a sum could reach 2^64.",
        "struct Acc { uint64_t c[4]; };",
        "// a canonical value v enters as v * 2^32 (mod p), so the final REDC returns v",
        "__device__ __forceinline__ Acc acc_of(FpExt a) {",
        "  return Acc{{uint64_t(a.c[0]) * kFoldC, uint64_t(a.c[1]) * kFoldC, uint64_t(a.c[2]) * kFoldC,",
        "              uint64_t(a.c[3]) * kFoldC}};",
        "}",
        "__device__ __forceinline__ Acc acc_of(uint32_t a) { return Acc{{uint64_t(a) * kFoldC, 0, 0, 0}}; }",
        "__device__ __forceinline__ Acc acc_fold(Acc a) {",
        "#pragma unroll",
        "  for (int i = 0; i < 4; i++) a.c[i] = fold64(a.c[i]);",
        "  return a;",
        "}",
        "__device__ __forceinline__ FpExt acc_red(Acc a) {",
        "  return FpExt{{mont_reduce(a.c[0]), mont_reduce(a.c[1]), mont_reduce(a.c[2]), mont_reduce(a.c[3])}};",
        "}",
        "__device__ __forceinline__ Acc acc_add(Acc a, Acc b) {",
        "#pragma unroll",
        "  for (int i = 0; i < 4; i++) a.c[i] += b.c[i];",
        "  return a;",
        "}",
        "// a += t * pm[k]  (t in Fp)",
        "__device__ __forceinline__ Acc acc_fp(Acc a, uint32_t t, const uint32_t* pm, int k) {",
        "#pragma unroll",
        "  for (int i = 0; i < 4; i++) a.c[i] += uint64_t(t) * pm[4 * k + i];",
        "  return a;",
        "}",
        "// a += t * pm[k]  (t in FpExt; x^4 = NBETA folded into pmn = NBETA * pm)",
        "__device__ __forceinline__ Acc acc_ext(Acc a, FpExt t, const uint32_t* pm, const uint32_t* pmn, int k) {",
        "  const uint32_t* q = pm + 4 * k;",
        "  const uint32_t* n = pmn + 4 * k;",
        "  a.c[0] += uint64_t(t.c[0]) * q[0] + uint64_t(t.c[1]) * n[3] + uint64_t(t.c[2]) * n[2] + uint64_t(t.c[3]) * n[1];",
        "  a.c[1] += uint64_t(t.c[0]) * q[1] + uint64_t(t.c[1]) * q[0] + uint64_t(t.c[2]) * n[3] + uint64_t(t.c[3]) * n[2];",
        "  a.c[2] += uint64_t(t.c[0]) * q[2] + uint64_t(t.c[1]) * q[1] + uint64_t(t.c[2]) * q[0] + uint64_t(t.c[3]) * n[3];",
        "  a.c[3] += uint64_t(t.c[0]) * q[3] + uint64_t(t.c[1]) * q[2] + uint64_t(t.c[2]) * q[1] + uint64_t(t.c[3]) * q[0];",
        "  return a;",
        "}",
    ]
    common_text = "\n".join(common) + "\n"

    stats = []
    PROD = (P - 1) ** 2
    LIM = 2**64
    RED = P * 2**32
    CANON = (P - 1) * (2**32 % P)  # bound of acc_of(canonical)

    def fold_bound(bd):
        return (bd >> 32) * (2**32 % P) + 2**32 - 1

    for ki, items in enumerate(kernels):
        roots = []
        for it in items:
            roots += [it[3]] if it[2] == "mat" else term_roots(it[3])
        need = pg.cone(roots)
        produced = set(it[3] for it in items if it[2] == "mat")
        loaded = set(v for v in need if v in pg.mat and v not in produced)
        first, last = ki == 0, ki == len(kernels) - 1
        mine = [it[3] for it in items if it[2] == "term"]
        # accumulate ops computed here stay lazy (Acc a<i>); canonical v<i> only where needed
        lazy = set(v for v in need if v not in loaded and pg.byid[v][0] in "ab")
        canon = set(produced & lazy)
        for v in need:
            if v in loaded:
                continue
            ins = pg.byid[v]
            ds = deps(ins)
            for n, d in enumerate(ds):
                if d in lazy and not (ins[0] in "ab" and n == 0):
                    canon.add(d)
        for e, f in mine:
            if f and e in lazy:
                canon.add(e)
            for x in f:
                if x[0] == "v" and x[1] in lazy:
                    canon.add(x[1])
        bound = {}
        L = []
        w = L.append

        # Trace taps and materialised values are re-loaded where they are used instead of
        # being kept live: the program is cut into chunks of CHUNK ops separated by a
        # compiler memory barrier, and a load is emitted (once) in each chunk that needs
        # it. Without this LLVM hoists all ~400 loads to the top and the kernels need
        # 450-512 VGPR+AGPR (one wave per SIMD, exposed load latency).
        remat = set(v for v in need if v in loaded or pg.byid[v][0] == "l") if CHUNK else set()
        chunk = {"n": 0, "ops": 0, "have": {}}

        def ref(x):
            if x not in remat:
                return f"v{x}"
            h = chunk["have"]
            if x not in h:
                nm = f"v{x}_{chunk['n']}"
                h[x] = nm
                if x in loaded:
                    kind, s_ = slot[x]
                    if kind == "f":
                        w(f"  const uint32_t {nm} = A.mf[uint64_t({s_}u) * A.domain + cycle];")
                    else:
                        w(f"  FpExt {nm}; {{ uint4 t = reinterpret_cast<const uint4*>(A.me)[uint64_t({s_}u) * A.domain"
                          f" + cycle]; {nm} = FpExt{{{{t.x, t.y, t.z, t.w}}}}; }}")
                else:
                    ins = pg.byid[x]
                    w(f"  const uint32_t {nm} = A.a[{ins[2]}][{ins[3]}u * A.domain + ((cycle - {4 * ins[4]}u) & mask)];")
            return h[x]

        def tick():
            chunk["ops"] += 1
            if CHUNK and chunk["ops"] >= CHUNK:
                w("  asm volatile(\"\" ::: \"memory\");")
                chunk["n"] += 1
                chunk["ops"] = 0
                chunk["have"] = {}

        def acc_src(x):
            """(expression, bound) of an Acc holding value x."""
            if x in lazy:
                return f"a{x}", bound[x]
            return f"acc_of({ref(x)})", CANON

        def room(expr, bd, k):
            """fold expr first if adding k more products could overflow 64 bits."""
            if bd + k * PROD >= LIM:
                return f"acc_fold({expr})", fold_bound(bd)
            return expr, bd

        def reduced(expr, bd):
            if bd >= RED:
                return f"acc_red(acc_fold({expr}))"
            return f"acc_red({expr})"

        def pmidx(k):
            return str(k)

        def add_prod(expr, bd, t, tty, k):
            """Acc expression for expr + t * pm[k]; t canonical of type tty."""
            n = 1 if tty == "f" else 4
            expr, bd = room(expr, bd, n)
            if tty == "f":
                return f"acc_fp({expr}, {t}, A.pm, {k})", bd + PROD
            return f"acc_ext({expr}, {t}, A.pm, A.pmn, {k})", bd + 4 * PROD

        # Each term is added to the running sum right after its last root is computed,
        # so term values do not stay live to the end of the kernel.
        acc_state = {"n": 0, "b": 0}
        kwaves = tune.get(ki, {}).get("waves", WAVES)
        kpf = tune.get(ki, {}).get("pf", PF)
        if ORDER == "dfs":
            byid_ = pg.byid
            leaves = set(v for v in need if v in loaded or byid_[v][0] in "clge")
            oroots = sorted(set(roots), key=lambda v: pg.order[v])
            body = [v for v in dfs_order(pg, need, oroots, leaves) if v not in leaves]
            first_use = {}
            for n_, v in enumerate(body):
                for d in deps(byid_[v]):
                    if d in leaves and d not in first_use:
                        first_use[d] = n_
            consts = [v for v in leaves if byid_[v][0] in "ceg"]
            slots = {}
            for v in leaves:
                if byid_[v][0] in "ceg":
                    continue
                slots.setdefault(max(0, first_use.get(v, 0) - kpf), []).append(v)
            seq = sorted(consts, key=lambda v: pg.order[v])
            for n_, v in enumerate(body):
                seq += sorted(slots.get(n_, []), key=lambda v: pg.order[v])
                seq.append(v)
            kprog = [byid_[v] for v in seq]
        else:
            kprog = [ins_ for ins_ in prog if ins_[0] != "r"]
        order_pos = {}
        for n_, ins_ in enumerate(kprog):
            order_pos[ins_[1]] = n_
        term_at = {}
        for ti, (e, f) in enumerate(mine):
            rts = [x for x in term_roots((e, f)) if x not in remat and pg.byid[x][0] not in "ceg"]
            term_at.setdefault(max([order_pos[x] for x in rts] + [-1]), []).append(ti)
        done_terms = set()

        def pending_terms():
            return [ti for pos in sorted(term_at) for ti in term_at[pos] if ti not in done_terms]

        def emit_term(ti):
            done_terms.add(ti)
            e, f = mine[ti]
            sn, sb = acc_state["n"], acc_state["b"]
            vals = [x[1] for x in f if x[0] == "v"]
            pms = tuple(sorted(x[1] for x in f if x[0] == "pm"))
            if not vals and not pms:
                src, bd = acc_src(e)
                cur, sb2 = f"s{sn}", sb
                if sb2 + bd >= LIM:
                    cur, sb2 = f"acc_fold({cur})", fold_bound(sb2)
                if sb2 + bd >= LIM:
                    src, bd = f"acc_fold({src})", fold_bound(bd)
                w(f"  const Acc s{sn + 1} = acc_add({cur}, {src});")
                acc_state["n"], acc_state["b"] = sn + 1, sb2 + bd
                return
            expr = ref(e)
            ety = types[e]
            for v in vals:
                expr = f"emul({expr}, {ref(v)})"
                if types[v] == "e":
                    ety = "e"
            if not pms:
                cur, sb2 = room(f"s{sn}", sb, 1)
                w(f"  const Acc s{sn + 1} = acc_add({cur}, acc_of({expr}));")
                acc_state["n"], acc_state["b"] = sn + 1, sb2 + CANON
                return
            if len(pms) == 1:
                k = pms[0]
            else:
                if pms not in combo_index:
                    combo_index[pms] = len(combo_index)
                k = f"NPM + {combo_index[pms]}"
            e2, sb = add_prod(f"s{sn}", sb, expr, ety, k)
            w(f"  const Acc s{sn + 1} = {e2};")
            acc_state["n"], acc_state["b"] = sn + 1, sb

        w(f"// GENERATED by tools/gen_eval_check.py from risc0_amd/circuits/{circuit}.poly.ir — do not edit.")
        w(common_text)
        lb = "256" if kwaves <= 1 else f"256, {kwaves}"
        w(f"__global__ __launch_bounds__({lb}) void k{ki}(Args A) {{")
        w("  const uint32_t cycle = A.base + blockIdx.x * 256u + threadIdx.x;")
        w("  if (cycle >= A.base + A.count) return;")
        w("  const uint32_t mask = A.domain - 1;")
        if mine or last:
            w("  const Acc s0 = Acc{{0, 0, 0, 0}};")
        for ins in kprog:
            op, i = ins[0], ins[1]
            if i not in need or op == "r" or i in remat:
                continue
            if i in loaded:
                kind, s_ = slot[i]
                if kind == "f":
                    w(f"  const uint32_t v{i} = A.mf[uint64_t({s_}u) * A.domain + cycle];")
                else:
                    w(f"  FpExt v{i}; {{ uint4 t = reinterpret_cast<const uint4*>(A.me)[uint64_t({s_}u) * A.domain + cycle];"
                      f" v{i} = FpExt{{{{t.x, t.y, t.z, t.w}}}}; }}")
                continue
            if op == "l":
                w(f"  const uint32_t v{i} = A.a[{ins[2]}][{ins[3]}u * A.domain + ((cycle - {4 * ins[4]}u) & mask)];")
                continue
            if op == "c":
                w(f"  const uint32_t v{i} = {enc(ins[2])}u;")
            elif op == "e":
                w(f"  const FpExt v{i} = FpExt{{{{{', '.join(str(enc(x)) + 'u' for x in ins[2:6])}}}}};")
            elif op == "g":
                w(f"  const uint32_t v{i} = A.a[{ins[2]}][{ins[3]}];")
            elif op in "ab":
                src, bd = acc_src(ins[2])
                if op == "a":
                    t, tty, k = ref(ins[3]), types[ins[3]], ins[4]
                else:
                    T, U, k = ins[3], ins[4], ins[5]
                    t = f"emul({ref(T)}, {ref(U)})"
                    tty = "e" if "e" in (types[T], types[U]) else "f"
                expr, bd = add_prod(src, bd, t, tty, k)
                w(f"  const Acc a{i} = {expr};")
                bound[i] = bd
                if i in canon:
                    w(f"  const FpExt v{i} = {reduced(f'a{i}', bd)};")
            else:
                a, b = ins[2], ins[3]
                ra, rb = ref(a), ref(b)
                if types[a] == "f" and types[b] == "f":
                    fn = {"+": "fp_add", "-": "fp_sub", "*": "fp_mul"}[op]
                    w(f"  const uint32_t v{i} = {fn}({ra}, {rb});")
                else:
                    fn = {"+": "eadd", "-": "esub", "*": "emul"}[op]
                    w(f"  const FpExt v{i} = {fn}({ra}, {rb});")
            if i in produced:
                kind, s_ = slot[i]
                if kind == "f":
                    w(f"  A.mf[uint64_t({s_}u) * A.domain + cycle] = v{i};")
                else:
                    w(f"  reinterpret_cast<uint4*>(A.me)[uint64_t({s_}u) * A.domain + cycle] ="
                      f" make_uint4(v{i}.c[0], v{i}.c[1], v{i}.c[2], v{i}.c[3]);")
            for ti in term_at.get(order_pos[i], []):
                emit_term(ti)
            if op not in "ceg":
                tick()
        if mine or last:
            # previous kernels' sum (if any) joins at the end; terms were added as they completed
            w("  uint4* accp = reinterpret_cast<uint4*>(A.acc) + cycle;")
            for ti in pending_terms():
                emit_term(ti)
            sn, sb = acc_state["n"], acc_state["b"]
            if not first:
                w(f"  Acc s{sn + 1}; {{ uint4 p = *accp; s{sn + 1} = acc_of(FpExt{{{{p.x, p.y, p.z, p.w}}}}); }}")
                cur, sb2 = room(f"s{sn}", sb, 1)
                w(f"  const Acc s{sn + 2} = acc_add({cur}, s{sn + 1});")
                sn, sb = sn + 2, sb2 + CANON
            w(f"  FpExt s = {reduced(f's{sn}', sb)};")
            if last:
                w("  s = fe_mul_fp(s, A.vinv[cycle & 3]);")
                w("  #pragma unroll")
                w("  for (int k = 0; k < 4; k++) A.check[uint64_t(k) * A.domain + cycle] = s.c[k];")
            else:
                w("  *accp = make_uint4(s.c[0], s.c[1], s.c[2], s.c[3]);")
        if first and not mine and not last:
            # keep the accumulator defined for later kernels
            w("  reinterpret_cast<uint4*>(A.acc)[cycle] = make_uint4(0u, 0u, 0u, 0u);")
        w("}")
        w(f"void launch_k{ki}(hipStream_t s, const Args& A) {{")
        w(f"  hipLaunchKernelGGL(k{ki}, dim3(div_up(A.count, 256)), dim3(256), 0, s, A);")
        w("  HIP_OK(hipGetLastError());")
        w("}")
        w(f"}}  // namespace ec_{circuit}")
        w("}  // namespace r0")
        with open(os.path.join(outdir, f"eval_check_{circuit}_k{ki}.hip"), "w") as f:
            f.write("\n".join(L) + "\n")
        stats.append(pg.cone_cost(roots))
    # accumulator initialisation: kernels after the first add into acc; if the first
    # kernel has no terms it zeroes it (above).
    flat = []
    for pms, j in sorted(combo_index.items(), key=lambda kv: kv[1]):
        flat += [len(pms)] + list(pms)
    L = []
    w = L.append
    w(f"// GENERATED by tools/gen_eval_check.py — {circuit}: {len(prog)} IR ops, {len(terms)} terms,")
    w(f"// {len(kernels)} kernels, {nf} Fp + {ne} FpExt materialised values per point.")
    w(common_text)
    for ki in range(len(kernels)):
        w(f"void launch_k{ki}(hipStream_t s, const Args& A);")
    w(f"const int kPmCombos[] = {{{', '.join(str(x) for x in flat) or '0'}}};")
    w(f"}}  // namespace ec_{circuit}")
    w(f"void eval_check_{circuit}_info(EvalCheckInfo* info) {{")
    w(f"  info->combos = ec_{circuit}::kPmCombos; info->ncombos = {len(combo_index)}; info->npm = ec_{circuit}::NPM;")
    w(f"  info->nargs = {nargs}; info->mat_fp = {nf}; info->mat_ext = {ne}; info->kernels = {len(kernels)};")
    w(f"  info->modmuls_per_point = {modmuls(pg) + 4};")
    w("}")
    w(f"void eval_check_{circuit}(hipStream_t s, const EvalCheckArgs& e) {{")
    w(f"  using namespace ec_{circuit};")
    w(f"  R0_REQUIRE(e.nargs == {nargs}, \"eval_check_{circuit}: wrong argument count\");")
    w("  Args A;")
    w(f"  for (int i = 0; i < {nargs}; i++) A.a[i] = e.args[i];")
    w("  A.pm = e.poly_mix; A.pmn = e.poly_mix_nb; A.acc = e.acc; A.check = e.check; A.vinv = e.vinv; A.domain = e.domain;")
    w("  A.mf = e.mat_fp; A.me = e.mat_ext;")
    w("  // tiles of e.tile points run every kernel before the next tile, so a tile's")
    w("  // trace columns are re-read from the Infinity Cache rather than HBM")
    w("  const uint32_t tile = e.tile ? e.tile : e.domain;")
    w("  for (uint32_t b = 0; b < e.domain; b += tile) {")
    w("    A.base = b;")
    w("    A.count = e.domain - b < tile ? e.domain - b : tile;")
    for ki in range(len(kernels)):
        w(f"    launch_k{ki}(s, A);")
    w("  }")
    w("}")
    w("}  // namespace r0")
    with open(os.path.join(outdir, f"eval_check_{circuit}.hip"), "w") as f:
        f.write("\n".join(L) + "\n")
    tot = sum(stats)
    base = pg.cone_cost([pg.res])
    print(f"{circuit}: {len(terms)} terms, {len(kernels)} kernels, mat {nf} Fp + {ne} FpExt, "
          f"work {tot} vs {base} ({tot / base:.2f}x), per-kernel cost {stats}")


if __name__ == "__main__":
    emit(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 4000)
