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
Products of several poly_mix powers are folded into host-computed constants, and values
that depend only on constants, mix and global words are evaluated once on the host
(Program.hoist_uniform). Per kernel (tuning file): sums of products as 64-bit sums with one
REDC per sum ("fuse"), and tap addressing by column base pointers ("wide").

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
        self.uprog, self.uslot = [], {}

    def hoist_uniform(self, terms):
        """Lane-independent values — cones of constants and `g` loads only (mix and global
        words, the same for every point) — that a point's arithmetic reads are evaluated once
        on the host (eval_check_<circuit>_uniform) and read by the kernels from a table
        (A.uv, scalar loads); every kernel that needed one recomputed its cone per lane.
        Applied after scheduling, so kernel packing (and its tuning) is unchanged."""
        uni = {}
        for ins in self.prog:
            op = ins[0]
            if op == "r":
                continue
            if op in "ceg":
                uni[ins[1]] = True
            elif op == "l":
                uni[ins[1]] = False
            else:
                uni[ins[1]] = all(uni[d] for d in deps(ins))
        need = set()
        for ins in self.prog:
            if ins[0] in "+-*ab" and not uni[ins[1]]:
                need.update(d for d in deps(ins) if uni[d])
        for t in terms:
            need.update(v for v in term_roots(t) if uni[v])
        need.update(v for v in self.mat if uni[v])  # a stored value that is the same everywhere
        hoist = sorted((v for v in need if self.byid[v][0] in "+-*ab"), key=self.order.get)
        self.mat -= set(hoist)
        cone, stack = set(), list(hoist)
        while stack:
            v = stack.pop()
            if v not in cone:
                cone.add(v)
                stack.extend(deps(self.byid[v]))
        self.uprog = [self.byid[v] for v in sorted(cone, key=self.order.get)]
        self.uslot = {v: n for n, v in enumerate(hoist)}
        for v in hoist:
            self.byid[v] = ("u", v, self.uslot[v])

    def cost(self, v):
        ins = self.byid[v]
        op = ins[0]
        ty = self.types
        if op in "clgeu":
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
                if v in roots or v in pg.mat or byid[v][0] in "clgeu":
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


# emission order: "ir" (the reference program's order) or "dfs" (each value computed
# right before its first use, accumulation chains first; loads hoisted EC_PF ops ahead)
ORDER = os.environ.get("EC_ORDER", "dfs")
PF = int(os.environ.get("EC_PF", "512"))
# minimum waves per SIMD requested from the register allocator (1 = no limit)
WAVES = int(os.environ.get("EC_WAVES", "2"))
# Variants measured on MI355X (per-kernel rocprofv3 sums, rv32im po2=20, tools/rehearsal/ec_variants.sh):
#   canonical results (default)                  28.6-28.8 ms
#   EC_CANON=0 lazy range analysis               34.3-34.8 ms: 2-11% fewer VALU instructions,
#                                                but more live registers -> spills in 6 kernels
#   EC_SADDR=1 saddr tap loads                   28.9-30.0 ms: -1.1k VALU per big kernel, no gain
#   EC_SPLIT=2 / 3 split accumulation chains     30.6 / 32.7 ms (register pressure)
#   poly_mix powers staged in LDS per kernel (instead of scalar loads, which the compiler
#   hoists and spills to VGPR lanes: ~640 v_writelane/v_readlane in k13)   not adopted:
#   plain, volatile and sched_barrier-fenced LDS reads all compiled k13 to 256 VGPRs +
#   256 AGPRs (1 wave/SIMD, AGPR spills) against 227 VGPRs at 2 waves with SGPR operands
#   xmul as a polynomial product (c_0..c_6, then NBETA * REDC(c_4..c_6) added back: 38
#   VALU against 43, no NBETA * b Montgomery products)   not adopted: 26.46 -> 27.29 ms;
#   k16 -0.1 ms but k27 +0.68 ms (256 VGPRs + AGPRs, one wave per SIMD) because LLVM no
#   longer shares NBETA * b between products with a common operand; a hybrid keeping the
#   shared form for operands of several products still took k23/k27 to 256 VGPRs
# The kernels are bound by register pressure and issue stalls (SQ_WAIT_INST_ANY 30-55% of
# wave cycles), not by the count of VALU instructions.
# EC_CANON=1: every Fp/FpExt result canonical; EC_CANON=0: the lazy range analysis below
CANON_ALL = os.environ.get("EC_CANON", "1") == "1"
# EC_CANON_FORCE=0/1 overrides the tuned per-kernel mode (tools/tune_ec_canon.py variants)
if "EC_CANON_FORCE" in os.environ:
    CANON_ALL = os.environ["EC_CANON_FORCE"] == "1"
# EC_SADDR=0: taps addressed as A.a[arg][col * domain + row] (64-bit VALU address per load);
# EC_SADDR=1: scalar column base (A.cp) + one 32-bit lane offset per `back`
SADDR = os.environ.get("EC_SADDR", "0") == "1"
# EC_SPLIT=n: each accumulation chain (ACC + T*pm[k], ...) runs as n interleaved partial
# sums, joined where the value is used, so consecutive products do not wait on each
# other's v_mad_u64_u32 results
SPLIT = int(os.environ.get("EC_SPLIT", "1"))
# EC_PIN=1: each poly_mix read goes through pin(), an empty asm that makes the table
# pointer depend on the running sum it is added to, so the scalar load of pm[k] cannot be
# hoisted ahead of that sum (hoisted loads were spilled from SGPRs to VGPR lanes)
# Measured (rv32im po2=20, sum of kernel means): pinned to the running sum itself 50.5 ms,
# 4 accumulations back 40.7 ms (volatile asm) / 45.3 ms (plain asm), against 26.9 ms for the
# hoisted-and-spilled default — the spills go away (k13: 302 -> 0) but the pinned scalar
# loads cannot be scheduled around; not adopted. Never-taken branches every 100/300
# statements (basic-block boundaries) made it worse: k13 630-666 SGPR spills, 1 wave/SIMD.
PIN = os.environ.get("EC_PIN", "0") == "1"
# EC_PMV=1 (or a kernel's "pmv" in the tuning file): the poly_mix power of each Fp
# accumulation (ACC + T*pm[k]) is a uint4 vector load with a uniform address, issued EC_PMD
# program positions before its use. Vector loads complete in order (vmcnt), so unlike the
# scalar loads (out of order: any use waits for all of them, and the compiler hoists and
# spills them to VGPR lanes) they can run ahead a fixed distance; the four words sit in
# VGPRs and feed the v_mad_u64_u32 directly.
# Measured (rv32im po2=20, tools/tune_ec_pmv.py, gpurun_out r3f): the lane spills go but
# every kernel gets 1.1-9x slower at distances 16/32/64 — a broadcast vector load still
# returns 16 B to each of the 64 lanes through the texture data path, ~360 per wave; not
# adopted.
PMV = os.environ.get("EC_PMV", "0") == "1"
# EC_FUSE=1 (or a kernel's "fuse" in the tuning file): sums of products are accumulated in
# 64 bits (one v_mad_u64_u32 per product, one REDC per sum) instead of a REDC per product
# and a reduction per addition; EC_FUSE_FORCE=0/1 overrides the tuning file
FUSE = os.environ.get("EC_FUSE", "0") == "1"
# EC_HOIST=0: every kernel computes the lane-independent values it reads itself (no host table)
HOIST = os.environ.get("EC_HOIST", "1") == "1"
PMD = int(os.environ.get("EC_PMD", "64"))
# EC_PINB=n (or a kernel's "pinb"): the poly_mix terms (acc_fp, acc_ext) go in batches of n;
# batch b's table pointer is pinned to the running sum after the first term of batch b-1,
# so batch b's scalar loads are issued once batch b-1's have landed and overlap the rest of
# batch b-1. Scalar loads return out of order (any use waits for all in flight), so a load
# per term pinned a few terms back (EC_PIN) made every term wait on the loads of the next
# ones; batches wait once per batch, on their own loads only, with ~8n SGPRs live.
PINB = int(os.environ.get("EC_PINB", "0"))
# ... pinned to the running sum EC_PIND accumulations back, so the load has that long to land
PIND = int(os.environ.get("EC_PIND", "4"))


def kernel_config(circuit, budget):
    """Per-kernel (waves, prefetch) chosen by tools/tune_eval_check.py on an MI355X and
    committed as risc0_amd/circuits/<circuit>.ectune.json; EC_WAVES/EC_PF (if set) or
    the defaults apply to kernels it does not list (or when EC_NOTUNE is set)."""
    path = os.path.join(ROOT, "risc0_amd", "circuits", circuit + ".ectune.json")
    keep = os.environ.get("EC_KEEPTUNE") == "1"  # EC_WAVES/EC_PF override only those two fields
    if (os.environ.get("EC_NOTUNE") or (not keep and ("EC_WAVES" in os.environ or "EC_PF" in os.environ))
            or not os.path.exists(path)):
        return {}
    import json
    with open(path) as f:
        t = json.load(f)
    if t.get("budget") != budget or t.get("order") != ORDER:
        return {}
    ks = {int(k): dict(v) for k, v in t["kernels"].items()}
    if keep:
        for v in ks.values():
            if "EC_WAVES" in os.environ:
                v["waves"] = int(os.environ["EC_WAVES"])
            if "EC_PF" in os.environ:
                v["pf"] = int(os.environ["EC_PF"])
    return ks


# ---- value-range analysis --------------------------------------------------------
# Every Fp word (and every limb of an FpExt) is kept as a 32-bit integer congruent to
# its Montgomery word mod p, below a bound M (inclusive maximum) that the generator
# knows exactly. Reductions are emitted only where an operation could overflow:
#   x + y                     M = Mx + My                      (< 2^32)
#   x - y = x + (k p - y)     M = Mx + k p,  k p >= My
#   lmul(x, y) (REDC, no min) M = (Mx My + (2^32 - 1) p) >> 32  (Mx My + (2^32-1) p < 2^64)
#   lred(x) = min(x, x - p)   M = max(p - 1, Mx - p)
# FpExt products form four 4-term sums in 64 bits (< 2^64), fold hi*(2^32 mod p)+lo and
# REDC. Anything that leaves the kernel (the accumulator, check, materialised values) is
# canonical, so outputs are the reference's words exactly.
U32 = 2**32 - 1
U64 = 2**64 - 1
FOLDC = 2**32 % P
NBW = (P - 11) * 2**32 % P  # kNBeta, Montgomery word of NBETA = -11 (x^4 = NBETA)


def redc_max(t):
    assert t + U32 * P <= U64
    return (t + U32 * P) >> 32


def fold_max(x):
    return (x >> 32) * FOLDC + U32


def mul_ok(ma, mb):
    t = ma * mb
    return t + U32 * P <= U64 and redc_max(t) <= U32


def emul_ok(ma, mb):
    # four products per limb, b's upper limbs enter as canonical NBETA*b
    return 4 * ma * max(mb, P - 1) <= U64


def mat_config(circuit, budget):
    """Sub-expressions materialised to HBM across kernels (tools/pick_ec_mat.py, committed in
    <circuit>.ectune.json as "mat"), so kernels read them instead of recomputing their cones.
    Applies whatever EC_WAVES/EC_PF say, since tuning variants must share the partition;
    EC_NOMAT=1 disables it."""
    path = os.path.join(ROOT, "risc0_amd", "circuits", circuit + ".ectune.json")
    if os.environ.get("EC_NOMAT") == "1" or not os.path.exists(path):
        return []
    import json
    with open(path) as f:
        t = json.load(f)
    if t.get("budget") != budget:
        return []
    return [int(v) for v in t.get("mat", [])]


def resplit_config(circuit, budget):
    """Kernels re-packed at a smaller cost budget after the schedule: {kernel: budget} from
    EC_RESPLIT ("5:2000,9:2500") or the tuning file's "resplit", with per-piece tuning
    overrides ("resplit_tune": {"5.1": {"waves": 3}}). A re-split kernel's pieces keep its
    tuning unless overridden; they carry fewer live values per lane, so they can run more waves
    per SIMD (the kernels whose issue stalls follow their register budget)."""
    spec = os.environ.get("EC_RESPLIT")
    over = {}
    if spec is None:
        path = os.path.join(ROOT, "risc0_amd", "circuits", circuit + ".ectune.json")
        if not os.path.exists(path):
            return {}, {}
        import json
        with open(path) as f:
            t = json.load(f)
        if t.get("budget") != budget:
            return {}, {}
        return {int(k): int(v) for k, v in t.get("resplit", {}).items()}, t.get("resplit_tune", {})
    out = {}
    for part in filter(None, spec.split(",")):
        k, b = part.split(":")
        out[int(k)] = int(b)
    for part in filter(None, os.environ.get("EC_RESPLIT_WAVES", "").split(",")):
        k, w = part.split(":")  # "5.1:3"
        over[k] = {"waves": int(w)}
    return out, over


def split_terms(pg, items, budget):
    """the linear split of schedule() step 1 applied again to one kernel's terms, down to
    `budget`: an accumulation term ACC + T*pm (or ACC + T*U*pm) becomes ACC's term and T's term
    with the extra factor, so each piece's cone is smaller (its pieces then recompute what
    they share)"""
    byid = pg.byid
    out = []
    for it in items:
        if it[2] != "term":
            out.append(it)
            continue
        pieces = [it[3]]
        while True:
            best, bestc = None, -1
            for i, t in enumerate(pieces):
                if byid[t[0]][0] in "ab":
                    c = pg.cone_cost(term_roots(t))
                    if c > bestc:
                        best, bestc = i, c
            if best is None or bestc <= budget:
                break
            e, f = pieces[best]
            ins = byid[e]
            if ins[0] == "a":
                new = [(ins[2], f), (ins[3], f + [("pm", ins[4])])]
            else:
                T, U = ins[3], ins[4]
                if byid[U][0] in "ab" and byid[T][0] not in "ab":
                    T, U = U, T
                new = [(ins[2], f), (T, f + [("v", U), ("pm", ins[5])])]
            pieces[best:best + 1] = new
        out += [(it[0], it[1], "term", t) for t in pieces]
    return out


def repack(pg, items, budget):
    """one kernel's items split (split_terms) and packed again under `budget`, first fit in
    decreasing cone cost: the items of one kernel are independent of each other (what they
    read was materialised by earlier kernels), so any grouping keeps the schedule valid"""
    items = split_terms(pg, items, budget)
    roots = lambda it: [it[3]] if it[2] == "mat" else term_roots(it[3])
    items.sort(key=lambda it: -pg.cone_cost(roots(it)))
    bins = []  # [items, roots]
    for it in items:
        r = roots(it)
        for b in bins:
            if pg.cone_cost(b[1] + r) <= budget:
                b[0].append(it)
                b[1] += r
                break
        else:
            bins.append([[it], list(r)])
    return [sorted(b[0], key=lambda it: (it[0], it[1])) for b in bins]


def uniform_fn(pg):
    """Host evaluation of the hoisted lane-independent values (Program.hoist_uniform), in
    program order with canonical host arithmetic (bb31.h); g[ARG] are host copies of the
    uniform arguments (mix, global), pm the poly_mix powers (FpExt AoS)."""
    ty = pg.types
    L = ["// lane-independent values (cones of constants, mix and global words), evaluated once",
         "// per eval_check on the host; slot s holds 4 words (an Fp value in word 0)",
         f"constexpr int NUV = {len(pg.uslot)};",
         "void uniform(const uint32_t* const* g, const uint32_t* pmw, uint32_t* out) {",
         "  const FpExt* pm = reinterpret_cast<const FpExt*>(pmw);",
         "  (void)g; (void)pm; (void)out;"]

    def x(v):
        return f"u{v}" if ty[v] == "e" else f"fe_from_fp(u{v})"

    for ins in pg.uprog:
        op, i = ins[0], ins[1]
        if op == "c":
            L.append(f"  const uint32_t u{i} = {enc(ins[2])}u;")
        elif op == "e":
            L.append(f"  const FpExt u{i} = FpExt{{{{{', '.join(str(enc(v)) + 'u' for v in ins[2:6])}}}}};")
        elif op == "g":
            L.append(f"  const uint32_t u{i} = g[{ins[2]}][{ins[3]}];")
        elif op in "+-*":
            a, b = ins[2], ins[3]
            if ty[i] == "f":
                fn = {"+": "fp_add", "-": "fp_sub", "*": "fp_mul"}[op]
                L.append(f"  const uint32_t u{i} = {fn}(u{a}, u{b});")
            else:
                fn = {"+": "fe_add", "-": "fe_sub", "*": "fe_mul"}[op]
                L.append(f"  const FpExt u{i} = {fn}({x(a)}, {x(b)});")
        elif op == "a":
            L.append(f"  const FpExt u{i} = fe_add(u{ins[2]}, fe_mul({x(ins[3])}, pm[{ins[4]}]));")
        elif op == "b":
            L.append(f"  const FpExt u{i} = fe_add(u{ins[2]}, fe_mul(fe_mul({x(ins[3])}, {x(ins[4])}), pm[{ins[5]}]));")
        else:
            raise RuntimeError(f"unexpected op {op} in a lane-independent cone")
    for v, n in sorted(pg.uslot.items(), key=lambda kv: kv[1]):
        if ty[v] == "f":
            L.append(f"  out[{4 * n}] = u{v}; out[{4 * n + 1}] = out[{4 * n + 2}] = out[{4 * n + 3}] = 0;")
        else:
            L.append(f"  for (int k = 0; k < 4; k++) out[{4 * n} + k] = u{v}.c[k];")
    L.append("}")
    return L


def emit(circuit, outdir, budget, host=False):
    pg = Program(circuit)
    pg.mat = set(mat_config(circuit, budget))
    terms, kernels = schedule(pg, budget)
    if HOIST:
        pg.hoist_uniform(terms)
    # uses of each value over the whole program (after hoisting); term roots and materialised
    # values count twice, so a fused sum never swallows a value something else reads
    nuse, consumer = {}, {}
    for ins in pg.byid.values():
        for d in deps(ins):
            nuse[d] = nuse.get(d, 0) + 1
            consumer[d] = ins[1]
    for t in terms:
        for r in term_roots(t):
            nuse[r] = nuse.get(r, 0) + 2
    for v in pg.mat:
        nuse[v] = nuse.get(v, 0) + 2
    tune0 = kernel_config(circuit, budget)
    resplit, piece_tune = resplit_config(circuit, budget)
    tune = {}
    split_kernels = []
    for k, items in enumerate(kernels):
        pieces = repack(pg, items, resplit[k]) if k in resplit else [items]
        for j, piece in enumerate(pieces):
            t = dict(tune0.get(k, {}))
            if len(pieces) > 1:
                t.update(piece_tune.get(f"{k}.{j}", {}))
            tune[len(split_kernels)] = t
            split_kernels.append(piece)
    kernels = split_kernels
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
    # trace columns read by the program: the host passes one base pointer per column
    # (A.cp), so a tap is a global load with a scalar base and a shared 32-bit lane
    # offset per `back` (no per-load 64-bit address arithmetic on the VALU)
    colslot = {}
    for ins in prog:
        if ins[0] == "l" and (ins[2], ins[3]) not in colslot:
            colslot[(ins[2], ins[3])] = len(colslot)
    if outdir:
        os.makedirs(outdir, exist_ok=True)

    common = [
        '#include "bb31.h"',
        "#if defined(R0_EC_HOST)",
        "#define EC_FN static inline",
        "#else",
        '#include "evalcheck.h"',
        "#define EC_FN __device__ __forceinline__",
        "#endif",
        "namespace r0 {",
        f"namespace ec_{circuit} {{",
        "struct Args {",
        f"  const uint32_t* a[{nargs}];",
        "  const uint32_t* const* cp;  // column base pointers (kColArg/kColIdx order)",
        "  const uint32_t* pm;   // poly_mix powers then folded products, FpExt AoS",
        "  const uint32_t* pmn;  // the same times NBETA",
        "  uint32_t* acc;        // FpExt AoS accumulator per point",
        "  uint32_t* check;      // 4 SoA planes",
        "  const uint32_t* vinv; // inv((3x)^N - 1) for cycle & 3",
        "  uint32_t* mf;         // materialised Fp values, [slot][domain]",
        "  uint32_t* me;         // materialised FpExt values, [slot][domain] AoS",
        "  uint32_t domain;",
        "  uint32_t base, count;  // this launch covers points [base, base + count)",
        "  uint64_t wide;         // bit k: kernel k takes its taps from the column bases (A.cp)",
        "  const uint32_t* uv;    // lane-independent values evaluated on the host, 4 words each",
        "};",
        f"constexpr int NPM = {npm};",
        "// one more than the largest tapped column index of any argument: 32-bit tap indices",
        "// are exact while kTapCols * domain <= 2^32",
        f"constexpr uint32_t kTapCols = {max(c for _, c in colslot) + 1 if colslot else 1}u;",
        "// lazy Fp/FpExt words: congruent mod p, below a generator-tracked bound (see",
        "// tools/gen_eval_check.py); lred/xred take one p off values >= p",
        "EC_FN uint32_t lmul(uint32_t a, uint32_t b) {",
        "  const uint64_t t = uint64_t(a) * b;",
        "  const uint32_t m = uint32_t(t) * kNegPinv;",
        "  return uint32_t((t + uint64_t(m) * kP) >> 32);",
        "}",
        "// tap load: scalar column base + 32-bit byte offset (saddr-form global load)",
        "EC_FN uint32_t ldc(const uint32_t* p, uint32_t off) {",
        "  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(p) + off);",
        "}",
        "// trace tap: W = false indexes in 32 bits (col * domain + row < 2^32 words); W = true",
        "// (columns x domain >= 2^32) takes the column's base from the host table A.cp (one",
        "// scalar load) plus a 32-bit byte offset, instead of a 64-bit col * domain per tap",
        "template <bool W> EC_FN uint32_t tap(const uint32_t* a, const uint32_t* const* cp, uint32_t slot, uint32_t col,",
        "                                     uint32_t domain, uint32_t row) {",
        "  if constexpr (W) return ldc(cp[slot], row * 4u);",
        "  else return a[col * domain + row];",
        "}",
        "EC_FN uint32_t lred(uint32_t x) { return umin(x, x - kP); }",
        "EC_FN uint32_t lsub(uint32_t a, uint32_t b, uint32_t kp) { return a + (kp - b); }",
        "EC_FN FpExt xred(FpExt a) { return FpExt{{lred(a.c[0]), lred(a.c[1]), lred(a.c[2]), lred(a.c[3])}}; }",
        "EC_FN FpExt xadd(FpExt a, FpExt b) { return FpExt{{a.c[0] + b.c[0], a.c[1] + b.c[1], a.c[2] + b.c[2], a.c[3] + b.c[3]}}; }",
        "EC_FN FpExt xaddf(FpExt a, uint32_t b) { a.c[0] += b; return a; }",
        "EC_FN FpExt xsub(FpExt a, FpExt b, uint32_t kp) {",
        "  return FpExt{{lsub(a.c[0], b.c[0], kp), lsub(a.c[1], b.c[1], kp), lsub(a.c[2], b.c[2], kp), lsub(a.c[3], b.c[3], kp)}};",
        "}",
        "EC_FN FpExt xsubf(FpExt a, uint32_t b, uint32_t kp) { a.c[0] = lsub(a.c[0], b, kp); return a; }",
        "EC_FN FpExt fsubx(uint32_t a, FpExt b, uint32_t kp) {",
        "  return FpExt{{lsub(a, b.c[0], kp), kp - b.c[1], kp - b.c[2], kp - b.c[3]}};",
        "}",
        "EC_FN FpExt xmulf(FpExt a, uint32_t b) { return FpExt{{lmul(a.c[0], b), lmul(a.c[1], b), lmul(a.c[2], b), lmul(a.c[3], b)}}; }",
        "// a * x (the extension generator, FpExt(0, 1, 0, 0)): a limb shift, x^4 = NBETA",
        "EC_FN FpExt xmulx(FpExt a) { return FpExt{{lmul(a.c[3], kNBeta), a.c[0], a.c[1], a.c[2]}}; }",
        "// extension product; b's upper limbs times NBETA are canonical; four 4-term sums,",
        "// folded and REDC'd without the final min",
        "EC_FN FpExt xmul(FpExt a, FpExt b) {",
        "  const uint32_t n1 = fp_mul(kNBeta, b.c[1]), n2 = fp_mul(kNBeta, b.c[2]), n3 = fp_mul(kNBeta, b.c[3]);",
        "  const uint64_t a0 = a.c[0], a1 = a.c[1], a2 = a.c[2], a3 = a.c[3];",
        "  const uint64_t s0 = a0 * b.c[0] + a1 * n3 + a2 * n2 + a3 * n1;",
        "  const uint64_t s1 = a0 * b.c[1] + a1 * b.c[0] + a2 * n3 + a3 * n2;",
        "  const uint64_t s2 = a0 * b.c[2] + a1 * b.c[1] + a2 * b.c[0] + a3 * n3;",
        "  const uint64_t s3 = a0 * b.c[3] + a1 * b.c[2] + a2 * b.c[1] + a3 * b.c[0];",
        "  auto r = [](uint64_t t) { t = fold64(t); const uint32_t m = uint32_t(t) * kNegPinv;",
        "                            return uint32_t((t + uint64_t(m) * kP) >> 32); };",
        "  return FpExt{{r(s0), r(s1), r(s2), r(s3)}};",
        "}",
        "// Lazy FpExt accumulator: four unreduced 64-bit sums of Montgomery products;",
        "// the generator tracks an upper bound and folds (hi * (2^32 mod p) + lo) before a",
        "// sum could reach 2^64.",
        "struct Acc { uint64_t c[4]; };",
        "// a value v enters as v * 2^32 (mod p), so the final REDC returns v",
        "EC_FN Acc acc_of(FpExt a) {",
        "  return Acc{{uint64_t(a.c[0]) * kFoldC, uint64_t(a.c[1]) * kFoldC, uint64_t(a.c[2]) * kFoldC,",
        "              uint64_t(a.c[3]) * kFoldC}};",
        "}",
        "EC_FN Acc acc_of(uint32_t a) { return Acc{{uint64_t(a) * kFoldC, 0, 0, 0}}; }",
        "EC_FN Acc acc_fold(Acc a) {",
        "#pragma unroll",
        "  for (int i = 0; i < 4; i++) a.c[i] = fold64(a.c[i]);",
        "  return a;",
        "}",
        "EC_FN FpExt acc_red(Acc a) {",
        "  return FpExt{{mont_reduce(a.c[0]), mont_reduce(a.c[1]), mont_reduce(a.c[2]), mont_reduce(a.c[3])}};",
        "}",
        "EC_FN uint32_t redc_lazy(uint64_t t) { const uint32_t m = uint32_t(t) * kNegPinv; return uint32_t((t + uint64_t(m) * kP) >> 32); }",
        "EC_FN FpExt acc_lred(Acc a) { return FpExt{{redc_lazy(a.c[0]), redc_lazy(a.c[1]), redc_lazy(a.c[2]), redc_lazy(a.c[3])}}; }",
        "EC_FN Acc acc_add(Acc a, Acc b) {",
        "#pragma unroll",
        "  for (int i = 0; i < 4; i++) a.c[i] += b.c[i];",
        "  return a;",
        "}",
        "// 64-bit sums of products (EC_FUSE): a term x enters as x * 2^32 (x * kFoldC), a product",
        "// a * b as itself, so one REDC of the sum gives the Montgomery word of the sum",
        "EC_FN Acc acc_mf(Acc s, FpExt a, uint32_t b) {",
        "#pragma unroll",
        "  for (int i = 0; i < 4; i++) s.c[i] += uint64_t(a.c[i]) * b;",
        "  return s;",
        "}",
        "EC_FN Acc acc_m0(Acc s, uint32_t a, uint32_t b) { s.c[0] += uint64_t(a) * b; return s; }",
        "EC_FN Acc acc_me(Acc s, FpExt a, FpExt b) {",
        "  const uint32_t n1 = fp_mul(kNBeta, b.c[1]), n2 = fp_mul(kNBeta, b.c[2]), n3 = fp_mul(kNBeta, b.c[3]);",
        "  s.c[0] += uint64_t(a.c[0]) * b.c[0] + uint64_t(a.c[1]) * n3 + uint64_t(a.c[2]) * n2 + uint64_t(a.c[3]) * n1;",
        "  s.c[1] += uint64_t(a.c[0]) * b.c[1] + uint64_t(a.c[1]) * b.c[0] + uint64_t(a.c[2]) * n3 + uint64_t(a.c[3]) * n2;",
        "  s.c[2] += uint64_t(a.c[0]) * b.c[2] + uint64_t(a.c[1]) * b.c[1] + uint64_t(a.c[2]) * b.c[0] + uint64_t(a.c[3]) * n3;",
        "  s.c[3] += uint64_t(a.c[0]) * b.c[3] + uint64_t(a.c[1]) * b.c[2] + uint64_t(a.c[2]) * b.c[1] + uint64_t(a.c[3]) * b.c[0];",
        "  return s;",
        "}",
        "EC_FN Acc acc_plus(Acc s, FpExt x) {",
        "#pragma unroll",
        "  for (int i = 0; i < 4; i++) s.c[i] += uint64_t(x.c[i]) * kFoldC;",
        "  return s;",
        "}",
        "EC_FN Acc acc_plusf(Acc s, uint32_t x) { s.c[0] += uint64_t(x) * kFoldC; return s; }",
        "EC_FN Acc acc_add0(Acc s, uint64_t x) { s.c[0] += x; return s; }",
        "EC_FN Acc acc_negk(Acc s, uint64_t k) {",
        "#pragma unroll",
        "  for (int i = 0; i < 4; i++) s.c[i] = k - s.c[i];",
        "  return s;",
        "}",
        "EC_FN FpExt xneg(FpExt a, uint32_t kp) { return FpExt{{kp - a.c[0], kp - a.c[1], kp - a.c[2], kp - a.c[3]}}; }",
        "// the table pointer, made to depend on `a` (no instruction): pm[k] is loaded after `a`",
        "#ifdef R0_EC_HOST",
        "EC_FN const uint32_t* pin(const uint32_t* p, const Acc&) { return p; }",
        "#else",
        "EC_FN const uint32_t* pin(const uint32_t* p, const Acc& a) {",
        "  const uint32_t d = uint32_t(a.c[0]);",
        "  asm(\"\" : \"+s\"(p) : \"v\"(d));",
        "  return p;",
        "}",
        "#endif",
        "// a += t * pm[k]  (t in Fp)",
        "EC_FN Acc acc_fp(Acc a, uint32_t t, const uint32_t* pm, int k) {",
        "#pragma unroll",
        "  for (int i = 0; i < 4; i++) a.c[i] += uint64_t(t) * pm[4 * k + i];",
        "  return a;",
        "}",
        "// poly_mix power k as a vector load (EC_PMV): z is a zero the compiler cannot see",
        "// through, so the uniform address still takes a global load into VGPRs",
        "EC_FN uint4 pm_vec(const uint32_t* pm, uint32_t z, int k) {",
        "  return *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(pm + 4 * k) + z);",
        "}",
        "EC_FN Acc acc_fpv(Acc a, uint32_t t, uint4 q) {",
        "  a.c[0] += uint64_t(t) * q.x;",
        "  a.c[1] += uint64_t(t) * q.y;",
        "  a.c[2] += uint64_t(t) * q.z;",
        "  a.c[3] += uint64_t(t) * q.w;",
        "  return a;",
        "}",
        "// a += t * pm[k]  (t in FpExt; x^4 = NBETA folded into pmn = NBETA * pm)",
        "EC_FN Acc acc_ext(Acc a, FpExt t, const uint32_t* pm, const uint32_t* pmn, int k) {",
        "  const uint32_t* q = pm + 4 * k;",
        "  const uint32_t* n = pmn + 4 * k;",
        "  a.c[0] += uint64_t(t.c[0]) * q[0] + uint64_t(t.c[1]) * n[3] + uint64_t(t.c[2]) * n[2] + uint64_t(t.c[3]) * n[1];",
        "  a.c[1] += uint64_t(t.c[0]) * q[1] + uint64_t(t.c[1]) * q[0] + uint64_t(t.c[2]) * n[3] + uint64_t(t.c[3]) * n[2];",
        "  a.c[2] += uint64_t(t.c[0]) * q[2] + uint64_t(t.c[1]) * q[1] + uint64_t(t.c[2]) * q[0] + uint64_t(t.c[3]) * n[3];",
        "  a.c[3] += uint64_t(t.c[0]) * q[3] + uint64_t(t.c[1]) * q[2] + uint64_t(t.c[2]) * q[1] + uint64_t(t.c[3]) * q[0];",
        "  return a;",
        "}",
        "// EC_PINB: the table pointer made to depend on `a` (no instruction), then read back",
        "// uniform (readfirstlane) in the constant address space, so its reads stay scalar loads",
        "// (an asm result is otherwise taken as divergent: per-lane flat loads)",
        "#ifdef R0_EC_HOST",
        "typedef const uint32_t* cptr;",
        "EC_FN cptr pinc(const uint32_t* p, const Acc&) { return p; }",
        "#else",
        "typedef const __attribute__((address_space(4))) uint32_t* cptr;",
        "EC_FN cptr pinc(const uint32_t* p, const Acc& a) {",
        "  const uint64_t v = reinterpret_cast<uint64_t>(p);",
        "  uint32_t lo = uint32_t(v), hi = uint32_t(v >> 32);",
        "  const uint32_t d = uint32_t(a.c[0]);",
        "  asm(\"\" : \"+s\"(lo), \"+s\"(hi) : \"v\"(d));",
        "  lo = __builtin_amdgcn_readfirstlane(lo);",
        "  hi = __builtin_amdgcn_readfirstlane(hi);",
        "  return reinterpret_cast<cptr>((uint64_t(hi) << 32) | lo);",
        "}",
        "#endif",
        "EC_FN Acc acc_fpc(Acc a, uint32_t t, cptr pm, int k) {",
        "#pragma unroll",
        "  for (int i = 0; i < 4; i++) a.c[i] += uint64_t(t) * pm[4 * k + i];",
        "  return a;",
        "}",
        "EC_FN Acc acc_extc(Acc a, FpExt t, cptr q, cptr n) {",
        "  a.c[0] += uint64_t(t.c[0]) * q[0] + uint64_t(t.c[1]) * n[3] + uint64_t(t.c[2]) * n[2] + uint64_t(t.c[3]) * n[1];",
        "  a.c[1] += uint64_t(t.c[0]) * q[1] + uint64_t(t.c[1]) * q[0] + uint64_t(t.c[2]) * n[3] + uint64_t(t.c[3]) * n[2];",
        "  a.c[2] += uint64_t(t.c[0]) * q[2] + uint64_t(t.c[1]) * q[1] + uint64_t(t.c[2]) * q[0] + uint64_t(t.c[3]) * n[3];",
        "  a.c[3] += uint64_t(t.c[0]) * q[3] + uint64_t(t.c[1]) * q[2] + uint64_t(t.c[2]) * q[1] + uint64_t(t.c[3]) * q[0];",
        "  return a;",
        "}",
    ]
    common_text = "\n".join(common) + "\n"

    stats = []
    bodies = []
    PM = P - 1  # bound of a canonical word / of every pm, pmn word
    RED = P * 2**32
    CANON = PM * FOLDC  # bound of acc_of(canonical)
    one, two, mone = enc(1), enc(2), enc(P - 1)

    for ki, items in enumerate(kernels):
        # per-kernel arithmetic mode: tuned "canon" (1 canonical, 0 range analysis) or EC_CANON
        kcanon = CANON_ALL if "EC_CANON_FORCE" in os.environ else bool(tune.get(ki, {}).get("canon", CANON_ALL))
        # (a scheduled "mat" item that hoist_uniform took out of pg.mat has nothing to store)
        items = [it for it in items if it[2] != "mat" or it[3] in pg.mat]
        roots = []
        for it in items:
            roots += [it[3]] if it[2] == "mat" else term_roots(it[3])
        need = pg.cone(roots)
        produced = set(it[3] for it in items if it[2] == "mat")
        loaded = set(v for v in need if v in pg.mat and v not in produced)
        first, last = ki == 0, ki == len(kernels) - 1
        mine = [it[3] for it in items if it[2] == "term"]
        # accumulate ops computed here stay lazy (Acc a<i>); FpExt v<i> only where needed
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
        parts = {}   # lazy accumulation value -> its partial sums [(Acc name, 64-bit bound)]
        chainpos = {}
        Mv = {}      # word bounds of v<i>
        cval = {}    # Fp constants: Montgomery word
        ecval = {}   # FpExt constants: Montgomery words of the four limbs
        red_memo = {}
        offs = set()
        acc_hist = []  # Acc variables in emission order (anchors of pin())
        pm_idx = []    # acc_hist index of each poly_mix term's result (EC_PINB anchors)
        tmp = {"n": 0}
        L = []
        w = L.append

        def fresh():
            tmp["n"] += 1
            return f"t{tmp['n']}"

        # EC_FUSE: a product whose only use is an addition or subtraction is deferred (pend:
        # its two operands), and a sum whose only use is another sum stays a 64-bit Fp sum or an
        # Acc (sums: kind, variable, bound); the value is reduced to a word where it is read
        kfuse = (os.environ["EC_FUSE_FORCE"] == "1" if "EC_FUSE_FORCE" in os.environ
                 else bool(tune.get(ki, {}).get("fuse", FUSE)))
        rootset = set(roots)
        fuse_ok = set()
        if kfuse:
            for v in need:
                ins_ = pg.byid[v]
                if (ins_[0] in "+-*" and nuse.get(v, 0) == 1 and v not in rootset and v not in produced
                        and v not in loaded and consumer[v] in need and pg.byid[consumer[v]][0] in "+-"):
                    fuse_ok.add(v)
        pend, sums = {}, {}
        qn = {"n": 0}

        def qname():
            qn["n"] += 1
            return f"q{qn['n']}"

        def f_reduce(expr, bd, name):
            """word of a 64-bit Fp sum (canonical in canonical kernels)"""
            if kcanon:
                if bd >= RED:
                    expr, bd = f"fold64({expr})", fold_max(bd)
                w(f"  const uint32_t {name} = mont_reduce({expr});")
                return PM
            if bd + U32 * P > U64 or redc_max(bd) > U32:
                expr, bd = f"fold64({expr})", fold_max(bd)
            w(f"  const uint32_t {name} = redc_lazy({expr});")
            return redc_max(bd)

        def materialize(x):
            if x in pend:
                a, b = pend.pop(x)
                Mv[x] = op_mul(a, b, name=f"v{x}")[1]
                return
            kind, var, bd = sums.pop(x)
            Mv[x] = acc_to_ext(var, bd, f"v{x}") if kind == "E" else f_reduce(var, bd, f"v{x}")

        def opd(x):
            if x not in Mv and (x in pend or x in sums):
                materialize(x)
            return (f"v{x}", Mv[x], types[x], x)

        def negw(o):
            """k p - o for a word operand (k p >= its bound, k p < 2^32)"""
            while -(-o[1] // P) * P > U32:
                o = reduce1(o)
            kp = max(1, -(-o[1] // P)) * P
            nm = fresh()
            if o[2] == "f":
                w(f"  const uint32_t {nm} = {kp}u - {o[0]};")
            else:
                w(f"  const FpExt {nm} = xneg({o[0]}, {kp}u);")
            return (nm, kp, o[2], None)

        LIM = U64 - fold_max(U64)

        def sum_of(i, op, xa, xb):
            """64-bit sum for x_a + x_b or x_a - x_b, operands deferred products, sums or words"""
            E = types[i] == "e"
            st = {"e": None, "b": 0}

            def push(make, tb):
                cur, cb = st["e"], st["b"]
                if cur is not None and cb + tb > U64:
                    nm = qname()
                    w(f"  const {'Acc' if E else 'uint64_t'} {nm} = {'acc_fold' if E else 'fold64'}({cur});")
                    cur, cb = nm, fold_max(cb)
                assert cb + tb <= U64
                nm = qname()
                if E:
                    w(f"  const Acc {nm} = {make(cur if cur is not None else 'Acc{{0, 0, 0, 0}}')};")
                else:
                    w(f"  const uint64_t {nm} = {make(cur)};")
                st["e"], st["b"] = nm, cb + tb

            def f_add(cur, term):
                return term if cur is None else f"{cur} + {term}"

            def contrib(x, neg):
                if x in sums:
                    kind, var, bd = sums.pop(x)
                    if bd > LIM:
                        nm = qname()
                        w(f"  const {'Acc' if kind == 'E' else 'uint64_t'} {nm} = "
                          f"{'acc_fold' if kind == 'E' else 'fold64'}({var});")
                        var, bd = nm, fold_max(bd)
                    if neg:
                        if -(-bd // P) * P > U64:
                            nm = qname()
                            w(f"  const {'Acc' if kind == 'E' else 'uint64_t'} {nm} = "
                              f"{'acc_fold' if kind == 'E' else 'fold64'}({var});")
                            var, bd = nm, fold_max(bd)
                        K = max(1, -(-bd // P)) * P
                        if kind == "E":
                            push(lambda c: f"acc_add({c}, acc_negk({var}, {K}ull))", K)
                        elif E:
                            push(lambda c: f"acc_add0({c}, {K}ull - {var})", K)
                        else:
                            push(lambda c: f_add(c, f"({K}ull - {var})"), K)
                    else:
                        if kind == "E":
                            push(lambda c: f"acc_add({c}, {var})", bd)
                        elif E:
                            push(lambda c: f"acc_add0({c}, {var})", bd)
                        else:
                            push(lambda c: f_add(c, var), bd)
                    return
                if x in pend:
                    a, b = pend.pop(x)
                    if a[2] == "f" and b[2] == "e":
                        a, b = b, a
                    # every term below LIM, so a folded running sum always has room for it
                    while (4 if a[2] == b[2] == "e" else 1) * a[1] * max(b[1], PM if a[2] == b[2] == "e" else 0) > LIM:
                        if a[1] >= b[1]:
                            a = reduce1(a)
                        else:
                            b = reduce1(b)
                    if a[2] == "e" and b[2] == "e":
                        if neg:
                            a = negw(a)
                        push(lambda c: f"acc_me({c}, {a[0]}, {b[0]})", 4 * a[1] * max(b[1], PM))
                    elif a[2] == "e":
                        if neg:
                            b = negw(b)
                        push(lambda c: f"acc_mf({c}, {a[0]}, {b[0]})", a[1] * b[1])
                    else:
                        if neg:
                            b = negw(b)
                        if E:
                            push(lambda c: f"acc_m0({c}, {a[0]}, {b[0]})", a[1] * b[1])
                        else:
                            push(lambda c: f_add(c, f"uint64_t({a[0]}) * {b[0]}"), a[1] * b[1])
                    return
                o = opd(x)
                if neg:
                    o = negw(o)
                if o[2] == "e":
                    push(lambda c: f"acc_plus({c}, {o[0]})", o[1] * FOLDC)
                elif E:
                    push(lambda c: f"acc_plusf({c}, {o[0]})", o[1] * FOLDC)
                else:
                    push(lambda c: f_add(c, f"uint64_t({o[0]}) * {FOLDC}u"), o[1] * FOLDC)

            contrib(xa, False)
            contrib(xb, op == "-")
            sums[i] = ("E" if E else "F", st["e"], st["b"])
            if i not in fuse_ok:
                materialize(i)

        def special_mul(a, b):
            """products op_mul shortcuts (constant operands 1, 2, -1; FpExt constants)"""
            if a[2] == "f" and b[2] == "f":
                return any(cval.get(x[3]) in (one, two, mone) for x in (a, b) if x[3] is not None)
            if a[2] == "e" and b[2] == "e":
                return any(x[3] is not None and x[3] in ecval for x in (a, b))
            return False

        def decl(ty):
            return "uint32_t" if ty == "f" else "FpExt"

        def reduce1(o):
            nm, M, ty, key = o
            assert M >= P
            if key is not None:
                for nm2, m2 in red_memo.get(key, []):
                    if m2 < M:
                        return (nm2, m2, ty, key)
            n2 = fresh()
            w(f"  const {decl(ty)} {n2} = {'lred' if ty == 'f' else 'xred'}({nm});")
            m2 = max(PM, M - P)
            if key is not None:
                red_memo.setdefault(key, []).append((n2, m2))
            return (n2, m2, ty, key)

        def canonical(o):
            while o[1] >= P:
                o = reduce1(o)
            return o

        def larger_first(a, b):
            return (a, b) if a[1] >= b[1] else (b, a)

        def out(ty, expr, M, name=None):
            """declare a value; in canonical kernels (kcanon) every result is reduced (the
            pre-range-analysis arithmetic), otherwise only where the range analysis needs it"""
            nm = name or fresh()
            if kcanon:
                r = "lred" if ty == "f" else "xred"
                while M >= P:
                    expr, M = f"{r}({expr})", max(PM, M - P)
            w(f"  const {decl(ty)} {nm} = {expr};")
            return (nm, M, ty, None)

        def op_add(a, b, name=None):
            while a[1] + b[1] > U32:
                if a[1] >= b[1]:
                    a = reduce1(a)
                else:
                    b = reduce1(b)
            ta, tb = a[2], b[2]
            M = a[1] + b[1]
            if ta == "f" and tb == "f":
                return out("f", f"{a[0]} + {b[0]}", M, name)
            if ta == "e" and tb == "e":
                return out("e", f"xadd({a[0]}, {b[0]})", M, name)
            if ta == "e":
                return out("e", f"xaddf({a[0]}, {b[0]})", M, name)
            return out("e", f"xaddf({b[0]}, {a[0]})", M, name)

        def op_sub(a, b, name=None):
            while True:
                k = max(1, -(-b[1] // P))
                kp = k * P
                if a[1] + kp <= U32:
                    break
                if a[1] >= b[1]:
                    a = reduce1(a)
                else:
                    b = reduce1(b)
            M = a[1] + kp
            ta, tb = a[2], b[2]
            if ta == "f" and tb == "f":
                return out("f", f"lsub({a[0]}, {b[0]}, {kp}u)", M, name)
            if ta == "e" and tb == "e":
                return out("e", f"xsub({a[0]}, {b[0]}, {kp}u)", M, name)
            if ta == "e":
                return out("e", f"xsubf({a[0]}, {b[0]}, {kp}u)", M, name)
            return out("e", f"fsubx({a[0]}, {b[0]}, {kp}u)", M, name)

        def op_mul(a, b, name=None):
            ta, tb = a[2], b[2]
            if ta == "f" and tb == "f":
                for x, y in ((a, b), (b, a)):
                    c = cval.get(x[3]) if x[3] is not None else None
                    if c == one:
                        return out("f", y[0], y[1], name)
                    if c == two and 2 * y[1] <= U32:
                        return out("f", f"{y[0]} + {y[0]}", 2 * y[1], name)
                    if c == mone:
                        kp = max(1, -(-y[1] // P)) * P
                        return out("f", f"{kp}u - {y[0]}", kp, name)
            if ta == "e" and tb == "e":
                # a constant operand (the program's `e` values: x, and Fp constants embedded
                # as FpExt) needs no full extension product
                for x, y in ((a, b), (b, a)):
                    c = ecval.get(x[3]) if x[3] is not None else None
                    if c is None:
                        continue
                    if c[1:] == [0, 0, 0]:
                        if c[0] == one:
                            return out("e", y[0], y[1], name)
                        while not mul_ok(y[1], c[0]):
                            y = reduce1(y)
                        return out("e", f"xmulf({y[0]}, {c[0]}u)", redc_max(y[1] * c[0]), name)
                    if c == [0, one, 0, 0]:
                        while not mul_ok(y[1], NBW):
                            y = reduce1(y)
                        return out("e", f"xmulx({y[0]})", max(y[1], redc_max(y[1] * NBW)), name)
                while not emul_ok(a[1], b[1]):
                    if a[1] >= b[1]:
                        a = reduce1(a)
                    else:
                        b = reduce1(b)
                M = redc_max(fold_max(4 * a[1] * max(b[1], PM)))
                return out("e", f"xmul({a[0]}, {b[0]})", M, name)
            while not mul_ok(a[1], b[1]):
                if a[1] >= b[1]:
                    a = reduce1(a)
                else:
                    b = reduce1(b)
            M = redc_max(a[1] * b[1])
            if ta == "f" and tb == "f":
                return out("f", f"lmul({a[0]}, {b[0]})", M, name)
            if ta == "e":
                return out("e", f"xmulf({a[0]}, {b[0]})", M, name)
            return out("e", f"xmulf({b[0]}, {a[0]})", M, name)

        joined = {}

        def acc_src(x):
            """(expression, bound) of an Acc holding value x (partial sums joined)."""
            if x not in lazy:
                return f"acc_of(v{x})", Mv[x] * FOLDC
            ps = parts[x]
            if len(ps) == 1:
                return ps[0]
            if x not in joined:
                e, b = ps[0]
                for n_, (e2, b2) in enumerate(ps[1:]):
                    if b + b2 > U64:
                        e2, b2 = f"acc_fold({e2})", fold_max(b2)
                    e, b = room(e, b, b2)
                    nm = f"a{x}_j{n_}"
                    w(f"  const Acc {nm} = acc_add({e}, {e2});")
                    e, b = nm, b + b2
                joined[x] = (e, b)
            return joined[x]

        def acc_parts(x):
            if x in lazy:
                return list(parts[x]), chainpos[x] + 1
            return [(f"acc_of(v{x})", Mv[x] * FOLDC)], 1

        def room(expr, bd, add):
            """fold expr first if adding `add` could overflow 64 bits."""
            if bd + add > U64:
                bd = fold_max(bd)
                expr = f"acc_fold({expr})"
                assert bd + add <= U64
            return expr, bd

        def add_prod(expr, bd, t, k, q=None):
            """Acc expression for expr + t * pm[k]; t an operand; q: pm[k] already loaded
            into a uint4 (EC_PMV)."""
            j = len(pm_idx)
            pm_idx.append(len(acc_hist))  # the caller appends this term's Acc next
            pinned = None
            if kpinb and j >= kpinb:
                pinned = acc_hist[pm_idx[(j // kpinb - 1) * kpinb]]
            if t[2] == "e":
                while 4 * t[1] * PM + fold_max(U64) > U64:
                    t = reduce1(t)
                add = 4 * t[1] * PM
                expr, bd = room(expr, bd, add)
                if PIN and len(acc_hist) >= PIND:
                    a_ = acc_hist[-PIND]
                    return f"acc_ext({expr}, {t[0]}, pin(A.pm, {a_}), pin(A.pmn, {a_}), {k})", bd + add
                if pinned:
                    kk = f"4 * ({k})"
                    return (f"acc_extc({expr}, {t[0]}, pinc(A.pm, {pinned}) + {kk}, pinc(A.pmn, {pinned}) + {kk})",
                            bd + add)
                return f"acc_ext({expr}, {t[0]}, A.pm, A.pmn, {k})", bd + add
            add = t[1] * PM
            expr, bd = room(expr, bd, add)
            if q is not None:
                return f"acc_fpv({expr}, {t[0]}, {q})", bd + add
            if PIN and len(acc_hist) >= PIND:
                return f"acc_fp({expr}, {t[0]}, pin(A.pm, {acc_hist[-PIND]}), {k})", bd + add
            if pinned:
                return f"acc_fpc({expr}, {t[0]}, pinc(A.pm, {pinned}), {k})", bd + add
            return f"acc_fp({expr}, {t[0]}, A.pm, {k})", bd + add

        def acc_to_ext(expr, bd, name):
            """lazy FpExt of an Acc (REDC without the final min)"""
            if bd + U32 * P > U64 or redc_max(bd) > U32:
                expr, bd = f"acc_fold({expr})", fold_max(bd)
            M = redc_max(bd)
            if kcanon:
                if bd >= RED:
                    expr = f"acc_fold({expr})"
                w(f"  const FpExt {name} = acc_red({expr});")
                return PM
            w(f"  const FpExt {name} = acc_lred({expr});")
            return M

        def canon_out(expr, bd):
            if bd >= RED:
                return f"acc_red(acc_fold({expr}))"
            return f"acc_red({expr})"

        acc_state = {"n": 0, "b": 0}
        kwaves = int(os.environ.get("EC_WAVES_OVERRIDE", tune.get(ki, {}).get("waves", WAVES)))
        kpf = tune.get(ki, {}).get("pf", PF)
        kpmv = PMV or bool(tune.get(ki, {}).get("pmv", 0))
        kpmd = int(os.environ.get("EC_PMD", tune.get(ki, {}).get("pmd", PMD)))
        kpinb = int(os.environ.get("EC_PINB", tune.get(ki, {}).get("pinb", PINB)))
        if ORDER == "dfs":
            byid_ = pg.byid
            leaves = set(v for v in need if v in loaded or byid_[v][0] in "clgeu")
            oroots = sorted(set(roots), key=lambda v: pg.order[v])
            body = [v for v in dfs_order(pg, need, oroots, leaves) if v not in leaves]
            first_use = {}
            for n_, v in enumerate(body):
                for d in deps(byid_[v]):
                    if d in leaves and d not in first_use:
                        first_use[d] = n_
            consts = [v for v in leaves if byid_[v][0] in "cegu"]
            slots = {}
            for v in leaves:
                if byid_[v][0] in "cegu":
                    continue
                slots.setdefault(max(0, first_use.get(v, 0) - kpf), []).append(v)
            seq = sorted(consts, key=lambda v: pg.order[v])
            pmslots = {}
            if kpmv:
                for n_, v in enumerate(body):
                    ins_ = byid_[v]
                    if ins_[0] == "a" and types[ins_[3]] == "f":
                        pmslots.setdefault(max(0, n_ - kpmd), []).append(("pmv", f"q{v}", ins_[4], v))
                    elif ins_[0] == "b" and types[ins_[3]] == "f" and types[ins_[4]] == "f":
                        pmslots.setdefault(max(0, n_ - kpmd), []).append(("pmv", f"q{v}", ins_[5], v))
            kprog = [byid_[v] for v in seq]
            for n_, v in enumerate(body):
                kprog += [byid_[x] for x in sorted(slots.get(n_, []), key=lambda v: pg.order[v])]
                kprog += pmslots.get(n_, [])
                kprog.append(byid_[v])
        else:
            kprog = [ins_ for ins_ in prog if ins_[0] != "r"]
        order_pos = {}
        for n_, ins_ in enumerate(kprog):
            if ins_[0] != "pmv":
                order_pos[ins_[1]] = n_
        qv = {}
        term_at = {}
        for ti, (e, f) in enumerate(mine):
            rts = [x for x in term_roots((e, f)) if pg.byid[x][0] not in "cegu"]
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
                if sb2 + bd > U64:
                    cur, sb2 = f"acc_fold({cur})", fold_max(sb2)
                if sb2 + bd > U64:
                    src, bd = f"acc_fold({src})", fold_max(bd)
                w(f"  const Acc s{sn + 1} = acc_add({cur}, {src});")
                acc_state["n"], acc_state["b"] = sn + 1, sb2 + bd
                return
            cur = opd(e)
            for v in vals:
                cur = op_mul(cur, opd(v))
            if not pms:
                add = cur[1] * FOLDC
                s, sb2 = room(f"s{sn}", sb, add)
                w(f"  const Acc s{sn + 1} = acc_add({s}, acc_of({cur[0]}));")
                acc_state["n"], acc_state["b"] = sn + 1, sb2 + add
                return
            if len(pms) == 1:
                k = pms[0]
            else:
                if pms not in combo_index:
                    combo_index[pms] = len(combo_index)
                k = f"NPM + {combo_index[pms]}"
            e2, sb = add_prod(f"s{sn}", sb, cur, k)
            w(f"  const Acc s{sn + 1} = {e2};")
            acc_hist.append(f"s{sn + 1}")
            acc_state["n"], acc_state["b"] = sn + 1, sb

        if mine or last:
            w("  const Acc s0 = Acc{{0, 0, 0, 0}};")
        if kpmv:
            w("  uint32_t pmz;")
            w("#ifdef R0_EC_HOST")
            w("  pmz = 0;")
            w("#else")
            w('  asm volatile("v_mov_b32 %0, 0" : "=v"(pmz));')
            w("#endif")
        for ins in kprog:
            op, i = ins[0], ins[1]
            if op == "pmv":
                w(f"  const uint4 {i} = pm_vec(A.pm, pmz, {ins[2]});")
                qv[ins[3]] = i
                continue
            if i not in need or op == "r":
                continue
            if i in loaded:
                kind, s_ = slot[i]
                if kind == "f":
                    w(f"  const uint32_t v{i} = A.mf[uint64_t({s_}u) * A.domain + cycle];")
                else:
                    w(f"  FpExt v{i}; {{ uint4 t = reinterpret_cast<const uint4*>(A.me)[uint64_t({s_}u) * A.domain + cycle];"
                      f" v{i} = FpExt{{{{t.x, t.y, t.z, t.w}}}}; }}")
                Mv[i] = PM
                continue
            if op == "l" and not SADDR:
                # tap<W>: 32-bit column index while columns x domain < 2^32 words (every
                # po2 <= 22), the column-pointer table above (211 columns x 2^26 points at
                # po2=24); each kernel is instantiated for both, the launcher picks by domain
                g, col, back = ins[2], ins[3], ins[4]
                w(f"  const uint32_t v{i} = tap<W>(A.a[{g}], A.cp, {colslot[(g, col)]}u, {col}u, A.domain, (cycle - {4 * back}u) & mask);")
                Mv[i] = PM
                continue
            if op == "l":
                back = ins[4]
                if back not in offs:
                    offs.add(back)
                    w(f"  const uint32_t o{back} = ((cycle - {4 * back}u) & mask) * 4u;")
                w(f"  const uint32_t v{i} = ldc(A.cp[{colslot[(ins[2], ins[3])]}], o{back});")
                Mv[i] = PM
                continue
            if op == "c":
                cval[i] = enc(ins[2])
                w(f"  const uint32_t v{i} = {cval[i]}u;")
                Mv[i] = cval[i]
            elif op == "e":
                ev = [enc(x) for x in ins[2:6]]
                ecval[i] = ev
                w(f"  const FpExt v{i} = FpExt{{{{{', '.join(str(x) + 'u' for x in ev)}}}}};")
                Mv[i] = max(ev)
            elif op == "g":
                w(f"  const uint32_t v{i} = A.a[{ins[2]}][{ins[3]}];")
                Mv[i] = PM
            elif op == "u":
                q = 4 * ins[2]
                if types[i] == "f":
                    w(f"  const uint32_t v{i} = A.uv[{q}];")
                else:
                    w(f"  const FpExt v{i} = FpExt{{{{A.uv[{q}], A.uv[{q + 1}], A.uv[{q + 2}], A.uv[{q + 3}]}}}};")
                Mv[i] = PM
            elif op in "ab":
                ps, pos = acc_parts(ins[2])
                if op == "a":
                    t, k = opd(ins[3]), ins[4]
                else:
                    t, k = op_mul(opd(ins[3]), opd(ins[4])), ins[5]
                idx = pos % SPLIT
                if idx >= len(ps):
                    ps.append(("Acc{{0, 0, 0, 0}}", 0))
                expr, bd = add_prod(ps[idx][0], ps[idx][1], t, k, qv.get(i) if t[2] == "f" else None)
                w(f"  const Acc a{i} = {expr};")
                acc_hist.append(f"a{i}")
                ps[idx] = (f"a{i}", bd)
                parts[i], chainpos[i] = ps, pos
                if i in canon:
                    e_, b_ = acc_src(i)
                    Mv[i] = acc_to_ext(e_, b_, f"v{i}")
            elif kfuse and op == "*" and i in fuse_ok and not special_mul(opd(ins[2]), opd(ins[3])):
                pend[i] = (opd(ins[2]), opd(ins[3]))
            elif kfuse and op in "+-" and any(x in pend or x in sums for x in (ins[2], ins[3])):
                sum_of(i, op, ins[2], ins[3])
            else:
                fn = {"+": op_add, "-": op_sub, "*": op_mul}[op]
                Mv[i] = fn(opd(ins[2]), opd(ins[3]), name=f"v{i}")[1]
            if i in produced:
                kind, s_ = slot[i]
                o = canonical(opd(i))
                if kind == "f":
                    w(f"  A.mf[uint64_t({s_}u) * A.domain + cycle] = {o[0]};")
                else:
                    w(f"  reinterpret_cast<uint4*>(A.me)[uint64_t({s_}u) * A.domain + cycle] ="
                      f" make_uint4({o[0]}.c[0], {o[0]}.c[1], {o[0]}.c[2], {o[0]}.c[3]);")
            for ti in term_at.get(order_pos[i], []):
                emit_term(ti)
        if mine or last:
            # previous kernels' sum (if any) joins at the end; terms were added as they completed
            w("  uint4* accp = reinterpret_cast<uint4*>(A.acc) + cycle;")
            for ti in pending_terms():
                emit_term(ti)
            sn, sb = acc_state["n"], acc_state["b"]
            if not first:
                w(f"  Acc s{sn + 1}; {{ uint4 p = *accp; s{sn + 1} = acc_of(FpExt{{{{p.x, p.y, p.z, p.w}}}}); }}")
                cur, sb2 = room(f"s{sn}", sb, CANON)
                w(f"  const Acc s{sn + 2} = acc_add({cur}, s{sn + 1});")
                sn, sb = sn + 2, sb2 + CANON
            w(f"  FpExt s = {canon_out(f's{sn}', sb)};")
            if last:
                w("  s = fe_mul_fp(s, A.vinv[cycle & 3]);")
                w("  #pragma unroll")
                w("  for (int k = 0; k < 4; k++) A.check[uint64_t(k) * A.domain + cycle] = s.c[k];")
            else:
                w("  *accp = make_uint4(s.c[0], s.c[1], s.c[2], s.c[3]);")
        if first and not mine and not last:
            # keep the accumulator defined for later kernels
            w("  reinterpret_cast<uint4*>(A.acc)[cycle] = make_uint4(0u, 0u, 0u, 0u);")
        bodies.append((L, kwaves))
        stats.append(pg.cone_cost(roots))

    flat = []
    for pms, j in sorted(combo_index.items(), key=lambda kv: kv[1]):
        flat += [len(pms)] + list(pms)
    head = (f"// GENERATED by tools/gen_eval_check.py from risc0_amd/circuits/{circuit}.poly.ir — do not edit.\n"
            + common_text)
    info = [
        f"void eval_check_{circuit}_info(EvalCheckInfo* info) {{",
        f"  info->combos = ec_{circuit}::kPmCombos; info->ncombos = {len(combo_index)}; info->npm = ec_{circuit}::NPM;",
        f"  info->nargs = {nargs}; info->mat_fp = {nf}; info->mat_ext = {ne}; info->kernels = {len(kernels)};",
        f"  info->modmuls_per_point = {modmuls(pg) + 4};",
        f"  info->ncols = {len(colslot)}; info->col_arg = ec_{circuit}::kColArg; info->col_idx = ec_{circuit}::kColIdx;",
        f"  info->n_uniform = ec_{circuit}::NUV; info->uniform = ec_{circuit}::uniform;",
        "}",
    ]
    combos_line = f"const int kPmCombos[] = {{{', '.join(str(x) for x in flat) or '0'}}};"
    cols = sorted(colslot, key=colslot.get)
    combos_line += (f"\nconst int kColArg[] = {{{', '.join(str(a) for a, _ in cols)}}};"
                    f"\nconst int kColIdx[] = {{{', '.join(str(c) for _, c in cols)}}};")
    if host:
        # one host translation unit: every kernel body as a per-point function, for the
        # CPU check of the generated arithmetic (tests/test_ec_host.py)
        T = ["#define R0_EC_HOST 1", "#include <stddef.h>", "#include <stdint.h>",
             "struct uint4 { uint32_t x, y, z, w; };",
             "static inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return uint4{x, y, z, w}; }",
             head]
        for ki, (L, _) in enumerate(bodies):
            T.append(f"static void k{ki}(const Args& A, uint32_t cycle) {{")
            T.append("  constexpr bool W = true;")
            T.append("  const uint32_t mask = A.domain - 1;")
            T += L
            T.append("}")
        T.append(f"constexpr int NK = {len(bodies)};")
        T.append(f"static void (*const kTable[NK])(const Args&, uint32_t) = {{{', '.join(f'k{i}' for i in range(len(bodies)))}}};")
        T.append(combos_line)
        T += uniform_fn(pg)
        T.append(f"}}  // namespace ec_{circuit}")
        T.append("}  // namespace r0")
        T += [
            f'extern "C" int ec_host_{circuit}_combos(const int** combos, int* npm) {{',
            f"  *combos = r0::ec_{circuit}::kPmCombos; *npm = r0::ec_{circuit}::NPM; return {len(combo_index)};",
            "}",
            f'extern "C" void ec_host_{circuit}(const uint32_t* const* args, const uint32_t* pm, const uint32_t* pmn,',
            "    const uint32_t* vinv, uint32_t* acc, uint32_t* mf, uint32_t* me, uint32_t* check, uint32_t domain) {",
            f"  using namespace r0::ec_{circuit};",
            "  Args A;",
            f"  for (int i = 0; i < {nargs}; i++) A.a[i] = args[i];",
            f"  const uint32_t* cp[{len(colslot)}];",
            f"  for (int i = 0; i < {len(colslot)}; i++) cp[i] = args[kColArg[i]] + size_t(kColIdx[i]) * domain;",
            "  A.cp = cp;",
            "  A.pm = pm; A.pmn = pmn; A.acc = acc; A.check = check; A.vinv = vinv; A.mf = mf; A.me = me;",
            "  A.domain = domain; A.base = 0; A.count = domain; A.wide = 0;",
            "  uint32_t uvt[4 * (NUV ? NUV : 1)];",
            "  uniform(args, pm, uvt);",
            "  A.uv = uvt;",
            "  for (int k = 0; k < NK; k++)",
            "    for (uint32_t c = 0; c < domain; c++) kTable[k](A, c);",
            "}",
        ]
        return "\n".join(T) + "\n"

    for ki, (L, kwaves) in enumerate(bodies):
        K = [head]
        lb = "256" if kwaves <= 1 else f"256, {kwaves}"
        K.append(f"template <bool W> __global__ __launch_bounds__({lb}) void k{ki}(Args A) {{")
        K.append("  const uint32_t cycle = A.base + blockIdx.x * 256u + threadIdx.x;")
        K.append("  if (cycle >= A.base + A.count) return;")
        K.append("  const uint32_t mask = A.domain - 1;")
        K += L
        K.append("}")
        K.append(f"void launch_k{ki}(hipStream_t s, const Args& A) {{")
        K.append(f"  if (((A.wide >> {ki}) & 1) || uint64_t(kTapCols) * A.domain > (uint64_t(1) << 32))")
        K.append(f"    hipLaunchKernelGGL(k{ki}<true>, dim3(div_up(A.count, 256)), dim3(256), 0, s, A);")
        K.append("  else")
        K.append(f"    hipLaunchKernelGGL(k{ki}<false>, dim3(div_up(A.count, 256)), dim3(256), 0, s, A);")
        K.append("  HIP_OK(hipGetLastError());")
        K.append("}")
        K.append(f"}}  // namespace ec_{circuit}")
        K.append("}  // namespace r0")
        with open(os.path.join(outdir, f"eval_check_{circuit}_k{ki}.hip"), "w") as f:
            f.write("\n".join(K) + "\n")
    # kernels tuned to the scalar-column-base tap form at every size ("wide" in the tuning file)
    assert len(kernels) <= 64
    wide_list = [k for k in range(len(kernels)) if tune.get(k, {}).get("wide")]
    wide_default = sum(1 << k for k in wide_list)
    L = [head]
    w = L.append
    for ki in range(len(kernels)):
        w(f"void launch_k{ki}(hipStream_t s, const Args& A);")
    w(combos_line)
    L += uniform_fn(pg)
    w(f"}}  // namespace ec_{circuit}")
    L += info
    w(f"void eval_check_{circuit}(hipStream_t s, const EvalCheckArgs& e) {{")
    w(f"  using namespace ec_{circuit};")
    w(f"  R0_REQUIRE(e.nargs == {nargs}, \"eval_check_{circuit}: wrong argument count\");")
    w("  Args A;")
    w(f"  for (int i = 0; i < {nargs}; i++) A.a[i] = e.args[i];")
    w("  A.cp = e.colptr;")
    w("  A.pm = e.poly_mix; A.pmn = e.poly_mix_nb; A.acc = e.acc; A.check = e.check; A.vinv = e.vinv; A.domain = e.domain;")
    w("  A.mf = e.mat_fp; A.me = e.mat_ext; A.uv = e.uniform;")
    w(f"  R0_REQUIRE(NUV == 0 || e.uniform, \"eval_check_{circuit}: no lane-independent value table\");")
    w(f"  A.wide = e.wide >= 0 ? uint64_t(e.wide) : {wide_default}ull;  // tuned: {wide_list}")
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
    if sys.argv[1] == "--host":
        # gen_eval_check.py --host CIRCUIT OUT.cpp [BUDGET]
        src = emit(sys.argv[2], None, int(sys.argv[4]) if len(sys.argv) > 4 else 4000, host=True)
        with open(sys.argv[3], "w") as f:
            f.write(src)
    else:
        emit(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 4000)
