#!/usr/bin/env python3
"""Emit the gfx950 kernels of a circuit's accumulation step from its block IR:

  recursion (risc0_amd/circuits/recursion.accum.ir, tools/gen_accum_ir.py):
    compute : per cycle, the accumulator factor (recursion-sys step_compute_accum.cpp)
    verify  : per cycle, the accum-group registers from the prefix product
              (recursion-sys step_verify_accum.cpp)
  rv32im (risc0_amd/circuits/rv32im.accum.ir, tools/gen_rv32im_accum_ir.py):
    compute : per cycle, phase 1 of the accumulation (rv32im-sys steps.cpp step_TopAccum)

One lane per cycle, values are canonical Montgomery words in VGPRs, `if (x != 0)` blocks
stay branches (selectors are one-hot per cycle, so a wave takes a few arms).
Each function is cut into kernels of at most LIMIT operations along its block structure:
a piece re-evaluates the pure definitions it uses from enclosing blocks (loads, constants,
arithmetic) and runs under the conjunction of its enclosing guards. Pieces run in program
order, so every register write of a cycle lands in the order the reference makes it.

Sums of products are fused into lazily reduced linear combinations first (fuse_sums).

  gen_accum.py CIRCUIT OUTDIR [LIMIT [INV_BATCH [LOAD_AHEAD [FUSE [PACK [SORT]]]]]]
PACK > 0 packs whole arms into kernels under that cone cost (arm_chunks) where the
program has the rv32im shape; LIMIT cuts the others. SORT (default 1) makes those kernels
arm-sorted over workgroup tiles of SORT lanes (emit_sorted; default 256, 0 = unsorted).
Writes OUTDIR/accum_k<i>.hip and OUTDIR/accum.hip (launchers of the functions).
"""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
P = 15 * 2**27 + 1


def load(circuit):
    fns, cur = {}, None
    for line in open(os.path.join(ROOT, "risc0_amd", "circuits", circuit + ".accum.ir")):
        if line.startswith("#") or not line.strip():
            continue
        t = line.split()
        if t[0] == "fn":
            cur = fns.setdefault(t[1], [])
            continue
        cur.append((t[0],) + tuple(int(x) for x in t[1:]))
    return fns


def tree(prog):
    """statements -> nested [('s', ins) | ('if', cond, children)]"""
    root, stack = [], []
    cur = root
    for ins in prog:
        if ins[0] == "if":
            node = ("if", ins[1], [])
            cur.append(node)
            stack.append(cur)
            cur = node[2]
        elif ins[0] == "end":
            cur = stack.pop()
        else:
            cur.append(("s", ins))
    assert not stack
    return root


def size(node):
    if node[0] == "s":
        return sum(st[0] == "t" for st in node[1][2]) if node[1][0] == "lc" else 1
    return 1 + sum(size(c) for c in node[2])


def chunks(children, guards, limit, out):
    cur, n = [], 0
    for c in children:
        s = size(c)
        if c[0] == "if" and s > limit:
            if cur:
                out.append((guards, cur))
                cur, n = [], 0
            chunks(c[2], guards + [c[1]], limit, out)
            continue
        if cur and n + s > limit:
            out.append((guards, cur))
            cur, n = [], 0
        cur.append(c)
        n += s
    if cur:
        out.append((guards, cur))


def op_cost(ins):
    """VALU instructions of one definition, roughly (the kernel-packing cost model)"""
    o = ins[0]
    if o == "lc":
        return len(ins[2]) + 4
    return {"*": 5, "+": 3, "-": 3, "n": 3, "i": 45, "z": 2, "l": 1}.get(o, 0)


def arm_chunks(prog, limit):
    """Kernels made of whole arms: the rv32im step computes every instruction arm and keeps
    each arm's register writes under one `if (arm)` block, so most of a block's input cone
    is its own. Units are the top-level observable items (a guarded block, an unguarded
    store); units whose cones load a column another unit stores are merged (they keep
    program order in one kernel). Units are packed greedily, each into the kernel whose
    cone cost (op_cost over the union of the units' input cones) it raises least, while
    that cost stays under `limit`. Kernel order does not matter beyond that: two units in
    different kernels never store the same column unless their guards are exclusive
    (checked: each guard is a conjunction of selector literals, and two such conjunctions
    are exclusive when one selector appears with both polarities).
    The units that store the BigInt state columns (accum 0..11) also read them at back 1;
    another cycle's lane may write that row in the same kernel, before or after the read,
    in either order (the unsorted kernels had the same race across waves). Both orders give
    the same words because the step writes exactly the state the host injected there
    (tests/test_bigint_accum.py checks the reference's own step rewrites every injected
    state unchanged).
    Returns None when the program is not of that shape (a guarded block that defines
    values, or nested blocks)."""
    defs = {}
    for ins in prog:
        for d in defined(ins):
            defs[d] = ins
    units, depth = [], 0
    for ins in prog:
        if ins[0] == "if":
            if depth:
                return None
            units.append([ins])
            depth = 1
        elif ins[0] == "end":
            units[-1].append(ins)
            depth = 0
        elif depth:
            if ins[0] not in ("w",):
                return None
            units[-1].append(ins)
        elif ins[0] in ("w", "wa"):
            units.append([ins])
    # guards as selector literal sets
    lit = {}
    for ins in prog:
        if ins[0] == "z":
            x = ins[2]
            if x in lit and len(lit[x]) == 1:
                (v, pol), = lit[x]
                lit[ins[1]] = frozenset({(v, 1 - pol)})
            elif x not in lit:
                lit[ins[1]] = frozenset({(x, 0)})
        elif ins[0] == "*" and ins[2] in lit and ins[3] in lit:
            lit[ins[1]] = lit[ins[2]] | lit[ins[3]]

    def guard(u):
        return u[0][1] if u[0][0] == "if" else None

    def exclusive(a, b):
        la, lb = lit.get(a), lit.get(b)
        return la is not None and lb is not None and any((v, 1 - p) in lb for v, p in la)

    memo = {}

    def cone(v):
        if v not in memo:
            s = {v}
            for u in used(defs[v]):
                s |= cone(u)
            memo[v] = frozenset(s)
        return memo[v]

    def ucone(u):
        s = set()
        for ins in u:
            for v in (used(ins) if ins[0] != "if" else [ins[1]]):
                s |= cone(v)
        return s

    def stores(u):
        return {(ins[1], ins[2]) for ins in u if ins[0] == "w"} | ({"vals"} if any(i[0] == "wa" for i in u) else set())

    # merge units that share a column with a non-exclusive guard, or read what another stores
    cones = [ucone(u) for u in units]
    loads = [{(defs[v][2], defs[v][3]) for v in c if defs[v][0] == "l"} | ({"vals"} if any(defs[v][0] == "ra" for v in c) else set())
             for c in cones]
    parent = list(range(len(units)))

    def find(i):
        while parent[i] != i:
            parent[i] = parent[parent[i]]
            i = parent[i]
        return i

    st = [stores(u) for u in units]
    for i in range(len(units)):
        for j in range(i + 1, len(units)):
            clash = st[i] & st[j] and not exclusive(guard(units[i]), guard(units[j]))
            if clash or st[i] & loads[j] or st[j] & loads[i]:
                parent[find(j)] = find(i)
    merged = {}
    for i in range(len(units)):
        merged.setdefault(find(i), []).append(i)
    groups = sorted(merged.values())
    cost = lambda s: sum(op_cost(defs[v]) for v in s)
    kernels = []  # [unit indices, cone]
    for g in sorted(groups, key=lambda g: -cost(set().union(*(cones[i] for i in g)))):
        c = set().union(*(cones[i] for i in g))
        best, bi = None, None
        for k, (idx, kc) in enumerate(kernels):
            nc = cost(kc | c)
            if nc <= limit and (best is None or nc - cost(kc) < best):
                best, bi = nc - cost(kc), k
        if bi is None:
            kernels.append([list(g), c])
        else:
            kernels[bi][0] += g
            kernels[bi][1] |= c
    kernels.sort(key=lambda k: min(k[0]))
    out = []
    for idx, _ in kernels:
        nodes = []
        for i in sorted(idx):
            u = units[i]
            nodes += tree(u)
        out.append(([], nodes))
    return out


def booleans(prog):
    """values that are 0 or R (Montgomery one): isz results and their products"""
    b = set()
    for ins in prog:
        if ins[0] == "z" or (ins[0] == "c" and ins[2] % P in (0, 1)):
            b.add(ins[1])
        elif ins[0] == "*" and ins[2] in b and ins[3] in b:
            b.add(ins[1])
    return b


DEFS = {"c", "l", "g", "+", "-", "*", "n", "i", "z", "ra", "lc"}

R32 = 2**32 % P                     # Montgomery one
FOLD_C = 2**32 % P                  # fold64: hi * (2^32 mod p) + lo


def fuse_sums(prog):
    """Collapse every tree of single-use +, -, n nodes into one linear combination ("lc").

    Its leaves are single-use products x*y (a constant operand is folded into the
    multiplier, a negative sign into p - y) and plain values v (as v * R or v * (p - R)).
    The emitted code accumulates 64-bit v_mad_u64_u32 products, folds (hi * (2^32 mod p)
    + lo, one mad) only when the generator's exact bound on the running sum would pass
    2^64, and ends in one Montgomery reduction (input below p * 2^32), so the result is
    the canonical word the unfused ops give, with one mad per term instead of a reduced
    multiply and a canonical add each. Every operand is canonical (< p): computed values
    are, and the words read are too — data and global are zeroized before the
    accumulation (rv32im witgen/mod.rs:166-169, recursion prove/witgen.rs:119-121), an
    accum column is read only after this step wrote it, and the mix is drawn canonical.

    Returns the program with each collapsed tree's root replaced by
    ("lc", out, steps) — steps: ("t", x, y) with y an int (a value id) or ("k", const) or
    ("neg", value id) — and the tree's other nodes removed. A tree is collapsed only when
    it has a product leaf or at least four leaves (otherwise the plain ops are cheaper)."""
    defs, ncons, cons = {}, {}, {}
    for ins in prog:
        for d in defined(ins):
            defs[d] = ins
        for u in used(ins) + ([ins[1]] if ins[0] == "if" else []):
            ncons[u] = ncons.get(u, 0) + 1
            cons[u] = ins
    in_tree = {}

    def inner(v):
        """v's node is absorbed into its single consumer's linear combination"""
        if v in in_tree:
            return in_tree[v]
        r = False
        if defs[v][0] in "+-n*" and ncons.get(v, 0) == 1:
            c = cons[v]
            r = c[0] in "+-" or (c[0] == "n" and inner(c[1]))
        in_tree[v] = r
        return r

    def bound(v):
        return P - 1

    const = {ins[1]: (ins[2] % P) * R32 % P for ins in prog if ins[0] == "c"}
    out, removed = [], set()
    for ins in prog:
        if ins[0] not in "+-" or inner(ins[1]):
            out.append(ins)
            continue
        leaves, nodes = [], []

        def walk(v, sign):
            d = defs[v]
            if d is not ins and not inner(v):
                leaves.append(("v", sign, v))
                return
            if d[0] in "+-":
                nodes.append(d)
                walk(d[2], sign)
                walk(d[3], sign if d[0] == "+" else -sign)
            elif d[0] == "n":
                nodes.append(d)
                walk(d[2], -sign)
            else:  # a single-use product
                nodes.append(d)
                leaves.append(("p", sign, d[2], d[3]))

        walk(ins[1], 1)
        nprod = sum(l[0] == "p" for l in leaves)
        if nprod == 0 and len(leaves) < 4:
            out.append(ins)
            continue
        steps, b = [], 0
        for l in leaves:
            if l[0] == "v":
                x, y, ym = l[2], ("k", R32 if l[1] > 0 else P - R32), R32 if l[1] > 0 else P - R32
            else:
                x, y = l[2], l[3]
                if x in const and y not in const:
                    x, y = y, x
                if y in const:
                    k = const[y] if l[1] > 0 else (P - const[y]) % P
                    y, ym = ("k", k), k
                elif l[1] > 0:
                    ym = bound(y)
                else:
                    y, ym = ("neg", y), P
            tb = bound(x) * ym
            if b + tb >= 2**64:
                steps.append(("f",))
                b = (b >> 32) * FOLD_C + 2**32 - 1
                assert b + tb < 2**64
            steps.append(("t", x, y))
            b += tb
        if b >= P * 2**32:
            steps.append(("f",))
        out.append(("lc", ins[1], tuple(steps)))
        removed.update(id(n) for n in nodes if n is not ins)
    return [ins for ins in out if id(ins) not in removed]


def lc_used(steps):
    r = []
    for s in steps:
        if s[0] == "t":
            r.append(s[1])
            if isinstance(s[2], int):
                r.append(s[2])
            elif s[2][0] == "neg":
                r.append(s[2][1])
    return r


def defined(ins):
    if ins[0] == "ra":
        return list(ins[1:5])
    return [ins[1]] if ins[0] in DEFS else []


def used(ins):
    op = ins[0]
    if op == "lc":
        return lc_used(ins[2])
    if op in "+-*":
        return [ins[2], ins[3]]
    if op in ("n", "i", "z"):
        return [ins[2]]
    if op == "w":
        return [ins[3]]
    if op == "wa":
        return list(ins[1:5])
    return []


def flat(nodes):
    for n in nodes:
        if n[0] == "s":
            yield n[1]
        else:
            yield ("if", n[1])
            yield from flat(n[2])
            yield ("end",)


def batch_inverses(run, width, written=()):
    """Reorder one straight-line run of a kernel (its prelude, or the statements between two
    control markers of its body) so its field inverses run in batches of `width`
    (Montgomery's trick, fp_inv_batch: 3 multiplies per inverse plus one addition chain
    instead of 41 multiplies each). An inverse's level is the number of inverses on its
    longest input path within the run; the inverses of one level are independent, so each
    batch is preceded by the not-yet-emitted cone of its inputs and followed by whatever is
    left, in program order. Only definitions move, and only earlier; a batch whose cone
    would lift a load of a `written` array (or a vals read) above a store of the run is not
    formed. Returns the run with ("ib", [(out, in), ...]) pseudo-ops."""
    if width <= 1 or sum(ins[0] == "i" for ins in run) < 2:
        return run
    by_val = {d: ins for ins in run for d in defined(ins)}
    pos = {id(ins): k for k, ins in enumerate(run)}
    first_store = next((k for k, ins in enumerate(run) if ins[0] in ("w", "wa")), len(run))

    def pinned(ins):
        return pos[id(ins)] > first_store and (ins[0] == "ra" or (ins[0] == "l" and ins[2] in written))

    level = {}
    for ins in run:
        lv = max((level.get(u, 0) for u in used(ins)), default=0)
        for d in defined(ins):
            level[d] = lv + (1 if ins[0] == "i" else 0)
    invs = [ins for ins in run if ins[0] == "i"]
    groups = []
    for lv in sorted(set(level[i[1]] for i in invs)):
        same = [i for i in invs if level[i[1]] == lv]
        groups += [same[k:k + width] for k in range(0, len(same), width)]
    done, out = set(), []
    for g in groups:
        if len(g) == 1:
            continue
        cone, stack = {}, [i[2] for i in g]
        while stack:
            v = stack.pop()
            ins = by_val.get(v)
            if ins is None or id(ins) in done or id(ins) in cone:
                continue
            cone[id(ins)] = ins
            stack += used(ins)
        if any(pinned(ins) for ins in cone.values()):
            continue
        for ins in sorted(cone.values(), key=lambda i: pos[id(i)]):
            out.append(ins)
            done.add(id(ins))
        out.append(("ib", [(i[1], i[2]) for i in g]))
        done.update(id(i) for i in g)
    out += [ins for ins in run if id(ins) not in done]
    return out


def batch_body(body, width, written):
    """batch_inverses over every straight-line run of a kernel body"""
    out, run = [], []
    for ins in body + [("end",)]:
        if ins[0] in ("if", "end"):
            out += batch_inverses(run, width, written)
            run = []
            out.append(ins)
        else:
            run.append(ins)
    return out[:-1]


def stmt_lines(ins, ind, bools):
    """the HIP lines of one statement"""
    L = []
    w = L.append
    op = ins[0]
    if op == "c":
        w(f"{ind}const uint32_t v{ins[1]} = {(ins[2] % P) * 2**32 % P}u;")
    elif op == "l":
        _, i, a, col, back = ins
        w(f"{ind}const uint32_t v{i} = A.a[{a}][uint64_t({col}u) * A.cycles + ((cycle - {back}u) & mask)];")
    elif op == "g":
        w(f"{ind}const uint32_t v{ins[1]} = A.a[{ins[2]}][{ins[3]}];")
    elif op == "*" and ins[2] in bools and ins[3] in bools:
        # both 0 or R: the product is their minimum
        w(f"{ind}const uint32_t v{ins[1]} = umin(v{ins[2]}, v{ins[3]});")
    elif op in "+-*":
        f = {"+": "fp_add", "-": "fp_sub", "*": "fp_mul"}[op]
        w(f"{ind}const uint32_t v{ins[1]} = {f}(v{ins[2]}, v{ins[3]});")
    elif op == "n":
        w(f"{ind}const uint32_t v{ins[1]} = fp_neg(v{ins[2]});")
    elif op == "i":
        w(f"{ind}const uint32_t v{ins[1]} = fp_inv(v{ins[2]});")
    elif op == "z":
        w(f"{ind}const uint32_t v{ins[1]} = v{ins[2]} == 0u ? kOne : 0u;")
    elif op == "lc":
        first = True
        for s in ins[2]:
            if s[0] == "f":
                w(f"{ind}t{ins[1]} = fold64(t{ins[1]});")
                continue
            y = s[2]
            ye = f"v{y}" if isinstance(y, int) else (f"{y[1]}u" if y[0] == "k" else f"(kP - v{y[1]})")
            if first:
                w(f"{ind}uint64_t t{ins[1]} = uint64_t(v{s[1]}) * {ye};")
                first = False
            else:
                w(f"{ind}t{ins[1]} += uint64_t(v{s[1]}) * {ye};")
        w(f"{ind}const uint32_t v{ins[1]} = mont_reduce(t{ins[1]});")
    elif op == "ib":
        n = len(ins[1])
        tag = ins[1][0][0]
        w(f"{ind}uint32_t ib{tag}[{n}] = {{{', '.join(f'v{x}' for _, x in ins[1])}}};")
        w(f"{ind}fp_inv_batch(ib{tag});")
        for k, (o, _) in enumerate(ins[1]):
            w(f"{ind}const uint32_t v{o} = ib{tag}[{k}];")
    elif op == "ra":
        w(f"{ind}const uint4 r{ins[1]} = A.vals[cycle];")
        for k, c in enumerate("xyzw"):
            w(f"{ind}const uint32_t v{ins[1 + k]} = r{ins[1]}.{c};")
    elif op == "wa":
        w(f"{ind}A.vals[cycle] = make_uint4(v{ins[1]}, v{ins[2]}, v{ins[3]}, v{ins[4]});")
    elif op == "w":
        _, a, col, i = ins
        w(f"{ind}A.a[{a}][uint64_t({col}u) * A.cycles + cycle] = v{i};")
    else:
        raise ValueError(op)
    return L


def cone_defs(vals, defs, avail):
    """the definitions `vals` need beyond the values in `avail`"""
    seen, stack = {}, [v for v in vals if v not in avail]
    while stack:
        ins = defs[stack.pop()]
        if id(ins) in seen:
            continue
        seen[id(ins)] = ins
        stack += [u for u in used(ins) if u not in avail]
    return list(seen.values())


def block(L, ind, items, extra, avail, defs, order, inv_batch, load_ahead, bools):
    """Emit at indent `ind` the definitions that `extra` and the stores `items` need beyond
    `avail` — depth-first, each just before the first item that needs it, inverses batched,
    trace loads issued `load_ahead` ahead — then the items. Returns the values defined."""
    vals = list(extra) + [u for it in items for u in used(it)]
    pre = batch_inverses(sorted(cone_defs(vals, defs, avail), key=lambda i: order[id(i)]), inv_batch)
    node_of = {}
    for k, ins in enumerate(pre):
        for d in ([o for o, _ in ins[1]] if ins[0] == "ib" else defined(ins)):
            node_of[d] = k
    uses_of = lambda ins: [x for _, x in ins[1]] if ins[0] == "ib" else used(ins)
    done, seq = set(), []

    def need(vs):
        stack = [(node_of[v], False) for v in reversed(list(vs)) if v in node_of]
        while stack:
            k, expanded = stack.pop()
            if k in done:
                continue
            if expanded:
                done.add(k)
                seq.append(("node", k))
                continue
            stack.append((k, True))
            stack += [(node_of[u], False) for u in reversed(uses_of(pre[k])) if u in node_of and node_of[u] not in done]

    need(extra)
    for it in items:
        need(used(it))
        seq.append(("item", it))
    loads = [k for t, k in seq if t == "node" and pre[k][0] == "l"]
    issued, seen = set(), 0
    for t, x in seq:
        if t == "node" and pre[x][0] == "l":
            seen += 1
        for k in loads[:seen + load_ahead]:
            if k not in issued:
                issued.add(k)
                L.extend(stmt_lines(pre[k], ind, bools))
        if t == "node":
            if x not in issued:
                issued.add(x)
                L.extend(stmt_lines(pre[x], ind, bools))
        else:
            L.extend(stmt_lines(x, ind, bools))
    return set(avail) | {d for ins in pre for d in ([o for o, _ in ins[1]] if ins[0] == "ib" else defined(ins))}


ACC_WAVES = {}


def emit_sorted(nodes, defs, order, inv_batch, load_ahead, bools, tile=256):
    """One arm-sorted kernel over whole units (arm_chunks): each cycle's key is the first of
    the kernel's arm guards it satisfies; the 256 cycles of a workgroup are counting-sorted
    by key (tile_sort_lane, accum_gen.h), so a wavefront holds few arms; then every unit
    runs as `if (guard) { its input cone; its stores }`, its cone computed inside the
    block, so a wave skips the arms none of its lanes take. Units keep program order."""
    guards = []
    for n in nodes:
        if n[0] == "if" and n[1] not in guards:
            guards.append(n[1])
    K = len(guards)
    assert K < 32
    L = ["  const uint32_t mask = A.cycles - 1;", f"  const uint32_t c0 = blockIdx.x * {tile}u + threadIdx.x;"]
    if K:
        L += [f"  uint32_t key = {K}u;", "  if (c0 < A.steps) {", "    const uint32_t cycle = c0;"]
        block(L, "    ", [], guards, set(), defs, order, 1, load_ahead, bools)
        sel = f"{K}u"
        for i in reversed(range(K)):
            sel = f"v{guards[i]} != 0u ? {i}u : {sel}"
        L += [f"    key = {sel};", "  }",
              f"  const uint32_t cycle = blockIdx.x * {tile}u + tile_sort_lane<{tile}>(key, {K + 1}u);"]
    else:
        L += ["  const uint32_t cycle = c0;"]
    L += ["  if (cycle >= A.steps) return;"]
    avail = block(L, "  ", [], guards, set(), defs, order, 1, load_ahead, bools)
    for n in nodes:
        if n[0] == "s":
            avail = block(L, "  ", [n[1]], [], avail, defs, order, inv_batch, load_ahead, bools)
        else:
            L.append(f"  if (v{n[1]} != 0u) {{")
            block(L, "    ", [c[1] for c in n[2]], [], avail, defs, order, inv_batch, load_ahead, bools)
            L.append("  }")
    return L


def emit_fn(name, prog, limit, kbase, inv_batch=1, load_ahead=0, pack=0, sort=0):
    """the kernels of one function: [(lines, own_header)]"""
    defs = {}
    order = {}
    for pos, ins in enumerate(prog):
        for d in defined(ins):
            defs[d] = ins
            order[id(ins)] = pos
    bools = booleans(prog)
    out = arm_chunks(prog, pack) if pack else None
    if out is not None and sort:
        return [(emit_sorted(nodes, defs, order, inv_batch, load_ahead, bools, sort), True) for _, nodes in out]
    if out is None:
        out = []
        chunks(tree(prog), [], limit, out)
    kernels = []
    for guards, nodes in out:
        body = list(flat(nodes))
        if not any(ins[0] in ("w", "wa") for ins in body):
            continue  # nothing observable (definitions only; their users re-evaluate them)
        have = set(d for ins in body if ins[0] in DEFS for d in defined(ins))
        need = set(guards)
        for ins in body:
            if ins[0] == "if":
                need.add(ins[1])
            need.update(used(ins))
        pre = {}
        stack = [v for v in need if v not in have]
        while stack:
            v = stack.pop()
            ins = defs[v]
            if id(ins) in pre:
                continue
            pre[id(ins)] = ins
            stack += [u for u in used(ins) if u not in have]
        written = {ins[1] for ins in body if ins[0] == "w"}
        vals_written = any(ins[0] == "wa" for ins in body)
        pinned = lambda ins: (ins[0] == "l" and ins[2] in written) or (ins[0] == "ra" and vals_written)
        # the value pool: the prelude and the body's top-level pure definitions, emitted on
        # demand; the items: everything else at the top level of the body, in order
        pool = sorted(pre.values(), key=lambda i: order[id(i)])
        items, lv, cur = [], 0, None
        for ins in body:
            if lv == 0 and ins[0] in DEFS and not pinned(ins):
                pool.append(ins)
            elif lv == 0 and ins[0] != "if":
                items.append([ins])
            else:
                if lv == 0:
                    cur = []
                    items.append(cur)
                cur.append(ins)
            lv += {"if": 1, "end": -1}.get(ins[0], 0)
        split = []
        for it in items:
            if it[0][0] == "if" and all(x[0] == "w" for x in it[1:-1]):
                split += [[it[0], x, it[-1]] for x in it[1:-1]]  # one guarded store per item
            elif it[0][0] == "if":
                split.append([it[0]] + batch_body(it[1:-1], inv_batch, written) + [it[-1]])
            else:
                split.append(it)
        items = split
        pre = batch_inverses(pool, inv_batch)
        L = []
        w = L.append
        ind = "  "

        def stmt(ins, ind):
            L.extend(stmt_lines(ins, ind, bools))

        # pool values are emitted depth-first, each just before the first top-level item that
        # needs it (short live ranges: program order kept every value live from its
        # definition to its last store and spilled); stores keep their order
        node_of = {}
        for k, ins in enumerate(pre):
            for d in ([o for o, _ in ins[1]] if ins[0] == "ib" else defined(ins)):
                node_of[d] = k
        uses_of = lambda ins: [x for _, x in ins[1]] if ins[0] == "ib" else used(ins)
        done = set()

        def need(vals, seq):
            stack = [(node_of[v], False) for v in reversed(list(vals)) if v in node_of]
            while stack:
                k, expanded = stack.pop()
                if k in done:
                    continue
                if expanded:
                    done.add(k)
                    seq.append(("node", k))
                    continue
                stack.append((k, True))
                for u in reversed(uses_of(pre[k])):
                    if u in node_of and node_of[u] not in done:
                        stack.append((node_of[u], False))

        gseq, seq = [], []
        need(guards, gseq)
        for item in items:
            vals = []
            for it in item:
                vals += [it[1]] if it[0] == "if" else ([] if it[0] == "end" else uses_of(it))
            need(vals, seq)
            seq.append(("item", item))
        need([d for ins in pre for d in defined(ins) if ins[0] != "ib"], seq)  # unused pool values
        for _, k in gseq:
            stmt(pre[k], ind)
        if guards:
            w(f"  if ({' && '.join(f'v{g} != 0u' for g in guards)}) {{")
            ind = "    "
        # trace loads run `load_ahead` loads ahead of their depth-first position, so a wave
        # has that many in flight instead of waiting on each right before its use
        loads = [k for t, k in seq if t == "node" and pre[k][0] == "l"]
        issued, seen = set(), 0
        depth = ind
        for t, x in seq:
            if t == "node" and pre[x][0] == "l":
                seen += 1
            for k in loads[:seen + load_ahead]:
                if k not in issued:
                    issued.add(k)
                    stmt(pre[k], ind)
            if t == "node":
                if x not in issued:
                    issued.add(x)
                    stmt(pre[x], ind)
                continue
            for ins in x:
                if ins[0] == "if":
                    w(f"{depth}if (v{ins[1]} != 0u) {{")
                    depth += "  "
                elif ins[0] == "end":
                    depth = depth[:-2]
                    w(f"{depth}}}")
                else:
                    stmt(ins, depth)
        if guards:
            w("  }")
        kernels.append((L, False))
    return kernels


CIRCUITS = {  # namespace, functions in launch order, launcher prefix
    "recursion": ("rec_accum", ("compute", "verify"), "recursion_accum_"),
    "rv32im": ("rv_accum", ("compute",), "rv32im_accum_"),
}


def head(circuit):
    ns = CIRCUITS[circuit][0]
    return (f"// GENERATED by tools/gen_accum.py from risc0_amd/circuits/{circuit}.accum.ir — do not edit.\n"
            f"#include \"accum_gen.h\"\nnamespace r0 {{\nnamespace {ns} {{\n")


def main():
    circuit, outdir = sys.argv[1], sys.argv[2]
    limit = int(sys.argv[3]) if len(sys.argv) > 3 else 1200
    inv_batch = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    load_ahead = int(sys.argv[5]) if len(sys.argv) > 5 else 64
    fuse = int(sys.argv[6]) if len(sys.argv) > 6 else 1
    # R0_ACC_WAVES="3" (every kernel) or "0:3,2:3" (kernel:waves): an occupancy target per
    # kernel (amdgpu_waves_per_eu); unset, the compiler picks the register budget
    global ACC_WAVES
    ACC_WAVES = {(-1 if ":" not in e else int(e.split(":")[0])): int(e.split(":")[-1])
                 for e in os.environ.get("R0_ACC_WAVES", "").split(",") if e}
    pack = int(sys.argv[7]) if len(sys.argv) > 7 else 20000
    sort = int(sys.argv[8]) if len(sys.argv) > 8 else 256
    ns, names, prefix = CIRCUITS[circuit]
    HEAD = head(circuit)
    fns = load(circuit)
    if fuse:
        fns = {k: fuse_sums(v) for k, v in fns.items()}
    os.makedirs(outdir, exist_ok=True)
    for f in os.listdir(outdir):
        if f.startswith("accum_k") and f.endswith(".hip"):
            os.remove(os.path.join(outdir, f))
    launch = {}
    k = 0
    for name in names:
        launch[name] = []
        for L, own in emit_fn(name, fns[name], limit, k, inv_batch, load_ahead, pack, sort):
            wg = sort if own else 256
            wv = ACC_WAVES.get(k, ACC_WAVES.get(-1, 0))
            occ = f" __attribute__((amdgpu_waves_per_eu({wv}, {wv})))" if wv else ""
            src = [HEAD, f"__global__ __launch_bounds__({wg}){occ} void k{k}(AccArgs A) {{"]
            if not own:
                src += ["  const uint32_t cycle = blockIdx.x * 256u + threadIdx.x;",
                        "  if (cycle >= A.steps) return;",
                        "  const uint32_t mask = A.cycles - 1;"]
            src += L
            src += ["}", f"void launch_k{k}(hipStream_t s, const AccArgs& A) {{",
                    f"  hipLaunchKernelGGL(k{k}, dim3(div_up(A.steps, {wg})), dim3({wg}), 0, s, A);",
                    "  HIP_OK(hipGetLastError());", "}", f"}}  // namespace {ns}", "}  // namespace r0"]
            with open(os.path.join(outdir, f"accum_k{k}.hip"), "w") as f:
                f.write("\n".join(src) + "\n")
            launch[name].append(k)
            k += 1
    L = [HEAD]
    for i in range(k):
        L.append(f"void launch_k{i}(hipStream_t s, const AccArgs& A);")
    L.append(f"}}  // namespace {ns}")
    for name in names:
        L.append(f"void {prefix}{name}(hipStream_t s, const AccArgs& A) {{")
        for i in launch[name]:
            L.append(f"  {ns}::launch_k{i}(s, A);")
        L.append("}")
    L.append("}  // namespace r0")
    with open(os.path.join(outdir, "accum.hip"), "w") as f:
        f.write("\n".join(L) + "\n")
    print(f"{circuit} accum: " + " + ".join(f"{len(launch[n])} {n}" for n in names) + " kernels")


if __name__ == "__main__":
    main()
