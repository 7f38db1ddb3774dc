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

  gen_accum.py CIRCUIT OUTDIR [LIMIT [INV_BATCH [LOAD_AHEAD]]]
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
    return 1 if node[0] == "s" else 1 + sum(size(c) for c in node[2])


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


DEFS = {"c", "l", "g", "+", "-", "*", "n", "i", "z", "ra"}


def defined(ins):
    if ins[0] == "ra":
        return list(ins[1:5])
    return [ins[1]] if ins[0] in DEFS else []


def used(ins):
    op = ins[0]
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


def emit_fn(name, prog, limit, kbase, inv_batch=1, load_ahead=0):
    defs = {}
    order = {}
    for pos, ins in enumerate(prog):
        for d in defined(ins):
            defs[d] = ins
            order[id(ins)] = pos
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
            op = ins[0]
            if op == "c":
                w(f"{ind}const uint32_t v{ins[1]} = {(ins[2] % P) * 2**32 % P}u;")
            elif op == "l":
                _, i, a, col, back = ins
                w(f"{ind}const uint32_t v{i} = A.a[{a}][uint64_t({col}u) * A.cycles + ((cycle - {back}u) & mask)];")
            elif op == "g":
                w(f"{ind}const uint32_t v{ins[1]} = A.a[{ins[2]}][{ins[3]}];")
            elif op in "+-*":
                f = {"+": "fp_add", "-": "fp_sub", "*": "fp_mul"}[op]
                w(f"{ind}const uint32_t v{ins[1]} = {f}(v{ins[2]}, v{ins[3]});")
            elif op == "n":
                w(f"{ind}const uint32_t v{ins[1]} = fp_neg(v{ins[2]});")
            elif op == "i":
                w(f"{ind}const uint32_t v{ins[1]} = fp_inv(v{ins[2]});")
            elif op == "z":
                w(f"{ind}const uint32_t v{ins[1]} = v{ins[2]} == 0u ? kOne : 0u;")
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
        kernels.append(L)
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
    ns, names, prefix = CIRCUITS[circuit]
    HEAD = head(circuit)
    fns = load(circuit)
    os.makedirs(outdir, exist_ok=True)
    launch = {}
    k = 0
    for name in names:
        launch[name] = []
        for L in emit_fn(name, fns[name], limit, k, inv_batch, load_ahead):
            src = [HEAD, f"__global__ __launch_bounds__(256) void k{k}(AccArgs A) {{",
                   "  const uint32_t cycle = blockIdx.x * 256u + threadIdx.x;",
                   "  if (cycle >= A.steps) return;",
                   "  const uint32_t mask = A.cycles - 1;"]
            src += L
            src += ["}", f"void launch_k{k}(hipStream_t s, const AccArgs& A) {{",
                    f"  hipLaunchKernelGGL(k{k}, dim3(div_up(A.steps, 256)), dim3(256), 0, s, A);",
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
