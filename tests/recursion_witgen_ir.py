"""The recursion witness generation IR (risc0_amd/circuits/recursion.witgen.ir, flattened by
tools/gen_witgen_ir.py from the reference's step_exec.cpp / step_verify_mem.cpp), run on the
CPU (test infrastructure only): each IR function is compiled to a Python function over raw
Montgomery words, and `witgen` drives them the way risc0_circuit_recursion_cpu_witgen does
(recursion-sys/kernels/cxx/ffi.cpp:57-205, externs extern.cpp): step_exec over the work
cycles, the WOM argument rows sorted, the exclusive scan of the per-cycle row counts,
injectWomBacks, then step_verify_mem over the work cycles. Cycles run in order (the
reference's forward mode; its parallel mode must give the same words)."""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 15 * 2**27 + 1
R = 2**32 % P
RINV = pow(2**32, P - 2, P)
INVALID = 0xFFFFFFFF
MAX_WOM_ROWS = 9  # kMaxWomRowsPerCycle (recursion-sys/kernels/cxx/context.h)


def enc(x):
    return (x % P) * R % P


def dec(w):
    return w * RINV % P


def mul(a, b):
    return a * b * RINV % P


def inv(a):
    return pow(dec(a), P - 2, P) * R % P if a else 0


class WitgenError(RuntimeError):
    pass


def load(path=None):
    fns, cur = {}, None
    for line in open(path or os.path.join(ROOT, "risc0_amd", "circuits", "recursion.witgen.ir")):
        if line.startswith("#") or not line.strip():
            continue
        t = line.split()
        if t[0] == "fn":
            cur = fns.setdefault(t[1], [])
            continue
        cur.append(t)
    return fns


def compile_fn(name, prog):
    """Python source of one step function: f(ctx, cycle) with ctx.args = [ctrl, global, data]
    (flat numpy uint32 arrays), ctx.steps and the extern state."""
    out = [f"def step_{name}(ctx, cycle):", "  args = ctx.args; steps = ctx.steps; mask = steps - 1"]
    ind = 1
    for t in prog:
        op, a = t[0], t[1:]
        pad = "  " * ind
        if op == "c":
            out.append(f"{pad}x{a[0]} = {enc(int(a[1]))}")
        elif op in ("l", "ld"):
            e = f"int(args[{a[1]}][{a[2]} * steps + ((cycle - {a[3]}) & mask)])"
            if op == "ld":
                out.append(f"{pad}x{a[0]} = {e}; x{a[0]} = 0 if x{a[0]} == {INVALID} else x{a[0]}")
            else:
                out.append(f"{pad}x{a[0]} = {e}")
        elif op == "g":
            out.append(f"{pad}x{a[0]} = int(args[{a[1]}][{a[2]}])")
        elif op == "+":
            out.append(f"{pad}x{a[0]} = (x{a[1]} + x{a[2]}) % {P}")
        elif op == "-":
            out.append(f"{pad}x{a[0]} = (x{a[1]} - x{a[2]}) % {P}")
        elif op == "*":
            out.append(f"{pad}x{a[0]} = x{a[1]} * x{a[2]} * {RINV} % {P}")
        elif op == "n":
            out.append(f"{pad}x{a[0]} = (-x{a[1]}) % {P}")
        elif op == "i":
            out.append(f"{pad}x{a[0]} = inv(x{a[1]})")
        elif op == "and":
            out.append(f"{pad}x{a[0]} = enc(dec(x{a[1]}) & dec(x{a[2]}))")
        elif op == "isz":
            out.append(f"{pad}x{a[0]} = {enc(1)} if x{a[1]} == 0 else 0")
        elif op == "if":
            out.append(f"{pad}if x{a[0]} != 0:")
            ind += 1
            out.append("  " * ind + "pass")
        elif op == "end":
            ind -= 1
        elif op == "w":
            out.append(f"{pad}args[{a[0]}][{a[1]} * steps + cycle] = x{a[2]}")
        elif op == "gw":
            out.append(f"{pad}args[{a[0]}][{a[1]}] = x{a[2]}")
        elif op == "chk":
            out.append(f"{pad}if x{a[0]} != 0: raise WitgenError('eqz failed at: zirgen/circuit/recursion/wom.cpp:{a[1]}')")
        elif op == "wr":
            out.append(f"{pad}x{a[0]}, x{a[1]}, x{a[2]}, x{a[3]} = ctx.wom_read(dec(x{a[4]}))")
        elif op == "pw":
            out.append(f"{pad}ctx.plonk_write(cycle, dec(x{a[0]}), (x{a[1]}, x{a[2]}, x{a[3]}, x{a[4]}))")
        elif op == "pr":
            out.append(f"{pad}x{a[0]}, x{a[1]}, x{a[2]}, x{a[3]}, x{a[4]} = ctx.plonk_read(cycle)")
        elif op == "iop":
            out.append(f"{pad}x{a[0]}, x{a[1]}, x{a[2]}, x{a[3]} = ctx.iop_body(cycle)")
        elif op == "rc":
            out.append(f"{pad}raise WitgenError('extern_readCoefficients not implemented')")
        else:
            raise ValueError(op)
    return "\n".join(out) + "\n"


_STEPS = None


def steps():
    global _STEPS
    if _STEPS is None:
        env = {"enc": enc, "dec": dec, "inv": inv, "WitgenError": WitgenError}
        for name, prog in load().items():
            exec(compile(compile_fn(name, prog), f"<witgen_{name}>", "exec"), env)
        _STEPS = env["step_exec"], env["step_verify"]
    return _STEPS


class Ctx:
    def __init__(self, ctrl, glob, data, n, wom, cycles, iops):
        self.args = [ctrl, glob, data]
        self.steps = n
        self.wom, self.iops = wom, iops
        self.iop_idx = [c[0] for c in cycles]
        ncyc = len(cycles)
        self.rows = [(INVALID, (INVALID,) * 4)] * (ncyc * MAX_WOM_ROWS)
        self.count = [0] * ncyc

    def wom_read(self, addr):
        return tuple(int(x) for x in self.wom[addr])

    def iop_body(self, cycle):
        i = self.iop_idx[cycle]
        self.iop_idx[cycle] += 1
        return tuple(int(x) for x in self.iops[i])

    def plonk_write(self, cycle, addr, value):
        i = self.count[cycle]
        assert i < MAX_WOM_ROWS
        self.rows[cycle * MAX_WOM_ROWS + i] = (addr, value)
        self.count[cycle] += 1

    def plonk_read(self, cycle):
        addr, v = self.rows[self.index[cycle]]
        self.index[cycle] += 1
        return (enc(addr),) + tuple(v)


def witgen(ctrl, data, glob, n, wom, cycles, iops):
    """In place on data (DATA x n) and glob: the reference's witgen over len(cycles) work
    cycles. wom / iops: (k, 4) Montgomery words; cycles: [(iop_idx, is_par_safe)]."""
    step_exec, step_verify = steps()
    ctx = Ctx(ctrl, glob, data, n, wom, cycles, iops)
    ncyc = len(cycles)
    for c in range(ncyc):
        step_exec(ctx, c)
    # verifyWom (ffi.cpp:118-135): sort by (addr, value as Fp: decoded words), exclusive scan
    ctx.rows.sort(key=lambda r: (r[0],) + tuple(dec(v) for v in r[1]))
    ctx.index, acc = [], 0
    for k in ctx.count:
        ctx.index.append(acc)
        acc += k
    # injectWomBacks (ffi.cpp:137-158)
    d = ctx.args[2]
    for c in range(1, ncyc):
        idx = ctx.index[c]
        vals = (enc(ctx.rows[idx - 1][0]),) + tuple(ctx.rows[idx - 1][1]) if idx else (0,) * 5
        for j in range(5):
            d[j * n + c - 1] = vals[j]
    for c in range(ncyc):
        step_verify(ctx, c)
