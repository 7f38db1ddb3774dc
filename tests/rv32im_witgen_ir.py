"""The rv32im witness-generation IR (risc0_amd/circuits/rv32im.witgen.ir, flattened by
tools/gen_rv32im_witgen_ir.py from the reference's steps.cpp step_Top), run on the CPU (test
infrastructure only): the IR is compiled to one Python function over raw Montgomery words
with the branches kept, and `witgen` drives it the way risc0_circuit_rv32im_cpu_witgen does
in forward mode (rv32im-sys/kernels/cxx/ffi.cpp:267-308), with the externs of
ffi.cpp:84-228 and the lookup tables of tables.h. Checked reads of unset words, inconsistent
re-stores (buffers.h:30-55), EQZ failures and the externs' own checks raise WitgenError
with the reference's message."""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 15 * 2**27 + 1
R = 2**32 % P
RINV = pow(2**32, P - 2, P)
INVALID = 0xFFFFFFFF


def enc(x):
    return (x % P) * R % P


def dec(w):
    return w * RINV % P


def inv(a):
    return pow(dec(a), P - 2, P) * R % P if a else 0


class WitgenError(RuntimeError):
    pass


def load(path=None):
    strings, consts, ops = {}, [], []
    for line in open(path or os.path.join(ROOT, "risc0_amd", "circuits", "rv32im.witgen.ir")):
        if line.startswith("#") or not line.strip():
            continue
        if line.startswith("s "):
            _, k, text = line.rstrip("\n").split(" ", 2)
            strings[int(k)] = text
            continue
        t = line.split()
        (consts if t[0] == "c" else ops).append(t)
    return strings, consts, ops


def compile_ir(strings, consts, ops):
    """Python source of step(ctx, cycle); ctx.data / ctx.glob flat uint32 arrays"""
    out = ["def step(ctx, cycle):", "  data = ctx.data; glob = ctx.glob; rows = ctx.rows; S = ctx.strings",
           "  ctx.begin(cycle)"]
    for t in consts:
        out.append(f"  x{t[1]} = {enc(int(t[2]))}")
    ind = 1
    frames = []
    prev = None
    for t in ops:
        op, a = t[0], t[1:]
        pad = "  " * ind
        if op == "l":
            out.append(f"{pad}x{a[0]} = ctx.get({a[1]}, (cycle - {a[2]}) % rows)")
        elif op == "g":
            out.append(f"{pad}x{a[0]} = ctx.gget({a[1]})")
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
        elif op == "z":
            out.append(f"{pad}x{a[0]} = {enc(1)} if x{a[1]} == 0 else 0")
        elif op == "and":
            out.append(f"{pad}x{a[0]} = enc(dec(x{a[1]}) & dec(x{a[2]}))")
        elif op == "mod":
            out.append(f"{pad}x{a[0]} = enc(dec(x{a[1]}) % dec(x{a[2]}))")
        elif op == "inr":
            out.append(f"{pad}x{a[0]} = {enc(1)} if dec(x{a[1]}) <= dec(x{a[2]}) < dec(x{a[3]}) else 0")
        elif op == "m":
            out.append(f"{pad}x{a[0]} = 0")
        elif op == "a":
            out.append(f"{pad}x{a[0]} = x{a[1]}")
        elif op == "if":
            if prev == "else":  # an else-if chain: `else:` + `pass` become `elif ...:` + `pass`
                assert out[-1].strip() == "pass" and out[-2].strip() == "else:"
                out[-2] = out[-2].replace("else:", f"elif x{a[0]} != 0:")
                frames.append(True)
            else:
                out.append(f"{pad}if x{a[0]} != 0:")
                ind += 1
                out.append("  " * ind + "pass")
                frames.append(False)
        elif op == "else":
            ind -= 1
            out.append("  " * ind + "else:")
            ind += 1
            out.append("  " * ind + "pass")
        elif op == "end":
            if not frames.pop():
                ind -= 1
        elif op == "w":
            out.append(f"{pad}ctx.set({a[0]}, cycle, x{a[1]})")
        elif op == "gw":
            out.append(f"{pad}ctx.gset({a[0]}, x{a[1]})")
        elif op == "eqz":
            out.append(f"{pad}if x{a[0]} != 0: ctx.eqz_fail(cycle, S[{a[1]}])")
        elif op == "unreachable":
            out.append(f"{pad}raise WitgenError('Reached unreachable mux arm')")
        elif op == "first":
            out.append(f"{pad}x{a[0]} = {enc(1)} if cycle == 0 else 0")
        elif op == "mm":
            out.append(f"{pad}x{a[0]}, x{a[1]} = ctx.major_minor(cycle)")
        elif op == "txn":
            out.append(f"{pad}x{a[0]}, x{a[1]}, x{a[2]}, x{a[3]}, x{a[4]} = ctx.txn(cycle, x{a[5]})")
        elif op == "lkd":
            out.append(f"{pad}ctx.lookup_delta(cycle, x{a[0]}, x{a[1]})")
        elif op == "lkc":
            out.append(f"{pad}x{a[0]} = ctx.lookup_current(x{a[1]}, x{a[2]})")
        elif op == "dc":
            out.append(f"{pad}x{a[0]} = ctx.diff_count(x{a[1]})")
        elif op == "div":
            out.append(f"{pad}x{a[0]}, x{a[1]}, x{a[2]}, x{a[3]} = ctx.divide(x{a[4]}, x{a[5]}, x{a[6]}, x{a[7]}, x{a[8]})")
        elif op == "hrp":
            out.append(f"{pad}x{a[0]} = ctx.host_word(cycle)")
        elif op == "hw":
            out.append(f"{pad}x{a[0]} = ctx.host_word(cycle)")
        elif op == "npi":
            out.append(f"{pad}x{a[0]}, x{a[1]} = ctx.paging(cycle)")
        elif op == "bi":
            out.append(f"{pad}" + ", ".join(f"x{v}" for v in a) + " = ctx.bigint(cycle)")
        else:
            raise ValueError(op)
        prev = op
    return "\n".join(out) + "\n"


_STEP = None


def step_fn():
    global _STEP
    if _STEP is None:
        strings, consts, ops = load()
        src = compile_ir(strings, consts, ops)
        env = {"enc": enc, "dec": dec, "inv": inv, "WitgenError": WitgenError}
        exec(compile(src, "<rv32im_witgen>", "exec"), env)
        _STEP = (env["step"], strings)
    return _STEP


def divide_rv32im(numer, denom, sign_type):  # ffi.cpp:54-82
    M = 0xFFFFFFFF
    ones = 1 if sign_type == 2 else 0
    neg_n = sign_type != 0 and numer >= 0x80000000
    neg_d = sign_type == 1 and denom >= 0x80000000
    if neg_n:
        numer = (-numer - ones) & M
    if neg_d:
        denom = (-denom - ones) & M
    if denom == 0:
        quot, rem = M, numer
    else:
        quot, rem = numer // denom, numer % denom
    qneg = (int(neg_n) ^ int(neg_d)) - (int(denom == 0) * int(neg_n))
    if qneg & M:
        quot = (-quot - ones) & M
    if neg_n:
        rem = (-rem - ones) & M
    return quot, rem


class Ctx:
    def __init__(self, data, glob, rows, cycles, txns, bigint=None):
        self.data, self.glob, self.rows = data, glob, rows
        self.cycles, self.txns = cycles, txns
        self.bigint_bytes = bigint if bigint is not None else np.zeros(0, np.uint8)
        self.u8 = np.zeros(1 << 8, np.int64)
        self.u16 = np.zeros(1 << 16, np.int64)
        self.strings = step_fn()[1]

    def begin(self, cycle):
        self.cur = int(self.cycles["txnIdx"][cycle])

    def get(self, col, row):
        w = int(self.data[col * self.rows + row])
        if w == INVALID:
            raise WitgenError(f"Read of unset value (row {row}, col {col})")
        return w

    def set(self, col, row, v):
        i = col * self.rows + row
        cur = int(self.data[i])
        if cur != INVALID and cur != v:
            raise WitgenError(f"Inconsistent set (row {row}, col {col}: {cur:#x} -> {v:#x})")
        self.data[i] = v

    def gget(self, idx):
        w = int(self.glob[idx])
        if w == INVALID:
            raise WitgenError(f"Read of unset value (global {idx})")
        return w

    def gset(self, idx, v):
        cur = int(self.glob[idx])
        if cur != INVALID and cur != v:
            raise WitgenError(f"Inconsistent set (global {idx})")
        self.glob[idx] = v

    def eqz_fail(self, cycle, msg):
        raise WitgenError(f"[{cycle}]: eqz failure at: {msg}")

    def major_minor(self, cycle):
        return enc(int(self.cycles["major"][cycle])), enc(int(self.cycles["minor"][cycle]))

    def txn(self, cycle, addr_w):
        t = self.txns[self.cur]
        self.cur += 1
        if int(t["cycle"]) // 2 != cycle:
            raise WitgenError("txn cycle mismatch")
        if int(t["addr"]) != dec(addr_w):
            raise WitgenError("memory peek not in preflight")
        pw, w = int(t["prevWord"]), int(t["word"])
        return enc(int(t["prevCycle"])), enc(pw & 0xFFFF), enc(pw >> 16), enc(w & 0xFFFF), enc(w >> 16)

    def lookup_delta(self, cycle, tab_w, idx_w):  # tables.h:33-53 (the count is not used)
        tab, idx = dec(tab_w), dec(idx_w)
        if tab == 0:
            return
        if tab not in (8, 16):
            raise WitgenError("Invalid lookup table")
        if idx >= (1 << tab):
            raise WitgenError("u8/16 table error")
        (self.u8 if tab == 8 else self.u16)[idx] += 1

    def lookup_current(self, tab_w, idx_w):
        tab, idx = dec(tab_w), dec(idx_w)
        if tab not in (8, 16):
            raise WitgenError("Invalid lookup table")
        return enc(int((self.u8 if tab == 8 else self.u16)[idx]))

    def diff_count(self, cyc_w):
        c = dec(cyc_w)
        return enc(int(self.cycles["diffCount"][c // 2][c % 2]))

    def divide(self, nl, nh, dl, dh, s):
        q, r = divide_rv32im(dec(nl) | (dec(nh) << 16), dec(dl) | (dec(dh) << 16), dec(s))
        return enc(q & 0xFFFF), enc(q >> 16), enc(r & 0xFFFF), enc(r >> 16)

    def host_word(self, cycle):
        return enc(int(self.txns[self.cur]["word"]))

    def paging(self, cycle):
        return enc(int(self.cycles["pagingIdx"][cycle])), enc(int(self.cycles["machineMode"][cycle]))

    def bigint(self, cycle):
        i = int(self.cycles["bigintIdx"][cycle])
        if i + 16 > len(self.bigint_bytes):
            raise WitgenError("bigint bytes past the preflight's")
        return tuple(enc(int(b)) for b in self.bigint_bytes[i:i + 16])


def witgen(data, glob, cycles, txns, rows, bigint=None):
    """In place on data (DATA x rows) and glob: the IR over every cycle in forward order
    (rows = the trace length, a power of two)."""
    step, _ = step_fn()
    ctx = Ctx(data, glob, rows, cycles, txns, bigint)
    for c in range(rows):
        step(ctx, c)
    return data, glob
