#!/usr/bin/env python3
"""Flatten the rv32im circuit's witness-generation step (stepExec -> step_Top in the
reference's rv32im-sys/kernels/cxx/steps.cpp, driven by risc0_circuit_rv32im_cpu_witgen,
rv32im-sys/kernels/cxx/ffi.cpp:230-308) into a branchy block IR that
tools/gen_rv32im_witgen.py compiles to gfx950 kernels. Run where the reference tree lives
(it reads the generated C++ as text); the output is committed circuit data:
risc0_amd/circuits/rv32im.witgen.ir and rv32im.witgen.json (the layout offsets the
injector and the tests need).

The front end is the zirgen-C++ evaluator of tools/gen_rv32im_accum_ir.py (layouts,
inlined calls, structs, map/reduce, FpExt lowered to four Fp), with the differences the
witness generator needs:
  * a mux `if (to_size_t(s0)) {..} else if ..` stays a branch: its arms call externs with
    side effects (getMemoryTxn advances the cycle's transaction cursor, lookupDelta counts
    table entries), so only the taken arm may run. Values the arms assign and that are used
    after the mux become phi registers (`m`, assigned with `a` at the end of each arm);
  * common subexpressions are shared only within the branch that defined them;
  * the checks stay: EQZ failures, checked reads of unset words and inconsistent re-stores
    (the reference's Buffer<checked=true>, rv32im-sys/kernels/cxx/buffers.h:30-55), the
    unreachable mux arm, and the externs' own checks all raise errors like the reference's
    throws;
  * the externs of ffi.cpp:84-228 become IR ops; memoryDelta, log, assert and print do
    nothing in the reference and are dropped.

IR (one statement per line; buffers: data (col, back) and global (index)):
  s K TEXT                 message K (EQZ locations)
  c ID VALUE               constant (plain integer; emitted first)
  l ID COL BACK            data[COL][(cycle - BACK) mod rows]   (checked read)
  g ID IDX                 global[IDX]                           (checked read)
  + - * ID A B | n ID A | i ID A (inverse, inv(0) = 0) | z ID A (isz) | and ID A B
  mod ID A B | inr ID LO MID HI
  m ID                     phi register, 0 until assigned
  a ID SRC                 phi ID = SRC
  if ID [major K | minor M] / else / end
                                   branch on xID != 0; `major K` tags the arms of Top's
                                   instruction mux (majorOnehot), `minor M` those of an arm's
                                   minor mux (minorOnehot)
  w COL ID                 data store at this cycle (checked set)
  gw IDX ID                global store (checked set)
  eqz ID K                 error unless xID == 0 (message K)
  unreachable              "Reached unreachable mux arm"
  first ID | mm MAJ MIN | txn PC OLO OHI NLO NHI ADDR | lkd TAB IDX CNT | lkc ID TAB IDX
  dc ID CYC | div Q0 Q1 R0 R1 NL NH DL DH SIGN | hrp ID FP LEN | hw ID FD AL AH LEN
  npi IDX MODE | bi B0 .. B15      the externs (ffi.cpp:84-228)

  gen_rv32im_witgen_ir.py [REFERENCE_ROOT]
"""
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_rv32im_accum_ir as A  # noqa: E402  (tokenizer, layouts, parser, FpExt helpers)

P = A.P
SRC = A.SRC
ROOT = os.path.join(HERE, "..")

MULTI_EXTERNS = {"getMemoryTxn": ("txn", 5), "divide": ("div", 4), "nextPagingIdx": ("npi", 2),
                 "bigIntExtern": ("bi", 16), "getMajorMinor": ("mm", 2)}
VALUE_EXTERNS = {"isFirstCycle_0": "first", "lookupCurrent": "lkc", "getDiffCount": "dc",
                 "hostReadPrepare": "hrp", "hostWrite": "hw"}
NOOP_EXTERNS = {"memoryDelta", "log", "assert", "print"}
PURE = {"+", "-", "*", "n", "i", "z", "and", "mod", "inr"}


class IR:
    """ops with branch-scoped common-subexpression sharing"""

    def __init__(self):
        self.ops = []
        self.n = 0
        self.consts = {}   # value -> id
        self.cval_of = {}  # id -> value
        self.memo = [{}]
        self.strings = []
        self.str_idx = {}

    def fresh(self):
        self.n += 1
        return A.V(self.n)

    def new(self, op, *args):
        key = (op,) + args
        if op in PURE:
            for m in reversed(self.memo):
                if key in m:
                    return m[key]
        v = self.fresh()
        self.ops.append((op, v) + args)
        if op in PURE:
            self.memo[-1][key] = v
        return v

    def emit(self, *op):
        self.ops.append(op)

    def const(self, v):
        v %= P
        if v not in self.consts:
            x = self.fresh()
            self.consts[v] = x
            self.cval_of[x] = v
        return self.consts[v]

    def cval(self, x):
        return self.cval_of.get(x)

    def msg(self, s):
        if s not in self.str_idx:
            self.str_idx[s] = len(self.strings)
            self.strings.append(s)
        return self.str_idx[s]


class Ctx(A.Ctx):
    def __init__(self, funcs, lay):
        self.funcs = funcs
        self.lay = lay
        self.split = None
        self.ir = IR()
        self.stored = [{}]  # (buf, col) -> id, scoped like the branches
        self.guard = []
        self._cv = {}

    def cv(self, x):
        return self.ir.cval(x) if isinstance(x, A.V) else None

    def push(self):
        self.ir.memo.append({})
        self.stored.append({})

    def pop(self):
        self.ir.memo.pop()
        self.stored.pop()

    def fwd(self, key):
        for s in reversed(self.stored):
            if key in s:
                return s[key]
        return None

    def load(self, bl, back, ext):
        buf, node = bl
        assert isinstance(node, int), node
        out = []
        for w in range(4 if ext else 1):
            col = node + w
            if buf == "global":
                assert back == 0
                v = self.fwd(("global", col))
                out.append(v if v is not None else self.ir.new("g", col))
                continue
            assert buf == "data", buf
            v = self.fwd(("data", col)) if back == 0 else None
            out.append(v if v is not None else self.ir.new("l", col, back))
        return A.Fe(out) if ext else out[0]

    def store(self, bl, val, ext):
        buf, node = bl
        assert isinstance(node, int) and buf in ("data", "global"), (buf, node)
        vals = self.ext(val).c if ext else (val,)
        for w, v in enumerate(vals):
            if type(v) is int:
                v = self.c(v)
            self.ir.emit("w" if buf == "data" else "gw", node + w, v)
            self.stored[-1][(buf, node + w)] = v

    # constant folding of constant operands (indices like inner[x4 + 16] inside map lambdas)
    def add(self, a, b):
        ca, cb = self.cv(a), self.cv(b)
        if ca is not None and cb is not None:
            return self.c(ca + cb)
        return super().add(a, b)

    def sub(self, a, b):
        ca, cb = self.cv(a), self.cv(b)
        if ca is not None and cb is not None:
            return self.c(ca - cb)
        return super().sub(a, b)

    def mul(self, a, b):
        ca, cb = self.cv(a), self.cv(b)
        if ca is not None and cb is not None:
            return self.c(ca * cb)
        return super().mul(a, b)

    def neg(self, a):
        ca = self.cv(a)
        if ca is not None:
            return self.c(-ca)
        return super().neg(a)

    def isz(self, a):
        ca = self.cv(a)
        if ca is not None:
            return self.c(1 if ca == 0 else 0)
        return self.ir.new("z", a)


class Ev(A.Ev):
    def __init__(self, ctx):
        super().__init__(ctx)
        self.fn_stack = []

    def call(self, f, vals):
        self.fn_stack.append(f.name)
        try:
            return super().call(f, vals)
        finally:
            self.fn_stack.pop()

    def scalar(self, v):
        return self.x.c(v) if type(v) is int else v

    # ---- statements
    def stmt(self, t, k, env):
        x = self.x
        if t[k] == "EQZ":
            assert t[k + 1] == "("
            v, k2 = self.expr(t, k + 2, env)
            assert t[k2] == ","
            msg = t[k2 + 1]
            assert msg.startswith('"') and t[k2 + 2] == ")" and t[k2 + 3] == ";", t[k2:k2 + 4]
            m = x.ir.msg(msg[1:-1])
            for e in (v.c if isinstance(v, A.Fe) else (v,)):
                e = self.scalar(e)
                if x.cv(e) == 0:
                    continue
                x.ir.emit("eqz", e, m)
            return k2 + 4
        if t[k] == "assert":
            # only in the unreachable arm of a mux: handled by mux()
            return self.skip_call(t, k) + 1
        if t[k] == "INVOKE_EXTERN":
            name = t[k + 4]
            assert t[k + 1:k + 4] == ["(", "ctx", ","], t[k:k + 6]
            if name in NOOP_EXTERNS:
                return self.skip_call(t, k) + 1
            assert name == "lookupDelta", name
            (tab, idx, cnt), k2 = self.args(t, k + 6, env) if t[k + 5] == "," else (None, None)
            assert t[k2] == ";"
            x.ir.emit("lkd", self.scalar(tab), self.scalar(idx), self.scalar(cnt))
            return k2 + 1
        if t[k] == "auto" and t[k + 1] == "[":
            j = k + 2
            names = []
            while t[j] != "]":
                if t[j] != ",":
                    names.append(t[j])
                j += 1
            assert t[j + 1] == "=" and t[j + 2] == "INVOKE_EXTERN", t[j:j + 5]
            name = t[j + 6]
            op, nout = MULTI_EXTERNS[name]
            assert len(names) == nout, (name, names)
            if t[j + 7] == ",":
                args, k2 = self.args(t, j + 8, env)
            else:
                assert t[j + 7] == ")"
                args, k2 = [], j + 8
            assert t[k2] == ";"
            outs = [x.ir.fresh() for _ in range(nout)]
            x.ir.emit(op, *outs, *[self.scalar(a) for a in args])
            for nm, o in zip(names, outs):
                env[nm] = o
            return k2 + 1
        return super().stmt(t, k, env)

    def mux(self, t, k, env):
        x = self.x
        arms = []
        has_else = False
        k0 = k
        while True:
            assert t[k] == "if" and t[k + 1] == "("
            sel, k = self.expr(t, k + 2, env)
            assert t[k] == ")" and t[k + 1] == "{"
            start = k + 2
            k = self.skip_block(t, start)
            arms.append((self.scalar(sel), start))
            if t[k] == "else" and t[k + 1] == "if":
                k += 1
                continue
            if t[k] == "else":
                assert t[k + 1] == "{"
                body = t[k + 2:self.skip_block(t, k + 2) - 1]
                assert body[:1] == ["assert"] and "0" in body[:4], body[:8]
                has_else = True
                k = self.skip_block(t, k + 2)
            break
        tag = self.fn_stack and self.fn_stack[-1] == "exec_Top" and len(arms) == 13
        # an arm's minor mux (`if (to_size_t(....minorOnehot._super[0]._super))` ...): tagged so
        # the kernel generator can specialise it as it does Top's major mux
        minor = not tag and "minorOnehot" in t[k0:k0 + 12]
        outer = dict(env)
        start_pos = len(x.ir.ops)
        phis = {}     # name -> phi structure
        m_ops = []
        depth = 0
        for ai, (sel, start) in enumerate(arms):
            if ai:
                x.ir.emit("else")
            x.ir.emit(*(("if", sel, "major", ai) if tag else ("if", sel, "minor", ai) if minor else ("if", sel)))
            depth += 1
            x.push()
            arm_env = dict(outer)
            self.block(t, start, arm_env)
            for name in outer:
                v = arm_env[name]
                if v is outer[name]:
                    continue
                if name not in phis:
                    phis[name] = self.phi_like(v, m_ops)
                self.assign(phis[name], v)
            x.pop()
        if has_else:
            x.ir.emit("else")
            x.ir.emit("unreachable")
        for _ in range(depth):
            x.ir.emit("end")
        x.ir.ops[start_pos:start_pos] = m_ops
        for name, ph in phis.items():
            env[name] = ph
        return k

    def phi_like(self, v, m_ops):
        if isinstance(v, dict):
            return {f: self.phi_like(w, m_ops) for f, w in v.items()}
        if isinstance(v, list):
            return [self.phi_like(w, m_ops) for w in v]
        if isinstance(v, tuple) and v and v[0] in ("data", "global"):
            return v  # a bound layout: every arm must bind the same one
        if isinstance(v, A.Fe):
            return A.Fe(self.phi_like(w, m_ops) for w in v.c)
        assert v is None or isinstance(v, (int, A.V)), v
        p = self.x.ir.fresh()
        m_ops.append(("m", p))
        return p

    def assign(self, ph, v):
        if isinstance(ph, dict):
            for f in ph:
                self.assign(ph[f], v[f] if v is not None else None)
        elif isinstance(ph, list):
            for i in range(len(ph)):
                self.assign(ph[i], v[i] if v is not None else None)
        elif isinstance(ph, tuple):
            assert v == ph, (v, ph)
        elif isinstance(ph, A.Fe):
            vv = self.x.ext(v) if v is not None else None
            for i in range(4):
                self.assign(ph.c[i], vv.c[i] if vv is not None else None)
        elif v is not None:
            self.x.ir.emit("a", ph, self.scalar(v))

    # ---- expressions
    def primary(self, t, k, env):
        x = self.x
        tok = t[k]
        if tok == "INVOKE_EXTERN":
            name = t[k + 4]
            op = VALUE_EXTERNS[name]
            if t[k + 5] == ",":
                args, k2 = self.args(t, k + 6, env)
            else:
                assert t[k + 5] == ")"
                args, k2 = [], k + 6
            v = x.ir.fresh()
            x.ir.emit(op, v, *[self.scalar(a) for a in args])
            return v, k2
        if tok == "bitAnd":
            (a, b), k = self.args(t, k + 2, env)
            return x.ir.new("and", *sorted((self.scalar(a), self.scalar(b)))), k
        if tok == "mod":
            (a, b), k = self.args(t, k + 2, env)
            return x.ir.new("mod", self.scalar(a), self.scalar(b)), k
        if tok == "neg_0":
            (a,), k = self.args(t, k + 2, env)
            return x.e_neg(self.scalar(a)), k
        if tok == "reduce":
            args, k = self.args(t, k + 2, env)
            if len(args) == 4:
                arr, acc, lay, fn = args
                for i in range(len(arr)):
                    acc = fn(acc, arr[i], self.index(lay, i))
            else:
                arr, acc, fn = args
                for i in range(len(arr)):
                    acc = fn(acc, arr[i])
            return acc, k
        if tok == "inRange":
            (lo, mid, hi), k = self.args(t, k + 2, env)
            return x.ir.new("inr", self.scalar(lo), self.scalar(mid), self.scalar(hi)), k
        return super().primary(t, k, env)


def dce(ops):
    """drop pure definitions nothing observable needs (loads, stores, checks, externs and
    branches stay)"""
    need = set()
    keep = [False] * len(ops)
    for i in range(len(ops) - 1, -1, -1):
        op = ops[i]
        o = op[0]
        if o in PURE:
            if op[1] in need:
                keep[i] = True
                need.update(a for a in op[2:] if isinstance(a, A.V))
        elif o == "m":
            keep[i] = op[1] in need
        elif o == "a":
            if op[1] in need:
                keep[i] = True
                need.add(op[2])
        else:
            keep[i] = True
            if o == "if":
                need.add(op[1])
            elif o in ("w", "gw"):
                need.add(op[2])
            elif o == "eqz":
                need.add(op[1])
            elif o in ("lkd",):
                need.update(op[1:])
            elif o in ("lkc", "dc", "hrp", "hw"):
                need.update(op[2:])
            elif o == "txn":
                need.add(op[6])
            elif o == "div":
                need.update(op[5:])
    return [op for op, k in zip(ops, keep) if k]


def layout_offsets(lay):
    """the layout columns the host-side injector (witgen/mod.rs:226-378) and the tests use"""
    top = lay.get("kLayout_Top")
    d = lambda v: lay.deref(v)
    leaf = lambda v: d(d(v)["_super"]) if isinstance(d(v), dict) else d(v)
    out = {"cycle": leaf(top["cycle"]), "next_pc_low": leaf(top["nextPcLow"]), "next_pc_high": leaf(top["nextPcHigh"]),
           "next_state_0": leaf(top["nextState_0"]), "next_machine_mode": leaf(top["nextMachineMode"])}
    res = d(top["instResult"])
    arm8 = d(res["arm8"])
    out["ecall_s"] = [leaf(arm8[f]) for f in ("s0", "s1", "s2")]
    st = d(d(res["arm9"])["state"])
    names = ["hasState", "stateAddr", "bufOutAddr", "isElem", "checkOut", "loadTxType", "nextState", "subState",
             "bufInAddr", "count", "mode"]
    p2 = [leaf(st[f]) for f in names] + [leaf(c) for c in d(st["inner"])]
    z = leaf(st["zcheck"])
    out["poseidon2_state"] = p2 + [z, z + 1, z + 2, z + 3]
    sha = d(d(res["arm11"])["state"])  # Sha2State::fp_offsets / u32_offsets (witgen/sha2.rs:28-50)
    out["sha2_fp"] = [leaf(sha[f]) for f in ("stateInAddr", "stateOutAddr", "dataAddr", "count", "kAddr", "round",
                                              "nextState")]
    out["sha2_u32"] = [leaf(d(sha[f])[0]) for f in ("a", "e", "w")]
    bi = d(d(res["arm12"])["state"])  # BigIntState::offsets (witgen/bigint.rs:185-211)
    out["bigint_state"] = [leaf(bi[f]) for f in ("isEcall", "mode", "pc", "polyOp", "coeff")] + \
        [leaf(b) for b in d(bi["bytes"])] + [leaf(bi["nextState"])]
    g = lay.get("kLayoutGlobal")

    def u32s(name):
        vals = d(d(g[name])["values"])
        return [[leaf(d(v)["low"]), leaf(d(v)["high"])] for v in vals]
    out["global"] = {"state_in": u32s("stateIn"), "state_out": u32s("stateOut"), "input": u32s("input"),
                     "output": u32s("output"), "povw_nonce": u32s("povwNonce"), "rng": leaf(g["rng"]),
                     "is_terminate": leaf(g["isTerminate"]), "shutdown_cycle": leaf(g["shutdownCycle"])}
    return out


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    steps = open(f"{ref}/{SRC}steps.cpp").read()
    lay = A.Layouts(open(f"{ref}/{SRC}layout.cpp.inc").read())
    funcs = A.parse_functions(steps)
    ctx = Ctx(funcs, lay)
    ev = Ev(ctx)
    ev.call(funcs["step_Top"], ["data", "global"])
    ops = dce(ctx.ir.ops)
    circ = os.path.join(ROOT, "risc0_amd", "circuits")
    with open(os.path.join(circ, "rv32im.witgen.ir"), "w") as f:
        f.write("# rv32im witness generation step (stepExec -> step_Top) flattened by tools/gen_rv32im_witgen_ir.py\n")
        f.write("# from the reference's rv32im-sys/kernels/cxx/steps.cpp (externs: ffi.cpp:84-228)\n")
        for i, s in enumerate(ctx.ir.strings):
            f.write(f"s {i} {s}\n")
        for v, x in sorted(ctx.ir.consts.items(), key=lambda kv: kv[1]):
            f.write(f"c {x} {v}\n")
        for op in ops:
            f.write(" ".join(str(a) for a in op) + "\n")
    with open(os.path.join(circ, "rv32im.witgen.json"), "w") as f:
        json.dump(layout_offsets(lay), f, indent=1)
    counts = {}
    for op in ops:
        counts[op[0]] = counts.get(op[0], 0) + 1
    print(f"rv32im witgen IR: {len(ops)} ops, {len(ctx.ir.consts)} constants, {len(ctx.ir.strings)} messages; {counts}",
          file=sys.stderr)


if __name__ == "__main__":
    main()
