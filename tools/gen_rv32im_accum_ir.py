#!/usr/bin/env python3
"""Flatten the rv32im circuit's per-cycle accumulation step (phase 1 of
risc0_circuit_rv32im_cpu_accum, rv32im-sys/kernels/cxx/ffi.cpp:238-247 -> step_TopAccum in
steps.cpp) into the block IR tools/gen_accum.py compiles to HIP. Run in the container where
the reference tree lives (reading its generated C++ as text); the output is committed
circuit data: risc0_amd/circuits/rv32im.accum.ir.

The step code is zirgen C++ (28 functions, exec_TopAccum and its callees): values are Val
(Fp) and ExtVal (FpExt) expressions over layout-bound buffer loads, struct values built with
designated initializers, muxes `if (to_size_t(sel)) ... else if ...` whose arms assign
struct values used after the mux, `map` over register arrays, and checks (EQZ,
INVOKE_EXTERN assert, inRange) that do not affect the outputs. This front end evaluates it
symbolically, inlining every call:
  * layouts come from layout.cpp.inc (designated initializers with /*offset=*/ leaves);
  * FpExt is lowered to four Fp values (x^4 = -11);
  * a mux evaluates every arm (pure arithmetic, harmless on any input) and merges the
    values assigned in the arms as sum_k c_k * v_k, where c_k = [arm k is the first arm
    whose selector is nonzero] (isz products, exactly 0 or 1); stores (the only side
    effects) run under `if (c_k != 0)` blocks;
  * a load of a location stored earlier in the same cycle returns the stored value; loads
    of machine accum columns (col >= kUserAccumSplit) at back > 0 read 0, as the
    reference's MutableBufObj(accum, zeroBack) does (ffi.cpp:243);
  * values feeding only checks are dropped (dead-code elimination from the stores), and
    the arms' pure definitions are hoisted out of their `if` blocks (the merged values are
    used after the mux), so the blocks hold only stores.

IR (one statement per line; buffers: 0 data, 1 accum, 2 global, 3 mix):
  c ID VALUE | l ID BUF COL BACK | g ID BUF IDX | + - * ID A B | n ID A | i ID A (inv, 0 -> 0)
  z ID A (1 if A == 0 else 0) | if ID ... end (if A != 0) | w BUF COL ID

  gen_rv32im_accum_ir.py [REFERENCE_ROOT] > risc0_amd/circuits/rv32im.accum.ir
"""
import re
import sys

SRC = "risc0/circuit/rv32im-sys/kernels/cxx/"
P = 15 * 2**27 + 1
NBETA = P - 11
BUFS = {"data": 0, "accum": 1, "global": 2, "mix": 3}

# ---------------------------------------------------------------- tokenizer
TOK = re.compile(r'\s+|//[^\n]*|/\*offset=\*/|/\*.*?\*/|"(?:\\.|[^"\\])*"|\d+|[A-Za-z_]\w*|::|->|==|!=|&&|\|\||<=|>=|.',
                 re.S)


def tokenize(text):
    out = []
    for m in TOK.finditer(text):
        t = m.group(0)
        if t.isspace() or t.startswith("//") or (t.startswith("/*") and t != "/*offset=*/"):
            continue
        out.append(t)
    return out


# ---------------------------------------------------------------- layouts
class Layouts:
    """constexpr T kLayout... = T{.field = value, ...}; leaves /*offset=*/N; array
    initializers positional; references to other kLayout constants."""

    def __init__(self, text):
        self.defs = {}
        for m in re.finditer(r"constexpr\s+\w+\s+(\w+)\s*=\s*(.*?);\s*(?=constexpr|$)", text, re.S):
            self.defs[m.group(1)] = m.group(2)
        self.cache = {}

    def get(self, name):
        if name not in self.cache:
            toks = tokenize(self.defs[name])
            v, k = self._value(toks, 0)
            assert k == len(toks), name
            self.cache[name] = v
        return self.cache[name]

    def _value(self, t, k):
        if t[k] == "/*offset=*/":
            return int(t[k + 1]), k + 2
        if t[k].startswith("kLayout"):
            return ("ref", t[k]), k + 1
        # Type{...}
        assert re.match(r"[A-Za-z_]\w*$", t[k]) and t[k + 1] == "{", t[k:k + 5]
        k += 2
        if t[k] == "}":
            return {}, k + 1
        if t[k] == ".":
            d = {}
            while True:
                assert t[k] == "."
                f = t[k + 1]
                assert t[k + 2] == "="
                v, k = self._value(t, k + 3)
                d[f] = v
                if t[k] == ",":
                    k += 1
                    continue
                assert t[k] == "}"
                return d, k + 1
        lst = []
        while True:
            v, k = self._value(t, k)
            lst.append(v)
            if t[k] == ",":
                k += 1
                continue
            assert t[k] == "}"
            return lst, k + 1

    def deref(self, v):
        while isinstance(v, tuple) and v[0] == "ref":
            v = self.get(v[1])
        return v


# ---------------------------------------------------------------- IR builder
class V(int):
    """an IR value id (literal integers of the source stay plain int)"""


class IR:
    def __init__(self):
        self.ops = []     # (op, id, args...) | ("if", id) | ("end",) | ("w", buf, col, id)
        self.n = 0
        self.consts = {}
        self.memo = {}

    def new(self, op, *args):
        key = (op,) + args
        if op != "l" and key in self.memo:
            return self.memo[key]
        self.n += 1
        self.ops.append((op, self.n) + args)
        v = V(self.n)
        self.memo[key] = v
        return v

    def const(self, v):
        v %= P
        if v not in self.consts:
            self.n += 1
            self.ops.append(("c", self.n, v))
            self.consts[v] = V(self.n)
        return self.consts[v]

    def cval(self, x):
        for op in self.ops:
            if op[0] == "c" and op[1] == x:
                return op[2]
        return None


class Fe:  # FpExt as four Fp ids
    __slots__ = ("c",)

    def __init__(self, c):
        self.c = tuple(c)


class Ctx:
    """symbolic evaluation of the step code of one cycle"""

    def __init__(self, funcs, lay, split):
        self.funcs = funcs
        self.lay = lay
        self.split = split
        self.ir = IR()
        self.stored = {}   # (buf, col) -> id (this cycle)
        self.guard = []    # condition ids of enclosing muxes (stores run under them)
        self._cv = {}

    # -- scalar helpers (constant-folding the obvious cases keeps the IR small)
    def cv(self, x):
        if x not in self._cv:
            self._cv[x] = self.ir.cval(x)
        return self._cv[x]

    def c(self, v):
        return self.ir.const(v)

    def add(self, a, b):
        if self.cv(a) == 0:
            return b
        if self.cv(b) == 0:
            return a
        return self.ir.new("+", *sorted((a, b)))

    def sub(self, a, b):
        if self.cv(b) == 0:
            return a
        return self.ir.new("-", a, b)

    def mul(self, a, b):
        ca, cb = self.cv(a), self.cv(b)
        if ca == 0 or cb == 0:
            return self.c(0)
        if ca == 1:
            return b
        if cb == 1:
            return a
        return self.ir.new("*", *sorted((a, b)))

    def neg(self, a):
        return self.ir.new("n", a)

    def isz(self, a):
        ca = self.cv(a)
        if ca is not None:
            return self.c(1 if ca == 0 else 0)
        return self.ir.new("z", a)

    def inv(self, a):
        return self.ir.new("i", a)

    # -- FpExt
    def ext(self, v):
        return v if isinstance(v, Fe) else Fe((v, self.c(0), self.c(0), self.c(0)))

    def e_add(self, a, b):
        if not isinstance(a, Fe) and not isinstance(b, Fe):
            return self.add(a, b)
        a, b = self.ext(a), self.ext(b)
        return Fe(self.add(x, y) for x, y in zip(a.c, b.c))

    def e_sub(self, a, b):
        if not isinstance(a, Fe) and not isinstance(b, Fe):
            return self.sub(a, b)
        a, b = self.ext(a), self.ext(b)
        return Fe(self.sub(x, y) for x, y in zip(a.c, b.c))

    def e_mul(self, a, b):
        if not isinstance(a, Fe) and not isinstance(b, Fe):
            return self.mul(a, b)
        if not isinstance(a, Fe):
            return Fe(self.mul(a, y) for y in b.c)
        if not isinstance(b, Fe):
            return Fe(self.mul(x, b) for x in a.c)
        r = [self.c(0)] * 4
        nb = self.c(NBETA)
        for i in range(4):
            for j in range(4):
                t = self.mul(a.c[i], b.c[j])
                if i + j >= 4:
                    r[i + j - 4] = self.add(r[i + j - 4], self.mul(nb, t))
                else:
                    r[i + j] = self.add(r[i + j], t)
        return Fe(r)

    def e_neg(self, a):
        if isinstance(a, Fe):
            return Fe(self.neg(x) for x in a.c)
        return self.neg(a)

    def e_inv(self, a):
        if not isinstance(a, Fe):
            return self.inv(a)
        # baby_bear.rs:448-481 (ExtElem::inv), with inv(0) = 0 giving inv_0(0) = 0
        a0, a1, a2, a3 = a.c
        beta = self.c(11)
        b0 = self.add(self.mul(a0, a0), self.mul(beta, self.sub(self.mul(a1, self.add(a3, a3)), self.mul(a2, a2))))
        b2 = self.add(self.sub(self.mul(a0, self.add(a2, a2)), self.mul(a1, a1)), self.mul(beta, self.mul(a3, a3)))
        cc = self.add(self.mul(b0, b0), self.mul(beta, self.mul(b2, b2)))
        ic = self.inv(cc)
        b0, b2 = self.mul(b0, ic), self.mul(b2, ic)
        nbeta = self.c(NBETA)
        return Fe((self.add(self.mul(a0, b0), self.mul(beta, self.mul(a2, b2))),
                   self.add(self.neg(self.mul(a1, b0)), self.mul(nbeta, self.mul(a3, b2))),
                   self.add(self.neg(self.mul(a0, b2)), self.mul(a2, b0)),
                   self.sub(self.mul(a1, b2), self.mul(a3, b0))))

    # -- memory
    def load(self, bl, back, ext):
        buf, node = bl
        assert isinstance(node, int), node
        words = 4 if ext else 1
        out = []
        for w in range(words):
            col = node + w
            if buf in ("global", "mix"):
                assert back == 0
                out.append(self.ir.new("g", BUFS[buf], col))
                continue
            if back == 0 and (buf, col) in self.stored:
                out.append(self.stored[(buf, col)])
                continue
            if buf == "accum" and back > 0 and col >= self.split:
                out.append(self.c(0))  # MutableBufObj zeroBack (ffi.cpp:243)
                continue
            if buf == "accum" and back == 0:
                raise ValueError(f"read of accum column {col} before it is set this cycle")
            out.append(self.ir.new("l", BUFS[buf], col, back))
        return Fe(out) if ext else out[0]

    def store(self, bl, val, ext):
        buf, node = bl
        assert isinstance(node, int) and buf in ("accum", "data"), (buf, node)
        vals = self.ext(val).c if ext else (val,)
        for w, v in enumerate(vals):
            self.ir.ops.append(("w", BUFS[buf], node + w, v))
            self.stored[(buf, node + w)] = v


# ---------------------------------------------------------------- step-code parser
class Fn:
    def __init__(self, name, params, body):
        self.name, self.params, self.body = name, params, body


def parse_functions(text):
    funcs = {}
    for m in re.finditer(r"^(\w[\w<>:, ]*?)\s+(\w+)\(ExecContext& ctx,?([^)]*)\)\s*\{", text, re.M):
        name = m.group(2)
        params = []
        for p in m.group(3).split(","):
            p = p.strip()
            if p:
                params.append(p.split()[-1])
        # body: brace matching from the opening brace
        k = m.end()
        depth = 1
        i = k
        while depth:
            ch = text[i]
            if ch == "{":
                depth += 1
            elif ch == "}":
                depth -= 1
            elif ch == '"':
                i += 1
                while text[i] != '"':
                    i += 2 if text[i] == "\\" else 1
            i += 1
        funcs[name] = Fn(name, params, tokenize(text[k:i - 1]))
    return funcs


class Return(Exception):
    def __init__(self, v):
        self.v = v


class Ev:
    """evaluates token streams of statements/expressions in a Ctx"""

    def __init__(self, ctx):
        self.x = ctx

    # ---- statements
    def block(self, t, k, env):
        """statements until the matching '}' (t[k-1] == '{'); returns index after '}'"""
        while t[k] != "}":
            k = self.stmt(t, k, env)
        return k + 1

    def stmt(self, t, k, env):
        x = self.x
        if t[k] == "if":
            return self.mux(t, k, env)
        if t[k] == "return":
            if t[k + 1] == ";":
                raise Return(None)
            v, k = self.expr(t, k + 1, env)
            assert t[k] == ";"
            raise Return(v)
        if t[k] in ("EQZ", "assert", "INVOKE_EXTERN"):
            return self.skip_call(t, k) + 1
        if t[k] in ("STORE", "STORE_EXT"):
            ext = t[k] == "STORE_EXT"
            assert t[k + 1] == "("
            bl, k = self.expr(t, k + 2, env)
            assert t[k] == ","
            v, k = self.expr(t, k + 1, env)
            assert t[k] == ")" and t[k + 1] == ";"
            x.store(bl, v, ext)
            return k + 2
        # assignment xN = expr;
        if re.match(r"x\d+$", t[k]) and t[k + 1] == "=":
            v, k2 = self.expr(t, k + 2, env)
            assert t[k2] == ";"
            env[t[k]] = v
            return k2 + 1
        # declaration: TYPE ... NAME (= expr)? ;
        j = k
        depth = 0
        while True:
            if t[j] == "<":
                depth += 1
            elif t[j] == ">":
                depth -= 1
            elif depth == 0 and re.match(r"x\d+$", t[j]) and t[j + 1] in ("=", ";"):
                break
            j += 1
            assert j - k < 40, t[k:k + 20]
        name = t[j]
        if t[j + 1] == ";":
            env[name] = None
            return j + 2
        v, k2 = self.expr(t, j + 2, env)
        assert t[k2] == ";", t[k2 - 3:k2 + 3]
        env[name] = v
        return k2 + 1

    def skip_call(self, t, k):
        """index of the ';' after NAME(...)"""
        assert t[k + 1] == "("
        depth = 0
        j = k + 1
        while True:
            if t[j] == "(":
                depth += 1
            elif t[j] == ")":
                depth -= 1
                if depth == 0:
                    break
            j += 1
        assert t[j + 1] == ";"
        return j + 1

    def mux(self, t, k, env):
        """if (to_size_t(s0)) {A0} else if (to_size_t(s1)) {A1} ... [else {unreachable}]"""
        x = self.x
        arms = []  # (selector id, token index of the block start)
        while True:
            assert t[k] == "if" and t[k + 1] == "("
            sel, k = self.expr(t, k + 2, env)
            assert t[k] == ")" and t[k + 1] == "{"
            start = k + 2
            k = self.skip_block(t, start)
            arms.append((sel, start))
            if t[k] == "else" and t[k + 1] == "if":
                k += 1
                continue
            if t[k] == "else":
                assert t[k + 1] == "{"
                k = self.skip_block(t, k + 2)  # the unreachable arm: nothing to evaluate
            break
        # condition of arm i: all earlier selectors zero, this one nonzero (0 or 1 each)
        conds = []
        none_before = None
        for sel, _ in arms:
            nz = x.isz(x.isz(sel))  # 1 if sel != 0
            c = nz if none_before is None else x.mul(none_before, nz)
            conds.append(c)
            z = x.isz(sel)
            none_before = z if none_before is None else x.mul(none_before, z)
        outer = dict(env)
        results = []
        for (sel, start), c in zip(arms, conds):
            if x.cv(c) == 0:
                continue
            arm_env = dict(outer)
            saved = dict(x.stored)
            x.ir.ops.append(("if", c))
            x.guard.append(c)
            self.block(t, start, arm_env)
            x.guard.pop()
            x.ir.ops.append(("end",))
            x.stored = saved  # stores made under the arm are not visible unconditionally
            results.append((c, arm_env))
        # merge the outer variables the arms assigned
        for name in outer:
            vals = [(c, e[name]) for c, e in results if e[name] is not outer[name]]
            if not vals:
                continue
            env[name] = self.merge([(c, e[name]) for c, e in results], outer[name])
        return k

    def merge(self, vals, old):
        x = self.x
        v0 = next(v for _, v in vals if v is not None) if any(v is not None for _, v in vals) else old
        if isinstance(v0, dict):
            return {f: self.merge([(c, (v or {}).get(f)) for c, v in vals], (old or {}).get(f) if isinstance(old, dict) else None)
                    for f in v0}
        if isinstance(v0, list):
            return [self.merge([(c, v[i] if v is not None else None) for c, v in vals],
                               old[i] if isinstance(old, list) else None) for i in range(len(v0))]
        if isinstance(v0, tuple) and v0 and v0[0] in BUFS:  # a bound layout: must agree
            return v0
        acc = None
        for c, v in vals:
            if v is None:
                continue
            term = x.e_mul(c, v)
            acc = term if acc is None else x.e_add(acc, term)
        return acc

    def skip_block(self, t, k):
        depth = 1
        while depth:
            if t[k] == "{":
                depth += 1
            elif t[k] == "}":
                depth -= 1
            k += 1
        return k

    # ---- expressions (precedence: postfix > unary > * > + -)
    def expr(self, t, k, env):
        a, k = self.term(t, k, env)
        while t[k] in ("+", "-"):
            op = t[k]
            b, k = self.term(t, k + 1, env)
            a = self.x.e_add(a, b) if op == "+" else self.x.e_sub(a, b)
        return a, k

    def term(self, t, k, env):
        a, k = self.unary(t, k, env)
        while t[k] == "*":
            b, k = self.unary(t, k + 1, env)
            a = self.x.e_mul(a, b)
        return a, k

    def unary(self, t, k, env):
        if t[k] == "-":
            a, k = self.unary(t, k + 1, env)
            return self.x.e_neg(a), k
        return self.postfix(t, k, env)

    def postfix(self, t, k, env):
        v, k = self.primary(t, k, env)
        while True:
            if t[k] == "." and re.match(r"[A-Za-z_]\w*$", t[k + 1]):
                v = self.field(v, t[k + 1])
                k += 2
            elif t[k] == "[":
                i, k = self.expr(t, k + 1, env)
                assert t[k] == "]"
                k += 1
                v = self.index(v, i)
            else:
                return v, k

    def field(self, v, f):
        if isinstance(v, tuple) and v[0] in BUFS:  # bound layout
            node = self.x.lay.deref(v[1])
            return (v[0], self.x.lay.deref(node[f]))
        return v[f]

    def index(self, v, i):
        i = self.intval(i)
        if isinstance(v, tuple) and v[0] in BUFS:
            node = self.x.lay.deref(v[1])
            return (v[0], self.x.lay.deref(node[i]))
        return v[i]

    def intval(self, i):
        if type(i) is int:
            return i
        c = self.x.cv(i)
        assert c is not None, i
        return c

    def args(self, t, k, env):
        """comma-separated expressions up to ')' (t[k-1] == '(')"""
        out = []
        if t[k] == ")":
            return out, k + 1
        while True:
            v, k = self.expr(t, k, env)
            out.append(v)
            if t[k] == ",":
                k += 1
                continue
            assert t[k] == ")", t[k - 5:k + 5]
            return out, k + 1

    def path(self, t, k):
        """a member path a.b.c up to the closing ')' of LAYOUT_LOOKUP"""
        parts = []
        while t[k] != ")":
            if t[k] != ".":
                parts.append(t[k])
            k += 1
        return parts, k + 1

    def primary(self, t, k, env):
        x = self.x
        tok = t[k]
        if tok == "(":
            if t[k + 1] == "[":
                return self.lambda_(t, k + 1, env)
            v, k = self.expr(t, k + 1, env)
            assert t[k] == ")"
            return v, k + 1
        if tok.isdigit():
            return int(tok), k + 1
        if tok == "LAYOUT_LOOKUP":
            bl, k = self.expr(t, k + 2, env)
            assert t[k] == ","
            parts, k = self.path(t, k + 1)
            for f in parts:
                bl = self.field(bl, f)
            return bl, k
        if tok == "LAYOUT_SUBSCRIPT":
            bl, k = self.expr(t, k + 2, env)
            assert t[k] == ","
            i, k = self.expr(t, k + 1, env)
            assert t[k] == ")"
            return self.index(bl, i), k + 1
        if tok == "BIND_LAYOUT":
            name = t[k + 2]
            assert t[k + 3] == ","
            buf = env[t[k + 4]]
            assert t[k + 5] == ")"
            return (buf, self.x.lay.get(name)), k + 6
        if tok in ("LOAD", "LOAD_EXT"):
            (bl, back), k = self.args(t, k + 2, env)
            return x.load(bl, self.intval(back), tok == "LOAD_EXT"), k
        if tok == "Val" and t[k + 1] == "(":
            (v,), k = self.args(t, k + 2, env)
            return x.c(self.intval(v)), k
        if tok == "ExtVal" and t[k + 1] == "(":
            vs, k = self.args(t, k + 2, env)
            vs = [x.c(v) if type(v) is int else v for v in vs]
            return Fe(vs + [x.c(0)] * (4 - len(vs))), k
        if tok == "inv_0":
            (v,), k = self.args(t, k + 2, env)
            return x.e_inv(v), k
        if tok == "isz":
            (v,), k = self.args(t, k + 2, env)
            assert not isinstance(v, Fe)
            return x.isz(v), k
        if tok == "to_size_t":
            (v,), k = self.args(t, k + 2, env)
            return v, k
        if tok == "inRange":
            # feeds only range checks (INVOKE_EXTERN assert), dropped by dead-code elimination
            _, k = self.args(t, k + 2, env)
            return x.c(1), k
        if tok == "map":
            (arr, lay, fn), k = self.args(t, k + 2, env)
            n = len(arr) if isinstance(arr, list) else len(self.x.lay.deref(lay[1]))
            return [fn(arr[i], self.index(lay, i)) for i in range(n)], k
        if tok in self.x.funcs and t[k + 1] == "(" and t[k + 2] == "ctx":
            f = self.x.funcs[tok]
            vals, k = self.args(t, k + 4, env) if t[k + 3] == "," else ([], k + 4)
            return self.call(f, vals), k
        if re.match(r"[A-Za-z_]\w*$", tok) and t[k + 1] == "{":
            return self.init(t, k + 2, env)
        if tok in env:
            return env[tok], k + 1
        raise ValueError(f"unknown token {tok!r} near {' '.join(t[k - 5:k + 8])}")

    def init(self, t, k, env):
        """Type{.f = e, ...} -> dict; Type{e, ...} -> list (t[k-1] == '{')"""
        if t[k] == "}":
            return {}, k + 1
        if t[k] == "." and t[k + 2] == "=":
            d = {}
            while True:
                f = t[k + 1]
                v, k = self.expr(t, k + 3, env)
                d[f] = v
                if t[k] == ",":
                    k += 1
                    continue
                assert t[k] == "}"
                return d, k + 1
        lst = []
        while True:
            v, k = self.expr(t, k, env)
            lst.append(self.x.c(v) if type(v) is int else v)
            if t[k] == ",":
                k += 1
                continue
            assert t[k] == "}"
            return lst, k + 1

    def lambda_(self, t, k, env):
        """([&](T a, T b) { body }) starting at '['; returns a Python callable"""
        assert t[k:k + 4] == ["[", "&", "]", "("]
        k += 4
        params = []
        depth = 0
        cur = []
        while True:
            if t[k] == "<":
                depth += 1
            elif t[k] == ">":
                depth -= 1
            if depth == 0 and t[k] in (",", ")"):
                params.append(cur[-1])
                cur = []
                if t[k] == ")":
                    break
            else:
                cur.append(t[k])
            k += 1
        assert t[k + 1] == "{"
        start = k + 2
        end = self.skip_block(t, start)
        assert t[end] == ")"
        outer = env

        def fn(*vals):
            e = dict(outer)
            e.update(zip(params, vals))
            try:
                self.block(t, start, e)
            except Return as r:
                return r.v
            return None
        return fn, end + 1

    def call(self, f, vals):
        env = dict(zip(f.params, vals))
        try:
            self.block(f.body + ["}"], 0, env)
        except Return as r:
            return r.v
        return None


# ---------------------------------------------------------------- driver
def dce(ops):
    """keep what the stores and their guards need"""
    need = set()
    keep = [False] * len(ops)
    for i in range(len(ops) - 1, -1, -1):
        op = ops[i]
        if op[0] == "w":
            keep[i] = True
            need.add(op[3])
        elif op[0] == "if":
            keep[i] = True
            need.add(op[1])
        elif op[0] == "end":
            keep[i] = True
        elif op[1] in need:
            keep[i] = True
            for a in op[2:]:
                if op[0] in ("+", "-", "*", "n", "i", "z"):
                    need.add(a)
    out = [op for op, k in zip(ops, keep) if k]
    # drop empty if-blocks
    res = []
    for op in out:
        if op[0] == "end" and res and res[-1][0] == "if":
            res.pop()
            continue
        res.append(op)
    return res


def hoist(ops):
    """move every pure definition made inside a mux arm in front of the arm's outermost
    `if` (order kept): arm values are merged after the mux, so they must be in scope
    there; only the stores stay guarded"""
    out, held, depth, pos = [], [], 0, 0
    for op in ops:
        if op[0] == "if":
            if depth == 0:
                pos = len(out)
            depth += 1
            out.append(op)
        elif op[0] == "end":
            depth -= 1
            out.append(op)
            if depth == 0 and held:
                out[pos:pos] = held
                held = []
        elif op[0] == "w" or depth == 0:
            out.append(op)
        else:
            held.append(op)
    return out


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    steps = open(f"{ref}/{SRC}steps.cpp").read()
    lay = Layouts(open(f"{ref}/{SRC}layout.cpp.inc").read())
    top_accum = lay.get("kLayout_TopAccum")
    split = lay.deref(top_accum["columns"])[0]  # kUserAccumSplit (ffi.cpp:52)
    funcs = parse_functions(steps)
    ctx = Ctx(funcs, lay, split)
    ev = Ev(ctx)
    ev.call(funcs["step_TopAccum"], ["accum", "data", "global", "mix"])
    ops = dce(hoist(ctx.ir.ops))
    print("# rv32im accumulation step (phase 1) flattened by tools/gen_rv32im_accum_ir.py from the reference's")
    print("# rv32im-sys/kernels/cxx/steps.cpp step_TopAccum; buffers 0 data, 1 accum, 2 global, 3 mix")
    print(f"# kUserAccumSplit {split}")
    print("fn compute")
    for op in ops:
        print(" ".join(str(a) for a in op))


if __name__ == "__main__":
    main()
