#!/usr/bin/env python3
"""Flatten a circuit's constraint polynomial into a compact SSA "constraint program".

Input : the reference's generated C++ `poly_fp` (a call tree of ~20 straight-line
        functions sharing constant-indexed arrays):
          rv32im    risc0/circuit/rv32im-sys/kernels/cxx/rust_poly_fp_{0..3}.cpp
          recursion risc0/circuit/recursion-sys/kernels/cxx/poly_fp.cpp
Output: risc0_amd/circuits/<circuit>.poly.ir — every call inlined, every array
        element scalarised, common subexpressions merged, dead values dropped.
        It is circuit *data* (the constraint system), consumed by
        tools/gen_eval_check.py to emit the gfx950 eval_check kernels.

IR lines (ids are dense, operands refer to earlier ids; types are inferred):
  c ID V            Fp constant (plain integer, Elem::new)
  e ID V0 V1 V2 V3  FpExt constant
  l ID ARG COL BACK load args[ARG][COL*domain + ((cycle - 4*BACK) & (domain-1))]
  g ID ARG IDX      uniform load args[ARG][IDX] (global buffers: mix, out)
  + ID A B | - ID A B | * ID A B
  a ID ACC T K      accumulate: ACC + T * poly_mix[K]
  b ID ACC T U K    accumulate: ACC + T * U * poly_mix[K]
  r ID              result
Runs in the build container only (reads /root/reference); the .ir is committed.
"""
import os
import re
import sys

REF = os.environ.get("R0_REFERENCE", "/root/reference")
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")

SOURCES = {
    "rv32im": [f"risc0/circuit/rv32im-sys/kernels/cxx/rust_poly_fp_{i}.cpp" for i in range(4)],
    "recursion": ["risc0/circuit/recursion-sys/kernels/cxx/poly_fp.cpp"],
}

HDR = re.compile(r"^FpExt (\w+)\(size_t cycle, size_t steps, FpExt\* poly_mix, (.*)\) \{$")
R_CONST = re.compile(r"^constexpr Fp (x\d+)\((\d+)\);$")
R_ECONST = re.compile(r"^constexpr FpExt (x\d+)\((\d+),(\d+),(\d+),(\d+)\);$")
R_LOAD = re.compile(r"^auto (x\d+) = (?:/\*\w+=\*/)?(\w+(?:\[\d+\])?)\[(\d+) \* steps \+ \(\(cycle - kInvRate \* (\d+)\) & mask\)\];$")
R_AREAD = re.compile(r"^auto (x\d+) = (\w+)\[(\d+)\];$")
R_AWRITE = re.compile(r"^(\w+)\[(\d+)\] = (\w+);$")
R_BIN = re.compile(r"^auto (x\d+) = (\w+) ([-+*]) (\w+);$")
R_ACC = re.compile(r"^FpExt (x\d+) = (\w+) \+ (\w+) \* poly_mix\[(\d+)\];$")
R_ACC2 = re.compile(r"^FpExt (x\d+) = (\w+) \+ (\w+) \* (\w+) \* poly_mix\[(\d+)\];$")
R_ARR = re.compile(r"^(Fp|FpExt) (x\d+)\[(\d+)\];$")
R_CALL = re.compile(r"^auto (x\d+) = (\w+)\(cycle, steps, poly_mix, (.*)\);$")
R_RET = re.compile(r"^return (\w+);$")
R_GREAD = re.compile(r"^auto (x\d+) = (?:/\*\w+=\*/)?args\[(\d+)\]\[(\d+)\];$")
R_EZERO = re.compile(r"^FpExt (x\d+) = FpExt\((\d+)\);$")


def strip(src):
    src = re.sub(r"/\*(?!\w+=\*/).*?\*/", "", src, flags=re.S)  # keep /*data=*/ tags
    out = []
    for line in src.split("\n"):
        i = line.find("//")
        if i >= 0:
            line = line[:i]
        line = line.strip()
        if line:
            out.append(line)
    return out


def parse(files):
    funcs = {}
    cur = None
    for path in files:
        for line in strip(open(os.path.join(REF, path)).read()):
            m = HDR.match(line)
            if m:
                params = [p.strip() for p in m.group(2).split(",")]
                cur = {"name": m.group(1), "params": [p.split()[-1] for p in params],
                       "ptypes": [" ".join(p.split()[:-1]) for p in params], "body": []}
                funcs[cur["name"]] = cur
                continue
            if cur is None:
                continue
            if line == "}":
                cur = None
                continue
            cur["body"].append(line)
    return funcs


class Builder:
    def __init__(self):
        self.nodes = []   # tuples
        self.types = []   # 'f' or 'e'
        self.memo = {}

    def add(self, node, ty):
        key = node
        if key in self.memo:
            return self.memo[key]
        i = len(self.nodes)
        self.nodes.append(node)
        self.types.append(ty)
        self.memo[key] = i
        return i


def run(funcs, b, name, args, arg_bufs):
    """Symbolically execute `name`. args: list of values (SSA id, ('arr', dict, ty) or ('buf', k))."""
    f = funcs[name]
    env = dict(zip(f["params"], args))
    P = 2013265921

    def val(tok):
        v = env[tok]
        assert isinstance(v, int), (name, tok, v)
        return v

    for line in f["body"]:
        if line == "size_t mask = steps - 1;":
            continue
        m = R_CONST.match(line)
        if m:
            env[m.group(1)] = b.add(("c", int(m.group(2)) % P), "f")
            continue
        m = R_ECONST.match(line)
        if m:
            env[m.group(1)] = b.add(("e",) + tuple(int(m.group(k)) % P for k in range(2, 6)), "e")
            continue
        m = R_EZERO.match(line)
        if m:
            env[m.group(1)] = b.add(("e", int(m.group(2)) % P, 0, 0, 0), "e")
            continue
        m = R_LOAD.match(line)
        if m:
            src = m.group(2)
            if src.startswith("args["):
                buf = int(src[5:-1])
            else:
                kind = env[src]
                assert kind[0] == "buf", (name, line)
                buf = kind[1]
            env[m.group(1)] = b.add(("l", buf, int(m.group(3)), int(m.group(4))), "f")
            continue
        m = R_GREAD.match(line)
        if m:
            env[m.group(1)] = b.add(("g", int(m.group(2)), int(m.group(3))), "f")
            continue
        m = R_AREAD.match(line)
        if m:
            arr = env[m.group(2)]
            if arr[0] == "buf":  # a global (mix / out) buffer indexed directly: uniform load
                env[m.group(1)] = b.add(("g", arr[1], int(m.group(3))), "f")
                continue
            assert arr[0] == "arr", line
            env[m.group(1)] = arr[1][int(m.group(3))]
            continue
        m = R_AWRITE.match(line)
        if m:
            arr = env[m.group(1)]
            assert arr[0] == "arr", line
            arr[1][int(m.group(2))] = val(m.group(3))
            continue
        m = R_BIN.match(line)
        if m:
            x, y = val(m.group(2)), val(m.group(4))
            ty = "e" if "e" in (b.types[x], b.types[y]) else "f"
            op = m.group(3)
            if op in "+*" and x > y:
                x, y = y, x  # canonical order for CSE of commutative ops
            env[m.group(1)] = b.add((op, x, y), ty)
            continue
        m = R_ACC.match(line)
        if m:
            env[m.group(1)] = b.add(("a", val(m.group(2)), val(m.group(3)), int(m.group(4))), "e")
            continue
        m = R_ACC2.match(line)
        if m:
            env[m.group(1)] = b.add(("b", val(m.group(2)), val(m.group(3)), val(m.group(4)), int(m.group(5))), "e")
            continue
        m = R_ARR.match(line)
        if m:
            env[m.group(2)] = ("arr", {}, m.group(1))
            continue
        m = R_CALL.match(line)
        if m:
            callee = m.group(2)
            cargs = []
            for tok in [t.strip() for t in m.group(3).split(",")]:
                if tok.startswith("/*"):
                    tok = tok.split("*/", 1)[1].strip()
                if tok.startswith("args["):
                    cargs.append(("buf", int(tok[5:-1])))
                else:
                    cargs.append(env[tok])
            env[m.group(1)] = run(funcs, b, callee, cargs, arg_bufs)
            continue
        m = R_RET.match(line)
        if m:
            return val(m.group(1))
        raise ValueError(f"{name}: unhandled statement: {line}")
    raise ValueError(f"{name}: no return")


def flatten(circuit):
    funcs = parse(SOURCES[circuit])
    b = Builder()
    res = run(funcs, b, "poly_fp", [("buf", k) for k in range(8)], None)
    # dead-code elimination + renumbering
    live = [False] * len(b.nodes)
    live[res] = True
    for i in range(len(b.nodes) - 1, -1, -1):
        if not live[i]:
            continue
        n = b.nodes[i]
        ops = {"+": n[1:3], "-": n[1:3], "*": n[1:3], "a": n[1:3], "b": n[1:4]}.get(n[0], ())
        for o in ops:
            live[o] = True
    remap = {}
    lines = []
    for i, n in enumerate(b.nodes):
        if not live[i]:
            continue
        j = len(remap)
        remap[i] = j
        if n[0] == "c":
            lines.append(f"c {j} {n[1]}")
        elif n[0] == "e":
            lines.append(f"e {j} {n[1]} {n[2]} {n[3]} {n[4]}")
        elif n[0] == "l":
            lines.append(f"l {j} {n[1]} {n[2]} {n[3]}")
        elif n[0] == "g":
            lines.append(f"g {j} {n[1]} {n[2]}")
        elif n[0] in "+-*":
            lines.append(f"{n[0]} {j} {remap[n[1]]} {remap[n[2]]}")
        elif n[0] == "a":
            lines.append(f"a {j} {remap[n[1]]} {remap[n[2]]} {n[3]}")
        elif n[0] == "b":
            lines.append(f"b {j} {remap[n[1]]} {remap[n[2]]} {remap[n[3]]} {n[4]}")
    lines.append(f"r {remap[res]}")
    return lines


def main():
    for circuit in sys.argv[1:] or list(SOURCES):
        lines = flatten(circuit)
        out = os.path.join(ROOT, "risc0_amd", "circuits", f"{circuit}.poly.ir")
        with open(out, "w") as f:
            f.write(f"# {circuit} constraint program (flattened by tools/gen_poly_ir.py)\n")
            f.write("\n".join(lines) + "\n")
        kinds = {}
        for ln in lines:
            kinds[ln[0]] = kinds.get(ln[0], 0) + 1
        print(circuit, len(lines), kinds)


if __name__ == "__main__":
    main()
