#!/usr/bin/env python3
"""Flatten the recursion circuit's generated witness-generation step functions into a block
IR that tools/gen_witgen.py compiles to HIP (run in the container where the reference tree
lives, reading it as text; the output is committed circuit data, like
risc0_amd/circuits/recursion.accum.ir):

  risc0/circuit/recursion-sys/kernels/cxx/step_exec.cpp        (the VM step: data columns)
  risc0/circuit/recursion-sys/kernels/cxx/step_verify_mem.cpp  (the sorted-WOM check rows)

as driven by risc0_circuit_recursion_cpu_witgen (recursion-sys/kernels/cxx/ffi.cpp:191-205)
with the externs of recursion-sys/kernels/cxx/extern.cpp. The step code is SSA over Fp with
nested `if (x != 0)` blocks (the control columns' one-hot selectors).

IR, one statement per line (IDs are the reference's xN numbers):
  fn exec|verify
  c ID VALUE                 constexpr Fp xID(VALUE)                   (plain integer)
  l ID ARG COL BACK          args[ARG][COL * steps + ((cycle - BACK) & mask)]
  ld ID ARG COL BACK         the same, then INVALID -> 0 (`if (x == Fp::invalid()) x = 0`)
  g ID ARG IDX               args[ARG][IDX]
  + - * ID A B | n ID A | i ID A (inverse, inv(0) = 0)
  and ID A B                 Fp(xA.asUInt32() & xB.asUInt32())
  isz ID A                   (xA == 0) ? Fp(1) : Fp(0)
  if ID / end                if (xID != 0) { ... }
  w ARG COL ID               args[ARG][COL * steps + cycle] = xID      (register write)
  gw ARG IDX ID              args[ARG][IDX] = xID                      (global write)
  chk ID LINE                if (xID != 0) throw "eqz failed at: zirgen/circuit/recursion/wom.cpp:LINE"
  wr D0 D1 D2 D3 ADDR        extern_womRead(ADDR): the preflight WOM at xADDR.asUInt32()
  pw ADDR V0 V1 V2 V3        extern_plonkWrite_wom: this cycle's next WOM argument row
  pr D0 D1 D2 D3 D4          extern_plonkRead_wom: the next sorted WOM row (addr as Fp, value)
  iop D0 D1 D2 D3            extern_readIOPBody: the cycle's next IOP value
  rc D0 .. D15               extern_readCoefficients (checked bytes): not implemented by the
                             reference's CPU witness generator (extern.cpp throws), so an error

  gen_witgen_ir.py [REFERENCE_ROOT] > risc0_amd/circuits/recursion.witgen.ir
"""
import re
import sys

SRC = "risc0/circuit/recursion-sys/kernels/cxx/"
X = r"x(\d+)"

PATTERNS = [
    (re.compile(rf"constexpr Fp {X}\((\d+)\);"), lambda m: f"c {m[1]} {m[2]}"),
    (re.compile(rf"auto {X} = args\[(\d+)\]\[(\d+) \* steps \+ \(\(cycle - (\d+)\) & mask\)\];"),
     lambda m: f"l {m[1]} {m[2]} {m[3]} {m[4]}"),
    (re.compile(rf"auto {X} = args\[(\d+)\]\[(\d+)\];"), lambda m: f"g {m[1]} {m[2]} {m[3]}"),
    (re.compile(rf"auto {X} = {X} ([-+*]) {X};"), lambda m: f"{m[3]} {m[1]} {m[2]} {m[4]}"),
    (re.compile(rf"auto {X} = -{X};"), lambda m: f"n {m[1]} {m[2]}"),
    (re.compile(rf"auto {X} = inv\({X}\);"), lambda m: f"i {m[1]} {m[2]}"),
    (re.compile(rf"auto {X} = Fp\({X}\.asUInt32\(\) & {X}\.asUInt32\(\)\);"), lambda m: f"and {m[1]} {m[2]} {m[3]}"),
    (re.compile(rf"auto {X} = \({X} == 0\) \? Fp\(1\) : Fp\(0\);"), lambda m: f"isz {m[1]} {m[2]}"),
    (re.compile(rf"if \({X} != 0\) \{{"), lambda m: f"if {m[1]}"),
    (re.compile(rf"if \({X} != 0\) throw std::runtime_error\(\"eqz failed at: zirgen/circuit/recursion/wom\.cpp:(\d+)\"\);"),
     lambda m: f"chk {m[1]} {m[2]}"),
    (re.compile(rf"args\[(\d+)\]\[(\d+)\] = {X};"), lambda m: f"gw {m[1]} {m[2]} {m[3]}"),
    (re.compile(rf"auto \[{X}, {X}, {X}, {X}\] = extern_womRead\(ctx, cycle, \"\", \{{{X}\}}\);"),
     lambda m: f"wr {m[1]} {m[2]} {m[3]} {m[4]} {m[5]}"),
    (re.compile(rf"extern_plonkWrite_wom\(ctx, cycle, \"wom\", \{{{X}, {X}, {X}, {X}, {X}\}}\);"),
     lambda m: f"pw {m[1]} {m[2]} {m[3]} {m[4]} {m[5]}"),
    (re.compile(rf"auto \[{X}, {X}, {X}, {X}, {X}\] = extern_plonkRead_wom\(ctx, cycle, \"wom\", \{{\}}\);"),
     lambda m: f"pr {m[1]} {m[2]} {m[3]} {m[4]} {m[5]}"),
    (re.compile(r"auto \[(x\d+(?:, x\d+){15})\] = extern_readCoefficients\(ctx, cycle, \"\", \{\}\);"),
     lambda m: "rc " + " ".join(v[1:] for v in m[1].split(", "))),
    (re.compile(rf"auto \[{X}, {X}, {X}, {X}\] = extern_readIOPBody\(ctx, cycle, \"\", \{{{X}, {X}, {X}\}}\);"),
     lambda m: f"iop {m[1]} {m[2]} {m[3]} {m[4]}"),
]
DEFAULT0 = re.compile(rf"if \({X} == Fp::invalid\(\)\) {X} = 0;")
REG = re.compile(r"auto& reg = args\[(\d+)\]\[(\d+) \* steps \+ cycle\];")
SET = re.compile(rf"reg = {X};")
# asserts, comments, logging and the no-op externs (extern.cpp: womWrite and readIOPHeader
# do nothing; log only prints)
SKIP = re.compile(r"^assert\(|^//|^#|^$|^namespace|^\} // namespace|^Fp step_|^size_t mask|^return x\d+;$|"
                  r"^extern_log\(|^extern_womWrite\(|^extern_readIOPHeader\(")


def flatten(path, name, fn_sig):
    out = [f"fn {name}"]
    lines = [l.strip() for l in open(path).read().split("\n")]
    start = next(i for i, l in enumerate(lines) if l.startswith(fn_sig))
    blocks = []
    pending = None
    for l in lines[start + 1:]:
        if SKIP.search(l):
            continue
        if l == "}":
            if not blocks:
                break  # end of the function
            if blocks.pop() == "if":
                out.append("end")
            continue
        if l == "{":
            blocks.append("{")
            continue
        m = REG.fullmatch(l)
        if m:
            pending = (m[1], m[2])
            continue
        m = SET.fullmatch(l)
        if m:
            assert pending, l
            out.append(f"w {pending[0]} {pending[1]} {m[1]}")
            pending = None
            continue
        m = DEFAULT0.fullmatch(l)
        if m:
            assert m[1] == m[2] and out[-1].startswith(f"l {m[1]} "), l
            out[-1] = "ld" + out[-1][1:]
            continue
        for pat, fmt in PATTERNS:
            m = pat.fullmatch(l)
            if m:
                s = fmt(m)
                out.append(s)
                if s.startswith("if "):
                    blocks.append("if")
                break
        else:
            raise SystemExit(f"{path}: unrecognised statement: {l}")
    return out


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    print("# recursion witness generation steps (flattened by tools/gen_witgen_ir.py from")
    print(f"# {SRC}step_exec.cpp and step_verify_mem.cpp)")
    for name, fname, sig in (("exec", "step_exec.cpp", "Fp step_exec("),
                             ("verify", "step_verify_mem.cpp", "Fp step_verify_mem(")):
        for s in flatten(f"{root}/{SRC}{fname}", name, sig):
            print(s)


if __name__ == "__main__":
    main()
