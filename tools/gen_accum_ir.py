#!/usr/bin/env python3
"""Flatten the recursion circuit's generated accumulation step functions into the block
IR that tools/gen_accum.py compiles to HIP (run in the container where the reference
tree lives; the output is committed circuit data, like risc0_amd/circuits/*.poly.ir):

  risc0/circuit/recursion-sys/kernels/cxx/step_compute_accum.cpp  (per-cycle factor)
  risc0/circuit/recursion-sys/kernels/cxx/step_verify_accum.cpp   (accum columns)

as driven by risc0_circuit_recursion_cpu_accum (recursion-sys/kernels/cxx/ffi.cpp:160-217):
compute_accum for every cycle, an inclusive prefix product of the per-cycle values, then
verify_accum for every cycle. The step code is SSA over Fp with nested `if (x != 0)`
blocks (the one-hot micro/macro-op selectors of the control columns).

IR, one statement per line:
  fn compute|verify
  c ID VALUE               constexpr Fp xID(VALUE)                 (plain integer)
  l ID ARG COL BACK        args[ARG][COL * steps + ((cycle - BACK) & mask)]
  g ID ARG IDX             args[ARG][IDX]                           (globals / mix)
  + ID A B | - ID A B | * ID A B | n ID A (negation) | i ID A (inverse, inv(0) = 0)
  if ID / end              if (xID != 0) { ... }
  w ARG COL ID             args[ARG][COL * steps + cycle] = xID     (register write)
  ra ID0 ID1 ID2 ID3       the cycle's accumulator value            (extern_plonkReadAccum_wom)
  wa ID0 ID1 ID2 ID3       set the cycle's accumulator value        (extern_plonkWriteAccum_wom)

  gen_accum_ir.py [REFERENCE_ROOT] > risc0_amd/circuits/recursion.accum.ir
"""
import re
import sys

SRC = "risc0/circuit/recursion-sys/kernels/cxx/"

PATTERNS = [
    (re.compile(r"constexpr Fp x(\d+)\((\d+)\);"), lambda m: f"c {m[1]} {m[2]}"),
    (re.compile(r"auto x(\d+) = args\[(\d+)\]\[(\d+) \* steps \+ \(\(cycle - (\d+)\) & mask\)\];"),
     lambda m: f"l {m[1]} {m[2]} {m[3]} {m[4]}"),
    (re.compile(r"auto x(\d+) = args\[(\d+)\]\[(\d+)\];"), lambda m: f"g {m[1]} {m[2]} {m[3]}"),
    (re.compile(r"auto x(\d+) = x(\d+) ([-+*]) x(\d+);"), lambda m: f"{m[3]} {m[1]} {m[2]} {m[4]}"),
    (re.compile(r"auto x(\d+) = -x(\d+);"), lambda m: f"n {m[1]} {m[2]}"),
    (re.compile(r"auto x(\d+) = inv\(x(\d+)\);"), lambda m: f"i {m[1]} {m[2]}"),
    (re.compile(r"if \(x(\d+) != 0\) \{"), lambda m: f"if {m[1]}"),
    (re.compile(r"auto \[x(\d+), x(\d+), x(\d+), x(\d+)\] = extern_plonkReadAccum_wom\(ctx, cycle, \"wom\", \{\}\);"),
     lambda m: f"ra {m[1]} {m[2]} {m[3]} {m[4]}"),
    (re.compile(r"extern_plonkWriteAccum_wom\(ctx, cycle, \"wom\", \{x(\d+), x(\d+), x(\d+), x(\d+)\}\);"),
     lambda m: f"wa {m[1]} {m[2]} {m[3]} {m[4]}"),
]
REG = re.compile(r"auto& reg = args\[(\d+)\]\[(\d+) \* steps \+ cycle\];")
SET = re.compile(r"reg = x(\d+);")
SKIP = re.compile(r"assert\(|^//|^#|^$|^namespace|^\} // namespace|^Fp step_|^size_t mask|^return x\d+;$")


def flatten(path, name):
    out = [f"fn {name}"]
    lines = [l.strip() for l in open(path).read().split("\n")]
    # the function body: from its signature to the closing brace at column 0
    start = next(i for i, l in enumerate(lines) if l.startswith(f"Fp step_{name}_accum("))
    depth = 0     # brace depth inside the function body
    blocks = []   # stack: "if" or "{"
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
    print("# recursion accumulation steps (flattened by tools/gen_accum_ir.py from")
    print(f"# {SRC}step_compute_accum.cpp and step_verify_accum.cpp)")
    for name in ("compute", "verify"):
        for s in flatten(f"{root}/{SRC}step_{name}_accum.cpp", name):
            print(s)


if __name__ == "__main__":
    main()
