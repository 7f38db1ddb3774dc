"""numpy interpreter of risc0_amd/circuits/rv32im.accum.ir (tools/gen_rv32im_accum_ir.py):
the rv32im accumulation step (phase 1) over every cycle at once, for checking the IR
against the compiled reference (tests/rv32im_accum_ref.py) on the CPU."""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
IR = os.path.join(ROOT, "risc0_amd", "circuits", "rv32im.accum.ir")
P = 15 * 2**27 + 1
R = 2**32 % P
RINV = pow(2**32, P - 2, P)


def load():
    ops = []
    for line in open(IR):
        if line.startswith("#") or line.startswith("fn") or not line.strip():
            continue
        t = line.split()
        ops.append((t[0],) + tuple(int(x) for x in t[1:]))
    return ops


def run(data, accum, glob, mix, rows, last_cycle, ops=None):
    """accum (column-major words) updated in place for cycles [0, last_cycle)"""
    ops = ops or load()
    bufs = [data, accum, glob, mix]
    cyc = np.arange(last_cycle, dtype=np.int64)
    v = {}
    mask = [np.ones(last_cycle, bool)]
    for op in ops:
        o = op[0]
        if o == "c":
            v[op[1]] = np.full(last_cycle, op[2] * R % P, np.int64)
        elif o == "l":
            _, i, b, col, back = op
            v[i] = bufs[b][col * rows + ((cyc - back) % rows)].astype(np.int64)
        elif o == "g":
            v[op[1]] = np.full(last_cycle, int(bufs[op[2]][op[3]]), np.int64)
        elif o == "+":
            v[op[1]] = (v[op[2]] + v[op[3]]) % P
        elif o == "-":
            v[op[1]] = (v[op[2]] - v[op[3]]) % P
        elif o == "*":
            v[op[1]] = (v[op[2]] * v[op[3]] % P) * RINV % P
        elif o == "n":
            v[op[1]] = (-v[op[2]]) % P
        elif o == "i":
            x = v[op[2]]
            v[op[1]] = np.array([pow(int(a), P - 2, P) * R % P * R % P if a else 0 for a in x], np.int64)
        elif o == "z":
            v[op[1]] = np.where(v[op[2]] == 0, R, 0).astype(np.int64)
        elif o == "if":
            mask.append(mask[-1] & (v[op[1]] != 0))
        elif o == "end":
            mask.pop()
        elif o == "w":
            _, b, col, i = op
            m = mask[-1]
            bufs[b][col * rows + cyc[m]] = v[i][m].astype(np.uint32)
        else:
            raise ValueError(o)
