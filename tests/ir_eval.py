"""Vectorised numpy interpreter for the flattened constraint programs
(risc0_amd/circuits/*.poly.ir). Test infrastructure: used to pin the IR against the
reference's own compiled poly_fp and to cross-check the emitted HIP kernels."""
import os

import numpy as np

P = 15 * 2**27 + 1
NB = P - 11
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_ir(name):
    prog = []
    with open(os.path.join(ROOT, "risc0_amd", "circuits", name + ".poly.ir")) as f:
        for line in f:
            if line.startswith("#") or not line.strip():
                continue
            t = line.split()
            prog.append((t[0],) + tuple(int(x) for x in t[1:]))
    return prog


def _emul(a, b):
    a0, a1, a2, a3 = a
    b0, b1, b2, b3 = b
    m = lambda x, y: (x * y) % P
    r0 = (m(a0, b0) + NB * ((m(a1, b3) + m(a2, b2) + m(a3, b1)) % P)) % P
    r1 = (m(a0, b1) + m(a1, b0) + NB * ((m(a2, b3) + m(a3, b2)) % P)) % P
    r2 = (m(a0, b2) + m(a1, b1) + m(a2, b0) + NB * m(a3, b3)) % P
    r3 = (m(a0, b3) + m(a1, b2) + m(a2, b1) + m(a3, b0)) % P
    return (r0, r1, r2, r3)


def evaluate(prog, args, domain, pm, inv_rate=4):
    """args: list of plain-integer numpy arrays (per buffer); pm: list of plain FpExt tuples.
    Returns 4 arrays (plain) of length `domain` = poly_fp(cycle) for every cycle. Taps read
    `back * inv_rate` rows back: 4 on the evaluation domain (the generated code's kInvRate),
    1 to evaluate the constraints on the trace rows themselves."""
    cyc = np.arange(domain, dtype=np.int64)
    mask = domain - 1
    val = {}
    z = np.zeros(domain, dtype=np.uint64)

    def ext(v):
        return v if isinstance(v, tuple) else (v, z, z, z)

    def add(a, b):
        if isinstance(a, tuple) or isinstance(b, tuple):
            a, b = ext(a), ext(b)
            return tuple((x + y) % P for x, y in zip(a, b))
        return (a + b) % P

    def sub(a, b):
        if isinstance(a, tuple) or isinstance(b, tuple):
            a, b = ext(a), ext(b)
            return tuple((x + P - y) % P for x, y in zip(a, b))
        return (a + P - b) % P

    def mul(a, b):
        if isinstance(a, tuple) and isinstance(b, tuple):
            return _emul(a, b)
        if isinstance(a, tuple):
            return tuple((x * b) % P for x in a)
        if isinstance(b, tuple):
            return tuple((a * y) % P for y in b)
        return (a * b) % P

    for ins in prog:
        op, i = ins[0], ins[1]
        if op == "c":
            val[i] = np.full(domain, ins[2], dtype=np.uint64)
        elif op == "e":
            val[i] = tuple(np.full(domain, x, dtype=np.uint64) for x in ins[2:6])
        elif op == "l":
            buf, col, back = ins[2:5]
            idx = col * domain + ((cyc - inv_rate * back) & mask)
            val[i] = args[buf][idx].astype(np.uint64)
        elif op == "g":
            val[i] = np.full(domain, int(args[ins[2]][ins[3]]), dtype=np.uint64)
        elif op == "+":
            val[i] = add(val[ins[2]], val[ins[3]])
        elif op == "-":
            val[i] = sub(val[ins[2]], val[ins[3]])
        elif op == "*":
            val[i] = mul(val[ins[2]], val[ins[3]])
        elif op == "a":
            k = tuple(np.full(domain, x, dtype=np.uint64) for x in pm[ins[4]])
            val[i] = add(val[ins[2]], mul(val[ins[3]], k))
        elif op == "b":
            k = tuple(np.full(domain, x, dtype=np.uint64) for x in pm[ins[5]])
            val[i] = add(val[ins[2]], mul(mul(val[ins[3]], val[ins[4]]), k))
        elif op == "r":
            return ext(val[i])
    raise ValueError("no result")
