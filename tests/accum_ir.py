"""TEST INFRASTRUCTURE — the recursion accumulation (risc0_amd/circuits/recursion.accum.ir,
flattened by tools/gen_accum_ir.py from recursion-sys/kernels/cxx/step_{compute,verify}_accum.cpp)
interpreted with numpy over all cycles at once, with the driver of
risc0_circuit_recursion_cpu_accum (recursion-sys/kernels/cxx/ffi.cpp:160-217): compute for
every cycle (the per-cycle value starts at FpExt 1), inclusive prefix product, verify.
Also the synthetic witness these tests use, and a ctypes binding of the reference's own
compiled risc0_circuit_recursion_cpu_accum (oracle/_ref/libref_recursion.so).
"""
import ctypes as C
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 15 * 2**27 + 1
RINV = pow(2**32, P - 2, P)
INVALID = 0xFFFFFFFF


def load_ir():
    fns = {}
    cur = None
    for line in open(os.path.join(ROOT, "risc0_amd", "circuits", "recursion.accum.ir")):
        if line.startswith("#") or not line.strip():
            continue
        t = line.split()
        if t[0] == "fn":
            cur = fns.setdefault(t[1], [])
            continue
        cur.append((t[0],) + tuple(int(x) for x in t[1:]))
    return fns


def synthetic(rng, oracle, po2, gs, out_size, mix_size):
    """Uniform canonical words, with the control columns' one-hot selectors made one-hot
    (micro/macro-op select, ctrl columns 1..7, and the macro-op kind, columns 9..17) as the
    recursion program's control rows are: the step code's `if` arms are then mutually
    exclusive per cycle, and the reference's own write asserts hold."""
    n = 1 << po2
    ctrl = oracle.rand_elems(rng, gs[1] * n)
    one = oracle.encode(1)
    for cols in (range(1, 8), range(9, 18)):
        cols = list(cols)
        sel = rng.integers(0, len(cols), n)
        for j, c in enumerate(cols):
            ctrl[c * n:(c + 1) * n] = np.where(sel == j, one, 0)
    data = oracle.rand_elems(rng, gs[2] * n)
    glob = oracle.rand_elems(rng, out_size)
    mix = oracle.rand_elems(rng, mix_size)
    return ctrl, glob, data, mix


def ref_accum(ctrl, glob, data, mix, accum, steps, cycles):
    """The reference's risc0_circuit_recursion_cpu_accum on host buffers (accum in place)."""
    lib = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref_recursion.so"))
    f = lib.risc0_circuit_recursion_cpu_accum
    f.restype = C.c_void_p

    class AB(C.Structure):
        _fields_ = [(k, C.c_void_p) for k in ("ctrl", "glob", "data", "mix", "accum")]

    ab = AB(*(a.ctypes.data for a in (ctrl, glob, data, mix, accum)))
    err = f(C.byref(ab), C.c_uint32(steps), C.c_uint32(cycles))
    if err:
        raise RuntimeError(C.cast(err, C.c_char_p).value.decode())


def _dec(w):
    return (w.astype(np.uint64) * RINV) % P


def _enc(v):
    return ((v.astype(np.uint64) << np.uint64(32)) % P).astype(np.uint32)


def _mul(a, b):
    return (a * b) % P


def _inv(a):
    r = np.ones_like(a)
    base = a.copy()
    e = P - 2
    while e:
        if e & 1:
            r = _mul(r, base)
        base = _mul(base, base)
        e >>= 1
    return r


def _emul(a, b):
    """FpExt product (x^4 = -11) of 4-tuples of plain ints"""
    r = [0, 0, 0, 0]
    for i in range(4):
        for j in range(4):
            if i + j < 4:
                r[i + j] += a[i] * b[j]
            else:
                r[i + j - 4] += (P - 11) * a[i] * b[j]
    return [x % P for x in r]


def run(fn, args, steps, cycles, accum_vals, accum_out):
    """Interpret one step function for cycles [0, steps) at once. args: 5 host arrays of
    Montgomery words (ctrl, global, data, mix, accum); accum_vals: per-cycle FpExt (plain,
    shape (steps, 4)) read by `ra` and written by `wa`; register writes go to accum_out."""
    mask = cycles - 1
    cyc = np.arange(steps, dtype=np.int64)
    v = {}
    guard = [np.ones(steps, dtype=bool)]
    for ins in fn:
        op = ins[0]
        if op == "c":
            v[ins[1]] = np.full(steps, ins[2] % P, np.uint64)
        elif op == "l":
            _, i, a, col, back = ins
            v[i] = _dec(args[a][col * cycles + ((cyc - back) & mask)])
        elif op == "g":
            v[ins[1]] = np.full(steps, int(_dec(np.array([args[ins[2]][ins[3]]]))[0]), np.uint64)
        elif op == "+":
            v[ins[1]] = (v[ins[2]] + v[ins[3]]) % P
        elif op == "-":
            v[ins[1]] = (v[ins[2]] + P - v[ins[3]]) % P
        elif op == "*":
            v[ins[1]] = _mul(v[ins[2]], v[ins[3]])
        elif op == "n":
            v[ins[1]] = (P - v[ins[2]]) % P
        elif op == "i":
            v[ins[1]] = _inv(v[ins[2]])
        elif op == "if":
            guard.append(guard[-1] & (v[ins[1]] != 0))
        elif op == "end":
            guard.pop()
        elif op == "w":
            _, a, col, i = ins
            g = guard[-1]
            assert a == 4
            accum_out[col * cycles + cyc[g]] = _enc(v[i][g])
        elif op == "ra":
            for k in range(4):
                v[ins[1 + k]] = accum_vals[:, k].copy()
        elif op == "wa":
            g = guard[-1]
            for k in range(4):
                accum_vals[g, k] = v[ins[1 + k]][g]
        else:
            raise ValueError(op)


def accum(ctrl, glob, data, mix, accum_buf, steps, cycles):
    """ffi.cpp:160-217 over the IR: returns the accum buffer after compute, prefix
    product and verify (a copy of accum_buf with the written registers)."""
    fns = load_ir()
    out = accum_buf.copy()
    args = [ctrl, glob, data, mix, out]
    vals = np.zeros((steps, 4), np.uint64)
    vals[:, 0] = 1
    run(fns["compute"], args, steps, cycles, vals, out)
    acc = [1, 0, 0, 0]
    for c in range(steps):
        acc = _emul(acc, [int(x) for x in vals[c]])
        vals[c] = acc
    run(fns["verify"], args, steps, cycles, vals, out)
    return out


def circuit():
    with open(os.path.join(ROOT, "risc0_amd", "circuits", "recursion.taps.json")) as f:
        return json.load(f)
