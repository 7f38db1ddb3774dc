"""The recursion circuit's own verifier constraint program, interpreted (test infrastructure).

risc0/circuit/recursion/src/poly_ext.rs holds `DEF: PolyExtStepDef`, the generated
constraint program the reference verifier evaluates at the out-of-domain point
(verify/mod.rs:556: `circuit.poly_ext(poly_mix, eval_u, &[out, &mix]).tot`). This module
reads that table as text where it lies under /root/reference (study of the source; nothing
of it is copied into the repo) and runs it with a restatement of the reference's
interpreter, PolyExtExecutor::step (risc0/zkp/src/adapter.rs:317-400), vectorised over many
inputs with numpy. tools/make_poly_ext_golden.py turns its outputs on seeded inputs into
the committed fixture tests/golden/poly_ext_recursion.npy.

Values are plain integers mod p (decoded from Montgomery words); FpExt is a (4, n) array.
"""
import os
import re

import numpy as np

P = 15 * 2**27 + 1
NB = P - 11  # x^4 = -11 (baby_bear.rs)
REF = "/root/reference/risc0/circuit/recursion/src/poly_ext.rs"
RINV = pow(2**32, P - 2, P)
R_MOD = 2**32 % P


def available():
    return os.path.exists(REF)


def parse(path=REF):
    """[(op, args)] of DEF.block and DEF.ret (poly_ext.rs: `PolyExtStep::Op(a, b), // loc`)."""
    text = open(path).read()
    steps = [(m.group(1), tuple(int(x) for x in m.group(2).split(",") if x.strip()) if m.group(2) else ())
             for m in re.finditer(r"PolyExtStep::(\w+)(?:\(([^)]*)\))?", text.split("pub const DEF")[1])]
    ret = int(re.search(r"ret:\s*(\d+)", text).group(1))
    return steps, ret


def dec(w):
    return (np.asarray(w, np.uint64) * np.uint64(RINV)) % np.uint64(P)


def enc(x):
    return ((np.asarray(x, np.uint64) % np.uint64(P)) * np.uint64(R_MOD)) % np.uint64(P)


def _mul(a, b):
    """FpExt product (baby_bear.rs:744-757), a, b: (4, n) uint64 < p"""
    out = np.zeros_like(a)
    for i in range(4):
        for j in range(4):
            t = (a[i] * b[j]) % np.uint64(P)
            if i + j >= 4:
                t = (t * np.uint64(NB)) % np.uint64(P)
            out[(i + j) % 4] = (out[(i + j) % 4] + t) % np.uint64(P)
    return out


def run(steps, ret, poly_mix, eval_u, glob, mix):
    """PolyExtStepDef::step over n inputs: poly_mix (4, n), eval_u (taps, 4, n), glob (out, n),
    mix (mix_size, n), all decoded values; returns MixState.tot as (4, n)."""
    n = poly_mix.shape[1]
    p = np.uint64(P)
    one = np.zeros((4, n), np.uint64)
    one[0] = 1
    zero = np.zeros((4, n), np.uint64)
    args = [glob, mix]  # &[out, &mix] (verify/mod.rs:556)
    fp, mixv = [], []
    for op, a in steps:
        if op == "Const":
            v = zero.copy()
            v[0] = a[0] % P
            fp.append(v)
        elif op == "ConstExt":
            fp.append(np.array([[x % P] * n for x in a], np.uint64))
        elif op == "Get":
            fp.append(eval_u[a[0]])
        elif op == "GetGlobal":
            v = zero.copy()
            v[0] = args[a[0]][a[1]]
            fp.append(v)
        elif op == "Add":
            fp.append((fp[a[0]] + fp[a[1]]) % p)
        elif op == "Sub":
            fp.append((fp[a[0]] + p - fp[a[1]]) % p)
        elif op == "Mul":
            fp.append(_mul(fp[a[0]], fp[a[1]]))
        elif op == "True":
            mixv.append((zero, one))
        elif op == "AndEqz":
            tot, mul = mixv[a[0]]
            mixv.append(((tot + _mul(mul, fp[a[1]])) % p, _mul(mul, poly_mix)))
        elif op == "AndCond":
            tot, mul = mixv[a[0]]
            itot, imul = mixv[a[2]]
            mixv.append(((tot + _mul(_mul(fp[a[1]], itot), mul)) % p, _mul(mul, imul)))
        else:
            raise ValueError(op)
    assert len(mixv) == ret + 1 and len(fp) == len(steps) - (ret + 1)
    return mixv[ret][0]


def inputs(oracle, n, num_taps, mix_size, output_size, seed=0x504F4C59):
    """n seeded input sets as Montgomery words (splitmix64 of (seed + k, index) mod p,
    oracle.splitmix_fill): poly_mix (n, 4), eval_u (n, 4 * taps), glob (n, out), mix (n, mix)."""
    width = 4 + 4 * num_taps + output_size + mix_size
    w = np.stack([oracle.splitmix_fill(seed + k, width) for k in range(n)])
    a = 4 + 4 * num_taps
    return w[:, :4], w[:, 4:a], w[:, a:a + output_size], w[:, a + output_size:]


def evaluate(steps, ret, poly_mix, eval_u, glob, mix, chunk=200):
    """Montgomery words in (as from inputs()), MixState.tot as Montgomery words (n, 4) out."""
    out = []
    for s in range(0, poly_mix.shape[0], chunk):
        sl = slice(s, s + chunk)
        pm = dec(poly_mix[sl]).T
        u = dec(eval_u[sl]).reshape(-1, eval_u.shape[1] // 4, 4).transpose(1, 2, 0)
        tot = run(steps, ret, pm, u, dec(glob[sl]).T, dec(mix[sl]).T)
        out.append(enc(tot).T.astype(np.uint32))
    return np.concatenate(out)
