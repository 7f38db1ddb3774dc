"""numpy interpreter of the C subset tools/gen_accum.py emits (one lane per cycle, all cycles
at once): runs the generated accumulation kernels' *source text* on the CPU, so the
generator's rewrites (batched inverses, depth-first emission, split guarded stores, load
look-ahead, lazily reduced sums of products, arm-sorted kernels) are checked against the IR
interpreter without a GPU. Test infrastructure.

The 64-bit sums of a fused linear combination run in uint64 with a check that no sum wraps
and that Montgomery REDC's input stays below p * 2^32, as the generator's bounds promise.
An arm-sorted kernel's tile sort only permutes which lane takes which cycle, so it runs
here as the identity."""
import re

import numpy as np

P = 15 * 2**27 + 1
R = 2**32 % P
RINV = pow(2**32, P - 2, P)

_V = r"v(\d+)"
_PATTERNS = [
    ("const", re.compile(r"const uint32_t v(\d+) = (\d+)u;$")),
    ("load", re.compile(r"const uint32_t v(\d+) = A\.a\[(\d+)\]\[uint64_t\((\d+)u\) \* A\.cycles \+ "
                        r"\(\(cycle - (\d+)u\) & mask\)\];$")),
    ("glob", re.compile(r"const uint32_t v(\d+) = A\.a\[(\d+)\]\[(\d+)\];$")),
    ("bin", re.compile(r"const uint32_t v(\d+) = (fp_add|fp_sub|fp_mul)\(v(\d+), v(\d+)\);$")),
    ("un", re.compile(r"const uint32_t v(\d+) = (fp_neg|fp_inv)\(v(\d+)\);$")),
    ("isz", re.compile(r"const uint32_t v(\d+) = v(\d+) == 0u \? kOne : 0u;$")),
    ("ibdef", re.compile(r"uint32_t ib(\d+)\[(\d+)\] = \{(.*)\};$")),
    ("ibrun", re.compile(r"fp_inv_batch\(ib(\d+)\);$")),
    ("ibget", re.compile(r"const uint32_t v(\d+) = ib(\d+)\[(\d+)\];$")),
    ("if", re.compile(r"if \((v\d+ != 0u(?: && v\d+ != 0u)*)\) \{$")),
    ("end", re.compile(r"\}$")),
    ("store", re.compile(r"A\.a\[(\d+)\]\[uint64_t\((\d+)u\) \* A\.cycles \+ cycle\] = v(\d+);$")),
    ("vread", re.compile(r"const uint4 r(\d+) = A\.vals\[cycle\];$")),
    ("vget", re.compile(r"const uint32_t v(\d+) = r(\d+)\.([xyzw]);$")),
    ("vwrite", re.compile(r"A\.vals\[cycle\] = make_uint4\(v(\d+), v(\d+), v(\d+), v(\d+)\);$")),
    ("umin", re.compile(r"const uint32_t v(\d+) = umin\(v(\d+), v(\d+)\);$")),
    ("tdef", re.compile(r"uint64_t t(\d+) = uint64_t\(v(\d+)\) \* (v\d+|\d+u|\(kP - v\d+\));$")),
    ("tadd", re.compile(r"t(\d+) \+= uint64_t\(v(\d+)\) \* (v\d+|\d+u|\(kP - v\d+\));$")),
    ("tfold", re.compile(r"t(\d+) = fold64\(t(\d+)\);$")),
    ("redc", re.compile(r"const uint32_t v(\d+) = mont_reduce\(t(\d+)\);$")),
    ("keyblk", re.compile(r"if \(c0 < A\.steps\) \{$")),
]
_SKIP = re.compile(r"^(const uint32_t (cycle|mask|c0) = .*|if \(cycle >= A\.steps\) return;|"
                   r"uint32_t key = \d+u;|key = .*;)$")
_FOLD_C = 2**32 % P
_NEG_PINV = (-pow(P, -1, 2**32)) % 2**32
_M32 = np.uint64(0xFFFFFFFF)


def kernel_body(src):
    """the statements of the one __global__ function of a generated file"""
    lines = src.split("\n")
    start = next(i for i, ln in enumerate(lines) if ln.startswith("__global__"))
    end = next(i for i in range(start, len(lines)) if lines[i] == "}")
    return [ln.strip() for ln in lines[start + 1:end] if ln.strip()]


def _inv(x):
    return np.array([pow(int(a), P - 2, P) * R % P * R % P if a else 0 for a in x], np.int64)


def run_kernel(src, bufs, rows, steps, vals=None):
    """Execute one generated kernel's statements for cycles [0, steps); bufs are the AccArgs
    arrays (numpy uint32, updated in place by the stores); vals (recursion) the per-cycle
    FpExt of A.vals, int64 Montgomery words of shape (steps, 4)."""
    cyc = np.arange(steps, dtype=np.int64)
    v, ib, rr, t = {}, {}, {}, {}

    def operand(e):
        if e.startswith("(kP - v"):
            return np.uint64(P) - v[int(e[7:-1])].astype(np.uint64)
        if e.startswith("v"):
            return v[int(e[1:])].astype(np.uint64)
        return np.full(steps, int(e[:-1]), np.uint64)

    mask = [np.ones(steps, bool)]
    for st in kernel_body(src):
        if _SKIP.match(st):
            continue
        for kind, pat in _PATTERNS:
            m = pat.match(st)
            if m:
                break
        else:
            raise ValueError(f"unparsed statement: {st}")
        g = m.groups()
        if kind == "const":
            v[int(g[0])] = np.full(steps, int(g[1]), np.int64)
        elif kind == "load":
            b, col, back = int(g[1]), int(g[2]), int(g[3])
            v[int(g[0])] = bufs[b][col * rows + ((cyc - back) % rows)].astype(np.int64)
        elif kind == "glob":
            v[int(g[0])] = np.full(steps, int(bufs[int(g[1])][int(g[2])]), np.int64)
        elif kind == "bin":
            a, c = v[int(g[2])], v[int(g[3])]
            v[int(g[0])] = {"fp_add": lambda: (a + c) % P, "fp_sub": lambda: (a - c) % P,
                            "fp_mul": lambda: (a * c % P) * RINV % P}[g[1]]()
        elif kind == "un":
            a = v[int(g[2])]
            v[int(g[0])] = (-a) % P if g[1] == "fp_neg" else _inv(a)
        elif kind == "isz":
            v[int(g[0])] = np.where(v[int(g[1])] == 0, R, 0).astype(np.int64)
        elif kind == "ibdef":
            names = [int(x.strip()[1:]) for x in g[2].split(",")]
            assert len(names) == int(g[1])
            ib[int(g[0])] = [v[n] for n in names]
        elif kind == "ibrun":
            ib[int(g[0])] = [_inv(x) for x in ib[int(g[0])]]  # Montgomery's trick is exact
        elif kind == "ibget":
            v[int(g[0])] = ib[int(g[1])][int(g[2])]
        elif kind == "if":
            m_ = mask[-1].copy()
            for name in re.findall(_V, g[0]):
                m_ &= v[int(name)] != 0
            mask.append(m_)
        elif kind == "end":
            mask.pop()
        elif kind == "vread":
            rr[int(g[0])] = vals.copy()
        elif kind == "vget":
            v[int(g[0])] = rr[int(g[1])][:, "xyzw".index(g[2])].copy()
        elif kind == "vwrite":
            sel = mask[-1]
            for k in range(4):
                vals[sel, k] = v[int(g[k])][sel]
        elif kind == "umin":
            v[int(g[0])] = np.minimum(v[int(g[1])], v[int(g[2])])
        elif kind == "tdef":
            t[int(g[0])] = v[int(g[1])].astype(np.uint64) * operand(g[2])
        elif kind == "tadd":
            old = t[int(g[0])]
            t[int(g[0])] = old + v[int(g[1])].astype(np.uint64) * operand(g[2])
            assert (t[int(g[0])] >= old).all(), "64-bit sum wrapped"
        elif kind == "tfold":
            x = t[int(g[1])]
            t[int(g[0])] = (x >> np.uint64(32)) * np.uint64(_FOLD_C) + (x & _M32)
        elif kind == "redc":
            x = t[int(g[1])]
            assert (x < np.uint64(P) << np.uint64(32)).all(), "REDC input not below p * 2^32"
            m = ((x & _M32) * np.uint64(_NEG_PINV)) & _M32
            r = (x + m * np.uint64(P)) >> np.uint64(32)
            v[int(g[0])] = np.where(r >= P, r - np.uint64(P), r).astype(np.int64)
        elif kind == "keyblk":
            mask.append(mask[-1].copy())
        elif kind == "store":
            b, col, i = int(g[0]), int(g[1]), int(g[2])
            sel = mask[-1]
            bufs[b][col * rows + cyc[sel]] = v[i][sel].astype(np.uint32)
    assert len(mask) == 1, "unbalanced blocks"
