"""tools/gen_accum.py's fuse_sums: the lazily reduced linear combinations it emits store the
same words as the unfused field operations, for both accumulation IRs.

The unfused program runs in exact field arithmetic; the fused one runs its "lc" steps the
way the emitted HIP does — 64-bit unsigned accumulation of products, fold64, Montgomery
REDC with its final min — asserting that no sum wraps 2^64 and that REDC's input is below
p * 2^32. Inputs are random canonical words and, separately, the largest canonical word
everywhere (the bound the generator plans for)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_accum as G  # noqa: E402

P = G.P
R = 2**32 % P
RINV = pow(2**32, P - 2, P)
NEG_PINV = (-pow(P, -1, 2**32)) % 2**32
M32 = np.uint64(0xFFFFFFFF)


def redc(t):
    assert (t < np.uint64(P) << np.uint64(32)).all(), "REDC input not below p * 2^32"
    m = ((t & M32) * np.uint64(NEG_PINV)) & M32
    r = (t + m * np.uint64(P)) >> np.uint64(32)
    return np.where(r >= P, r - np.uint64(P), r)


def run(prog, bufs, vals, n, fused):
    v = {}
    mask = [np.ones(n, bool)]
    cyc = np.arange(n)
    stores = []
    for ins in prog:
        o = ins[0]
        if o == "c":
            v[ins[1]] = np.full(n, ins[2] % P * R % P, np.uint64)
        elif o == "l":
            _, i, a, col, back = ins
            v[i] = bufs[a][col, (cyc - back) % n].astype(np.uint64)
        elif o == "g":
            v[ins[1]] = np.full(n, bufs[ins[2]][ins[3], 0], np.uint64)
        elif o == "ra":
            for k in range(4):
                v[ins[1 + k]] = vals[:, k].astype(np.uint64)
        elif o == "+":
            v[ins[1]] = (v[ins[2]] + v[ins[3]]) % np.uint64(P)
        elif o == "-":
            v[ins[1]] = (v[ins[2]] + np.uint64(P) - v[ins[3]]) % np.uint64(P)
        elif o == "*":
            v[ins[1]] = (v[ins[2]] * v[ins[3]] % np.uint64(P)) * np.uint64(RINV) % np.uint64(P)
        elif o == "n":
            v[ins[1]] = (np.uint64(P) - v[ins[2]]) % np.uint64(P)
        elif o == "i":
            x = v[ins[2]]
            v[ins[1]] = np.array([pow(int(a), P - 2, P) * R % P * R % P if a else 0 for a in x], np.uint64)
        elif o == "z":
            v[ins[1]] = np.where(v[ins[2]] == 0, R, 0).astype(np.uint64)
        elif o == "lc":
            assert fused
            t = None
            for s in ins[2]:
                if s[0] == "f":
                    t = (t >> np.uint64(32)) * np.uint64(G.FOLD_C) + (t & M32)
                    continue
                y = s[2]
                if isinstance(y, int):
                    ye = v[y]
                elif y[0] == "k":
                    ye = np.full(n, y[1], np.uint64)
                else:
                    ye = np.uint64(P) - v[y[1]]
                term = v[s[1]] * ye
                if t is None:
                    t = term
                else:
                    nt = t + term
                    assert (nt >= t).all(), "64-bit sum wrapped"
                    t = nt
            v[ins[1]] = redc(t)
        elif o == "if":
            mask.append(mask[-1] & (v[ins[1]] != 0))
        elif o == "end":
            mask.pop()
        elif o == "w":
            stores.append((ins[1], ins[2], np.where(mask[-1], v[ins[3]], np.uint64(2**32 - 1))))
        elif o == "wa":
            stores.append(("vals", 0, np.stack([np.where(mask[-1], v[x], 0) for x in ins[1:5]])))
        else:
            raise ValueError(o)
    return stores


def inputs(prog, n, rng, extreme):
    cols = {}
    for ins in prog:
        if ins[0] == "l":
            cols[ins[2]] = max(cols.get(ins[2], 0), ins[3] + 1)
        elif ins[0] == "g":
            cols[ins[2]] = max(cols.get(ins[2], 0), ins[3] + 1)
    if extreme:
        bufs = {a: np.full((c, n), P - 1, np.uint64) for a, c in cols.items()}
        vals = np.full((n, 4), P - 1, np.uint64)
    else:
        bufs = {a: rng.integers(0, P, (c, n), dtype=np.uint64) for a, c in cols.items()}
        vals = rng.integers(0, P, (n, 4), dtype=np.uint64)
    return bufs, vals


@pytest.mark.parametrize("circuit,fn", [("rv32im", "compute"), ("recursion", "compute"), ("recursion", "verify")])
@pytest.mark.parametrize("extreme", [False, True])
def test_fused_sums_store_the_same_words(circuit, fn, extreme):
    prog = G.load(circuit)[fn]
    fused = G.fuse_sums(prog)
    assert sum(i[0] == "lc" for i in fused) > 0.15 * sum(i[0] == "*" for i in prog)
    n = 48
    bufs, vals = inputs(prog, n, np.random.default_rng(7), extreme)
    a = run(prog, bufs, vals, n, False)
    b = run(fused, bufs, vals, n, True)
    assert len(a) == len(b)
    for (ka, ca, xa), (kb, cb, xb) in zip(a, b):
        assert (ka, ca) == (kb, cb)
        np.testing.assert_array_equal(xa, xb)


def test_fused_kernels_emit():
    """the generator emits every circuit's kernels with fusion on"""
    for circuit in G.CIRCUITS:
        fns = {k: G.fuse_sums(v) for k, v in G.load(circuit).items()}
        for name in G.CIRCUITS[circuit][1]:
            ks = G.emit_fn(name, fns[name], 1200, 0, 8, 64)
            assert ks and any("mont_reduce(t" in line for L, _ in ks for line in L)


def test_arm_sorted_kernels_store_each_column_write_once_under_its_guard():
    """the arm-sorted rv32im kernels (gen_accum.py PACK/SORT, the build's default) hold every
    register write of the step exactly once, inside its own arm's `if` (or unguarded, as in
    the IR), and each kernel sorts its tile by its own arms' guards"""
    import re
    prog = G.fuse_sums(G.load("rv32im")["compute"])
    want, guard = [], []
    for ins in prog:
        if ins[0] == "if":
            guard.append(ins[1])
        elif ins[0] == "end":
            guard.pop()
        elif ins[0] == "w":
            want.append((ins[1], ins[2], ins[3], tuple(guard)))
    got = []
    ks = G.emit_fn("compute", prog, 1200, 0, 8, 64, 20000, 256)
    assert len(ks) > 1 and all(own for _, own in ks)
    for L, _ in ks:
        assert any("tile_sort_lane<256>" in line for line in L)
        stack = []
        for line in L:
            m = re.match(r"\s*if \(v(\d+) != 0u\) \{$", line)
            if m:
                stack.append(int(m.group(1)))
            elif line.strip() == "}" and stack:
                stack.pop()
            m = re.match(r"\s*A\.a\[(\d)\]\[uint64_t\((\d+)u\) \* A\.cycles \+ cycle\] = v(\d+);", line)
            if m:
                got.append((int(m.group(1)), int(m.group(2)), int(m.group(3)), tuple(stack)))
    assert sorted(got) == sorted(want)


def test_arm_chunks_merges_non_exclusive_writers_and_readers():
    """arm_chunks keeps in one kernel, in program order, the units that store one column
    under guards that are not provably exclusive, and the units whose cones read a column
    another unit stores; units under exclusive selector literals may split."""
    # v1, v2: two selector loads; g_a = [v1 == 0], g_b = [v1 != 0] (exclusive), g_c = [v2 == 0]
    prog = [
        ("l", 1, 0, 1, 0), ("l", 2, 0, 2, 0), ("l", 3, 0, 3, 0),
        ("z", 10, 1), ("z", 11, 10), ("z", 12, 2),
        ("*", 20, 3, 3), ("*", 21, 20, 3),
        ("if", 10), ("w", 1, 5, 20), ("end",),
        ("if", 11), ("w", 1, 5, 21), ("end",),   # same column, exclusive with the first
        ("if", 12), ("w", 1, 6, 20), ("end",),
        ("if", 12), ("w", 1, 5, 3), ("end",),    # column 5 again, not exclusive with g_a/g_b
        ("l", 30, 1, 6, 1), ("*", 31, 30, 3),
        ("if", 10), ("w", 1, 7, 31), ("end",),   # reads column 6, which the third unit stores
    ]
    out = G.arm_chunks(prog, 10**9)
    assert out is not None
    kern = lambda guard_col: next(k for k, (_, nodes) in enumerate(out)
                                  for n in nodes if n[0] == "if" and (n[1], n[2][0][1][2]) == guard_col)
    assert kern((10, 5)) == kern((12, 5)) == kern((11, 5))  # column 5: non-exclusive pairs merge
    assert kern((12, 6)) == kern((10, 7))                    # column 6: stored by one, read by another
    # one unit per kernel at a tiny cost cap: the merged groups still cannot split
    tiny = G.arm_chunks(prog, 1)
    ks = {}
    for k, (_, nodes) in enumerate(tiny):
        for n in nodes:
            ks.setdefault(k, []).append((n[1], n[2][0][1][2]))
    together = [k for k, us in ks.items() if (10, 5) in us]
    assert together and {(12, 5), (11, 5)} <= set(ks[together[0]])
