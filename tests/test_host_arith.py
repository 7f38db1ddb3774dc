"""Host-side equivalence of the product's lean arithmetic (lazy Montgomery, 64-bit
M_EXT + Barrett Poseidon2, lazy extension multiply) with step-by-step restatements.
Builds tests/native/field_equiv.cpp with g++ against risc0_amd/csrc headers."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_field_and_poseidon2_equivalence(tmp_path):
    exe = tmp_path / "field_equiv"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "risc0_amd", "csrc"), "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "field_equiv.cpp")], check=True)
    out = subprocess.run([str(exe), "50000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("OK")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_bn254_poseidon254_host(tmp_path):
    """The product's 29-bit-limb lazy Montgomery BN254 arithmetic and Poseidon254
    (risc0_amd/csrc/bn254.h, poseidon254.h) against Python integers and p254_ref."""
    import random

    import p254_ref as ref
    exe = tmp_path / "p254_host"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "risc0_amd", "csrc"), "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "p254_host.cpp")], check=True)
    r, R, M = ref.MOD, 2**261, (1 << 29) - 1
    val = lambda ls: sum(int(x) << (29 * i) for i, x in enumerate(ls))
    limbs = lambda x: [(x >> (29 * i)) & M for i in range(9)]
    rnd = random.Random(254)

    def operand(kind):
        # normalised values up to 2.2r, or limbwise sums of two normalised values (limbs < 2^30)
        if kind == "max":
            return [2 * M] * 8 + [2 * (int(2.2 * r) >> 232)]
        if kind == "sum":
            a, b = limbs(rnd.randrange(int(1.1 * r))), limbs(rnd.randrange(r))
            return [x + y for x, y in zip(a, b)]
        return limbs(rnd.choice([0, 1, r - 1, r, int(2.2 * r), rnd.randrange(int(2.2 * r))]))

    lines, checks = [], []
    for t in range(600):
        kind = ["max", "sum", "norm"][t % 3]
        a, b = operand(kind), operand(["sum", "norm", "max"][t % 3])
        lines.append("mul " + " ".join(map(str, a + b)))
        checks.append(("mul", val(a) * val(b)))
        lines.append("sqr " + " ".join(map(str, a)))
        checks.append(("sqr", val(a) ** 2))
        ms = [limbs(rnd.randrange(r)) for _ in range(3)]
        ss = [operand(rnd.choice(["sum", "norm"])) for _ in range(3)]
        c = limbs(rnd.randrange(r))
        lines.append("dot3 " + " ".join(" ".join(map(str, x)) for x in ms + ss + [c]))
        checks.append(("dot3", sum(val(m) * val(s) for m, s in zip(ms, ss)) + val(c) * R))
        x = limbs(rnd.randrange(int(2.2 * r)))
        lines.append("canon " + " ".join(map(str, x)))
        checks.append(("canon", val(x)))
    for n in [0, 1, 8, 9, 16, 17, 32, 40]:
        v = [rnd.choice([0, 1, ref.BB - 1, rnd.randrange(ref.BB)]) for _ in range(n)]
        lines.append("hash %d " % n + " ".join(map(str, v)))
        checks.append(("hash", ref.hash_elems(v)))
    a, b = ref.hash_elems([7]), ref.hash_elems([8, 9])
    lines.append("pair " + " ".join(map(str, a + b)))
    checks.append(("pair", ref.hash_pair(a, b)))
    for _ in range(300):  # random and extreme canonical digests through whole permutations
        a, b = (ref.to_words(rnd.choice([0, r - 1, rnd.randrange(r)])) for _ in range(2))
        lines.append("pair " + " ".join(map(str, a + b)))
        checks.append(("pair", ref.hash_pair(a, b)))
    out = subprocess.run([str(exe)], input="\n".join(lines) + "\n", capture_output=True, text=True, check=True)
    rinv = pow(R, -1, r)
    res = out.stdout.split("\n")
    assert len(res) >= len(checks)
    for (op, want), line in zip(checks, res):
        got = [int(x) for x in line.split()]
        if op in ("hash", "pair"):
            assert got == want, op
            continue
        assert all(x <= M for x in got), (op, got)
        g = val(got)
        if op == "canon":
            assert g == want * rinv % r
        else:
            assert g % r == want * rinv % r, op
            assert g < 2.2 * r, op
