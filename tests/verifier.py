"""TEST INFRASTRUCTURE — a Python restatement of the reference STARK verifier
(risc0/zkp/src/verify/{mod.rs,merkle.rs,fri.rs,read_iop.rs}, rv32im wrapper
circuit/rv32im/src/lib.rs:78-92), used to check seals from the HIP prover at sizes the
CPU oracle cannot prove (po2 20-24): transcript replay, every Merkle opening, every FRI
fold and the final polynomial, plus the DEEP-ALI combination of the taps.

The validity check (poly_ext(z) == check(z) * (3z)^N - 1, mod.rs:356-386) only holds
for a witness that satisfies the circuit's constraints; synthetic witnesses do not, so
it is reported separately (`validity`) and the tests check everything else. Hashes and
the Fiat-Shamir RNG come from the CPU oracle (oracle/), field arithmetic is plain
Python integers. Test infrastructure only — never used by the product.
"""
import json
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 15 * 2**27 + 1
RINV = pow(2**32, P - 2, P)
NB = P - 11  # x^4 = -11
QUERIES, INV_RATE, FRI_FOLD, FRI_MIN_DEGREE, CHECK_SIZE = 50, 4, 16, 256, 16
PROOF_SYSTEM_INFO = b"RISC0_STARK:v1__"  # zkp/src/adapter.rs:120


class VerificationError(Exception):
    pass


def _rou(name):
    src = open(os.path.join(ROOT, "risc0_amd", "csrc", "bb31.h")).read()
    body = re.search(name + r"\[28\] = \{([^}]*)\}", src).group(1)
    return [int(x) for x in re.findall(r"\d+", body)]


ROU_FWD, ROU_REV = _rou("kRouFwd"), _rou("kRouRev")


def dec(w):
    return int(w) * RINV % P


def enc(x):
    return (x % P) * 2**32 % P


# ---- FpExt as 4-tuples of plain integers (baby_bear.rs:375-790) ----
def eadd(a, b):
    return tuple((x + y) % P for x, y in zip(a, b))


def esub(a, b):
    return tuple((x - y) % P for x, y in zip(a, b))


def emul(a, b):
    r = [0, 0, 0, 0]
    for i in range(4):
        if a[i]:
            for j in range(4):
                if i + j < 4:
                    r[i + j] += a[i] * b[j]
                else:
                    r[i + j - 4] += NB * a[i] * b[j]
    return tuple(x % P for x in r)


def escal(a, s):
    return tuple(x * s % P for x in a)


def efp(x):
    return (x % P, 0, 0, 0)


def epow(a, n):
    r = (1, 0, 0, 0)
    while n:
        if n & 1:
            r = emul(r, a)
        a = emul(a, a)
        n >>= 1
    return r


def einv(a):
    # baby_bear.rs:448-481 (same formula as risc0_amd/csrc/bb31.h fe_inv)
    a0, a1, a2, a3 = a
    b0 = (a0 * a0 + 11 * (a1 * 2 * a3 - a2 * a2)) % P
    b2 = (a0 * 2 * a2 - a1 * a1 + 11 * a3 * a3) % P
    c = (b0 * b0 + 11 * b2 * b2) % P
    ic = pow(c, P - 2, P)
    b0, b2 = b0 * ic % P, b2 * ic % P
    return ((a0 * b0 + 11 * a2 * b2) % P, (-a1 * b0 + NB * a3 * b2) % P, (-a0 * b2 + a2 * b0) % P,
            (a1 * b2 - a3 * b0) % P)


def poly_eval(coeffs, x):
    tot = (0, 0, 0, 0)
    for c in reversed(coeffs):
        tot = eadd(emul(tot, x), c)
    return tot


def ext_words(words):
    w = [dec(x) for x in words]
    return [tuple(w[4 * i:4 * i + 4]) for i in range(len(w) // 4)]


class ReadIOP:
    """read_iop.rs:20-84"""

    def __init__(self, oracle, seal, suite):
        self.o = oracle
        self.words = np.ascontiguousarray(seal, dtype=np.uint32)
        self.pos = 0
        self.suite = suite
        self.rng = oracle.Rng(suite)

    def read(self, n):
        if self.pos + n > self.words.size:
            raise VerificationError("seal too short")
        out = self.words[self.pos:self.pos + n]
        self.pos += n
        return np.ascontiguousarray(out)

    def commit(self, digest):
        self.rng.mix(digest)

    def random_bits(self, bits):
        return int(self.rng.random_bits(bits))

    def random_elem(self):
        return int(self.rng.random_elem())

    def random_ext_elem(self):
        return tuple(dec(x) for x in self.rng.random_ext_elem())

    def hash_elems(self, words):
        return self.o.hash_elems(self.suite, np.ascontiguousarray(words, dtype=np.uint32))

    def hash_pair(self, a, b):
        return self.o.hash_pair(self.suite, np.ascontiguousarray(a, dtype=np.uint32),
                                np.ascontiguousarray(b, dtype=np.uint32))


class MerkleVerifier:
    """verify/merkle.rs:79-186 with MerkleTreeParams (zkp/src/merkle.rs:36-66)"""

    def __init__(self, iop, row_size, col_size, queries=QUERIES):
        layers = row_size.bit_length() - 1
        assert 1 << layers == row_size
        top_layer = 0
        for i in range(1, layers):
            if (1 << i) > queries:
                break
            top_layer = i
        self.row_size, self.col_size, self.top_size = row_size, col_size, 1 << top_layer
        ts = self.top_size
        self.top = iop.read(ts * 8).reshape(ts, 8)
        self.rest = {}
        for i in reversed(range(ts // 2, ts)):
            self.rest[i] = iop.hash_pair(self.top[2 * i - ts], self.top[2 * i + 1 - ts])
        for i in reversed(range(1, ts // 2)):
            self.rest[i] = iop.hash_pair(self.rest[2 * i], self.rest[2 * i + 1])
        self.root = self.rest[1] if self.rest else self.top[0]
        iop.commit(self.root)

    def verify(self, iop, idx):
        if idx >= self.row_size:
            raise VerificationError("merkle query out of range")
        out = iop.read(self.col_size)
        cur = iop.hash_elems(out)
        idx += self.row_size
        while idx >= 2 * self.top_size:
            low = idx % 2
            other = iop.read(8)
            idx //= 2
            cur = iop.hash_pair(other, cur) if low else iop.hash_pair(cur, other)
        present = self.top[idx - self.top_size] if idx >= self.top_size else self.rest[idx]
        if not np.array_equal(present, cur):
            raise VerificationError("merkle path mismatch")
        return out


class Taps:
    def __init__(self, circuit):
        with open(os.path.join(ROOT, "risc0_amd", "circuits", circuit + ".taps.json")) as f:
            self.d = d = json.load(f)
        self.taps = d["taps"]  # [offset, back, group, combo, skip]
        self.combo_taps, self.combo_begin = d["combo_taps"], d["combo_begin"]
        self.combos_count, self.tot_combo_backs = d["combos_count"], d["tot_combo_backs"]
        self.group_sizes, self.num_taps = d["group_sizes"], d["group_begin"][-1]
        self.regs = []  # (cursor, group, offset, combo, size) — taps.rs:202-224
        cur = 0
        while cur < self.num_taps:
            t = self.taps[cur]
            self.regs.append((cur, t[2], t[0], t[3], t[4]))
            cur += t[4]


def verify(oracle, circuit, seal, suite, check_validity=False):
    """zkp/src/verify/mod.rs:615-680 (+ rv32im lib.rs:78-92). Returns a dict of facts;
    raises VerificationError on any failed check."""
    taps = Taps(circuit)
    if circuit == "rv32im":
        if int(seal[0]) != 2:
            raise VerificationError("bad rv32im seal version")
        seal = seal[1:]
    iop = ReadIOP(oracle, seal, suite)
    iop.commit(iop.hash_elems(np.array([enc(b) for b in PROOF_SYSTEM_INFO], np.uint32)))
    iop.commit(iop.hash_elems(np.array([enc(ord(ch)) for ch in taps.d["circuit_info"]], np.uint32)))
    out_size, mix_size = taps.d["output_size"], taps.d["mix_size"]
    header = iop.read(out_size + 1)
    iop.commit(iop.hash_elems(header))
    po2 = int(header[-1])
    n = 1 << po2
    domain = INV_RATE * n
    merkles = [None, None, None]
    merkles[1] = MerkleVerifier(iop, domain, taps.group_sizes[1])  # code
    merkles[2] = MerkleVerifier(iop, domain, taps.group_sizes[2])  # data
    mix = [iop.random_elem() for _ in range(mix_size)]
    merkles[0] = MerkleVerifier(iop, domain, taps.group_sizes[0])  # accum
    # verify_validity (mod.rs:290-474)
    poly_mix = iop.random_ext_elem()
    check_merkle = MerkleVerifier(iop, domain, CHECK_SIZE)
    z = iop.random_ext_elem()
    back_one = ROU_REV[po2]
    coeff_u_words = iop.read((taps.num_taps + CHECK_SIZE) * 4)
    iop.commit(oracle.hash_ext_elems(suite, coeff_u_words))
    coeff_u = ext_words(coeff_u_words)
    eval_u, pos = [], 0
    for cur, group, offset, combo, size in taps.regs:
        for i in range(size):
            x = escal(z, pow(back_one, taps.taps[cur + i][1], P))
            eval_u.append(poly_eval(coeff_u[pos:pos + size], x))
        pos += size
    nt = taps.num_taps
    check = (0, 0, 0, 0)
    remap = [0, 2, 1, 3]
    for i, rmi in enumerate(remap):
        zi = epow(z, i)
        for k in range(4):
            unit = tuple(1 if j == k else 0 for j in range(4))
            check = eadd(check, emul(emul(coeff_u[nt + rmi + 4 * k], zi), unit))
    check = emul(check, esub(epow(escal(z, 3), n), (1, 0, 0, 0)))
    validity = None
    if check_validity:
        validity = check == poly_ext(circuit, taps, poly_mix, eval_u, header[:out_size], mix)
    fri_mix = iop.random_ext_elem()
    combo_u = [(0, 0, 0, 0)] * (taps.tot_combo_backs + 1)
    cur_mix, pos, tap_mix_pows = (1, 0, 0, 0), 0, []
    for cur, group, offset, combo, size in taps.regs:
        for i in range(size):
            k = taps.combo_begin[combo] + i
            combo_u[k] = eadd(combo_u[k], emul(cur_mix, coeff_u[pos + i]))
        tap_mix_pows.append(cur_mix)
        cur_mix = emul(cur_mix, fri_mix)
        pos += size
    check_mix_pows = []
    for _ in range(CHECK_SIZE):
        combo_u[-1] = eadd(combo_u[-1], emul(cur_mix, coeff_u[pos]))
        pos += 1
        check_mix_pows.append(cur_mix)
        cur_mix = emul(cur_mix, fri_mix)
    gen = ROU_FWD[domain.bit_length() - 1]

    def inner(idx):  # mod.rs:244-283 fri_eval_taps
        x = efp(pow(gen, idx, P))
        rows = [[dec(w) for w in m.verify(iop, idx)] for m in merkles]
        check_row = [dec(w) for w in check_merkle.verify(iop, idx)]
        tot = [(0, 0, 0, 0)] * (taps.combos_count + 1)
        for (cur, group, offset, combo, size), m in zip(taps.regs, tap_mix_pows):
            tot[combo] = eadd(tot[combo], escal(m, rows[group][offset]))
        for i in range(CHECK_SIZE):
            tot[-1] = eadd(tot[-1], escal(check_mix_pows[i], check_row[i]))
        ret = (0, 0, 0, 0)
        for i in range(taps.combos_count):
            num = esub(tot[i], poly_eval(combo_u[taps.combo_begin[i]:taps.combo_begin[i + 1]], x))
            div = (1, 0, 0, 0)
            for back in taps.combo_taps[taps.combo_begin[i]:taps.combo_begin[i + 1]]:
                div = emul(div, esub(x, escal(z, pow(back_one, back, P))))
            ret = eadd(ret, emul(num, einv(div)))
        check_num = esub(tot[-1], combo_u[taps.tot_combo_backs])
        ret = eadd(ret, emul(check_num, einv(esub(x, epow(z, INV_RATE)))))
        return ret

    fri_verify(iop, n, inner)
    if iop.pos != iop.words.size:
        raise VerificationError("trailing words in seal")
    return {"po2": po2, "validity": validity, "words": int(iop.pos)}


def fri_verify(iop, degree, inner):
    """verify/fri.rs:80-155"""
    orig_domain = INV_RATE * degree
    domain = orig_domain
    rounds = []
    while degree > FRI_MIN_DEGREE:
        d = domain // FRI_FOLD
        merkle = MerkleVerifier(iop, d, FRI_FOLD * 4)
        rounds.append((d, merkle, iop.random_ext_elem()))
        domain //= FRI_FOLD
        degree //= FRI_FOLD
    final_words = iop.read(4 * degree)
    iop.commit(iop.hash_elems(final_words))
    final = [dec(w) for w in final_words]
    poly = [tuple(final[j * degree + i] for j in range(4)) for i in range(degree)]
    gen = ROU_FWD[domain.bit_length() - 1]
    inv16 = pow(FRI_FOLD, P - 2, P)
    w16 = ROU_REV[4]
    for _ in range(QUERIES):
        pos = iop.random_bits(orig_domain.bit_length() - 1)
        goal = inner(pos)
        for rdom, merkle, mix in rounds:  # verify_query, fri.rs:52-78
            quot, group = pos // rdom, pos % rdom
            data = [dec(w) for w in merkle.verify(iop, group)]
            data_ext = [tuple(data[j * FRI_FOLD + i] for j in range(4)) for i in range(FRI_FOLD)]
            if data_ext[quot] != goal:
                raise VerificationError("FRI fold mismatch")
            root_po2 = (FRI_FOLD * rdom).bit_length() - 1
            inv_wk = pow(ROU_REV[root_po2], group, P)
            # interpolate_ntt + bit_reverse = natural-order coefficients of the fold
            coeffs = []
            for k in range(FRI_FOLD):
                acc = (0, 0, 0, 0)
                for jj in range(FRI_FOLD):
                    acc = eadd(acc, escal(data_ext[jj], pow(w16, jj * k, P)))
                coeffs.append(escal(acc, inv16))
            goal = poly_eval(coeffs, escal(mix, inv_wk))
            pos = group
        if poly_eval(poly, efp(pow(gen, pos, P))) != goal:
            raise VerificationError("FRI final polynomial mismatch")


def poly_ext(circuit, taps, poly_mix, eval_u, out, mix):
    """The constraint polynomial at z from the tap evaluations, by interpreting the
    circuit's flattened program (risc0_amd/circuits/<c>.poly.ir) over FpExt."""
    import ir_eval
    prog = ir_eval.load_ir(circuit)
    d = taps.d
    names = d["eval_args"]
    gid = {"accum": 0, "code": 1, "data": 2}
    tap_index = {}
    for t_i, t in enumerate(taps.taps):
        tap_index[(t[2], t[0], t[1])] = t_i
    pows = [epow(poly_mix, k) for k in d["poly_mix_powers"]]
    val = {}

    def ext(v):
        return v if isinstance(v, tuple) else efp(v)

    for ins in prog:
        op, i = ins[0], ins[1]
        if op == "c":
            val[i] = efp(ins[2])
        elif op == "e":
            val[i] = tuple(x % P for x in ins[2:6])
        elif op == "l":
            buf, col, back = ins[2:5]
            val[i] = eval_u[tap_index[(gid[names[buf]], col, back)]]
        elif op == "g":
            src = {"mix": mix, "global": [int(x) for x in out]}[names[ins[2]]]
            val[i] = efp(dec(src[ins[3]]))
        elif op == "+":
            val[i] = eadd(ext(val[ins[2]]), ext(val[ins[3]]))
        elif op == "-":
            val[i] = esub(ext(val[ins[2]]), ext(val[ins[3]]))
        elif op == "*":
            val[i] = emul(ext(val[ins[2]]), ext(val[ins[3]]))
        elif op == "a":
            val[i] = eadd(val[ins[2]], emul(ext(val[ins[3]]), pows[ins[4]]))
        elif op == "b":
            val[i] = eadd(val[ins[2]], emul(emul(ext(val[ins[3]]), ext(val[ins[4]])), pows[ins[5]]))
        elif op == "r":
            return ext(val[i])
    raise ValueError("no result")
