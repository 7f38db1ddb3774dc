"""TEST INFRASTRUCTURE — the reference STARK prover driven through the per-op Hal entry
points, as a Rust `HipHal` behind `risc0_zkp::hal::Hal` would drive them.

This is the call sequence of
  risc0/zkp/src/prove/prover.rs:38-393        (make_coeffs, commit_group, finalize)
  risc0/zkp/src/prove/poly_group.rs:55-83     (PolyGroup::new)
  risc0/zkp/src/prove/merkle.rs:54-140        (MerkleTreeProver::{new, commit, prove})
  risc0/zkp/src/prove/fri.rs:39-126           (ProveRoundInfo, fri_prove)
  risc0/circuit/rv32im/src/prove/hal/mod.rs:143-224 (prove_core: version word, header,
                                               group order; recursion: prove/mod.rs:160-230)
restated over any object with the Hal method names (risc0_amd.HipHal: one C-ABI symbol
per call). Every buffer lives on the device; the host holds what the reference host
holds: the transcript (WriteIOP with the suite's RNG), the out-of-domain evaluations and
the register polynomials. Like the reference, it uses the CPU HashSuite for host-side
hashing and the RNG (`hal.get_hash_suite()`, cuda.rs:974-976) — here the oracle's.
has_unified_memory() is false, so openings go through gather_sample (merkle.rs:111-129)
and every `get_at`/`view` is a device-to-host copy.
Used by tests/test_gpu_parity.py only; never part of the product.
"""
import numpy as np

from verifier import (CHECK_SIZE, FRI_FOLD, FRI_MIN_DEGREE, INV_RATE, P, PROOF_SYSTEM_INFO, QUERIES, ROU_REV, Taps,
                      dec, eadd, einv, emul, enc, epow, escal, esub)


def ewords(vals):
    """host FpExt values (plain ints) -> Montgomery words, AoS"""
    return np.array([enc(c) for v in vals for c in v], dtype=np.uint32)


def log2(n):
    k = n.bit_length() - 1
    assert 1 << k == n
    return k


class WriteIOP:
    """prove/write_iop.rs:24-76"""

    def __init__(self, oracle, suite):
        self.o, self.suite = oracle, suite
        self.proof = []
        self.rng = oracle.Rng(suite)

    def write(self, words):
        self.proof.extend(int(x) for x in np.asarray(words, dtype=np.uint32).reshape(-1))

    def commit(self, digest):
        self.rng.mix(np.ascontiguousarray(digest, dtype=np.uint32))

    def random_elem(self):
        return int(self.rng.random_elem())

    def random_ext_elem(self):
        return tuple(dec(x) for x in self.rng.random_ext_elem())

    def random_bits(self, bits):
        return int(self.rng.random_bits(bits))

    def hash_elems(self, words):
        return self.o.hash_elems(self.suite, np.ascontiguousarray(words, dtype=np.uint32))


class MerkleTreeProver:
    """prove/merkle.rs:26-140 + merkle.rs:39-67 (MerkleTreeParams)"""

    def __init__(self, hal, matrix, rows, cols, queries=QUERIES):
        assert matrix.size == rows * cols
        self.hal, self.matrix, self.rows, self.cols = hal, matrix, rows, cols
        layers = log2(rows)
        top_layer = 0
        for i in range(1, layers):
            if (1 << i) > queries:
                break
            top_layer = i
        self.top_size = 1 << top_layer
        self.nodes = hal.alloc_digest("nodes", rows * 2)
        hal.hash_rows(self.nodes.slice(rows, rows), matrix)
        for i in reversed(range(layers)):
            hal.hash_fold(self.nodes, (1 << i) * 2, 1 << i)
        self.root = self.get_at(1)

    def get_at(self, i):
        return self.nodes.slice(i, 1).to_numpy()

    def commit(self, iop):
        iop.write(self.nodes.slice(self.top_size, self.top_size).to_numpy())
        iop.commit(self.root)

    def prove(self, iop, idx):
        assert idx < self.rows
        sample = self.hal.alloc_elem("sample", self.cols)
        self.hal.gather_sample(sample, self.matrix, idx, self.cols, self.rows)
        out = sample.to_numpy()
        iop.write(out)
        idx += self.rows
        while idx >= 2 * self.top_size:
            low = idx % 2
            idx //= 2
            iop.write(self.get_at(2 * idx + (1 - low)))
        return out


class PolyGroup:
    """prove/poly_group.rs:55-83"""

    def __init__(self, hal, coeffs, count, size):
        assert coeffs.size == count * size
        domain = size * INV_RATE
        self.coeffs, self.count = coeffs, count
        self.evaluated = hal.alloc_elem("evaluated", count * domain)
        hal.batch_expand_into_evaluate_ntt(self.evaluated, coeffs, count, log2(INV_RATE))
        hal.batch_bit_reverse(coeffs, count)
        self.merkle = MerkleTreeProver(hal, self.evaluated, domain, count)


def poly_divide(p, z):
    """core/poly.rs:81-89: in-place division by (x - z), returns the remainder"""
    cur = (0, 0, 0, 0)
    for i in reversed(range(len(p))):
        nxt = eadd(emul(z, cur), p[i])
        p[i] = cur
        cur = nxt
    return cur


def poly_eval(c, x):
    tot, mul = (0, 0, 0, 0), (1, 0, 0, 0)
    for ci in c:
        tot = eadd(tot, emul(ci, mul))
        mul = emul(mul, x)
    return tot


def poly_interpolate(out, xs, fxs, size):
    """core/poly.rs:41-78 (clears out[0..len) like the reference)"""
    if size == 1:
        out[0] = fxs[0]
        return
    if size == 2:
        out[1] = emul(esub(fxs[1], fxs[0]), einv(esub(xs[1], xs[0])))
        out[0] = esub(fxs[0], emul(out[1], xs[0]))
        return
    ft = [(0, 0, 0, 0)] * (size + 1)
    ft[0] = (1, 0, 0, 0)
    for i in range(size):
        for j in reversed(range(i + 1)):
            value = ft[j]
            ft[j + 1] = eadd(ft[j + 1], value)
            ft[j] = emul(ft[j], esub((0, 0, 0, 0), xs[i]))
    for i in range(len(out)):
        out[i] = (0, 0, 0, 0)
    for i in range(size):
        fr = list(ft)
        poly_divide(fr, xs[i])
        mul = emul(fxs[i], einv(poly_eval(fr, xs[i])))
        for j in range(size):
            out[j] = eadd(out[j], emul(mul, fr[j]))


class Prover:
    """prove/prover.rs:28-393 over a Hal"""

    def __init__(self, oracle, hal, circuit):
        self.o, self.hal, self.circuit = oracle, hal, circuit
        self.taps = Taps(circuit)
        self.iop = WriteIOP(oracle, hal.suite)
        self.groups = [None, None, None]
        self.po2 = self.cycles = None

    def set_po2(self, po2):
        self.po2, self.cycles = po2, 1 << po2

    def commit_group(self, g, witness):
        gs = self.taps.group_sizes[g]
        assert witness.size == gs * self.cycles
        coeffs = self.hal.alloc_elem("coeffs", witness.size)  # make_coeffs, prover.rs:38-48
        self.hal.eltwise_copy_elem(coeffs, witness)
        self.hal.batch_interpolate_ntt(coeffs, gs)
        self.hal.zk_shift(coeffs, gs)
        self.groups[g] = PolyGroup(self.hal, coeffs, gs, self.cycles)
        self.groups[g].merkle.commit(self.iop)

    def finalize(self, mix_buf, global_buf):
        hal, taps, iop = self.hal, self.taps, self.iop
        poly_mix = iop.random_ext_elem()
        domain = self.cycles * INV_RATE
        check = hal.alloc_elem("check_poly", 4 * domain)
        hal.eval_check(self.circuit, check, [g.evaluated for g in self.groups], mix_buf, global_buf,
                       ewords([poly_mix]), self.po2)
        hal.batch_interpolate_ntt(check, 4)
        check_group = PolyGroup(hal, check, CHECK_SIZE, self.cycles)
        check_group.merkle.commit(iop)
        z = iop.random_ext_elem()
        back_one = ROU_REV[self.po2]
        all_xs, eval_u = [], []
        for gid, pg in enumerate(self.groups):
            which, xs = [], []
            for t in range(taps.d["group_begin"][gid], taps.d["group_begin"][gid + 1]):
                which.append(taps.taps[t][0])
                x = escal(z, pow(back_one, taps.taps[t][1], P))
                xs.append(x)
                all_xs.append(x)
            dw = hal.copy_from_u32("which", np.array(which, np.uint32))
            dx = hal.copy_from_extelem("xs", ewords(xs))
            out = hal.alloc_extelem("out", len(which))
            hal.batch_evaluate_any(pg.coeffs, pg.count, dw, dx, out)
            w = out.to_numpy()
            eval_u += [tuple(dec(x) for x in w[4 * i:4 * i + 4]) for i in range(len(which))]
        coeff_u = [(0, 0, 0, 0)] * len(eval_u)
        pos = 0
        for cur, group, offset, combo, size in taps.regs:
            seg = coeff_u[pos:]
            poly_interpolate(seg, all_xs[pos:], eval_u[pos:], size)
            coeff_u[pos:] = seg
            pos += size
        z_pow = epow(z, 4)
        dw = hal.copy_from_u32("which", np.arange(CHECK_SIZE, dtype=np.uint32))
        dx = hal.copy_from_extelem("xs", ewords([z_pow] * CHECK_SIZE))
        out = hal.alloc_extelem("out", CHECK_SIZE)
        hal.batch_evaluate_any(check_group.coeffs, CHECK_SIZE, dw, dx, out)
        w = out.to_numpy()
        coeff_u += [tuple(dec(x) for x in w[4 * i:4 * i + 4]) for i in range(CHECK_SIZE)]
        cu = ewords(coeff_u)
        iop.write(cu)
        iop.commit(self.o.hash_ext_elems(iop.suite, cu))
        mix = iop.random_ext_elem()
        combo_count = taps.combos_count
        combos = hal.alloc_extelem_zeroed("combos", self.cycles * (combo_count + 1))
        cur_mix = (1, 0, 0, 0)
        for gid, pg in enumerate(self.groups):
            gs = taps.group_sizes[gid]
            which = np.array([combo for cur, group, offset, combo, size in taps.regs if group == gid], np.uint32)
            assert which.size == gs
            hal.mix_poly_coeffs(combos, ewords([cur_mix]), ewords([mix]), pg.coeffs, which, gs, self.cycles)
            cur_mix = emul(cur_mix, epow(mix, gs))
        hal.mix_poly_coeffs(combos, ewords([cur_mix]), ewords([mix]), check_group.coeffs,
                            np.full(CHECK_SIZE, combo_count, np.uint32), CHECK_SIZE, self.cycles)
        reg_sizes = np.array([r[4] for r in taps.regs], np.uint32)
        reg_combo_ids = np.array([r[3] for r in taps.regs], np.uint32)
        hal.combos_prepare(combos, cu, combo_count, self.cycles, reg_sizes, reg_combo_ids, ewords([mix]))
        pows, begin = [], [0]
        for i in range(combo_count):
            for back in taps.combo_taps[taps.combo_begin[i]:taps.combo_begin[i + 1]]:
                pows.append(escal(z, pow(back_one, back, P)))
            begin.append(len(pows))
        pows.append(z_pow)
        begin.append(len(pows))
        bad = hal.combos_divide(combos, ewords(pows), np.array(begin, np.uint32), self.cycles)
        assert bad < 0, f"combos_divide: nonzero remainder in chunk {bad}"
        final = hal.alloc_elem("final_poly_coeffs", self.cycles * 4)
        hal.eltwise_sum_extelem(final, combos)
        hal.batch_bit_reverse(final, 4)
        self.fri_prove(final, check_group)
        return np.array(iop.proof, dtype=np.uint32)

    def fri_prove(self, coeffs, check_group):
        """fri.rs:86-126"""
        hal, iop = self.hal, self.iop
        orig_domain = coeffs.size // 4 * INV_RATE
        rounds = []
        while coeffs.size // 4 > FRI_MIN_DEGREE:
            size = coeffs.size // 4
            domain = size * INV_RATE
            evaluated = hal.alloc_elem("evaluated", domain * 4)
            hal.batch_expand_into_evaluate_ntt(evaluated, coeffs, 4, log2(INV_RATE))
            merkle = MerkleTreeProver(hal, evaluated, domain // FRI_FOLD, FRI_FOLD * 4)
            merkle.commit(iop)
            fold_mix = iop.random_ext_elem()
            out = hal.alloc_elem("out_coeffs", size // FRI_FOLD * 4)
            hal.fri_fold(out, coeffs, ewords([fold_mix]))
            rounds.append((domain, merkle, evaluated))
            coeffs = out
        final = hal.alloc_elem("final_coeffs", coeffs.size)
        hal.eltwise_copy_elem(final, coeffs)
        hal.batch_bit_reverse(final, 4)
        fw = final.to_numpy()
        iop.write(fw)
        iop.commit(iop.hash_elems(fw))
        for _ in range(QUERIES):
            pos = iop.random_bits(log2(orig_domain))
            for pg in self.groups:
                pg.merkle.prove(iop, pos)
            check_group.merkle.prove(iop, pos)
            for domain, merkle, _ in rounds:
                group = pos % (domain // FRI_FOLD)
                merkle.prove(iop, group)
                pos = group


def prove_segment(oracle, hal, circuit, po2, code, data, accum, glob, accumulate=None):
    """rv32im prove_core (circuit/rv32im/src/prove/hal/mod.rs:143-224) / recursion
    (circuit/recursion/src/prove/mod.rs:160-230) over device witness buffers. The mix is
    drawn from the transcript after code and data are committed; `accum` is taken as given,
    or filled by accumulate(mix_buf, mix) between the mix draw and the accum commit (the
    circuit HAL's accumulation, witgen/mod.rs:178-221). Returns (seal, mix)."""
    p = Prover(oracle, hal, circuit)
    if circuit == "rv32im":
        p.iop.write([2])  # RV32IM_SEAL_VERSION
    p.iop.commit(p.iop.hash_elems([enc(b) for b in PROOF_SYSTEM_INFO]))
    p.iop.commit(p.iop.hash_elems([enc(ord(ch)) for ch in p.taps.d["circuit_info"]]))
    g = glob.to_numpy()  # global.view_mut: INVALID -> 0, written back
    g = np.where(g >= P, 0, g).astype(np.uint32)
    glob.copy_from(g)
    header = np.concatenate([g, np.array([po2], np.uint32)])  # po2 as a raw word
    p.iop.commit(p.iop.hash_elems(header))
    p.iop.write(header)
    p.set_po2(po2)
    p.commit_group(1, code)
    p.commit_group(2, data)
    mix = np.array([p.iop.random_elem() for _ in range(p.taps.d["mix_size"])], np.uint32)
    mix_buf = hal.copy_from_elem("mix", mix)
    if accumulate is not None:
        accumulate(mix_buf, mix)
    p.commit_group(0, accum)
    return p.finalize(mix_buf, glob), mix
