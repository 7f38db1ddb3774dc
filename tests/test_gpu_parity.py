"""GPU parity: every HIP HAL op against the CPU oracle on identical seeded inputs.

Mirrors the reference's DualHal tests (risc0/zkp/src/hal/mod.rs:319-616, shapes
noted per test) plus what DualHal does not cover (combos_prepare/combos_divide,
eval_check, whole-segment seals). The bar is bit-exact equality of u32 words.
"""
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P = 15 * 2**27 + 1


@pytest.fixture(scope="module")
def hal():
    return H("poseidon2")


@pytest.fixture(scope="module")
def hal_sha():
    return H("sha-256")


_HALS = {}


def H(suite):
    """one HipHal per hash suite ("poseidon2", "sha-256", "poseidon_254"), made on first use"""
    import risc0_amd as r
    if suite not in _HALS:
        _HALS[suite] = r.HipHal(suite)
    return _HALS[suite]


def S(oracle, suite):
    return {"poseidon2": oracle.POSEIDON2, "sha-256": oracle.SHA256, "poseidon_254": oracle.POSEIDON254}[suite]


def rnd(oracle, seed, n):
    return oracle.rand_elems(np.random.default_rng(seed), n)


def dev(hal, a):
    return hal.copy_from_elem("x", a)


@pytest.mark.parametrize("count,log_n", [(224, 14), (224, 12), (3, 1), (5, 2), (7, 5), (1, 10), (2, 11), (4, 14), (1, 20)])
def test_batch_bit_reverse(hal, oracle, count, log_n):
    # hal/mod.rs:354-366 (224 x 2^14)
    a = rnd(oracle, 1, count << log_n)
    d = dev(hal, a)
    hal.batch_bit_reverse(d, count)
    oracle.batch_bit_reverse(a, count)
    assert np.array_equal(d.to_numpy(), a)


@pytest.mark.parametrize("count,log_in", [(224, 16), (224, 12), (1, 1), (3, 2), (5, 8), (2, 10), (9, 11), (4, 16), (1, 20)])
def test_batch_expand_into_evaluate_ntt(hal, oracle, count, log_in):
    # hal/mod.rs:389-404 (224 x 2^16 -> 2^18)
    a = rnd(oracle, 2, count << log_in)
    out = hal.alloc_elem("out", count << (log_in + 2))
    hal.batch_expand_into_evaluate_ntt(out, dev(hal, a), count, 2)
    ref = np.zeros(count << (log_in + 2), np.uint32)
    oracle.batch_expand_into_evaluate_ntt(ref, a, count, 2)
    assert np.array_equal(out.to_numpy(), ref)


@pytest.mark.parametrize("count,log_n", [(224, 18), (224, 14), (1, 1), (3, 3), (2, 12), (3, 13), (1, 17), (2, 22)])
def test_batch_interpolate_ntt(hal, oracle, count, log_n):
    # hal/mod.rs:406-418 (224 x 2^18)
    a = rnd(oracle, 3, count << log_n)
    d = dev(hal, a)
    hal.batch_interpolate_ntt(d, count)
    oracle.batch_interpolate_ntt(a, count)
    assert np.array_equal(d.to_numpy(), a)


@pytest.mark.parametrize("log_n", [22, 24, 26])
def test_ntt_roundtrip_full_size(hal, oracle, log_n):
    # size-independent property at prover sizes (po2 = 20 and 24 domains):
    # interpolate, bit-reverse back to natural order, re-evaluate == identity
    a = rnd(oracle, 4, 1 << log_n)
    d = dev(hal, a)
    hal.batch_interpolate_ntt(d, 1)
    hal.batch_bit_reverse(d, 1)
    hal.batch_bit_reverse(d, 1)
    out = hal.alloc_elem("out", 1 << log_n)
    hal.batch_expand_into_evaluate_ntt(out, d, 1, 0)
    assert np.array_equal(out.to_numpy(), a)


@pytest.mark.parametrize("poly_count,log_n", [(1000, 8), (900, 12), (3, 1), (1, 20)])
def test_zk_shift(hal, oracle, poly_count, log_n):
    # hal/mod.rs:605-615
    a = rnd(oracle, 5, poly_count << log_n)
    d = dev(hal, a)
    hal.zk_shift(d, poly_count)
    oracle.zk_shift(a, poly_count)
    assert np.array_equal(d.to_numpy(), a)


@pytest.mark.parametrize("poly_count,log_n,evals,kind", [
    (223, 16, 865, "reference"),  # hal/mod.rs:368-387 exactly: which = 0, every x = z^4
    (223, 16, 865, "mixed"),      # every polynomial, distinct points
    (16, 20, 16, "check"),        # the prover's check evaluation (prover.rs:253-262): 16 x 2^20 at z^4
    (223, 12, 865, "mixed"),
    (3, 1, 5, "mixed"),           # shorter than one 64-coefficient lane chunk
])
def test_batch_evaluate_any(hal, oracle, poly_count, log_n, evals, kind):
    # polynomials longer than one 16384-coefficient chunk (log_n >= 15) go through the
    # multi-chunk Horner combine (eltwise.hip)
    rng = np.random.default_rng(6)
    coeffs = oracle.rand_elems(rng, poly_count << log_n)
    if kind == "mixed":
        which = rng.integers(0, poly_count, evals).astype(np.uint32)
        xs = oracle.rand_elems(rng, 4 * evals)
    else:
        which = (np.zeros(evals) if kind == "reference" else np.arange(evals)).astype(np.uint32)
        z = oracle.rand_elems(rng, 4)
        zp = z
        for _ in range(3):
            zp = oracle.ext_mul(zp, z)
        xs = np.tile(zp, evals).astype(np.uint32)
    out = hal.alloc_extelem("out", evals)
    hal.batch_evaluate_any(dev(hal, coeffs), poly_count, dev(hal, which), hal.copy_from_extelem("xs", xs), out)
    ref = np.zeros(4 * evals, np.uint32)
    oracle.batch_evaluate_any(coeffs, poly_count, which, xs, ref)
    assert np.array_equal(out.to_numpy(), ref)


@pytest.mark.parametrize("count", [1, 9, 12, 1001, 1024, 1025, 1 << 20])
def test_fri_fold(hal, oracle, count):
    # hal/mod.rs:507-520 (COUNTS)
    rng = np.random.default_rng(7)
    inp = oracle.rand_elems(rng, count * 4 * 16)
    mix = oracle.rand_elems(rng, 4)
    out = hal.alloc_elem("out", count * 4)
    hal.fri_fold(out, dev(hal, inp), mix)
    ref = np.zeros(count * 4, np.uint32)
    oracle.fri_fold(ref, inp, mix)
    assert np.array_equal(out.to_numpy(), ref)


@pytest.mark.parametrize("combos_kind", ["zeros", "spread"])
def test_mix_poly_coeffs(hal, oracle, combos_kind):
    # hal/mod.rs:522-549 (combo_count 100, steps 2^12, CHECK_SIZE inputs)
    rng = np.random.default_rng(8)
    combo_count, steps = 100, 1 << 12
    input_size = 16 if combos_kind == "zeros" else 40
    combos = (np.zeros(input_size) if combos_kind == "zeros" else rng.integers(0, 6, input_size)).astype(np.uint32)
    inp = oracle.rand_elems(rng, input_size * steps)
    start = oracle.rand_elems(rng, 4)
    mix = oracle.rand_elems(rng, 4)
    init = oracle.rand_elems(rng, 4 * steps * (combo_count + 1))
    out = hal.copy_from_extelem("out", init)
    hal.mix_poly_coeffs(out, start, mix, dev(hal, inp), combos, input_size, steps)
    ref = init.copy()
    oracle.mix_poly_coeffs(ref, start, mix, inp, combos, input_size, steps)
    assert np.array_equal(out.to_numpy(), ref)


def test_eltwise_ops(hal, oracle):
    # hal/mod.rs:452-505 (COUNTS; sum_extelem 2^20)
    rng = np.random.default_rng(9)
    for count in [1, 9, 12, 1001, 1024, 1025, 1 << 20]:
        a, b = oracle.rand_elems(rng, count), oracle.rand_elems(rng, count)
        o = hal.alloc_elem("o", count)
        hal.eltwise_add_elem(o, dev(hal, a), dev(hal, b))
        ref = np.zeros(count, np.uint32)
        oracle.eltwise_add_elem(ref, a, b)
        assert np.array_equal(o.to_numpy(), ref)
        hal.eltwise_copy_elem(o, dev(hal, a))
        assert np.array_equal(o.to_numpy(), a)
    z = oracle.rand_elems(rng, 5000)
    z[::7] = 0xFFFFFFFF
    dz = dev(hal, z)
    hal.eltwise_zeroize_elem(dz)
    oracle.eltwise_zeroize_elem(z)
    assert np.array_equal(dz.to_numpy(), z)
    count = 1 << 20
    for to_add in (1, 5):
        inp = oracle.rand_elems(rng, 4 * count * to_add)
        out = hal.alloc_elem("out", 4 * count)
        hal.eltwise_sum_extelem(out, hal.copy_from_extelem("in", inp))
        ref = np.zeros(4 * count, np.uint32)
        oracle.eltwise_sum_extelem(ref, inp)
        assert np.array_equal(out.to_numpy(), ref)


def test_gather_scatter_slice_prefix(hal, oracle):
    rng = np.random.default_rng(10)
    # hal/mod.rs:420-444
    rows, cols, idx = 1000, 900, 400
    src = oracle.rand_elems(rng, rows * cols)
    dst = hal.alloc_elem("dst", rows)
    hal.gather_sample(dst, dev(hal, src), idx, rows, cols)
    assert np.array_equal(dst.to_numpy(), src.reshape(rows, cols)[:, idx])
    # the same straight to the host (r0hip_gather_sample_host), and a Merkle-opening shape:
    # 211 columns of a 2^16-row matrix at the last row
    dsrc = dev(hal, src)
    assert np.array_equal(hal.gather_sample_host(dsrc, idx, rows, cols), src.reshape(rows, cols)[:, idx])
    assert hal.gather_sample_host(dsrc, idx, 0, cols).size == 0
    m = oracle.rand_elems(rng, 211 << 16)
    assert np.array_equal(hal.gather_sample_host(dev(hal, m), (1 << 16) - 1, 211, 1 << 16),
                          m.reshape(211, 1 << 16)[:, -1])
    # scatter (cpu.rs:598-615): CSR per cycle
    cycles = 300
    counts = rng.integers(0, 5, cycles)
    index = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint32)
    offsets = rng.permutation(4096)[: index[-1]].astype(np.uint32)
    values = oracle.rand_elems(rng, index[-1])
    into = oracle.rand_elems(rng, 4096)
    d = dev(hal, into)
    hal.scatter(d, index, offsets, values)
    oracle.scatter(into, index, offsets, values)
    assert np.array_equal(d.to_numpy(), into)
    hal.scatter(d, np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.uint32))  # empty: no-op
    # eltwise_copy_elem_slice (cpu.rs:617-635)
    frm = oracle.rand_elems(rng, 50 * 40)
    into = oracle.rand_elems(rng, 4000)
    d = dev(hal, into)
    hal.eltwise_copy_elem_slice(d, frm, 20, 7, 3, 40, 11, 60)
    oracle.eltwise_copy_elem_slice(into, frm, 20, 7, 3, 40, 11, 60)
    assert np.array_equal(d.to_numpy(), into)
    # prefix_products (cpu.rs:637-642, KAT at cpu.rs:735-753)
    io = oracle.rand_elems(rng, 4 * 777)
    d = hal.copy_from_extelem("io", io)
    hal.prefix_products(d)
    oracle.prefix_products(io)
    assert np.array_equal(d.to_numpy(), io)


@pytest.mark.parametrize("suite", ["poseidon2", "sha-256", "poseidon_254"])
def test_hash_rows(hal, hal_sha, oracle, suite):
    # hal/mod.rs:575-589 (rows {1,2,3,4,10} x cols {16,32,64,128}) + ragged column counts
    h, s = H(suite), S(oracle, suite)
    rng = np.random.default_rng(11)
    shapes = [(r, c) for r in (1, 2, 3, 4, 10) for c in (16, 32, 64, 128)]
    shapes += [(4096, 1), (4096, 211), (1000, 103), (257, 17), (1 << 16, 16), (4097, 1), (1001, 12), (513, 16)]
    for rows, cols in shapes:
        m = oracle.rand_elems(rng, rows * cols)
        out = h.alloc_digest("out", rows)
        h.hash_rows(out, dev(h, m))
        ref = np.zeros(rows * 8, np.uint32)
        oracle.hash_rows(s, ref, m)
        assert np.array_equal(out.to_numpy(), ref), (rows, cols)
    # hal/mod.rs:591-603: hash into a slice of a larger node buffer
    rows, cols = 4096, 256
    m = oracle.rand_elems(rng, rows * cols)
    nodes = h.alloc_digest("nodes", rows * 2)
    h.hash_rows(nodes.slice(rows, rows), dev(h, m))
    ref = np.zeros(rows * 8, np.uint32)
    oracle.hash_rows(s, ref, m)
    assert np.array_equal(nodes.to_numpy()[rows * 8:], ref)


@pytest.mark.parametrize("suite,inputs", [("poseidon2", 1024), ("sha-256", 1024), ("poseidon_254", 1024),
                                          ("poseidon2", 1 << 17)])
def test_hash_fold(hal, hal_sha, oracle, suite, inputs):
    # hal/mod.rs:551-573 (1024 inputs; digests of reduced words for Poseidon2); 2^17
    # inputs cross the Poseidon2 one-quad-per-node threshold (layers <= 32768 nodes)
    h, s = H(suite), S(oracle, suite)
    rng = np.random.default_rng(12)
    io = np.zeros(inputs * 2 * 8, np.uint32)
    io[inputs * 8:] = (rng.integers(0, 2**32, inputs * 8, dtype=np.uint64) // 3).astype(np.uint32)
    if suite == "poseidon_254":  # digests are canonical BN254 Fr values (< r < 2^254, mod.rs:94-98)
        io[inputs * 8 + 7::8] &= 0x0FFFFFFF
    d = h.copy_from_digest("io", io)
    layer = inputs
    while layer > 1:
        h.hash_fold(d, layer, layer // 2)
        oracle.hash_fold(s, io, layer, layer // 2)
        layer //= 2
    assert np.array_equal(d.to_numpy(), io)


@pytest.mark.parametrize("suite", ["poseidon2", "sha-256"])
@pytest.mark.parametrize("rows,cols,pattern", [
    (4096, 1, "zero"), (4096, 16, "zero"), (1 << 17, 1, "zero"), (4096, 211, "zero"),
    (1 << 16, 1, "half"), (4096, 1, "one"), (4096, 16, "blocks"), (1 << 17, 1, "sparse"),
    (1 << 15, 17, "blocks"), (2, 1, "zero"), (1, 1, "zero")])
def test_merkle_tree_zero_subtrees(hal, hal_sha, oracle, suite, rows, cols, pattern):
    """r0hip_merkle_tree (MerkleTreeProver::new in one call, prove/merkle.rs:54-81) equals the
    oracle's hash_rows + hash_fold of every layer. Zero rows exercise the zero-subtree
    path (hash.hip, ZeroSub; Poseidon2 and SHA-256): whole trees of zero rows (rv32im's code group), zero halves, one
    nonzero row, 64-row and misaligned 96-row runs that give waves of mixed hits, and sparse rows."""
    h, s = H(suite), S(oracle, suite)
    rng = np.random.default_rng(rows * 31 + cols)
    m = oracle.rand_elems(rng, rows * cols).reshape(cols, rows)
    if pattern == "zero":
        m[:] = 0
    elif pattern == "half":
        m[:, : rows // 2] = 0
    elif pattern == "one":
        m[:] = 0
        m[:, 777] = 1
    elif pattern == "blocks":
        idx = np.arange(rows)
        m[:, ((idx // 64) % 2 == 0) | ((idx // 96) % 3 == 1)] = 0
    elif pattern == "sparse":
        m[:, rng.random(rows) > 0.01] = 0
    m = np.ascontiguousarray(m).reshape(-1)
    nodes = h.alloc_digest("nodes", rows * 2)
    h.merkle_tree(nodes, dev(h, m), rows)
    io = np.zeros(rows * 2 * 8, np.uint32)
    leaves = np.zeros(rows * 8, np.uint32)
    oracle.hash_rows(s, leaves, m)
    io[rows * 8:] = leaves
    layer = rows
    while layer > 1:
        oracle.hash_fold(s, io, layer, layer // 2)
        layer //= 2
    assert np.array_equal(nodes.to_numpy()[8:], io[8:])
    # the per-op form (hash_rows into the heap's leaf range, then hash_fold per layer, as
    # MerkleTreeProver::new drives a HAL): the library's heap note gives the folds their height
    ops = h.alloc_digest("nodes_ops", rows * 2)
    h.hash_rows(ops.slice(rows, rows), dev(h, m))
    layer = rows
    while layer > 1:
        h.hash_fold(ops, layer, layer // 2)
        layer //= 2
    assert np.array_equal(ops.to_numpy()[8:], io[8:])
    # degenerate folds on a noted heap: an empty fold is a no-op, a bad size is reported
    h.hash_fold(ops, 0, 0)
    with pytest.raises(Exception):
        h.hash_fold(ops, 6, 4)
    # the same heap refilled with other leaves (a stale note): still the oracle's words
    if rows >= 4:
        other = rng.integers(0, 2**32, rows * 8, dtype=np.uint64).astype(np.uint32) // 3
        if suite == "poseidon2":
            other[: rows * 4] = 0  # half the leaves equal to no Z_k: words, not zero digests
        io2 = np.zeros(rows * 2 * 8, np.uint32)
        io2[rows * 8:] = other
        ops.copy_from(io2)  # same base as the noted heap
        layer = rows
        while layer > 1:
            h.hash_fold(ops, layer, layer // 2)
            oracle.hash_fold(s, io2, layer, layer // 2)
            layer //= 2
        assert np.array_equal(ops.to_numpy()[8:], io2[8:])


@pytest.mark.parametrize("po2,last", [(4, 16), (10, 1000), (12, 4096), (20, (1 << 20) - 7), (16, 1), (13, 4097)])
def test_rv32im_accum_finalize(hal, oracle, po2, last):
    # accumulation phases 2-3 (rv32im-sys/kernels/cxx/ffi.cpp:326-360): 103 accum columns,
    # prefix sums over [0, last) including ragged tiles and a single row; rows past `last` untouched
    rows, cols = 1 << po2, 103
    a = rnd(oracle, 40 + po2, rows * cols)
    d = dev(hal, a)
    hal.rv32im_accum_finalize(d, rows, cols, last)
    ref = a.copy()
    oracle.rv32im_accum_finalize(ref, rows, cols, 23, last)
    assert np.array_equal(d.to_numpy(), ref)


@pytest.mark.parametrize("po2,last", [(10, 1024), (12, 3000), (14, 1 << 14)])
def test_rv32im_accum_finalize_matches_reference(hal, po2, last):
    """Phases 2-3 on the GPU against the compiled reference itself: the reference's phase-1
    output (stepAccum on random data rows, accum allocated all-INVALID as the prover does)
    finished by r0hip_rv32im_accum_finalize equals the reference's whole
    risc0_circuit_rv32im_cpu_accum (ffi.cpp:313-368)."""
    import rv32im_accum_ref as R
    if not R.available():
        pytest.skip("oracle/_ref/libref_rv32im_accum.so not built")
    rows = 1 << po2
    rng = np.random.default_rng(po2 * 7 + last)
    draw = lambda n: rng.integers(0, R.P, n, dtype=np.uint64).astype(np.uint32)
    data, glob, mix = draw(R.DATA_COLS * rows), draw(R.GLOBAL_WORDS), draw(R.MIX_WORDS)
    p1 = R.accum(data, glob, mix, rows, last, phase1_only=True)
    full = R.accum(data, glob, mix, rows, last)
    d = dev(hal, p1)
    hal.rv32im_accum_finalize(d, rows, R.ACCUM_COLS, last)
    assert np.array_equal(d.to_numpy(), full)


@pytest.mark.parametrize("po2,last", [(10, 1024), (12, 3000), (20, 1 << 20)])
def test_rv32im_accum_matches_reference(hal, po2, last):
    """The whole rv32im accumulation on the GPU (r0hip_rv32im_accum: the generated
    per-cycle step, then the scan and finalize) against the compiled reference's
    risc0_circuit_rv32im_cpu_accum (ffi.cpp:313-368) on random data rows, each taking one of
    the 13 instruction arms (tests/test_rv32im_accum_ir.py:rows_for_arms)."""
    import rv32im_accum_ref as R
    from test_rv32im_accum_ir import rows_for_arms
    if not R.available():
        pytest.skip("oracle/_ref/libref_rv32im_accum.so not built")
    rows = 1 << po2
    rng = np.random.default_rng(po2 * 31 + last)
    data = rows_for_arms(rng, rows, list(rng.integers(0, 13, rows)))
    glob = rng.integers(0, R.P, R.GLOBAL_WORDS, dtype=np.uint64).astype(np.uint32)
    mix = rng.integers(0, R.P, R.MIX_WORDS, dtype=np.uint64).astype(np.uint32)
    ref = R.accum(data, glob, mix, rows, last)
    d_acc = dev(hal, np.full(R.ACCUM_COLS * rows, R.INVALID, np.uint32))
    hal.rv32im_accum(dev(hal, data), d_acc, dev(hal, glob), dev(hal, mix), rows, last)
    got = d_acc.to_numpy()
    bad = np.nonzero(got != ref)[0]
    assert bad.size == 0, f"{bad.size} words differ, first at column {bad[0] // rows} row {bad[0] % rows}"


def test_combos_prepare_and_divide(hal, oracle):
    # hal/mod.rs:202-257: prepare, then divide by (x - z*w^-back); remainders must vanish.
    # Build combos whose rows have the required roots by construction.
    rng = np.random.default_rng(13)
    for cycles in (1 << 10, 1 << 16, 8):
        combos_count = 4
        mix = oracle.rand_elems(rng, 4)
        reg_sizes = np.array([1, 2, 3, 2, 1, 6, 1], np.uint32)
        reg_ids = np.array([0, 1, 2, 3, 0, 2, 1], np.uint32)
        coeff_u = oracle.rand_elems(rng, 4 * (int(reg_sizes.sum()) + 16))
        combos = oracle.rand_elems(rng, 4 * cycles * (combos_count + 1))
        d = hal.copy_from_extelem("combos", combos)
        hal.combos_prepare(d, coeff_u, combos_count, cycles, reg_sizes, reg_ids, mix)
        oracle.combos_prepare(combos, coeff_u, combos_count, cycles, reg_sizes, reg_ids, mix)
        assert np.array_equal(d.to_numpy(), combos)
        # divide: nonzero remainders are reported identically (first bad chunk)
        pows = oracle.rand_elems(rng, 4 * 7)
        begin = np.array([0, 1, 3, 3, 6, 7], np.uint32)
        bad_gpu = hal.combos_divide(d, pows, begin, cycles)
        bad_ref = oracle.combos_divide(combos, pows, begin, cycles)
        assert bad_gpu == bad_ref
        assert np.array_equal(d.to_numpy(), combos)


def test_poly_divide_exact(hal, oracle):
    """A polynomial with root z divides exactly (poly_divide, core/poly.rs:81-89): p = q(x)(x - z)
    for a random q of degree n - 2 comes back as q with a zero remainder (no bad chunk), and
    the same p plus one leaves the nonzero remainder reported."""
    import poly_ext_def as D
    rng = np.random.default_rng(14)
    n = 1 << 20
    q = oracle.rand_elems(rng, 4 * n).reshape(n, 4)
    q[-1] = 0  # degree n - 2
    z = oracle.rand_elems(rng, 4)
    qd = D.dec(q).T  # (4, n) plain values
    zd = np.repeat(D.dec(z).reshape(4, 1), n, axis=1)
    shifted = np.concatenate([np.zeros((4, 1), np.uint64), qd[:, :-1]], axis=1)  # q_{i-1}
    pd = (shifted + np.uint64(D.P) - D._mul(zd, qd)) % np.uint64(D.P)  # p_i = q_{i-1} - z q_i
    p = D.enc(pd).T.astype(np.uint32).reshape(-1)
    d = hal.copy_from_extelem("p", p)
    begin = np.array([0, 1], np.uint32)
    assert hal.combos_divide(d, z, begin, n) == -1
    assert np.array_equal(d.to_numpy(), q.reshape(-1))
    p1 = p.copy()
    p1[0] = oracle.encode(np.array([oracle.decode(np.array([p[0]]))[0] + 1]))[0]
    d1 = hal.copy_from_extelem("p", p1)
    assert hal.combos_divide(d1, z, begin, n) == 0
    ref = p1.copy()
    oracle.combos_divide(ref, z, begin, n)
    assert np.array_equal(d1.to_numpy(), ref)


@pytest.mark.parametrize("circuit", ["rv32im", "recursion"])
@pytest.mark.parametrize("po2", [5, 8])
def test_eval_check(hal, oracle, circuit, po2):
    # CircuitHal::eval_check (rv32im/src/prove/hal/cpu.rs:145-207) vs the reference's
    # compiled C++ poly_fp; DualCircuitHal (hal/dual.rs:418-500) covers the same op.
    if oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    d = oracle.load_circuit_json(circuit)
    rng = np.random.default_rng(15 + po2)
    D = 4 << po2
    gs = d["group_sizes"]
    groups = [oracle.rand_elems(rng, gs[g] * D) for g in range(3)]
    mix = oracle.rand_elems(rng, d["mix_size"])
    glob = oracle.rand_elems(rng, d["output_size"])
    pm = oracle.rand_elems(rng, 4)
    ref = np.zeros(4 * D, np.uint32)
    oracle.eval_check(circuit, ref, groups, mix, glob, pm, po2)
    out = hal.alloc_elem("check", 4 * D)
    hal.eval_check(circuit, out, [dev(hal, g) for g in groups], dev(hal, mix), dev(hal, glob), pm, po2)
    assert np.array_equal(out.to_numpy(), ref)


@pytest.mark.parametrize("circuit", ["rv32im", "recursion"])
@pytest.mark.parametrize("wide", ["0", "0xffffffff"])
def test_eval_check_both_tap_forms(hal, oracle, circuit, wide, monkeypatch):
    """Every generated kernel is built with 32-bit tap indices and with column base pointers;
    the tuning file picks one per kernel below po2=24 (the other runs only if R0_EC_WIDE asks
    for it), so both forms of every kernel are checked against the compiled poly_fp here."""
    if oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    monkeypatch.setenv("R0_EC_WIDE", wide)
    po2 = 6
    d = oracle.load_circuit_json(circuit)
    rng = np.random.default_rng(77)
    D = 4 << po2
    gs = d["group_sizes"]
    groups = [oracle.rand_elems(rng, gs[g] * D) for g in range(3)]
    mix = oracle.rand_elems(rng, d["mix_size"])
    glob = oracle.rand_elems(rng, d["output_size"])
    pm = oracle.rand_elems(rng, 4)
    ref = np.zeros(4 * D, np.uint32)
    oracle.eval_check(circuit, ref, groups, mix, glob, pm, po2)
    out = hal.alloc_elem("check", 4 * D)
    hal.eval_check(circuit, out, [dev(hal, g) for g in groups], dev(hal, mix), dev(hal, glob), pm, po2)
    assert np.array_equal(out.to_numpy(), ref)


@pytest.mark.parametrize("circuit,suite,po2", [("rv32im", "poseidon2", 8), ("rv32im", "poseidon2", 11),
                                               ("rv32im", "sha-256", 9), ("recursion", "poseidon2", 9),
                                               ("recursion", "sha-256", 8), ("recursion", "poseidon_254", 8),
                                               ("rv32im", "poseidon2", 12), ("recursion", "sha-256", 13),
                                               ("rv32im", "poseidon2", 14)])
def test_prove_segment_seal_identical(hal, hal_sha, oracle, circuit, suite, po2):
    """Whole-segment seals (Vec<u32>) are bit-identical to the CPU oracle's. From po2 12 the
    prover keeps coefficient rows bit-reversed (prover.cpp: coeffs_stay_bitrev), so the
    po2 >= 12 cases pin that order through evaluate_any, mix and the combos reversal."""
    if oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    import risc0_amd as r
    h, s = H(suite), S(oracle, suite)
    d = oracle.load_circuit_json(circuit)
    rng = np.random.default_rng(0x5249534330 + po2)
    n = 1 << po2
    gs = d["group_sizes"]
    code, data, accum = (oracle.rand_elems(rng, gs[g] * n) for g in (1, 2, 0))
    glob = oracle.rand_elems(rng, d["output_size"])
    glob[3] = 0xFFFFFFFF  # INVALID globals are zeroized into the header
    version = 2 if circuit == "rv32im" else None
    seal, mix = r.prove_segment(h, circuit, po2, dev(h, code), dev(h, data), dev(h, accum), dev(h, glob),
                                version=version)
    ref_seal, ref_mix, _ = oracle.prove_segment(circuit, s, po2, code, data, accum, glob, version=version)
    assert np.array_equal(mix, ref_mix)
    assert seal.size == ref_seal.size
    assert np.array_equal(seal, ref_seal)


# ---- golden fixtures (tests/golden, from the reference's compiled poly_fp; no oracle/_ref needed) ----
import test_golden as G  # noqa: E402


@pytest.mark.parametrize("case", G.INDEX["eval_check"], ids=lambda c: f"{c['circuit']}-po2{c['po2']}")
def test_eval_check_golden(hal, oracle, case):
    groups, mix, glob, pm = G.eval_inputs(oracle, case["circuit"], case["po2"], case["seed"])
    out = hal.alloc_elem("check", 4 * (4 << case["po2"]))
    hal.eval_check(case["circuit"], out, [dev(hal, g) for g in groups], dev(hal, mix), dev(hal, glob), pm,
                   case["po2"])
    assert np.array_equal(out.to_numpy(), np.load(G.os.path.join(G.GOLD, case["file"])))


@pytest.mark.parametrize("case", G.INDEX["seals"], ids=lambda c: f"{c['circuit']}-{c['suite']}-po2{c['po2']}")
def test_prove_segment_seal_golden(hal, hal_sha, oracle, case):
    import risc0_amd as r
    circuit, po2 = case["circuit"], case["po2"]
    h = H(case["suite"])
    code, data, accum, glob = G.seal_inputs(oracle, circuit, po2)
    seal, mix = r.prove_segment(h, circuit, po2, dev(h, code), dev(h, data), dev(h, accum), dev(h, glob),
                                version=2 if circuit == "rv32im" else None)
    assert seal.size == case["seal_words"]
    assert G.digest(seal) == case["seal_sha256"]
    assert [int(x) for x in mix] == case["mix"]


def test_prove_segments_concurrently_golden(hal, hal_sha, oracle):
    """Segments in flight: host threads, each on its own HIP stream and buffer pool,
    prove different golden cases at once; every seal still matches its fixture."""
    import threading

    import risc0_amd as r
    cases = G.INDEX["seals"]
    inputs = []
    for case in cases:
        h = H(case["suite"])
        code, data, accum, glob = G.seal_inputs(oracle, case["circuit"], case["po2"])
        inputs.append((h, case, [dev(h, x) for x in (code, data, accum, glob)]))
    out = [None] * len(inputs)

    def run(i):
        h, case, (c, d, a, g) = inputs[i]
        for _ in range(2):
            out[i] = r.prove_segment(h, case["circuit"], case["po2"], c, d, a, g,
                                     version=2 if case["circuit"] == "rv32im" else None)

    ts = [threading.Thread(target=run, args=(i,)) for i in range(len(inputs))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for (h, case, _), (seal, mix) in zip(inputs, out):
        assert G.digest(seal) == case["seal_sha256"], case
        assert [int(x) for x in mix] == case["mix"]


def test_prove_segment_from_pinned_host(oracle):
    """The end-to-end path of bench.py's `end_to_end` leg: witness groups in page-locked
    host memory (r0hip_host_alloc), uploaded with r0hip_memcpy_h2d, then proved; the seal
    matches its golden fixture."""
    import ctypes

    import risc0_amd as r
    case = G.INDEX["seals"][0]
    h = H(case["suite"])
    lib = r.lib()
    bufs, hosts = [], []
    try:
        for a in G.seal_inputs(oracle, case["circuit"], case["po2"]):
            p = ctypes.c_void_p()
            r.check(lib.r0hip_host_alloc(ctypes.byref(p), a.size * 4))
            hosts.append(p.value)
            np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint32)), shape=(a.size,))[:] = a
            b = h.alloc_elem("w", a.size)
            r.check(lib.r0hip_memcpy_h2d(b.ptr, p.value, a.size * 4))
            bufs.append(b)
        seal, mix = r.prove_segment(h, case["circuit"], case["po2"], *bufs,
                                    version=2 if case["circuit"] == "rv32im" else None)
    finally:
        for p in hosts:
            r.check(lib.r0hip_host_free(p))
    assert G.digest(seal) == case["seal_sha256"]
    assert [int(x) for x in mix] == case["mix"]


@pytest.mark.parametrize("case", G.INDEX["seals"], ids=lambda c: f"{c['circuit']}-{c['suite']}-po2{c['po2']}")
def test_prove_segments_pipeline_golden(hal, hal_sha, oracle, case):
    """The native segment pipeline (r0hip_prove_segments): uploader + 2 provers over 5
    jobs from host witnesses, groups of more than 48 columns committed chunk by chunk as
    they upload (Poseidon2 / SHA-256); every seal matches its golden fixture."""
    import risc0_amd as r
    h = H(case["suite"])
    w = G.seal_inputs(oracle, case["circuit"], case["po2"])
    out = r.prove_segments(h, case["circuit"], case["po2"], [w] * 5,
                           version=2 if case["circuit"] == "rv32im" else None, in_flight=2)
    assert len(out) == 5
    for seal, mix in out:
        assert G.digest(seal) == case["seal_sha256"]
        assert [int(x) for x in mix] == case["mix"]


@pytest.mark.parametrize("circuit,suite,po2", [("rv32im", "poseidon2", 16), ("rv32im", "sha-256", 14),
                                               ("recursion", "poseidon2", 14), ("rv32im", "poseidon2", 20)])
def test_prove_segments_streamed_matches_resident(hal, hal_sha, oracle, circuit, suite, po2):
    """A segment proved through the pipeline (chunked upload, streamed commits: interpolate,
    evaluate, bit-reverse and row-hash ranges per 48-column chunk) gives the same seal as
    the resident-witness prover on the same witness."""
    import risc0_amd as r
    h = H(suite)
    w = G.seal_inputs(oracle, circuit, po2)
    version = 2 if circuit == "rv32im" else None
    seal, mix = r.prove_segment(h, circuit, po2, *(dev(h, a) for a in w), version=version)
    out = r.prove_segments(h, circuit, po2, [w] * 2, version=version, in_flight=1)
    for s2, m2 in out:
        assert np.array_equal(m2, mix)
        assert np.array_equal(s2, seal)


def device_witness(h, n, seed):
    """Uniform canonical BabyBear words generated on the device (r0hip_fill_uniform) for
    sizes whose host generation would take minutes."""
    import risc0_amd as r
    b = h.alloc_elem("w", n)
    r.check(r.lib().r0hip_fill_uniform(b.ptr, n, seed))
    return b


def ec_sample_cycles(po2, rng, n_random=4096):
    """Cycles for the full-size eval_check checks: the domain's ends, the back-wrap
    region (taps reach back 4*68 points), every cycle & 3 coset, 256-point launch-block
    edges, the 2^k boundaries, and random points."""
    D = 4 << po2
    s = set(range(8)) | set(range(D - 8, D)) | set(range(4 * 68 - 4, 4 * 68 + 8))
    s |= set(range(D - 4 * 68 - 4, D - 4 * 68 + 4))
    for k in range(8, po2 + 2):
        s |= {(1 << k) - 1, 1 << k, (1 << k) + 1}
    for b in rng.integers(1, D // 256, 64):
        s |= {int(b) * 256 - 1, int(b) * 256}
    s |= {int(x) for x in rng.integers(0, D, n_random)}
    return np.array(sorted(x for x in s if 0 <= x < D), np.uint64)


@pytest.mark.parametrize("circuit,po2", [("rv32im", 20), ("rv32im", 24), ("recursion", 18)])
def test_eval_check_full_size(hal, oracle, circuit, po2):
    """eval_check at the BASELINE sizes (configs[1] po2=20, configs[2] po2=24, configs[4]
    recursion po2=18) equals the reference's compiled poly_fp x inv((3x)^N - 1)
    (rv32im/src/prove/hal/cpu.rs:145-207) word for word at >= 4096 sampled cycles. The
    evaluated groups are drawn on the device; the checker recomputes any tap from its
    index (oracle.eval_check_sampled)."""
    import risc0_amd as r
    if oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    d = oracle.load_circuit_json(circuit)
    D = 4 << po2
    gs = d["group_sizes"]
    seeds = [0x45430000 + 16 * po2 + g for g in range(3)]
    rng = np.random.default_rng(0x4543 + po2)
    bufs = [device_witness(hal, gs[g] * D, seeds[g]) for g in range(3)]
    mix = oracle.rand_elems(rng, d["mix_size"])
    glob = oracle.rand_elems(rng, d["output_size"])
    pm = oracle.rand_elems(rng, 4)
    out = hal.alloc_elem("check", 4 * D)
    hal.eval_check(circuit, out, bufs, dev(hal, mix), dev(hal, glob), pm, po2)
    for b in bufs:
        b.free()
    got = out.to_numpy().reshape(4, D)
    out.free()
    cycles = ec_sample_cycles(po2, rng)
    assert cycles.size >= 4096
    ref = oracle.eval_check_sampled(circuit, seeds, mix, glob, pm, po2, cycles)
    bad = np.nonzero((got[:, cycles.astype(np.int64)].T != ref).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} of {cycles.size} cycles differ, first at {cycles[bad[:8]]}"


@pytest.mark.parametrize("circuit,suite,po2", [("rv32im", "poseidon2", 20), ("rv32im", "poseidon2", 16),
                                               ("recursion", "sha-256", 18), ("recursion", "poseidon_254", 18),
                                               ("rv32im", "poseidon2", 24)])
def test_full_size_seal_verifies(hal, hal_sha, oracle, circuit, suite, po2):
    """At BASELINE sizes the CPU oracle cannot prove (configs[1] po2=20 and configs[2] po2=24,
    the maximum segment), the HIP seal passes the reference verifier's checks
    (tests/verifier.py: transcript, all Merkle openings, DEEP-ALI combination, every FRI
    fold and the final polynomial); flipped bits are rejected."""
    import risc0_amd as r
    import verifier
    h, s = H(suite), S(oracle, suite)
    d = oracle.load_circuit_json(circuit)
    rng = np.random.default_rng(0x5249534330 + po2)
    n = 1 << po2
    gs = d["group_sizes"]
    if po2 >= 22:
        bufs = [device_witness(h, gs[g] * n, 0x5249534330 + po2 + g) for g in (1, 2, 0)]
    else:
        bufs = [dev(h, oracle.rand_elems(rng, gs[g] * n)) for g in (1, 2, 0)]
    glob = dev(h, oracle.rand_elems(rng, d["output_size"]))
    seal, _mix = r.prove_segment(h, circuit, po2, *bufs, glob, version=2 if circuit == "rv32im" else None)
    for b in bufs:
        b.free()
    res = verifier.verify(oracle, circuit, seal, s)
    assert res["po2"] == po2
    assert r.verify_seal(circuit, s, seal, check_validity=False) == po2  # the native verifier agrees
    for where in (seal.size // 3, seal.size - 5):
        bad = seal.copy()
        bad[where] ^= np.uint32(1 << 9)
        with pytest.raises(verifier.VerificationError):
            verifier.verify(oracle, circuit, bad, s)
        with pytest.raises(r.R0HipError):
            r.verify_seal(circuit, s, bad, check_validity=False)


@pytest.mark.parametrize("suite,po2", [("poseidon2", 20), ("sha-256", 16), ("poseidon_254", 16)])
def test_valid_witness_seal_passes_validity(hal, hal_sha, oracle, suite, po2):
    """A witness that satisfies the recursion circuit (all-zero code/data/accum; its
    constraints hold for any globals and mix) proved on the GPU passes every check of the
    reference verifier including the validity equation (mod.rs:340-394), in the native
    verifier and in the restatement."""
    import risc0_amd as r
    import verifier
    h, s = H(suite), S(oracle, suite)
    d = oracle.load_circuit_json("recursion")
    n, gs = 1 << po2, d["group_sizes"]
    bufs = [dev(h, np.zeros(gs[g] * n, np.uint32)) for g in (1, 2, 0)]
    glob = dev(h, oracle.rand_elems(np.random.default_rng(po2), d["output_size"]))
    seal, _mix = r.prove_segment(h, "recursion", po2, *bufs, glob)
    for b in bufs:
        b.free()
    assert r.verify_seal("recursion", s, seal) == po2
    assert verifier.verify(oracle, "recursion", seal, s, check_validity=True)["validity"] is True


def test_abi_errors_are_reported_not_fatal(hal, oracle):
    """The C ABI's error contract (risc0/sys/src/lib.rs:53-75): bad arguments come back as
    messages, the library stays usable, and the pipeline reports the failing job."""
    import ctypes

    import risc0_amd as r
    L = r.lib()
    d = hal.alloc_digest("d", 8)
    m = hal.alloc_elem("m", 8 * 16)
    with pytest.raises(r.R0HipError, match="suite"):
        r.check(L.r0hip_hash_rows(7, d.ptr, m.ptr, 8, 16))
    with pytest.raises(r.R0HipError, match="input_size"):
        r.check(L.r0hip_hash_fold(0, d.ptr, 6, 4))
    with pytest.raises(r.R0HipError, match="NTT size"):
        r.check(L.r0hip_batch_interpolate_ntt(m.ptr, 1, 40))
    with pytest.raises(r.R0HipError, match="circuit"):
        r.check(L.r0hip_eval_check(b"keccak", m.ptr, None, m.ptr, m.ptr, None, 4))
    case = G.INDEX["seals"][0]
    code, data, accum, glob = (dev(hal, x) for x in G.seal_inputs(oracle, case["circuit"], case["po2"]))
    with pytest.raises(r.R0HipError, match="seal buffer too small"):
        r.prove_segment(hal, case["circuit"], case["po2"], code, data, accum, glob, version=2, seal_cap=16)
    w = G.seal_inputs(oracle, case["circuit"], case["po2"])
    with pytest.raises(r.R0HipError, match="segment 1"):
        r.prove_segments(hal, case["circuit"], case["po2"], [w, (w[0], 0, w[2], w[3])], version=2)
    # still healthy afterwards
    h_ok = hal.alloc_elem("ok", 8 * 16)
    h_ok.copy_from(oracle.rand_elems(np.random.default_rng(3), 8 * 16))
    out = hal.alloc_digest("o", 8)
    hal.hash_rows(out, h_ok)
    ref = np.zeros(8 * 8, np.uint32)
    oracle.hash_rows(oracle.POSEIDON2, ref, h_ok.to_numpy())
    assert np.array_equal(out.to_numpy(), ref)


def test_steady_state_proving_makes_no_hipmalloc(oracle):
    """Locks in ae46b24: once a segment size has been proved, proofs on NEW host threads
    (the bench and the pipeline start fresh ones) reuse the pooled blocks and scratch that
    exited threads left: zero hipMalloc calls (r0hip_mem_stats, the MemoryTracker
    equivalent), identical seals, and the peak live bytes reported."""
    import threading

    import risc0_amd as r
    case = G.INDEX["seals"][0]
    h = H(case["suite"])
    code, data, accum, glob = G.seal_inputs(oracle, case["circuit"], case["po2"])
    bufs = [dev(h, x) for x in (code, data, accum)]
    globs = [dev(h, glob) for _ in range(2)]
    version = 2 if case["circuit"] == "rv32im" else None
    seals = {}
    # start from a clean pool: blocks other tests' calls left (other sizes) would be matched
    # up to 25% larger in whatever order threads race for them. Every entry point hands its
    # thread's idle blocks back to the shared pool before it returns (release_thread_memory,
    # runtime.cpp), so nothing lands in the pool after the call that used it has returned
    r.trim()

    def batch(tag):
        def run(i):
            seals[(tag, i)] = r.prove_segment(h, case["circuit"], case["po2"], *bufs, globs[i], version=version)[0]
        ts = [threading.Thread(target=run, args=(i,)) for i in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()

    # warm until a whole batch allocates nothing: some slots are asked small and then grown
    # within a proof, and blocks go back to a shared pool at the end of each call, so which thread
    # finds which block depends on the race; once the pool holds blocks of every size both
    # interleavings need, proving allocates no more (a leak would keep allocating here)
    # (three batches in a row, since one or two interleavings that happen to allocate nothing
    # do not mean the pool holds enough for the others)
    quiet = 0
    for k in range(16):
        m0 = r.mem_stats()["mallocs"]
        batch(f"warm{k}")
        quiet = quiet + 1 if k and r.mem_stats()["mallocs"] == m0 else 0
        if quiet == 3:
            break
    else:
        raise AssertionError("warm batches kept allocating device memory")
    r.mem_reset_peak()
    before = r.mem_stats()
    os.write(2, b"steady batch begins\n")  # brackets R0HIP_TRACE_MALLOC=1 output
    batch("steady")
    os.write(2, b"steady batch ends\n")
    after = r.mem_stats()
    assert after["mallocs"] == before["mallocs"], (before, after)
    # no thread keeps a proof's blocks past its call: live bytes are the test's own buffers again
    assert after["live"] == before["live"], (before, after)
    assert after["peak_live"] > after["live"] >= 0
    assert after["reserved"] >= after["peak_live"]
    for i in range(2):
        assert G.digest(seals[("steady", i)]) == case["seal_sha256"]


@pytest.mark.parametrize("idx", range(len(G.INDEX["seals"])))
def test_per_op_abi_prover_matches_golden_seal(idx, oracle):
    """The drop-in path at seal level: the reference Prover call sequence (prover.rs,
    poly_group.rs, merkle.rs, fri.rs, restated in tests/hal_prover.py) drives ONLY the
    per-op Hal symbols of include/r0hip.h (alloc/memcpy, NTTs, zk_shift, bit_reverse,
    hash_rows/hash_fold, eval_check, batch_evaluate_any, mix_poly_coeffs,
    combos_prepare/combos_divide, eltwise ops, fri_fold, gather_sample openings as with
    has_unified_memory() = false) — what a Rust HipHal would call — and the seal equals
    the golden digest for every (circuit, suite, po2) case, as r0hip_prove_segment's does."""
    import hal_prover
    case = G.INDEX["seals"][idx]
    h = H(case["suite"])
    code, data, accum, glob = G.seal_inputs(oracle, case["circuit"], case["po2"])
    bufs = [dev(h, x) for x in (code, data, accum, glob)]
    seal, mix = hal_prover.prove_segment(oracle, h, case["circuit"], case["po2"], *bufs)
    assert [int(x) for x in mix] == case["mix"]
    assert G.digest(seal) == case["seal_sha256"], case


@pytest.mark.parametrize("po2,short", [(10, 0), (12, 7), (16, 0), (18, 0), (4, 3)])
def test_recursion_accum_matches_reference(hal, oracle, po2, short):
    """Recursion accumulation on the GPU (r0hip_recursion_accum: compute, prefix product,
    verify; kernels generated from risc0_amd/circuits/recursion.accum.ir) against the
    reference's own compiled risc0_circuit_recursion_cpu_accum (recursion-sys
    kernels/cxx/ffi.cpp:208-217, oracle/_ref/libref_recursion.so) on the same synthetic rows:
    every accum word identical, including the cells neither writes (INVALID); work cycles
    below the total leave the ZK tail rows alone."""
    import accum_ir as A
    d = A.circuit()
    gs = d["group_sizes"]
    n = 1 << po2
    rng = np.random.default_rng(100 + po2)
    ctrl, glob, data, mix = A.synthetic(rng, oracle, po2, gs, d["output_size"], d["mix_size"])
    acc0 = np.full(gs[0] * n, A.INVALID, np.uint32)
    steps = n - short
    ref = acc0.copy()
    A.ref_accum(ctrl, glob, data, mix, ref, steps, n)
    dacc = dev(hal, acc0)
    hal.recursion_accum(dev(hal, ctrl), dev(hal, glob), dev(hal, data), dev(hal, mix), dacc, steps, n)
    got = dacc.to_numpy()
    assert np.array_equal(got, ref), int((got != ref).sum())


@pytest.mark.parametrize("circuit,suite,po2", [("rv32im", "poseidon2", 10), ("rv32im", "sha-256", 9),
                                               ("recursion", "poseidon2", 9)])
def test_prove_segment_accum_matches_reference(hal, hal_sha, oracle, circuit, suite, po2):
    """The prove core with the accumulation on the device (r0hip_prove_segment_accum: commit
    code and data, draw mix, accumulate, zeroize, commit accum, finalize), as the reference's
    prove_core runs it (rv32im prove/hal/mod.rs:205-212, recursion prove/mod.rs:212-218).
    Checked in two halves against the reference: the device-filled accum group equals the
    compiled reference accumulation (oracle/_ref) run on the same rows with the mix the
    transcript drew, INVALID words zeroized; and the seal equals the oracle prover's on that
    accum group."""
    import risc0_amd as r
    if oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    h, s = H(suite), S(oracle, suite)
    d = oracle.load_circuit_json(circuit)
    gs = d["group_sizes"]
    n = 1 << po2
    rng = np.random.default_rng(0x41434355 + po2)
    INVALID = 0xFFFFFFFF
    if circuit == "rv32im":
        import rv32im_accum_ref as R
        from test_rv32im_accum_ir import rows_for_arms
        if not R.available():
            pytest.skip("oracle/_ref/libref_rv32im_accum.so not built")
        code = oracle.rand_elems(rng, gs[1] * n)
        data = rows_for_arms(rng, n, list(rng.integers(0, 13, n)))
        glob = oracle.rand_elems(rng, d["output_size"])
        acc0 = np.full(gs[0] * n, INVALID, np.uint32)
        work, version = n, 2
    else:
        import accum_ir as A
        code, glob, data, _ = A.synthetic(rng, oracle, po2, gs, d["output_size"], d["mix_size"])
        acc0 = np.full(gs[0] * n, INVALID, np.uint32).reshape(gs[0], n)
        acc0[:, n - 8:] = oracle.rand_elems(rng, gs[0] * 8).reshape(gs[0], 8)  # ZK noise rows
        acc0 = acc0.reshape(-1)
        work, version = n - 8, None
    dacc = dev(h, acc0)
    seal, mix = r.prove_segment_accum(h, circuit, po2, dev(h, code), dev(h, data), dacc, work, dev(h, glob),
                                      version=version)
    glob_z = np.where(glob == INVALID, 0, glob).astype(np.uint32)
    if circuit == "rv32im":
        ref_acc = R.accum(data, glob_z, mix, n, work)
    else:
        ref_acc = acc0.copy()
        A.ref_accum(code, glob_z, data, mix, ref_acc, work, n)
    ref_acc = np.where(ref_acc == INVALID, 0, ref_acc).astype(np.uint32)
    got = dacc.to_numpy()
    assert np.array_equal(got, ref_acc), int((got != ref_acc).sum())
    ref_seal, ref_mix, _ = oracle.prove_segment(circuit, s, po2, code, data, ref_acc, glob, version=version)
    assert np.array_equal(mix, ref_mix)
    assert np.array_equal(seal, ref_seal)


@pytest.mark.parametrize("suite,po2", [("poseidon2", 10), ("sha-256", 9)])
def test_prove_segments_device_accum_matches_fused(hal, hal_sha, oracle, suite, po2):
    """The segment pipeline with no host accum group (rv32im): each prover accumulates on
    the device after the mix draw. Seals equal r0hip_prove_segment_accum's on the same
    witness (which test_prove_segment_accum_matches_reference pins to the reference), for
    more jobs than buffer sets, so sets are reused and refilled with INVALID words."""
    import risc0_amd as r
    from test_rv32im_accum_ir import rows_for_arms
    h = H(suite)
    d = oracle.load_circuit_json("rv32im")
    n = 1 << po2
    jobs, want = [], []
    for i in range(4):
        rng = np.random.default_rng(0x50495045 + 7 * po2 + i)
        code = oracle.rand_elems(rng, d["group_sizes"][1] * n)
        data = rows_for_arms(rng, n, list(rng.integers(0, 13, n)))
        glob = oracle.rand_elems(rng, d["output_size"])
        dacc = dev(h, np.full(d["group_sizes"][0] * n, 0xFFFFFFFF, np.uint32))
        seal, mix = r.prove_segment_accum(h, "rv32im", po2, dev(h, code), dev(h, data), dacc, n, dev(h, glob),
                                          version=2)
        want.append((seal, mix))
        jobs.append((code, data, None, glob))
    got = r.prove_segments(h, "rv32im", po2, jobs, version=2, in_flight=2)
    for (s1, m1), (s2, m2) in zip(got, want):
        assert np.array_equal(m1, m2)
        assert np.array_equal(s1, s2)


# ---- rv32im BigInt cycles: the accumulator states WitnessGenerator::accum injects with the
# final mix before the step (witgen/mod.rs:178-205; tests/bigint_accum.py) ----

def _bigint_witness(po2, seed, calls):
    import bigint_accum as B
    rng = np.random.default_rng(seed)
    n = 1 << po2
    data, recs = B.lay_out(rng, n, calls)
    return rng, data, recs


@pytest.mark.parametrize("po2,calls", [(10, 60), (20, 1500)])
def test_rv32im_accum_bigint_matches_reference(hal, po2, calls):
    """r0hip_rv32im_bigint_accum_inject + r0hip_rv32im_accum against the compiled reference
    accumulation (risc0_circuit_rv32im_cpu_accum) on rows whose arm-12 cycles run every PolyOp,
    both starting from the group with the reference's injected states. Without the injection
    the device result differs (the step reads the previous cycle's state at back 1)."""
    import risc0_amd as r
    import bigint_accum as B
    import rv32im_accum_ref as R
    if not R.available():
        pytest.skip("oracle/_ref/libref_rv32im_accum.so not built")
    n = 1 << po2
    rng, data, recs = _bigint_witness(po2, 0xB1 + po2, calls)
    assert {rec[1] for rec in recs} == set(range(7))
    glob = rng.integers(0, R.P, R.GLOBAL_WORDS, dtype=np.uint64).astype(np.uint32)
    mix = rng.integers(0, R.P, R.MIX_WORDS, dtype=np.uint64).astype(np.uint32)
    acc0 = np.full(R.ACCUM_COLS * n, R.INVALID, np.uint32)
    ref = R.accum(data, glob, mix, n, n, accum_init=B.inject(acc0.copy(), n, mix, recs))
    dd, dg, dm = dev(hal, data), dev(hal, glob), dev(hal, mix)
    d_acc = dev(hal, acc0)
    r.bigint_accum_inject(d_acc, n, mix, recs)
    hal.rv32im_accum(dd, d_acc, dg, dm, n, n)
    got = d_acc.to_numpy()
    bad = np.nonzero(got != ref)[0]
    assert bad.size == 0, f"{bad.size} words differ, first at column {bad[0] // n} row {bad[0] % n}"
    if po2 <= 12:
        d_plain = dev(hal, acc0)
        hal.rv32im_accum(dd, d_plain, dg, dm, n, n)
        assert not np.array_equal(d_plain.to_numpy(), ref)


@pytest.mark.parametrize("suite,po2,calls", [("poseidon2", 10, 60), ("sha-256", 9, 30), ("poseidon2", 20, 1500)])
def test_prove_segment_accum_bigint_matches_reference(hal, hal_sha, oracle, suite, po2, calls):
    """r0hip_prove_segment_accum with the trace's BigInt backs: the states are computed with
    the mix the transcript draws inside the call and injected before the step. The device
    accum group equals the compiled reference accumulation on the same rows with the
    reference's injection; the seal equals the oracle prover's on that group (po2 <= 12), and
    at po2 20 the seal passes the verifier's structural checks."""
    import risc0_amd as r
    import bigint_accum as B
    import rv32im_accum_ref as R
    if oracle.ref_lib() is None or not R.available():
        pytest.skip("oracle/_ref not built")
    h, s = H(suite), S(oracle, suite)
    d = oracle.load_circuit_json("rv32im")
    n = 1 << po2
    rng, data, recs = _bigint_witness(po2, 0xB2 + po2, calls)
    code = oracle.rand_elems(rng, d["group_sizes"][1] * n)
    glob = oracle.rand_elems(rng, d["output_size"])
    acc0 = np.full(d["group_sizes"][0] * n, R.INVALID, np.uint32)
    dacc = dev(h, acc0)
    seal, mix = r.prove_segment_accum(h, "rv32im", po2, dev(h, code), dev(h, data), dacc, n, dev(h, glob),
                                      version=2, bigint=recs)
    glob_z = np.where(glob == R.INVALID, 0, glob).astype(np.uint32)
    ref_acc = R.accum(data, glob_z, mix, n, n, accum_init=B.inject(acc0.copy(), n, mix, recs))
    ref_acc = np.where(ref_acc == R.INVALID, 0, ref_acc).astype(np.uint32)
    got = dacc.to_numpy()
    assert np.array_equal(got, ref_acc), int((got != ref_acc).sum())
    if po2 <= 12:
        ref_seal, ref_mix, _ = oracle.prove_segment("rv32im", s, po2, code, data, ref_acc, glob, version=2)
        assert np.array_equal(mix, ref_mix)
        assert np.array_equal(seal, ref_seal)
    else:
        assert r.verify_seal("rv32im", s, seal, check_validity=False) == po2


def test_prove_segment_accum_rejects_invalid_bigint_eqz(hal, oracle):
    """An EqZero whose integer identity fails stops the proof with the reference's error
    (byte_poly.rs:458 "Invalid eqz in bigint accum"), as WitnessGenerator::accum does."""
    import risc0_amd as r
    import bigint_accum as B
    po2 = 8
    n = 1 << po2
    d = oracle.load_circuit_json("rv32im")
    rng, data, recs = _bigint_witness(po2, 0xB3, 6)
    recs = [[row, op, c, list(by)] for row, op, c, by in recs]
    eqz = next(i for i, rec in enumerate(recs) if rec[1] == B.EQ_ZERO)
    recs[eqz][3][0] ^= 1
    code = oracle.rand_elems(rng, d["group_sizes"][1] * n)
    glob = oracle.rand_elems(rng, d["output_size"])
    dacc = dev(hal, np.full(d["group_sizes"][0] * n, 0xFFFFFFFF, np.uint32))
    with pytest.raises(r.R0HipError, match="Invalid eqz in bigint accum"):
        r.prove_segment_accum(hal, "rv32im", po2, dev(hal, code), dev(hal, data), dacc, n, dev(hal, glob),
                              version=2, bigint=recs)
    # the library stays usable after the error
    seal, _ = r.prove_segment_accum(hal, "rv32im", po2, dev(hal, code), dev(hal, data),
                                    dev(hal, np.full(d["group_sizes"][0] * n, 0xFFFFFFFF, np.uint32)), n,
                                    dev(hal, glob), version=2, bigint=[tuple(x) for x in recs[:eqz]])
    assert seal.size > 0


@pytest.mark.parametrize("suite,po2", [("poseidon2", 10), ("sha-256", 9)])
def test_prove_segments_bigint_matches_fused(hal, hal_sha, oracle, suite, po2):
    """The segment pipeline's device accumulation with per-job BigInt backs equals
    r0hip_prove_segment_accum on the same jobs (4 jobs over 3 reused buffer sets; one job
    without BigInt cycles), and a job that gives backs with a host accum group is refused."""
    import risc0_amd as r
    h = H(suite)
    d = oracle.load_circuit_json("rv32im")
    n = 1 << po2
    jobs, want = [], []
    for i in range(4):
        rng, data, recs = _bigint_witness(po2, 0x50 + 7 * po2 + i, 0 if i == 2 else 40)
        code = oracle.rand_elems(rng, d["group_sizes"][1] * n)
        glob = oracle.rand_elems(rng, d["output_size"])
        dacc = dev(h, np.full(d["group_sizes"][0] * n, 0xFFFFFFFF, np.uint32))
        want.append(r.prove_segment_accum(h, "rv32im", po2, dev(h, code), dev(h, data), dacc, n, dev(h, glob),
                                          version=2, bigint=recs))
        jobs.append((code, data, None, glob, recs))
    got = r.prove_segments(h, "rv32im", po2, jobs, version=2, in_flight=2)
    for (s1, m1), (s2, m2) in zip(got, want):
        assert np.array_equal(m1, m2)
        assert np.array_equal(s1, s2)
    code, data, _, glob, recs = jobs[0]
    acc = np.zeros(d["group_sizes"][0] * n, np.uint32)
    with pytest.raises(r.R0HipError, match="without a device accumulation"):
        r.prove_segments(h, "rv32im", po2, [(code, data, acc, glob, recs)], version=2)


# ---- a satisfying, non-trivial recursion witness proven on the GPU (tests/recursion_program.py) ----

@pytest.mark.parametrize("suite,po2", [("poseidon2", 16), ("sha-256", 16), ("poseidon2", 18)])
def test_satisfying_recursion_program_gpu_seal_passes_validity(hal, hal_sha, oracle, suite, po2):
    """A hand-encoded recursion program filling the segment (every row but the ZK rows),
    through the restated preflight and the reference's compiled witness generator, proven by
    r0hip_prove_segment_accum (accumulation on the device). The device accum group equals the
    reference accumulation with the drawn mix; the seal passes r0hip_verify_seal with the
    validity equation and the restated verifier; at po2 16 Poseidon2 it equals the oracle
    prover's seal; flipping one data word makes the native verifier reject the new seal."""
    import recursion_program as RP
    import risc0_amd as r
    import verifier
    if not RP.available() or oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    h, s = H(suite), S(oracle, suite)
    w = RP.satisfying_witness(1000 + po2, po2)
    assert w["work"] > (1 << po2) - RP.ZK_CYCLES - 64
    dacc = dev(h, w["acc0"])
    seal, mix = r.prove_segment_accum(h, "recursion", po2, dev(h, w["ctrl"]), dev(h, w["data"]), dacc, w["work"],
                                      dev(h, w["glob"]))
    ref_acc = RP.accumulate(w, mix, po2)
    got = dacc.to_numpy()
    assert np.array_equal(got, ref_acc), int((got != ref_acc).sum())
    assert r.verify_seal("recursion", s, seal) == po2
    assert verifier.verify(oracle, "recursion", seal, s, check_validity=True)["validity"] is True
    if po2 == 16 and suite == "poseidon2":
        ref_seal, ref_mix, _ = oracle.prove_segment("recursion", s, po2, w["ctrl"], w["data"], ref_acc, w["glob"])
        assert np.array_equal(mix, ref_mix)
        assert np.array_equal(seal, ref_seal)
    bad = w["data"].copy()
    bad[9 * (1 << po2) + 100] ^= 1
    seal_b, _ = r.prove_segment_accum(h, "recursion", po2, dev(h, w["ctrl"]), dev(h, bad), dev(h, w["acc0"]),
                                      w["work"], dev(h, w["glob"]))
    with pytest.raises(r.R0HipError):
        r.verify_seal("recursion", s, seal_b)
    assert r.verify_seal("recursion", s, seal_b, check_validity=False) == po2


def test_pinned_host_buffers_are_pooled(hal):
    """r0hip_host_free keeps the block page-locked for the next r0hip_host_alloc of its size
    (unpinning stalled later proofs); r0hip_trim returns idle blocks; a pointer
    the library did not allocate and a second free of one block are refused."""
    import ctypes
    import risc0_amd as r
    lib = r.lib()
    a, b = ctypes.c_void_p(), ctypes.c_void_p()
    r.check(lib.r0hip_host_alloc(ctypes.byref(a), 3 << 20))
    arr = np.ctypeslib.as_array(ctypes.cast(a, ctypes.POINTER(ctypes.c_uint32)), shape=(3 << 18,))
    arr[:] = np.arange(3 << 18, dtype=np.uint32)
    d = hal.alloc_elem("x", 3 << 18)
    r.check(lib.r0hip_memcpy_h2d(d.ptr, a, 3 << 20))
    assert np.array_equal(d.to_numpy(), np.arange(3 << 18, dtype=np.uint32))
    r.check(lib.r0hip_host_free(a))
    r.check(lib.r0hip_host_alloc(ctypes.byref(b), 3 << 20))
    assert b.value == a.value
    r.check(lib.r0hip_host_free(b))
    # a second free of the same block is refused (it would hand one buffer to two callers)
    with pytest.raises(r.R0HipError, match="double free"):
        r.check(lib.r0hip_host_free(b))
    c, e = ctypes.c_void_p(), ctypes.c_void_p()
    r.check(lib.r0hip_host_alloc(ctypes.byref(c), 3 << 20))
    r.check(lib.r0hip_host_alloc(ctypes.byref(e), 3 << 20))
    assert c.value != e.value
    r.check(lib.r0hip_host_free(c))
    r.check(lib.r0hip_host_free(e))
    with pytest.raises(r.R0HipError, match="not returned by r0hip_host_alloc"):
        r.check(lib.r0hip_host_free(ctypes.c_void_p(arr.ctypes.data + 4096)))
    r.trim()


# ---- recursion witness generation on the GPU (r0hip_recursion_witgen, r0hip_prove_recursion) ----

@pytest.mark.parametrize("po2,rows,blocks", [
    (14, None, ("arith", "bits", "mix_rng", "iop", "poseidon2")),
    (18, None, ("arith", "bits", "mix_rng", "iop", "poseidon2")),
    (12, 1500, ("poseidon2",)),
    (12, 1500, ("iop", "mix_rng", "bits")),
])
def test_recursion_witgen_matches_reference(hal, po2, rows, blocks):
    """r0hip_recursion_witgen (generated step_exec / step_verify_mem kernels, the WOM
    argument sorted and scanned on the device, injectWomBacks) writes the same data group and
    globals, INVALID words included, as the reference's compiled
    risc0_circuit_recursion_cpu_witgen on a program filling the segment (restated preflight,
    tests/recursion_program.py)."""
    import recursion_program as RP
    import risc0_amd as r
    if not RP.available():
        pytest.skip("oracle/_ref/libref_recursion.so not built")
    n = 1 << po2
    rng = np.random.default_rng(2000 + po2 + (rows or 0))
    prog, inp = RP.random_program(rng, rows or n - RP.ZK_CYCLES - 1, blocks)
    pf = RP.preflight(prog, inp)
    ctrl, data, glob = RP.witgen(prog, pf, po2, raw=True)
    wom, cyc, iops = RP.trace_arrays(pf)
    dd = dev(hal, np.full(RP.DATA * n, RP.INVALID, np.uint32))
    dg = dev(hal, np.full(RP.OUT, RP.INVALID, np.uint32))
    r.recursion_witgen(dev(hal, ctrl), dd, dg, n, wom, cyc, iops)
    got = dd.to_numpy()
    bad = np.nonzero(got != data)[0]
    assert bad.size == 0, f"{bad.size} words differ; first col {bad[0] // n} row {bad[0] % n}"
    assert np.array_equal(dg.to_numpy(), glob)


def test_recursion_witgen_reports_a_failed_check(hal):
    """A hole in the write-once memory fails the sorted-memory check as in the reference
    (eqz at zirgen/circuit/recursion/wom.cpp:74), and the library stays usable."""
    import recursion_program as RP
    import risc0_amd as r
    po2, n = 11, 1 << 11
    b = RP.Builder(np.random.default_rng(5))
    b.consts([(3, 0), (4, 0)])
    b.next += 1
    b.consts([(5, 0)])
    prog, inp = b.finish()
    pf = RP.preflight(prog, inp)
    wom, cyc, iops = RP.trace_arrays(pf)
    dd = dev(hal, np.full(RP.DATA * n, RP.INVALID, np.uint32))
    dg = dev(hal, np.full(RP.OUT, RP.INVALID, np.uint32))
    with pytest.raises(r.R0HipError, match="wom.cpp:74"):
        r.recursion_witgen(dev(hal, RP.ctrl_group(prog, po2)), dd, dg, n, wom, cyc, iops)
    hal.synchronize()


@pytest.mark.parametrize("suite,po2", [("poseidon2", 14), ("sha-256", 16), ("poseidon2", 18)])
def test_prove_recursion_from_program(hal, hal_sha, oracle, suite, po2):
    """r0hip_prove_recursion: a recursion proof from the program (control group) and its
    preflight alone — witness generation, ZK noise, accumulation and the proof on the device.
    The seal passes r0hip_verify_seal with the validity equation; at po2 14 it equals the
    oracle prover's seal on the witness the reference's compiled witgen and accumulation make
    with the same noise words (r0hip_fill_uniform's generator, oracle.splitmix_fill)."""
    import recursion_program as RP
    import risc0_amd as r
    import verifier
    if not RP.available() or oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    h, s = H(suite), S(oracle, suite)
    n = 1 << po2
    rng = np.random.default_rng(3000 + po2)
    prog, inp = RP.random_program(rng, n - RP.ZK_CYCLES - 1)
    pf = RP.preflight(prog, inp)
    wom, cyc, iops = RP.trace_arrays(pf)
    ctrl = RP.ctrl_group(prog, po2)
    seed = 0x5EED + po2
    seal, mix = r.prove_recursion(h, po2, dev(h, ctrl), wom, cyc, iops, seed)
    assert r.verify_seal("recursion", s, seal) == po2
    if po2 == 14:
        assert verifier.verify(oracle, "recursion", seal, s, check_validity=True)["validity"] is True
        _, data, glob = RP.witgen(prog, pf, po2, raw=True)
        data = data.reshape(RP.DATA, n)
        data[:, n - RP.ZK_CYCLES:] = oracle.splitmix_fill(seed, RP.DATA * RP.ZK_CYCLES).reshape(RP.DATA, RP.ZK_CYCLES)
        data = np.where(data == RP.INVALID, 0, data).astype(np.uint32).reshape(-1)
        glob = np.where(glob == RP.INVALID, 0, glob).astype(np.uint32)
        acc0 = np.full((RP.ACCUM, n), RP.INVALID, np.uint32)
        acc0[:, n - RP.ZK_CYCLES:] = oracle.splitmix_fill(seed + 1, RP.ACCUM * RP.ZK_CYCLES).reshape(RP.ACCUM,
                                                                                                  RP.ZK_CYCLES)
        w = dict(ctrl=ctrl, data=data, glob=glob, work=len(prog.rows), acc0=acc0.reshape(-1))
        acc = RP.accumulate(w, mix, po2)
        ref_seal, ref_mix, _ = oracle.prove_segment("recursion", s, po2, ctrl, data, acc, glob)
        assert np.array_equal(mix, ref_mix)
        assert np.array_equal(seal, ref_seal)


@pytest.mark.gpu
def test_async_mirror_copy(hal):
    """r0hip_memcpy_d2h_start / r0hip_copy_finish (the HAL's node-heap mirrors): a copy into
    page-locked memory runs beside later calls and lands word for word, polled (block = 0) or
    waited; a pageable destination and an empty copy are done on return (NULL handle)."""
    import ctypes
    import risc0_amd as r
    lib = r.lib()
    n = 1 << 24  # 64 MB: long enough to still be in flight at the first poll
    src = np.random.default_rng(7).integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    d = hal.copy_from_elem("src", src)
    h = ctypes.c_void_p()
    r.check(lib.r0hip_host_alloc(ctypes.byref(h), n * 4))
    try:
        arr = np.ctypeslib.as_array(ctypes.cast(h, ctypes.POINTER(ctypes.c_uint32)), shape=(n,))
        arr[:] = 0
        for block in (0, 1):
            c, done = ctypes.c_void_p(), ctypes.c_int(-1)
            r.check(lib.r0hip_memcpy_d2h_start(h, d.ptr, n * 4, ctypes.byref(c)))
            assert c.value
            r.check(lib.r0hip_eltwise_zeroize_elem(hal.alloc_elem("other", 1 << 20).ptr, 1 << 20))  # a later call
            polls = 0
            while True:
                r.check(lib.r0hip_copy_finish(c, block, ctypes.byref(done)))
                if done.value:
                    break
                polls += 1
                assert polls < 10**7
            assert np.array_equal(arr, src)
            arr[:] = 0
        # pageable destination: copied before return, no handle
        page = np.zeros(n, dtype=np.uint32)
        c = ctypes.c_void_p(1)
        r.check(lib.r0hip_memcpy_d2h_start(page.ctypes.data, d.ptr, n * 4, ctypes.byref(c)))
        assert c.value is None and np.array_equal(page, src)
        r.check(lib.r0hip_memcpy_d2h_start(h, d.ptr, 0, ctypes.byref(c)))
        assert c.value is None
        done = ctypes.c_int(-1)
        r.check(lib.r0hip_copy_finish(None, 0, ctypes.byref(done)))
        assert done.value == 1
    finally:
        r.check(lib.r0hip_host_free(h))


@pytest.mark.gpu
def test_empty_inputs_are_no_ops(hal):
    """Every per-op entry point takes a zero count as the reference CPU HAL does (an empty loop,
    hal/cpu.rs:263-651): it returns success and writes nothing — no zero-sized grid reaches the
    runtime (a HIP launch of 0 workgroups is an error) and no word of the buffers changes."""
    import ctypes
    import risc0_amd as r
    lib = r.lib()
    sentinel = np.full(4096, 0x1234567, dtype=np.uint32)
    a, b, c = (hal.copy_from_elem(n, sentinel) for n in ("a", "b", "c"))
    u32 = ctypes.POINTER(ctypes.c_uint32)
    fe = (ctypes.c_uint32 * 4)(1, 2, 3, 4)
    which = (ctypes.c_uint32 * 1)(0)
    host = np.zeros(4, dtype=np.uint32)
    calls = {
        "memset32": lambda: lib.r0hip_memset32(a.ptr, 7, 0),
        "memcpy_h2d": lambda: lib.r0hip_memcpy_h2d(a.ptr, host.ctypes.data, 0),
        "memcpy_d2h": lambda: lib.r0hip_memcpy_d2h(host.ctypes.data, a.ptr, 0),
        "memcpy_d2d": lambda: lib.r0hip_memcpy_d2d(a.ptr, b.ptr, 0),
        "expand_evaluate": lambda: lib.r0hip_batch_expand_into_evaluate_ntt(a.ptr, b.ptr, 0, 6, 2),
        "interpolate": lambda: lib.r0hip_batch_interpolate_ntt(a.ptr, 0, 6),
        "zk_shift": lambda: lib.r0hip_zk_shift(a.ptr, 0, 6),
        "bit_reverse": lambda: lib.r0hip_batch_bit_reverse(a.ptr, 0, 6),
        "evaluate_any": lambda: lib.r0hip_batch_evaluate_any(a.ptr, b.ptr, 1, 6, c.ptr, c.ptr, 0),
        "mix_poly_coeffs": lambda: lib.r0hip_mix_poly_coeffs(a.ptr, b.ptr, ctypes.cast(which, u32),
                                                             ctypes.cast(fe, u32), ctypes.cast(fe, u32), 0, 64),
        "fri_fold": lambda: lib.r0hip_fri_fold(a.ptr, b.ptr, ctypes.cast(fe, u32), 0),
        "add_elem": lambda: lib.r0hip_eltwise_add_elem(a.ptr, b.ptr, c.ptr, 0),
        "copy_elem": lambda: lib.r0hip_eltwise_copy_elem(a.ptr, b.ptr, 0),
        "zeroize": lambda: lib.r0hip_eltwise_zeroize_elem(a.ptr, 0),
        "sum_extelem": lambda: lib.r0hip_eltwise_sum_extelem(a.ptr, b.ptr, 5, 0),
        "gather_sample": lambda: lib.r0hip_gather_sample(a.ptr, b.ptr, 3, 0, 64),
        "prefix_products": lambda: lib.r0hip_prefix_products(a.ptr, 0),
        "hash_rows": lambda: lib.r0hip_hash_rows(0, a.ptr, b.ptr, 0, 16),
        "hash_fold": lambda: lib.r0hip_hash_fold(0, a.ptr, 0, 0),
        "hash_rows_sha": lambda: lib.r0hip_hash_rows(1, a.ptr, b.ptr, 0, 16),
        "hash_fold_sha": lambda: lib.r0hip_hash_fold(1, a.ptr, 0, 0),
    }
    for name, call in calls.items():
        r.check(call())
        for buf in (a, b, c):
            assert np.array_equal(buf.to_numpy(), sentinel), name
    # a CSR scatter over zero cycles (index holds its one entry, 0)
    idx = hal.copy_from_elem("idx", np.zeros(1, dtype=np.uint32))
    r.check(lib.r0hip_scatter(a.ptr, idx.ptr, b.ptr, c.ptr, 0))
    assert np.array_equal(a.to_numpy(), sentinel)
