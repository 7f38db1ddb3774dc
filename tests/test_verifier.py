"""The Python restatement of the reference verifier (tests/verifier.py) accepts the
oracle's seals and rejects tampered ones — the checker the GPU full-size tests use."""
import numpy as np
import pytest

import test_golden as G
import verifier

CASES = [("rv32im", "poseidon2", 8), ("rv32im", "sha-256", 9), ("recursion", "poseidon2", 9),
         ("recursion", "sha-256", 8), ("recursion", "poseidon_254", 8)]
SUITES = {"poseidon2": 0, "sha-256": 1, "poseidon_254": 2}


@pytest.mark.parametrize("circuit,suite,po2", CASES)
def test_verifier_accepts_oracle_seals(oracle, circuit, suite, po2):
    if oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    code, data, accum, glob = G.seal_inputs(oracle, circuit, po2)
    s = SUITES[suite]
    seal, _mix, _ = oracle.prove_segment(circuit, s, po2, code, data, accum, glob,
                                         version=2 if circuit == "rv32im" else None)
    r = verifier.verify(oracle, circuit, seal, s, check_validity=True)
    assert r["po2"] == po2 and r["words"] == seal.size - (1 if circuit == "rv32im" else 0)
    # synthetic witnesses do not satisfy the constraints, so DEEP-ALI validity fails
    assert r["validity"] is False
    # a flipped bit anywhere — header, Merkle data, U coefficients, FRI — is rejected
    for where in (2, seal.size // 4, seal.size // 2, seal.size - 3):
        bad = seal.copy()
        bad[where] ^= np.uint32(1 << 7)
        with pytest.raises(verifier.VerificationError):
            verifier.verify(oracle, circuit, bad, s)


@pytest.mark.parametrize("circuit,suite,po2", CASES)
def test_native_verifier_matches_restatement(oracle, circuit, suite, po2):
    """r0hip_verify_seal (risc0_amd/csrc/verify.cpp) — host code, no GPU — accepts what the
    restatement accepts and rejects the same tampered, truncated and padded seals."""
    import os
    import risc0_amd as r
    from risc0_amd.hal import LIB_PATH
    if oracle.ref_lib() is None or not os.path.exists(LIB_PATH):
        pytest.skip("oracle/_ref or libr0hip.so not built")
    code, data, accum, glob = G.seal_inputs(oracle, circuit, po2)
    s = SUITES[suite]
    seal, _mix, _ = oracle.prove_segment(circuit, s, po2, code, data, accum, glob,
                                         version=2 if circuit == "rv32im" else None)
    assert r.verify_seal(circuit, s, seal, check_validity=False) == po2
    # synthetic witnesses break the constraints: both verifiers see it
    with pytest.raises(r.R0HipError, match="proof is invalid"):
        r.verify_seal(circuit, s, seal)
    rng = np.random.default_rng(po2 * 7 + s)
    for where in [1, 2, 9, seal.size // 4, seal.size // 2, seal.size - 3] + list(rng.integers(0, seal.size, 6)):
        bad = seal.copy()
        bad[where] ^= np.uint32(1 << int(rng.integers(0, 31)))
        with pytest.raises(verifier.VerificationError):
            verifier.verify(oracle, circuit, bad, s)
        with pytest.raises(r.R0HipError):
            r.verify_seal(circuit, s, bad, check_validity=False)
    for bad, msg in ((seal[:-1], "seal too short"), (np.append(seal, np.uint32(0)), "trailing words")):
        with pytest.raises(r.R0HipError, match=msg):
            r.verify_seal(circuit, s, bad, check_validity=False)
    with pytest.raises(r.R0HipError):  # another suite's transcript
        r.verify_seal(circuit, (s + 1) % 3, seal, check_validity=False)
    with pytest.raises(r.R0HipError, match="unknown circuit"):
        r.verify_seal("nope", s, seal)


def _native_lib_or_skip(oracle):
    import os
    from risc0_amd.hal import LIB_PATH
    if oracle.ref_lib() is None or not os.path.exists(LIB_PATH):
        pytest.skip("oracle/_ref or libr0hip.so not built")


@pytest.mark.parametrize("circuit", ["rv32im", "recursion"])
def test_native_poly_ext_matches_restatement(oracle, circuit):
    """r0hip_poly_ext (the constraint program run over FpExt on the host) equals the
    Python IR interpretation on random out-of-domain inputs."""
    import risc0_amd as r
    _native_lib_or_skip(oracle)
    taps = verifier.Taps(circuit)
    d = taps.d
    rng = np.random.default_rng(11)
    for _ in range(3):
        mix = oracle.rand_elems(rng, d["mix_size"])
        glob = oracle.rand_elems(rng, d["output_size"])
        eval_u = oracle.rand_elems(rng, 4 * taps.num_taps)
        pm = oracle.rand_elems(rng, 4)
        got = tuple(verifier.dec(w) for w in r.poly_ext(circuit, mix, glob, eval_u, pm))
        want = verifier.poly_ext(circuit, taps, tuple(verifier.dec(w) for w in pm),
                                 verifier.ext_words(eval_u), glob, mix)
        assert got == want


@pytest.mark.parametrize("circuit", ["rv32im", "recursion"])
def test_native_poly_ext_matches_compiled_poly_fp(oracle, circuit):
    """r0hip_poly_ext against the reference's own compiled constraint code: on 1000 random
    base-field tap assignments, the validity polynomial the verifier evaluates over FpExt
    (each tap embedded as (u, 0, 0, 0)) equals the reference's risc0_circuit_<c>_cpu_poly_fp
    (rv32im-sys/kernels/cxx/eval_check.cpp:31-39, recursion-sys poly_fp.cpp) at a cycle whose
    taps read those values (oracle_poly_fp_at_taps), with a random FpExt poly_mix, mix and
    globals. For rv32im this is the reference-code pin of the constraint program (its
    poly_ext.rs is not in the reference tree)."""
    import risc0_amd as r
    _native_lib_or_skip(oracle)
    taps = verifier.Taps(circuit)
    d = taps.d
    rng = np.random.default_rng(0x50465450)
    for _ in range(1000):
        u = oracle.rand_elems(rng, taps.num_taps)
        mix = oracle.rand_elems(rng, d["mix_size"])
        glob = oracle.rand_elems(rng, d["output_size"])
        pm = oracle.rand_elems(rng, 4)
        eval_u = np.zeros(4 * taps.num_taps, np.uint32)
        eval_u[0::4] = u
        got = r.poly_ext(circuit, mix, glob, eval_u, pm)
        want = oracle.poly_fp_at_taps(circuit, u, mix, glob, pm)
        assert np.array_equal(got, want), (got, want)


def _poly_ext_golden_inputs(oracle, n):
    import poly_ext_def as D
    d = oracle.load_circuit_json("recursion")
    return D.inputs(oracle, n, verifier.Taps("recursion").num_taps, d["mix_size"], d["output_size"])


def test_native_poly_ext_matches_reference_constraint_program(oracle):
    """r0hip_poly_ext("recursion") equals the reference verifier's own constraint program on
    1000 seeded (poly_mix, eval_u, global, mix) inputs: the DEF table of
    risc0/circuit/recursion/src/poly_ext.rs run by a restatement of PolyExtExecutor
    (zkp/src/adapter.rs:317-400), whose outputs are the committed fixture
    tests/golden/poly_ext_recursion.npy (tools/make_poly_ext_golden.py). The Python
    restatement (tests/verifier.py poly_ext, over the IR the library embeds) agrees too."""
    import os
    import risc0_amd as r
    from risc0_amd.hal import LIB_PATH
    if not os.path.exists(LIB_PATH):
        pytest.skip("libr0hip.so not built")
    want = np.load(os.path.join(os.path.dirname(__file__), "golden", "poly_ext_recursion.npy"))
    pm, u, g, m = _poly_ext_golden_inputs(oracle, want.shape[0])
    got = np.stack([r.poly_ext("recursion", m[k], g[k], u[k], pm[k]) for k in range(want.shape[0])])
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} of {want.shape[0]} inputs differ, first {bad[0]}"
    taps = verifier.Taps("recursion")
    for k in range(5):
        ours = verifier.poly_ext("recursion", taps, tuple(verifier.dec(w) for w in pm[k]), verifier.ext_words(u[k]),
                                 g[k], m[k])
        assert tuple(verifier.enc(x) for x in ours) == tuple(int(x) for x in want[k])


def test_poly_ext_golden_is_the_reference_constraint_program(oracle):
    """The fixture above re-derived from the reference's poly_ext.rs where it lies (skipped
    without /root/reference): the first 100 vectors, and the table's shape."""
    import os
    import poly_ext_def as D
    if not D.available():
        pytest.skip("/root/reference not present")
    steps, ret = D.parse()
    assert len(steps) == 12359 and ret == 1228
    want = np.load(os.path.join(os.path.dirname(__file__), "golden", "poly_ext_recursion.npy"))[:100]
    pm, u, g, m = _poly_ext_golden_inputs(oracle, 100)
    assert np.array_equal(D.evaluate(steps, ret, pm, u, g, m), want)


@pytest.mark.parametrize("suite", ["poseidon2", "sha-256", "poseidon_254"])
def test_valid_recursion_seal_passes_validity(oracle, suite):
    """A witness that satisfies the recursion circuit (all-zero code/data/accum; the
    constraints hold for any globals and mix) gives a seal whose validity equation holds in
    the restatement and in the native verifier; a flipped coefficient breaks it."""
    import risc0_amd as r
    _native_lib_or_skip(oracle)
    po2, s = 8, SUITES[suite]
    d = oracle.load_circuit_json("recursion")
    n, gs = 1 << po2, d["group_sizes"]
    code, data, accum = (np.zeros(gs[g] * n, np.uint32) for g in (1, 2, 0))
    glob = oracle.rand_elems(np.random.default_rng(5), d["output_size"])
    seal, _mix, _ = oracle.prove_segment("recursion", s, po2, code, data, accum, glob, version=None)
    assert verifier.verify(oracle, "recursion", seal, s, check_validity=True)["validity"] is True
    assert r.verify_seal("recursion", s, seal) == po2


@pytest.mark.parametrize("suite", ["poseidon2", "sha-256", "poseidon_254"])
def test_satisfying_recursion_program_seal_passes_validity(oracle, suite):
    """A non-trivial satisfying witness: a hand-encoded recursion program (arithmetic, bit
    ops, MIX_RNG, IOP reads, Poseidon2; tests/recursion_program.py) run through a restatement
    of the reference preflight (prove/preflight.rs) and the reference's own compiled witness
    generator and accumulation. Its constraints hold on every row; the oracle's seal of it
    passes the validity equation in the restated verifier and in r0hip_verify_seal, and one
    flipped witness word breaks both."""
    import recursion_program as RP
    import risc0_amd as r
    _native_lib_or_skip(oracle)
    if not RP.available():
        pytest.skip("oracle/_ref/libref_recursion.so not built")
    po2, s = 11, SUITES[suite]
    w = RP.satisfying_witness(77, po2)
    assert w["work"] > 900 and len(w["preflight"].iops) > 0
    _, mix, _ = oracle.prove_segment("recursion", s, po2, w["ctrl"], w["data"], w["acc0"] * 0, w["glob"])
    acc = RP.accumulate(w, mix, po2)
    rc = RP.row_constraints(w["ctrl"], w["data"], acc, w["glob"], mix, po2)
    assert not rc.any(), f"constraints fail on rows {np.nonzero(rc.any(axis=0))[0][:8]}"
    seal, mix2, _ = oracle.prove_segment("recursion", s, po2, w["ctrl"], w["data"], acc, w["glob"])
    assert np.array_equal(mix, mix2)
    assert verifier.verify(oracle, "recursion", seal, s, check_validity=True)["validity"] is True
    assert r.verify_seal("recursion", s, seal) == po2
    bad = w["data"].copy()
    bad[7 * (1 << po2) + 5] ^= 1
    _, mixb, _ = oracle.prove_segment("recursion", s, po2, w["ctrl"], bad, acc, w["glob"])
    seal_b, _, _ = oracle.prove_segment("recursion", s, po2, w["ctrl"], bad, RP.accumulate(dict(w, data=bad), mixb, po2),
                                        w["glob"])
    assert verifier.verify(oracle, "recursion", seal_b, s, check_validity=True)["validity"] is False
    with pytest.raises(r.R0HipError):
        r.verify_seal("recursion", s, seal_b)


def test_native_verifier_rejects_garbage(oracle):
    """Malformed seals (empty, random words, a valid prefix with a tampered po2 or cut
    anywhere) come back as errors, never as a crash or an out-of-bounds read."""
    import risc0_amd as r
    _native_lib_or_skip(oracle)
    rng = np.random.default_rng(99)
    for circuit in ("rv32im", "recursion"):
        for s in (0, 1, 2):
            for n in (0, 1, 5, 64, 4096):
                junk = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
                if circuit == "rv32im" and n:
                    junk[0] = 2
                with pytest.raises(r.R0HipError):
                    r.verify_seal(circuit, s, junk, check_validity=False)
    code, data, accum, glob = G.seal_inputs(oracle, "recursion", 8)
    seal, _mix, _ = oracle.prove_segment("recursion", 0, 8, code, data, accum, glob)
    po2_at = verifier.Taps("recursion").d["output_size"]
    for po2 in (0, 1, 9, 25, 2**31):
        bad = seal.copy()
        bad[po2_at] = po2
        with pytest.raises(r.R0HipError):
            r.verify_seal("recursion", 0, bad, check_validity=False)
    for cut in rng.integers(1, seal.size, 20):
        with pytest.raises(r.R0HipError, match="seal too short"):
            r.verify_seal("recursion", 0, seal[:cut], check_validity=False)


def test_native_verifier_binds_code_root_and_canonical_words(oracle):
    """check_code (zkp/src/verify/mod.rs:531): the code root comes back and an allow-list
    is enforced; field words >= p are rejected as read_field_elem_slice's checked cast
    rejects them (read_iop.rs:45-48), even though they are congruent to valid words."""
    import risc0_amd as r
    _native_lib_or_skip(oracle)
    po2, s = 8, 0
    d = oracle.load_circuit_json("recursion")
    n, gs = 1 << po2, d["group_sizes"]
    code, data, accum = (np.zeros(gs[g] * n, np.uint32) for g in (1, 2, 0))
    glob = oracle.rand_elems(np.random.default_rng(6), d["output_size"])
    seal, _mix, _ = oracle.prove_segment("recursion", s, po2, code, data, accum, glob, version=None)
    got, root = r.verify_seal("recursion", s, seal, return_code_root=True)
    assert got == po2 and root.any()
    other = root.copy()
    other[0] ^= 1
    assert r.verify_seal("recursion", s, seal, code_roots=np.concatenate([other, root])) == po2
    with pytest.raises(r.R0HipError, match="code root"):
        r.verify_seal("recursion", s, seal, code_roots=other)
    bad = seal.copy()
    bad[0] += np.uint32(oracle.P)  # a header global, congruent to the original
    with pytest.raises(r.R0HipError, match="non-canonical"):
        r.verify_seal("recursion", s, bad, check_validity=False)
    rng = np.random.default_rng(7)
    for where in rng.choice(np.nonzero(seal < np.uint32(2**32 - oracle.P))[0], 60, replace=False):
        bad = seal.copy()
        bad[where] += np.uint32(oracle.P)
        with pytest.raises(r.R0HipError):
            r.verify_seal("recursion", s, bad, check_validity=False)
