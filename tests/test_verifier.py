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
    assert r.verify_seal(circuit, s, seal) == po2
    rng = np.random.default_rng(po2 * 7 + s)
    for where in [1, 2, 9, seal.size // 4, seal.size // 2, seal.size - 3] + list(rng.integers(0, seal.size, 6)):
        bad = seal.copy()
        bad[where] ^= np.uint32(1 << int(rng.integers(0, 31)))
        with pytest.raises(verifier.VerificationError):
            verifier.verify(oracle, circuit, bad, s)
        with pytest.raises(r.R0HipError):
            r.verify_seal(circuit, s, bad)
    for bad, msg in ((seal[:-1], "seal too short"), (np.append(seal, np.uint32(0)), "trailing words")):
        with pytest.raises(r.R0HipError, match=msg):
            r.verify_seal(circuit, s, bad)
    with pytest.raises(r.R0HipError):  # another suite's transcript
        r.verify_seal(circuit, (s + 1) % 3, seal)
    with pytest.raises(r.R0HipError, match="unknown circuit"):
        r.verify_seal("nope", s, seal)
