"""CPU pinning of tests/hal_prover.py, the reference Prover call sequence over the Hal
methods: run over the CPU oracle (tests/oracle_hal.py, the CpuHal role), it reproduces
the golden seal digests that r0hip_prove_segment and the oracle's own C++ prover match.
The GPU test test_per_op_abi_prover_matches_golden_seal runs the same sequence over
risc0_amd.HipHal, so a mismatch there is in the HIP ops, not in this restatement."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import test_golden as G  # noqa: E402

SMALL = [i for i, c in enumerate(G.INDEX["seals"]) if c["po2"] <= 9]


@pytest.mark.parametrize("idx", SMALL)
def test_hal_prover_over_oracle_matches_golden(idx, oracle):
    import hal_prover
    from oracle_hal import OracleHal
    case = G.INDEX["seals"][idx]
    suite = {"poseidon2": oracle.POSEIDON2, "sha-256": oracle.SHA256, "poseidon_254": oracle.POSEIDON254}[case["suite"]]
    h = OracleHal(oracle, suite)
    code, data, accum, glob = G.seal_inputs(oracle, case["circuit"], case["po2"])
    bufs = [h.copy_from_elem("x", x) for x in (code, data, accum, glob)]
    seal, mix = hal_prover.prove_segment(oracle, h, case["circuit"], case["po2"], *bufs)
    assert [int(x) for x in mix] == case["mix"]
    assert G.digest(seal) == case["seal_sha256"], case
