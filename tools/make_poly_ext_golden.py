"""Golden vectors for the recursion verifier's constraint program: the reference's own
DEF table (risc0/circuit/recursion/src/poly_ext.rs, read in place) run by the restated
interpreter (tests/poly_ext_def.py, adapter.rs:317-400) on N seeded inputs
(poly_ext_def.inputs: splitmix64 words, seed 0x504F4C59 + k). Writes only the outputs,
MixState.tot as Montgomery words, to tests/golden/poly_ext_recursion.npy (N x 4 u32); the
inputs are regenerated from the seed by the test.

    python3 tools/make_poly_ext_golden.py [N]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), ROOT]

import oracle  # noqa: E402
import poly_ext_def as D  # noqa: E402
import verifier  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    steps, ret = D.parse()
    d = oracle.load_circuit_json("recursion")
    taps = verifier.Taps("recursion")
    pm, u, g, m = D.inputs(oracle, n, taps.num_taps, d["mix_size"], d["output_size"])
    out = D.evaluate(steps, ret, pm, u, g, m)
    path = os.path.join(ROOT, "tests", "golden", "poly_ext_recursion.npy")
    np.save(path, out)
    print(f"{path}: {out.shape}")


if __name__ == "__main__":
    main()
