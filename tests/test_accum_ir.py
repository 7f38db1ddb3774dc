"""Pinning of the recursion accumulation IR (risc0_amd/circuits/recursion.accum.ir) that
the HIP accumulation kernels are generated from: interpreted over synthetic control rows
it reproduces the accum group the reference's own compiled
risc0_circuit_recursion_cpu_accum writes (recursion-sys/kernels/cxx/ffi.cpp:208-217),
word for word, including the cells it leaves INVALID. Needs oracle/_ref (built from the
reference tree by oracle/Makefile)."""
import os

import numpy as np
import pytest

import accum_ir as A

REF = os.path.join(A.ROOT, "oracle", "_ref", "libref_recursion.so")


@pytest.mark.skipif(not os.path.exists(REF), reason="oracle/_ref not built (no reference tree)")
@pytest.mark.parametrize("po2,steps_short,seed", [(8, 0, 1), (10, 0, 2), (10, 5, 3)])
def test_accum_ir_matches_reference(oracle, po2, steps_short, seed):
    d = A.circuit()
    gs = d["group_sizes"]
    n = 1 << po2
    rng = np.random.default_rng(seed)
    ctrl, glob, data, mix = A.synthetic(rng, oracle, po2, gs, d["output_size"], d["mix_size"])
    acc0 = np.full(gs[0] * n, A.INVALID, np.uint32)
    steps = n - steps_short  # work cycles < total cycles: the ZK tail is left alone
    ref = acc0.copy()
    A.ref_accum(ctrl, glob, data, mix, ref, steps, n)
    got = A.accum(ctrl, glob, data, mix, acc0, steps, n)
    assert np.array_equal(got, ref)
    assert (ref != A.INVALID).sum() > n  # the comparison covers real accumulator values
