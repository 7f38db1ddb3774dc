"""rv32im BigInt accumulator states (WitnessGenerator::accum's injection,
risc0/circuit/rv32im/src/prove/witgen/mod.rs:178-205) on the CPU:

* the product's host restatement of BigIntAccum (risc0_amd/csrc/bigint.cpp,
  r0hip_rv32im_bigint_accum_states; no GPU needed) equals the Python restatement
  (tests/bigint_accum.py, byte_poly.rs:381-470) and fails where the reference fails;
* with those states injected, the rv32im accumulation step IR equals the reference's own
  compiled stepAccum on rows whose arm-12 cycles run every PolyOp, and so does the
  reference's whole accumulation (phases 1-3);
* the compiled reference, run in row order, rewrites every injected state with the same
  words: the host states are exactly what the circuit's step computes.
"""
import os

import numpy as np
import pytest

import bigint_accum as B
import rv32im_accum_ref as R


def _lib_or_skip():
    from risc0_amd.hal import LIB_PATH
    if not os.path.exists(LIB_PATH):
        pytest.skip("libr0hip.so not built")


def _mix(rng):
    return rng.integers(0, B.P, R.MIX_WORDS, dtype=np.uint64).astype(np.uint32)


@pytest.mark.parametrize("seed", range(4))
def test_native_states_match_restatement(seed):
    import risc0_amd as r
    _lib_or_skip()
    rng = np.random.default_rng(0xB16 + seed)
    mix = _mix(rng)
    _, recs = B.lay_out(rng, 1 << 10, 40)
    assert {rec[1] for rec in recs} == set(range(7))
    got = r.bigint_accum_states(mix, recs, 1 << 10)
    assert np.array_equal(got, B.states(mix, recs))
    assert r.bigint_accum_states(mix, [], 16).shape == (0, 12)


def test_native_states_fail_as_the_reference():
    import risc0_amd as r
    _lib_or_skip()
    rng = np.random.default_rng(7)
    mix = _mix(rng)
    _, recs = B.lay_out(rng, 256, 9)
    recs = [(row, op, c, list(by)) for row, op, c, by in recs]
    eqz = next(i for i, rec in enumerate(recs) if rec[1] == B.EQ_ZERO)
    bad = [[row, op, c, list(by)] for row, op, c, by in recs]
    bad[eqz][3][0] ^= 1  # the integer identity no longer holds
    with pytest.raises(ValueError, match="Invalid eqz"):
        B.states(mix, bad)
    with pytest.raises(r.R0HipError, match="Invalid eqz in bigint accum"):
        r.bigint_accum_states(mix, bad, 256)
    bad = [[row, op, c, list(by)] for row, op, c, by in recs]
    bad[1][1] = 7
    with pytest.raises(r.R0HipError, match="invalid poly_op"):
        r.bigint_accum_states(mix, bad, 256)
    with pytest.raises(r.R0HipError, match="increasing row order"):
        r.bigint_accum_states(mix, [recs[1], recs[0]], 256)
    with pytest.raises(r.R0HipError, match="outside the segment"):
        r.bigint_accum_states(mix, recs, recs[-1][0])


@pytest.mark.skipif(not R.available(), reason="oracle/_ref/libref_rv32im_accum.so not built")
@pytest.mark.parametrize("rows,calls", [(128, 6), (512, 30)])
def test_accum_ir_with_bigint_cycles_matches_reference(rows, calls):
    import rv32im_accum_ir as IRI
    rng = np.random.default_rng(rows + calls)
    glob, mix = (rng.integers(0, B.P, n, dtype=np.uint64).astype(np.uint32) for n in (R.GLOBAL_WORDS, R.MIX_WORDS))
    data, recs = B.lay_out(rng, rows, calls)
    assert {rec[1] for rec in recs} == set(range(7))
    acc0 = B.inject(np.full(R.ACCUM_COLS * rows, R.INVALID, np.uint32), rows, mix, recs)
    ref = R.accum(data, glob, mix, rows, rows, phase1_only=True, accum_init=acc0)
    ours = acc0.copy()
    IRI.run(data.copy(), ours, glob, mix, rows, rows)
    bad = np.nonzero(ours != ref)[0]
    assert bad.size == 0, f"{bad.size} words differ; first at col {bad[0] // rows} row {bad[0] % rows}"
    # the reference's step, run in row order, writes the same states the host injected
    st = ref.reshape(R.ACCUM_COLS, rows)[:12, [rec[0] for rec in recs]].T
    assert np.array_equal(st, B.states(mix, recs))
    # and its whole accumulation accepts the injected group (phases 2-3 on top)
    full = R.accum(data, glob, mix, rows, rows, accum_init=acc0)
    assert np.array_equal(full.reshape(R.ACCUM_COLS, rows)[:12], ref.reshape(R.ACCUM_COLS, rows)[:12])
