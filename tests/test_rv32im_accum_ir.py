"""The rv32im accumulation step flattened to block IR (risc0_amd/circuits/rv32im.accum.ir,
tools/gen_rv32im_accum_ir.py) against the reference's own compiled phase 1 (stepAccum,
oracle/_ref/libref_rv32im_accum.so): same accum words on random data rows taking each of
the 13 instruction arms (and a mix of them)."""
import numpy as np
import pytest

import rv32im_accum_ir as IRI
import rv32im_accum_ref as R


SELECTORS = list(range(1, 14))  # instResult._selector[k]._super: data columns 1..13 (layout.cpp.inc)


def rows_for_arms(rng, rows, arms):
    """random rows; row r takes instruction arm arms[r] (its earlier selectors zeroed, the
    first nonzero selector wins as in the reference's if/else-if mux)"""
    draw = lambda n: rng.integers(1, R.P, n, dtype=np.uint64).astype(np.uint32)
    data = draw(R.DATA_COLS * rows).reshape(R.DATA_COLS, rows)
    for r, a in enumerate(arms):
        data[SELECTORS[:a], r] = 0
        if a == 12:
            # the big-integer arm's polyOp (data column 32) must decode one-hot (EQZ at
            # one_hot.zir:9); 0 selects BigIntPolyOpNop. The other ops read the previous
            # cycle's BigInt accumulator state (back 1), which the witness generator injects
            # before the step (witgen/mod.rs:178-205): rows running them come from
            # tests/bigint_accum.py with their states (tests/test_bigint_accum.py and the
            # *_bigint_* GPU tests).
            data[32, r] = 0
    return data.reshape(-1)


@pytest.mark.skipif(not R.available(), reason="oracle/_ref/libref_rv32im_accum.so not built")
@pytest.mark.parametrize("rows,last,arm", [(64, 64, 0), (128, 100, 0), (256, 256, "mixed")] +
                         [(32, 32, a) for a in range(1, 13)])
def test_accum_ir_matches_reference_phase1(rows, last, arm):
    rng = np.random.default_rng(rows + last + (99 if arm == "mixed" else arm))
    draw = lambda n: rng.integers(0, R.P, n, dtype=np.uint64).astype(np.uint32)
    glob, mix = draw(R.GLOBAL_WORDS), draw(R.MIX_WORDS)
    data = rows_for_arms(rng, rows, list(rng.integers(0, 13, rows)) if arm == "mixed" else [arm] * rows)
    ref = R.accum(data, glob, mix, rows, last, phase1_only=True)
    ours = np.full(R.ACCUM_COLS * rows, R.INVALID, np.uint32)
    IRI.run(data.copy(), ours, glob, mix, rows, last)
    bad = np.nonzero(ours != ref)[0]
    assert bad.size == 0, f"{bad.size} words differ; first at col {bad[0] // rows} row {bad[0] % rows}"
