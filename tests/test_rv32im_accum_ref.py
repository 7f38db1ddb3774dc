"""rv32im accumulation phases 2-3 (the scan of the last 4 accum columns and the totals
added to the machine columns, rv32im-sys/kernels/cxx/ffi.cpp:326-360) pinned to the
reference itself: its phase 1 (stepAccum) output, finished by the oracle's restatement,
must equal its whole risc0_circuit_rv32im_cpu_accum (tests/rv32im_accum_ref.py)."""
import numpy as np
import pytest

import rv32im_accum_ref as R

pytestmark = pytest.mark.skipif(not R.available(), reason="oracle/_ref/libref_rv32im_accum.so not built")

SPLIT = 23  # kUserAccumSplit = kLayout_TopAccum.columns[0].col (ffi.cpp:52)


def inputs(rows, seed):
    rng = np.random.default_rng(seed)
    draw = lambda n: rng.integers(0, R.P, n, dtype=np.uint64).astype(np.uint32)
    return draw(R.DATA_COLS * rows), draw(R.GLOBAL_WORDS), draw(R.MIX_WORDS)


@pytest.mark.parametrize("rows,last", [(64, 64), (256, 200)])
def test_accum_phases_2_3_restatement_matches_reference(oracle, rows, last):
    data, glob, mix = inputs(rows, rows + last)
    p1 = R.accum(data, glob, mix, rows, last, phase1_only=True)
    full = R.accum(data, glob, mix, rows, last)
    # phase 1 wrote the accumulator columns of the arm the rows select (every row of them),
    # including the 4 running-sum columns phase 2 scans; phases 2-3 changed them
    used = p1.reshape(R.ACCUM_COLS, rows)[:, :last]
    written = [c for c in range(R.ACCUM_COLS) if not np.any(used[c] == R.INVALID)]
    assert set(range(R.ACCUM_COLS - 4, R.ACCUM_COLS)) <= set(written)
    assert not np.array_equal(p1, full)
    ours = p1.copy()
    oracle.rv32im_accum_finalize(ours, rows, R.ACCUM_COLS, SPLIT, last)
    assert np.array_equal(ours, full)


def test_zero_rows_stop_at_an_unreachable_mux_arm():
    """All-zero data rows select no arm of the top-level state mux (exec_TopExtract): the
    reference's phase 1 aborts, which is why the synthetic rows above are random."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import numpy as np, rv32im_accum_ref as R; "
            "R.accum(np.zeros(R.DATA_COLS * 16, np.uint32), np.zeros(R.GLOBAL_WORDS, np.uint32), "
            "np.zeros(R.MIX_WORDS, np.uint32), 16, 16, phase1_only=True)") % __import__("os").path.dirname(__file__)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "unreachable mux arm" in r.stderr


def test_reference_accum_rate():
    """the compiled reference's whole accumulation at 2^14 rows (sizes the GPU parity test)"""
    import time
    rows = 1 << 14
    rng = np.random.default_rng(5)
    data, glob, mix = inputs(rows, 5)
    t = time.perf_counter()
    R.accum(data, glob, mix, rows, rows)
    print(f"reference rv32im cpu_accum: {rows / (time.perf_counter() - t):.0f} rows/s")
