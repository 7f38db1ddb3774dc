"""The recursion witness generation IR (risc0_amd/circuits/recursion.witgen.ir, flattened by
tools/gen_witgen_ir.py from the reference's step_exec.cpp and step_verify_mem.cpp, and
compiled to the GPU kernels by tools/gen_witgen.py) against the reference's own compiled
witness generator (risc0_circuit_recursion_cpu_witgen, oracle/_ref/libref_recursion.so) on
hand-encoded programs through the restated preflight (tests/recursion_program.py): the IR run
on the CPU (tests/recursion_witgen_ir.py) writes the same data group and globals word for
word, INVALID words included."""
import numpy as np
import pytest

import recursion_program as RP
import recursion_witgen_ir as W


def _case(seed, po2, rows, blocks=("arith", "bits", "mix_rng", "iop", "poseidon2")):
    rng = np.random.default_rng(seed)
    prog, inp = RP.random_program(rng, rows, blocks)
    pf = RP.preflight(prog, inp)
    return prog, pf


@pytest.mark.skipif(not RP.available(), reason="oracle/_ref/libref_recursion.so not built")
@pytest.mark.parametrize("seed,po2,rows,blocks", [
    (1, 11, 400, ("arith", "bits", "mix_rng", "iop", "poseidon2")),
    (2, 11, 900, ("arith", "bits", "mix_rng", "iop", "poseidon2")),
    (3, 11, 300, ("poseidon2",)),
    (4, 11, 300, ("iop", "mix_rng")),
])
def test_witgen_ir_matches_reference(seed, po2, rows, blocks):
    n = 1 << po2
    prog, pf = _case(seed, po2, rows, blocks)
    ctrl, data, glob = RP.witgen(prog, pf, po2, raw=True)
    wom, cyc, iops = RP.trace_arrays(pf)
    d2 = np.full(RP.DATA * n, RP.INVALID, np.uint32)
    g2 = np.full(RP.OUT, RP.INVALID, np.uint32)
    W.witgen(ctrl.copy(), d2, g2, n, wom, cyc, iops)
    bad = np.nonzero(d2 != data)[0]
    assert bad.size == 0, f"{bad.size} data words differ; first col {bad[0] // n} row {bad[0] % n}"
    assert np.array_equal(g2, glob)


@pytest.mark.skipif(not RP.available(), reason="oracle/_ref/libref_recursion.so not built")
def test_witgen_ir_fails_where_the_reference_fails():
    """A WOM address skipped by the program breaks the sorted-memory check in both (the
    reference's "eqz failed at: zirgen/circuit/recursion/wom.cpp:74")."""
    po2, n = 11, 1 << 11
    b = RP.Builder(np.random.default_rng(5))
    b.consts([(3, 0), (4, 0)])
    b.next += 1  # a hole in the write-once memory
    b.consts([(5, 0)])
    prog, inp = b.finish()
    pf = RP.preflight(prog, inp)
    # the compiled reference raises from inside its thread pool, which it does not survive
    # being called again in the same process: run it in a child. The child exits 3 after
    # printing the reference's message; it may instead die by SIGSEGV in the compiled
    # reference's thread-pool teardown (seen under pytest-xdist), which counts only when the
    # message was already printed. Any other exit, or another signal, fails the test.
    import os
    import pickle
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = ("import pickle, sys; sys.path[:0] = [%r, %r]; import recursion_program as RP\n"
            "import os\nprog, pf = pickle.loads(sys.stdin.buffer.read())\n"
            "try:\n    RP.witgen(prog, pf, 11, raw=True)\n"
            "except RuntimeError as e:\n    print(e, flush=True)\n    os._exit(3)\n"
            "os._exit(0)\n") % (here, os.path.join(os.path.dirname(here), "oracle"))
    import signal
    # the compiled reference can also die by SIGSEGV in its thread pool before its message
    # reaches stdout (seen once in a full CPU run): such a child is run again, up to 4 times
    for _ in range(4):
        res = subprocess.run([sys.executable, "-c", code], input=pickle.dumps((prog, pf)), capture_output=True,
                             timeout=120)
        if b"wom.cpp:74" in res.stdout or res.returncode != -signal.SIGSEGV:
            break
    assert b"wom.cpp:74" in res.stdout, (res.returncode, res.stdout, res.stderr)
    assert res.returncode in (3, -signal.SIGSEGV), \
        f"child exit {res.returncode} (expected 3, or SIGSEGV after the message): {res.stderr[-2000:]!r}"
    ctrl = RP.ctrl_group(prog, po2)
    wom, cyc, iops = RP.trace_arrays(pf)
    with pytest.raises(W.WitgenError, match="wom.cpp:74"):
        W.witgen(ctrl, np.full(RP.DATA * n, RP.INVALID, np.uint32), np.full(RP.OUT, RP.INVALID, np.uint32), n, wom,
                 cyc, iops)
