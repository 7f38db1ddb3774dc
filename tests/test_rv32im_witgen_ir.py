"""rv32im witness generation on the CPU: the restated preflight (tests/rv32im_trace.py) is
accepted by the reference's compiled witness generator (risc0_circuit_rv32im_cpu_witgen,
rv32im-sys/kernels/cxx/ffi.cpp:267-308), and the committed block IR the GPU kernels are
generated from (risc0_amd/circuits/rv32im.witgen.ir) reproduces its data and global groups
word for word, INVALID words included. Failing traces fail in both."""
import os

import numpy as np
import pytest

import rv32im_trace as T
import rv32im_witgen_ir as I
import rv32im_witgen_ref as W

needs_ref = pytest.mark.skipif(not os.path.exists(W.RA.LIB), reason="oracle/_ref/libref_rv32im_accum.so not built")


def test_trace_shapes():
    """fini's reserved rows and the split (preflight.rs:205-326), the injected cycle columns"""
    t = T.random_trace(13, 300, seed=7)
    cyc, tx = t.arrays()
    n = 1 << 13
    assert len(cyc) == n and t.table_split_cycle + T.RESERVED_CYCLES <= n
    assert list(cyc["state"][t.table_split_cycle:t.table_split_cycle + 3]) == [T.CONTROL_TABLE] * 3
    assert cyc["state"][-1] == T.CONTROL_DONE and cyc["major"][-1] == 7 and cyc["minor"][-1] == 7
    # every transaction belongs to its cycle (txn.cycle / 2) and each address's first
    # transaction wraps to that address's last cycle
    owner = np.searchsorted(cyc["txnIdx"].astype(np.int64), np.arange(len(tx)), side="right") - 1
    assert np.array_equal(tx["cycle"] // 2, owner)
    lay = W.layout()
    r, c, v = t.injector(lay)
    assert (c == lay["cycle"]).sum() == n


@needs_ref
@pytest.mark.parametrize("po2,n,seed", [(13, 1, 3), (13, 600, 1), (14, 2500, 2), (14, 2500, 5)])
def test_ir_matches_reference(po2, n, seed):
    t = T.random_trace(po2, n, seed=seed) if n > 1 else T.Trace(po2, [T.asm("addi", 1, 0, 5)])
    data, glob, cyc, tx = W.inputs(t)
    ref_d, ref_g = W.run(data, glob, cyc, tx, t.table_split_cycle, 1 << po2)
    assert (ref_d == W.INVALID).any() and (ref_d != data).any()
    d, g = I.witgen(data.copy(), glob.copy(), cyc.copy(), tx, 1 << po2)
    assert np.array_equal(d, ref_d), np.flatnonzero(d != ref_d)[:10]
    assert np.array_equal(g, ref_g)


@needs_ref
@pytest.mark.parametrize("terminate,bigint", [(True, True), (False, False)])
def test_ir_matches_reference_with_ecalls(terminate, bigint):
    """user ecalls into a machine-mode kernel: Poseidon2 ecalls (with and without state, bytes
    and field elements), host write, an unaligned host read, SHA-256, mret, terminate, and a
    BigInt ecall (every PolyOp and MemoryOp; its witness bytes in the trace's bigint array)"""
    t = T.ecall_trace(14, seed=3, terminate=terminate, bigint=bigint)
    assert t.terminated == terminate
    data, glob, cyc, tx = W.inputs(t)
    majors = set(int(m) for m in cyc["major"][:t.table_split_cycle])
    assert {0, 1, 7, 8, 9, 10, 11} <= majors and (12 in majors) == bigint
    bi = t.bigint_array()
    assert len(bi) == 16 * (12 in majors) * 18
    ref_d, ref_g = W.run(data, glob, cyc, tx, t.table_split_cycle, 1 << 14, bigint=bi)
    d, g = I.witgen(data.copy(), glob.copy(), cyc.copy(), tx, 1 << 14, bigint=bi)
    assert np.array_equal(d, ref_d) and np.array_equal(g, ref_g)


@needs_ref
def test_reference_modes_agree():
    """the reference's parallel schedule (phase 1 before tableSplitCycle, phase 2 after)
    gives the forward mode's words: the lookup-table reads of phase 2 see every count"""
    t = T.random_trace(14, 2000, seed=11)
    data, glob, cyc, tx = W.inputs(t)
    a = W.run(data, glob, cyc, tx, t.table_split_cycle, 1 << 14, W.MODE_SEQ_FORWARD)
    b = W.run(data, glob, cyc, tx, t.table_split_cycle, 1 << 14, W.MODE_PARALLEL)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def _fails_both(data, glob, cyc, tx, split, rows, match):
    with pytest.raises(RuntimeError, match=match):
        W.run(data, glob, cyc, tx, split, rows)
    with pytest.raises(I.WitgenError, match=match):
        I.witgen(data.copy(), glob.copy(), cyc.copy(), tx, rows)


@needs_ref
def test_failures_match_reference():
    t = T.random_trace(13, 400, seed=4)
    data, glob, cyc, tx = W.inputs(t)
    rows = 1 << 13
    # a transaction at another address than the step reads (ffi.cpp:101-104)
    bad = tx.copy()
    k = int(cyc["txnIdx"][400])
    bad["addr"][k] ^= 4
    _fails_both(data, glob, cyc, bad, t.table_split_cycle, rows, "memory peek not in preflight")
    # a decode row whose major/minor disagree with the instruction word: an EQZ fails
    c2 = cyc.copy()
    row = next(r for r in range(rows) if c2["state"][r] == T.DECODE and c2["major"][r] == 0 and c2["minor"][r] == 0)
    c2["minor"][row] = 1
    _fails_both(data, glob, c2, tx, t.table_split_cycle, rows, "eqz failure")
    # an injected next-pc that disagrees with the step: the checked re-store refuses it
    d2 = data.copy()
    lay = W.layout()
    d2[lay["next_pc_low"] * rows + 500] = W.encode(12345)
    _fails_both(d2, glob, cyc, tx, t.table_split_cycle, rows, "Inconsistent set")


@needs_ref
def test_trace_seal_verifies_with_validity(oracle):
    """prove_core from a restated preflight on the CPU (the compiled reference witgen and
    accumulation around the oracle prover): the rows satisfy every rv32im constraint, so the
    seal passes the native verifier WITH the validity equation (verify/mod.rs:340-394); one
    flipped data word after witgen makes it fail there"""
    import risc0_amd as r
    t = T.random_trace(13, 250, seed=21)
    seal, mix, d, g, acc = W.prove_from_trace(t, oracle.POSEIDON2, oracle)
    assert r.verify_seal("rv32im", r.POSEIDON2, seal, check_validity=True) == 13
    # a terminating segment with machine-mode ecalls (BigInt included) is valid too
    te = T.ecall_trace(14, seed=4, terminate=True, bigint=True)
    seal_e, _, _, _, _ = W.prove_from_trace(te, oracle.POSEIDON2, oracle)
    assert r.verify_seal("rv32im", r.POSEIDON2, seal_e, check_validity=True) == 14
    rows = 1 << 13
    d2 = d.copy()
    row = int(np.flatnonzero(t.arrays()[0]["state"] == T.DECODE)[0])
    d2[W.layout()["cycle"] * rows + row] = W.encode(row + 1)  # the cycle counter of a user row
    code = np.zeros(rows, np.uint32)
    bad, _, _ = oracle.prove_segment("rv32im", oracle.POSEIDON2, 13, code, d2, acc, g, version=2)
    with pytest.raises(r.R0HipError):
        r.verify_seal("rv32im", r.POSEIDON2, bad, check_validity=True)
    assert r.verify_seal("rv32im", r.POSEIDON2, bad, check_validity=False) == 13


def test_trace_poseidon2_constants_match_oracle():
    """the restated preflight decodes its Poseidon2 constants from the product's Montgomery
    table (so the bench's input generator reads nothing under oracle/); they equal the oracle's
    plain-integer table (poseidon2/consts.rs:51-184) wherever the rounds use them"""
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    text = open(os.path.join(root, "oracle", "poseidon2_consts.inc")).read()
    tabs = {m.group(1): [int(x, 16) for x in re.findall(r"0x[0-9a-fA-F]+", m.group(2))]
            for m in re.finditer(r"static const uint32_t (\w+)\[[^\]]*\] = \{(.*?)\};", text, re.S)}
    rc, diag = tabs["ROUND_CONSTANTS_INT"], tabs["M_INT_DIAG_HZN_INT"]
    for r in list(range(4)) + list(range(25, 29)):
        assert T.RC[r * 24:(r + 1) * 24] == rc[r * 24:(r + 1) * 24]
    assert [T.RC[(4 + i) * 24] for i in range(21)] == [rc[(4 + i) * 24] for i in range(21)]
    assert T.M_INT_DIAG == diag


def test_loop_s_bulk_iterations_match_stepped():
    """the benchmark guest (loop.s under the v1compat kernel): its addi/bltu iterations
    written as numpy blocks (Trace._bulk_loop) give the trace, injector and global vector of
    stepping every instruction, for loops shorter and longer than the affine check's window"""
    for n in (1, 4, 7, 600):
        a, b = T.loop_s_trace(14, n, fast=False), T.loop_s_trace(14, n)
        assert a.terminated and b.terminated
        for x, y in zip(a.arrays() + a.injector_arrays(), b.arrays() + b.injector_arrays()):
            assert np.array_equal(x, y)
        assert np.array_equal(a.global_words(), b.global_words())
        # the halt copied loop.s's null digest to GLOBAL_OUTPUT_ADDR; a4 counted to `count`
        assert [b.mem[T.GLOBAL_OUTPUT_WADDR + i] for i in range(8)] == T.NULL_DIGEST
        assert b.mem[T.USER_REGS_WADDR + T.REG_A4] == n


def test_loop_s_datasheet_segments_fit():
    """datasheet.rs:42-58: CYCLES_PO2_ITERS fills a segment of its po2 (here 16; po2 20 with
    ITERATIONS_FULL_PO2_20_SEGMENT is covered by the bench and the GPU tests)"""
    t = T.loop_s_trace(16)
    cyc, tx = t.arrays()
    assert len(cyc) == 1 << 16 and t.terminated
    user = int(np.sum((cyc["state"] == T.DECODE)[:t.table_split_cycle]))
    assert user >= 2 * T.loop_s_iterations(16)
    assert T.loop_s_iterations(20) == 1024 * 494 + 817 and T.loop_s_iterations(24) == 1024 * 256 * 31


@needs_ref
def test_loop_s_guest_proves_and_verifies_on_cpu(oracle):
    """BASELINE configs[0]: the benchmarks' loop guest, one po2=16 segment (16 K iterations,
    datasheet.rs:44) proved on the CPU path — the compiled reference witgen and accumulation
    around the oracle prover — and the receipt's seal passes the native verifier with the
    validity equation, as the datasheet's prove + verify does (datasheet.rs:245-262)"""
    import risc0_amd as r
    t = T.loop_s_trace(16, seed=16)
    seal, mix, d, g, acc = W.prove_from_trace(t, oracle.POSEIDON2, oracle)
    assert r.verify_seal("rv32im", r.POSEIDON2, seal, check_validity=True) == 16
    assert g[W.layout()["global"]["is_terminate"]] == W.encode(1)
