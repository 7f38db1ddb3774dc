"""rv32im witness generation on the GPU (r0hip_rv32im_witgen, generated from the reference's
step_Top) against the reference's compiled risc0_circuit_rv32im_cpu_witgen
(rv32im-sys/kernels/cxx/ffi.cpp:267-308, forward mode) on traces of the restated preflight
(tests/rv32im_trace.py): the data and global groups word for word, INVALID words included,
and the same failures."""
import numpy as np
import pytest

import rv32im_trace as T
import rv32im_witgen_ref as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hal():
    import risc0_amd as r
    return r.HipHal("poseidon2")


def gpu_witgen(hal, data, glob, cyc, tx, split, mode=0, bigint=None):
    import risc0_amd as r
    dd = hal.copy_from_elem("data", data)
    dg = hal.copy_from_elem("global", glob)
    r.rv32im_witgen(dd, dg, cyc, tx, split, bigint=bigint, mode=mode)
    return dd.to_numpy(), dg.to_numpy()


@pytest.mark.parametrize("po2,n,seed", [(13, 1, 1), (13, 300, 2), (14, 2500, 3), (16, 12000, 4), (20, 60000, 5)])
def test_rv32im_witgen_matches_reference(hal, po2, n, seed):
    t = T.random_trace(po2, n, seed=seed) if n > 1 else T.Trace(po2, [T.asm("addi", 1, 0, 5)])
    data, glob, cyc, tx = W.inputs(t)
    ref_d, ref_g = W.run(data, glob, cyc, tx, t.table_split_cycle, 1 << po2)
    d, g = gpu_witgen(hal, data, glob, cyc, tx, t.table_split_cycle)
    bad = np.flatnonzero(d != ref_d)
    assert bad.size == 0, f"{bad.size} words differ; first (col, row): {[(int(i) >> po2, int(i) & ((1 << po2) - 1)) for i in bad[:8]]}"
    assert np.array_equal(g, ref_g)
    assert (d == W.INVALID).any()  # columns no arm of a row writes stay INVALID, as in the reference


@pytest.mark.parametrize("terminate,bigint", [(True, True), (False, False)])
def test_rv32im_witgen_ecalls_match_reference(hal, terminate, bigint):
    """machine-mode rows: user ecall, Poseidon2 ecalls (state / no state, bytes / elements),
    host write, unaligned host read, SHA-256, mret, terminate, and a BigInt ecall (arm 12:
    every PolyOp and MemoryOp, the witness bytes from the trace's bigint array)"""
    import risc0_amd as r
    t = T.ecall_trace(14, seed=3, terminate=terminate, bigint=bigint)
    data, glob, cyc, tx = W.inputs(t)
    bi = t.bigint_array()
    assert (12 in set(cyc["major"][:t.table_split_cycle].tolist())) == bigint
    ref_d, ref_g = W.run(data, glob, cyc, tx, t.table_split_cycle, 1 << 14, bigint=bi)
    d, g = gpu_witgen(hal, data, glob, cyc, tx, t.table_split_cycle, bigint=bi)
    assert np.array_equal(d, ref_d) and np.array_equal(g, ref_g)
    if bigint:  # cut inside the bytes of the call's first Write row (its 4th cycle): refused, not read past
        with pytest.raises(r.R0HipError, match="bigint bytes past"):
            gpu_witgen(hal, data, glob, cyc, tx, t.table_split_cycle, bigint=bi[:56])


def test_rv32im_witgen_ecall_heavy_matches_reference(hal, oracle):
    """30 passes of the machine-mode ecalls (Poseidon2, SHA-256, BigInt, host I/O) at po2=16:
    the ecall arms fill many wavefronts per bin (SHA-256 4230 rows, Poseidon2 5881, BigInt
    540), across the minor-ordered bins and their stored-slot masks. Data and global groups
    equal the reference's; the proof from the trace equals the CPU path's and is valid."""
    import risc0_amd as r
    t = T.ecall_trace(16, seed=5, bigint=True, reps=30)
    data, glob, cyc, tx = W.inputs(t)
    bi = t.bigint_array()
    ref_d, ref_g = W.run(data, glob, cyc, tx, t.table_split_cycle, 1 << 16, W.MODE_PARALLEL, bigint=bi)
    d, g = gpu_witgen(hal, data, glob, cyc, tx, t.table_split_cycle, bigint=bi)
    bad = np.flatnonzero(d != ref_d)
    assert bad.size == 0, f"{bad.size} words differ; first (col, row): {[(int(i) >> 16, int(i) & 0xFFFF) for i in bad[:8]]}"
    assert np.array_equal(g, ref_g)
    ref_seal, ref_mix, _, _, _ = W.prove_from_trace(t, oracle.POSEIDON2, oracle)
    idx, off, val = W.injector_arrays(t)
    seal, mix = r.prove_segment_trace(hal, 16, W.global_words(t), idx, off, val, cyc, tx, t.table_split_cycle,
                                      bigint=bi, bigint_records=t.bigint_records())
    assert np.array_equal(mix, ref_mix) and np.array_equal(seal, ref_seal)
    assert r.verify_seal("rv32im", hal.suite, seal, check_validity=True) == 16


def test_rv32im_witgen_modes(hal):
    """every mode runs the same schedule and gives the reference's forward-mode words"""
    t = T.random_trace(13, 500, seed=9)
    data, glob, cyc, tx = W.inputs(t)
    ref = W.run(data, glob, cyc, tx, t.table_split_cycle, 1 << 13)
    for mode in (0, 1, 2):
        d, g = gpu_witgen(hal, data, glob, cyc, tx, t.table_split_cycle, mode)
        assert np.array_equal(d, ref[0]) and np.array_equal(g, ref[1])


def test_rv32im_witgen_failures(hal):
    """the reference's throws are errors here too, and a failed call leaves the next one clean"""
    import risc0_amd as r
    t = T.random_trace(13, 400, seed=4)
    data, glob, cyc, tx = W.inputs(t)
    rows = 1 << 13
    bad = tx.copy()
    bad["addr"][int(cyc["txnIdx"][400])] ^= 4
    with pytest.raises(r.R0HipError, match="memory peek not in preflight"):
        gpu_witgen(hal, data, glob, cyc, bad, t.table_split_cycle)
    c2 = cyc.copy()
    row = next(i for i in range(rows) if c2["state"][i] == T.DECODE and c2["major"][i] == 0 and c2["minor"][i] == 0)
    c2["minor"][row] = 1
    with pytest.raises(r.R0HipError, match="eqz failure"):
        gpu_witgen(hal, data, glob, c2, tx, t.table_split_cycle)
    d2 = data.copy()
    d2[W.layout()["next_pc_low"] * rows + 500] = W.encode(12345)
    with pytest.raises(r.R0HipError, match="Inconsistent set"):
        gpu_witgen(hal, d2, glob, cyc, tx, t.table_split_cycle)
    c3 = cyc.copy()
    c3["major"][77] = 13
    with pytest.raises(r.R0HipError, match="selects no instruction arm"):
        gpu_witgen(hal, data, glob, c3, tx, t.table_split_cycle)
    ref = W.run(data, glob, cyc, tx, t.table_split_cycle, rows)
    d, g = gpu_witgen(hal, data, glob, cyc, tx, t.table_split_cycle)
    assert np.array_equal(d, ref[0]) and np.array_equal(g, ref[1])


@pytest.mark.parametrize("trace", ["random", "ecalls"])
def test_rv32im_witgen_first_failure_matches_reference(hal, trace):
    """one row of every instruction arm with its minor moved to the next one: the call fails
    with the reference's message for its first failed check, word for word for an EQZ (its
    zirgen source location and the cycle), in each arm kernel: the checks kept in program
    order (arms 4 and 11) and the rest, and the arms that reload injected cells (10, 11)"""
    import risc0_amd as r
    t = T.random_trace(13, 400, seed=4) if trace == "random" else T.ecall_trace(14, seed=3, bigint=True)
    data, glob, cyc, tx = W.inputs(t)
    rows = 1 << (13 if trace == "random" else 14)
    bi = t.bigint_array()
    arms = 0
    for arm in range(13):
        cand = [i for i in range(t.table_split_cycle) if cyc["major"][i] == arm]
        if not cand:
            continue
        row = cand[len(cand) // 2]
        c2 = cyc.copy()
        c2["minor"][row] = (int(c2["minor"][row]) + 1) % 8
        with pytest.raises(RuntimeError) as ref:
            W.run(data, glob, c2, tx, t.table_split_cycle, rows, bigint=bi)
        with pytest.raises(r.R0HipError) as got:
            gpu_witgen(hal, data, glob, c2, tx, t.table_split_cycle, bigint=bi)
        want = str(ref.value)
        if "eqz failure" in want:
            assert want in str(got.value), (arm, want, str(got.value))
        else:
            assert want.split(":")[0] in str(got.value), (arm, want, str(got.value))
        arms += 1
    assert arms == (10 if trace == "random" else 13)


@pytest.mark.parametrize("po2,n,suite,seed", [(13, 250, "poseidon2", 21), (14, 2500, "poseidon2", 3),
                                              (14, 2000, "sha-256", 8), (14, 0, "poseidon2", 4)])
def test_prove_segment_trace_matches_oracle(po2, n, suite, seed, oracle):
    """r0hip_prove_segment_trace (injector scatter, stepExec, zeroize, accumulation and the
    prove core on the device, rv32im prove/hal/mod.rs:143-224) gives the seal and mix of the
    CPU path: the compiled reference witgen and accumulation around the oracle prover. The
    rows satisfy the circuit, so the seal verifies with the validity equation."""
    import risc0_amd as r
    h = r.HipHal(suite)
    # n = 0: the ecall trace, with a BigInt ecall whose accumulator states the prover injects
    t = T.random_trace(po2, n, seed=seed) if n else T.ecall_trace(po2, seed=seed, bigint=True)
    s = {"poseidon2": oracle.POSEIDON2, "sha-256": oracle.SHA256}[suite]
    ref_seal, ref_mix, _, _, _ = W.prove_from_trace(t, s, oracle)
    cyc, tx = t.arrays()
    idx, off, val = W.injector_arrays(t)
    seal, mix = r.prove_segment_trace(h, po2, W.global_words(t), idx, off, val, cyc, tx, t.table_split_cycle,
                                      bigint=t.bigint_array(), bigint_records=t.bigint_records())
    assert np.array_equal(mix, ref_mix)
    assert seal.size == ref_seal.size and np.array_equal(seal, ref_seal)
    assert r.verify_seal("rv32im", h.suite, seal, check_validity=True) == po2


def test_prove_segment_trace_full_size_verifies(hal):
    """BASELINE configs[1] shape from a trace: a po2=20 segment of a random program proved from
    its preflight on the device; its seal passes the native verifier with the validity
    equation (the CPU path would take minutes at this size)"""
    import risc0_amd as r
    t = T.random_trace(20, 60000, seed=5)
    cyc, tx = t.arrays()
    idx, off, val = W.injector_arrays(t)
    seal, mix = r.prove_segment_trace(hal, 20, W.global_words(t), idx, off, val, cyc, tx, t.table_split_cycle)
    assert r.verify_seal("rv32im", hal.suite, seal, check_validity=True) == 20


def test_prove_segment_trace_resident_matches_host_path(hal):
    """the benchmark's form (global vector, injector and preflight already in device memory,
    r0hip_prove_segment_trace_resident) proves the same seal as the host-pointer ABI, also with
    two segments in flight on their own threads"""
    import threading
    import risc0_amd as r
    t = T.loop_trace(14, body_len=24, seed=13)
    cyc, tx = t.arrays()
    idx, off, val = W.injector_arrays(t)
    g = W.global_words(t)
    seal, mix = r.prove_segment_trace(hal, 14, g, idx, off, val, cyc, tx, t.table_split_cycle)
    rt = r.ResidentTrace(hal, 14, g, idx, off, val, cyc, tx, t.table_split_cycle)
    out = [None, None]

    def run(i):
        out[i] = r.prove_segment_trace_resident(hal, rt)
    ts = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for x in ts:
        x.start()
    for x in ts:
        x.join()
    for s2, m2 in out:
        assert np.array_equal(s2, seal) and np.array_equal(m2, mix)
    assert r.verify_seal("rv32im", hal.suite, seal, check_validity=True) == 14
    # with BigInt bytes resident too
    te = T.ecall_trace(14, seed=6, bigint=True)
    cyc, tx = te.arrays()
    idx, off, val = W.injector_arrays(te)
    args = (W.global_words(te), idx, off, val, cyc, tx, te.table_split_cycle)
    seal, mix = r.prove_segment_trace(hal, 14, *args, bigint=te.bigint_array(), bigint_records=te.bigint_records())
    rt = r.ResidentTrace(hal, 14, *args, bigint=te.bigint_array())
    s2, m2 = r.prove_segment_trace_resident(hal, rt, bigint_records=te.bigint_records())
    assert np.array_equal(s2, seal) and np.array_equal(m2, mix)
    assert r.verify_seal("rv32im", hal.suite, seal, check_validity=True) == 14


def _trace_job(r, t, pinned=False):
    cyc, tx = t.arrays()
    idx, off, val = W.injector_arrays(t)
    arrs = [W.global_words(t), idx, off, val, cyc, tx]
    if pinned:
        arrs = [r.pinned_copy(a) for a in arrs]
    return r.TraceJob(*arrs, t.table_split_cycle, bigint=t.bigint_array(), bigint_records=t.bigint_records())


def test_prove_segments_trace_jobs_match_single(hal):
    """the segment pipeline's trace jobs (r0hip_prove_trace_segments: an uploader stages each
    preflight trace into one of in_flight + 1 device trace sets while the provers run, as r0vm's
    GPU queue does): six distinct po2=14 segments — loop guests of different lengths, a random
    loop body, a BigInt ecall trace; page-locked and pageable inputs — over 2 provers and 3 sets
    give the seals and mixes of r0hip_prove_segment_trace, job by job"""
    import risc0_amd as r
    traces = [T.loop_s_trace(14, 300 + 97 * i, seed=40 + i) for i in range(3)] + \
        [T.loop_trace(14, body_len=24, seed=13), T.ecall_trace(14, seed=6, bigint=True), T.loop_s_trace(14, 5, seed=9)]
    jobs = [_trace_job(r, t, pinned=i % 2 == 1) for i, t in enumerate(traces)]
    got = r.prove_trace_segments(hal, 14, jobs, in_flight=2)
    for t, j, (seal, mix) in zip(traces, jobs, got):
        ref_seal, ref_mix = r.prove_segment_trace(hal, 14, j.glob, j.index, j.offsets, j.values, j.cycles, j.txns,
                                                  t.table_split_cycle, bigint=t.bigint_array(),
                                                  bigint_records=t.bigint_records())
        assert np.array_equal(seal, ref_seal) and np.array_equal(mix, ref_mix)
        assert r.verify_seal("rv32im", hal.suite, seal, check_validity=True) == 14
    assert len({s.tobytes() for s, _ in got}) == len(traces)
    # one in-flight prover, more jobs than sets: the same seals
    again = r.prove_trace_segments(hal, 14, jobs[:4], in_flight=1)
    assert all(np.array_equal(a[0], b[0]) for a, b in zip(again, got[:4]))


def test_prove_segments_trace_job_errors(hal):
    """a trace job whose injector index decreases fails with the host check's message (the other
    jobs still prove), and the next call is clean"""
    import risc0_amd as r
    t = T.loop_s_trace(14, 100, seed=3)
    good = _trace_job(r, t)
    bad = _trace_job(r, t)
    bad.index[1001] = bad.index[1000] - 1
    with pytest.raises(r.R0HipError, match="segment 1: .*injector index decreases"):
        r.prove_trace_segments(hal, 14, [good, bad, good], in_flight=2)
    (seal, mix), = r.prove_trace_segments(hal, 14, [good])
    ref = r.prove_segment_trace(hal, 14, good.glob, good.index, good.offsets, good.values, good.cycles, good.txns,
                                t.table_split_cycle)
    assert np.array_equal(seal, ref[0])


def test_prove_trace_segments_verification_fails_the_job(hal, monkeypatch):
    """r0hip_prove_trace_segments checks every seal with the native verifier (validity equation
    included) on a host thread beside the proofs, as ProverImpl::prove_segment_core verifies a
    receipt before it returns it (prover_impl.rs:262-280): every job of a clean call is verified;
    a job whose seal fails the check (a bit flipped in its first Merkle root by the testing hook
    R0HIP_TESTING_CORRUPT_SEAL_JOB) reports "receipt verification failed" and the other jobs still
    return their verified seals"""
    import risc0_amd as r
    traces = [T.loop_s_trace(14, 150 + 31 * i, seed=70 + i) for i in range(4)]
    jobs = [_trace_job(r, t) for t in traces]
    clean = r.prove_trace_segments(hal, 14, jobs, in_flight=2, per_job=True)
    assert all(e is None and ms > 0 and pms > 0 for _, _, e, ms, pms in clean)
    monkeypatch.setenv("R0HIP_TESTING_CORRUPT_SEAL_JOB", "2")
    got = r.prove_trace_segments(hal, 14, jobs, in_flight=2, per_job=True)
    monkeypatch.delenv("R0HIP_TESTING_CORRUPT_SEAL_JOB")
    for i, ((seal, mix, err, _, _), (cseal, cmix, _, _, _)) in enumerate(zip(got, clean)):
        if i == 2:
            assert err and "receipt verification failed" in err, err
            assert not np.array_equal(seal, cseal)
        else:
            assert err is None and np.array_equal(seal, cseal) and np.array_equal(mix, cmix)
    with pytest.raises(r.R0HipError, match="segment 2: receipt verification failed"):
        monkeypatch.setenv("R0HIP_TESTING_CORRUPT_SEAL_JOB", "2")
        try:
            r.prove_trace_segments(hal, 14, jobs, in_flight=2)
        finally:
            monkeypatch.delenv("R0HIP_TESTING_CORRUPT_SEAL_JOB")
    # without the check the flipped seal is returned as proved (what verify=1 guards against)
    monkeypatch.setenv("R0HIP_TESTING_CORRUPT_SEAL_JOB", "2")
    unchecked = r.prove_trace_segments(hal, 14, jobs, in_flight=2, verify=False)
    monkeypatch.delenv("R0HIP_TESTING_CORRUPT_SEAL_JOB")
    with pytest.raises(r.R0HipError):
        r.verify_seal("rv32im", hal.suite, unchecked[2][0], check_validity=True)


def test_prove_segment_trace_pinned_inputs_match_pageable(hal):
    """r0hip_prove_segment_trace copies host arrays of 64 KiB or more that lie in r0hip_host_alloc
    blocks straight to the device (no staging): the cycles, transactions and injector arrays in
    page-locked memory give the seal and mix of the same arrays in pageable memory"""
    import risc0_amd as r
    t = T.loop_s_trace(16, seed=77)
    cyc, tx = t.arrays()
    idx, off, val = W.injector_arrays(t)
    assert min(a.nbytes for a in (cyc, tx, idx, off, val)) >= 64 << 10
    g = W.global_words(t)
    ref = r.prove_segment_trace(hal, 16, g, idx, off, val, cyc, tx, t.table_split_cycle)
    pin = [r.pinned_copy(a) for a in (idx, off, val, cyc, tx)]
    got = r.prove_segment_trace(hal, 16, g, *pin[:3], pin[3], pin[4], t.table_split_cycle)
    assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1])


def test_loop_s_guest_seal_matches_cpu_path(hal, oracle):
    """BASELINE configs[0] on the device: the datasheet's loop guest (loop.s under the v1compat
    kernel, 16 K iterations at po2=16) from its preflight trace gives the CPU path's seal and mix
    (compiled reference witgen + accumulation around the oracle prover), and it is valid"""
    import risc0_amd as r
    t = T.loop_s_trace(16, seed=16)
    ref_seal, ref_mix, _, _, _ = W.prove_from_trace(t, oracle.POSEIDON2, oracle)
    cyc, tx = t.arrays()
    idx, off, val = W.injector_arrays(t)
    seal, mix = r.prove_segment_trace(hal, 16, W.global_words(t), idx, off, val, cyc, tx, t.table_split_cycle)
    assert np.array_equal(mix, ref_mix) and np.array_equal(seal, ref_seal)
    assert r.verify_seal("rv32im", hal.suite, seal, check_validity=True) == 16


def test_loop_s_witgen_po2_22_matches_reference(hal):
    """po2=22 (the datasheet's 1,835,008 iterations, 14.7 M memory transactions): the GPU
    witness generation equals the compiled reference's word for word"""
    import risc0_amd as r
    t = T.loop_s_trace(22, seed=22)
    data, glob, cyc, tx = W.inputs(t)
    ref_d, ref_g = W.run(data, glob, cyc, tx, t.table_split_cycle, 1 << 22, W.MODE_PARALLEL)
    d, g = gpu_witgen(hal, data, glob, cyc, tx, t.table_split_cycle)
    del data
    bad = np.flatnonzero(d != ref_d)
    assert bad.size == 0, f"{bad.size} words differ; first (col, row): {[(int(i) >> 22, int(i) & ((1 << 22) - 1)) for i in bad[:8]]}"
    assert np.array_equal(g, ref_g)
    r.trim()


def test_loop_s_trace_po2_24_proves_and_verifies(hal):
    """BASELINE configs[2] from a trace: the maximum segment (po2=24, the datasheet's 8,126,464
    loop iterations, 16.25 M user cycles, 211 x 2^24 data words) proved from its preflight —
    witness generation, accumulation, prove — passes the native verifier with the validity
    equation"""
    import risc0_amd as r
    r.trim()
    t = T.loop_s_trace(24, seed=24)
    job = _trace_job(r, t)
    del t
    (seal, _mix), = r.prove_trace_segments(hal, 24, [job], in_flight=1)
    del job
    assert r.verify_seal("rv32im", hal.suite, seal, check_validity=True) == 24
    r.trim()


def _with_entry(idx, off, val, row, offset, word):
    """the injector with one more entry at the end of `row` (Injector::set order)"""
    at = int(idx[row + 1])
    idx2 = idx.copy()
    idx2[row + 1:] += 1
    return idx2, np.insert(off, at, offset), np.insert(val, at, word)


def test_injector_words_outside_the_arms_columns_match_reference(hal, oracle):
    """a word set before the arms run in a column the row's arm does not take from the
    injector is treated as the reference's Buffer::set treats it (buffers.h:30-42): kept when the
    arm does not store the column, accepted when the arm stores the same value, "Inconsistent set"
    when it stores another. The public witgen's data group equals the compiled reference's word for
    word; the prover (an injector entry there) equals the CPU path's seal; the next call is clean."""
    import risc0_amd as r
    po2, rows = 14, 1 << 14
    t = T.loop_s_trace(po2, 200, seed=5)
    cyc, tx = t.arrays()
    lay = W.layout()
    data, glob, _, _ = W.inputs(t)
    ref_d, ref_g = W.run(data, glob, cyc, tx, t.table_split_cycle, rows)
    row = int(np.flatnonzero((cyc["state"] == T.DECODE) & (cyc["major"] == 0))[5])
    keep_col = lay["sha2_u32"][0]  # the arm neither reads nor writes it: a set word is kept
    assert ref_d[keep_col * rows + row] == W.INVALID
    # a column the row's arm writes that the injector left INVALID
    stored = [c for c in range(W.DATA_COLS) if data[c * rows + row] == W.INVALID and ref_d[c * rows + row] != W.INVALID]
    same_col = stored[len(stored) // 2]
    same = int(ref_d[same_col * rows + row])
    other = (same + 1) % T.P  # another canonical word
    for col, word, fails in ((keep_col, W.encode(1), False), (same_col, same, False), (same_col, other, True)):
        d2 = data.copy()
        d2[col * rows + row] = word
        if fails:
            with pytest.raises(RuntimeError, match="Inconsistent set"):
                W.run(d2, glob, cyc, tx, t.table_split_cycle, rows)
            with pytest.raises(r.R0HipError, match="Inconsistent set"):
                gpu_witgen(hal, d2, glob, cyc, tx, t.table_split_cycle)
        else:
            rd, rg = W.run(d2, glob, cyc, tx, t.table_split_cycle, rows)
            gd, gg = gpu_witgen(hal, d2, glob, cyc, tx, t.table_split_cycle)
            assert np.array_equal(gd, rd) and np.array_equal(gg, rg), (col, int((gd != rd).sum()))
    idx, off, val = W.injector_arrays(t)
    # the prover: an injector entry in a column the arm does not take (kept, then zeroized-in)
    patch = [(keep_col * rows + row, int(W.encode(1)))]
    ref_seal, ref_mix, _, _, _ = W.prove_from_trace(t, oracle.POSEIDON2, oracle, data_patch=patch)
    idx2, off2, val2 = _with_entry(idx, off, val, row, *patch[0])
    seal, mix = r.prove_segment_trace(hal, po2, W.global_words(t), idx2, off2, val2, cyc, tx, t.table_split_cycle)
    assert np.array_equal(mix, ref_mix) and np.array_equal(seal, ref_seal)
    # an entry of another row is refused on the host (Injector::set writes its own row)
    idx3, off3, val3 = _with_entry(idx, off, val, row, keep_col * rows + row + 1, int(W.encode(1)))
    with pytest.raises(r.R0HipError, match="of another row"):
        r.prove_segment_trace(hal, po2, W.global_words(t), idx3, off3, val3, cyc, tx, t.table_split_cycle)
    seal, _ = r.prove_segment_trace(hal, po2, W.global_words(t), idx, off, val, cyc, tx, t.table_split_cycle)
    assert r.verify_seal("rv32im", hal.suite, seal, check_validity=True) == po2


def test_loop_s_session_segments_match_reference_and_verify(hal):
    """configs[3]'s input: ONE loop.s session cut into consecutive po2=20
    segments where the executor cuts it (rv32im_trace.LoopSession): each segment after the first
    resumes mid-loop from the previous one's final memory with its pages loaded, and its pre-state
    root is the previous post-state root. Segments 0, 1 and the last: the GPU witness equals the
    compiled reference witgen's word for word, and the three seals (one r0hip_prove_trace_segments
    call, receipts checked) pass r0hip_verify_seal with the validity equation."""
    import risc0_amd as r
    po2, K = 20, 3
    S = T.LoopSession(po2, T.loop_s_session_iterations(po2, K), seed=11)
    traces = list(S)
    assert len(traces) == K and traces[-1].terminated and not traces[0].terminated
    for a, b in zip(traces, traces[1:]):
        assert b.root == a.post_root
    for t in traces:
        data, glob, cyc, tx = W.inputs(t)
        ref_d, ref_g = W.run(data, glob, cyc, tx, t.table_split_cycle, 1 << po2, W.MODE_PARALLEL)
        d, g = gpu_witgen(hal, data, glob, cyc, tx, t.table_split_cycle)
        assert np.array_equal(d, ref_d) and np.array_equal(g, ref_g)
    got = r.prove_trace_segments(hal, po2, [_trace_job(r, t) for t in traces], in_flight=2)
    assert len({s.tobytes() for s, _ in got}) == K
    for seal, _ in got:
        assert r.verify_seal("rv32im", hal.suite, seal, check_validity=True) == po2

