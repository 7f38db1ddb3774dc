"""The drop-in per-op path at the BASELINE sizes: the reference prover
driven through ONLY the per-op r0hip_* symbols — natively (integration/hal_prover.cpp,
libr0hip_halprover.so, what a Rust HipHal behind risc0_zkp::hal::Hal would call) and from
Python (tests/hal_prover.py over risc0_amd.HipHal) — against the fused prover on the same
inputs: rv32im prove_core from a loop-guest trace at po2 16 and 20 (Poseidon2; the fused seal
at po2 20 is pinned to the CPU path by the bench's cpu_baseline), and a recursion program at
po2 18 with SHA-256. Seals and mixes must be identical."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

import rv32im_trace as T
import rv32im_witgen_ref as W

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "integration"))


def _trace_job(r, t):
    cyc, tx = t.arrays()
    idx, off, val = t.injector_arrays()
    return r.TraceJob(t.global_words(), idx, off, val, cyc, tx, t.table_split_cycle, bigint=t.bigint_array(),
                      bigint_records=t.bigint_records())


def test_driver_imports_only_per_op_symbols():
    """the native driver binds the per-op Hal symbols and nothing fused (no r0hip_prove_*)"""
    import subprocess
    import halprover
    out = subprocess.check_output(["nm", "-D", "--undefined-only", halprover.LIB_PATH], text=True)
    used = {ln.split()[-1] for ln in out.splitlines() if "r0hip_" in ln}
    assert "r0hip_eval_check" in used and "r0hip_hash_fold" in used
    assert not any(u.startswith("r0hip_prove") for u in used), used


@pytest.mark.parametrize("po2", [16, 20])
def test_per_op_path_rv32im_matches_fused(oracle, po2):
    """rv32im prove_core from the loop guest's preflight trace: the per-op path (the injector
    scatter, r0hip_rv32im_witgen, zeroize, the prover with r0hip_rv32im_accum between the mix
    draw and the accum commit) gives the fused r0hip_prove_segment_trace's seal and mix, natively
    and from Python"""
    import halprover
    import hal_prover
    import risc0_amd as r
    hal = r.HipHal("poseidon2")
    t = T.loop_s_trace(po2, T.loop_s_iterations(po2) - 11, seed=900 + po2)
    job = _trace_job(r, t)
    fused_seal, fused_mix = r.prove_segment_trace(hal, po2, job.glob, job.index, job.offsets, job.values, job.cycles,
                                                  job.txns, t.table_split_cycle, bigint=t.bigint_array(),
                                                  bigint_records=t.bigint_records())
    seal, mix = halprover.prove_trace(hal, po2, job)
    assert np.array_equal(mix, fused_mix) and np.array_equal(seal, fused_seal)
    # the same sequence from Python over HipHal, from the per-op witness generation
    n = 1 << po2
    data = hal.alloc_elem_init("data", 211 * n, 0xFFFFFFFF)
    glob = hal.copy_from_elem("global", job.glob)
    hal.scatter(data, job.index, job.offsets, job.values)
    r.rv32im_witgen(data, glob, job.cycles, job.txns, t.table_split_cycle, bigint=t.bigint_array())
    hal.eltwise_zeroize_elem(data)
    hal.eltwise_zeroize_elem(glob)
    code = hal.alloc_elem_init("code", n, 0)
    accum = hal.alloc_elem("accum", 103 * n)

    def accumulate(mix_buf, mix_words):  # WitnessGenerator::accum (witgen/mod.rs:178-221)
        r.check(r.lib().r0hip_memset32(accum.ptr, 0xFFFFFFFF, accum.size))
        r.bigint_accum_inject(accum, n, mix_words, t.bigint_records())
        r.check(r.lib().r0hip_rv32im_accum(data.ptr, accum.ptr, glob.ptr, mix_buf.ptr, n, 103, n))
        hal.eltwise_zeroize_elem(accum)
    pseal, pmix = hal_prover.prove_segment(oracle, hal, "rv32im", po2, code, data, accum, glob, accumulate=accumulate)
    assert np.array_equal(pmix, fused_mix) and np.array_equal(pseal, fused_seal)
    assert r.verify_seal("rv32im", hal.suite, seal, check_validity=True) == po2


def test_per_op_path_recursion_sha256_matches_fused(oracle):
    """a recursion program at po2 18 with SHA-256 (configs[4]'s suite): the per-op path
    (r0hip_recursion_witgen, the ZK noise by r0hip_fill_uniform + r0hip_eltwise_copy_elem_slice,
    zeroize, the prover with r0hip_recursion_accum) gives r0hip_prove_recursion's seal and mix,
    natively and from Python"""
    import halprover
    import hal_prover
    import recursion_program as RP
    import risc0_amd as r
    if not RP.available():
        pytest.skip("oracle/_ref not built")
    hal = r.HipHal("sha-256")
    po2 = 18
    n, zk = 1 << po2, RP.ZK_CYCLES
    rng = np.random.default_rng(4242)
    prog, inp = RP.random_program(rng, n - zk - 1)
    pf = RP.preflight(prog, inp)
    wom, cyc, iops = RP.trace_arrays(pf)
    ctrl = hal.copy_from_elem("ctrl", RP.ctrl_group(prog, po2))
    seed = 0x5EED18
    fused_seal, fused_mix = r.prove_recursion(hal, po2, ctrl, wom, cyc, iops, seed)
    lib = r.lib()

    def witness():  # WitnessGenerator::new (circuit/recursion/src/prove/witgen.rs:44-133), per op
        data = hal.alloc_elem_init("data", RP.DATA * n, 0xFFFFFFFF)
        glob = hal.alloc_elem_init("global", RP.OUT, 0xFFFFFFFF)
        r.recursion_witgen(ctrl, data, glob, n, wom, cyc, iops)
        noise = hal.alloc_elem("noise", max(RP.DATA, RP.ACCUM) * zk)
        r.check(lib.r0hip_fill_uniform(noise.ptr, RP.DATA * zk, seed))
        r.check(lib.r0hip_eltwise_copy_elem_slice(data.ptr, noise.ptr, RP.DATA, zk, 0, zk, n - zk, n))
        hal.eltwise_zeroize_elem(data)
        accum = hal.alloc_elem_init("accum", RP.ACCUM * n, 0xFFFFFFFF)
        r.check(lib.r0hip_fill_uniform(noise.ptr, RP.ACCUM * zk, seed + 1))
        r.check(lib.r0hip_eltwise_copy_elem_slice(accum.ptr, noise.ptr, RP.ACCUM, zk, 0, zk, n - zk, n))
        return data, glob, accum
    data, glob, accum = witness()
    seal, mix = halprover.prove_segment(hal, "recursion", po2, ctrl, data, accum, glob, accum_mode=2,
                                        work_cycles=len(prog.rows))
    assert np.array_equal(mix, fused_mix) and np.array_equal(seal, fused_seal)
    data, glob, accum = witness()

    def accumulate(mix_buf, mix_words):  # prove/witgen.rs:162-177
        r.check(lib.r0hip_recursion_accum(ctrl.ptr, glob.ptr, data.ptr, mix_buf.ptr, accum.ptr, len(prog.rows), n))
        hal.eltwise_zeroize_elem(accum)
    pseal, pmix = hal_prover.prove_segment(oracle, hal, "recursion", po2, ctrl, data, accum, glob, accumulate=accumulate)
    assert np.array_equal(pmix, fused_mix) and np.array_equal(pseal, fused_seal)
    assert r.verify_seal("recursion", hal.suite, seal, check_validity=True) == po2
