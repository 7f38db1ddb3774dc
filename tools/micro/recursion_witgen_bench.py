#!/usr/bin/env python3
"""Recursion witness generation (r0hip_recursion_witgen) and accumulation
(r0hip_recursion_accum) against the reference's compiled CPU witgen and accumulation (risc0_circuit_recursion_cpu_witgen in oracle/_ref/libref_recursion.so, parallel
mode, every host core) on the same program: a random recursion program filling a segment
of 2^po2 rows (tests/recursion_program.py, restated preflight).

Reports the GPU's HIP-event times per phase (exec, WOM sort + back injection, verify), the
call's wall time including the preflight upload from host memory, the reference's wall
time, and whether the two data groups are equal word for word.

  recursion_witgen_bench.py [PO2 [REPS]]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # oracle.py: the preflight's Poseidon2 (test code)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import recursion_program as RP  # noqa: E402
import risc0_amd as r  # noqa: E402


def main():
    po2 = int(sys.argv[1]) if len(sys.argv) > 1 else 18
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    n = 1 << po2
    rng = np.random.default_rng(18)
    prog, inp = RP.random_program(rng, n - RP.ZK_CYCLES - 1)
    pf = RP.preflight(prog, inp)
    t0 = time.perf_counter()
    ctrl, data, glob = RP.witgen(prog, pf, po2, raw=True)
    cpu_s = time.perf_counter() - t0
    # the C call's own cost: the trace as contiguous u32 arrays up front (the ctypes wrapper
    # would otherwise convert the Python list of cycles on every call)
    wom, cyc, iops = (np.ascontiguousarray(np.asarray(x, np.uint32)) for x in RP.trace_arrays(pf))
    hal = r.HipHal("poseidon2")
    d_ctrl = hal.copy_from_elem("ctrl", ctrl)
    inval = np.full(RP.DATA * n, RP.INVALID, np.uint32)
    dd = hal.copy_from_elem("data", inval)
    dg = hal.copy_from_elem("glob", np.full(RP.OUT, RP.INVALID, np.uint32))
    r.recursion_witgen(d_ctrl, dd, dg, n, wom, cyc, iops)  # warm
    equal = bool(np.array_equal(dd.to_numpy(), data)) and bool(np.array_equal(dg.to_numpy(), glob))
    plain = []
    for _ in range(reps):
        dd.copy_from(inval)
        hal.synchronize()
        t0 = time.perf_counter()
        r.recursion_witgen(d_ctrl, dd, dg, n, wom, cyc, iops)
        plain.append((time.perf_counter() - t0) * 1e3)
    phases, walls = [], []
    for _ in range(reps):
        dd.copy_from(inval)
        hal.synchronize()
        r.set_kernel_timing(True)
        t0 = time.perf_counter()
        r.recursion_witgen(d_ctrl, dd, dg, n, wom, cyc, iops)
        walls.append((time.perf_counter() - t0) * 1e3)
        t = r.kernel_times()
        r.set_kernel_timing(False)
        phases.append({k: round(v[0], 3) for k, v in t.items()})
    # the accumulation (r0hip_recursion_accum) on the same program's witness as the prover
    # hands it over (ZK noise rows, INVALID zeroized), against the compiled
    # risc0_circuit_recursion_cpu_accum with the same mix
    import accum_ir as A
    w_ctrl, w_data, w_glob = RP.witgen(prog, pf, po2, noise_seed=5)
    acc0 = RP.accum_init(po2, noise_seed=6)
    mix = np.random.default_rng(7).integers(0, RP.P, RP.MIX, dtype=np.uint64).astype(np.uint32)
    want = acc0.copy()
    t0 = time.perf_counter()
    A.ref_accum(w_ctrl, w_glob, w_data, mix, want, len(prog.rows), n)
    acc_cpu_s = time.perf_counter() - t0
    dc, dgl, dda, dmx = (hal.copy_from_elem(nm, x) for nm, x in
                         (("c", w_ctrl), ("g", w_glob), ("d", w_data), ("m", mix)))
    dacc = hal.copy_from_elem("acc", acc0)
    hal.recursion_accum(dc, dgl, dda, dmx, dacc, len(prog.rows), n)  # warm
    acc_equal = bool(np.array_equal(dacc.to_numpy(), want))
    acc_ms = []
    for _ in range(reps):
        dacc.copy_from(acc0)
        hal.synchronize()
        r.set_kernel_timing(True)
        hal.recursion_accum(dc, dgl, dda, dmx, dacc, len(prog.rows), n)
        t = r.kernel_times()
        r.set_kernel_timing(False)
        acc_ms.append(sum(v[0] for v in t.values()))
    print(json.dumps({
        "po2": po2, "cycles": len(prog.rows), "equal_to_reference": equal,
        "accumulation": {"gpu_ms": round(float(np.median(acc_ms)), 3), "reference_cpu_ms": round(acc_cpu_s * 1e3, 1),
                         "equal_to_reference": acc_equal},
        "gpu_ms_by_phase": phases[-1],
        "gpu_ms_wall_with_upload": round(float(np.median(plain)), 3),
        "gpu_ms_wall_with_upload_and_kernel_timing": round(float(np.median(walls)), 3),
        "trace_bytes": int(wom.nbytes + cyc.nbytes + iops.nbytes),
        "reference_cpu_ms": round(cpu_s * 1e3, 1),
        "reference_cpu_threads": {"affinity": len(os.sched_getaffinity(0)), "hardware_concurrency": os.cpu_count(),
                                  "note": "poolstl's default pool starts hardware_concurrency threads"},
    }))


if __name__ == "__main__":
    main()
