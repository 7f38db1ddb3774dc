#!/usr/bin/env python3
"""rv32im witness generation (r0hip_rv32im_witgen) against the reference's compiled CPU witgen
(risc0_circuit_rv32im_cpu_witgen in oracle/_ref/libref_rv32im_accum.so, parallel mode) on the
same preflight: the bench's loop guest (tests/rv32im_trace.py loop_trace, 32-instruction body)
filling a segment of 2^po2 rows.

Reports the GPU's HIP-event times per phase (bucketing, phase 1 = cycles before the table
split, phase 2 = table and done rows), the call's wall time including the preflight upload
from host memory, the reference's wall time, and whether the data and global groups are equal
word for word. R0_RVWG_SORT=0 selects the unsorted (atomic-cursor) bucketing.

  rv32im_witgen_bench.py [PO2 [REPS]]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import risc0_amd as r  # noqa: E402
import rv32im_trace as T  # noqa: E402
import rv32im_witgen_ref as W  # noqa: E402


def main():
    po2 = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    n = 1 << po2
    t0 = time.perf_counter()
    t = T.loop_trace(po2, body_len=32, seed=0x5249534330)
    build_s = time.perf_counter() - t0
    data, glob, cyc, tx = W.inputs(t)
    split = t.table_split_cycle
    hal = r.HipHal("poseidon2")
    dd = hal.copy_from_elem("data", data)
    dg = hal.copy_from_elem("global", glob)
    r.rv32im_witgen(dd, dg, cyc, tx, split)  # warm
    gpu_d, gpu_g = dd.to_numpy(), dg.to_numpy()
    walls, phases = [], []
    for _ in range(reps):
        dd.copy_from(data)
        dg.copy_from(glob)
        hal.synchronize()
        r.set_kernel_timing(True)
        t0 = time.perf_counter()
        r.rv32im_witgen(dd, dg, cyc, tx, split)
        walls.append((time.perf_counter() - t0) * 1e3)
        kt = r.kernel_times()
        r.set_kernel_timing(False)
        phases.append({k: round(v[0], 3) for k, v in kt.items()})
    out = {"po2": po2, "cycles": n, "table_split_cycle": split, "txns": int(len(tx)),
           "sorted_buckets": os.environ.get("R0_RVWG_SORT", "1") != "0",
           "trace_build_s": round(build_s, 2),
           "gpu_wall_ms_incl_upload": sorted(round(w, 3) for w in walls),
           "gpu_phase_ms": phases[len(phases) // 2]}
    if "--no-ref" not in sys.argv:
        t0 = time.perf_counter()
        ref_d, ref_g = W.run(data, glob, cyc, tx, split, n, W.MODE_PARALLEL)
        out["ref_cpu_parallel_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
        out["cpu_threads"] = len(os.sched_getaffinity(0))
        out["equal"] = bool(np.array_equal(gpu_d, ref_d) and np.array_equal(gpu_g, ref_g))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
