#!/usr/bin/env python3
"""rv32im witness generation on an ecall-heavy trace (tests/rv32im_trace.py ecall_trace with
REPS passes of the machine-mode Poseidon2, SHA-256, BigInt and host I/O ecalls): per-phase
HIP-event times, for the per-arm kernel times under rocprofv3.

  rv32im_witgen_ecall_bench.py [PO2 [REPS [RUNS]]]
"""
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import risc0_amd as r  # noqa: E402
import rv32im_trace as T  # noqa: E402
import rv32im_witgen_ref as W  # noqa: E402


def main():
    po2 = int(sys.argv[1]) if len(sys.argv) > 1 else 18
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 120
    runs = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    t = T.ecall_trace(po2, seed=5, bigint=True, reps=reps)
    data, glob, cyc, tx = W.inputs(t)
    bi = t.bigint_array()
    hal = r.HipHal("poseidon2")
    dd, dg = hal.copy_from_elem("data", data), hal.copy_from_elem("global", glob)
    phases = []
    for k in range(runs + 1):
        dd.copy_from(data)
        dg.copy_from(glob)
        hal.synchronize()
        r.set_kernel_timing(True)
        r.rv32im_witgen(dd, dg, cyc, tx, t.table_split_cycle, bigint=bi)
        kt = r.kernel_times()
        r.set_kernel_timing(False)
        if k:
            phases.append({n: round(v[0], 3) for n, v in kt.items()})
    majors = np.bincount(cyc["major"][:t.table_split_cycle], minlength=13)
    print(json.dumps({"po2": po2, "reps": reps, "rows_by_arm": [int(x) for x in majors],
                      "gpu_phase_ms": phases[len(phases) // 2]}))


if __name__ == "__main__":
    main()
