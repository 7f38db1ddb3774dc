#!/usr/bin/env python3
"""rv32im accumulation (r0hip_rv32im_accum) at po2=20 on random rows over all instruction
arms: HIP-event times of the generated per-cycle step and of the scan/finalize; with
--reference also the compiled reference accumulation's time on the same rows and equality."""
import json
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import risc0_amd as r  # noqa: E402
from test_rv32im_accum_ir import rows_for_arms  # noqa: E402

P = 15 * 2**27 + 1


def main():
    po2 = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    rows = 1 << po2
    hal = r.HipHal("poseidon2")
    rng = np.random.default_rng(3)
    data = rows_for_arms(rng, rows, list(rng.integers(0, 13, rows)))
    d_data = hal.copy_from_elem("data", data)
    glob = rng.integers(0, P, 90, dtype=np.uint64).astype(np.uint32)
    mix = rng.integers(0, P, 36, dtype=np.uint64).astype(np.uint32)
    d_glob = hal.copy_from_elem("g", glob)
    d_mix = hal.copy_from_elem("m", mix)
    inval = np.full(103 * rows, 0xFFFFFFFF, np.uint32)
    acc = hal.copy_from_elem("acc", inval)
    hal.rv32im_accum(d_data, acc, d_glob, d_mix, rows, rows)  # warm
    out = {}
    for rep in range(3):
        acc.copy_from(inval)
        hal.synchronize()
        r.set_kernel_timing(True)
        hal.rv32im_accum(d_data, acc, d_glob, d_mix, rows, rows)
        t = r.kernel_times()
        r.set_kernel_timing(False)
        out[rep] = {k: round(v[0], 3) for k, v in t.items()}
    res = {"po2": po2, "ms": out}
    if "--reference" in sys.argv:
        # the reference's compiled risc0_circuit_rv32im_cpu_accum (all three phases) on the
        # same rows, on every host thread its pool starts; and word-for-word equality
        import time
        import rv32im_accum_ref as R
        t0 = time.perf_counter()
        want = R.accum(data, glob, mix, rows, rows)
        res["reference_cpu_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
        res["reference_cpu_threads"] = os.cpu_count()
        res["equal_to_reference"] = bool(np.array_equal(acc.to_numpy(), want))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
