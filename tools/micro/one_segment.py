#!/usr/bin/env python3
"""One rv32im po2=20 segment through r0hip_prove_segments from pinned host memory, after
a warm-up call: the single-segment latency leg of bench.py's end_to_end, alone, for a
rocprofv3 --kernel-trace --memory-copy-trace timeline (tools/timeline.py)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import risc0_amd as r  # noqa: E402

P = 15 * 2**27 + 1


def main():
    po2 = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    with open(os.path.join(ROOT, "risc0_amd", "circuits", "rv32im.taps.json")) as f:
        circ = json.load(f)
    hal = r.HipHal("poseidon2")
    rng = np.random.default_rng(7)
    n = 1 << po2
    gs = circ["group_sizes"]
    sizes = [gs[1] * n, gs[2] * n, gs[0] * n, circ["output_size"]]
    lib = r.lib()
    hosts = []
    for sz in sizes:
        p = ctypes.c_void_p()
        r.check(lib.r0hip_host_alloc(ctypes.byref(p), sz * 4))
        hosts.append(p.value)
        np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint32)), shape=(sz,))[:] = \
            rng.integers(0, P, size=sz, dtype=np.uint64).astype(np.uint32)
    job = [tuple(hosts)]
    r.prove_segments(hal, "rv32im", po2, job * 2, version=2, in_flight=2)  # warm
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        r.prove_segments(hal, "rv32im", po2, job, version=2, in_flight=1)
        ts.append(round(1000 * (time.perf_counter() - t0), 1))
    print(json.dumps({"ms_one_segment": ts, "h2d_bytes": sum(sizes) * 4}))
    for hp in hosts:
        r.check(lib.r0hip_host_free(hp))


if __name__ == "__main__":
    main()
