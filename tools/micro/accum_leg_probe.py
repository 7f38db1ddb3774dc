#!/usr/bin/env python3
"""Why the resident with_accumulation leg is slower than the pipeline's device-accumulation
leg: time 6 po2=20 proofs over 2 threads with and without the per-proof INVALID fill."""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import risc0_amd as r  # noqa: E402

n = 1 << 20
hal = r.HipHal("poseidon2")
rng = np.random.default_rng(1)
code, data, _a, glob = bench.synthetic_witness(rng, {"group_sizes": [103, 1, 211], "output_size": 90}, 20)
dc, dd = hal.copy_from_elem("c", code), hal.copy_from_elem("d", bench.mixed_arm_rows(data, n))
accs = [hal.alloc_elem("a", 103 * n) for _ in range(2)]
globs = [hal.copy_from_elem("g", glob) for _ in range(2)]


def run(slot, cnt, fill, fused):
    for _ in range(cnt):
        if fill:
            r.check(r.lib().r0hip_memset32(accs[slot].ptr, 0xFFFFFFFF, accs[slot].size))
        if fused:
            r.prove_segment_accum(hal, "rv32im", 20, dc, dd, accs[slot], n, globs[slot], version=2)
        else:
            r.prove_segment(hal, "rv32im", 20, dc, dd, accs[slot], globs[slot], version=2)


def batch(cnt, fill, fused):
    ts = [threading.Thread(target=run, args=(i, cnt // 2, fill, fused)) for i in range(2)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    hal.synchronize()
    return 1000 * (time.perf_counter() - t0) / cnt


for fill, fused in ((False, False), (True, False), (False, True), (True, True), (False, True)):
    batch(4, fill, fused)
    print(f"fill={fill} fused={fused}: {batch(8, fill, fused):.1f} ms/segment", flush=True)
