#!/usr/bin/env python3
"""Poseidon2 Merkle layer latency, one lane per node vs one quad per node
(risc0_amd/csrc/hash.hip p2_fold_kernel / p2_fold_quad_kernel, poseidon2.h).

Times r0hip_hash_fold on layers of n nodes: K back-to-back launches then one
synchronize, as merkle_tree issues them. The lane/quad choice is the library's
R0_P2_QUAD_MAX (read once per process), so run this once per setting:
    R0_P2_QUAD_MAX=0 python3 tools/micro/fold_latency.py      # one lane per node
    R0_P2_QUAD_MAX=1000000 python3 tools/micro/fold_latency.py  # one quad per node
Prints one JSON line {"quad_max": .., "us_per_layer": {n: us}}.
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from risc0_amd.hal import HipHal  # noqa: E402


def main():
    hal = HipHal("poseidon2")
    rng = np.random.default_rng(1)
    out = {}
    K = 200
    for lg in range(6, 20):
        n = 1 << lg
        io = np.zeros(4 * n * 8, np.uint32)
        io[2 * n * 8:] = (rng.integers(0, 2**31, 2 * n * 8, dtype=np.uint64) % 2013265921).astype(np.uint32)
        d = hal.copy_from_digest("io", io)
        for _ in range(5):
            hal.hash_fold(d, 2 * n, n)
        hal.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            hal.hash_fold(d, 2 * n, n)
        hal.synchronize()
        out[n] = round((time.perf_counter() - t0) / K * 1e6, 2)
        del d
    print(json.dumps({"quad_max": os.environ.get("R0_P2_QUAD_MAX", "default"), "us_per_layer": out}))


if __name__ == "__main__":
    main()
