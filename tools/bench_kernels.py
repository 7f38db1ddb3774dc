#!/usr/bin/env python3
"""Micro-benchmarks of individual HAL ops at prover shapes (po2=20 rv32im data group),
timed with the library's HIP-event kernel timer. Run under rocprofv3 for per-kernel splits."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import risc0_amd as r  # noqa: E402

P = 15 * 2**27 + 1


def main():
    which = sys.argv[1:] or ["ntt", "hash"]
    hal = r.HipHal("poseidon2")
    rng = np.random.default_rng(1)
    if "ec" in which:
        import json
        name = os.environ.get("R0_EC_CIRCUIT", "rv32im")
        circ = json.load(open(os.path.join(ROOT, "risc0_amd", "circuits", name + ".taps.json")))
        po2 = 20 if name == "rv32im" else 18
        D = 4 << po2
        gs = circ["group_sizes"]
        groups = [hal.copy_from_elem("g", rng.integers(0, P, gs[g] * D, dtype=np.uint64).astype(np.uint32))
                  for g in range(3)]
        mix = hal.copy_from_elem("mix", rng.integers(0, P, circ["mix_size"], dtype=np.uint64).astype(np.uint32))
        glob = hal.copy_from_elem("glob", rng.integers(0, P, circ["output_size"], dtype=np.uint64).astype(np.uint32))
        out = hal.alloc_elem("check", 4 * D)
        pm = rng.integers(0, P, 4, dtype=np.uint64).astype(np.uint32)
        hal.eval_check(name, out, groups, mix, glob, pm, po2)
        hal.synchronize()
        r.set_kernel_timing(True)
        for _ in range(3):
            hal.eval_check(name, out, groups, mix, glob, pm, po2)
        hal.synchronize()
        for k, v in sorted(r.kernel_times().items()):
            print(f"{os.environ.get('R0HIP_LIB', 'default')}: {k} {v[0] / v[1]:.3f} ms/launch")
        return
    if "fold" in which:
        # the Merkle layers of one po2=20 tree (2^22 leaves) down to 1024 nodes
        D = 4 << 20
        nodes = hal.copy_from_elem("nodes", rng.integers(0, P, 2 * D * 8, dtype=np.uint64).astype(np.uint32))
        r.set_kernel_timing(True)
        for _ in range(5):
            size = D
            while size > 1024:
                hal.hash_fold(nodes, size, size // 2)
                size //= 2
        hal.synchronize()
        for k, (ms, calls, b, _mm) in sorted(r.kernel_times().items()):
            print(f"{k:28s} {ms / calls:9.3f} ms/launch")
        return
    if "rows" in which:
        # leaf rows of the narrow groups: 16 columns (check) and 1 column at 2^22 rows
        D = 4 << 20
        for c in (16, 1):
            m = hal.copy_from_elem(f"m{c}", rng.integers(0, P, c * D, dtype=np.uint64).astype(np.uint32))
            d = hal.alloc_digest(f"d{c}", D)
            r.set_kernel_timing(True)
            for _ in range(5):
                hal.hash_rows(d, m)
            hal.synchronize()
            for k, (ms, calls, b, _mm) in sorted(r.kernel_times().items()):
                print(f"cols={c:2d} {k:28s} {ms / calls:9.3f} ms/launch")
            r.set_kernel_timing(False)
        return
    cols, po2 = 211, 20
    n = 1 << po2
    inp = hal.copy_from_elem("in", rng.integers(0, P, cols * n, dtype=np.uint64).astype(np.uint32))
    out = hal.alloc_elem("out", cols * 4 * n)
    reps = 5
    r.set_kernel_timing(True)
    for _ in range(reps):
        if "ntt" in which:
            hal.batch_expand_into_evaluate_ntt(out, inp, cols, 2)
            hal.batch_interpolate_ntt(inp, cols)
        if "hash" in which:
            d = hal.alloc_digest("d", 4 * n)
            hal.hash_rows(d, out)
    hal.synchronize()
    for k, (ms, calls, b, _mm) in sorted(r.kernel_times().items()):
        print(f"{k:28s} {ms / calls:9.3f} ms/launch  {b / calls / 1e9:7.3f} GB alg  {b / (ms / 1e3) / 1e9:8.1f} GB/s")


if __name__ == "__main__":
    main()
