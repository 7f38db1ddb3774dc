"""Per-op Merkle tree over an all-zero 1-column matrix (rv32im's code group at po2=20: 4M
rows): r0hip_hash_rows into the heap's leaf range, then r0hip_hash_fold per layer, as
MerkleTreeProver::new drives a HAL. Prints ms per tree (run with R0_P2_ZERO=0 / 1)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import risc0_amd as r  # noqa: E402
from risc0_amd import hal as H  # noqa: E402

rows = 1 << 22
h = r.HipHal("poseidon2")
m = h.copy_from_elem("m", np.zeros(rows, np.uint32))
nodes = h.alloc_digest("nodes", 2 * rows)
for it in range(4):
    H.check(H.lib().r0hip_synchronize())
    t = time.perf_counter()
    h.hash_rows(nodes.slice(rows, rows), m)
    layer = rows
    while layer > 1:
        h.hash_fold(nodes, layer, layer // 2)
        layer //= 2
    H.check(H.lib().r0hip_synchronize())
    dt = (time.perf_counter() - t) * 1e3
print(f"R0_P2_ZERO={os.environ.get('R0_P2_ZERO', '1')} per-op zero tree 2^22 rows: {dt:.3f} ms; root {nodes.to_numpy()[8:16]}")
