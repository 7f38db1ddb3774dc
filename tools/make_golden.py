#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ from the reference itself.

Run in the build container (needs /root/reference for oracle/_ref): the eval_check
outputs come from the reference's own compiled C++ poly_fp (rv32im
rust_poly_fp_*.cpp / recursion ffi.cpp, built by `make -C oracle ref`) driven by the
oracle's CircuitHal::eval_check restatement; the seals come from the oracle's C++
restatement of Prover + CpuHal with that poly_fp. Fixtures are data only (seeds,
input digests, outputs); tests regenerate the inputs from the seeds.

  python tools/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")

# (circuit, po2, seed) — eval_check fixtures (D = 4 * 2^po2 points)
EVAL_CASES = [("rv32im", 4, 0x4543_0004), ("rv32im", 6, 0x4543_0006), ("recursion", 4, 0x4543_1004),
              ("recursion", 6, 0x4543_1006)]
# (circuit, suite, po2) — whole-segment seals, seed 0x5249534330 + po2 (as tests/test_gpu_parity.py)
SEAL_CASES = [("rv32im", "poseidon2", 8), ("rv32im", "poseidon2", 11), ("rv32im", "sha-256", 9),
              ("recursion", "poseidon2", 9), ("recursion", "sha-256", 8), ("recursion", "poseidon_254", 8)]
SUITE_IDS = {"poseidon2": oracle.POSEIDON2, "sha-256": oracle.SHA256, "poseidon_254": oracle.POSEIDON254}


def eval_inputs(circuit, po2, seed):
    d = oracle.load_circuit_json(circuit)
    rng = np.random.default_rng(seed)
    D = 4 << po2
    gs = d["group_sizes"]
    groups = [oracle.rand_elems(rng, gs[g] * D) for g in range(3)]
    mix = oracle.rand_elems(rng, d["mix_size"])
    glob = oracle.rand_elems(rng, d["output_size"])
    pm = oracle.rand_elems(rng, 4)
    return groups, mix, glob, pm


def seal_inputs(circuit, po2):
    d = oracle.load_circuit_json(circuit)
    rng = np.random.default_rng(0x5249534330 + po2)
    n = 1 << po2
    gs = d["group_sizes"]
    code, data, accum = (oracle.rand_elems(rng, gs[g] * n) for g in (1, 2, 0))
    glob = oracle.rand_elems(rng, d["output_size"])
    glob[3] = 0xFFFFFFFF  # INVALID globals are zeroized into the header
    return code, data, accum, glob


def digest(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a, dtype=np.uint32).tobytes())
    return h.hexdigest()


def main():
    oracle.build(ref=True)
    if oracle.ref_lib() is None:
        sys.exit("oracle/_ref (the reference's compiled poly_fp) is required; run in the build container")
    os.makedirs(OUT, exist_ok=True)
    index = {"eval_check": [], "seals": []}
    for circuit, po2, seed in EVAL_CASES:
        groups, mix, glob, pm = eval_inputs(circuit, po2, seed)
        check = np.zeros(4 * (4 << po2), np.uint32)
        oracle.eval_check(circuit, check, groups, mix, glob, pm, po2)
        name = f"eval_check_{circuit}_po2_{po2}.npy"
        np.save(os.path.join(OUT, name), check)
        index["eval_check"].append({"circuit": circuit, "po2": po2, "seed": seed, "file": name,
                                    "inputs_sha256": digest(*groups, mix, glob, pm)})
    for circuit, suite, po2 in SEAL_CASES:
        code, data, accum, glob = seal_inputs(circuit, po2)
        s = SUITE_IDS[suite]
        seal, mix, _ = oracle.prove_segment(circuit, s, po2, code, data, accum, glob,
                                            version=2 if circuit == "rv32im" else None)
        index["seals"].append({"circuit": circuit, "suite": suite, "po2": po2,
                               "inputs_sha256": digest(code, data, accum, glob), "seal_words": int(seal.size),
                               "seal_sha256": digest(seal), "seal_head": [int(x) for x in seal[:16]],
                               "mix": [int(x) for x in mix]})
    with open(os.path.join(OUT, "index.json"), "w") as f:
        json.dump(index, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
