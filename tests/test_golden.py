"""Golden fixtures (tests/golden/, made by tools/make_golden.py from the reference's own
compiled C++ poly_fp and the oracle's Prover restatement) pinning, on the CPU:
  * the flattened constraint programs (risc0_amd/circuits/*.poly.ir) the HIP eval_check
    kernels are generated from — evaluated by tests/ir_eval.py, no reference needed;
  * the oracle's eval_check and whole-segment seals (when oracle/_ref is built).
The GPU side of the same fixtures is in tests/test_gpu_parity.py."""
import hashlib
import json
import os
import re

import numpy as np
import pytest

import ir_eval

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
P = 15 * 2**27 + 1
NB = P - 11

with open(os.path.join(GOLD, "index.json")) as f:
    INDEX = json.load(f)


def digest(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a, dtype=np.uint32).tobytes())
    return h.hexdigest()


def eval_inputs(oracle, circuit, po2, seed):
    d = oracle.load_circuit_json(circuit)
    rng = np.random.default_rng(seed)
    D = 4 << po2
    gs = d["group_sizes"]
    groups = [oracle.rand_elems(rng, gs[g] * D) for g in range(3)]
    mix = oracle.rand_elems(rng, d["mix_size"])
    glob = oracle.rand_elems(rng, d["output_size"])
    pm = oracle.rand_elems(rng, 4)
    return groups, mix, glob, pm


def seal_inputs(oracle, circuit, po2):
    d = oracle.load_circuit_json(circuit)
    rng = np.random.default_rng(0x5249534330 + po2)
    n = 1 << po2
    gs = d["group_sizes"]
    code, data, accum = (oracle.rand_elems(rng, gs[g] * n) for g in (1, 2, 0))
    glob = oracle.rand_elems(rng, d["output_size"])
    glob[3] = 0xFFFFFFFF
    return code, data, accum, glob


def rou_fwd():
    src = open(os.path.join(ROOT, "risc0_amd", "csrc", "bb31.h")).read()
    body = re.search(r"kRouFwd\[28\] = \{([^}]*)\}", src).group(1)
    return [int(x) for x in re.findall(r"\d+", body)]


def e_mul(a, b):
    r = [0, 0, 0, 0]
    for i in range(4):
        for j in range(4):
            if i + j < 4:
                r[i + j] += a[i] * b[j]
            else:
                r[i + j - 4] += NB * a[i] * b[j]
    return tuple(x % P for x in r)


def e_pow(a, n):
    r = (1, 0, 0, 0)
    while n:
        if n & 1:
            r = e_mul(r, a)
        a = e_mul(a, a)
        n >>= 1
    return r


@pytest.mark.parametrize("case", INDEX["eval_check"], ids=lambda c: f"{c['circuit']}-po2{c['po2']}")
def test_ir_program_matches_reference_poly_fp(oracle, case):
    """The IR the HIP kernels are generated from reproduces the reference's own poly_fp."""
    circuit, po2 = case["circuit"], case["po2"]
    groups, mix, glob, pm = eval_inputs(oracle, circuit, po2, case["seed"])
    assert digest(*groups, mix, glob, pm) == case["inputs_sha256"], "numpy RNG stream changed"
    gold = np.load(os.path.join(GOLD, case["file"]))
    d = oracle.load_circuit_json(circuit)
    bufs = {"accum": groups[0], "code": groups[1], "data": groups[2], "mix": mix, "global": glob}
    args = [oracle.decode(bufs[a]).astype(np.uint64) for a in d["eval_args"]]
    poly_mix = tuple(int(x) for x in oracle.decode(pm))
    pows = [e_pow(poly_mix, k) for k in d["poly_mix_powers"]]
    D = 4 << po2
    fp = ir_eval.evaluate(ir_eval.load_ir(circuit), args, D, pows)
    # check = poly_fp(x) / ((3x)^N - 1), x = w_D^cycle (rv32im/src/prove/hal/cpu.rs:145-207)
    w = rou_fwd()[po2 + 2]
    out = np.zeros((4, D), np.uint64)
    for c in range(D):
        x = 3 * pow(w, c, P) % P
        inv = pow((pow(x, 1 << po2, P) - 1) % P, P - 2, P)
        for k in range(4):
            out[k, c] = int(fp[k][c]) * inv % P
    assert np.array_equal(oracle.encode(out.reshape(-1)), gold)


@pytest.mark.parametrize("case", INDEX["eval_check"], ids=lambda c: f"{c['circuit']}-po2{c['po2']}")
def test_oracle_eval_check_matches_golden(oracle, case):
    if oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built (needs the reference sources)")
    groups, mix, glob, pm = eval_inputs(oracle, case["circuit"], case["po2"], case["seed"])
    check = np.zeros(4 * (4 << case["po2"]), np.uint32)
    oracle.eval_check(case["circuit"], check, groups, mix, glob, pm, case["po2"])
    assert np.array_equal(check, np.load(os.path.join(GOLD, case["file"])))


@pytest.mark.parametrize("case", INDEX["seals"], ids=lambda c: f"{c['circuit']}-{c['suite']}-po2{c['po2']}")
def test_oracle_seal_matches_golden(oracle, case):
    circuit, po2 = case["circuit"], case["po2"]
    code, data, accum, glob = seal_inputs(oracle, circuit, po2)
    assert digest(code, data, accum, glob) == case["inputs_sha256"]
    if oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built (needs the reference sources)")
    s = {"poseidon2": oracle.POSEIDON2, "sha-256": oracle.SHA256, "poseidon_254": oracle.POSEIDON254}[case["suite"]]
    seal, mix, _ = oracle.prove_segment(circuit, s, po2, code, data, accum, glob,
                                        version=2 if circuit == "rv32im" else None)
    assert seal.size == case["seal_words"]
    assert digest(seal) == case["seal_sha256"]
    assert [int(x) for x in mix] == case["mix"]
