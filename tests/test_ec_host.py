"""CPU check of the generated eval_check arithmetic (tools/gen_eval_check.py).

The generator emits the same per-point kernel bodies the gfx950 build compiles as one
host translation unit (`--host`), compiled here with g++. Its lazy value-range analysis
(reductions only where a word or a 64-bit sum could overflow) is exercised on:
  * the golden fixtures made from the reference's own compiled poly_fp
    (tests/golden, risc0/circuit/*/src/prove/hal/cpu.rs eval_check semantics);
  * extreme inputs (every word p-1, or mixes of 0, 1, p-2, p-1) checked against the
    numpy IR interpreter, where every bound is hit as tightly as the data allows.
The device kernels are checked on the GPU by tests/test_gpu_parity.py."""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import ir_eval
from test_golden import GOLD, INDEX, e_mul, e_pow, eval_inputs, rou_fwd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 15 * 2**27 + 1
u32p = C.POINTER(C.c_uint32)


# generator variants: the default (tuned per kernel), the lazy range analysis with saddr tap
# loads and split accumulation chains, and 64-bit sums of products (EC_FUSE) in canonical and
# lazy kernels (tools/gen_eval_check.py knobs)
VARIANTS = {"canonical": {}, "lazy": {"EC_CANON": "0", "EC_SADDR": "1", "EC_SPLIT": "2"},
            "fused": {"EC_FUSE_FORCE": "1"}, "fused_canon": {"EC_FUSE_FORCE": "1", "EC_CANON_FORCE": "1"},
            "fused_lazy": {"EC_FUSE_FORCE": "1", "EC_CANON_FORCE": "0"}}


@pytest.fixture(scope="module", params=sorted(VARIANTS))
def host_ec(request, tmp_path_factory):
    libs = {}
    d = tmp_path_factory.mktemp("ec_host_" + request.param)
    env = dict(os.environ, **VARIANTS[request.param])
    for circuit in ("rv32im", "recursion"):
        src = d / f"ec_{circuit}.cpp"
        so = d / f"ec_{circuit}.so"
        subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "gen_eval_check.py"), "--host", circuit,
                               str(src)], stdout=subprocess.DEVNULL, env=env)
        subprocess.check_call(["g++", "-O0", "-std=c++17", "-shared", "-fPIC",
                               "-I" + os.path.join(ROOT, "risc0_amd", "csrc"), str(src), "-o", str(so)])
        libs[circuit] = C.CDLL(str(so))
    return libs


def ptr(a):
    return a.ctypes.data_as(u32p)


def enc(x):
    return np.array([(int(v) % P) * 2**32 % P for v in x], dtype=np.uint32)


def run_host(lib, circuit, args_plain_words, poly_mix, po2):
    """args: Montgomery word arrays in eval_args order; poly_mix: plain FpExt tuple."""
    d = json.load(open(os.path.join(ROOT, "risc0_amd", "circuits", circuit + ".taps.json")))
    combos = C.POINTER(C.c_int)()
    npm = C.c_int()
    ncomb = getattr(lib, f"ec_host_{circuit}_combos")(C.byref(combos), C.byref(npm))
    pows = [e_pow(poly_mix, k) for k in d["poly_mix_powers"]][:npm.value]
    k = 0
    for _ in range(ncomb):
        n = combos[k]
        prod = (1, 0, 0, 0)
        for q in range(n):
            prod = e_mul(prod, pows[combos[k + 1 + q]])
        k += 1 + n
        pows.append(prod)
    pm = enc([x for t in pows for x in t])
    pmn = enc([x * (P - 11) for t in pows for x in t])
    D = 4 << po2
    w = rou_fwd()[po2 + 2]
    vinv = enc([pow((pow(3 * pow(w, q, P) % P, 1 << po2, P) - 1) % P, P - 2, P) for q in range(4)])
    acc = np.zeros(4 * D, np.uint32)
    # materialised sub-expressions (tools/pick_ec_mat.py): up to 64 Fp and 64 FpExt slots
    mf = np.zeros(64 * D, np.uint32)
    me = np.zeros(64 * 4 * D, np.uint32)
    check = np.zeros(4 * D, np.uint32)
    arrs = [np.ascontiguousarray(a, dtype=np.uint32) for a in args_plain_words]
    argv = (u32p * len(arrs))(*[ptr(a) for a in arrs])
    getattr(lib, f"ec_host_{circuit}")(argv, ptr(pm), ptr(pmn), ptr(vinv), ptr(acc), ptr(mf), ptr(me), ptr(check),
                                       C.c_uint32(D))
    return check


@pytest.mark.parametrize("case", INDEX["eval_check"], ids=lambda c: f"{c['circuit']}-po2{c['po2']}")
def test_generated_eval_check_matches_golden(host_ec, oracle, case):
    circuit, po2 = case["circuit"], case["po2"]
    groups, mix, glob, pm = eval_inputs(oracle, circuit, po2, case["seed"])
    d = oracle.load_circuit_json(circuit)
    bufs = {"accum": groups[0], "code": groups[1], "data": groups[2], "mix": mix, "global": glob}
    args = [bufs[a] for a in d["eval_args"]]
    poly_mix = tuple(int(x) for x in oracle.decode(pm))
    out = run_host(host_ec[circuit], circuit, args, poly_mix, po2)
    assert np.array_equal(out, np.load(os.path.join(GOLD, case["file"])))


@pytest.mark.parametrize("circuit", ["rv32im", "recursion"])
@pytest.mark.parametrize("mode", ["all_pm1", "edge_mix"])
def test_generated_eval_check_extreme_inputs(host_ec, oracle, circuit, mode):
    po2 = 2
    D = 4 << po2
    d = oracle.load_circuit_json(circuit)
    rng = np.random.default_rng(7)
    gs = d["group_sizes"]
    sizes = {"accum": gs[0] * D, "code": gs[1] * D, "data": gs[2] * D, "mix": d["mix_size"],
             "global": d["output_size"]}
    edge = np.array([0, 1, 2, P - 2, P - 1], dtype=np.uint64)
    plain = {}
    for k, n in sizes.items():
        plain[k] = np.full(n, P - 1, np.uint64) if mode == "all_pm1" else rng.choice(edge, size=n)
    poly_mix = (P - 1, P - 1, P - 1, P - 1) if mode == "all_pm1" else (P - 2, 1, P - 1, 2)
    args_plain = [plain[a] for a in d["eval_args"]]
    out = run_host(host_ec[circuit], circuit, [enc(a) for a in args_plain], poly_mix, po2)
    pows = [e_pow(poly_mix, k) for k in d["poly_mix_powers"]]
    fp = ir_eval.evaluate(ir_eval.load_ir(circuit), args_plain, D, pows)
    w = rou_fwd()[po2 + 2]
    ref = np.zeros((4, D), np.uint64)
    for c in range(D):
        x = 3 * pow(w, c, P) % P
        inv = pow((pow(x, 1 << po2, P) - 1) % P, P - 2, P)
        for k in range(4):
            ref[k, c] = int(fp[k][c]) * inv % P
    assert np.array_equal(out, enc(ref.reshape(-1)))
