"""ORACLE — test infrastructure only.

ctypes binding of the CPU restatement (oracle/liboracle.so) and of the reference's
own generated C++ constraint code (oracle/_ref/libref_polyfp.so, built from the
reference sources by oracle/Makefile). Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module; the product never does.
"""
import ctypes as C
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libref_polyfp.so")
CIRCUITS = os.path.join(ROOT, "risc0_amd", "circuits")

P = 15 * 2**27 + 1
POSEIDON2, SHA256, POSEIDON254 = 0, 1, 2

u32p = C.POINTER(C.c_uint32)
_lib = None
_ref = None


def build(ref=True):
    import subprocess
    subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])
    if ref and os.path.isdir(os.environ.get("R0_REFERENCE", "/root/reference")) and not os.path.exists(REF_PATH):
        subprocess.check_call(["make", "-s", "-j8", "-C", HERE, "ref"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build(ref=False)
        _lib = C.CDLL(LIB_PATH)
        _lib.oracle_prove_segment.restype = C.c_void_p
        _lib.oracle_eval_check.restype = C.c_void_p
        _lib.oracle_eval_check_sampled.restype = C.c_void_p
        _lib.oracle_combos_divide.restype = C.c_long
        _lib.oracle_rng_new.restype = C.c_void_p
        for f in ("oracle_rng_free", "oracle_rng_mix", "oracle_rng_random_bits", "oracle_rng_random_elem"):
            getattr(_lib, f).argtypes = [C.c_void_p] + ([u32p] if f == "oracle_rng_mix" else
                                                         [C.c_size_t] if f == "oracle_rng_random_bits" else [])
        _lib.oracle_rng_random_bits.restype = C.c_uint32
        _lib.oracle_rng_random_elem.restype = C.c_uint32
        _lib.oracle_rng_random_ext_elem.argtypes = [C.c_void_p, u32p]
        _lib.oracle_rng_random_ext_elem.restype = None
        _lib.oracle_encode.restype = C.c_uint32
        _lib.oracle_decode.restype = C.c_uint32
        _lib.oracle_elem_pow.restype = C.c_uint32
        _lib.oracle_elem_pow.argtypes = [C.c_uint32, C.c_uint64]
        _lib.oracle_num_threads.restype = C.c_size_t
    return _lib


def ref_lib():
    """The reference's compiled poly_fp (checker only); None if it was never built."""
    global _ref
    if _ref is None and os.path.exists(REF_PATH):
        _ref = C.CDLL(REF_PATH)
    return _ref


def ptr(a):
    assert a.dtype == np.uint32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(u32p)


def sz(n):
    return C.c_size_t(int(n))


def encode(x):
    """Elem::new (plain integer -> Montgomery word)."""
    x = np.asarray(x, dtype=np.uint64) % P
    return ((x << np.uint64(32)) % np.uint64(P)).astype(np.uint32)


def decode(x):
    x = np.asarray(x, dtype=np.uint64)
    inv_r = pow(2**32, P - 2, P)
    return ((x * np.uint64(inv_r)) % np.uint64(P)).astype(np.uint32)


def rand_elems(rng, n):
    """Uniform canonical Montgomery words (any canonical word is a valid element)."""
    return (rng.integers(0, P, size=n, dtype=np.uint64)).astype(np.uint32)


# ---------------------------------------------------------------------------
# HAL ops (restatement of risc0/zkp/src/hal/cpu.rs)
def batch_expand_into_evaluate_ntt(out, inp, count, expand_bits):
    lib().oracle_batch_expand_into_evaluate_ntt(ptr(out), sz(out.size), ptr(inp), sz(inp.size), sz(count), sz(expand_bits))


def batch_interpolate_ntt(io, count):
    lib().oracle_batch_interpolate_ntt(ptr(io), sz(io.size), sz(count))


def batch_bit_reverse(io, count):
    lib().oracle_batch_bit_reverse(ptr(io), sz(io.size), sz(count))


def batch_evaluate_any(coeffs, poly_count, which, xs, out):
    lib().oracle_batch_evaluate_any(ptr(coeffs), sz(coeffs.size), sz(poly_count), ptr(which), ptr(xs),
                                    ptr(out), sz(which.size))


def zk_shift(io, poly_count):
    lib().oracle_zk_shift(ptr(io), sz(io.size), sz(poly_count))


def mix_poly_coeffs(out, mix_start, mix, inp, combos, input_size, count):
    lib().oracle_mix_poly_coeffs(ptr(out), sz(out.size // 4), ptr(mix_start), ptr(mix), ptr(inp), ptr(combos),
                                 sz(input_size), sz(count))


def eltwise_add_elem(out, a, b):
    lib().oracle_eltwise_add_elem(ptr(out), ptr(a), ptr(b), sz(out.size))


def eltwise_sum_extelem(out, inp):
    lib().oracle_eltwise_sum_extelem(ptr(out), sz(out.size), ptr(inp), sz(inp.size // 4))


def eltwise_zeroize_elem(io):
    lib().oracle_eltwise_zeroize_elem(ptr(io), sz(io.size))


def fri_fold(out, inp, mix):
    lib().oracle_fri_fold(ptr(out), sz(out.size), ptr(inp), ptr(mix))


def hash_rows(suite, out, matrix):
    rows = out.size // 8
    lib().oracle_hash_rows(C.c_int(suite), ptr(out), sz(rows), ptr(matrix), sz(matrix.size))


def hash_fold(suite, io, input_size, output_size):
    lib().oracle_hash_fold(C.c_int(suite), ptr(io), sz(input_size), sz(output_size))


def gather_sample(dst, src, idx, size, stride):
    lib().oracle_gather_sample(ptr(dst), ptr(src), sz(idx), sz(size), sz(stride))


def scatter(into, index, offsets, values):
    lib().oracle_scatter(ptr(into), ptr(index), sz(index.size), ptr(offsets), ptr(values))


def eltwise_copy_elem_slice(into, frm, from_rows, from_cols, from_offset, from_stride, into_offset, into_stride):
    lib().oracle_eltwise_copy_elem_slice(ptr(into), ptr(frm), sz(from_rows), sz(from_cols), sz(from_offset),
                                         sz(from_stride), sz(into_offset), sz(into_stride))


def rv32im_accum_finalize(accum, rows, cols, split, last_cycle):
    lib().oracle_rv32im_accum_finalize(ptr(accum), sz(rows), sz(cols), sz(split), sz(last_cycle))


def prefix_products(io):
    lib().oracle_prefix_products(ptr(io), sz(io.size // 4))


def combos_prepare(combos, coeff_u, combo_count, cycles, reg_sizes, reg_combo_ids, mix):
    lib().oracle_combos_prepare(ptr(combos), ptr(coeff_u), sz(combo_count), sz(cycles), ptr(reg_sizes),
                                ptr(reg_combo_ids), sz(reg_sizes.size), ptr(mix))


def combos_divide(combos, chunk_pows, chunk_begin, cycles):
    return lib().oracle_combos_divide(ptr(combos), sz(chunk_begin.size - 1), ptr(chunk_pows), ptr(chunk_begin),
                                      sz(cycles))


# primitives
def poseidon2_mix(cells):
    lib().oracle_poseidon2_mix(ptr(cells))


def hash_elems(suite, elems):
    out = np.zeros(8, np.uint32)
    lib().oracle_hash_elems(C.c_int(suite), ptr(elems), sz(elems.size), ptr(out))
    return out


def hash_ext_elems(suite, elems):
    out = np.zeros(8, np.uint32)
    lib().oracle_hash_ext_elems(C.c_int(suite), ptr(elems), sz(elems.size // 4), ptr(out))
    return out


def hash_pair(suite, a, b):
    out = np.zeros(8, np.uint32)
    lib().oracle_hash_pair(C.c_int(suite), ptr(a), ptr(b), ptr(out))
    return out


def sha256_bytes(data: bytes):
    out = np.zeros(8, np.uint32)
    buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    lib().oracle_sha256_bytes(buf, sz(len(data)), ptr(out))
    return out


def ext_mul(a, b):
    out = np.zeros(4, np.uint32)
    lib().oracle_ext_mul(ptr(a), ptr(b), ptr(out))
    return out


def ext_inv(a):
    out = np.zeros(4, np.uint32)
    lib().oracle_ext_inv(ptr(a), ptr(out))
    return out


def elem_pow(x, n):
    return lib().oracle_elem_pow(C.c_uint32(int(x)), C.c_uint64(int(n)))


class Rng:
    def __init__(self, suite):
        self.h = lib().oracle_rng_new(C.c_int(suite))

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_rng_free(self.h)

    def mix(self, digest):
        d = np.ascontiguousarray(digest, dtype=np.uint32)
        lib().oracle_rng_mix(self.h, ptr(d))

    def random_bits(self, bits):
        return lib().oracle_rng_random_bits(self.h, sz(bits))

    def random_elem(self):
        return lib().oracle_rng_random_elem(self.h)

    def random_ext_elem(self):
        out = np.zeros(4, np.uint32)
        lib().oracle_rng_random_ext_elem(self.h, ptr(out))
        return out


# ---------------------------------------------------------------------------
# circuits + prover
class Circuit(C.Structure):
    _fields_ = [("taps", u32p), ("n_taps", C.c_size_t), ("combo_taps", u32p), ("combo_begin", u32p),
                ("combos_count", C.c_size_t), ("group_begin", u32p), ("n_groups", C.c_size_t),
                ("poly_mix_powers", u32p), ("n_poly_mix", C.c_size_t), ("circuit_info", C.POINTER(C.c_uint8)),
                ("mix_size", C.c_size_t), ("output_size", C.c_size_t), ("eval_args", C.POINTER(C.c_int32)),
                ("n_eval_args", C.c_size_t), ("poly_fp", C.c_void_p)]


def load_circuit_json(name):
    with open(os.path.join(CIRCUITS, name + ".taps.json")) as f:
        return json.load(f)


def make_circuit(name):
    """Returns (Circuit struct, keepalive). poly_fp = the reference's compiled C++ when built."""
    d = load_circuit_json(name)
    keep = {}
    keep["taps"] = np.array(d["taps"], dtype=np.uint32).reshape(-1)
    keep["combo_taps"] = np.array(d["combo_taps"], dtype=np.uint32)
    keep["combo_begin"] = np.array(d["combo_begin"], dtype=np.uint32)
    keep["group_begin"] = np.array(d["group_begin"], dtype=np.uint32)
    keep["pows"] = np.array(d["poly_mix_powers"], dtype=np.uint32)
    keep["info"] = (C.c_uint8 * 16).from_buffer_copy(d["circuit_info"].encode())
    amap = {"accum": 0, "code": 1, "data": 2, "mix": -1, "global": -2}
    keep["args"] = np.array([amap[a] for a in d["eval_args"]], dtype=np.int32)
    fp = None
    r = ref_lib()
    if r is not None:
        fp = C.cast(getattr(r, f"ref_{name}_poly_fp"), C.c_void_p).value
    c = Circuit(ptr(keep["taps"]), len(d["taps"]), ptr(keep["combo_taps"]), ptr(keep["combo_begin"]),
                d["combos_count"], ptr(keep["group_begin"]), len(d["group_names"]), ptr(keep["pows"]),
                len(d["poly_mix_powers"]), C.cast(keep["info"], C.POINTER(C.c_uint8)), d["mix_size"],
                d["output_size"], keep["args"].ctypes.data_as(C.POINTER(C.c_int32)), len(d["eval_args"]), fp)
    return c, keep, d


def _check(err):
    if err:
        msg = C.cast(err, C.c_char_p).value.decode()
        raise RuntimeError(msg)


def eval_check(name, check, groups, mix, glob, poly_mix, po2):
    c, keep, _ = make_circuit(name)
    arr = (u32p * len(groups))(*[ptr(g) for g in groups])
    _check(lib().oracle_eval_check(C.byref(c), ptr(check), arr, ptr(mix), ptr(glob), ptr(poly_mix),
                                   C.c_uint32(po2)))


def splitmix_fill(seed, n, start=0):
    """The synthetic words r0hip_fill_uniform writes (splitmix64 of (seed, index) mod p),
    for indices [start, start + n)."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (np.arange(start, start + n, dtype=np.uint64) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return (z % np.uint64(P)).astype(np.uint32)


def eval_check_sampled(name, group_seeds, mix, glob, poly_mix, po2, cycles):
    """eval_check over groups filled by r0hip_fill_uniform(group_seeds[g]) (group ids:
    accum 0, code 1, data 2), evaluated only at `cycles`; returns (len(cycles), 4)."""
    c, keep, _ = make_circuit(name)
    seeds = np.ascontiguousarray(group_seeds, dtype=np.uint64)
    cyc = np.ascontiguousarray(cycles, dtype=np.uint64)
    out = np.zeros(4 * cyc.size, np.uint32)
    u64p = C.POINTER(C.c_uint64)
    _check(lib().oracle_eval_check_sampled(C.byref(c), seeds.ctypes.data_as(u64p), ptr(mix), ptr(glob),
                                           ptr(poly_mix), C.c_uint32(po2), cyc.ctypes.data_as(u64p),
                                           sz(cyc.size), ptr(out)))
    return out.reshape(-1, 4)


def prove_segment(name, suite, po2, code, data, accum, glob, version=None):
    c, keep, d = make_circuit(name)
    glob = glob.copy()
    cap = 1 << 24
    seal = np.zeros(cap, np.uint32)
    n = C.c_size_t(0)
    mix = np.zeros(d["mix_size"], np.uint32)
    _check(lib().oracle_prove_segment(C.byref(c), C.c_int(suite), C.c_uint32(po2), ptr(code), ptr(data),
                                      ptr(accum), ptr(glob), C.c_int(version is not None),
                                      C.c_uint32(version or 0), ptr(seal), sz(cap), C.byref(n), ptr(mix)))
    return seal[: n.value].copy(), mix, glob


def poly_fp_at_taps(name, tap_values, mix, glob, poly_mix):
    """the reference's compiled poly_fp at a cycle whose taps read tap_values (one base-field
    Montgomery word per tap, tap order): the mixed constraint sum, 4 words"""
    c, keep, _ = make_circuit(name)
    out = np.zeros(4, np.uint32)
    _check(lib().oracle_poly_fp_at_taps(C.byref(c), ptr(np.ascontiguousarray(tap_values, np.uint32)), ptr(mix),
                                        ptr(glob), ptr(np.ascontiguousarray(poly_mix, np.uint32)), ptr(out)))
    return out


ACCUM_CB = C.CFUNCTYPE(C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_void_p)


def prove_segment_cb(name, suite, po2, code, data, glob, fill_accum, accum_words, version=None):
    """oracle_prove_segment_cb: the prover with the accum group filled by
    fill_accum(mix) -> accum (numpy uint32, accum_words) once the mix is drawn, as prove_core
    runs WitnessGenerator::accum between the data commit and the accum commit."""
    c, keep, d = make_circuit(name)
    glob = glob.copy()
    cap = 1 << 24
    seal = np.zeros(cap, np.uint32)
    n = C.c_size_t(0)
    mix = np.zeros(d["mix_size"], np.uint32)
    accum = np.zeros(accum_words, np.uint32)
    err = []

    def cb(mix_p, acc_p, _ctx):
        try:
            m = np.ctypeslib.as_array(mix_p, shape=(d["mix_size"],)).copy()
            a = np.ascontiguousarray(fill_accum(m), dtype=np.uint32)
            assert a.size == accum_words
            np.ctypeslib.as_array(acc_p, shape=(accum_words,))[:] = a
            return None
        except Exception as e:  # reported through the prover's error (the buffer outlives the call)
            err.append(e)
            msg = C.create_string_buffer(str(e).encode())
            err.append(msg)
            return C.cast(msg, C.c_void_p).value

    fcb = ACCUM_CB(cb)
    f = lib().oracle_prove_segment_cb
    f.restype = C.c_void_p
    e = f(C.byref(c), C.c_int(suite), C.c_uint32(po2), ptr(code), ptr(data), ptr(accum), fcb, None, ptr(glob),
          C.c_int(version is not None), C.c_uint32(version or 0), ptr(seal), sz(cap), C.byref(n), ptr(mix))
    if err:
        raise err[0]
    _check(e)
    return seal[: n.value].copy(), mix, glob, accum


def num_threads():
    return lib().oracle_num_threads()


def op_times(reset=True):
    """{hal_op: (seconds, calls)} of the oracle proofs since the last reset (the CPU
    baseline's per-op breakdown)."""
    f = lib().oracle_op_times
    f.restype = C.c_size_t
    f.argtypes = [C.c_char_p, C.c_size_t, C.c_int]
    buf = C.create_string_buffer(f(None, 0, 0) + 1)
    f(buf, len(buf), int(reset))
    out = {}
    for item in buf.value.decode().split(";"):
        if item:
            k, v = item.split("=")
            t, n = v.split(":")
            out[k] = (float(t), int(n))
    return out
