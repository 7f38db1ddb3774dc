"""ctypes binding of the per-op driver (integration/hal_prover.h, libr0hip_halprover.so): the
reference prover over ONLY the per-op r0hip_* symbols, what a Rust HipHal behind
risc0_zkp::hal::Hal delivers. Used by tests/ (seal parity with the fused prover) and by
bench.py's per_op_abi leg. Not part of the product; no oracle."""
import ctypes as C
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "lib", "libr0hip_halprover.so")
_lib = None


class Taps(C.Structure):
    """struct halp_taps"""
    _fields_ = [("taps", C.c_void_p), ("n_taps", C.c_size_t), ("combo_taps", C.c_void_p), ("combo_begin", C.c_void_p),
                ("combos_count", C.c_size_t), ("group_begin", C.c_void_p), ("group_sizes", C.c_void_p),
                ("circuit_info", C.c_char_p), ("mix_size", C.c_size_t), ("output_size", C.c_size_t)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is not built (make -C integration)")
        import risc0_amd  # noqa: F401  (loads libr0hip.so first)
        _lib = C.CDLL(LIB_PATH)
        vp, sz = C.c_void_p, C.c_size_t
        _lib.halp_prove_segment.restype = vp
        _lib.halp_prove_segment.argtypes = [C.c_char_p, vp, C.c_int, C.c_uint32, vp, vp, vp, vp, C.c_int, sz, vp, sz,
                                            C.c_int, C.c_uint32, vp, sz, C.POINTER(sz), vp]
        _lib.halp_prove_trace.restype = vp
        _lib.halp_prove_trace.argtypes = [vp, C.c_int, C.c_uint32, C.c_uint32, vp, vp, sz, vp, vp, vp, vp, sz, vp, sz,
                                          C.POINTER(sz), vp]
        _lib.halp_last_profile.restype = vp
        _lib.halp_last_profile.argtypes = [C.c_char_p, sz]
    return _lib


class CircuitTaps:
    """a circuit's TapSet from risc0_amd/circuits/<c>.taps.json, kept alive with its struct"""

    def __init__(self, circuit):
        with open(os.path.join(ROOT, "risc0_amd", "circuits", circuit + ".taps.json")) as f:
            d = json.load(f)
        u = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.uint32).reshape(-1))
        self.arrays = [u(d["taps"]), u(d["combo_taps"]), u(d["combo_begin"]), u(d["group_begin"]), u(d["group_sizes"])]
        self.info = d["circuit_info"].encode()
        self.mix_size = d["mix_size"]
        t, ct, cb, gb, gs = self.arrays
        self.struct = Taps(t.ctypes.data, len(d["taps"]), ct.ctypes.data, cb.ctypes.data, d["combos_count"], gb.ctypes.data,
                           gs.ctypes.data, self.info, d["mix_size"], d["output_size"])


def _check(err):
    if err:
        msg = C.cast(err, C.c_char_p).value.decode()
        C.CDLL(None).free(C.c_void_p(err))
        from risc0_amd import R0HipError
        raise R0HipError(msg)


def last_profile():
    buf = C.create_string_buffer(4096)
    lib().halp_last_profile(buf, 4096)
    out = {}
    for kv in buf.value.decode().split(";"):
        if "=" in kv:
            k, v = kv.split("=")
            out[k] = out.get(k, 0.0) + float(v)
    return out


def prove_segment(hal, circuit, po2, code, data, accum, glob, accum_mode=0, work_cycles=0, bigint_records=None,
                  version=None, seal_cap=1 << 22):
    """halp_prove_segment over device buffers (risc0_amd Buffers); returns (seal, mix)"""
    from risc0_amd.hal import bigint_backs
    taps = CircuitTaps(circuit)
    backs = bigint_backs(bigint_records)
    seal = np.zeros(seal_cap, np.uint32)
    mix = np.zeros(taps.mix_size, np.uint32)
    n = C.c_size_t(0)
    _check(lib().halp_prove_segment(circuit.encode(), C.addressof(taps.struct), hal.suite, po2, code.ptr, data.ptr,
                                    accum.ptr, glob.ptr, accum_mode, work_cycles,
                                    None if backs is None else C.cast(backs, C.c_void_p).value,
                                    0 if backs is None else len(backs), int(version is not None), version or 0,
                                    seal.ctypes.data, seal_cap, C.byref(n), mix.ctypes.data))
    return seal[: n.value].copy(), mix


def prove_trace(hal, po2, job, seal_cap=1 << 22):
    """halp_prove_trace over a risc0_amd.TraceJob (its host arrays); returns (seal, mix)"""
    taps = CircuitTaps("rv32im")
    t = job.struct
    seal = np.zeros(seal_cap, np.uint32)
    mix = np.zeros(taps.mix_size, np.uint32)
    n = C.c_size_t(0)
    backs = job.backs
    _check(lib().halp_prove_trace(C.addressof(taps.struct), hal.suite, po2, t.mode, t.h_global, t.h_inj_index, t.inj_rows,
                                  t.h_inj_offsets, t.h_inj_values, C.addressof(t.preflight),
                                  None if backs is None else C.cast(backs, C.c_void_p).value,
                                  0 if backs is None else len(backs), seal.ctypes.data, seal_cap, C.byref(n),
                                  mix.ctypes.data))
    return seal[: n.value].copy(), mix
