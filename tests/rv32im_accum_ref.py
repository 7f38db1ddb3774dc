"""The reference's rv32im accumulation, compiled from /root/reference by oracle/Makefile into
oracle/_ref/libref_rv32im_accum.so (test infrastructure only): risc0_circuit_rv32im_cpu_accum
(rv32im-sys/kernels/cxx/ffi.cpp:313-368, all three phases) and ref_rv32im_accum_phase1
(oracle/ref_rv32im_glue.cpp: the same stepAccum, phase 1 alone)."""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_ref", "libref_rv32im_accum.so")
P = 15 * 2**27 + 1
INVALID = 0xFFFFFFFF  # Fp::invalid() (risc0/sys/cxx/fp.h)
DATA_COLS, ACCUM_COLS, GLOBAL_WORDS, MIX_WORDS = 211, 103, 90, 36


class Buffer(C.Structure):
    """risc0::Buffer<isGlobal> (rv32im-sys/kernels/cxx/buffers.h)"""
    _fields_ = [("buf", C.c_void_p), ("rows", C.c_size_t), ("cols", C.c_size_t), ("checked", C.c_bool)]


class AccumBuffers(C.Structure):
    """witgen.h: data, accum, global, mix"""
    _fields_ = [("data", Buffer), ("accum", Buffer), ("glob", Buffer), ("mix", Buffer)]


class PreflightTrace(C.Structure):
    """preflight.h (unused by the accumulation step; zeroed)"""
    _fields_ = [("cycles", C.c_void_p), ("txns", C.c_void_p), ("bigintBytes", C.c_void_p), ("txnsLen", C.c_uint32),
                ("bigintBytesLen", C.c_uint32), ("tableSplitCycle", C.c_uint32)]


def available():
    return os.path.exists(LIB)


def _lib():
    lib = C.CDLL(LIB)
    lib.risc0_circuit_rv32im_cpu_accum.restype = C.c_void_p
    lib.risc0_circuit_rv32im_cpu_accum.argtypes = [C.POINTER(AccumBuffers), C.POINTER(PreflightTrace), C.c_uint32]
    lib.ref_rv32im_accum_phase1.restype = C.c_void_p
    lib.ref_rv32im_accum_phase1.argtypes = [C.POINTER(AccumBuffers), C.c_uint32]
    return lib


def _buffers(data, accum, glob, mix, rows):
    return AccumBuffers(Buffer(data.ctypes.data, rows, DATA_COLS, True), Buffer(accum.ctypes.data, rows, ACCUM_COLS, True),
                        Buffer(glob.ctypes.data, 1, GLOBAL_WORDS, True), Buffer(mix.ctypes.data, 1, MIX_WORDS, True))


def _check(err):
    if err:
        raise RuntimeError(C.cast(err, C.c_char_p).value.decode())


def accum(data, glob, mix, rows, last_cycle, phase1_only=False, accum_init=None):
    """Accum group (column-major, ACCUM_COLS x rows, raw Montgomery words) the reference
    computes from `data` (DATA_COLS x rows), starting from an all-INVALID buffer as the
    prover allocates it, or from `accum_init` (e.g. with the BigInt states injected, as
    WitnessGenerator::accum hands it to step_accum, witgen/mod.rs:187-215)."""
    data = np.ascontiguousarray(data, np.uint32)
    glob = np.ascontiguousarray(glob, np.uint32)
    mix = np.ascontiguousarray(mix, np.uint32)
    if accum_init is None:
        out = np.full(ACCUM_COLS * rows, INVALID, np.uint32)
    else:
        out = np.array(accum_init, dtype=np.uint32).reshape(-1)
        assert out.size == ACCUM_COLS * rows
    bufs = _buffers(data, out, glob, mix, rows)
    lib = _lib()
    if phase1_only:
        _check(lib.ref_rv32im_accum_phase1(C.byref(bufs), last_cycle))
    else:
        pf = PreflightTrace()
        _check(lib.risc0_circuit_rv32im_cpu_accum(C.byref(bufs), C.byref(pf), last_cycle))
    return out
