"""The reference's rv32im witness generator, compiled from /root/reference by oracle/Makefile
into oracle/_ref/libref_rv32im_accum.so (test infrastructure only):
risc0_circuit_rv32im_cpu_witgen (rv32im-sys/kernels/cxx/ffi.cpp:267-308) over the buffers
WitnessGenerator::hal_generate_witness hands it (witgen/mod.rs:135-176): the global vector
and the data group filled with Val::INVALID, the injector scattered into data."""
import ctypes as C
import json
import os

import numpy as np

import bigint_accum as BA
import rv32im_accum_ref as RA
import rv32im_trace as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = T.P
INVALID = RA.INVALID
DATA_COLS, GLOBAL_WORDS = RA.DATA_COLS, RA.GLOBAL_WORDS
MODE_PARALLEL, MODE_SEQ_FORWARD, MODE_SEQ_REVERSE = 0, 1, 2


class ExecBuffers(C.Structure):
    """witgen.h:36-39"""
    _fields_ = [("glob", RA.Buffer), ("data", RA.Buffer)]


def layout():
    return T.layout()


encode = T.encode


def inputs(trace, lay=None):
    """(data, global, cycles, txns) as hal_generate_witness prepares them: data all INVALID
    with the injector scattered in, globals INVALID except build_global_vec's words"""
    lay = lay or layout()
    rows = 1 << trace.po2
    data = np.full(DATA_COLS * rows, INVALID, np.uint32)
    r, c, v = trace.injector(lay)
    data[c.astype(np.int64) * rows + r] = encode(v)
    g = trace.global_values(lay)
    glob = np.array([INVALID if x is None else int(encode(x)) for x in g], np.uint32)
    cyc, tx = trace.arrays()
    return data, glob, cyc, tx


def global_words(trace, lay=None):
    """build_global_vec as Montgomery words (INVALID where unset)"""
    return trace.global_words(lay)


def injector_arrays(trace, lay=None):
    """the Injector (witgen/mod.rs:329-378) as hal.scatter takes it"""
    return trace.injector_arrays(lay)


def prove_from_trace(trace, suite, oracle, mode=MODE_SEQ_FORWARD, data_patch=()):
    """the reference's prove_core from a preflight on the CPU (SegmentProverImpl::prove_core,
    prove/hal/mod.rs:143-224): the compiled reference witgen, zeroize, the oracle prover with
    the compiled reference accumulation run on the drawn mix (oracle_prove_segment_cb), INVALID
    accum words zeroized. data_patch: (offset, word) pairs set in the data group after the
    injector (extra injector entries). Returns (seal, mix, data, global, accum)."""
    rows = 1 << trace.po2
    data, glob, cyc, tx = inputs(trace)
    for off, word in data_patch:
        data[off] = word
    d, g = run(data, glob, cyc, tx, trace.table_split_cycle, rows, mode, trace.bigint_array())
    d = np.where(d == INVALID, 0, d).astype(np.uint32)
    g = np.where(g == INVALID, 0, g).astype(np.uint32)
    code = np.zeros(rows, np.uint32)

    records = trace.bigint_records()

    def fill(mix):
        init = None
        if records:  # WitnessGenerator::accum's BigIntAccum injection (witgen/mod.rs:187-205)
            init = BA.inject(np.full(RA.ACCUM_COLS * rows, INVALID, np.uint32), rows, mix, records)
        acc = RA.accum(d, g, mix, rows, rows, accum_init=init)
        return np.where(acc == INVALID, 0, acc).astype(np.uint32)
    seal, mix, _, acc = oracle.prove_segment_cb("rv32im", suite, trace.po2, code, d, g, fill, RA.ACCUM_COLS * rows,
                                                version=2)
    return seal, mix, d, g, acc


def witgen(trace, mode=MODE_SEQ_FORWARD, lay=None):
    """(data, global) after the reference's witness generation; raises RuntimeError with the
    reference's message when it throws"""
    data, glob, cyc, tx = inputs(trace, lay)
    return run(data, glob, cyc, tx, trace.table_split_cycle, 1 << trace.po2, mode, trace.bigint_array())


def run(data, glob, cyc, tx, split, rows, mode=MODE_SEQ_FORWARD, bigint=None):
    data = np.array(data, np.uint32)
    glob = np.array(glob, np.uint32)
    cyc = np.array(cyc)  # the reference advances txnIdx in place
    tx = np.ascontiguousarray(tx)
    n_bigint = 0 if bigint is None else len(bigint)
    bigint = np.concatenate([np.zeros(0, np.uint8) if bigint is None else np.asarray(bigint, np.uint8),
                             np.zeros(16, np.uint8)])
    lib = C.CDLL(RA.LIB)
    f = lib.risc0_circuit_rv32im_cpu_witgen
    f.restype = C.c_void_p
    f.argtypes = [C.c_uint32, C.POINTER(ExecBuffers), C.POINTER(RA.PreflightTrace), C.c_uint32]
    bufs = ExecBuffers(RA.Buffer(glob.ctypes.data, 1, GLOBAL_WORDS, True), RA.Buffer(data.ctypes.data, rows, DATA_COLS, True))
    pf = RA.PreflightTrace(cyc.ctypes.data, tx.ctypes.data, bigint.ctypes.data, len(tx), n_bigint, split)
    err = f(mode, C.byref(bufs), C.byref(pf), rows)
    if err:
        raise RuntimeError(C.cast(err, C.c_char_p).value.decode())
    return data, glob
