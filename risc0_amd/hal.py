"""Python mirror of the risc0_zkp `Hal` trait over the r0hip C ABI.

`HipHal` exposes the same method names and argument meanings as
risc0/zkp/src/hal/mod.rs:55-258 (buffers are device allocations of u32 words:
Elem = 1 word, ExtElem = 4, Digest = 8), so the parity tests read like the
reference's DualHal tests (risc0/zkp/src/hal/mod.rs:319-616). It is a thin
ctypes layer: every operation runs in libr0hip.so on the GPU. There is no CPU
fallback; a missing library or device raises.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# R0HIP_LIB selects an alternative build of the same library (tools/ experiments only)
LIB_PATH = os.environ.get("R0HIP_LIB") or os.path.join(_HERE, "lib", "libr0hip.so")

POSEIDON2, SHA256, POSEIDON254 = 0, 1, 2
SUITES = {"poseidon2": POSEIDON2, "sha-256": SHA256, "poseidon_254": POSEIDON254, "poseidon254": POSEIDON254}

_lib = None
u32p = C.POINTER(C.c_uint32)


class R0HipError(RuntimeError):
    pass


def lib():
    """Load libr0hip.so (built by __graft_entry__.build()); raise if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise R0HipError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(LIB_PATH)
        _declare(L)
        _lib = L
    return _lib


def _declare(L):
    sz = C.c_size_t
    vp = C.c_void_p
    sig = {
        "r0hip_init": [C.c_int],
        "r0hip_device_info": [C.c_char_p, sz, C.POINTER(C.c_uint64)],
        "r0hip_alloc": [C.POINTER(vp), sz],
        "r0hip_free": [vp],
        "r0hip_memset32": [vp, C.c_uint32, sz],
        "r0hip_memcpy_h2d": [vp, vp, sz],
        "r0hip_memcpy_d2h": [vp, vp, sz],
        "r0hip_memcpy_d2d": [vp, vp, sz],
        "r0hip_host_alloc": [C.POINTER(vp), sz],
        "r0hip_host_free": [vp],
        "r0hip_memcpy_d2h_start": [vp, vp, sz, C.POINTER(vp)],
        "r0hip_copy_finish": [vp, C.c_int, C.POINTER(C.c_int)],
        "r0hip_fill_uniform": [vp, sz, C.c_uint64],
        "r0hip_rv32im_accum_finalize": [vp, sz, sz, sz],
        "r0hip_rv32im_accum": [vp, vp, vp, vp, sz, sz, sz],
        "r0hip_recursion_accum": [vp, vp, vp, vp, vp, sz, sz],
        "r0hip_prove_segments": [C.c_char_p, C.c_int, C.c_uint32, C.c_int, C.c_uint32, C.c_void_p, sz, C.c_uint32],
        "r0hip_prove_trace_segments": [C.c_int, C.c_uint32, C.c_void_p, sz, C.c_uint32, C.c_int],
        "r0hip_verify_seal": [C.c_char_p, C.c_int, u32p, sz, u32p, sz, u32p, C.POINTER(C.c_uint32)],
        "r0hip_testing_verify_seal_structure": [C.c_char_p, C.c_int, u32p, sz, C.POINTER(C.c_uint32)],
        "r0hip_poly_ext": [C.c_char_p, u32p, u32p, u32p, u32p, u32p],
        "r0hip_synchronize": [],
        "r0hip_batch_expand_into_evaluate_ntt": [vp, vp, sz, C.c_uint32, C.c_uint32],
        "r0hip_batch_interpolate_ntt": [vp, sz, C.c_uint32],
        "r0hip_zk_shift": [vp, sz, C.c_uint32],
        "r0hip_batch_bit_reverse": [vp, sz, C.c_uint32],
        "r0hip_batch_evaluate_any": [vp, vp, sz, C.c_uint32, vp, vp, sz],
        "r0hip_mix_poly_coeffs": [vp, vp, u32p, u32p, u32p, sz, sz],
        "r0hip_fri_fold": [vp, vp, u32p, sz],
        "r0hip_combos_prepare": [vp, u32p, sz, sz, u32p, u32p, sz, u32p],
        "r0hip_poly_divide": [vp, sz, u32p, u32p],
        "r0hip_combos_divide": [vp, sz, u32p, u32p, sz, C.POINTER(C.c_int64)],
        "r0hip_eltwise_add_elem": [vp, vp, vp, sz],
        "r0hip_eltwise_copy_elem": [vp, vp, sz],
        "r0hip_eltwise_zeroize_elem": [vp, sz],
        "r0hip_eltwise_sum_extelem": [vp, vp, sz, sz],
        "r0hip_eltwise_copy_elem_slice": [vp, vp, sz, sz, sz, sz, sz, sz],
        "r0hip_gather_sample": [vp, vp, sz, sz, sz],
        "r0hip_gather_sample_host": [vp, vp, sz, sz, sz],
        "r0hip_scatter": [vp, vp, vp, vp, sz],
        "r0hip_prefix_products": [vp, sz],
        "r0hip_hash_rows": [C.c_int, vp, vp, sz, sz],
        "r0hip_hash_fold": [C.c_int, vp, sz, sz],
        "r0hip_merkle_tree": [C.c_int, vp, vp, sz, sz],
        "r0hip_eval_check": [C.c_char_p, vp, C.POINTER(vp), vp, vp, u32p, C.c_uint32],
        "r0hip_prove_segment": [C.c_char_p, C.c_int, C.c_uint32, vp, vp, vp, vp, C.c_int, C.c_uint32, u32p, sz,
                                C.POINTER(sz), u32p],
        "r0hip_prove_segment_accum": [C.c_char_p, C.c_int, C.c_uint32, vp, vp, vp, sz, vp, sz, vp, C.c_int,
                                      C.c_uint32, u32p, sz, C.POINTER(sz), u32p],
        "r0hip_rv32im_bigint_accum_states": [u32p, vp, sz, sz, u32p],
        "r0hip_recursion_witgen": [vp, vp, vp, sz, u32p, sz, u32p, sz, u32p, sz],
        "r0hip_rv32im_witgen": [C.c_uint32, vp, vp, C.c_uint32],
        "r0hip_prove_segment_trace_resident": [C.c_int, C.c_uint32, C.c_uint32, vp, vp, sz, vp, vp, vp, vp, sz,
                                               u32p, sz, C.POINTER(sz), u32p],
        "r0hip_prove_segment_trace": [C.c_int, C.c_uint32, C.c_uint32, u32p, u32p, sz, u32p, u32p, vp, vp, sz, u32p,
                                      sz, C.POINTER(sz), u32p],
        "r0hip_prove_recursion": [C.c_int, C.c_uint32, vp, u32p, sz, u32p, sz, u32p, sz, C.c_uint64, u32p, sz,
                                  C.POINTER(sz), u32p],
        "r0hip_rv32im_bigint_accum_inject": [vp, sz, u32p, vp, sz],
        "r0hip_last_profile": [C.c_char_p, sz],
        "r0hip_set_kernel_timing": [C.c_int],
        "r0hip_kernel_times": [C.c_char_p, sz],
        "r0hip_mem_stats": [C.POINTER(C.c_uint64)],
        "r0hip_mem_reset_peak": [],
        "r0hip_trim": [],
    }
    for name, args in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = C.c_void_p
    L.r0hip_free_error.argtypes = [C.c_void_p]
    L.r0hip_free_error.restype = None


def check(err):
    if err:
        msg = C.cast(err, C.c_char_p).value.decode()
        lib().r0hip_free_error(err)
        raise R0HipError(msg)


def exported_symbols():
    """Every r0hip_* entry point declared in include/r0hip.h."""
    hdr = os.path.join(os.path.dirname(_HERE), "include", "r0hip.h")
    import re
    return sorted(set(re.findall(r"\b(r0hip_\w+)\s*\(", open(hdr).read())))


def _h(a):
    a = np.ascontiguousarray(a, dtype=np.uint32)
    return a, a.ctypes.data_as(u32p)


class Buffer:
    """A device allocation of `size` elements of `words` u32 each (hal/mod.rs:39-53)."""

    def __init__(self, hal, name, size, words=1, ptr=None, owner=True):
        self.hal, self.name, self.size, self.words = hal, name, size, words
        self._owner = owner
        if ptr is None:
            p = C.c_void_p()
            check(lib().r0hip_alloc(C.byref(p), max(1, size * words) * 4))
            ptr = p.value
        self.ptr = ptr

    @property
    def nwords(self):
        return self.size * self.words

    def slice(self, offset, size):
        return Buffer(self.hal, self.name, size, self.words, self.ptr + offset * self.words * 4, owner=False)

    def to_numpy(self):
        out = np.empty(self.nwords, dtype=np.uint32)
        if self.nwords:
            check(lib().r0hip_memcpy_d2h(out.ctypes.data, self.ptr, self.nwords * 4))
        return out

    def copy_from(self, arr):
        a = np.ascontiguousarray(arr, dtype=np.uint32).reshape(-1)
        assert a.size == self.nwords, (a.size, self.nwords)
        if a.size:
            check(lib().r0hip_memcpy_h2d(self.ptr, a.ctypes.data, a.size * 4))

    def free(self):
        if self._owner and self.ptr:
            check(lib().r0hip_free(self.ptr))
        self.ptr = 0

    def __del__(self):
        try:
            if self._owner and self.ptr and _lib is not None:
                _lib.r0hip_free(self.ptr)
        except Exception:
            pass


def _lg(n):
    l = int(n).bit_length() - 1
    assert 1 << l == n, f"{n} is not a power of two"
    return l


class HipHal:
    """risc0_zkp::hal::Hal on MI355X (one instance per process/device)."""

    EXT_SIZE = 4
    CHECK_SIZE = 16

    def __init__(self, hashfn="poseidon2", device=0):
        self.suite = SUITES[hashfn] if isinstance(hashfn, str) else int(hashfn)
        check(lib().r0hip_init(device))

    # ---- allocation (hal/mod.rs:67-100) ----
    def alloc_elem(self, name, size):
        return Buffer(self, name, size, 1)

    def alloc_extelem(self, name, size):
        return Buffer(self, name, size, 4)

    def alloc_digest(self, name, size):
        return Buffer(self, name, size, 8)

    def alloc_u32(self, name, size):
        return Buffer(self, name, size, 1)

    def alloc_elem_init(self, name, size, value):
        b = self.alloc_elem(name, size)
        check(lib().r0hip_memset32(b.ptr, value, size))
        return b

    def alloc_extelem_zeroed(self, name, size):
        b = self.alloc_extelem(name, size)
        check(lib().r0hip_memset32(b.ptr, 0, size * 4))
        return b

    def copy_from_elem(self, name, arr):
        a = np.ascontiguousarray(arr, dtype=np.uint32).reshape(-1)
        b = self.alloc_elem(name, a.size)
        b.copy_from(a)
        return b

    copy_from_u32 = copy_from_elem

    def copy_from_extelem(self, name, arr):
        a = np.ascontiguousarray(arr, dtype=np.uint32).reshape(-1)
        b = self.alloc_extelem(name, a.size // 4)
        b.copy_from(a)
        return b

    def copy_from_digest(self, name, arr):
        a = np.ascontiguousarray(arr, dtype=np.uint32).reshape(-1)
        b = self.alloc_digest(name, a.size // 8)
        b.copy_from(a)
        return b

    def has_unified_memory(self):
        return False

    # ---- HAL ops ----
    def batch_expand_into_evaluate_ntt(self, output, input, count, expand_bits):
        out_size = output.size // count
        check(lib().r0hip_batch_expand_into_evaluate_ntt(output.ptr, input.ptr, count, _lg(out_size), expand_bits))

    def batch_interpolate_ntt(self, io, count):
        check(lib().r0hip_batch_interpolate_ntt(io.ptr, count, _lg(io.size // count)))

    def batch_bit_reverse(self, io, count):
        check(lib().r0hip_batch_bit_reverse(io.ptr, count, _lg(io.size // count)))

    def zk_shift(self, io, count):
        check(lib().r0hip_zk_shift(io.ptr, count, _lg(io.size // count)))

    def batch_evaluate_any(self, coeffs, poly_count, which, xs, out):
        check(lib().r0hip_batch_evaluate_any(out.ptr, coeffs.ptr, poly_count, _lg(coeffs.size // poly_count),
                                             which.ptr, xs.ptr, which.size))

    def mix_poly_coeffs(self, out, mix_start, mix, input, combos, input_size, count):
        cb, cp = _h(combos)
        ms, msp = _h(mix_start)
        mx, mxp = _h(mix)
        check(lib().r0hip_mix_poly_coeffs(out.ptr, input.ptr, cp, msp, mxp, input_size, count))

    def eltwise_add_elem(self, output, input1, input2):
        assert output.size == input1.size == input2.size
        check(lib().r0hip_eltwise_add_elem(output.ptr, input1.ptr, input2.ptr, output.size))

    def eltwise_sum_extelem(self, output, input):
        count = output.size // 4
        check(lib().r0hip_eltwise_sum_extelem(output.ptr, input.ptr, input.size // count, count))

    def eltwise_copy_elem(self, output, input):
        assert output.size == input.size
        check(lib().r0hip_eltwise_copy_elem(output.ptr, input.ptr, output.size))

    def eltwise_copy_elem_slice(self, into, frm, from_rows, from_cols, from_offset, from_stride, into_offset,
                                into_stride):
        src = self.copy_from_elem("from", frm)
        check(lib().r0hip_eltwise_copy_elem_slice(into.ptr, src.ptr, from_rows, from_cols, from_offset, from_stride,
                                                  into_offset, into_stride))

    def eltwise_zeroize_elem(self, elems):
        check(lib().r0hip_eltwise_zeroize_elem(elems.ptr, elems.size))

    def fri_fold(self, output, input, mix):
        m, mp = _h(mix)
        check(lib().r0hip_fri_fold(output.ptr, input.ptr, mp, output.size // 4))

    def hash_rows(self, output, matrix):
        rows = output.size
        check(lib().r0hip_hash_rows(self.suite, output.ptr, matrix.ptr, rows, matrix.size // rows))

    def hash_fold(self, io, input_size, output_size):
        check(lib().r0hip_hash_fold(self.suite, io.ptr, input_size, output_size))

    def merkle_tree(self, nodes, matrix, rows):
        """nodes (2*rows digests) <- leaves and every layer (r0hip_merkle_tree)"""
        check(lib().r0hip_merkle_tree(self.suite, nodes.ptr, matrix.ptr, rows, matrix.size // rows))

    def gather_sample(self, dst, src, idx, size, stride):
        check(lib().r0hip_gather_sample(dst.ptr, src.ptr, idx, size, stride))

    def gather_sample_host(self, src, idx, size, stride):
        """src[idx + i*stride], i < size, as a host array (r0hip_gather_sample_host)"""
        out = np.zeros(size, np.uint32)
        check(lib().r0hip_gather_sample_host(out.ctypes.data, src.ptr, idx, size, stride))
        return out

    def scatter(self, into, index, offsets, values):
        index = np.asarray(index, dtype=np.uint32)
        if index.size == 0:
            return
        di, dof, dv = (self.copy_from_u32("index", index), self.copy_from_u32("offsets", offsets),
                       self.copy_from_elem("values", values))
        check(lib().r0hip_scatter(into.ptr, di.ptr, dof.ptr, dv.ptr, index.size - 1))

    def rv32im_accum_finalize(self, accum, rows, cols, last_cycle):
        """accumulation phases 2-3 of risc0_circuit_rv32im_cuda_accum (ffi.cu:480-509)"""
        check(lib().r0hip_rv32im_accum_finalize(accum.ptr, rows, cols, last_cycle))

    def rv32im_accum(self, data, accum, glob, mix, rows, last_cycle):
        """the whole rv32im accumulation, phases 1-3 (risc0_circuit_rv32im_cuda_accum,
        ffi.cu:362-514): `accum` (103 columns of `rows`) starts all-INVALID"""
        check(lib().r0hip_rv32im_accum(data.ptr, accum.ptr, glob.ptr, mix.ptr, rows, 103, last_cycle))

    def recursion_accum(self, ctrl, glob, data, mix, accum, work_cycles, total_cycles):
        """CircuitAccumulator::accumulate of the recursion circuit (witgen.rs:162-170 ->
        risc0_circuit_recursion_cuda_accum): compute, prefix product, verify"""
        check(lib().r0hip_recursion_accum(ctrl.ptr, glob.ptr, data.ptr, mix.ptr, accum.ptr, work_cycles,
                                          total_cycles))

    def prefix_products(self, io):
        check(lib().r0hip_prefix_products(io.ptr, io.size))

    def combos_prepare(self, combos, coeff_u, combo_count, cycles, reg_sizes, reg_combo_ids, mix):
        u, up = _h(coeff_u)
        rs, rsp = _h(reg_sizes)
        rc, rcp = _h(reg_combo_ids)
        m, mp = _h(mix)
        check(lib().r0hip_combos_prepare(combos.ptr, up, combo_count, cycles, rsp, rcp, rs.size, mp))

    def combos_divide(self, combos, chunk_pows, chunk_begin, cycles):
        pw, pwp = _h(chunk_pows)
        bg, bgp = _h(chunk_begin)
        bad = C.c_int64(0)
        check(lib().r0hip_combos_divide(combos.ptr, bg.size - 1, pwp, bgp, cycles, C.byref(bad)))
        return bad.value

    def eval_check(self, circuit, check_buf, groups, mix, glob, poly_mix, po2):
        arr = (C.c_void_p * len(groups))(*[g.ptr for g in groups])
        pm, pmp = _h(poly_mix)
        check(lib().r0hip_eval_check(circuit.encode(), check_buf.ptr, arr, mix.ptr, glob.ptr, pmp, po2))

    def synchronize(self):
        check(lib().r0hip_synchronize())


def prove_segment(hal, circuit, po2, code, data, accum, glob, version=None, seal_cap=1 << 24):
    """Prove one segment from device-resident witness groups; returns (seal, mix)."""
    from json import load
    with open(os.path.join(_HERE, "circuits", circuit + ".taps.json")) as f:
        mix_size = load(f)["mix_size"]
    seal = np.zeros(seal_cap, dtype=np.uint32)
    n = C.c_size_t(0)
    mix = np.zeros(mix_size, dtype=np.uint32)
    check(lib().r0hip_prove_segment(circuit.encode(), hal.suite, po2, code.ptr, data.ptr, accum.ptr, glob.ptr,
                                    int(version is not None), version or 0, seal.ctypes.data_as(u32p), seal_cap,
                                    C.byref(n), mix.ctypes.data_as(u32p)))
    return seal[: n.value].copy(), mix


class BigIntBack(C.Structure):
    """struct r0hip_bigint_back (include/r0hip.h): one Back::BigInt record of the rv32im
    preflight trace (witgen/preflight.rs:55-56; BigIntState, witgen/bigint.rs:36-44)"""
    _fields_ = [("row", C.c_uint32), ("poly_op", C.c_uint32), ("coeff", C.c_uint32), ("bytes", C.c_uint8 * 16)]


def bigint_backs(records):
    """ctypes array of BigIntBack from [(row, poly_op, coeff, bytes16), ...] (None/[] -> None)"""
    if records is None or len(records) == 0:
        return None
    arr = (BigIntBack * len(records))()
    for a, (row, op, coeff, by) in zip(arr, records):
        a.row, a.poly_op, a.coeff = int(row), int(op), int(coeff)
        for i, b in enumerate(by):
            a.bytes[i] = int(b)
    return arr


def bigint_accum_states(mix, records, rows):
    """r0hip_rv32im_bigint_accum_states (host-only): BigIntAccum::step over the records with the
    final mix (byte_poly.rs:381-470); returns (len(records), 12) Montgomery words"""
    arr = bigint_backs(records)
    n = 0 if arr is None else len(arr)
    m, mp = _h(mix)
    out = np.zeros(max(1, n * 12), np.uint32)
    check(lib().r0hip_rv32im_bigint_accum_states(mp, None if arr is None else C.cast(arr, C.c_void_p), n, rows,
                                                 out.ctypes.data_as(u32p)))
    return out[: n * 12].reshape(n, 12)


def bigint_accum_inject(accum, rows, mix, records):
    """r0hip_rv32im_bigint_accum_inject: the states scattered into accum columns 0..11"""
    arr = bigint_backs(records)
    m, mp = _h(mix)
    check(lib().r0hip_rv32im_bigint_accum_inject(accum.ptr, rows, mp, None if arr is None else C.cast(arr, C.c_void_p),
                                                 0 if arr is None else len(arr)))


def prove_segment_accum(hal, circuit, po2, code, data, accum, work_cycles, glob, version=None, seal_cap=1 << 24,
                        bigint=None):
    """Prove one segment with the circuit's accumulation on the device between the mix draw and
    the accum commit (r0hip_prove_segment_accum): `accum` holds the group as the witness
    generator allocated it (INVALID words) and is filled in place; `bigint` (rv32im) is the
    trace's BigInt backs [(row, poly_op, coeff, bytes16)], injected with the drawn mix.
    Returns (seal, mix)."""
    backs = bigint_backs(bigint)
    from json import load
    with open(os.path.join(_HERE, "circuits", circuit + ".taps.json")) as f:
        mix_size = load(f)["mix_size"]
    seal = np.zeros(seal_cap, dtype=np.uint32)
    n = C.c_size_t(0)
    mix = np.zeros(mix_size, dtype=np.uint32)
    check(lib().r0hip_prove_segment_accum(circuit.encode(), hal.suite, po2, code.ptr, data.ptr, accum.ptr,
                                          work_cycles, None if backs is None else C.cast(backs, C.c_void_p),
                                          0 if backs is None else len(backs), glob.ptr, int(version is not None),
                                          version or 0,
                                          seal.ctypes.data_as(u32p), seal_cap, C.byref(n),
                                          mix.ctypes.data_as(u32p)))
    return seal[: n.value].copy(), mix


def _trace(wom, cycles, iops):
    w = np.ascontiguousarray(np.asarray(wom, dtype=np.uint32).reshape(-1))
    c = np.ascontiguousarray(np.asarray(cycles, dtype=np.uint32).reshape(-1))
    i = np.ascontiguousarray(np.asarray(iops, dtype=np.uint32).reshape(-1))
    assert w.size % 4 == 0 and c.size % 2 == 0 and i.size % 4 == 0
    return w, c, i


def recursion_witgen(ctrl, data, glob, total_cycles, wom, cycles, iops):
    """r0hip_recursion_witgen: the recursion circuit's witness generation on the device from
    the control group and the preflight trace (wom: (k, 4) words, cycles: [(iop_idx,
    is_par_safe)], iops: (m, 4) words); data and glob must arrive INVALID-filled."""
    w, c, i = _trace(wom, cycles, iops)
    check(lib().r0hip_recursion_witgen(ctrl.ptr, data.ptr, glob.ptr, total_cycles, w.ctypes.data_as(u32p), w.size // 4,
                                       c.ctypes.data_as(u32p), c.size // 2, i.ctypes.data_as(u32p), i.size // 4))


def prove_recursion(hal, po2, ctrl, wom, cycles, iops, noise_seed, seal_cap=1 << 24):
    """r0hip_prove_recursion: a whole recursion proof from the program's control group and its
    preflight trace (witness generation, ZK noise from noise_seed, accumulation, prove).
    Returns (seal, mix)."""
    w, c, i = _trace(wom, cycles, iops)
    seal = np.zeros(seal_cap, dtype=np.uint32)
    n = C.c_size_t(0)
    mix = np.zeros(20, dtype=np.uint32)
    check(lib().r0hip_prove_recursion(hal.suite, po2, ctrl.ptr, w.ctypes.data_as(u32p), w.size // 4,
                                      c.ctypes.data_as(u32p), c.size // 2, i.ctypes.data_as(u32p), i.size // 4,
                                      noise_seed, seal.ctypes.data_as(u32p), seal_cap, C.byref(n),
                                      mix.ctypes.data_as(u32p)))
    return seal[: n.value].copy(), mix


class RawBuffer(C.Structure):
    """struct r0hip_raw_buffer (RawBuffer, rv32im-sys/src/lib.rs:63-69)"""
    _fields_ = [("buf", C.c_void_p), ("rows", C.c_size_t), ("cols", C.c_size_t), ("checked", C.c_bool)]


class RawExecBuffers(C.Structure):
    """struct r0hip_raw_exec_buffers (RawExecBuffers, lib.rs:71-75)"""
    _fields_ = [("glob", RawBuffer), ("data", RawBuffer)]


class RawPreflightTrace(C.Structure):
    """struct r0hip_raw_preflight_trace (RawPreflightTrace, lib.rs:53-61): host pointers"""
    _fields_ = [("cycles", C.c_void_p), ("txns", C.c_void_p), ("bigint_bytes", C.c_void_p), ("txns_len", C.c_uint32),
                ("bigint_bytes_len", C.c_uint32), ("table_split_cycle", C.c_uint32)]


def rv32im_witgen(data, glob, cycles, txns, table_split, bigint=None, mode=0):
    """r0hip_rv32im_witgen: the rv32im witness generation (step_Top per cycle, two phases) on
    the device. data (211 x rows) and glob (90 words) are device buffers as the witness
    generator prepares them (INVALID with the injector scattered in); cycles / txns are the
    preflight's RawPreflightCycle / RawMemoryTransaction arrays (numpy structured or raw bytes,
    one record per row)."""
    cyc = np.ascontiguousarray(cycles)
    tx = np.ascontiguousarray(txns)
    bi = np.ascontiguousarray(bigint if bigint is not None else np.zeros(0, np.uint8), dtype=np.uint8)
    rows = data.size // 211
    assert cyc.nbytes == 36 * rows and tx.nbytes % 20 == 0
    bufs = RawExecBuffers(RawBuffer(glob.ptr, 1, glob.size, True), RawBuffer(data.ptr, rows, 211, True))
    pf = RawPreflightTrace(cyc.ctypes.data, tx.ctypes.data if tx.nbytes else None, bi.ctypes.data if bi.size else None,
                           tx.nbytes // 20, bi.size, table_split)
    check(lib().r0hip_rv32im_witgen(mode, C.byref(bufs), C.byref(pf), rows))


def prove_segment_trace(hal, po2, glob, inj_index, inj_offsets, inj_values, cycles, txns, table_split, bigint=None,
                        bigint_records=None, mode=0, seal_cap=1 << 24):
    """r0hip_prove_segment_trace: rv32im prove_core from a preflight trace on the device
    (injector scatter, stepExec, zeroize, accumulation, prove). glob: build_global_vec's 90
    Montgomery words (INVALID where unset); the injector as index / offsets / Montgomery
    values. Returns (seal, mix)."""
    u = lambda a: np.ascontiguousarray(a, dtype=np.uint32)
    g, ix, off, val = u(glob), u(inj_index), u(inj_offsets), u(inj_values)
    cyc, tx = np.ascontiguousarray(cycles), np.ascontiguousarray(txns)
    bi = np.ascontiguousarray(bigint if bigint is not None else np.zeros(0, np.uint8), dtype=np.uint8)
    pf = RawPreflightTrace(cyc.ctypes.data, tx.ctypes.data if tx.nbytes else None, bi.ctypes.data if bi.size else None,
                           tx.nbytes // 20, bi.size, table_split)
    backs = bigint_backs(bigint_records)
    nb = 0 if backs is None else len(backs)
    backs = None if backs is None else C.cast(backs, C.c_void_p)
    seal = np.zeros(seal_cap, dtype=np.uint32)
    n = C.c_size_t(0)
    mix = np.zeros(36, dtype=np.uint32)
    check(lib().r0hip_prove_segment_trace(hal.suite, po2, mode, g.ctypes.data_as(u32p), ix.ctypes.data_as(u32p),
                                          ix.size - 1, off.ctypes.data_as(u32p), val.ctypes.data_as(u32p), C.byref(pf),
                                          backs, nb, seal.ctypes.data_as(u32p), seal_cap, C.byref(n),
                                          mix.ctypes.data_as(u32p)))
    return seal[: n.value].copy(), mix


class ResidentTrace:
    """a preflight trace, its injector and global vector uploaded once to device memory, for
    r0hip_prove_segment_trace_resident (the benchmark's inputs-in-HBM form of
    prove_segment_trace)"""

    def __init__(self, hal, po2, glob, inj_index, inj_offsets, inj_values, cycles, txns, table_split, bigint=None):
        u = lambda a: np.ascontiguousarray(a, dtype=np.uint32).reshape(-1)
        self.po2 = po2
        self.glob = hal.copy_from_elem("global", u(glob))
        self.index = hal.copy_from_elem("inj_index", u(inj_index))
        self.inj_rows = self.index.size - 1
        n_inj = max(1, int(np.asarray(inj_index)[-1]))
        self.offsets = hal.copy_from_elem("inj_offsets", u(inj_offsets) if len(inj_offsets) else np.zeros(n_inj, np.uint32))
        self.values = hal.copy_from_elem("inj_values", u(inj_values) if len(inj_values) else np.zeros(n_inj, np.uint32))
        cyc = np.ascontiguousarray(cycles).view(np.uint32).reshape(-1)
        tx = np.ascontiguousarray(txns).view(np.uint32).reshape(-1)
        self.cycles = hal.copy_from_elem("cycles", cyc)
        self.txns = hal.copy_from_elem("txns", tx if tx.size else np.zeros(5, np.uint32))
        bi = np.ascontiguousarray(bigint if bigint is not None else np.zeros(4, np.uint8), dtype=np.uint8)
        pad = (-bi.size) % 4
        self.bigint = hal.copy_from_elem("bigint", np.concatenate([bi, np.zeros(pad, np.uint8)]).view(np.uint32))
        self.pf = RawPreflightTrace(self.cycles.ptr, self.txns.ptr if tx.size else None,
                                    self.bigint.ptr if bigint is not None and len(bigint) else None, tx.size // 5,
                                    0 if bigint is None else len(bigint), table_split)


def prove_segment_trace_resident(hal, t, mode=0, bigint_records=None, seal_cap=1 << 24):
    """r0hip_prove_segment_trace_resident over a ResidentTrace; returns (seal, mix)"""
    backs = bigint_backs(bigint_records)
    nb = 0 if backs is None else len(backs)
    backs = None if backs is None else C.cast(backs, C.c_void_p)
    seal = np.zeros(seal_cap, dtype=np.uint32)
    n = C.c_size_t(0)
    mix = np.zeros(36, dtype=np.uint32)
    check(lib().r0hip_prove_segment_trace_resident(hal.suite, t.po2, mode, t.glob.ptr, t.index.ptr, t.inj_rows,
                                                   t.offsets.ptr, t.values.ptr, C.byref(t.pf), backs, nb,
                                                   seal.ctypes.data_as(u32p), seal_cap, C.byref(n),
                                                   mix.ctypes.data_as(u32p)))
    return seal[: n.value].copy(), mix


class TraceInput(C.Structure):
    """struct r0hip_trace_input (include/r0hip.h): one preflight trace, host pointers"""
    _fields_ = [("mode", C.c_uint32), ("h_global", C.c_void_p), ("h_inj_index", C.c_void_p), ("inj_rows", C.c_size_t),
                ("h_inj_offsets", C.c_void_p), ("h_inj_values", C.c_void_p), ("preflight", RawPreflightTrace)]


class SegmentJob(C.Structure):
    """struct r0hip_segment_job (include/r0hip.h)"""
    _fields_ = [("h_code", C.c_void_p), ("h_data", C.c_void_p), ("h_accum", C.c_void_p), ("h_global", C.c_void_p),
                ("h_bigint", C.c_void_p), ("n_bigint", C.c_size_t), ("h_seal", C.c_void_p),
                ("seal_cap", C.c_size_t), ("seal_len", C.c_size_t), ("h_mix_out", C.c_void_p), ("error", C.c_void_p)]


class TraceJobStruct(C.Structure):
    """struct r0hip_trace_job (include/r0hip.h)"""
    _fields_ = [("trace", TraceInput), ("h_bigint", C.c_void_p), ("n_bigint", C.c_size_t), ("h_seal", C.c_void_p),
                ("seal_cap", C.c_size_t), ("seal_len", C.c_size_t), ("h_mix_out", C.c_void_p), ("error", C.c_void_p),
                ("verified", C.c_int), ("verify_ms", C.c_double), ("prove_ms", C.c_double)]


class TraceJob:
    """one rv32im segment's preflight trace as the segment pipeline takes it (r0hip_trace_input):
    the global vector, the injector (index / offsets / Montgomery values), the cycle and
    transaction records, the BigInt bytes and backs. The arrays are kept as given (page-locked
    views from host_array() copy at full PCIe rate; others are staged)."""

    def __init__(self, glob, inj_index, inj_offsets, inj_values, cycles, txns, table_split, bigint=None,
                 bigint_records=None, mode=0):
        u = lambda a: a if isinstance(a, np.ndarray) and a.dtype == np.uint32 and a.flags.c_contiguous \
            else np.ascontiguousarray(a, dtype=np.uint32)
        self.glob, self.index, self.offsets, self.values = u(glob), u(inj_index), u(inj_offsets), u(inj_values)
        self.cycles, self.txns = np.ascontiguousarray(cycles), np.ascontiguousarray(txns)
        self.table_split = table_split
        self.bigint = None if bigint is None or not len(bigint) else np.ascontiguousarray(bigint, dtype=np.uint8)
        self.records = bigint_records
        self.backs = bigint_backs(bigint_records)
        pf = RawPreflightTrace(self.cycles.ctypes.data, self.txns.ctypes.data if self.txns.nbytes else None,
                               None if self.bigint is None else self.bigint.ctypes.data, self.txns.nbytes // 20,
                               0 if self.bigint is None else self.bigint.size, table_split)
        self.struct = TraceInput(mode, self.glob.ctypes.data, self.index.ctypes.data, self.index.size - 1,
                                 self.offsets.ctypes.data if self.offsets.size else None,
                                 self.values.ctypes.data if self.values.size else None, pf)

    def h2d_bytes(self):
        return sum(a.nbytes for a in (self.glob, self.index, self.offsets, self.values, self.cycles, self.txns)) + \
            (0 if self.bigint is None else self.bigint.nbytes)


def host_array(shape, dtype):
    """a numpy array over page-locked host memory (r0hip_host_alloc); the block goes back with
    r0hip_host_free when the last view of it is gone"""
    dtype = np.dtype(dtype)
    count = int(np.prod(shape))
    nbytes = max(1, count * dtype.itemsize)
    p = C.c_void_p()
    check(lib().r0hip_host_alloc(C.byref(p), nbytes))
    block = (C.c_uint8 * nbytes).from_address(p.value)
    block._owner = _HostBlock(p.value)  # the ctypes array is every view's base
    return np.frombuffer(block, dtype=dtype, count=count).reshape(shape)


def pinned_copy(a):
    """a copy of `a` in page-locked host memory (host_array)"""
    a = np.ascontiguousarray(a)
    out = host_array(a.shape, a.dtype)
    out[...] = a
    return out


class _HostBlock:
    def __init__(self, ptr):
        self.ptr = ptr

    def __del__(self):
        if self.ptr:
            lib().r0hip_host_free(C.c_void_p(self.ptr))
            self.ptr = None


def prove_trace_segments(hal, po2, traces, in_flight=2, seal_cap=1 << 22, verify=True, per_job=False):
    """The GPU worker unit (r0hip_prove_trace_segments): each TraceJob is one rv32im prove_core
    from its preflight trace; an uploader copies the traces into in_flight + 1 device trace sets
    while in_flight provers run, and (verify) every seal is checked by the native verifier, the
    validity equation included, on a host thread beside the proofs. Returns [(seal, mix)] in job
    order and raises on any failed job; per_job=True returns [(seal, mix, error or None,
    verify_ms, prove_ms)] instead, without raising for a job's own failure (prove_ms: from a
    prover taking the job to its seal in host memory)."""
    jobs = (TraceJobStruct * len(traces))()
    seals, mixes, keep = [], [], []
    for j, t in zip(jobs, traces):
        keep.append(t)
        j.trace = t.struct
        if t.backs is not None:
            j.h_bigint, j.n_bigint = C.cast(t.backs, C.c_void_p).value, len(t.backs)
        seals.append(np.zeros(seal_cap, dtype=np.uint32))
        mixes.append(np.zeros(36, dtype=np.uint32))
        j.h_seal, j.seal_cap, j.h_mix_out = seals[-1].ctypes.data, seal_cap, mixes[-1].ctypes.data
    err = lib().r0hip_prove_trace_segments(hal.suite, po2, C.cast(jobs, C.c_void_p), len(traces), in_flight,
                                           int(bool(verify)))
    errors = []
    for j in jobs:
        errors.append(C.cast(j.error, C.c_char_p).value.decode() if j.error else None)
        if j.error:
            libc_free(j.error)
    if per_job:
        if err and not any(errors):
            check(err)  # a failure of the call itself, not of a job
        elif err:
            libc_free(err)
        return [(seal[: j.seal_len].copy(), mix, e, j.verify_ms, j.prove_ms) for j, seal, mix, e in zip(jobs, seals, mixes, errors)]
    check(err)
    if verify:
        assert all(j.verified for j in jobs)
    return [(seal[: j.seal_len].copy(), mix) for j, seal, mix in zip(jobs, seals, mixes)]


def prove_segments(hal, circuit, po2, witnesses, version=None, in_flight=2, seal_cap=1 << 24):
    """The native segment pipeline (r0hip_prove_segments): `witnesses` is a list of
    (code, data, accum, global) host arrays (numpy uint32, ideally views of page-locked
    memory) or raw host pointers; returns [(seal, mix)] in job order. For rv32im, accum may
    be None: the prover then runs the accumulation on the device (r0hip_prove_segment_accum's
    path) and nothing of that group crosses PCIe; a 5th element then gives the job's BigInt
    backs [(row, poly_op, coeff, bytes16)]."""
    from json import load
    with open(os.path.join(_HERE, "circuits", circuit + ".taps.json")) as f:
        mix_size = load(f)["mix_size"]
    jobs = (SegmentJob * len(witnesses))()
    keep, seals, mixes = [], [], []
    for j, w in zip(jobs, witnesses):
        ptrs = []
        backs = bigint_backs(w[4]) if len(w) > 4 else None
        if backs is not None:
            keep.append(backs)
            j.h_bigint, j.n_bigint = C.cast(backs, C.c_void_p).value, len(backs)
        for a in w[:4]:
            if isinstance(a, np.ndarray):
                a = np.ascontiguousarray(a, dtype=np.uint32)
                keep.append(a)
                ptrs.append(a.ctypes.data)
            else:
                ptrs.append(0 if a is None else int(a))
        j.h_code, j.h_data, j.h_accum, j.h_global = ptrs
        seals.append(np.zeros(seal_cap, dtype=np.uint32))
        mixes.append(np.zeros(mix_size, dtype=np.uint32))
        j.h_seal, j.seal_cap, j.h_mix_out = seals[-1].ctypes.data, seal_cap, mixes[-1].ctypes.data
    err = lib().r0hip_prove_segments(circuit.encode(), hal.suite, po2, int(version is not None), version or 0,
                                     C.cast(jobs, C.c_void_p), len(witnesses), in_flight)
    for j in jobs:
        if j.error:
            libc_free(j.error)
    check(err)
    return [(seal[: j.seal_len].copy(), mix) for j, seal, mix in zip(jobs, seals, mixes)]


def verify_seal(circuit, suite, seal, check_validity=True, code_roots=None, return_code_root=False):
    """r0hip_verify_seal: the native seal verifier (host-only, no GPU); returns the
    segment po2 (and the code root, 8 words, with return_code_root), raises R0HipError
    naming the failed check. code_roots: allowed code/control roots (check_code,
    zkp/src/verify/mod.rs:531). check_validity=False calls the test-only
    r0hip_testing_verify_seal_structure instead (no constraint equation, no code-root check),
    for seals of synthetic witnesses."""
    seal = np.ascontiguousarray(seal, dtype=np.uint32)
    po2 = C.c_uint32(0)
    sid = SUITES[suite] if isinstance(suite, str) else suite
    if not check_validity:
        assert code_roots is None and not return_code_root, "the structure check binds no code root"
        check(lib().r0hip_testing_verify_seal_structure(circuit.encode(), sid, seal.ctypes.data_as(u32p), seal.size,
                                                        C.byref(po2)))
        return po2.value
    roots = np.ascontiguousarray(np.zeros(0, np.uint32) if code_roots is None else code_roots, dtype=np.uint32)
    assert roots.size % 8 == 0
    root_out = np.zeros(8, np.uint32)
    check(lib().r0hip_verify_seal(circuit.encode(), sid, seal.ctypes.data_as(u32p), seal.size,
                                  roots.ctypes.data_as(u32p), roots.size // 8, root_out.ctypes.data_as(u32p),
                                  C.byref(po2)))
    return (po2.value, root_out) if return_code_root else po2.value


def poly_ext(circuit, mix, glob, eval_u, poly_mix):
    """r0hip_poly_ext (host-only): Montgomery words in, the FpExt result as 4 Montgomery words."""
    arrs = [np.ascontiguousarray(a, dtype=np.uint32) for a in (mix, glob, eval_u, poly_mix)]
    out = np.zeros(4, np.uint32)
    check(lib().r0hip_poly_ext(circuit.encode(), *(a.ctypes.data_as(u32p) for a in arrs), out.ctypes.data_as(u32p)))
    return out


def libc_free(p):
    C.CDLL(None).free(C.c_void_p(p))


def last_profile():
    buf = C.create_string_buffer(4096)
    check(lib().r0hip_last_profile(buf, 4096))
    out = {}
    for kv in buf.value.decode().split(";"):
        if "=" in kv:
            k, v = kv.split("=")
            out[k] = float(v)
    return out


def set_kernel_timing(on):
    check(lib().r0hip_set_kernel_timing(int(bool(on))))


def kernel_times():
    """{kernel: (total_ms, calls, algorithmic_bytes, modmul_equivalents)} since timing was enabled."""
    buf = C.create_string_buffer(16384)
    check(lib().r0hip_kernel_times(buf, 16384))
    out = {}
    for kv in buf.value.decode().split(";"):
        if "=" in kv:
            k, v = kv.split("=")
            ms, calls, b, mm = v.split(":")
            out[k] = (float(ms), int(calls), float(b), float(mm))
    return out


def mem_stats():
    """The library's MemoryTracker (zkp/src/hal/mod.rs:292-317): live and reserved device
    bytes, their peaks since mem_reset_peak(), and how many hipMalloc calls it has made."""
    out = (C.c_uint64 * 5)()
    check(lib().r0hip_mem_stats(out))
    return dict(zip(("live", "peak_live", "reserved", "peak_reserved", "mallocs"), (int(x) for x in out)))


def mem_reset_peak():
    check(lib().r0hip_mem_reset_peak())


def trim():
    """r0hip_trim: release idle pooled device memory (this thread's and exited threads')."""
    check(lib().r0hip_trim())
