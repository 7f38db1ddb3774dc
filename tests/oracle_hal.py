"""TEST INFRASTRUCTURE — the CPU oracle behind the same Hal method names as
risc0_amd.HipHal (the reference CpuHal's role in its DualHal tests,
risc0/zkp/src/hal/mod.rs:319-616). Buffers are numpy arrays; slices are views. Used on
the CPU to pin tests/hal_prover.py (the reference Prover call sequence) against the
golden seals, so the GPU test of the same sequence checks only the HIP ops."""
import numpy as np


class Buf:
    def __init__(self, arr, words):
        self.a, self.words = arr, words
        self.size = arr.size // words

    def slice(self, offset, size):
        return Buf(self.a[offset * self.words:(offset + size) * self.words], self.words)

    def to_numpy(self):
        return self.a.copy()

    def copy_from(self, arr):
        self.a[:] = np.asarray(arr, dtype=np.uint32).reshape(-1)


class OracleHal:
    def __init__(self, oracle, suite, circuit_name=None):
        self.o = oracle
        self.suite = suite

    def _alloc(self, size, words):
        return Buf(np.zeros(size * words, np.uint32), words)

    def alloc_elem(self, name, size):
        return self._alloc(size, 1)

    def alloc_extelem(self, name, size):
        return self._alloc(size, 4)

    def alloc_digest(self, name, size):
        return self._alloc(size, 8)

    def alloc_extelem_zeroed(self, name, size):
        return self._alloc(size, 4)

    def copy_from_elem(self, name, arr):
        return Buf(np.array(arr, dtype=np.uint32).reshape(-1), 1)

    copy_from_u32 = copy_from_elem

    def copy_from_extelem(self, name, arr):
        return Buf(np.array(arr, dtype=np.uint32).reshape(-1), 4)

    def has_unified_memory(self):
        return False

    def eltwise_copy_elem(self, out, inp):
        out.a[:] = inp.a

    def batch_interpolate_ntt(self, io, count):
        self.o.batch_interpolate_ntt(io.a, count)

    def zk_shift(self, io, count):
        self.o.zk_shift(io.a, count)

    def batch_expand_into_evaluate_ntt(self, out, inp, count, expand_bits):
        self.o.batch_expand_into_evaluate_ntt(out.a, inp.a, count, expand_bits)

    def batch_bit_reverse(self, io, count):
        self.o.batch_bit_reverse(io.a, count)

    def hash_rows(self, out, matrix):
        self.o.hash_rows(self.suite, out.a, matrix.a)

    def hash_fold(self, io, input_size, output_size):
        self.o.hash_fold(self.suite, io.a, input_size, output_size)

    def gather_sample(self, dst, src, idx, size, stride):
        self.o.gather_sample(dst.a, src.a, idx, size, stride)

    def eval_check(self, circuit, check, groups, mix, glob, poly_mix, po2):
        self.o.eval_check(circuit, check.a, [g.a for g in groups], mix.a, glob.a,
                          np.asarray(poly_mix, np.uint32), po2)

    def batch_evaluate_any(self, coeffs, poly_count, which, xs, out):
        self.o.batch_evaluate_any(coeffs.a, poly_count, which.a, xs.a, out.a)

    def mix_poly_coeffs(self, out, mix_start, mix, inp, combos, input_size, count):
        self.o.mix_poly_coeffs(out.a, np.asarray(mix_start, np.uint32), np.asarray(mix, np.uint32), inp.a,
                               np.asarray(combos, np.uint32), input_size, count)

    def combos_prepare(self, combos, coeff_u, combo_count, cycles, reg_sizes, reg_combo_ids, mix):
        self.o.combos_prepare(combos.a, np.asarray(coeff_u, np.uint32), combo_count, cycles,
                              np.asarray(reg_sizes, np.uint32), np.asarray(reg_combo_ids, np.uint32),
                              np.asarray(mix, np.uint32))

    def combos_divide(self, combos, chunk_pows, chunk_begin, cycles):
        return self.o.combos_divide(combos.a, np.asarray(chunk_pows, np.uint32), np.asarray(chunk_begin, np.uint32),
                                    cycles)

    def eltwise_sum_extelem(self, out, inp):
        self.o.eltwise_sum_extelem(out.a, inp.a)

    def fri_fold(self, out, inp, mix):
        self.o.fri_fold(out.a, inp.a, np.asarray(mix, np.uint32))
