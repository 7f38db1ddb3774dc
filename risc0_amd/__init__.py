"""risc0_amd — MI355X-native STARK prover backend for risc0-zkp.

The product is libr0hip.so (risc0_amd/lib, built from risc0_amd/csrc by
__graft_entry__.build()): hand-written HIP kernels for gfx950 behind the C ABI
in include/r0hip.h, plus a C++ segment prover. This package is a thin ctypes
mirror of the reference's `Hal` trait for tests and the benchmark.
"""
from .hal import (POSEIDON2, POSEIDON254, SHA256, BigIntBack, Buffer, HipHal, R0HipError, bigint_accum_inject,
                  bigint_accum_states, check, prove_recursion, recursion_witgen, rv32im_witgen, prove_segment_trace, ResidentTrace,
                  prove_segment_trace_resident, exported_symbols, kernel_times,
                  last_profile, lib, mem_reset_peak, mem_stats, trim, prove_segment, prove_segment_accum, prove_segments,
                  set_kernel_timing, poly_ext, verify_seal, TraceJob, prove_trace_segments, host_array, pinned_copy)

__all__ = ["POSEIDON2", "POSEIDON254", "SHA256", "BigIntBack", "bigint_accum_inject", "bigint_accum_states", "prove_recursion", "recursion_witgen", "rv32im_witgen", "prove_segment_trace", "ResidentTrace", "prove_segment_trace_resident", "Buffer", "HipHal", "R0HipError", "check", "exported_symbols", "last_profile",
           "lib", "mem_reset_peak", "mem_stats", "trim", "prove_segment", "prove_segment_accum", "prove_segments",
           "kernel_times", "set_kernel_timing", "poly_ext", "verify_seal", "TraceJob", "prove_trace_segments",
           "host_array", "pinned_copy"]
