// risc0/sys/src/hip.rs — raw bindings of libr0hip (include/r0hip.h), behind `feature = "hip"`.
//
// Replaces for the HIP backend what risc0/sys/src/cuda.rs:19-80 (sppark_* and
// supra_poly_divide) and the risc0_zkp_cuda_* block bound by risc0/zkp/src/hal/cuda.rs
// provide for CUDA, plus the device/memory calls the `cust` crate makes there (cust does
// not run on ROCm). Every function returns NULL on success or a malloc'd message; wrap the
// call in `risc0_sys::ffi_wrap` (risc0/sys/src/lib.rs:53-75), which frees it.
//
// NOT COMPILED IN THIS REPOSITORY: the image has no Rust toolchain. The declarations are
// checked against include/r0hip.h by tests/test_integration_sources.py (every r0hip_* symbol
// the header declares is bound here with the same arity).
//
// build.rs of risc0-sys, `hip` feature (the kernels are prebuilt for gfx950 by
// `python -c "import __graft_entry__ as g; g.build()"`):
//     if env::var("CARGO_FEATURE_HIP").is_ok() {
//         let dir = env::var("R0HIP_LIB_DIR").expect("R0HIP_LIB_DIR: directory of libr0hip.so");
//         println!("cargo:rustc-link-search=native={dir}");
//         println!("cargo:rustc-link-lib=dylib=r0hip");
//         println!("cargo:rerun-if-env-changed=R0HIP_LIB_DIR");
//     }

use std::os::raw::{c_char, c_int, c_void};

/// Hash suite selectors of r0hip_hash_rows / r0hip_hash_fold / r0hip_prove_segment.
pub const R0HIP_POSEIDON2: c_int = 0;
pub const R0HIP_SHA256: c_int = 1;
pub const R0HIP_POSEIDON254: c_int = 2;

/// One Back::BigInt record of the rv32im preflight trace (struct r0hip_bigint_back).
#[repr(C)]
pub struct R0HipBigIntBack {
    pub row: u32,
    pub poly_op: u32,
    pub coeff: u32,
    pub bytes: [u8; 16],
}

/// A preflight trace as a job of r0hip_prove_trace_segments takes it (struct r0hip_trace_input):
/// host pointers; `preflight` has the repr(C) layout of risc0_circuit_rv32im_sys::RawPreflightTrace.
#[repr(C)]
pub struct R0HipTraceInput {
    pub mode: u32,
    pub h_global: *const u32,
    pub h_inj_index: *const u32,
    pub inj_rows: usize,
    pub h_inj_offsets: *const u32,
    pub h_inj_values: *const u32,
    pub preflight: risc0_circuit_rv32im_sys::RawPreflightTrace,
}

/// One job of r0hip_prove_segments: host witness groups in, seal out (struct r0hip_segment_job).
#[repr(C)]
pub struct R0HipSegmentJob {
    pub h_code: *const u32,
    pub h_data: *const u32,
    pub h_accum: *const u32,
    pub h_global: *const u32,
    pub h_bigint: *const R0HipBigIntBack,
    pub n_bigint: usize,
    pub h_seal: *mut u32,
    pub seal_cap: usize,
    pub seal_len: usize,
    pub h_mix_out: *mut u32,
    pub error: *const c_char,
}

/// One job of r0hip_prove_trace_segments (struct r0hip_trace_job): the rv32im prove_core of one
/// preflight trace; seal out, and with `verify` the receipt check's outcome.
#[repr(C)]
pub struct R0HipTraceJob {
    pub trace: R0HipTraceInput,
    pub h_bigint: *const R0HipBigIntBack,
    pub n_bigint: usize,
    pub h_seal: *mut u32,
    pub seal_cap: usize,
    pub seal_len: usize,
    pub h_mix_out: *mut u32,
    pub error: *const c_char,
    pub verified: c_int,
    pub verify_ms: f64,
    pub prove_ms: f64,
}

#[link(name = "r0hip")]
unsafe extern "C" {
    // ---- device and memory (cust's role in hal/cuda.rs:235-421) ----
    pub fn r0hip_init(device_ordinal: c_int) -> *const c_char;
    pub fn r0hip_device_info(name: *mut c_char, name_cap: usize, total_mem: *mut u64) -> *const c_char;
    pub fn r0hip_alloc(d_ptr: *mut *mut c_void, bytes: usize) -> *const c_char;
    pub fn r0hip_free(d_ptr: *mut c_void) -> *const c_char;
    pub fn r0hip_memset32(d_dst: *mut c_void, value: u32, count: usize) -> *const c_char;
    pub fn r0hip_memcpy_h2d(d_dst: *mut c_void, h_src: *const c_void, bytes: usize) -> *const c_char;
    pub fn r0hip_memcpy_d2h(h_dst: *mut c_void, d_src: *const c_void, bytes: usize) -> *const c_char;
    pub fn r0hip_memcpy_d2d(d_dst: *mut c_void, d_src: *const c_void, bytes: usize) -> *const c_char;
    pub fn r0hip_host_alloc(h_ptr: *mut *mut c_void, bytes: usize) -> *const c_char;
    pub fn r0hip_host_free(h_ptr: *mut c_void) -> *const c_char;
    pub fn r0hip_synchronize() -> *const c_char;
    pub fn r0hip_free_error(err: *const c_char);
    // a device-to-host copy beside later calls (the HAL's node-heap mirrors, hal_hip.rs)
    pub fn r0hip_memcpy_d2h_start(h_dst: *mut c_void, d_src: *const c_void, bytes: usize,
                                  h_copy: *mut *mut c_void) -> *const c_char;
    pub fn r0hip_copy_finish(h_copy: *mut c_void, block: c_int, done: *mut c_int) -> *const c_char;

    // ---- NTT family (sppark_batch_expand/NTT/iNTT/zk_shift, cuda_batch_bit_reverse) ----
    pub fn r0hip_batch_expand_into_evaluate_ntt(
        d_out: *mut u32,
        d_in: *const u32,
        count: usize,
        lg_out: u32,
        expand_bits: u32,
    ) -> *const c_char;
    pub fn r0hip_batch_interpolate_ntt(d_io: *mut u32, count: usize, lg_size: u32) -> *const c_char;
    pub fn r0hip_zk_shift(d_io: *mut u32, count: usize, lg_size: u32) -> *const c_char;
    pub fn r0hip_batch_bit_reverse(d_io: *mut u32, count: usize, lg_size: u32) -> *const c_char;

    // ---- polynomial ops ----
    pub fn r0hip_batch_evaluate_any(
        d_out: *mut u32,
        d_coeffs: *const u32,
        poly_count: usize,
        lg_poly_size: u32,
        d_which: *const u32,
        d_xs: *const u32,
        eval_count: usize,
    ) -> *const c_char;
    pub fn r0hip_mix_poly_coeffs(
        d_out: *mut u32,
        d_in: *const u32,
        h_combos: *const u32,
        h_mix_start: *const u32,
        h_mix: *const u32,
        input_size: usize,
        count: usize,
    ) -> *const c_char;
    pub fn r0hip_fri_fold(d_out: *mut u32, d_in: *const u32, h_mix: *const u32, count: usize) -> *const c_char;
    pub fn r0hip_combos_prepare(
        d_combos: *mut u32,
        h_coeff_u: *const u32,
        combo_count: usize,
        cycles: usize,
        h_reg_sizes: *const u32,
        h_reg_combo_ids: *const u32,
        reg_count: usize,
        h_mix: *const u32,
    ) -> *const c_char;
    pub fn r0hip_poly_divide(d_poly: *mut u32, size: usize, h_remainder: *mut u32, h_z: *const u32) -> *const c_char;
    pub fn r0hip_combos_divide(
        d_combos: *mut u32,
        nchunks: usize,
        h_pows: *const u32,
        h_begin: *const u32,
        cycles: usize,
        bad_chunk: *mut i64,
    ) -> *const c_char;

    // ---- element-wise ----
    pub fn r0hip_eltwise_add_elem(d_out: *mut u32, d_a: *const u32, d_b: *const u32, count: usize) -> *const c_char;
    pub fn r0hip_eltwise_copy_elem(d_out: *mut u32, d_in: *const u32, count: usize) -> *const c_char;
    pub fn r0hip_eltwise_zeroize_elem(d_io: *mut u32, count: usize) -> *const c_char;
    pub fn r0hip_eltwise_sum_extelem(d_out: *mut u32, d_in: *const u32, to_add: usize, count: usize) -> *const c_char;
    pub fn r0hip_eltwise_copy_elem_slice(
        d_into: *mut u32,
        d_from: *const u32,
        from_rows: usize,
        from_cols: usize,
        from_offset: usize,
        from_stride: usize,
        into_offset: usize,
        into_stride: usize,
    ) -> *const c_char;
    pub fn r0hip_gather_sample(d_dst: *mut u32, d_src: *const u32, idx: usize, size: usize, stride: usize)
        -> *const c_char;
    pub fn r0hip_gather_sample_host(h_dst: *mut u32, d_src: *const u32, idx: usize, size: usize, stride: usize)
        -> *const c_char;
    pub fn r0hip_scatter(
        d_into: *mut u32,
        d_index: *const u32,
        d_offsets: *const u32,
        d_values: *const u32,
        cycles: usize,
    ) -> *const c_char;
    pub fn r0hip_prefix_products(d_io: *mut u32, count: usize) -> *const c_char;
    pub fn r0hip_fill_uniform(d_out: *mut u32, count: usize, seed: u64) -> *const c_char;

    // ---- hashing (sppark_poseidon2_*, risc0_zkp_cuda_sha_*, sppark_poseidon254_*) ----
    pub fn r0hip_hash_rows(suite: c_int, d_out: *mut u32, d_matrix: *const u32, rows: usize, cols: usize)
        -> *const c_char;
    pub fn r0hip_hash_fold(suite: c_int, d_io: *mut u32, input_size: usize, output_size: usize) -> *const c_char;
    pub fn r0hip_merkle_tree(suite: c_int, d_nodes: *mut u32, d_matrix: *const u32, rows: usize, cols: usize)
        -> *const c_char;

    // ---- circuits ----
    pub fn r0hip_eval_check(
        circuit: *const c_char,
        d_check: *mut u32,
        d_groups: *const *const u32,
        d_mix: *const u32,
        d_global: *const u32,
        h_poly_mix: *const u32,
        po2: u32,
    ) -> *const c_char;
    pub fn r0hip_rv32im_accum_finalize(d_accum: *mut u32, rows: usize, cols: usize, last_cycle: usize)
        -> *const c_char;
    pub fn r0hip_rv32im_accum(
        d_data: *const u32,
        d_accum: *mut u32,
        d_global: *const u32,
        d_mix: *const u32,
        rows: usize,
        cols: usize,
        last_cycle: usize,
    ) -> *const c_char;
    pub fn r0hip_recursion_accum(
        d_ctrl: *const u32,
        d_global: *const u32,
        d_data: *const u32,
        d_mix: *const u32,
        d_accum: *mut u32,
        work_cycles: usize,
        total_cycles: usize,
    ) -> *const c_char;

    // ---- whole segments ----
    pub fn r0hip_prove_segment(
        circuit: *const c_char,
        suite: c_int,
        po2: u32,
        d_code: *const u32,
        d_data: *const u32,
        d_accum: *const u32,
        d_global: *mut u32,
        write_version: c_int,
        version: u32,
        h_seal: *mut u32,
        seal_cap: usize,
        seal_len: *mut usize,
        h_mix_out: *mut u32,
    ) -> *const c_char;
    /// prove_core with WitnessGenerator::accum inside (accum group given as witgen allocated it)
    pub fn r0hip_prove_segment_accum(
        circuit: *const c_char,
        suite: c_int,
        po2: u32,
        d_code: *const u32,
        d_data: *const u32,
        d_accum: *mut u32,
        work_cycles: usize,
        h_bigint: *const R0HipBigIntBack,
        n_bigint: usize,
        d_global: *mut u32,
        write_version: c_int,
        version: u32,
        h_seal: *mut u32,
        seal_cap: usize,
        seal_len: *mut usize,
        h_mix_out: *mut u32,
    ) -> *const c_char;
    /// WitnessGenerator::accum's BigInt state injection (witgen/mod.rs:178-205)
    pub fn r0hip_rv32im_bigint_accum_states(
        h_mix: *const u32,
        h_backs: *const R0HipBigIntBack,
        n: usize,
        rows: usize,
        h_states: *mut u32,
    ) -> *const c_char;
    pub fn r0hip_rv32im_bigint_accum_inject(
        d_accum: *mut u32,
        rows: usize,
        h_mix: *const u32,
        h_backs: *const R0HipBigIntBack,
        n: usize,
    ) -> *const c_char;
    /// risc0_circuit_rv32im_cuda_witgen's role (rv32im-sys ffi.cu:431-472): `buffers` and
    /// `preflight` point at risc0_circuit_rv32im_sys::{RawExecBuffers, RawPreflightTrace}
    /// (identical repr(C) layouts: struct r0hip_raw_exec_buffers / r0hip_raw_preflight_trace)
    pub fn r0hip_rv32im_witgen(
        mode: u32,
        buffers: *const c_void,
        preflight: *const c_void,
        cycles: u32,
    ) -> *const c_char;
    /// rv32im SegmentProverImpl::prove_core from a preflight trace (prove/hal/mod.rs:143-224)
    pub fn r0hip_prove_segment_trace(
        suite: c_int,
        po2: u32,
        mode: u32,
        h_global: *const u32,
        h_inj_index: *const u32,
        inj_rows: usize,
        h_inj_offsets: *const u32,
        h_inj_values: *const u32,
        preflight: *const c_void,
        h_bigint: *const R0HipBigIntBack,
        n_bigint: usize,
        h_seal: *mut u32,
        seal_cap: usize,
        seal_len: *mut usize,
        h_mix_out: *mut u32,
    ) -> *const c_char;
    /// r0hip_prove_segment_trace with every input resident on the device
    pub fn r0hip_prove_segment_trace_resident(
        suite: c_int,
        po2: u32,
        mode: u32,
        d_global: *const u32,
        d_inj_index: *const u32,
        inj_rows: usize,
        d_inj_offsets: *const u32,
        d_inj_values: *const u32,
        d_preflight: *const c_void,
        h_bigint: *const R0HipBigIntBack,
        n_bigint: usize,
        h_seal: *mut u32,
        seal_cap: usize,
        seal_len: *mut usize,
        h_mix_out: *mut u32,
    ) -> *const c_char;
    /// risc0_circuit_recursion_cuda_witgen's role (recursion-sys ffi.cpp:191-205)
    pub fn r0hip_recursion_witgen(
        d_ctrl: *const u32,
        d_data: *mut u32,
        d_global: *mut u32,
        total_cycles: usize,
        h_wom: *const u32,
        n_wom: usize,
        h_cycles: *const u32,
        n_cycles: usize,
        h_iops: *const u32,
        n_iops: usize,
    ) -> *const c_char;
    /// RecursionProverImpl::prove from the program and its preflight (recursion prove/mod.rs:160-230)
    pub fn r0hip_prove_recursion(
        suite: c_int,
        po2: u32,
        d_ctrl: *const u32,
        h_wom: *const u32,
        n_wom: usize,
        h_cycles: *const u32,
        n_cycles: usize,
        h_iops: *const u32,
        n_iops: usize,
        noise_seed: u64,
        h_seal: *mut u32,
        seal_cap: usize,
        seal_len: *mut usize,
        h_mix_out: *mut u32,
    ) -> *const c_char;
    pub fn r0hip_prove_segments(
        circuit: *const c_char,
        suite: c_int,
        po2: u32,
        write_version: c_int,
        version: u32,
        jobs: *mut R0HipSegmentJob,
        njobs: usize,
        in_flight: u32,
    ) -> *const c_char;
    pub fn r0hip_prove_trace_segments(
        suite: c_int,
        po2: u32,
        jobs: *mut R0HipTraceJob,
        njobs: usize,
        in_flight: u32,
        verify: c_int,
    ) -> *const c_char;

    // ---- verification (host-only) ----
    pub fn r0hip_verify_seal(
        circuit: *const c_char,
        suite: c_int,
        seal: *const u32,
        seal_len: usize,
        h_code_roots: *const u32,
        n_code_roots: usize,
        h_code_root_out: *mut u32,
        po2_out: *mut u32,
    ) -> *const c_char;
    pub fn r0hip_testing_verify_seal_structure(
        circuit: *const c_char,
        suite: c_int,
        seal: *const u32,
        seal_len: usize,
        po2_out: *mut u32,
    ) -> *const c_char;
    pub fn r0hip_poly_ext(
        circuit: *const c_char,
        h_mix: *const u32,
        h_global: *const u32,
        h_eval_u: *const u32,
        h_poly_mix: *const u32,
        h_out: *mut u32,
    ) -> *const c_char;

    // ---- diagnostics (scope! spans and the MemoryTracker) ----
    pub fn r0hip_set_kernel_timing(on: c_int) -> *const c_char;
    pub fn r0hip_kernel_times(buf: *mut c_char, cap: usize) -> *const c_char;
    pub fn r0hip_last_profile(buf: *mut c_char, cap: usize) -> *const c_char;
    pub fn r0hip_mem_stats(out: *mut u64) -> *const c_char;
    pub fn r0hip_mem_reset_peak() -> *const c_char;
    pub fn r0hip_trim() -> *const c_char;
}
