/*
 * r0hip — MI355X (gfx950) HAL for risc0-zkp: the C ABI a Rust `HipHal` binds.
 *
 * Drop-in boundary: every entry point below replaces one `extern "C"` symbol the
 * reference's CUDA HAL binds (risc0/zkp/src/hal/cuda.rs -> risc0/sys) or one piece
 * of the `cust` driver crate that cannot run on ROCm. Conventions, mirroring
 * risc0/sys/src/lib.rs:53-75 and SURVEY.md §8(b):
 *   - return NULL on success, else a malloc'd message the caller frees with free()
 *     (the reference's ffi_wrap contract); r0hip_free_error() is provided too;
 *   - pointers are device pointers to raw Montgomery u32 words unless named h_*;
 *     FpExt = 4 consecutive words (AoS), digests = 8 words, matrices column-major;
 *   - sizes/counts are 64-bit element counts (the CUDA ABI's u32 overflows at po2=24);
 *   - every call is complete when it returns (cuda.h:77-100 semantics): results are
 *     visible to the next call and to D2H copies. Work is queued on one HIP stream
 *     per process; r0hip_prove_segment runs whole proofs without per-op syncs.
 * Suites: R0HIP_POSEIDON2 = 0, R0HIP_SHA256 = 1, R0HIP_POSEIDON254 = 2 (zkp/src/core/hash/mod.rs:90-100;
 * the CUDA HAL's CudaHashPoseidon254, zkp/src/hal/cuda.rs:179-233).
 */
#ifndef R0HIP_H
#define R0HIP_H
#include <stddef.h>
#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define R0HIP_POSEIDON2 0
#define R0HIP_SHA256 1
#define R0HIP_POSEIDON254 2

/* ---- device / memory (replaces the `cust` crate; zkp/src/hal/cuda.rs:235-381,397-421) ---- */
const char* r0hip_init(int device_ordinal);                       /* sppark_init (sys/src/cuda.rs:20) */
const char* r0hip_device_info(char* name, size_t name_cap, uint64_t* total_mem);
const char* r0hip_alloc(void** d_ptr, size_t bytes);
const char* r0hip_free(void* d_ptr);
const char* r0hip_memset32(void* d_dst, uint32_t value, size_t count); /* alloc_elem_init (hal/mod.rs:72-83) */
const char* r0hip_memcpy_h2d(void* d_dst, const void* h_src, size_t bytes);
const char* r0hip_memcpy_d2h(void* h_dst, const void* d_src, size_t bytes);
const char* r0hip_memcpy_d2d(void* d_dst, const void* d_src, size_t bytes);
/* page-locked host memory for full-rate witness uploads (cust's LockedBuffer role) */
const char* r0hip_host_alloc(void** h_ptr, size_t bytes);
const char* r0hip_host_free(void* h_ptr);
const char* r0hip_synchronize(void);
void r0hip_free_error(const char* err);
/* A device-to-host copy that runs beside the caller's later calls, for a HAL's host mirrors
 * (hal_hip.rs: a Merkle node heap, read node by node by MerkleTreeProver::prove, merkle.rs:
 * 108-140). The copy goes on a process-wide copy stream; d_src is read as the caller's earlier
 * calls left it (every call is complete on return), and must not be written or freed until the
 * copy finished. *h_copy = a handle for r0hip_copy_finish, or NULL when the copy is already
 * done (bytes == 0, or h_dst is not r0hip_host_alloc memory: then it is copied before return).
 * r0hip_copy_finish: *done = 1 when the bytes are in h_dst (the handle is then released; a
 * NULL handle is done), 0 if not yet (only with block == 0). */
const char* r0hip_memcpy_d2h_start(void* h_dst, const void* d_src, size_t bytes, void** h_copy);
const char* r0hip_copy_finish(void* h_copy, int block, int* done);

/* ---- NTT family (sppark_batch_* in sys/src/cuda.rs:22-46; CPU semantics cpu.rs:305-408) ----
 * Inputs must be canonical field words (< p), as every buffer the Hal hands over is: the first
 * butterfly stage skips its unit twiddle (no Montgomery multiply reduces a staged word), so a
 * non-canonical input word is not reduced there. */
/* expand each of `count` polys of 2^(lg_out-expand_bits) bit-reversed coeffs into out (count x 2^lg_out)
 * and evaluate: Hal::batch_expand_into_evaluate_ntt (hal/mod.rs:102-108; cuda.rs:529-570) */
const char* r0hip_batch_expand_into_evaluate_ntt(uint32_t* d_out, const uint32_t* d_in, size_t count,
                                                 uint32_t lg_out, uint32_t expand_bits);
/* Hal::batch_interpolate_ntt (hal/mod.rs:110; cuda.rs:572-590 -> sppark_batch_iNTT) */
const char* r0hip_batch_interpolate_ntt(uint32_t* d_io, size_t count, uint32_t lg_size);
/* Hal::zk_shift (hal/mod.rs:123; cuda.rs:690-708 -> sppark_batch_zk_shift) */
const char* r0hip_zk_shift(uint32_t* d_io, size_t count, uint32_t lg_size);
/* Hal::batch_bit_reverse (risc0_zkp_cuda_batch_bit_reverse, ffi.cu:89-91) */
const char* r0hip_batch_bit_reverse(uint32_t* d_io, size_t count, uint32_t lg_size);

/* ---- polynomial ops ---- */
/* risc0_zkp_cuda_batch_evaluate_any (ffi.cu:93-101): out[k] = sum_i coeffs[which[k]][i] * xs[k]^i */
const char* r0hip_batch_evaluate_any(uint32_t* d_out, const uint32_t* d_coeffs, size_t poly_count,
                                     uint32_t lg_poly_size, const uint32_t* d_which, const uint32_t* d_xs,
                                     size_t eval_count);
/* risc0_zkp_cuda_mix_poly_coeffs (ffi.cu:79-87); mix_start / mix are host FpExt (4 words) */
const char* r0hip_mix_poly_coeffs(uint32_t* d_out, const uint32_t* d_in, const uint32_t* h_combos,
                                  const uint32_t* h_mix_start, const uint32_t* h_mix, size_t input_size,
                                  size_t count);
/* risc0_zkp_cuda_fri_fold (ffi.cu:75-77): out is 4 x count, in is 4 x 16 x count (SoA planes) */
const char* r0hip_fri_fold(uint32_t* d_out, const uint32_t* d_in, const uint32_t* h_mix, size_t count);
/* risc0_zkp_cuda_combos_prepare (ffi.cu:125-143); host arrays, CHECK_SIZE = 16 */
const char* r0hip_combos_prepare(uint32_t* d_combos, const uint32_t* h_coeff_u, size_t combo_count,
                                 size_t cycles, const uint32_t* h_reg_sizes, const uint32_t* h_reg_combo_ids,
                                 size_t reg_count, const uint32_t* h_mix);
/* supra_poly_divide (sys/src/cuda.rs:74-79): in-place division of a poly of `size` FpExt by (x - z);
 * h_remainder receives the remainder (Hal::combos_divide asserts it is zero, hal/mod.rs:236-257) */
const char* r0hip_poly_divide(uint32_t* d_poly, size_t size, uint32_t* h_remainder, const uint32_t* h_z);
/* Hal::combos_divide batched over all combos: chunk i divides combos[i*cycles..] by each z in
 * h_pows[h_begin[i]..h_begin[i+1]); *bad_chunk = first chunk with a nonzero remainder or -1 */
const char* r0hip_combos_divide(uint32_t* d_combos, size_t nchunks, const uint32_t* h_pows,
                                const uint32_t* h_begin, size_t cycles, int64_t* bad_chunk);

/* ---- element-wise (ffi.cu:27-73) ---- */
const char* r0hip_eltwise_add_elem(uint32_t* d_out, const uint32_t* d_a, const uint32_t* d_b, size_t count);
const char* r0hip_eltwise_copy_elem(uint32_t* d_out, const uint32_t* d_in, size_t count);
const char* r0hip_eltwise_zeroize_elem(uint32_t* d_io, size_t count);
/* out (4 x count SoA) = sum over to_add of in (to_add x count FpExt) */
const char* r0hip_eltwise_sum_extelem(uint32_t* d_out, const uint32_t* d_in, size_t to_add, size_t count);
const char* r0hip_eltwise_copy_elem_slice(uint32_t* d_into, const uint32_t* d_from, size_t from_rows,
                                          size_t from_cols, size_t from_offset, size_t from_stride,
                                          size_t into_offset, size_t into_stride);
const char* r0hip_gather_sample(uint32_t* d_dst, const uint32_t* d_src, size_t idx, size_t size, size_t stride);
/* gather_sample straight to the host: h_dst[i] = d_src[idx + i*stride], i < size (no CUDA
 * counterpart). For a HAL whose gather_sample destination is read back before the device uses it
 * (MerkleTreeProver::prove's sample, merkle.rs:111-129: gather_sample, then view): one kernel,
 * one copy and one sync instead of a device allocation, gather_sample, view and free. */
const char* r0hip_gather_sample_host(uint32_t* h_dst, const uint32_t* d_src, size_t idx, size_t size,
                                     size_t stride);
/* CSR scatter (ffi.cu:108-114): index has cycles+1 entries */
const char* r0hip_scatter(uint32_t* d_into, const uint32_t* d_index, const uint32_t* d_offsets,
                          const uint32_t* d_values, size_t cycles);
const char* r0hip_prefix_products(uint32_t* d_io, size_t count);
/* not a reference symbol: synthetic witness words (uniform canonical BabyBear values from a
 * counter hash of seed and index) for benches and tests at full size */
const char* r0hip_fill_uniform(uint32_t* d_out, size_t count, uint64_t seed);

/* ---- hashing (sppark_poseidon2_{rows,fold}, sppark_poseidon254_{rows,fold}, risc0_zkp_cuda_sha_{rows,fold};
 * sys/src/cuda.rs:49-72) ---- */
/* out[row] = H(matrix[col*rows + row] for col < cols). Poseidon2 / Poseidon254 inputs must be
 * canonical field words (< p): the Poseidon2 full rounds read a word as a signed 32-bit value,
 * which is its value mod p for any word below 2^31 (tests/native/field_equiv.cpp pins
 * [p, 2^31)) but not above. */
const char* r0hip_hash_rows(int suite, uint32_t* d_out, const uint32_t* d_matrix, size_t rows, size_t cols);
/* io[output_size + i] = H(io[input_size + 2i], io[input_size + 2i + 1]) (cpu.rs:569-581) */
const char* r0hip_hash_fold(int suite, uint32_t* d_io, size_t input_size, size_t output_size);
/* A whole tree in one call: MerkleTreeProver::new's hash_rows into nodes[rows..2rows) and
 * hash_fold of every layer down to the root at nodes[1] (prove/merkle.rs:54-81); d_nodes
 * holds 2*rows digests, rows a power of two. Same words as those calls; the fused form knows
 * each layer's height, so Poseidon2 and SHA-256 layers over all-zero rows store the zero-subtree digests
 * instead of hashing them. */
const char* r0hip_merkle_tree(int suite, uint32_t* d_nodes, const uint32_t* d_matrix, size_t rows, size_t cols);

/* ---- circuits (risc0_circuit_{rv32im,recursion}_cuda_eval_check) ---- */
/* circuit: "rv32im" | "recursion". groups[g] = evaluated register group g (accum=0, code=1, data=2),
 * d_check = 4 x 4*2^po2, h_poly_mix = the poly_mix FpExt (powers are expanded on the host) */
const char* r0hip_eval_check(const char* circuit, uint32_t* d_check, const uint32_t* const* d_groups,
                             const uint32_t* d_mix, const uint32_t* d_global, const uint32_t* h_poly_mix,
                             uint32_t po2);

/* ---- whole segment proof (risc0_zkp::prove::Prover driven as by the circuit's segment prover:
 * circuit/rv32im/src/prove/hal/mod.rs:143-224, circuit/recursion/src/prove/mod.rs:164-230) ----
 * Witness groups are device buffers (column-major, 2^po2 rows); d_global (output_size words) is
 * zeroized in place; h_mix_out (optional) receives the mix values drawn from the transcript.
 * The seal (Vec<u32>) is written to h_seal; *seal_len is its length in words. */
const char* r0hip_prove_segment(const char* circuit, int suite, uint32_t po2, const uint32_t* d_code,
                                const uint32_t* d_data, const uint32_t* d_accum, uint32_t* d_global,
                                int write_version, uint32_t version, uint32_t* h_seal, size_t seal_cap,
                                size_t* seal_len, uint32_t* h_mix_out);
/* ---- rv32im BigInt accumulator states (the witness generator's accum injection,
 * circuit/rv32im/src/prove/witgen/mod.rs:178-205) ----
 * One Back::BigInt record of the preflight trace (witgen/preflight.rs:55-56, 471-479), holding
 * the fields of BigIntState (witgen/bigint.rs:36-44) that BigIntAccum::step reads: the cycle
 * (row), poly_op (PolyOp, bigint.rs:62-70: 0 Reset, 1 Shift, 2 SetTerm, 3 AddTotal, 4 Carry1,
 * 5 Carry2, 6 EqZero), coeff (BigIntState::coeff = the instruction's coefficient + 4) and the
 * 16 bytes. Records are passed in trace order (strictly increasing rows). */
typedef struct r0hip_bigint_back {
  uint32_t row;
  uint32_t poly_op;
  uint32_t coeff;
  uint8_t bytes[16];
} r0hip_bigint_back;
/* BigIntAccum::new(final mix) then ::step per record (witgen/byte_poly.rs:381-470): the state
 * after each record, 12 Montgomery words (poly, term, total; BigIntAccumState::as_array) per
 * record into h_states. h_mix is the whole rv32im mix (36 words; the last 4 are the final
 * mix). Fails as the reference does on an EqZero whose goal is nonzero ("Invalid eqz in
 * bigint accum"). Host-only. */
const char* r0hip_rv32im_bigint_accum_states(const uint32_t* h_mix, const r0hip_bigint_back* h_backs, size_t n,
                                             size_t rows, uint32_t* h_states);
/* The states above scattered into accum columns 0..11 (BigIntAccumState::offsets,
 * byte_poly.rs:362-377) of each record's row of d_accum (column-major, `rows` rows): what
 * WitnessGenerator::accum does before step_accum (witgen/mod.rs:187-205). */
const char* r0hip_rv32im_bigint_accum_inject(uint32_t* d_accum, size_t rows, const uint32_t* h_mix,
                                             const r0hip_bigint_back* h_backs, size_t n);

/* ---- whole segment proof with the accumulation on the device: the prove_core sequence above,
 * with the circuit's accumulation between the mix draw and the accum commit, as the reference
 * runs it (rv32im: WitnessGenerator::accum, circuit/rv32im/src/prove/witgen/mod.rs:178-221, over
 * risc0_circuit_rv32im_cuda_accum; recursion: prove/witgen.rs:138-177 over
 * risc0_circuit_recursion_cuda_accum). d_accum is the accum group as the witness generator
 * allocated it: every word INVALID (0xFFFFFFFF), plus for recursion the ZK noise rows the caller
 * draws (witgen.rs:143-158). rv32im: h_bigint/n_bigint are the trace's BigInt backs; their
 * accumulator states, computed with the mix this call draws, are injected before the step
 * (r0hip_rv32im_bigint_accum_inject; witgen/mod.rs:182-205). Recursion takes none. The group is
 * accumulated over work_cycles cycles (rv32im: the preflight cycle count, 2^po2; recursion:
 * work_cycles), INVALID words are zeroized, and the group is committed. The other arguments
 * are r0hip_prove_segment's. */
const char* r0hip_prove_segment_accum(const char* circuit, int suite, uint32_t po2, const uint32_t* d_code,
                                      const uint32_t* d_data, uint32_t* d_accum, size_t work_cycles,
                                      const r0hip_bigint_back* h_bigint, size_t n_bigint, uint32_t* d_global,
                                      int write_version, uint32_t version, uint32_t* h_seal, size_t seal_cap,
                                      size_t* seal_len, uint32_t* h_mix_out);
/* ---- rv32im witness side: accumulation phases 2-3 (risc0_circuit_rv32im_cuda_accum after its
 * stepAccum kernel, rv32im-sys/kernels/cuda/ffi.cu:480-509; CPU ffi.cpp:326-360): inclusive
 * prefix sums of the last 4 accum columns over rows [0, last_cycle), then every row adds the
 * previous row's prefix values to the machine columns [23, cols - 4). d_accum is the accum
 * group, column-major with `rows` rows, after the per-cycle phase (r0hip_rv32im_accum runs both). */
const char* r0hip_rv32im_accum_finalize(uint32_t* d_accum, size_t rows, size_t cols, size_t last_cycle);
/* ---- rv32im witness side: the whole accumulation (risc0_circuit_rv32im_cuda_accum,
 * rv32im-sys/kernels/cuda/ffi.cu:362-514; CPU risc0_circuit_rv32im_cpu_accum, ffi.cpp:313-368):
 * phase 1, the per-cycle accumulation step (stepAccum, ffi.cpp:238-247, generated from the
 * reference's step_TopAccum), for cycles [0, last_cycle), then phases 2-3 as above. d_data is
 * the data group (211 columns), d_accum the accum group (cols = 103) as the prover allocates
 * it (every word INVALID, 0xFFFFFFFF); d_global (90 words) and d_mix (36 words) as in
 * AccumBuffers (witgen.h). Columns are `rows` long. */
const char* r0hip_rv32im_accum(const uint32_t* d_data, uint32_t* d_accum, const uint32_t* d_global,
                               const uint32_t* d_mix, size_t rows, size_t cols, size_t last_cycle);

/* ---- rv32im witness generation (risc0_circuit_rv32im_cuda_witgen / _cpu_witgen,
 * rv32im-sys/kernels/cuda/ffi.cu:431-472, kernels/cxx/ffi.cpp:267-308; bound in
 * rv32im-sys/src/lib.rs:55-86 and called from circuit/rv32im/src/prove/hal/cuda.rs:60-101) ----
 * The same three structs the reference passes (RawBuffer, RawExecBuffers, RawPreflightTrace,
 * rv32im-sys/src/lib.rs:20-76), field for field. buffers->global (rows 1, cols 90) and
 * buffers->data (cols 211, rows a power of two) are DEVICE pointers: the global vector as
 * build_global_vec makes it and the data group all INVALID with the injector scattered in
 * (witgen/mod.rs:146-162; r0hip_scatter). preflight's arrays are HOST pointers, as in the
 * reference: `cycles` RawPreflightCycle records (36 bytes), txns RawMemoryTransaction (20
 * bytes), bigint_bytes. step_Top runs for cycles [0, cycles) in the reference's two phases
 * (before and after table_split_cycle). mode (0 parallel, 1 forward, 2 reverse) is checked and
 * every mode runs the parallel schedule, which gives the same words on any trace the
 * reference accepts. Fails as the reference throws: EQZ ("eqz failure at: ..."), a
 * transaction at another cycle or address, reads of unset words, inconsistent re-stores, bad
 * lookups. Zeroize stays the caller's (witgen/mod.rs:166-170). */
typedef struct r0hip_raw_buffer {
  uint32_t* buf;
  size_t rows;
  size_t cols;
  bool checked;
} r0hip_raw_buffer;
typedef struct r0hip_raw_exec_buffers {
  r0hip_raw_buffer global;
  r0hip_raw_buffer data;
} r0hip_raw_exec_buffers;
typedef struct r0hip_raw_preflight_trace {
  const void* cycles;
  const void* txns;
  const uint8_t* bigint_bytes;
  uint32_t txns_len;
  uint32_t bigint_bytes_len;
  uint32_t table_split_cycle;
} r0hip_raw_preflight_trace;
const char* r0hip_rv32im_witgen(uint32_t mode, const r0hip_raw_exec_buffers* buffers,
                                const r0hip_raw_preflight_trace* preflight, uint32_t cycles);

/* ---- rv32im prove_core from a preflight trace: SegmentProverImpl::prove_core
 * (circuit/rv32im/src/prove/hal/mod.rs:143-224) over WitnessGenerator::new and ::accum
 * (witgen/mod.rs:106-223), every step on the device ----
 * h_global: build_global_vec's 90 Montgomery words (INVALID where unset, witgen/mod.rs:272-327).
 * The injector (Injector, witgen/mod.rs:329-378) as hal.scatter takes it: h_inj_index
 * (inj_rows + 1 entries), h_inj_offsets / h_inj_values (h_inj_index[inj_rows] entries:
 * col * 2^po2 + row, Montgomery value). preflight as r0hip_rv32im_witgen takes it (cycles =
 * 2^po2 records); mode as there. h_bigint / n_bigint: the trace's Back::BigInt records, as
 * r0hip_prove_segment_accum takes them. Runs: data INVALID, scatter, stepExec (both phases),
 * zeroize, then the prove_core sequence with the version word 2 (RV32IM_SEAL_VERSION) and the
 * accumulation on the device. Seal and mix out as r0hip_prove_segment. */
/* Host arrays of 64 KiB or more that lie inside r0hip_host_alloc blocks are copied to the
 * device directly; others are staged through the calling thread's page-locked arena. */
const char* r0hip_prove_segment_trace(int suite, uint32_t po2, uint32_t mode, const uint32_t* h_global,
                                      const uint32_t* h_inj_index, size_t inj_rows, const uint32_t* h_inj_offsets,
                                      const uint32_t* h_inj_values, const r0hip_raw_preflight_trace* preflight,
                                      const r0hip_bigint_back* h_bigint, size_t n_bigint, uint32_t* h_seal,
                                      size_t seal_cap, size_t* seal_len, uint32_t* h_mix_out);

/* The same with every input already resident in device memory (the global vector, the
 * injector arrays, and d_preflight's cycles / txns / bigint_bytes are DEVICE pointers; the
 * struct itself and h_bigint are on the host): what the benchmark times, inputs in HBM.
 * Injector offsets outside the data group are skipped. */
const char* r0hip_prove_segment_trace_resident(int suite, uint32_t po2, uint32_t mode, const uint32_t* d_global,
                                               const uint32_t* d_inj_index, size_t inj_rows,
                                               const uint32_t* d_inj_offsets, const uint32_t* d_inj_values,
                                               const r0hip_raw_preflight_trace* d_preflight,
                                               const r0hip_bigint_back* h_bigint, size_t n_bigint, uint32_t* h_seal,
                                               size_t seal_cap, size_t* seal_len, uint32_t* h_mix_out);

/* ---- recursion witness side: the accumulation step (risc0_circuit_recursion_cuda_accum,
 * recursion-sys/kernels/cuda/ffi.cu; CPU driver recursion-sys/kernels/cxx/ffi.cpp:160-217,
 * called from circuit/recursion/src/prove/witgen.rs:162-170): for cycles [0, work_cycles) the
 * per-cycle accumulator factors (step_compute_accum), their inclusive prefix product, and the
 * accum-group registers (step_verify_accum) written into d_accum. Groups are column-major with
 * total_cycles rows (a power of two); d_mix holds the mix values, d_global the globals. Cells
 * no step writes are left as they were (the reference leaves them INVALID for the caller to
 * zeroize, witgen.rs:172-175). */
const char* r0hip_recursion_accum(const uint32_t* d_ctrl, const uint32_t* d_global, const uint32_t* d_data,
                                  const uint32_t* d_mix, uint32_t* d_accum, size_t work_cycles,
                                  size_t total_cycles);

/* ---- recursion witness generation (risc0_circuit_recursion_cuda_witgen / _cpu_witgen,
 * recursion-sys/kernels/cxx/ffi.cpp:191-205, driven by circuit/recursion/src/prove/witgen.rs:
 * 91-100 in StepMode::Parallel) ----
 * From the control group (d_ctrl, 23 columns x total_cycles rows, the program's rows first)
 * and the preflight trace (RawPreflightTrace, prove/preflight.rs): h_wom the write-once
 * memory (n_wom FpExt, 4 Montgomery words each), h_cycles {iopIdx, isParSafe} per work
 * cycle (n_cycles pairs of words), h_iops the IOP values read (n_iops FpExt). Fills d_data
 * (128 columns x total_cycles, INVALID-filled by the caller as witgen.rs:68-72 allocates it)
 * and d_global (32 words, INVALID-filled): step_exec per cycle (runs of non-parallel-safe
 * cycles in order), the WOM argument sorted and scanned, injectWomBacks, step_verify_mem.
 * Fails with the reference's message on a failed check ("eqz failed at: ..."). ZK noise and
 * zeroize stay the caller's (witgen.rs:101-123). */
const char* r0hip_recursion_witgen(const uint32_t* d_ctrl, uint32_t* d_data, uint32_t* d_global, size_t total_cycles,
                                   const uint32_t* h_wom, size_t n_wom, const uint32_t* h_cycles, size_t n_cycles,
                                   const uint32_t* h_iops, size_t n_iops);
/* A whole recursion proof from a program and its preflight (RecursionProverImpl::prove,
 * circuit/recursion/src/prove/mod.rs:160-230): witness generation as above, ZK noise in the
 * last 1024 rows of data and accum (per-cell values of r0hip_fill_uniform(noise_seed) and
 * (noise_seed + 1), laid out as witgen.rs:101-158 copies its noise matrices), zeroize, then
 * r0hip_prove_segment_accum's sequence with work cycles = n_cycles. po2 >= 11 and n_cycles <=
 * 2^po2 - 1024 (program.rs:57). Seal and mix out as r0hip_prove_segment. */
const char* r0hip_prove_recursion(int suite, uint32_t po2, const uint32_t* d_ctrl, const uint32_t* h_wom, size_t n_wom,
                                  const uint32_t* h_cycles, size_t n_cycles, const uint32_t* h_iops, size_t n_iops,
                                  uint64_t noise_seed, uint32_t* h_seal, size_t seal_cap, size_t* seal_len,
                                  uint32_t* h_mix_out);

/* ---- segment pipeline (r0vm's per-GPU worker queue, r0vm/src/actors/worker.rs:75-76, over the
 * zkvm's per-segment prove loop, zkvm/src/host/server/prove/prover_impl.rs:84-94) ----
 * Proves njobs segments of one (circuit, suite, po2) from HOST witness groups: an uploader thread
 * copies each job's groups into one of in_flight+1 device buffer sets, in 48-column chunks, while
 * in_flight provers (in_flight - 1 threads and the calling thread) prove on their own streams; a
 * prover starts a job at once and commits each group chunk by chunk as it lands (Poseidon2 and
 * SHA-256; Poseidon254 waits for whole groups). Host buffers must stay valid until the call
 * returns and should be page-locked (r0hip_host_alloc) for full PCIe rate. Per job: seal into
 * h_seal (seal_cap words), its length in seal_len, mix values into h_mix_out (optional), and
 * error = NULL or a malloc'd message (free() it). Returns NULL when every job succeeded. Seals
 * equal r0hip_prove_segment's. (Round 5 appended a `trace` pointer to this struct; trace jobs
 * now have their own entry point below and this struct has its round-4 layout again.) */
typedef struct r0hip_segment_job {
  const uint32_t* h_code;
  const uint32_t* h_data;
  const uint32_t* h_accum;  /* rv32im: NULL = accumulate on the device (as r0hip_prove_segment_accum,
                               work cycles 2^po2); the group then never crosses PCIe */
  const uint32_t* h_global; /* output_size words; zeroized on the device copy only */
  const r0hip_bigint_back* h_bigint; /* device accumulation only: the trace's BigInt backs, as */
  size_t n_bigint;                   /* r0hip_prove_segment_accum takes them (NULL, 0 if none) */
  uint32_t* h_seal;
  size_t seal_cap;
  size_t seal_len;
  uint32_t* h_mix_out;
  const char* error;
} r0hip_segment_job;
const char* r0hip_prove_segments(const char* circuit, int suite, uint32_t po2, int write_version, uint32_t version,
                                 r0hip_segment_job* jobs, size_t njobs, uint32_t in_flight);

/* ---- the GPU worker unit from preflight traces: rv32im SegmentProverImpl::prove_core
 * (circuit/rv32im/src/prove/hal/mod.rs:143-224) per job, as r0vm's GPU worker runs it from the
 * executor's segments (r0vm/src/actors/worker.rs:186-260, job/proof.rs:238-323), with the CUDA
 * prove_core's trace upload (circuit/rv32im/src/prove/witgen/mod.rs:135-176) done by an uploader
 * thread: the trace, the injector and the global vector go into one of in_flight+1 device trace
 * sets while in_flight provers (in_flight - 1 threads and the calling thread) run witness
 * generation, accumulation and the proof from the others. The injector is checked on the host as
 * r0hip_prove_segment_trace checks it. Seals equal r0hip_prove_segment_trace's (version word 2).
 * verify != 0: every seal is checked by r0hip_verify_seal (the validity equation included) on a
 * host thread while the GPU proves the next jobs, as ProverImpl::prove_segment_core verifies a
 * receipt before returning it (zkvm/src/host/server/prove/prover_impl.rs:262-280); a seal that
 * fails sets that job's error ("receipt verification failed: ...") and the other jobs still
 * return. Host arrays must stay valid until the call returns. */
typedef struct r0hip_trace_input {
  uint32_t mode;                      /* as r0hip_rv32im_witgen */
  const uint32_t* h_global;           /* build_global_vec's 90 Montgomery words */
  const uint32_t* h_inj_index;        /* inj_rows + 1 entries */
  size_t inj_rows;
  const uint32_t* h_inj_offsets;      /* h_inj_index[inj_rows] entries each */
  const uint32_t* h_inj_values;
  r0hip_raw_preflight_trace preflight; /* host pointers; 2^po2 cycle records */
} r0hip_trace_input;
typedef struct r0hip_trace_job {
  r0hip_trace_input trace;
  const r0hip_bigint_back* h_bigint;  /* the trace's BigInt backs (NULL, 0 if none) */
  size_t n_bigint;
  uint32_t* h_seal;                   /* out: the seal (seal_cap words), its length in seal_len */
  size_t seal_cap;
  size_t seal_len;
  uint32_t* h_mix_out;                /* out (optional): the 36 mix words */
  const char* error;                  /* out: NULL or a malloc'd message (free() it) */
  int verified;                       /* out: 1 when the seal passed r0hip_verify_seal */
  double verify_ms;                   /* out: host milliseconds of that check */
  double prove_ms;                    /* out: host milliseconds from a prover taking the job to its
                                         seal in host memory (the wait for its upload included) */
} r0hip_trace_job;
const char* r0hip_prove_trace_segments(int suite, uint32_t po2, r0hip_trace_job* jobs, size_t njobs,
                                       uint32_t in_flight, int verify);

/* ---- seal verification (risc0/zkp/src/verify/mod.rs:500-560 `verify`, with merkle.rs:79-186,
 * fri.rs:36-155, read_iop.rs:20-84; rv32im seals lead with the version word 2,
 * circuit/rv32im/src/lib.rs:78-92) ----
 * Replays the transcript and checks the constraint validity equation poly_ext(z) ==
 * check(z) * ((3z)^N - 1) (mod.rs:340-394), every Merkle opening, every FRI fold, the final
 * FRI polynomial, that every field word read is canonical (read_field_elem_slice,
 * read_iop.rs:45-48) and the seal length. check_code (mod.rs:531): the code/control root is
 * written to h_code_root_out (8 words, if non-NULL), and when n_code_roots > 0 it must equal
 * one of the n_code_roots digests at h_code_roots (8 words each) — the recursion circuit's
 * control-id allow-list (zkvm/src/receipt/succinct.rs:143-157). Host-only: needs no GPU and
 * no r0hip_init. Returns NULL when the seal verifies (po2 of the segment in *po2_out, if
 * non-NULL), else the failed check. */
const char* r0hip_verify_seal(const char* circuit, int suite, const uint32_t* seal, size_t seal_len,
                              const uint32_t* h_code_roots, size_t n_code_roots, uint32_t* h_code_root_out,
                              uint32_t* po2_out);
/* TESTING ONLY — never use it to accept a receipt. r0hip_verify_seal without the validity
 * equation and without a code-root check, for seals of synthetic witnesses (which do not
 * satisfy the constraints) in the parity tests. */
const char* r0hip_testing_verify_seal_structure(const char* circuit, int suite, const uint32_t* seal,
                                                size_t seal_len, uint32_t* po2_out);
/* PolyExt::poly_ext of the circuit (its generated poly_ext.rs, called at mod.rs:356-386): the
 * constraint polynomial at the out-of-domain point. h_mix (mix_size) and h_global
 * (output_size) are Montgomery words, h_eval_u one FpExt (4 words) per tap in tap order,
 * h_poly_mix one FpExt; the result FpExt goes to h_out. Host-only. */
const char* r0hip_poly_ext(const char* circuit, const uint32_t* h_mix, const uint32_t* h_global,
                           const uint32_t* h_eval_u, const uint32_t* h_poly_mix, uint32_t* h_out);

/* kernel-level timing with HIP events on the library stream: enable, run, then read
 * "name=total_ms:calls:alg_bytes;..." (alg_bytes = algorithmic HBM bytes) */
const char* r0hip_set_kernel_timing(int on);
const char* r0hip_kernel_times(char* buf, size_t cap);
/* per-phase device timings (ms) of the last r0hip_prove_segment, as "name=ms;..." */
const char* r0hip_last_profile(char* buf, size_t cap);

/* Device-memory accounting, replacing the reference HAL's MemoryTracker
 * (risc0/zkp/src/hal/mod.rs:292-317, reported as the datasheet's `ram`,
 * risc0/zkvm/examples/datasheet.rs:251). out[5] = {live bytes (buffers handed out),
 * peak live bytes, reserved bytes (held from hipMalloc incl. the free pool), peak
 * reserved bytes, number of hipMalloc calls}. Peaks are since the last reset. Host-only. */
const char* r0hip_mem_stats(uint64_t* out);
const char* r0hip_mem_reset_peak(void);
/* Release the idle device memory the library holds: the calling thread's free pool and
 * the blocks exited threads left (pool and scratch). Blocks in use are untouched. For a
 * caller switching segment sizes, and for tests that need a clean pool. */
const char* r0hip_trim(void);

#ifdef __cplusplus
}
#endif
#endif /* R0HIP_H */
