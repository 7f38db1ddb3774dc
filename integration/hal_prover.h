/*
 * The drop-in per-op path, driven natively: the reference's segment prover
 * (risc0_zkp::prove::Prover, zkp/src/prove/prover.rs:38-393, with poly_group.rs, merkle.rs,
 * fri.rs) and the rv32im prove_core around it (circuit/rv32im/src/prove/hal/mod.rs:143-224,
 * witgen/mod.rs:106-223) restated in C++ over ONLY the per-op symbols of include/r0hip.h, one
 * call per Hal / CircuitHal method, exactly as integration/rust/hal_hip.rs and
 * circuit_hal_hip.rs bind them. This is what a Rust `HipHal` behind `risc0_zkp::hal::Hal`
 * delivers (every call synchronous, `has_unified_memory() = false`, so Merkle openings are one
 * device-to-host copy per node), measured without Rust, which this image lacks.
 *
 * Not part of the product: libr0hip_halprover.so links libr0hip.so and calls no fused entry
 * point (tests/test_abi.py checks its undefined symbols). Host-side hashing and the transcript
 * use the product's host transcript (risc0_amd/csrc/transcript.h), the role of risc0-zkp's CPU
 * HashSuite in the reference (hal.get_hash_suite(), cuda.rs:974-976).
 */
#ifndef R0HIP_HAL_PROVER_H
#define R0HIP_HAL_PROVER_H
#include <stddef.h>
#include <stdint.h>

#include "../include/r0hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* A circuit's TapSet (zkp/src/taps.rs:57-66) and CircuitInfo (adapter.rs:122-126), as the circuit
 * crate supplies them to the prover: risc0_amd/circuits/<c>.taps.json. */
typedef struct halp_taps {
  const uint32_t* taps;        /* n_taps x {offset, back, group, combo, skip} */
  size_t n_taps;
  const uint32_t* combo_taps;  /* combo_begin[combos_count] entries */
  const uint32_t* combo_begin; /* combos_count + 1 */
  size_t combos_count;
  const uint32_t* group_begin; /* 4: taps of group g are [group_begin[g], group_begin[g + 1]) */
  const uint32_t* group_sizes; /* 3: accum, code, data */
  const char* circuit_info;    /* 16 bytes */
  size_t mix_size;
  size_t output_size;
} halp_taps;

/* Per-phase host milliseconds of the last call on this thread, "name=ms;..." */
const char* halp_last_profile(char* buf, size_t cap);

/* The prove core over device witness groups (Prover::commit_group x3 + finalize), with the
 * accumulation between the mix draw and the accum commit when accum_mode != 0:
 *   0  d_accum holds the finished accum group;
 *   1  rv32im WitnessGenerator::accum (witgen/mod.rs:178-221): d_accum INVALID-filled by this
 *      call, the BigInt states injected (r0hip_rv32im_bigint_accum_inject), r0hip_rv32im_accum
 *      over work_cycles cycles, zeroize;
 *   2  recursion (prove/witgen.rs:138-177): d_accum as the caller prepared it (INVALID plus ZK
 *      noise rows), r0hip_recursion_accum over work_cycles, zeroize.
 * d_global (output_size words) is zeroized in place; seal and mix out as r0hip_prove_segment. */
const char* halp_prove_segment(const char* circuit, const halp_taps* taps, int suite, uint32_t po2,
                               const uint32_t* d_code, const uint32_t* d_data, uint32_t* d_accum, uint32_t* d_global,
                               int accum_mode, size_t work_cycles, const r0hip_bigint_back* h_bigint, size_t n_bigint,
                               int write_version, uint32_t version, uint32_t* h_seal, size_t seal_cap, size_t* seal_len,
                               uint32_t* h_mix_out);

/* rv32im SegmentProverImpl::prove_core from a preflight trace (host arrays, as
 * r0hip_prove_segment_trace takes them) over the per-op path: WitnessGenerator::new
 * (witgen/mod.rs:106-176: data INVALID, r0hip_scatter of the injector, r0hip_rv32im_witgen,
 * zeroize; code all 0), then halp_prove_segment with accum_mode 1 and the version word 2. */
const char* halp_prove_trace(const halp_taps* taps, int suite, uint32_t po2, uint32_t mode, const uint32_t* h_global,
                             const uint32_t* h_inj_index, size_t inj_rows, const uint32_t* h_inj_offsets,
                             const uint32_t* h_inj_values, const r0hip_raw_preflight_trace* preflight,
                             const r0hip_bigint_back* h_bigint, size_t n_bigint, uint32_t* h_seal, size_t seal_cap,
                             size_t* seal_len, uint32_t* h_mix_out);

#ifdef __cplusplus
}
#endif
#endif /* R0HIP_HAL_PROVER_H */
