// ORACLE (test infrastructure only — never linked into the product path).
//
// C ABI of the CPU oracle library (oracle/liboracle.so). Only tests/, the smoke
// check in __graft_entry__.py and bench.py's cpu_baseline leg load it.
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// Per-point constraint polynomial, the reference's generated C++ `poly_fp`
// (rv32im-sys/kernels/cxx/eval_check.cpp:30-39 signature). Built from the
// reference sources by oracle/Makefile into oracle/_ref/ (checker only).
typedef const char* (*oracle_poly_fp_fn)(size_t cycle, size_t steps, const uint32_t* poly_mix,
                                         const uint32_t** args, uint32_t* result);

// Circuit description; mirrors risc0_zkp::taps::TapSet (zkp/src/taps.rs:57-66)
// plus the circuit's CircuitInfo (adapter.rs:122-126) and eval_check arg order.
typedef struct {
  const uint32_t* taps;  // n_taps x {offset, back, group, combo, skip}
  size_t n_taps;
  const uint32_t* combo_taps;
  const uint32_t* combo_begin;  // combos_count + 1 entries
  size_t combos_count;
  const uint32_t* group_begin;  // n_groups + 1 entries
  size_t n_groups;
  const uint32_t* poly_mix_powers;
  size_t n_poly_mix;
  const uint8_t* circuit_info;  // 16 bytes
  size_t mix_size;
  size_t output_size;
  const int32_t* eval_args;  // >=0: register group id; -1: mix global; -2: out global
  size_t n_eval_args;
  oracle_poly_fp_fn poly_fp;
} oracle_circuit_t;

// Proves one segment with the CPU oracle: restates the circuit segment prover
// (circuit/rv32im/src/prove/hal/mod.rs:143-224, circuit/recursion/src/prove/mod.rs:164-230)
// on top of risc0_zkp::prove::Prover (zkp/src/prove/prover.rs). `global` is
// zeroized in place (valid_or_zero). Mix values are drawn from the transcript and
// returned in mix_out (mix_size words). Returns NULL or an error string.
const char* oracle_prove_segment(const oracle_circuit_t* c, int suite, uint32_t po2,
                                 const uint32_t* code, const uint32_t* data,
                                 const uint32_t* accum, uint32_t* global, int write_version,
                                 uint32_t version, uint32_t* seal, size_t seal_cap,
                                 size_t* seal_len, uint32_t* mix_out);

// eval_check with the reference C++ poly_fp (rv32im/src/prove/hal/cpu.rs:145-207).
// groups[g] = evaluated group g (size[g] x domain), check = 4 x domain.
const char* oracle_eval_check(const oracle_circuit_t* c, uint32_t* check, const uint32_t** groups,
                              const uint32_t* mix, const uint32_t* global,
                              const uint32_t* poly_mix, uint32_t po2);

// eval_check of groups filled by r0hip_fill_uniform(group_seeds[g]) at po2, evaluated only
// at the n given cycles (out: n x 4 words, point-major), for full-size parity tests.
const char* oracle_eval_check_sampled(const oracle_circuit_t* c, const uint64_t* group_seeds,
                                      const uint32_t* mix, const uint32_t* global,
                                      const uint32_t* poly_mix, uint32_t po2, const uint64_t* cycles,
                                      size_t n, uint32_t* out);

#ifdef __cplusplus
}
#endif
