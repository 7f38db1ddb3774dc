// Circuit descriptions compiled into the library: the TapSet
// (risc0/zkp/src/taps.rs:57-66), CircuitInfo (adapter.rs:122-126), the order of the
// eval_check argument buffers, and the generated eval_check entry points.
// The tables come from risc0_amd/circuits/*.taps.json via tools/gen_circuits_inc.py.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>

#include "evalcheck.h"

namespace r0 {

struct CircuitDef {
  const char* name;
  const uint32_t* taps;  // n_taps x {offset, back, group, combo, skip}
  size_t n_taps;
  const uint32_t* combo_taps;
  size_t n_combo_taps;
  const uint32_t* combo_begin;  // combos_count + 1
  size_t combos_count;
  const uint32_t* group_begin;  // n_groups + 1
  size_t n_groups;
  const uint32_t* group_sizes;
  const uint32_t* poly_mix_powers;
  size_t n_poly_mix;
  const char* circuit_info;  // 16 bytes
  size_t mix_size, output_size;
  const int* eval_args;  // >= 0 register group, -1 mix, -2 out (global)
  size_t n_eval_args;
  void (*eval_check)(hipStream_t, const EvalCheckArgs&);
  void (*info)(EvalCheckInfo*);
  // the constraint program for the host poly_ext (verify.cpp): n_ir records of
  // {op, dst, a, b, c, d}, op index into "celg+-*abr", dst dense 0..n_ir-1
  const uint32_t* ir;
  size_t n_ir;

  struct Tap {
    uint32_t offset, back, group, combo, skip;
  };
  const Tap& tap(size_t i) const { return reinterpret_cast<const Tap*>(taps)[i]; }
  size_t group_size(size_t g) const { return tap(group_begin[g + 1] - 1).offset + 1; }
  // RegisterIter (taps.rs:202-227): calls f(first tap index of each register)
  template <typename F>
  void regs(size_t begin, size_t end, F f) const {
    size_t cur = begin;
    while (cur < n_taps) {
      size_t next = cur + tap(cur).skip;
      if (next > end) break;
      f(cur);
      cur = next;
    }
  }
};

const CircuitDef* find_circuit(const std::string& name);

}  // namespace r0
