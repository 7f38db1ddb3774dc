// Interface between the host driver and the generated per-circuit eval_check
// kernels (risc0_amd/csrc/gen/eval_check_<circuit>.hip, emitted at build time by
// tools/gen_eval_check.py from risc0_amd/circuits/<circuit>.poly.ir).
#pragma once
#include "runtime.h"

namespace r0 {

struct EvalCheckArgs {
  const uint32_t* const* args;  // poly_fp argument buffers, circuit order
  size_t nargs;
  const uint32_t* const* colptr;  // device table: base pointer of every column the program reads
  const uint32_t* poly_mix;     // poly_mix powers + folded products (FpExt AoS, Montgomery)
  const uint32_t* poly_mix_nb;  // the same table times NBETA = -11 (lazy extension products)
  uint32_t* acc;                // scratch: domain x FpExt
  uint32_t* check;              // out: 4 x domain
  const uint32_t* vinv;         // 4 values: inv((3 w^c)^N - 1) for c = 0..3
  uint32_t* mat_fp;             // scratch: mat_fp x domain words
  uint32_t* mat_ext;            // scratch: mat_ext x domain FpExt
  uint32_t domain;
  uint32_t tile = 0;            // points per tile (0 = whole domain per launch)
  int64_t wide = -1;            // bit k: kernel k addresses taps from colptr (-1 = tuned default)
  const uint32_t* uniform = nullptr;  // info.uniform's table (4 words per value), on the device
};

struct EvalCheckInfo {
  const int* combos;  // for each folded product: count, then indices into the powers
  int ncombos;
  int npm;            // number of poly_mix powers the kernels index directly
  int nargs;
  int mat_fp, mat_ext, kernels;
  double modmuls_per_point;  // field multiplications of the restated poly_fp (+4 for the 1/Z scale)
  int ncols;             // columns the program reads: (argument, column) pairs
  const int* col_arg;
  const int* col_idx;
  // lane-independent values the kernels read (4 words each), evaluated on the host from host
  // copies of the eval_check arguments (only mix and global are read: g[i] null otherwise)
  // and the poly_mix powers (FpExt AoS)
  int n_uniform;
  void (*uniform)(const uint32_t* const* g, const uint32_t* poly_mix, uint32_t* out);
};

void eval_check_rv32im(hipStream_t s, const EvalCheckArgs& e);
void eval_check_rv32im_info(EvalCheckInfo* info);
void eval_check_recursion(hipStream_t s, const EvalCheckArgs& e);
void eval_check_recursion_info(EvalCheckInfo* info);

}  // namespace r0
