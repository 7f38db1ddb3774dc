// ORACLE (test infrastructure only — never linked into the product path).
//
// C-ABI restatement of risc0_zkp::hal::cpu::CpuHal (risc0/zkp/src/hal/cpu.rs:263-651)
// plus the default trait methods combos_prepare / combos_divide
// (risc0/zkp/src/hal/mod.rs:202-257). Buffers are host arrays of raw Montgomery
// u32 words; ExtElem buffers are 4 consecutive words per element (AoS), Digest
// buffers 8 words per digest. Sizes are in elements of the buffer's type.
#include <cstring>
#include <vector>

#include "core.h"
#include "oracle.h"

using namespace oracle;

static inline Elem* E(uint32_t* p) { return reinterpret_cast<Elem*>(p); }
static inline const Elem* E(const uint32_t* p) { return reinterpret_cast<const Elem*>(p); }
static inline ExtElem* X(uint32_t* p) { return reinterpret_cast<ExtElem*>(p); }
static inline const ExtElem* X(const uint32_t* p) { return reinterpret_cast<const ExtElem*>(p); }
static inline Digest* D(uint32_t* p) { return reinterpret_cast<Digest*>(p); }

extern "C" {

// cpu.rs:305-340
void oracle_batch_expand_into_evaluate_ntt(uint32_t* output, size_t out_size, const uint32_t* input,
                                           size_t in_size, size_t count, size_t expand_bits) {
  size_t out_row = out_size / count, in_row = in_size / count;
  size_t eb = log2_ceil(out_row / in_row);
  parallel_for(count, [&](size_t b, size_t e) {
    for (size_t r = b; r < e; r++) expand(E(output) + r * out_row, E(input) + r * in_row, in_row, eb);
  });
  parallel_for(count, [&](size_t b, size_t e) {
    for (size_t r = b; r < e; r++) evaluate_ntt(E(output) + r * out_row, out_row, expand_bits);
  });
}

// cpu.rs:342-350
void oracle_batch_interpolate_ntt(uint32_t* io, size_t size, size_t count) {
  size_t row = size / count;
  parallel_for(count, [&](size_t b, size_t e) {
    for (size_t r = b; r < e; r++) interpolate_ntt(E(io) + r * row, row);
  });
}

// cpu.rs:352-360
void oracle_batch_bit_reverse(uint32_t* io, size_t size, size_t count) {
  size_t row = size / count;
  parallel_for(count, [&](size_t b, size_t e) {
    for (size_t r = b; r < e; r++) bit_reverse(E(io) + r * row, row);
  });
}

// cpu.rs:362-393
void oracle_batch_evaluate_any(const uint32_t* coeffs, size_t coeffs_size, size_t poly_count,
                               const uint32_t* which, const uint32_t* xs, uint32_t* out,
                               size_t eval_count) {
  size_t po2 = log2_ceil(coeffs_size / poly_count);
  size_t count = size_t(1) << po2;
  parallel_for(eval_count, [&](size_t b, size_t e) {
    for (size_t k = b; k < e; k++) {
      ExtElem tot = ExtElem::zero(), cur = ExtElem::one();
      ExtElem x = X(xs)[k];
      const Elem* local = E(coeffs) + count * which[k];
      for (size_t i = 0; i < count; i++) {
        tot += cur * local[i];
        cur *= x;
      }
      X(out)[k] = tot;
    }
  });
}

// cpu.rs:395-408
void oracle_zk_shift(uint32_t* io, size_t size, size_t poly_count) {
  size_t bits = log2_ceil(size / poly_count);
  parallel_for(size, [&](size_t b, size_t e) {
    for (size_t idx = b; idx < e; idx++) {
      size_t pos = idx & ((size_t(1) << bits) - 1);
      uint32_t rev = bits ? (bit_rev_32((uint32_t)pos) >> (32 - bits)) : 0;
      Elem pow3 = Elem::from(3).pow(rev);
      E(io)[idx] = E(io)[idx] * pow3;
    }
  });
}

// cpu.rs:410-455
void oracle_mix_poly_coeffs(uint32_t* output, size_t out_size, const uint32_t* mix_start,
                            const uint32_t* mix, const uint32_t* input, const uint32_t* combos,
                            size_t input_size, size_t count) {
  ExtElem mix_cur = ExtElem::raw(mix_start), m = ExtElem::raw(mix);
  std::vector<ExtElem> mix_pows(input_size);
  for (size_t i = 0; i < input_size; i++) {
    mix_pows[i] = mix_cur;
    mix_cur *= m;
  }
  size_t chunks = out_size / count;
  parallel_for(chunks, [&](size_t b, size_t e) {
    for (size_t id = b; id < e; id++) {
      ExtElem* out_chunk = X(output) + id * count;
      for (size_t i = 0; i < input_size; i++) {
        if (combos[i] != id) continue;
        for (size_t idx = 0; idx < count; idx++)
          out_chunk[idx] += mix_pows[i] * E(input)[count * i + idx];
      }
    }
  });
}

// cpu.rs:457-473
void oracle_eltwise_add_elem(uint32_t* out, const uint32_t* a, const uint32_t* b, size_t n) {
  for (size_t i = 0; i < n; i++) E(out)[i] = E(a)[i] + E(b)[i];
}

// cpu.rs:475-500
void oracle_eltwise_sum_extelem(uint32_t* output, size_t out_size, const uint32_t* input,
                                size_t in_size) {
  size_t count = out_size / 4, to_add = in_size / count;
  parallel_for(count, [&](size_t b, size_t e) {
    for (size_t idx = b; idx < e; idx++) {
      ExtElem sum = ExtElem::zero();
      for (size_t i = 0; i < to_add; i++) sum += X(input)[i * count + idx];
      for (size_t i = 0; i < 4; i++) E(output)[i * count + idx] = sum.e[i];
    }
  });
}

// cpu.rs:502-516
void oracle_eltwise_copy_elem(uint32_t* out, const uint32_t* in, size_t n) {
  memcpy(out, in, n * 4);
}

// cpu.rs:518-522
void oracle_eltwise_zeroize_elem(uint32_t* io, size_t n) {
  for (size_t i = 0; i < n; i++) E(io)[i] = E(io)[i].valid_or_zero();
}

// cpu.rs:524-553 (FRI_FOLD = 16)
void oracle_fri_fold(uint32_t* output, size_t out_size, const uint32_t* input, const uint32_t* mix) {
  const size_t FOLD = 16;
  size_t count = out_size / 4;
  ExtElem m = ExtElem::raw(mix);
  for (size_t idx = 0; idx < count; idx++) {
    ExtElem tot = ExtElem::zero(), cur = ExtElem::one();
    for (size_t i = 0; i < FOLD; i++) {
      size_t rev_i = bit_rev_32((uint32_t)i) >> (32 - log2_ceil(FOLD));
      size_t rev_idx = rev_i * count + idx;
      ExtElem f;
      for (size_t k = 0; k < 4; k++) f.e[k] = E(input)[k * count * FOLD + rev_idx];
      tot += cur * f;
      cur *= m;
    }
    for (size_t k = 0; k < 4; k++) E(output)[count * k + idx] = tot.e[k];
  }
}

// cpu.rs:555-567
void oracle_hash_rows(int suite, uint32_t* output, size_t rows, const uint32_t* matrix,
                      size_t matrix_size) {
  size_t cols = matrix_size / rows;
  parallel_for(rows, [&](size_t b, size_t e) {
    std::vector<Elem> column(cols);
    for (size_t idx = b; idx < e; idx++) {
      for (size_t i = 0; i < cols; i++) column[i] = E(matrix)[i * rows + idx];
      D(output)[idx] = hash_elem_slice(suite, column.data(), cols);
    }
  });
}

// cpu.rs:569-581
void oracle_hash_fold(int suite, uint32_t* io, size_t input_size, size_t output_size) {
  Digest* d = D(io);
  parallel_for(output_size, [&](size_t b, size_t e) {
    for (size_t idx = b; idx < e; idx++)
      d[output_size + idx] = hash_pair(suite, d[input_size + 2 * idx], d[input_size + 2 * idx + 1]);
  });
}

// cpu.rs:583-596
void oracle_gather_sample(uint32_t* dst, const uint32_t* src, size_t idx, size_t size, size_t stride) {
  for (size_t g = 0; g < size; g++) dst[g] = src[g * stride + idx];
}

// cpu.rs:598-615
void oracle_scatter(uint32_t* into, const uint32_t* index, size_t index_len, const uint32_t* offsets,
                    const uint32_t* values) {
  if (index_len == 0) return;
  for (size_t cycle = 0; cycle + 1 < index_len; cycle++)
    for (uint32_t i = index[cycle]; i < index[cycle + 1]; i++) into[offsets[i]] = values[i];
}

// cpu.rs:617-635
void oracle_eltwise_copy_elem_slice(uint32_t* into, const uint32_t* from, size_t from_rows,
                                    size_t from_cols, size_t from_offset, size_t from_stride,
                                    size_t into_offset, size_t into_stride) {
  for (size_t r = 0; r < from_rows; r++)
    for (size_t c = 0; c < from_cols; c++)
      into[into_offset + r * into_stride + c] = from[from_offset + r * from_stride + c];
}

// cpu.rs:637-642
// rv32im accumulation, phases 2 and 3 of risc0_circuit_rv32im_cpu_accum
// (risc0/circuit/rv32im-sys/kernels/cxx/ffi.cpp:326-360): inclusive prefix sums of the
// last 4 accum columns over rows [0, last_cycle), then every row adds the previous row's
// (cyclically) prefix values to the machine columns [split, cols - 4), 4 at a time.
void oracle_rv32im_accum_finalize(uint32_t* accum, size_t rows, size_t cols, size_t split, size_t last_cycle) {
  Elem* a = E(accum);
  for (size_t j = 0; j < 4; j++) {
    Elem* c = a + (cols - 4 + j) * rows;
    for (size_t i = 1; i < last_cycle; i++) c[i] = c[i] + c[i - 1];
  }
  size_t machine_columns = (cols - split) / 4;
  for (size_t row = 0; row < last_cycle; row++) {
    size_t back1 = (row + last_cycle - 1) % last_cycle;
    Elem prev[4];
    for (size_t k = 0; k < 4; k++) prev[k] = a[(cols - 4 + k) * rows + back1];
    for (size_t j = 0; j + 1 < machine_columns; j++)
      for (size_t k = 0; k < 4; k++) {
        size_t col = split + j * 4 + k;
        a[col * rows + row] = a[col * rows + row] + prev[k];
      }
  }
}

void oracle_prefix_products(uint32_t* io, size_t n) {
  for (size_t i = 1; i < n; i++) X(io)[i] = X(io)[i] * X(io)[i - 1];
}

// hal/mod.rs:202-234 (CHECK_SIZE = INV_RATE * EXT_SIZE = 16)
void oracle_combos_prepare(uint32_t* combos, const uint32_t* coeff_u, size_t combo_count,
                           size_t cycles, const uint32_t* reg_sizes, const uint32_t* reg_combo_ids,
                           size_t reg_count, const uint32_t* mix) {
  ExtElem* c = X(combos);
  const ExtElem* u = X(coeff_u);
  ExtElem m = ExtElem::raw(mix);
  size_t cur_pos = 0;
  ExtElem cur = ExtElem::one();
  for (size_t r = 0; r < reg_count; r++) {
    for (size_t i = 0; i < reg_sizes[r]; i++) c[cycles * reg_combo_ids[r] + i] -= cur * u[cur_pos + i];
    cur *= m;
    cur_pos += reg_sizes[r];
  }
  for (size_t i = 0; i < 16; i++) {
    c[cycles * combo_count] -= cur * u[cur_pos];
    cur_pos++;
    cur *= m;
  }
}

// core/poly.rs:81-89
static ExtElem poly_divide(ExtElem* p, size_t n, ExtElem z) {
  ExtElem cur = ExtElem::zero();
  for (size_t i = n; i-- > 0;) {
    ExtElem next = z * cur + p[i];
    p[i] = cur;
    cur = next;
  }
  return cur;
}

// hal/mod.rs:236-257. chunk_pows: flattened z-powers; chunk_begin: prefix offsets
// (chunk i divides combos[i*cycles..] by each z in chunk_pows[chunk_begin[i]..chunk_begin[i+1]]).
// Returns the index of the first chunk with a nonzero remainder, or -1.
long oracle_combos_divide(uint32_t* combos, size_t nchunks, const uint32_t* chunk_pows,
                          const uint32_t* chunk_begin, size_t cycles) {
  std::vector<long> bad(nchunks, 0);
  parallel_for(nchunks, [&](size_t b, size_t e) {
    for (size_t i = b; i < e; i++)
      for (uint32_t k = chunk_begin[i]; k < chunk_begin[i + 1]; k++) {
        ExtElem rem = poly_divide(X(combos) + i * cycles, cycles, X(chunk_pows)[k]);
        if (rem != ExtElem::zero()) bad[i] = 1;
      }
  });
  for (size_t i = 0; i < nchunks; i++)
    if (bad[i]) return (long)i;
  return -1;
}

// ---- primitives exposed for known-answer tests ----------------------------
void oracle_poseidon2_mix(uint32_t* cells) { poseidon2_mix(E(cells)); }
void oracle_hash_elems(int suite, const uint32_t* e, size_t n, uint32_t* out) {
  *D(out) = hash_elem_slice(suite, E(e), n);
}
void oracle_hash_ext_elems(int suite, const uint32_t* e, size_t n, uint32_t* out) {
  *D(out) = hash_ext_elem_slice(suite, X(e), n);
}
void oracle_hash_pair(int suite, const uint32_t* a, const uint32_t* b, uint32_t* out) {
  *D(out) = hash_pair(suite, *reinterpret_cast<const Digest*>(a), *reinterpret_cast<const Digest*>(b));
}
void oracle_sha256_bytes(const uint8_t* b, size_t n, uint32_t* out) { *D(out) = sha256_hash_bytes(b, n); }
void oracle_interpolate_ntt(uint32_t* io, size_t n) { interpolate_ntt(E(io), n); }
void oracle_evaluate_ntt(uint32_t* io, size_t n, size_t expand_bits) { evaluate_ntt(E(io), n, expand_bits); }
void oracle_ext_mul(const uint32_t* a, const uint32_t* b, uint32_t* out) {
  (ExtElem::raw(a) * ExtElem::raw(b)).store(out);
}
void oracle_ext_inv(const uint32_t* a, uint32_t* out) { ExtElem::raw(a).inv().store(out); }
uint32_t oracle_encode(uint32_t x) { return Elem::from(x).v; }
uint32_t oracle_decode(uint32_t x) { return Elem::raw(x).as_u32(); }
uint32_t oracle_elem_pow(uint32_t x, uint64_t n) { return Elem::raw(x).pow(n).v; }

void* oracle_rng_new(int suite) { return new_rng(suite).release(); }
void oracle_rng_free(void* r) { delete static_cast<Rng*>(r); }
void oracle_rng_mix(void* r, const uint32_t* d) { static_cast<Rng*>(r)->mix(*reinterpret_cast<const Digest*>(d)); }
uint32_t oracle_rng_random_bits(void* r, size_t bits) { return static_cast<Rng*>(r)->random_bits(bits); }
uint32_t oracle_rng_random_elem(void* r) { return static_cast<Rng*>(r)->random_elem().v; }
void oracle_rng_random_ext_elem(void* r, uint32_t* out) {
  ExtElem e = static_cast<Rng*>(r)->random_ext_elem();
  for (int i = 0; i < 4; i++) out[i] = e.e[i].v;
}
size_t oracle_num_threads() { return num_threads(); }

}  // extern "C"
