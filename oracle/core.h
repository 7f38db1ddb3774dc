// ORACLE (test infrastructure only — never linked into the product path).
// CPU restatement of risc0-zkp's core primitives: NTT, Poseidon2, SHA-256 and the
// Fiat-Shamir RNGs. Each function cites the reference code it follows.
#pragma once
#include <cstdint>
#include <cstddef>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "field.h"

namespace oracle {

// ---- threading (rayon stand-in) -------------------------------------------
size_t num_threads();
void parallel_for(size_t n, const std::function<void(size_t begin, size_t end)>& f);

// ---- NTT: risc0/zkp/src/core/ntt.rs ---------------------------------------
uint32_t bit_rev_32(uint32_t x);                           // ntt.rs:34-45
size_t log2_ceil(size_t v);                                // core/mod.rs:52
void bit_reverse(Elem* io, size_t n);                      // ntt.rs:64-73
void interpolate_ntt(Elem* io, size_t n);                  // ntt.rs:232-281
void evaluate_ntt(Elem* io, size_t n, size_t expand_bits); // ntt.rs:284-330
void expand(Elem* out, const Elem* in, size_t in_n, size_t expand_bits);  // ntt.rs:334-342

// ---- Digest ----------------------------------------------------------------
struct Digest {
  uint32_t w[8];
  bool operator==(const Digest& o) const {
    for (int i = 0; i < 8; i++)
      if (w[i] != o.w[i]) return false;
    return true;
  }
};

// ---- Poseidon2: risc0/zkp/src/core/hash/poseidon2/mod.rs -------------------
void poseidon2_mix(Elem cells[24]);                        // mod.rs:193-216
Digest poseidon2_hash_elems(const Elem* e, size_t n);      // mod.rs:221-245 + to_digest
Digest poseidon2_hash_pair(const Digest& a, const Digest& b);  // mod.rs:47-59

// ---- SHA-256: risc0/zkp/src/core/hash/sha/cpu.rs ---------------------------
void sha256_compress(uint32_t state[8], const uint8_t block[64]);  // FIPS 180-4 compress256
Digest sha256_hash_bytes(const uint8_t* b, size_t n);            // cpu.rs:39-49 (padded)
Digest sha256_hash_raw_words(const uint32_t* w, size_t n);       // cpu.rs:56-77 (unpadded)
Digest sha256_hash_pair(const Digest& a, const Digest& b);       // sha/mod.rs:96-98, cpu.rs:81-105

// ---- HashSuite -------------------------------------------------------------
// ---- Poseidon254: risc0/zkp/src/core/hash/poseidon_254/mod.rs (poseidon254.cpp) ----
Digest poseidon254_hash_elems(const Elem* e, size_t n);        // mod.rs:107-133
Digest poseidon254_hash_pair(const Digest& a, const Digest& b);  // mod.rs:136-142

enum Suite { SUITE_POSEIDON2 = 0, SUITE_SHA256 = 1, SUITE_POSEIDON254 = 2 };
Digest hash_elem_slice(int suite, const Elem* e, size_t n);
Digest hash_ext_elem_slice(int suite, const ExtElem* e, size_t n);
Digest hash_pair(int suite, const Digest& a, const Digest& b);

struct Rng {
  virtual ~Rng() {}
  virtual void mix(const Digest& d) = 0;
  virtual uint32_t random_bits(size_t bits) = 0;
  virtual Elem random_elem() = 0;
  virtual ExtElem random_ext_elem() = 0;
};
std::unique_ptr<Rng> new_rng(int suite);
std::unique_ptr<Rng> new_poseidon254_rng();  // mod.rs:146-209

}  // namespace oracle
