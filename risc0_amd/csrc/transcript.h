// Host-side Fiat-Shamir for the driver: the HashSuite hash functions over host
// data (PROOF_SYSTEM_INFO / header / U coefficients / final FRI coefficients) and
// the transcript RNGs. Follows
//   poseidon2/mod.rs:47-100,221-245, poseidon2/rng.rs:50-89   (suite "poseidon2")
//   sha/cpu.rs:36-105, sha/rng.rs:24-101                      (suite "sha-256")
//   poseidon_254/mod.rs:107-209                                (suite "poseidon_254")
//   prove/write_iop.rs:24-76                                   (WriteIOP)
#pragma once
#include <stdint.h>
#include <string.h>

#include <memory>
#include <vector>

#include "bb31.h"
#include "poseidon2.h"
#include "poseidon254.h"

namespace r0 {

struct Digest {
  uint32_t w[8];
};

namespace sha {
static const uint32_t K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
// w: 16 big-endian message words
inline void compress(uint32_t* s, const uint32_t* m) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++) w[i] = m[i];
  for (int i = 16; i < 64; i++)
    w[i] = w[i - 16] + (rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3)) + w[i - 7] +
           (rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10));
  uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
  for (int i = 0; i < 64; i++) {
    uint32_t t1 = h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
    uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
}
inline void init(uint32_t* s) {
  static const uint32_t IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(s, IV, 32);
}
inline Digest out(const uint32_t* s) {
  Digest d;
  for (int i = 0; i < 8; i++) d.w[i] = __builtin_bswap32(s[i]);
  return d;
}
// unpadded hash of LE words (cpu.rs:56-77)
inline Digest hash_words(const uint32_t* words, size_t n) {
  uint32_t s[8], m[16];
  init(s);
  for (size_t i = 0; i < n; i += 16) {
    for (size_t k = 0; k < 16; k++) m[k] = i + k < n ? __builtin_bswap32(words[i + k]) : 0u;
    compress(s, m);
  }
  return out(s);
}
// standard padded SHA-256 of bytes (cpu.rs:39-49)
inline Digest hash_bytes(const uint8_t* b, size_t n) {
  std::vector<uint8_t> buf(b, b + n);
  buf.push_back(0x80);
  while (buf.size() % 64 != 56) buf.push_back(0);
  uint64_t bits = uint64_t(n) * 8;
  for (int i = 7; i >= 0; i--) buf.push_back(uint8_t(bits >> (8 * i)));
  uint32_t s[8], m[16];
  init(s);
  for (size_t i = 0; i < buf.size(); i += 64) {
    for (int k = 0; k < 16; k++)
      m[k] = (uint32_t(buf[i + 4 * k]) << 24) | (uint32_t(buf[i + 4 * k + 1]) << 16) |
             (uint32_t(buf[i + 4 * k + 2]) << 8) | uint32_t(buf[i + 4 * k + 3]);
    compress(s, m);
  }
  return out(s);
}
inline Digest hash_pair(const Digest& a, const Digest& b) {
  uint32_t s[8], m[16];
  init(s);
  for (int k = 0; k < 8; k++) {
    m[k] = __builtin_bswap32(a.w[k]);
    m[8 + k] = __builtin_bswap32(b.w[k]);
  }
  compress(s, m);
  return out(s);
}
}  // namespace sha

// poseidon2 sponge over raw Montgomery words (mod.rs:221-245)
inline Digest p2_hash_words(const uint32_t* e, size_t n) {
  uint32_t st[24] = {0};
  size_t unmixed = 0;
  for (size_t k = 0; k < n; k++) {
    st[unmixed++] = e[k];
    if (unmixed == 16) {
      poseidon2_mix(st);
      unmixed = 0;
    }
  }
  if (unmixed != 0 || n == 0) {
    for (size_t i = unmixed; i < 16; i++) st[i] = 0;
    poseidon2_mix(st);
  }
  Digest d;
  memcpy(d.w, st, 32);
  return d;
}

// poseidon_254 unpadded_hash over Elem::as_u32 of raw Montgomery words (mod.rs:107-133)
inline Digest p254_hash_words(const uint32_t* e, size_t n) {
  std::vector<uint32_t> v(n);
  for (size_t i = 0; i < n; i++) v[i] = fp_decode(e[i]);
  Digest d;
  p254_hash_canonical(v.data(), n, d.w);
  return d;
}

inline Digest hash_elems(int suite, const uint32_t* e, size_t n) {
  return suite == 0 ? p2_hash_words(e, n) : suite == 1 ? sha::hash_words(e, n) : p254_hash_words(e, n);
}

struct Rng {
  virtual ~Rng() {}
  virtual void mix(const Digest& d) = 0;
  virtual uint32_t random_bits(size_t bits) = 0;
  virtual uint32_t random_elem() = 0;  // Montgomery word
  FpExt random_ext_elem() {
    FpExt r;
    for (int i = 0; i < 4; i++) r.c[i] = random_elem();
    return r;
  }
};

struct Poseidon2Rng : Rng {
  uint32_t cells[24] = {0};
  size_t pool_used = 0;
  void mix(const Digest& d) override {
    if (pool_used != 0) {
      poseidon2_mix(cells);
      pool_used = 0;
    }
    for (int i = 0; i < 8; i++) cells[i] = fp_add(cells[i], d.w[i]);
    poseidon2_mix(cells);
  }
  uint32_t random_bits(size_t bits) override {
    uint32_t val = fp_decode(random_elem());
    for (int i = 0; i < 3; i++) {
      uint32_t nv = fp_decode(random_elem());
      if (val == 0) val = nv;
    }
    return uint32_t((uint64_t(1) << bits) - 1) & val;
  }
  uint32_t random_elem() override {
    if (pool_used == 16) {
      poseidon2_mix(cells);
      pool_used = 0;
    }
    return cells[pool_used++];
  }
};

struct ShaRng : Rng {
  Digest pool0, pool1;
  size_t pool_used = 0;
  ShaRng() {
    pool0 = sha::hash_bytes(reinterpret_cast<const uint8_t*>("Hello"), 5);
    pool1 = sha::hash_bytes(reinterpret_cast<const uint8_t*>("World"), 5);
  }
  void step() {
    pool0 = sha::hash_pair(pool0, pool1);
    pool1 = sha::hash_pair(pool0, pool1);
    pool_used = 0;
  }
  uint32_t next_u32() {
    if (pool_used == 8) step();
    return pool0.w[pool_used++];
  }
  void mix(const Digest& d) override {
    for (int i = 0; i < 8; i++) pool0.w[i] ^= d.w[i];
    step();
  }
  uint32_t random_bits(size_t bits) override { return uint32_t((uint64_t(1) << bits) - 1) & next_u32(); }
  uint32_t random_elem() override {  // baby_bear.rs:110-140
    uint64_t v = 0;
    for (int i = 0; i < 6; i++) {
      v = ((v << 32) + next_u32()) % kP;
    }
    return fp_encode(uint32_t(v));
  }
};

// poseidon_254/mod.rs:146-209: draws read the canonical value of cell 2, then permute
struct Poseidon254Rng : Rng {
  bn::Fr cells[3] = {p254_zero(), p254_zero(), p254_zero()};
  void mix(const Digest& d) override {
    cells[1] = bn::add_norm(cells[1], p254_from_digest(d.w).l);
    p254_mix(cells);
  }
  void next_source(uint32_t* w) {
    p254_to_digest(cells[2], w);
    p254_mix(cells);
  }
  uint32_t random_bits(size_t bits) override {
    uint32_t w[8];
    next_source(w);
    return uint32_t((uint64_t(1) << bits) - 1) & w[0];
  }
  uint32_t random_elem() override {  // low 160 bits of the source, mod p
    uint32_t w[8];
    next_source(w);
    uint64_t v = 0;
    for (int i = 4; i >= 0; i--) v = ((v << 32) | w[i]) % kP;
    return fp_encode(uint32_t(v));
  }
};

inline std::unique_ptr<Rng> make_rng(int suite) {
  if (suite == 2) return std::unique_ptr<Rng>(new Poseidon254Rng());
  if (suite == 0) return std::unique_ptr<Rng>(new Poseidon2Rng());
  return std::unique_ptr<Rng>(new ShaRng());
}

// write_iop.rs
struct WriteIOP {
  std::vector<uint32_t> proof;
  std::unique_ptr<Rng> rng;
  explicit WriteIOP(int suite) : rng(make_rng(suite)) {}
  void write(const uint32_t* p, size_t n) { proof.insert(proof.end(), p, p + n); }
  void commit(const Digest& d) { rng->mix(d); }
};

}  // namespace r0
