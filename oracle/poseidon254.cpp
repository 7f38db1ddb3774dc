// ORACLE (test infrastructure only — never linked into the product path).
//
// CPU restatement of the Poseidon254 hash suite (risc0/zkp/src/core/hash/poseidon_254):
//   BN254 scalar field Fr (consts.rs:19-23, ff::PrimeField derive: Montgomery form,
//   R = 2^256, little-endian repr), Poseidon t=3 alpha=8 with 4+42+4 rounds
//   (mod.rs:33-89), unpadded_hash packing 8 canonical BabyBear values per Fr in base p
//   (mod.rs:107-133), hash_pair (mod.rs:136-142) and Poseidon254Rng (mod.rs:157-209).
// Field arithmetic here is 4 x u64 limbs with unsigned __int128 (an independent
// formulation from the product's 8 x u32 device code).
#include <cstring>

#include "core.h"

namespace oracle {
namespace {

#include "poseidon254_consts.inc"

using u64 = uint64_t;
using u128 = unsigned __int128;

struct Fr {
  u64 v[4];  // Montgomery form, canonical (< modulus)
};

bool geq_mod(const u64* a) {
  for (int i = 3; i >= 0; i--) {
    if (a[i] != P254_MODULUS[i]) return a[i] > P254_MODULUS[i];
  }
  return true;
}
void sub_mod(u64* a) {
  u64 borrow = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = u128(a[i]) - P254_MODULUS[i] - borrow;
    a[i] = u64(d);
    borrow = u64(d >> 64) & 1;
  }
}
Fr add(const Fr& a, const Fr& b) {
  Fr r;
  u64 carry = 0;
  for (int i = 0; i < 4; i++) {
    u128 s = u128(a.v[i]) + b.v[i] + carry;
    r.v[i] = u64(s);
    carry = u64(s >> 64);
  }
  if (carry || geq_mod(r.v)) sub_mod(r.v);  // a + b < 2^255 for canonical inputs: carry is 0
  return r;
}
u64 inv64() {  // -modulus^-1 mod 2^64 by Newton iteration
  u64 x = 1;
  for (int i = 0; i < 7; i++) x *= 2 - P254_MODULUS[0] * x;
  return ~x + 1;
}
const u64 NINV = inv64();
// CIOS Montgomery product a*b/R mod modulus
Fr mul(const Fr& a, const Fr& b) {
  u64 t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u64 c = 0;
    for (int j = 0; j < 4; j++) {
      u128 s = u128(a.v[j]) * b.v[i] + t[j] + c;
      t[j] = u64(s);
      c = u64(s >> 64);
    }
    u128 s = u128(t[4]) + c;
    t[4] = u64(s);
    t[5] = u64(s >> 64);
    u64 m = t[0] * NINV;
    s = u128(m) * P254_MODULUS[0] + t[0];
    c = u64(s >> 64);
    for (int j = 1; j < 4; j++) {
      s = u128(m) * P254_MODULUS[j] + t[j] + c;
      t[j - 1] = u64(s);
      c = u64(s >> 64);
    }
    s = u128(t[4]) + c;
    t[3] = u64(s);
    t[4] = t[5] + u64(s >> 64);
  }
  Fr r;
  memcpy(r.v, t, 32);
  if (t[4] || geq_mod(r.v)) sub_mod(r.v);
  return r;
}
Fr canonical_to_fr(const u64* x);
Fr R2() {  // 2^512 mod modulus, by doubling 1
  Fr x{{1, 0, 0, 0}};
  for (int i = 0; i < 512; i++) x = add(x, x);
  return x;
}
const Fr kR2 = R2();
Fr canonical_to_fr(const u64* x) {
  Fr c;
  memcpy(c.v, x, 32);
  return mul(c, kR2);
}
void fr_to_canonical(const Fr& a, u64* out) {
  Fr one{{1, 0, 0, 0}};
  Fr r = mul(a, one);
  memcpy(out, r.v, 32);
}
Fr from_u64(u64 x) {
  u64 c[4] = {x, 0, 0, 0};
  return canonical_to_fr(c);
}
const Fr kZero{{0, 0, 0, 0}};

struct Consts {
  Fr rc[150], mds[9];
  Consts() {
    for (int i = 0; i < 150; i++) rc[i] = canonical_to_fr(P254_ROUND_CONSTANTS[i]);
    for (int i = 0; i < 9; i++) mds[i] = canonical_to_fr(P254_MDS[i]);
  }
};
const Consts& consts() {
  static Consts c;
  return c;
}

// mod.rs:39-43
Fr sbox(const Fr& x) {
  Fr x2 = mul(x, x);
  Fr x4 = mul(x2, x2);
  return mul(x4, x4);
}
// mod.rs:33-89
void poseidon_mix(Fr* cells) {
  const Consts& k = consts();
  for (int round = 0; round < 50; round++) {
    bool full = round < 4 || round >= 46;
    for (int i = 0; i < 3; i++) cells[i] = add(cells[i], k.rc[round * 3 + i]);
    if (full) {
      for (int i = 0; i < 3; i++) cells[i] = sbox(cells[i]);
    } else {
      cells[0] = sbox(cells[0]);
    }
    Fr old[3] = {cells[0], cells[1], cells[2]};
    for (int i = 0; i < 3; i++) {
      Fr tot = kZero;
      for (int j = 0; j < 3; j++) tot = add(tot, mul(k.mds[i * 3 + j], old[j]));
      cells[i] = tot;
    }
  }
}
// mod.rs:94-105: Digest <-> Fr through the little-endian canonical repr
Fr digest_to_fr(const Digest& d) {
  u64 x[4];
  for (int i = 0; i < 4; i++) x[i] = u64(d.w[2 * i]) | (u64(d.w[2 * i + 1]) << 32);
  return canonical_to_fr(x);
}
Digest fr_to_digest(const Fr& f) {
  u64 x[4];
  fr_to_canonical(f, x);
  Digest d;
  for (int i = 0; i < 4; i++) {
    d.w[2 * i] = uint32_t(x[i]);
    d.w[2 * i + 1] = uint32_t(x[i] >> 32);
  }
  return d;
}

}  // namespace

// mod.rs:107-133 over canonical values (Elem::as_u32)
Digest poseidon254_hash_elems(const Elem* e, size_t n) {
  Fr cells[3] = {kZero, kZero, kZero};
  const Fr p = from_u64(P);
  Fr m = from_u64(1);
  int idx = 1, count = 0;
  for (size_t k = 0; k < n; k++) {
    cells[idx] = add(cells[idx], mul(m, from_u64(e[k].as_u32())));
    m = mul(m, p);
    if (++count == 8) {
      m = from_u64(1);
      count = 0;
      idx++;
    }
    if (idx == 3) {
      poseidon_mix(cells);
      cells[1] = kZero;
      cells[2] = kZero;
      idx = 1;
    }
  }
  if (idx != 1 || count != 0) poseidon_mix(cells);
  return fr_to_digest(cells[0]);
}

// mod.rs:136-142
Digest poseidon254_hash_pair(const Digest& a, const Digest& b) {
  Fr cells[3] = {kZero, digest_to_fr(a), digest_to_fr(b)};
  poseidon_mix(cells);
  return fr_to_digest(cells[0]);
}

// mod.rs:146-209
struct Poseidon254Rng : Rng {
  Fr cells[3] = {kZero, kZero, kZero};
  void mix(const Digest& d) override {
    cells[1] = add(cells[1], digest_to_fr(d));
    poseidon_mix(cells);
  }
  // the bit loop of random_bits / random_elem peels the canonical value's low bits
  void next_source(u64* src) {
    fr_to_canonical(cells[2], src);
    poseidon_mix(cells);
  }
  uint32_t random_bits(size_t bits) override {
    u64 src[4];
    next_source(src);
    return uint32_t(src[0] & ((u64(1) << bits) - 1));
  }
  Elem random_elem() override {
    u64 src[4];
    next_source(src);
    Elem out = Elem::zero(), m = Elem::one(), two = Elem::from(2);
    for (int i = 0; i < 160; i++) {
      if ((src[i / 64] >> (i % 64)) & 1) out += m;
      m *= two;
    }
    return out;
  }
  ExtElem random_ext_elem() override {
    ExtElem r;
    for (int i = 0; i < 4; i++) r.e[i] = random_elem();
    return r;
  }
};

std::unique_ptr<Rng> new_poseidon254_rng() { return std::unique_ptr<Rng>(new Poseidon254Rng()); }

}  // namespace oracle
