// Poseidon over BN254 Fr, t = 3, alpha = 8, 4 + 42 + 4 rounds — the permutation and hash
// functions of risc0/zkp/src/core/hash/poseidon_254/mod.rs, host+device:
//   poseidon_mix                :33-89  (round constants, sbox x^8, dense 3x3 MDS)
//   unpadded_hash               :107-133 (8 canonical BabyBear values per Fr, base p, rate 2)
//   hash_pair                   :136-142
// Cells live in bn254.h's lazy Montgomery form. Each round's MDS product and the next
// round's constants share one reduction: REDC(sum_j M_ij s_j + RC_i * R).
#pragma once
#include "bn254.h"

namespace r0 {

#if defined(__HIP_DEVICE_COMPILE__)
__constant__ static const uint32_t kP254Rc[153][9] = P254_RC_L29;
__constant__ static const uint32_t kP254Mds[9][9] = P254_MDS_L29;
__constant__ static const uint32_t kP254Pack[8][9] = P254_PACK_L29;
#else
static const uint32_t kP254Rc[153][9] = P254_RC_L29;
static const uint32_t kP254Mds[9][9] = P254_MDS_L29;
static const uint32_t kP254Pack[8][9] = P254_PACK_L29;
#endif

R0_HD bn::Fr p254_sbox(const bn::Fr& x) { return bn::sqr(bn::sqr(bn::sqr(x))); }

// c: Montgomery cells < 2.2r with limbs < 2^29. Rounds stay rolled (a round is ~2.7k
// instructions; unrolled, the 50 rounds would not fit the instruction cache).
R0_HD void p254_mix(bn::Fr* c) {
#pragma unroll
  for (int i = 0; i < 3; i++) c[i] = bn::add_norm(c[i], kP254Rc[i]);
#pragma unroll 1
  for (int r = 0; r < 50; r++) {
    const bool full = r < 4 || r >= 46;
    c[0] = p254_sbox(c[0]);
    if (full) {
      c[1] = p254_sbox(c[1]);
      c[2] = p254_sbox(c[2]);
    }
    const bn::Fr s0 = c[0], s1 = c[1], s2 = c[2];
    // the next round's constants (row 150 of the table is zero: nothing after round 49)
    c[0] = bn::dot3_add(kP254Mds[0], kP254Mds[1], kP254Mds[2], s0, s1, s2, kP254Rc[3 * r + 3]);
    c[1] = bn::dot3_add(kP254Mds[3], kP254Mds[4], kP254Mds[5], s0, s1, s2, kP254Rc[3 * r + 4]);
    c[2] = bn::dot3_add(kP254Mds[6], kP254Mds[7], kP254Mds[8], s0, s1, s2, kP254Rc[3 * r + 5]);
  }
}

// Montgomery form of sum_k v[k] * p^k for up to 8 canonical BabyBear values (the rest 0):
// REDC(sum_k v_k * PACK_k) with PACK_k = p^k R^2 mod r. A column holds 8 products
// v_k (< 2^31) x limb (< 2^29) < 2^60.
R0_HD bn::Fr p254_pack8(const uint32_t* v) {
  bn::Fr o;
  bn::redc(o, [&](int k, uint64_t acc) {
    if (k < 9) {
#pragma unroll
      for (int j = 0; j < 8; j++) acc = bn::mac(v[j], kP254Pack[j][k], acc);
    }
    return acc;
  });
  return o;
}

R0_HD bn::Fr p254_zero() { return bn::Fr{{0, 0, 0, 0, 0, 0, 0, 0, 0}}; }

// digest (canonical LE words) -> Montgomery cell, and back (mod.rs:94-105)
R0_HD bn::Fr p254_from_digest(const uint32_t* w) { return bn::to_mont(bn::from_words(w)); }
R0_HD void p254_to_digest(const bn::Fr& x, uint32_t* w) { bn::to_words(bn::to_canonical(x), w); }

// mod.rs:136-142
R0_HD void p254_hash_pair(const uint32_t* a, const uint32_t* b, uint32_t* out) {
  bn::Fr c[3] = {p254_zero(), p254_from_digest(a), p254_from_digest(b)};
  p254_mix(c);
  p254_to_digest(c[0], out);
}

// mod.rs:107-133 over canonical values v[0..n)
R0_HD void p254_hash_canonical(const uint32_t* v, size_t n, uint32_t* out) {
  bn::Fr c[3] = {p254_zero(), p254_zero(), p254_zero()};
  size_t k = 0;
  for (; k + 16 <= n; k += 16) {
    c[1] = p254_pack8(v + k);
    c[2] = p254_pack8(v + k + 8);
    p254_mix(c);
  }
  if (k < n) {
    uint32_t t[16] = {0};
    for (size_t i = k; i < n; i++) t[i - k] = v[i];
    c[1] = p254_pack8(t);
    c[2] = n - k > 8 ? p254_pack8(t + 8) : p254_zero();
    p254_mix(c);
  }
  p254_to_digest(c[0], out);
}

}  // namespace r0
