// Poseidon over BN254 Fr, t = 3, alpha = 8, 4 + 42 + 4 rounds — the permutation and hash
// functions of risc0/zkp/src/core/hash/poseidon_254/mod.rs, host+device:
//   poseidon_mix                :33-89  (round constants, sbox x^8, dense 3x3 MDS)
//   unpadded_hash               :107-133 (8 canonical BabyBear values per Fr, base p, rate 2)
//   hash_pair                   :136-142
// Cells live in bn254.h's lazy Montgomery form. Each round's MDS product and the next
// round's constants share one reduction: REDC(sum_j M_ij s_j + RC_i * R); partial rounds
// use the equivalent sparse matrices (Poseidon paper, appendix B).
#pragma once
#include "bn254.h"

namespace r0 {

#if defined(__HIP_DEVICE_COMPILE__)
#define R0_P254_TABLE __constant__ static const
#else
#define R0_P254_TABLE static const
#endif
R0_P254_TABLE uint32_t kP254Rc0[3][9] = P254_RC0_L29;
R0_P254_TABLE uint32_t kP254FullMat[2][9][9] = P254_FULL_MAT_L29;
R0_P254_TABLE uint32_t kP254FullRc[8][3][9] = P254_FULL_RC_L29;
R0_P254_TABLE uint32_t kP254Partial[42][8][9] = P254_PARTIAL_L29;
R0_P254_TABLE uint32_t kP254Pack[8][9] = P254_PACK_L29;
#undef R0_P254_TABLE

R0_HD bn::Fr p254_sbox(const bn::Fr& x) { return bn::sqr(bn::sqr(bn::sqr(x))); }

// c: Montgomery cells, limbs < 2^29. The 42 partial rounds use the sparse equivalent
// matrices of tools/extract_poseidon254.py: cell 0 takes a 3-term row, cells 1 and 2 take
// w_i * s0 + cell_i, so a partial round costs 5 products instead of 9. Cells 1 and 2 are
// not reduced there and grow by < 2.1r a round, to < 88r < 2^260.1 before the next full
// round's S-boxes (which bring them back below 2.1r): all within bn254.h's column bounds.
// Rounds stay rolled (one full round is ~2.7k instructions, the partial round ~1.3k).
R0_HD void p254_mix(bn::Fr* c) {
#pragma unroll
  for (int i = 0; i < 3; i++) c[i] = bn::add_norm(c[i], kP254Rc0[i]);
#pragma unroll 1
  for (int f = 0; f < 8; f++) {
    if (f == 4) {
#pragma unroll 1
      for (int k = 0; k < 42; k++) {
        const uint32_t* t = &kP254Partial[k][0][0];
        const bn::Fr s0 = p254_sbox(c[0]);
        uint32_t e1[9], e2[9];
#pragma unroll
        for (int i = 0; i < 9; i++) {
          e1[i] = c[1].l[i] + t[54 + i];
          e2[i] = c[2].l[i] + t[63 + i];
        }
        c[0] = bn::dot3_add(t, t + 9, t + 18, s0, c[1], c[2], t + 45);
        c[1] = bn::mul_add(t + 27, s0, e1);
        c[2] = bn::mul_add(t + 36, s0, e2);
      }
    }
    const bn::Fr s0 = p254_sbox(c[0]), s1 = p254_sbox(c[1]), s2 = p254_sbox(c[2]);
    const uint32_t* m = &kP254FullMat[f == 3 ? 1 : 0][0][0];
    const uint32_t* n = &kP254FullRc[f][0][0];
    c[0] = bn::dot3_add(m, m + 9, m + 18, s0, s1, s2, n);
    c[1] = bn::dot3_add(m + 27, m + 36, m + 45, s0, s1, s2, n + 9);
    c[2] = bn::dot3_add(m + 54, m + 63, m + 72, s0, s1, s2, n + 18);
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
