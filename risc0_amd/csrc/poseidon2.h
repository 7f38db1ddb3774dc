// Poseidon2 over BabyBear, width 24 / rate 16 / 8 output cells, 4+21+4 rounds —
// the permutation of risc0/zkp/src/core/hash/poseidon2/mod.rs:102-216 with the
// parameters of poseidon2/consts.rs (Montgomery-encoded by tools/extract_poseidon2.py).
// Host+device: the device hashes Merkle rows/nodes, the host driver uses the same
// code for the Fiat-Shamir transcript (Poseidon2Rng, poseidon2/rng.rs:50-89).
#pragma once
#include "bb31.h"
#include "poseidon2_consts.inc"

namespace r0 {

#if defined(__HIP_DEVICE_COMPILE__)
__constant__ static const uint32_t kP2Full[8 * 24] = P2_FULL_RC_MONT;
__constant__ static const uint32_t kP2Partial[21] = P2_PARTIAL_RC_MONT;
__constant__ static const uint32_t kP2Diag[24] = P2_DIAG_MONT;
#else
static const uint32_t kP2Full[8 * 24] = P2_FULL_RC_MONT;
static const uint32_t kP2Partial[21] = P2_PARTIAL_RC_MONT;
static const uint32_t kP2Diag[24] = P2_DIAG_MONT;
#endif

R0_HD uint32_t p2_sbox(uint32_t x) {
  uint32_t x2 = fp_mul(x, x);
  uint32_t x4 = fp_mul(x2, x2);
  uint32_t x6 = fp_mul(x4, x2);
  return fp_mul(x6, x);
}

// 4x4 circulant block of M_EXT (Poseidon2 paper, appendix B): mod.rs:137-148
R0_HD void p2_m4(uint32_t* x) {
  uint32_t t0 = fp_add(x[0], x[1]);
  uint32_t t1 = fp_add(x[2], x[3]);
  uint32_t t2 = fp_add(fp_add(x[1], x[1]), t1);
  uint32_t t3 = fp_add(fp_add(x[3], x[3]), t0);
  uint32_t t1_2 = fp_add(t1, t1), t0_2 = fp_add(t0, t0);
  uint32_t t4 = fp_add(fp_add(t1_2, t1_2), t3);
  uint32_t t5 = fp_add(fp_add(t0_2, t0_2), t2);
  uint32_t t6 = fp_add(t3, t5);
  uint32_t t7 = fp_add(t2, t4);
  x[0] = t6;
  x[1] = t5;
  x[2] = t7;
  x[3] = t4;
}

// M_EXT: mod.rs:150-173
R0_HD void p2_m_ext(uint32_t* c) {
#pragma unroll
  for (int i = 0; i < 6; i++) p2_m4(c + 4 * i);
  uint32_t s[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    s[j] = fp_add(fp_add(fp_add(c[j], c[4 + j]), fp_add(c[8 + j], c[12 + j])), fp_add(c[16 + j], c[20 + j]));
  }
#pragma unroll
  for (int i = 0; i < 24; i++) c[i] = fp_add(c[i], s[i & 3]);
}

// M_INT = 1 + diag: mod.rs:129-135
R0_HD void p2_m_int(uint32_t* c) {
  uint32_t sum = 0;
#pragma unroll
  for (int i = 0; i < 24; i++) sum = fp_add(sum, c[i]);
#pragma unroll
  for (int i = 0; i < 24; i++) c[i] = fp_add(sum, fp_mul(kP2Diag[i], c[i]));
}

R0_HD void p2_full_round(uint32_t* c, int r) {
#pragma unroll
  for (int i = 0; i < 24; i++) c[i] = p2_sbox(fp_add(c[i], kP2Full[r * 24 + i]));
  p2_m_ext(c);
}

// mod.rs:193-216
R0_HD void poseidon2_mix(uint32_t* c) {
  p2_m_ext(c);
#pragma unroll
  for (int r = 0; r < 4; r++) p2_full_round(c, r);
#pragma unroll
  for (int r = 0; r < 21; r++) {
    c[0] = p2_sbox(fp_add(c[0], kP2Partial[r]));
    p2_m_int(c);
  }
#pragma unroll
  for (int r = 4; r < 8; r++) p2_full_round(c, r);
}

}  // namespace r0
