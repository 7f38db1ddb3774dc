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

// ---- reference formulation (mod.rs:102-216 step by step, every value canonical) ----
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
  for (int i = 0; i < 6; i++) p2_m4(c + 4 * i);
  uint32_t s[4];
  for (int j = 0; j < 4; j++) {
    s[j] = fp_add(fp_add(fp_add(c[j], c[4 + j]), fp_add(c[8 + j], c[12 + j])), fp_add(c[16 + j], c[20 + j]));
  }
  for (int i = 0; i < 24; i++) c[i] = fp_add(c[i], s[i & 3]);
}

// M_INT = 1 + diag: mod.rs:129-135
R0_HD void p2_m_int(uint32_t* c) {
  uint32_t sum = 0;
  for (int i = 0; i < 24; i++) sum = fp_add(sum, c[i]);
  for (int i = 0; i < 24; i++) c[i] = fp_add(sum, fp_mul(kP2Diag[i], c[i]));
}

R0_HD void p2_full_round(uint32_t* c, int r) {
  for (int i = 0; i < 24; i++) c[i] = p2_sbox(fp_add(c[i], kP2Full[r * 24 + i]));
  p2_m_ext(c);
}

R0_HD void poseidon2_mix_simple(uint32_t* c) {
  p2_m_ext(c);
  for (int r = 0; r < 4; r++) p2_full_round(c, r);
  for (int r = 0; r < 21; r++) {
    c[0] = p2_sbox(fp_add(c[0], kP2Partial[r]));
    p2_m_int(c);
  }
  for (int r = 4; r < 8; r++) p2_full_round(c, r);
}

// ---- VALU-lean formulation (same permutation, ~30% fewer instructions) ----------
// Poseidon2 is integer-VALU bound on CDNA4 (one v_* per 4 cycles per SIMD), so the
// count of instructions is the cost. Bounds (p < 2^31):
//  * sbox: x^2 canonical, then three REDCs without the final umin: each product has
//    one factor < p and one < 2p, so t < 2p^2 < p*2^32 and the result is < 2p;
//  * M_EXT runs in 64-bit on those lazy (< 2p) cells: every output is a combination
//    with coefficient sum <= 112, so y < 224p < 2^39; the next round constant is
//    added in 64-bit and one lazy REDC feeds the S-box (scaled rounds, below);
//  * M_INT: c_i*d_i + S = REDC(c_i*d_i + S*2^32) and S*2^32 is congruent to
//    fold64(sum c_i * (2^32 mod p)) < 2^60, so multiply, add and reduce are one
//    v_mad_u64_u32 plus one REDC (t < p^2 + 2^60 < p*2^32).
R0_HD uint32_t p2_red39(uint64_t y) {
  uint32_t q = uint32_t((uint64_t(uint32_t(y >> 7)) * 273u) >> 32);
  uint32_t r = uint32_t(y) - q * kP;  // in [0, 2p)
  return umin(r, r - kP);
}
R0_HD uint32_t mont_lazy(uint64_t t) {  // t < p*2^32 -> t*2^-32 mod p in [0, 2p)
  uint32_t m = uint32_t(t) * kNegPinv;
  return uint32_t((t + uint64_t(m) * kP) >> 32);
}
// acc + a * b as one v_mad_u64_u32. Written as inline asm on the device so LLVM keeps
// the multiply-accumulate: for sum(c_i * C) it otherwise factors C out and sums the
// zero-extended c_i with a v_mov + v_lshl_add_u64 pair per cell.
R0_HD uint64_t mad64(uint32_t a, uint32_t b, uint64_t acc) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(P2_NO_ASM)
  uint64_t r, carry;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(carry) : "v"(a), "v"(b), "v"(acc));
  return r;
#else
  return uint64_t(a) * b + acc;
#endif
}
R0_HD uint32_t p2_sbox_lazy(uint32_t x) {  // x canonical -> x^7 in [0, 2p)
  uint32_t x2 = fp_mul(x, x);
  uint32_t x4 = mont_lazy(uint64_t(x2) * x2);
  uint32_t x6 = mont_lazy(uint64_t(x4) * x2);
  return mont_lazy(uint64_t(x6) * x);
}
// y = M_EXT * x over the integers (x < 2p). The 32-bit cells enter the 64-bit sums
// through v_mad_u64_u32 (x * 1 + acc, x * 2 + acc): a plain zero-extended add costs a
// v_mov of the high word per cell first (49 per round in p2_fold_kernel).
R0_HD void p2_m_ext64(const uint32_t* x, uint64_t* y) {
#pragma unroll
  for (int b = 0; b < 6; b++) {
    const uint32_t* v = x + 4 * b;
    uint64_t t0 = mad64(v[0], 1u, mad64(v[1], 1u, 0));
    uint64_t t1 = mad64(v[2], 1u, mad64(v[3], 1u, 0));
    uint64_t t2 = mad64(v[1], 2u, t1);
    uint64_t t3 = mad64(v[3], 2u, t0);
    uint64_t t4 = (t1 << 2) + t3;
    uint64_t t5 = (t0 << 2) + t2;
    y[4 * b] = t3 + t5;
    y[4 * b + 1] = t5;
    y[4 * b + 2] = t2 + t4;
    y[4 * b + 3] = t4;
  }
#pragma unroll
  for (int j = 0; j < 4; j++) {
    uint64_t s = ((y[j] + y[4 + j]) + (y[8 + j] + y[12 + j])) + (y[16 + j] + y[20 + j]);
#pragma unroll
    for (int b = 0; b < 6; b++) y[4 * b + j] += s;
  }
}

// ---- signed Montgomery for the full rounds -----------------------------------------
// Values are int32 in (-p, p). sredc(t) = (t - m p) / 2^32 with m = t * p^-1 mod 2^32 taken
// signed, so |result| < |t| / 2^32 + p/2: a product of two values below p in magnitude
// comes back below 0.969p, closed under multiplication with no correction step (the
// unsigned REDC needs a canonical square before x^4). Overflow bound: |t| + 2^31 p < 2^63,
// i.e. |t| < 1.2 p^2, which every product below keeps (bounds at each use). Same R^-1 per
// reduction as mont_lazy, so the scaled round constants of P2Scaled apply unchanged.
constexpr uint32_t kPinv = 0u - kNegPinv;  // p^-1 mod 2^32
R0_HD int64_t smad64(int32_t a, int32_t b, int64_t acc) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(P2_NO_ASM)
  int64_t r;
  uint64_t carry;
  asm("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(carry) : "v"(a), "v"(b), "v"(acc));
  return r;
#else
  return int64_t(a) * b + acc;
#endif
}
R0_HD int32_t sredc(int64_t t) {
  const int32_t m = int32_t(uint32_t(uint64_t(t)) * kPinv);
  return int32_t(uint64_t(t - int64_t(m) * int64_t(kP)) >> 32);  // low word is 0: exact
}
R0_HD int32_t smul(int32_t a, int32_t b) { return sredc(int64_t(a) * b); }
// |x| < 0.5p + 60 (after sredc of an M_EXT output) or x canonical: x^7 with every
// intermediate below 0.969p in magnitude (products at most 0.94 p^2)
R0_HD int32_t p2_sbox_s(int32_t x) {
  const int32_t x2 = smul(x, x);
  const int32_t x4 = smul(x2, x2);
  const int32_t x6 = smul(x4, x2);
  return smul(x6, x);
}
R0_HD uint32_t s_canon(int32_t r) {  // (-p, p) -> [0, p)
  const uint32_t u = uint32_t(r);
  return umin(u, u + kP);
}
// y = M_EXT x over the integers, signed (|x| < 0.969p: |y| < 112 * 0.969p < 2^37)
R0_HD void p2_m_ext64s(const int32_t* x, int64_t* y) {
#pragma unroll
  for (int b = 0; b < 6; b++) {
    const int32_t* v = x + 4 * b;
    int64_t t0 = smad64(v[0], 1, smad64(v[1], 1, 0));
    int64_t t1 = smad64(v[2], 1, smad64(v[3], 1, 0));
    int64_t t2 = smad64(v[1], 2, t1);
    int64_t t3 = smad64(v[3], 2, t0);
    int64_t t4 = int64_t(uint64_t(t1) << 2) + t3;
    int64_t t5 = int64_t(uint64_t(t0) << 2) + t2;
    y[4 * b] = t3 + t5;
    y[4 * b + 1] = t5;
    y[4 * b + 2] = t2 + t4;
    y[4 * b + 3] = t4;
  }
#pragma unroll
  for (int j = 0; j < 4; j++) {
    int64_t s = ((y[j] + y[4 + j]) + (y[8 + j] + y[12 + j])) + (y[16 + j] + y[20 + j]);
#pragma unroll
    for (int b = 0; b < 6; b++) y[4 * b + j] += s;
  }
}

// Full rounds without Barrett steps. A full round's M_EXT output y (< 224p + p with the
// next round constant) goes straight into a lazy REDC, which returns y * 2^-32 mod p in
// [0, p + 106) in two instructions instead of p2_red39's seven; that is small enough for
// the S-box's first Montgomery square. The REDC leaves the state scaled by 2^-32, so in
// round r the stored cells are X * sigma_r (X the true value, R = 2^32 mod p):
//   sigma_{r+1} = (sigma_r R^-1)^7 R^-6      (one REDC, then the S-box's four)
// and the round constants are stored pre-multiplied by sigma_r R^-1. One Montgomery
// multiply by R^3 / sigma restores the Montgomery form (X * R) before the partial rounds
// and at the end. Rounds 0 and 5 start from sigma = R, so their constants are unchanged.
//
// The constant enters the REDC's low word (round 6): with rcs = rc + (2^32 mod p) mod p (p if
// that is 0), sredc(y + rcs - 2^32) is congruent to sredc(y + rc), and its REDC multiplier
// m = lo(y + rcs - 2^32) p^-1 = (lo(y) + rcs) p^-1 needs only the 32-bit sum. The result is
// then exactly hi(y - m p): the low word of y - m p is 2^32 - rcs (the REDC zeroes the low word
// of y + rcs - 2^32 - m p), so adding rcs - 2^32 carries out and cancels. One full-rate
// v_add_u32 replaces the 64-bit add of rc per cell (sredc_rc). |y + rcs - 2^32| < 110.6p, so
// the output stays below 0.5p + 52.
struct P2Scaled {
  uint32_t rc[8 * 24];   // rounds 0-3 and 5-7 (round 4 uses kP2Full as it is)
  uint32_t k_mid, k_end;
  uint32_t rcs[8 * 24];  // rc + (2^32 mod p) mod p, in [1, p], for sredc_rc
};
constexpr uint32_t p2c_mul(uint32_t a, uint32_t b) { return uint32_t(uint64_t(a) * b % kP); }
constexpr uint32_t p2c_pow(uint32_t a, uint64_t e) {
  uint32_t r = 1;
  while (e) {
    if (e & 1) r = p2c_mul(r, a);
    a = p2c_mul(a, a);
    e >>= 1;
  }
  return r;
}
constexpr P2Scaled p2_make_scaled() {
  P2Scaled t{};
  const uint32_t full[8 * 24] = P2_FULL_RC_MONT;
  const uint32_t R = uint32_t((uint64_t(1) << 32) % kP), Rinv = p2c_pow(R, kP - 2);
  const uint32_t R3 = p2c_pow(R, 3), Rm6 = p2c_pow(Rinv, 6);
  for (int half = 0; half < 2; half++) {
    const int r0 = half ? 5 : 0, r1 = half ? 8 : 4;
    uint32_t sigma = R;
    for (int r = r0; r < r1; r++) {
      const uint32_t s = p2c_mul(sigma, Rinv);
      for (int i = 0; i < 24; i++) t.rc[r * 24 + i] = p2c_mul(full[r * 24 + i], s);
      sigma = p2c_mul(p2c_pow(s, 7), Rm6);
    }
    const uint32_t k = p2c_mul(R3, p2c_pow(sigma, kP - 2));
    if (half) t.k_end = k;
    else t.k_mid = k;
  }
  for (int i = 0; i < 24; i++) t.rc[4 * 24 + i] = full[4 * 24 + i];
  for (int i = 0; i < 8 * 24; i++) {
    const uint32_t v = uint32_t((uint64_t(t.rc[i]) + R) % kP);
    t.rcs[i] = v ? v : kP;
  }
  return t;
}
// sredc(y + rc) (mod p) for the stored round constant rcs = rc + (2^32 mod p): above
R0_HD int32_t sredc_rc(int64_t y, uint32_t rcs) {
  const int32_t m = int32_t((uint32_t(uint64_t(y)) + rcs) * kPinv);
  return int32_t(uint64_t(y - int64_t(m) * int64_t(kP)) >> 32);
}
#if defined(__HIP_DEVICE_COMPILE__)
__constant__ static const P2Scaled kP2S = p2_make_scaled();
#else
static constexpr P2Scaled kP2S = p2_make_scaled();
#endif

R0_HD void poseidon2_mix(uint32_t* c) {
  int64_t y[24];
  int32_t x[24];
#pragma unroll
  for (int i = 0; i < 24; i++) x[i] = int32_t(c[i]);  // canonical: below p < 2^31
  p2_m_ext64s(x, y);
  // Full rounds in signed Montgomery (above): |y + rc| < 113p, so sredc returns below
  // 0.5p + 54, the S-box's input. Rolled: each round's 24 constants are loaded at the top
  // of its iteration instead of all 168 living in SGPRs (which spill to VGPR lanes in
  // hash_rows).
#pragma unroll 1
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 24; i++) x[i] = p2_sbox_s(sredc_rc(y[i], kP2S.rcs[r * 24 + i]));
    p2_m_ext64s(x, y);
  }
#pragma unroll
  for (int i = 0; i < 24; i++) c[i] = s_canon(smul(sredc(y[i]), int32_t(kP2S.k_mid)));
#pragma unroll
  // Partial rounds keep every cell lazy in [0, 2p): with cells c < X the M_INT output
  // REDC(c*d + sf) < 0.469 X + sf/2^32 + p, whose fixed point (sf < 2^57 + 2^32 after
  // two folds) is 3.86e9 < 2p < 2^32, so nothing is canonicalised until the end. The
  // sum is two 12-term halves (12 * 2p * (2^32 mod p) < 2^64).
  for (int r = 0; r < 21; r++) {
    c[0] = p2_sbox_lazy(fp_add(umin(c[0], c[0] - kP), kP2Partial[r]));
    uint64_t s0 = 0, s1 = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {  // two interleaved chains: no dependent back-to-back mads
      s0 = mad64(c[i], kFoldC, s0);
      s1 = mad64(c[12 + i], kFoldC, s1);
    }
    const uint64_t sf = fold64(fold64(s0) + fold64(s1));
#pragma unroll
    for (int i = 0; i < 24; i++) c[i] = mont_lazy(uint64_t(c[i]) * kP2Diag[i] + sf);
  }
#pragma unroll
  for (int i = 0; i < 24; i++) c[i] = umin(c[i], c[i] - kP);
#pragma unroll
  for (int i = 0; i < 24; i++) x[i] = p2_sbox_s(int32_t(fp_add(c[i], kP2Full[4 * 24 + i])));
  p2_m_ext64s(x, y);
#pragma unroll 1
  for (int r = 5; r < 8; r++) {
#pragma unroll
    for (int i = 0; i < 24; i++) x[i] = p2_sbox_s(sredc_rc(y[i], kP2S.rcs[r * 24 + i]));
    p2_m_ext64s(x, y);
  }
#pragma unroll
  for (int i = 0; i < 24; i++) c[i] = s_canon(smul(sredc(y[i]), int32_t(kP2S.k_end)));
}

#if defined(__HIP__)
// ---- one permutation over a lane quad (wavefront-shuffle formulation) -------------
// Lane q = lane & 3 of a quad holds cells 4j + q (j = 0..5): position q of every 4x4 block
// of M_EXT. The block mix needs the other three positions of the block (three DPP
// quad_perm moves per block, no LDS); the block sum s[q] of M_EXT and the per-cell
// M_INT diagonal are lane-local; the M_INT sum over all 24 cells is a two-step quad
// all-reduce. Same arithmetic and bounds as poseidon2_mix, so the words are identical.
// About 2.6k VALU instructions per lane against 7.6k for one lane per permutation: a
// third of the latency for 1.4x the issued work, so it pays only where a layer leaves
// SIMDs idle (Merkle tree tops), not in the throughput-bound leaf and layer hashing.
__device__ __forceinline__ uint32_t p2q_dpp(uint32_t v, int sel) {
  switch (sel) {  // quad_perm lane selectors for q^1, q^2, q^3
    case 1: return uint32_t(__builtin_amdgcn_mov_dpp(int(v), 0xB1, 0xF, 0xF, false));
    case 2: return uint32_t(__builtin_amdgcn_mov_dpp(int(v), 0x4E, 0xF, 0xF, false));
    default: return uint32_t(__builtin_amdgcn_mov_dpp(int(v), 0x1B, 0xF, 0xF, false));
  }
}
__device__ __forceinline__ uint64_t p2q_dpp64(uint64_t v, int sel) {
  return (uint64_t(p2q_dpp(uint32_t(v >> 32), sel)) << 32) | p2q_dpp(uint32_t(v), sel);
}
// M4 rows (p2_m4 as a matrix): [5 7 1 3] [4 6 1 1] [1 3 5 7] [1 1 4 6]; m[d] = M4[q][q ^ d]
struct P2Quad {
  uint32_t m[4];
  uint32_t q;
  __device__ __forceinline__ explicit P2Quad(uint32_t lane) : q(lane & 3) {
    constexpr uint32_t M4[16] = {5, 7, 1, 3, 4, 6, 1, 1, 1, 3, 5, 7, 1, 1, 4, 6};
#pragma unroll
    for (uint32_t d = 0; d < 4; d++) {
      uint32_t v = 0;
#pragma unroll
      for (uint32_t qq = 0; qq < 4; qq++) v = q == qq ? M4[qq * 4 + (qq ^ d)] : v;
      m[d] = v;
    }
  }
  // y = M_EXT x over the integers for this lane's six cells (x < 2p)
  __device__ __forceinline__ void m_ext(const uint32_t* x, uint64_t* y) const {
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < 6; j++) {
      uint64_t t = uint64_t(x[j]) * m[0];
      t = mad64(p2q_dpp(x[j], 1), m[1], t);
      t = mad64(p2q_dpp(x[j], 2), m[2], t);
      t = mad64(p2q_dpp(x[j], 3), m[3], t);
      y[j] = t;
      s += t;
    }
#pragma unroll
    for (int j = 0; j < 6; j++) y[j] += s;
  }
};

__device__ __forceinline__ void poseidon2_mix_quad(uint32_t* c) {
  const P2Quad Q(threadIdx.x);
  const uint32_t q = Q.q;
  uint64_t y[6];
  uint32_t x[6];
  Q.m_ext(c, y);
#pragma unroll 1
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int j = 0; j < 6; j++) x[j] = p2_sbox_lazy(mont_lazy(y[j] + kP2S.rc[r * 24 + 4 * j + q]));
    Q.m_ext(x, y);
  }
#pragma unroll
  for (int j = 0; j < 6; j++) c[j] = fp_mul(mont_lazy(y[j]), kP2S.k_mid);
  uint32_t diag[6];
#pragma unroll
  for (int j = 0; j < 6; j++) diag[j] = kP2Diag[4 * j + q];
#pragma unroll 1
  for (int r = 0; r < 21; r++) {
    const uint32_t u = p2_sbox_lazy(fp_add(umin(c[0], c[0] - kP), kP2Partial[r]));
    c[0] = q == 0 ? u : c[0];  // cell 0 lives in lane 0 of the quad
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < 6; j++) s = mad64(c[j], kFoldC, s);
    s = fold64(s);
    s += p2q_dpp64(s, 1);
    s += p2q_dpp64(s, 2);
    const uint64_t sf = fold64(s);
#pragma unroll
    for (int j = 0; j < 6; j++) c[j] = mont_lazy(uint64_t(c[j]) * diag[j] + sf);
  }
#pragma unroll
  for (int j = 0; j < 6; j++) c[j] = umin(c[j], c[j] - kP);
#pragma unroll
  for (int j = 0; j < 6; j++) x[j] = p2_sbox_lazy(fp_add(c[j], kP2Full[4 * 24 + 4 * j + q]));
  Q.m_ext(x, y);
#pragma unroll 1
  for (int r = 5; r < 8; r++) {
#pragma unroll
    for (int j = 0; j < 6; j++) x[j] = p2_sbox_lazy(mont_lazy(y[j] + kP2S.rc[r * 24 + 4 * j + q]));
    Q.m_ext(x, y);
  }
#pragma unroll
  for (int j = 0; j < 6; j++) c[j] = fp_mul(mont_lazy(y[j]), kP2S.k_end);
}
#endif

}  // namespace r0
