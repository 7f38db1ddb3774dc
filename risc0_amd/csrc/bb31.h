// BabyBear field (p = 15*2^27 + 1) and its quartic extension F_p[x]/(x^4 + 11) for
// CDNA4 device code and the host driver.
//
// Representation is the reference's: raw Montgomery words with R = 2^32
// (risc0/core/src/field/baby_bear.rs:40-42, 323-360), so buffers, digests and
// seals are bit-compatible with the CPU HAL. Every result is canonical (< p).
//
// Arithmetic is written for the gfx950 integer pipe: the reductions use an
// unsigned min() instead of compare+branch (one v_min_u32), and the Montgomery
// step multiplies by -p^-1 so t + m*p folds into one 64-bit multiply-add.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define R0_HD __host__ __device__ __forceinline__
#else
#define R0_HD inline
#endif

namespace r0 {

constexpr uint32_t kP = 0x78000001u;        // 2013265921
constexpr uint32_t kNegPinv = 0x77ffffffu;  // -p^-1 mod 2^32
constexpr uint32_t kR2 = 1172168163u;       // 2^64 mod p

R0_HD uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

R0_HD uint32_t fp_add(uint32_t a, uint32_t b) {
  uint32_t s = a + b;  // < 2p < 2^32
  return umin(s, s - kP);
}
R0_HD uint32_t fp_sub(uint32_t a, uint32_t b) {
  uint32_t d = a - b;
  return umin(d, d + kP);
}
R0_HD uint32_t fp_neg(uint32_t a) { return fp_sub(0, a); }

// Montgomery REDC of t < p * 2^32: returns t * 2^-32 mod p, canonical.
R0_HD uint32_t mont_reduce(uint64_t t) {
  uint32_t m = uint32_t(t) * kNegPinv;
  uint32_t r = uint32_t((t + uint64_t(m) * kP) >> 32);
  return umin(r, r - kP);
}
R0_HD uint32_t fp_mul(uint32_t a, uint32_t b) { return mont_reduce(uint64_t(a) * b); }

// Congruent fold of any 64-bit value below 2^60 + 2^32: hi * (2^32 mod p) + lo —
// one v_mad_u64_u32; lets sums of several Montgomery products stay unreduced.
constexpr uint32_t kFoldC = uint32_t((uint64_t(1) << 32) % kP);  // 268435454
R0_HD uint64_t fold64(uint64_t x) { return uint64_t(uint32_t(x >> 32)) * kFoldC + uint32_t(x); }

constexpr uint32_t mont_mul_c(uint32_t a, uint32_t b) {
  // constexpr twin of fp_mul for compile-time constants
  return (uint32_t((uint64_t(a) * b + uint64_t(uint32_t(uint64_t(a) * b) * kNegPinv) * kP) >> 32) >= kP)
             ? uint32_t((uint64_t(a) * b + uint64_t(uint32_t(uint64_t(a) * b) * kNegPinv) * kP) >> 32) - kP
             : uint32_t((uint64_t(a) * b + uint64_t(uint32_t(uint64_t(a) * b) * kNegPinv) * kP) >> 32);
}
constexpr uint32_t fp_encode(uint32_t x) { return mont_mul_c(kR2, x % kP); }  // Elem::new
constexpr uint32_t fp_decode(uint32_t x) { return mont_mul_c(1, x); }
constexpr uint32_t kOne = fp_encode(1);
constexpr uint32_t kNBeta = fp_encode(kP - 11);
constexpr uint32_t kBeta = fp_encode(11);

R0_HD uint32_t fp_pow(uint32_t x, uint64_t n) {
  uint32_t tot = kOne;
  while (n) {
    if (n & 1) tot = fp_mul(tot, x);
    n >>= 1;
    x = fp_mul(x, x);
  }
  return tot;
}
// x^(p-2) (inv(0) = 0): p - 2 = 0x77FFFFFF = 0b1110111 then 24 ones, so x^7, then
// x^119 = (x^7)^16 * x^7, then eight 3-bit windows r = r^8 * x^7: 30 squarings and 11
// multiplies instead of square-and-multiply's 31 + 30
R0_HD uint32_t fp_inv(uint32_t x) {
  const uint32_t x2 = fp_mul(x, x), x3 = fp_mul(x2, x), x7 = fp_mul(fp_mul(x3, x3), x);
  uint32_t r = x7;
  for (int i = 0; i < 4; i++) r = fp_mul(r, r);
  r = fp_mul(r, x7);
  for (int w = 0; w < 8; w++) {
    r = fp_mul(r, r);
    r = fp_mul(r, r);
    r = fp_mul(fp_mul(r, r), x7);
  }
  return r;
}

// x[i] <- x[i]^-1 for N independent values (inv(0) = 0, as fp_inv): Montgomery's trick, one
// addition chain and 3(N-1) multiplies; zeros enter the running product as one
template <int N>
R0_HD void fp_inv_batch(uint32_t (&x)[N]) {
  uint32_t pre[N];
  uint32_t acc = x[0] == 0u ? kOne : x[0];
#pragma unroll
  for (int i = 1; i < N; i++) {
    pre[i] = acc;
    acc = fp_mul(acc, x[i] == 0u ? kOne : x[i]);
  }
  uint32_t inv = fp_inv(acc);
#pragma unroll
  for (int i = N - 1; i > 0; i--) {
    const uint32_t xi = x[i];
    const uint32_t o = fp_mul(inv, pre[i]);
    inv = fp_mul(inv, xi == 0u ? kOne : xi);
    x[i] = xi == 0u ? 0u : o;
  }
  x[0] = x[0] == 0u ? 0u : inv;
}

struct FpExt {
  uint32_t c[4];
};

R0_HD FpExt fe_zero() { return FpExt{{0, 0, 0, 0}}; }
R0_HD FpExt fe_one() { return FpExt{{kOne, 0, 0, 0}}; }
R0_HD FpExt fe_from_fp(uint32_t a) { return FpExt{{a, 0, 0, 0}}; }
R0_HD FpExt fe_add(FpExt a, FpExt b) {
  return FpExt{{fp_add(a.c[0], b.c[0]), fp_add(a.c[1], b.c[1]), fp_add(a.c[2], b.c[2]), fp_add(a.c[3], b.c[3])}};
}
R0_HD FpExt fe_sub(FpExt a, FpExt b) {
  return FpExt{{fp_sub(a.c[0], b.c[0]), fp_sub(a.c[1], b.c[1]), fp_sub(a.c[2], b.c[2]), fp_sub(a.c[3], b.c[3])}};
}
R0_HD FpExt fe_neg(FpExt a) { return fe_sub(fe_zero(), a); }
R0_HD FpExt fe_mul_fp(FpExt a, uint32_t b) {
  return FpExt{{fp_mul(a.c[0], b), fp_mul(a.c[1], b), fp_mul(a.c[2], b), fp_mul(a.c[3], b)}};
}

R0_HD FpExt fe_mul(FpExt a, FpExt b) {
  // Extension multiply (equal to baby_bear.rs:744-757) with lazy reduction: x^4 =
  // NBETA is applied to b's upper limbs first, then each output limb is a sum of
  // four 62-bit products (< 2^64), folded below p * 2^32 and reduced once.
  // Results are canonical, hence bit-identical to the reference.
  const uint32_t n1 = fp_mul(kNBeta, b.c[1]), n2 = fp_mul(kNBeta, b.c[2]), n3 = fp_mul(kNBeta, b.c[3]);
  const uint64_t a0 = a.c[0], a1 = a.c[1], a2 = a.c[2], a3 = a.c[3];
  uint64_t s0 = a0 * b.c[0] + a1 * n3 + a2 * n2 + a3 * n1;
  uint64_t s1 = a0 * b.c[1] + a1 * b.c[0] + a2 * n3 + a3 * n2;
  uint64_t s2 = a0 * b.c[2] + a1 * b.c[1] + a2 * b.c[0] + a3 * n3;
  uint64_t s3 = a0 * b.c[3] + a1 * b.c[2] + a2 * b.c[1] + a3 * b.c[0];
  return FpExt{{mont_reduce(fold64(s0)), mont_reduce(fold64(s1)), mont_reduce(fold64(s2)), mont_reduce(fold64(s3))}};
}
R0_HD FpExt fe_pow(FpExt x, uint64_t n) {
  FpExt tot = fe_one();
  while (n) {
    if (n & 1) tot = fe_mul(tot, x);
    n >>= 1;
    x = fe_mul(x, x);
  }
  return tot;
}
// baby_bear.rs:448-481
R0_HD FpExt fe_inv(FpExt x) {
  const uint32_t* a = x.c;
  uint32_t b0 = fp_add(fp_mul(a[0], a[0]),
                       fp_mul(kBeta, fp_sub(fp_mul(a[1], fp_add(a[3], a[3])), fp_mul(a[2], a[2]))));
  uint32_t b2 = fp_add(fp_sub(fp_mul(a[0], fp_add(a[2], a[2])), fp_mul(a[1], a[1])),
                       fp_mul(kBeta, fp_mul(a[3], a[3])));
  uint32_t c = fp_add(fp_mul(b0, b0), fp_mul(kBeta, fp_mul(b2, b2)));
  uint32_t ic = fp_inv(c);
  b0 = fp_mul(b0, ic);
  b2 = fp_mul(b2, ic);
  return FpExt{{fp_add(fp_mul(a[0], b0), fp_mul(kBeta, fp_mul(a[2], b2))),
                fp_add(fp_neg(fp_mul(a[1], b0)), fp_mul(kNBeta, fp_mul(a[3], b2))),
                fp_add(fp_neg(fp_mul(a[0], b2)), fp_mul(a[2], b0)),
                fp_sub(fp_mul(a[1], b2), fp_mul(a[3], b0))}};
}
R0_HD bool fe_eq(FpExt a, FpExt b) {
  return a.c[0] == b.c[0] && a.c[1] == b.c[1] && a.c[2] == b.c[2] && a.c[3] == b.c[3];
}

// Roots of unity (baby_bear.rs:184-197), plain integers; encode before use.
constexpr uint32_t kRouFwd[28] = {
    1,          2013265920, 284861408,  1801542727, 567209306,  740045640,  918899846,
    1881002012, 1453957774, 65325759,   1538055801, 515192888,  483885487,  157393079,
    1695124103, 2005211659, 1540072241, 88064245,   1542985445, 1269900459, 1461624142,
    825701067,  682402162,  1311873874, 1164520853, 352275361,  18769,      137};
constexpr uint32_t kRouRev[28] = {
    1,          2013265920, 1728404513, 1592366214, 196396260,  1253260071, 72041623,
    1091445674, 145223211,  1446820157, 1030796471, 2010749425, 1827366325, 1239938613,
    246299276,  596347512,  1893145354, 246074437,  1525739923, 1194341128, 1463599021,
    704606912,  95395244,   15672543,   647517488,  584175179,  137728885,  749463956};

R0_HD uint32_t bitrev32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_bitreverse32(x);
#else
  x = ((x & 0xaaaaaaaau) >> 1) | ((x & 0x55555555u) << 1);
  x = ((x & 0xccccccccu) >> 2) | ((x & 0x33333333u) << 2);
  x = ((x & 0xf0f0f0f0u) >> 4) | ((x & 0x0f0f0f0fu) << 4);
  x = ((x & 0xff00ff00u) >> 8) | ((x & 0x00ff00ffu) << 8);
  return (x << 16) | (x >> 16);
#endif
}
// reverse the low `bits` bits of x (bits may be 0)
R0_HD uint32_t bitrev_n(uint32_t x, uint32_t bits) { return bits ? bitrev32(x) >> (32 - bits) : 0u; }

}  // namespace r0
