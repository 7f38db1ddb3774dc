// BN254 scalar field Fr (r = 21888242871839275222246405745257275088548364400416034343698204186575808495617,
// risc0/zkp/src/core/hash/poseidon_254/consts.rs:19-23) for the Poseidon254 hash suite, host+device.
//
// Representation (this backend's own, internal to hashing): 9 limbs of 29 bits, little-endian,
// Montgomery form with R = 2^261. Digests cross the boundary as the reference's canonical
// little-endian 8 x u32 words (mod.rs:94-105), converted at the edges.
//
// Why 29-bit limbs on CDNA4: every limb product is < 2^58, so one 64-bit accumulator takes a
// whole column of products — up to 36 of them — with one v_mad_u64_u32 each and no carry
// instructions. A Montgomery product is product scanning with the REDC interleaved per
// column (81 + 81 multiply-adds plus ~3 ops per column), against ~3 VALU ops per limb product
// for 32-bit limbs with explicit carry chains.
//
// Lazy values: r < 2^254 is 2^-7 of R, so REDC(T) < T/R + r stays a hair above r for every
// T used here; cells stay below ~2.1r and are canonicalised only when a digest is written.
// Column bounds (products of limbs < 2^30 where an unreduced sum fed a product) are
// documented at each use and checked by tests/native/p254_host.cpp on extreme inputs.
#pragma once
#include "bb31.h"
#include "poseidon254_consts.inc"

namespace r0 {
namespace bn {

constexpr int kL = 29;
constexpr uint32_t kMask = (1u << kL) - 1;
constexpr uint32_t kMod[9] = P254_MOD_L29;
constexpr uint32_t kNinv = P254_NINV_L29;  // -r^-1 mod 2^29
constexpr uint32_t kR2[9] = P254_R2_L29;

struct Fr {
  uint32_t l[9];
};

// acc + a*b: one v_mad_u64_u32
R0_HD uint64_t mac(uint32_t a, uint32_t b, uint64_t acc) { return uint64_t(a) * b + acc; }

// out = (T + c*R) / R mod r for the T whose column k (sum of the limb products of weight
// 2^(29k), k = 0..16) is added by cols(k, acc); c (optional, 9 limbs < 2^29) lands in the
// high columns. Every column sum plus the m*r terms (<= 9 * 2^58) must stay below 2^64.
template <class Cols>
R0_HD void redc(Fr& out, Cols cols, const uint32_t* c = nullptr) {
  uint64_t acc = 0;
  uint32_t m[9];
#pragma unroll
  for (int k = 0; k < 17; k++) {
    acc = cols(k, acc);
#pragma unroll
    for (int i = 0; i < 9; i++)
      if (i < k && k - i <= 8) acc = mac(m[i], kMod[k - i], acc);
    if (k < 9) {
      m[k] = (uint32_t(acc) * kNinv) & kMask;
      acc = mac(m[k], kMod[0], acc);  // low 29 bits become zero
    } else {
      if (c) acc += c[k - 9];
      out.l[k - 9] = uint32_t(acc) & kMask;
    }
    acc >>= kL;
  }
  out.l[8] = uint32_t(acc) + (c ? c[8] : 0u);
}

// a*b/R. Limbs of a and b < 2^30: a column has <= 9 products < 2^60 (9 * 2^60 + 9 * 2^58 < 2^64).
R0_HD Fr mul(const Fr& a, const Fr& b) {
  Fr o;
  redc(o, [&](int k, uint64_t acc) {
#pragma unroll
    for (int i = 0; i < 9; i++)
      if (k - i >= 0 && k - i <= 8) acc = mac(a.l[i], b.l[k - i], acc);
    return acc;
  });
  return o;
}

// a^2/R: cross products once with a doubled factor (45 products instead of 81). Limbs of a
// < 2^30: a column has <= 4 doubled products < 2^61 and one square < 2^60 (11.25 * 2^60 < 2^64).
R0_HD Fr sqr(const Fr& a) {
  uint32_t d[9];
#pragma unroll
  for (int i = 0; i < 9; i++) d[i] = a.l[i] << 1;
  Fr o;
  redc(o, [&](int k, uint64_t acc) {
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j > i && j <= 8) acc = mac(d[i], a.l[j], acc);
    }
    if ((k & 1) == 0 && k / 2 <= 8) acc = mac(a.l[k / 2], a.l[k / 2], acc);
    return acc;
  });
  return o;
}

// (sum_j m[j] * s[j] + c*R) / R: three products share one reduction. Limbs of m < 2^29 and
// of s < 2^30: a column has <= 27 products < 2^59 (13.5 * 2^60 + 2.25 * 2^60 < 2^64).
R0_HD Fr dot3_add(const uint32_t* m0, const uint32_t* m1, const uint32_t* m2, const Fr& s0, const Fr& s1,
                  const Fr& s2, const uint32_t* c) {
  Fr o;
  redc(
      o,
      [&](int k, uint64_t acc) {
#pragma unroll
        for (int i = 0; i < 9; i++) {
          const int j = k - i;
          if (j >= 0 && j <= 8) {
            acc = mac(s0.l[i], m0[j], acc);
            acc = mac(s1.l[i], m1[j], acc);
            acc = mac(s2.l[i], m2[j], acc);
          }
        }
        return acc;
      },
      c);
  return o;
}

// (w * s + e*R) / R for a constant w: one product and the addend e (limbs < 2^30) in the
// high columns.
R0_HD Fr mul_add(const uint32_t* w, const Fr& s, const uint32_t* e) {
  Fr o;
  redc(
      o,
      [&](int k, uint64_t acc) {
#pragma unroll
        for (int i = 0; i < 9; i++)
          if (k - i >= 0 && k - i <= 8) acc = mac(s.l[i], w[k - i], acc);
        return acc;
      },
      e);
  return o;
}

// x/R (leaves Montgomery form), then the single conditional subtraction to canonical:
// x < 2.2r gives x/R < r + 1 before it.
R0_HD Fr to_canonical(const Fr& x) {
  Fr o;
  redc(o, [&](int k, uint64_t acc) { return k < 9 ? acc + x.l[k] : acc; });
  // o - r with borrows in 29-bit limbs; keep it when nonnegative
  Fr d;
  int64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    int64_t t = int64_t(o.l[i]) - int64_t(kMod[i]) + borrow;
    d.l[i] = uint32_t(t) & kMask;
    borrow = t >> kL;
  }
  return borrow < 0 ? o : d;
}

// canonical 8 x u32 little-endian words <-> 9 x 29-bit limbs (plain integers)
R0_HD Fr from_words(const uint32_t* w) {
  Fr o;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int bit = kL * i, wi = bit / 32, sh = bit % 32;
    uint64_t v = uint64_t(w[wi]) >> sh;
    if (wi + 1 < 8) v |= uint64_t(w[wi + 1]) << (32 - sh);
    o.l[i] = uint32_t(v) & kMask;
  }
  return o;
}
R0_HD void to_words(const Fr& x, uint32_t* w) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int bit = 32 * i, li = bit / kL, sh = bit % kL;
    uint64_t v = uint64_t(x.l[li]) >> sh;
    if (li + 1 < 9) v |= uint64_t(x.l[li + 1]) << (kL - sh);
    if (li + 2 < 9 && kL - sh + kL < 32) v |= uint64_t(x.l[li + 2]) << (2 * kL - sh);
    w[i] = uint32_t(v);
  }
}

// plain integer x (limbs < 2^29, x < 2^261) -> Montgomery x*R mod r
R0_HD Fr to_mont(const Fr& x) {
  const Fr r2{P254_R2_L29};
  return mul(x, r2);
}

// a + b with carries propagated (normalised limbs)
R0_HD Fr add_norm(const Fr& a, const uint32_t* b) {
  Fr o;
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint32_t s = a.l[i] + b[i] + carry;
    o.l[i] = s & kMask;
    carry = s >> kL;
  }
  o.l[8] += carry << kL;
  return o;
}

}  // namespace bn
}  // namespace r0
