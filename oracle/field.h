// ORACLE (test infrastructure only — never linked into the product path).
//
// CPU restatement of the BabyBear field and its degree-4 extension exactly as
// the reference defines them:
//   risc0/core/src/field/baby_bear.rs:40-42   (Montgomery constants M, R2)
//   risc0/core/src/field/baby_bear.rs:84      (P = 15*2^27 + 1)
//   risc0/core/src/field/baby_bear.rs:323-360 (add / sub / mul / encode / decode)
//   risc0/core/src/field/baby_bear.rs:184-197 (ROU_FWD / ROU_REV tables)
//   risc0/core/src/field/baby_bear.rs:433-481 (ExtElem pow / inv)
//   risc0/core/src/field/baby_bear.rs:744-757 (ExtElem mul, x^4 + 11)
// Elements are held as raw Montgomery words, as the reference buffers hold them.
#pragma once
#include <cstdint>
#include <cstddef>

namespace oracle {

constexpr uint32_t P = 15u * (1u << 27) + 1u;  // 2013265921
constexpr uint32_t M = 0x88000001u;             // P^-1 mod 2^32
constexpr uint32_t R2 = 1172168163u;            // 2^64 mod P
constexpr uint32_t INVALID = 0xffffffffu;

// baby_bear.rs:324-327
inline uint32_t add(uint32_t a, uint32_t b) {
  uint32_t x = a + b;
  return x >= P ? x - P : x;
}
// baby_bear.rs:330-333
inline uint32_t sub(uint32_t a, uint32_t b) {
  uint32_t x = a - b;
  return x > P ? x + P : x;
}
// baby_bear.rs:337-350
inline uint32_t mul(uint32_t a, uint32_t b) {
  uint64_t o64 = uint64_t(a) * uint64_t(b);
  uint32_t low = 0u - uint32_t(o64);
  uint32_t red = M * low;
  o64 += uint64_t(red) * uint64_t(P);
  uint32_t ret = uint32_t(o64 >> 32);
  return ret >= P ? ret - P : ret;
}
inline uint32_t encode(uint32_t a) { return mul(R2, a % P); }  // Elem::new
inline uint32_t decode(uint32_t a) { return mul(1, a); }       // Elem::as_u32

struct Elem {
  uint32_t v;  // Montgomery form
  static Elem raw(uint32_t x) { return Elem{x}; }
  static Elem from(uint64_t x) { return Elem{encode(uint32_t(x % P))}; }
  static Elem zero() { return Elem{0}; }
  static Elem one() { return from(1); }
  Elem operator+(Elem o) const { return Elem{add(v, o.v)}; }
  Elem operator-(Elem o) const { return Elem{sub(v, o.v)}; }
  Elem operator*(Elem o) const { return Elem{mul(v, o.v)}; }
  Elem operator-() const { return Elem{sub(0, v)}; }
  Elem& operator+=(Elem o) { v = add(v, o.v); return *this; }
  Elem& operator-=(Elem o) { v = sub(v, o.v); return *this; }
  Elem& operator*=(Elem o) { v = mul(v, o.v); return *this; }
  bool operator==(Elem o) const { return v == o.v; }
  bool operator!=(Elem o) const { return v != o.v; }
  uint32_t as_u32() const { return decode(v); }
  // field/mod.rs Elem::pow: square-and-multiply
  Elem pow(uint64_t n) const {
    Elem tot = one(), x = *this;
    while (n) {
      if (n & 1) tot *= x;
      n >>= 1;
      x *= x;
    }
    return tot;
  }
  Elem inv() const { return pow(P - 2); }  // baby_bear.rs:105-107
  Elem valid_or_zero() const { return v == INVALID ? zero() : *this; }
};

// ROU tables, baby_bear.rs:184-197 (given as plain integers, stored encoded).
extern const uint32_t ROU_FWD_INT[28];
extern const uint32_t ROU_REV_INT[28];
inline Elem rou_fwd(size_t n) { return Elem::from(ROU_FWD_INT[n]); }
inline Elem rou_rev(size_t n) { return Elem::from(ROU_REV_INT[n]); }

struct ExtElem {
  Elem e[4];
  static ExtElem zero() { return ExtElem{{Elem::zero(), Elem::zero(), Elem::zero(), Elem::zero()}}; }
  static ExtElem one() { return ExtElem{{Elem::one(), Elem::zero(), Elem::zero(), Elem::zero()}}; }
  static ExtElem from_fp(Elem x) { return ExtElem{{x, Elem::zero(), Elem::zero(), Elem::zero()}}; }
  static ExtElem raw(const uint32_t* w) {
    return ExtElem{{Elem::raw(w[0]), Elem::raw(w[1]), Elem::raw(w[2]), Elem::raw(w[3])}};
  }
  void store(uint32_t* w) const {
    for (int i = 0; i < 4; i++) w[i] = e[i].v;
  }
  ExtElem operator+(const ExtElem& o) const {
    ExtElem r;
    for (int i = 0; i < 4; i++) r.e[i] = e[i] + o.e[i];
    return r;
  }
  ExtElem operator-(const ExtElem& o) const {
    ExtElem r;
    for (int i = 0; i < 4; i++) r.e[i] = e[i] - o.e[i];
    return r;
  }
  ExtElem operator-() const { return zero() - *this; }
  ExtElem operator*(Elem b) const {
    ExtElem r;
    for (int i = 0; i < 4; i++) r.e[i] = e[i] * b;
    return r;
  }
  // baby_bear.rs:744-757
  ExtElem operator*(const ExtElem& o) const {
    const Elem* a = e;
    const Elem* b = o.e;
    const Elem NBETA = Elem::from(P - 11);
    ExtElem r;
    r.e[0] = a[0] * b[0] + NBETA * (a[1] * b[3] + a[2] * b[2] + a[3] * b[1]);
    r.e[1] = a[0] * b[1] + a[1] * b[0] + NBETA * (a[2] * b[3] + a[3] * b[2]);
    r.e[2] = a[0] * b[2] + a[1] * b[1] + a[2] * b[0] + NBETA * (a[3] * b[3]);
    r.e[3] = a[0] * b[3] + a[1] * b[2] + a[2] * b[1] + a[3] * b[0];
    return r;
  }
  ExtElem& operator+=(const ExtElem& o) { return *this = *this + o; }
  ExtElem& operator-=(const ExtElem& o) { return *this = *this - o; }
  ExtElem& operator*=(const ExtElem& o) { return *this = *this * o; }
  ExtElem& operator*=(Elem o) { return *this = *this * o; }
  bool operator==(const ExtElem& o) const {
    for (int i = 0; i < 4; i++)
      if (e[i] != o.e[i]) return false;
    return true;
  }
  bool operator!=(const ExtElem& o) const { return !(*this == o); }
  // baby_bear.rs:433-445
  ExtElem pow(uint64_t n) const {
    ExtElem tot = one(), x = *this;
    while (n) {
      if (n & 1) tot *= x;
      n >>= 1;
      x *= x;
    }
    return tot;
  }
  // baby_bear.rs:448-481
  ExtElem inv() const {
    const Elem BETA = Elem::from(11), NBETA = Elem::from(P - 11);
    const Elem* a = e;
    Elem b0 = a[0] * a[0] + BETA * (a[1] * (a[3] + a[3]) - a[2] * a[2]);
    Elem b2 = a[0] * (a[2] + a[2]) - a[1] * a[1] + BETA * (a[3] * a[3]);
    Elem c = b0 * b0 + BETA * b2 * b2;
    Elem ic = c.inv();
    b0 *= ic;
    b2 *= ic;
    ExtElem r;
    r.e[0] = a[0] * b0 + BETA * a[2] * b2;
    r.e[1] = -a[1] * b0 + NBETA * a[3] * b2;
    r.e[2] = -a[0] * b2 + a[2] * b0;
    r.e[3] = a[1] * b2 - a[3] * b0;
    return r;
  }
};

}  // namespace oracle
