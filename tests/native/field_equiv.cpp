// Host-side equivalence checks of the product's lean field/hash formulations against
// their step-by-step restatements (tests/test_host_arith.py builds and runs this).
#include <cstdio>
#include <cstdlib>
#include <random>

#include "poseidon2.h"

using namespace r0;

static int fails = 0;
#define EXPECT(c, ...)            \
  do {                            \
    if (!(c)) {                   \
      if (fails++ < 10) std::printf(__VA_ARGS__); \
    }                             \
  } while (0)

// reference extension multiply: baby_bear.rs:744-757 with canonical ops only
static FpExt fe_mul_simple(FpExt a, FpExt b) {
  uint32_t r[4];
  for (int k = 0; k < 4; k++) r[k] = 0;
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      uint32_t p = fp_mul(a.c[i], b.c[j]);
      if (i + j < 4) r[i + j] = fp_add(r[i + j], p);
      else r[i + j - 4] = fp_add(r[i + j - 4], fp_mul(kNBeta, p));
    }
  return FpExt{{r[0], r[1], r[2], r[3]}};
}

int main(int argc, char** argv) {
  int n = argc > 1 ? std::atoi(argv[1]) : 20000;
  std::mt19937_64 rng(12345);
  auto elem = [&](int mode) -> uint32_t {
    switch (mode) {
      case 0: return 0;
      case 1: return kP - 1;
      case 2: return kP - 1 - uint32_t(rng() % 8);
      default: return uint32_t(rng() % kP);
    }
  };
  for (int it = 0; it < n; it++) {
    int mode = it < 64 ? it % 4 : 3;
    uint32_t a[24], b[24];
    for (int i = 0; i < 24; i++) a[i] = b[i] = (it < 64 && (rng() & 1)) ? elem(mode) : elem(3);
    poseidon2_mix(a);
    poseidon2_mix_simple(b);
    for (int i = 0; i < 24; i++) EXPECT(a[i] == b[i], "poseidon2 mismatch it=%d cell=%d\n", it, i);
    // the signed full rounds read a word as int32: words in [p, 2^31) are still the right
    // value mod p (the tolerated range); the simple permutation gets their canonical form
    if (it < 2000) {
      for (int i = 0; i < 24; i++) {
        b[i] = uint32_t(rng() % kP);
        a[i] = (b[i] < 0x80000000u - kP && (rng() & 1)) ? b[i] + kP : b[i];
      }
      poseidon2_mix(a);
      poseidon2_mix_simple(b);
      for (int i = 0; i < 24; i++) EXPECT(a[i] == b[i], "poseidon2 [p, 2^31) input mismatch it=%d cell=%d\n", it, i);
    }
    FpExt x{{elem(mode), elem(3), elem(mode), elem(3)}}, y{{elem(3), elem(mode), elem(mode), elem(3)}};
    FpExt u = fe_mul(x, y), v = fe_mul_simple(x, y);
    for (int k = 0; k < 4; k++) EXPECT(u.c[k] == v.c[k], "fe_mul mismatch it=%d\n", it);
    uint64_t t = (uint64_t(rng()) >> 4);
    EXPECT(mont_reduce(fold64(t)) == mont_reduce(fold64(fold64(t))), "fold64 it=%d\n", it);
  }
  std::printf("%s (%d cases)\n", fails ? "FAIL" : "OK", n);
  return fails ? 1 : 0;
}
