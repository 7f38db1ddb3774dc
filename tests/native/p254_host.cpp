// Host build of the product's BN254 / Poseidon254 code (risc0_amd/csrc/bn254.h,
// poseidon254.h) driven line by line from stdin by tests/test_host_arith.py, which
// checks every answer against Python integers and tests/p254_ref.py.
//   mul  a[9] b[9]        -> 9 limbs of a*b/R          (limbs of a, b may be < 2^30)
//   sqr  a[9]             -> 9 limbs of a^2/R
//   dot3 m0 m1 m2 s0 s1 s2 c (9 limbs each) -> (sum m_j s_j + c R)/R
//   canon a[9]            -> 9 limbs of a/R, canonical
//   hash n v[0..n)        -> digest words of unpadded_hash over canonical values
//   pair a[8] b[8]        -> digest words of hash_pair
#include <cstdio>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "poseidon254.h"

using namespace r0;

static bn::Fr read_fr() {
  bn::Fr x;
  for (int i = 0; i < 9; i++) std::cin >> x.l[i];
  return x;
}
static void put(const uint32_t* v, int n) {
  for (int i = 0; i < n; i++) std::printf(i ? " %u" : "%u", v[i]);
  std::printf("\n");
}

int main() {
  std::string op;
  while (std::cin >> op) {
    if (op == "mul") {
      bn::Fr a = read_fr(), b = read_fr();
      put(bn::mul(a, b).l, 9);
    } else if (op == "sqr") {
      bn::Fr a = read_fr();
      put(bn::sqr(a).l, 9);
    } else if (op == "dot3") {
      bn::Fr m[3], s[3], c;
      for (auto& x : m) x = read_fr();
      for (auto& x : s) x = read_fr();
      c = read_fr();
      put(bn::dot3_add(m[0].l, m[1].l, m[2].l, s[0], s[1], s[2], c.l).l, 9);
    } else if (op == "canon") {
      bn::Fr a = read_fr();
      put(bn::to_canonical(a).l, 9);
    } else if (op == "hash") {
      size_t n;
      std::cin >> n;
      std::vector<uint32_t> v(n);
      for (auto& x : v) std::cin >> x;
      uint32_t d[8];
      p254_hash_canonical(v.data(), n, d);
      put(d, 8);
    } else if (op == "pair") {
      uint32_t a[8], b[8], d[8];
      for (auto& x : a) std::cin >> x;
      for (auto& x : b) std::cin >> x;
      p254_hash_pair(a, b, d);
      put(d, 8);
    }
    std::fflush(stdout);
  }
  return 0;
}
