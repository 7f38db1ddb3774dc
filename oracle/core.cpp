// ORACLE (test infrastructure only — never linked into the product path).
#include "core.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace oracle {

// baby_bear.rs:184-197
const uint32_t ROU_FWD_INT[28] = {
    1,          2013265920, 284861408,  1801542727, 567209306,  740045640,  918899846,
    1881002012, 1453957774, 65325759,   1538055801, 515192888,  483885487,  157393079,
    1695124103, 2005211659, 1540072241, 88064245,   1542985445, 1269900459, 1461624142,
    825701067,  682402162,  1311873874, 1164520853, 352275361,  18769,      137};
const uint32_t ROU_REV_INT[28] = {
    1,          2013265920, 1728404513, 1592366214, 196396260,  1253260071, 72041623,
    1091445674, 145223211,  1446820157, 1030796471, 2010749425, 1827366325, 1239938613,
    246299276,  596347512,  1893145354, 246074437,  1525739923, 1194341128, 1463599021,
    704606912,  95395244,   15672543,   647517488,  584175179,  137728885,  749463956};

// ---------------------------------------------------------------------------
size_t num_threads() {
  static size_t n = [] {
    const char* s = getenv("ORACLE_THREADS");
    if (s && atoi(s) > 0) return (size_t)atoi(s);
    // every hardware thread unless the caller says otherwise (bench.py passes the CPUs the
    // process may use: its affinity mask, capped by the cgroup CPU quota)
    size_t hc = std::thread::hardware_concurrency();
    return hc ? hc : size_t(1);
  }();
  return n;
}

void parallel_for(size_t n, const std::function<void(size_t, size_t)>& f) {
  size_t nt = std::min(num_threads(), n);
  if (nt <= 1) {
    if (n) f(0, n);
    return;
  }
  std::vector<std::thread> ts;
  size_t chunk = (n + nt - 1) / nt;
  for (size_t t = 0; t < nt; t++) {
    size_t b = t * chunk, e = std::min(n, b + chunk);
    if (b >= e) break;
    ts.emplace_back([&f, b, e] { f(b, e); });
  }
  for (auto& t : ts) t.join();
}

// ---------------------------------------------------------------------------
// ntt.rs:34-45
uint32_t bit_rev_32(uint32_t x) {
  x = ((x & 0xaaaaaaaau) >> 1) | ((x & 0x55555555u) << 1);
  x = ((x & 0xccccccccu) >> 2) | ((x & 0x33333333u) << 2);
  x = ((x & 0xf0f0f0f0u) >> 4) | ((x & 0x0f0f0f0fu) << 4);
  x = ((x & 0xff00ff00u) >> 8) | ((x & 0x00ff00ffu) << 8);
  return (x << 16) | (x >> 16);
}

size_t log2_ceil(size_t value) {
  size_t r = 0;
  while ((size_t(1) << r) < value) r++;
  return r;
}

// ntt.rs:64-73
void bit_reverse(Elem* io, size_t len) {
  size_t n = log2_ceil(len);
  if (len <= 1) return;
  for (size_t i = 0; i < len; i++) {
    size_t rev = bit_rev_32((uint32_t)i) >> (32 - n);
    if (i < rev) std::swap(io[i], io[rev]);
  }
}

// ntt.rs:91-112 (fwd_butterfly_$n, recursive DIT)
static void fwd_butterfly(Elem* io, size_t n, size_t expand_bits) {
  if (n == 0 || n == expand_bits) return;
  size_t half = size_t(1) << (n - 1);
  fwd_butterfly(io, n - 1, expand_bits);
  fwd_butterfly(io + half, n - 1, expand_bits);
  Elem step = rou_fwd(n);
  Elem cur = Elem::one();
  for (size_t i = 0; i < half; i++) {
    Elem a = io[i];
    Elem b = io[i + half] * cur;
    io[i] = a + b;
    io[i + half] = a - b;
    cur *= step;
  }
}

// ntt.rs:115-133 (rev_butterfly_$n, recursive DIF)
static void rev_butterfly(Elem* io, size_t n) {
  if (n == 0) return;
  size_t half = size_t(1) << (n - 1);
  Elem step = rou_rev(n);
  Elem cur = Elem::one();
  for (size_t i = 0; i < half; i++) {
    Elem a = io[i];
    Elem b = io[i + half];
    io[i] = a + b;
    io[i + half] = (a - b) * cur;
    cur *= step;
  }
  rev_butterfly(io, n - 1);
  rev_butterfly(io + half, n - 1);
}

// ntt.rs:232-281
void interpolate_ntt(Elem* io, size_t size) {
  size_t n = log2_ceil(size);
  rev_butterfly(io, n);
  Elem norm = Elem::from(size).inv();
  for (size_t i = 0; i < size; i++) io[i] = io[i] * norm;
}

// ntt.rs:284-330
void evaluate_ntt(Elem* io, size_t size, size_t expand_bits) {
  size_t n = log2_ceil(size);
  fwd_butterfly(io, n, expand_bits);
}

// ntt.rs:334-342
void expand(Elem* out, const Elem* in, size_t in_n, size_t expand_bits) {
  size_t out_n = in_n << expand_bits;
  for (size_t i = 0; i < out_n; i++) out[i] = in[i >> expand_bits];
}

// ---------------------------------------------------------------------------
// Poseidon2 (poseidon2/mod.rs, consts.rs)
#include "poseidon2_consts.inc"

namespace {
struct P2Consts {
  Elem rc[29 * 24];
  Elem diag[24];
  P2Consts() {
    for (int i = 0; i < 29 * 24; i++) rc[i] = Elem::from(ROUND_CONSTANTS_INT[i]);
    for (int i = 0; i < 24; i++) diag[i] = Elem::from(M_INT_DIAG_HZN_INT[i]);
  }
};
const P2Consts& p2c() {
  static P2Consts c;
  return c;
}
constexpr int CELLS = 24, ROUNDS_HALF_FULL = 4, ROUNDS_PARTIAL = 21, CELLS_RATE = 16,
              CELLS_OUT = 8;

// mod.rs:112-117
inline Elem sbox(Elem x) {
  Elem x2 = x * x;
  Elem x4 = x2 * x2;
  Elem x6 = x4 * x2;
  return x6 * x;
}
// mod.rs:129-135
void multiply_by_m_int(Elem* cells) {
  Elem sum = Elem::zero();
  for (int i = 0; i < CELLS; i++) sum += cells[i];
  for (int i = 0; i < CELLS; i++) cells[i] = sum + p2c().diag[i] * cells[i];
}
// mod.rs:137-148
void mul_4x4_circulant(const Elem* x, Elem* out) {
  Elem two = Elem::from(2), four = Elem::from(4);
  Elem t0 = x[0] + x[1];
  Elem t1 = x[2] + x[3];
  Elem t2 = two * x[1] + t1;
  Elem t3 = two * x[3] + t0;
  Elem t4 = four * t1 + t3;
  Elem t5 = four * t0 + t2;
  Elem t6 = t3 + t5;
  Elem t7 = t2 + t4;
  out[0] = t6;
  out[1] = t5;
  out[2] = t7;
  out[3] = t4;
}
// mod.rs:150-173
void multiply_by_m_ext(Elem* cells) {
  Elem old[CELLS];
  for (int i = 0; i < CELLS; i++) old[i] = cells[i];
  Elem tmp[4] = {Elem::zero(), Elem::zero(), Elem::zero(), Elem::zero()};
  for (int i = 0; i < CELLS; i++) cells[i] = Elem::zero();
  for (int i = 0; i < CELLS / 4; i++) {
    Elem out[4];
    mul_4x4_circulant(old + i * 4, out);
    for (int j = 0; j < 4; j++) {
      tmp[j] += out[j];
      cells[i * 4 + j] += out[j];
    }
  }
  for (int i = 0; i < CELLS; i++) cells[i] += tmp[i % 4];
}
}  // namespace

// mod.rs:193-216
void poseidon2_mix(Elem* cells) {
  const P2Consts& c = p2c();
  int round = 0;
  multiply_by_m_ext(cells);
  for (int r = 0; r < ROUNDS_HALF_FULL; r++, round++) {
    for (int i = 0; i < CELLS; i++) cells[i] += c.rc[round * CELLS + i];
    for (int i = 0; i < CELLS; i++) cells[i] = sbox(cells[i]);
    multiply_by_m_ext(cells);
  }
  for (int r = 0; r < ROUNDS_PARTIAL; r++, round++) {
    cells[0] += c.rc[round * CELLS];
    cells[0] = sbox(cells[0]);
    multiply_by_m_int(cells);
  }
  for (int r = 0; r < ROUNDS_HALF_FULL; r++, round++) {
    for (int i = 0; i < CELLS; i++) cells[i] += c.rc[round * CELLS + i];
    for (int i = 0; i < CELLS; i++) cells[i] = sbox(cells[i]);
    multiply_by_m_ext(cells);
  }
}

// mod.rs:221-245, to_digest mod.rs:94-100
Digest poseidon2_hash_elems(const Elem* e, size_t n) {
  Elem state[CELLS];
  for (int i = 0; i < CELLS; i++) state[i] = Elem::zero();
  size_t count = 0, unmixed = 0;
  for (size_t k = 0; k < n; k++) {
    state[unmixed] = e[k];
    count++;
    unmixed++;
    if (unmixed == (size_t)CELLS_RATE) {
      poseidon2_mix(state);
      unmixed = 0;
    }
  }
  if (unmixed != 0 || count == 0) {
    for (size_t i = unmixed; i < (size_t)CELLS_RATE; i++) state[i] = Elem::zero();
    poseidon2_mix(state);
  }
  Digest d;
  for (int i = 0; i < CELLS_OUT; i++) d.w[i] = state[i].v;
  return d;
}

// mod.rs:47-59 (inputs must be reduced; the reference asserts it)
Digest poseidon2_hash_pair(const Digest& a, const Digest& b) {
  Elem both[16];
  for (int i = 0; i < 8; i++) {
    both[i] = Elem::raw(a.w[i]);
    both[8 + i] = Elem::raw(b.w[i]);
  }
  for (int i = 0; i < 16; i++)
    if (both[i].v >= P) abort();
  return poseidon2_hash_elems(both, 16);
}

// ---------------------------------------------------------------------------
// SHA-256 (FIPS 180-4). The reference uses the sha2 crate's compress256.
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
static const uint32_t IV256[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                  0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
static inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
static inline uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

void sha256_compress(uint32_t s[8], const uint8_t blk[64]) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = (uint32_t(blk[4 * i]) << 24) | (uint32_t(blk[4 * i + 1]) << 16) |
           (uint32_t(blk[4 * i + 2]) << 8) | uint32_t(blk[4 * i + 3]);
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
  for (int i = 0; i < 64; i++) {
    uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + K256[i] + w[i];
    uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
}

// Digest words hold the big-endian digest bytes in memory order (sha/cpu.rs:41-48,73-76).
static Digest state_to_digest(const uint32_t s[8]) {
  Digest d;
  for (int i = 0; i < 8; i++) d.w[i] = bswap(s[i]);
  return d;
}

Digest sha256_hash_bytes(const uint8_t* bytes, size_t n) {
  uint32_t s[8];
  memcpy(s, IV256, sizeof(s));
  size_t full = n / 64;
  for (size_t i = 0; i < full; i++) sha256_compress(s, bytes + 64 * i);
  uint8_t last[128];
  memset(last, 0, sizeof(last));
  size_t rem = n - 64 * full;
  memcpy(last, bytes + 64 * full, rem);
  last[rem] = 0x80;
  size_t tot = (rem + 1 + 8 <= 64) ? 64 : 128;
  uint64_t bits = uint64_t(n) * 8;
  for (int i = 0; i < 8; i++) last[tot - 1 - i] = uint8_t(bits >> (8 * i));
  sha256_compress(s, last);
  if (tot == 128) sha256_compress(s, last + 64);
  return state_to_digest(s);
}

// cpu.rs:56-77: compress the LE bytes of the words, zero-fill the last block, no trailer
Digest sha256_hash_raw_words(const uint32_t* words, size_t n) {
  uint32_t s[8];
  memcpy(s, IV256, sizeof(s));
  const uint8_t* bytes = reinterpret_cast<const uint8_t*>(words);
  size_t nb = n * 4, full = nb / 64;
  for (size_t i = 0; i < full; i++) sha256_compress(s, bytes + 64 * i);
  size_t rem = nb - 64 * full;
  if (rem) {
    uint8_t last[64];
    memset(last, 0, 64);
    memcpy(last, bytes + 64 * full, rem);
    sha256_compress(s, last);
  }
  return state_to_digest(s);
}

// sha/mod.rs:96-98 + cpu.rs:81-105: one compression of a||b from the IV
Digest sha256_hash_pair(const Digest& a, const Digest& b) {
  uint32_t s[8];
  memcpy(s, IV256, sizeof(s));
  uint8_t blk[64];
  memcpy(blk, a.w, 32);
  memcpy(blk + 32, b.w, 32);
  sha256_compress(s, blk);
  return state_to_digest(s);
}

Digest hash_elem_slice(int suite, const Elem* e, size_t n) {
  if (suite == SUITE_POSEIDON2) return poseidon2_hash_elems(e, n);
  if (suite == SUITE_POSEIDON254) return poseidon254_hash_elems(e, n);
  return sha256_hash_raw_words(reinterpret_cast<const uint32_t*>(e), n);
}
Digest hash_ext_elem_slice(int suite, const ExtElem* e, size_t n) {
  if (suite == SUITE_POSEIDON2) return poseidon2_hash_elems(&e[0].e[0], 4 * n);
  if (suite == SUITE_POSEIDON254) return poseidon254_hash_elems(&e[0].e[0], 4 * n);
  return sha256_hash_raw_words(reinterpret_cast<const uint32_t*>(e), 4 * n);
}
Digest hash_pair(int suite, const Digest& a, const Digest& b) {
  if (suite == SUITE_POSEIDON2) return poseidon2_hash_pair(a, b);
  if (suite == SUITE_POSEIDON254) return poseidon254_hash_pair(a, b);
  return sha256_hash_pair(a, b);
}

// ---------------------------------------------------------------------------
// poseidon2/rng.rs:26-89
struct Poseidon2Rng : Rng {
  Elem cells[24];
  size_t pool_used = 0;
  Poseidon2Rng() {
    for (int i = 0; i < 24; i++) cells[i] = Elem::zero();
  }
  void mix(const Digest& d) override {
    if (pool_used != 0) {
      poseidon2_mix(cells);
      pool_used = 0;
    }
    for (int i = 0; i < 8; i++) cells[i] += Elem::raw(d.w[i]);
    poseidon2_mix(cells);
  }
  uint32_t random_bits(size_t bits) override {
    uint32_t val = random_elem().as_u32();
    for (int i = 0; i < 3; i++) {
      uint32_t nv = random_elem().as_u32();
      if (val == 0) val = nv;
    }
    return uint32_t((uint64_t(1) << bits) - 1) & val;
  }
  Elem random_elem() override {
    if (pool_used == (size_t)CELLS_RATE) {
      poseidon2_mix(cells);
      pool_used = 0;
    }
    return cells[pool_used++];
  }
  ExtElem random_ext_elem() override {
    ExtElem r;
    for (int i = 0; i < 4; i++) r.e[i] = random_elem();
    return r;
  }
};

// sha/rng.rs:26-101
struct ShaRng : Rng {
  Digest pool0, pool1;
  size_t pool_used = 0;
  ShaRng() {
    pool0 = sha256_hash_bytes(reinterpret_cast<const uint8_t*>("Hello"), 5);
    pool1 = sha256_hash_bytes(reinterpret_cast<const uint8_t*>("World"), 5);
  }
  void step() {
    pool0 = sha256_hash_pair(pool0, pool1);
    pool1 = sha256_hash_pair(pool0, pool1);
    pool_used = 0;
  }
  uint32_t next_u32() {
    if (pool_used == 8) step();
    return pool0.w[pool_used++];
  }
  void mix(const Digest& d) override {
    for (int i = 0; i < 8; i++) pool0.w[i] ^= d.w[i];
    step();
  }
  uint32_t random_bits(size_t bits) override { return uint32_t((uint64_t(1) << bits) - 1) & next_u32(); }
  // baby_bear.rs:110-140
  Elem random_elem() override {
    uint64_t val = 0;
    for (int i = 0; i < 6; i++) {
      val <<= 32;
      val += next_u32();
      val %= P;
    }
    return Elem::from(val);
  }
  ExtElem random_ext_elem() override {
    ExtElem r;
    for (int i = 0; i < 4; i++) r.e[i] = random_elem();
    return r;
  }
};

std::unique_ptr<Rng> new_rng(int suite) {
  if (suite == SUITE_POSEIDON2) return std::unique_ptr<Rng>(new Poseidon2Rng());
  if (suite == SUITE_POSEIDON254) return new_poseidon254_rng();
  return std::unique_ptr<Rng>(new ShaRng());
}

}  // namespace oracle
