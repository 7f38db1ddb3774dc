// Merkle leaf and node hashing on CDNA4: Poseidon2 and SHA-256 row hashes
// (hash_rows) and pair compressions (hash_fold), and a fused tree builder.
//
//   hash_rows : risc0/zkp/src/hal/cpu.rs:555-567 -> HashFn::hash_elem_slice of one
//               row of a column-major matrix (poseidon2/mod.rs:221-245 unpadded
//               sponge; sha/cpu.rs:56-77 unpadded SHA-256 over LE word bytes)
//   hash_fold : cpu.rs:569-581 -> HashFn::hash_pair (poseidon2/mod.rs:47-59;
//               sha/mod.rs:96-98 single compression from the IV)
// One lane hashes one row: consecutive lanes read consecutive rows of each
// column, so every column read is a fully coalesced 256-byte wave access; the
// 24-cell state lives in VGPRs. Poseidon2 is integer-VALU bound (~1.4k modmul per
// permutation), not HBM bound.
#include "poseidon2.h"
#include "poseidon254.h"
#include "runtime.h"
#include "transcript.h"

#include <map>
#include <mutex>
#include <tuple>

namespace r0 {
namespace {

constexpr int kThreads = 256;
constexpr double kP2Modmuls = 8 * 24 * 4 + 21 * 4 + 21 * 24;

__device__ __forceinline__ void store_digest(uint32_t* out, const uint32_t* d) {
  uint4* o = reinterpret_cast<uint4*>(out);
  o[0] = make_uint4(d[0], d[1], d[2], d[3]);
  o[1] = make_uint4(d[4], d[5], d[6], d[7]);
}

// ---- zero subtrees (Poseidon2, SHA-256) -------------------------------------------------
// An all-zero row hashes to a constant of the hash (Z_0: one permutation / compression of
// a zero block for rows of <= 16 columns), and a node whose two children are both Z_k is
// Z_{k+1} = hash_pair(Z_k, Z_k): the empty-subtree digests of a sparse Merkle tree.
// rv32im's code group is one column of zeros in every proof (the reference allocates it
// zero-filled and zeroizes it: rv32im/src/prove/witgen/mod.rs:152,168), so its leaves and
// every layer above them are these constants. A wave whose rows (or child pairs) all match
// stores the constant and skips the permutation; any other wave hashes as before, so the
// words are the same for every input (the host computes the chain with the transcript's
// hash functions, transcript.h, whose words the row and fold tests pin to the kernels').
struct ZeroSub {
  uint32_t in[8];   // Z_k: the digest both children must equal (fold kernels)
  uint32_t out[8];  // Z_{k+1} (fold kernels) or Z_0 (row kernels)
  uint32_t on;
};
__device__ __forceinline__ bool wave_all(bool p) { return __ballot(!p) == 0; }
__device__ __forceinline__ bool eq_digest(uint4 a, uint4 b, const uint32_t* z) {
  return ((a.x ^ z[0]) | (a.y ^ z[1]) | (a.z ^ z[2]) | (a.w ^ z[3]) | (b.x ^ z[4]) | (b.y ^ z[5]) | (b.z ^ z[6]) |
          (b.w ^ z[7])) == 0;
}
// z[q] for a lane-dependent q < 4 as selects (no dynamic indexing of a kernel argument)
__device__ __forceinline__ uint32_t sel4(const uint32_t* z, uint32_t q) {
  return q == 0 ? z[0] : q == 1 ? z[1] : q == 2 ? z[2] : z[3];
}

// FIRST/LAST: a column range of a longer row (hash_rows_range) starts from the capacity
// cells 16..23 saved in `state` and ends by saving them there (overwrite-mode sponge: the
// rate cells are replaced by the next block, so the capacity is the whole carried state)
template <bool FIRST, bool LAST>
__global__ __launch_bounds__(kThreads) void p2_rows_kernel(uint32_t* out, uint32_t* state,
                                                         const uint32_t* __restrict__ m, uint64_t rows,
                                                         uint32_t cols, ZeroSub z) {
  uint64_t row = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (row >= rows) return;
  uint32_t c[24];
#pragma unroll
  for (int i = 0; i < 16; i++) c[i] = 0;
  if (FIRST) {
#pragma unroll
    for (int i = 16; i < 24; i++) c[i] = 0;
  } else {
    const uint4* st = reinterpret_cast<const uint4*>(state + row * 8);
    const uint4 a = st[0], b = st[1];
    c[16] = a.x; c[17] = a.y; c[18] = a.z; c[19] = a.w; c[20] = b.x; c[21] = b.y; c[22] = b.z; c[23] = b.w;
  }
  // blocks of 16 columns (the last one zero-padded; cols == 0 is one all-zero block),
  // software-pipelined: the next block's loads are in flight while the current block is
  // permuted. One permutation call site keeps the kernel small for the instruction cache.
  const uint32_t nblk = cols ? (cols + 15) / 16 : 1;
  uint32_t nxt[16];
  auto load = [&](uint32_t col) {
    if (col + 16 <= cols) {
#pragma unroll
      for (int i = 0; i < 16; i++) nxt[i] = m[uint64_t(col + i) * rows + row];
    } else {
#pragma unroll
      for (int i = 0; i < 16; i++) nxt[i] = col + i < cols ? m[uint64_t(col + i) * rows + row] : 0u;
    }
  };
  load(0);
  if (FIRST && LAST && nblk == 1 && z.on) {  // one block: a zero row hashes to Z_0
    uint32_t any = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) any |= nxt[i];
    if (wave_all(any == 0)) {
      store_digest(out + row * 8, z.out);
      return;
    }
  }
  for (uint32_t b = 0; b < nblk; b++) {
#pragma unroll
    for (int i = 0; i < 16; i++) c[i] = nxt[i];
    if (b + 1 < nblk) load((b + 1) * 16);
    poseidon2_mix(c);
  }
  if (LAST) store_digest(out + row * 8, c);
  else store_digest(state + row * 8, c + 16);
}

__global__ __launch_bounds__(kThreads) void p2_fold_kernel(uint32_t* io, uint64_t in_off, uint64_t out_off,
                                                         uint64_t n, ZeroSub z) {
  uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (i >= n) return;
  const uint4* src = reinterpret_cast<const uint4*>(io + (in_off + 2 * i) * 8);
  uint32_t c[24];
  uint4 a = src[0], b = src[1], d = src[2], e = src[3];
  if (z.on && wave_all(eq_digest(a, b, z.in) && eq_digest(d, e, z.in))) {
    store_digest(io + (out_off + i) * 8, z.out);
    return;
  }
  c[0] = a.x; c[1] = a.y; c[2] = a.z; c[3] = a.w; c[4] = b.x; c[5] = b.y; c[6] = b.z; c[7] = b.w;
  c[8] = d.x; c[9] = d.y; c[10] = d.z; c[11] = d.w; c[12] = e.x; c[13] = e.y; c[14] = e.z; c[15] = e.w;
#pragma unroll
  for (int k = 16; k < 24; k++) c[k] = 0;
  poseidon2_mix(c);
  store_digest(io + (out_off + i) * 8, c);
}

// Wide layers, two nodes per lane: lane i hashes node i, then node i + m (m = ceil(n/2)), whose
// two child digests are loaded before the first permutation, so those loads are in flight
// while it runs (one node per lane waits for its loads with nothing to overlap them).
__global__ __launch_bounds__(kThreads) void p2_fold2_kernel(uint32_t* io, uint64_t in_off, uint64_t out_off,
                                                          uint64_t n, ZeroSub z) {
  const uint64_t m = (n + 1) / 2;
  const uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (i >= m) return;
  const uint64_t j = i + m;
  const bool two = j < n;
  const uint4* s1 = reinterpret_cast<const uint4*>(io + (in_off + 2 * i) * 8);
  uint4 a = s1[0], b = s1[1], d = s1[2], e = s1[3];
  uint4 a2 = make_uint4(0, 0, 0, 0), b2 = a2, d2 = a2, e2 = a2;
  if (two) {
    const uint4* s2 = reinterpret_cast<const uint4*>(io + (in_off + 2 * j) * 8);
    a2 = s2[0], b2 = s2[1], d2 = s2[2], e2 = s2[3];
  }
  uint32_t c[24];
  if (z.on && wave_all(eq_digest(a, b, z.in) && eq_digest(d, e, z.in))) {
    store_digest(io + (out_off + i) * 8, z.out);
  } else {
    c[0] = a.x; c[1] = a.y; c[2] = a.z; c[3] = a.w; c[4] = b.x; c[5] = b.y; c[6] = b.z; c[7] = b.w;
    c[8] = d.x; c[9] = d.y; c[10] = d.z; c[11] = d.w; c[12] = e.x; c[13] = e.y; c[14] = e.z; c[15] = e.w;
#pragma unroll
    for (int k = 16; k < 24; k++) c[k] = 0;
    poseidon2_mix(c);
    store_digest(io + (out_off + i) * 8, c);
  }
  if (!two) return;
  if (z.on && wave_all(eq_digest(a2, b2, z.in) && eq_digest(d2, e2, z.in))) {
    store_digest(io + (out_off + j) * 8, z.out);
    return;
  }
  c[0] = a2.x; c[1] = a2.y; c[2] = a2.z; c[3] = a2.w; c[4] = b2.x; c[5] = b2.y; c[6] = b2.z; c[7] = b2.w;
  c[8] = d2.x; c[9] = d2.y; c[10] = d2.z; c[11] = d2.w; c[12] = e2.x; c[13] = e2.y; c[14] = e2.z; c[15] = e2.w;
#pragma unroll
  for (int k = 16; k < 24; k++) c[k] = 0;
  poseidon2_mix(c);
  store_digest(io + (out_off + j) * 8, c);
}

// Small layers: four lanes per node (poseidon2_mix_quad), so a layer of n nodes keeps 4n
// lanes busy. Lane q loads cells 4j + q (j < 4) of the two child digests and stores
// digest words q and 4 + q.
// Lane q's words of Z_k are z[q] and z[4 + q] (left child words 0, 1; right 2, 3).
__device__ __forceinline__ bool quad_zero(const uint32_t* c, const uint32_t* zin, uint32_t q) {
  const uint32_t z0 = sel4(zin, q), z1 = sel4(zin + 4, q);
  return ((c[0] ^ z0) | (c[1] ^ z1) | (c[2] ^ z0) | (c[3] ^ z1)) == 0;
}

__global__ __launch_bounds__(kThreads) void p2_fold_quad_kernel(uint32_t* io, uint64_t in_off, uint64_t out_off,
                                                              uint64_t n, ZeroSub z) {
  const uint64_t t = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  const uint64_t i = t >> 2;
  if (i >= n) return;  // whole quads: n * 4 lanes
  const uint32_t q = threadIdx.x & 3;
  const uint32_t* src = io + (in_off + 2 * i) * 8;
  uint32_t c[6];
#pragma unroll
  for (int j = 0; j < 4; j++) c[j] = src[4 * j + q];
  uint32_t* dst = io + (out_off + i) * 8;
  if (z.on && wave_all(quad_zero(c, z.in, q))) {
    dst[q] = sel4(z.out, q);
    dst[4 + q] = sel4(z.out + 4, q);
    return;
  }
  c[4] = c[5] = 0;
  poseidon2_mix_quad(c);
  dst[q] = c[0];
  dst[4 + q] = c[1];
}

// ---- Poseidon254 (BN254 Fr, poseidon_254/mod.rs) ---------------------------------
// One lane per row as above; the 3-cell state is 27 VGPRs of 29-bit limbs. Row values are
// decoded from Montgomery to canonical (Elem::as_u32) and packed 8 per cell.
__device__ __forceinline__ void p254_load8(uint32_t* v, const uint32_t* __restrict__ m, uint64_t rows,
                                           uint64_t row, uint32_t col, uint32_t cols) {
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = col + i < cols ? mont_reduce(m[uint64_t(col + i) * rows + row]) : 0u;
}

__global__ __launch_bounds__(kThreads) void p254_rows_kernel(uint32_t* out, const uint32_t* __restrict__ m,
                                                           uint64_t rows, uint32_t cols) {
  uint64_t row = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (row >= rows) return;
  bn::Fr c[3] = {p254_zero(), p254_zero(), p254_zero()};
  for (uint32_t col = 0; col < cols; col += 16) {
    uint32_t v[8];
    p254_load8(v, m, rows, row, col, cols);
    c[1] = p254_pack8(v);
    if (col + 8 < cols) {
      p254_load8(v, m, rows, row, col + 8, cols);
      c[2] = p254_pack8(v);
    } else {
      c[2] = p254_zero();
    }
    p254_mix(c);
  }
  uint32_t d[8];
  p254_to_digest(c[0], d);
  store_digest(out + row * 8, d);
}

__device__ __forceinline__ void p254_node(const uint32_t* src, uint32_t* d) {
  uint32_t a[8], b[8];
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  uint4 x0 = s4[0], x1 = s4[1], x2 = s4[2], x3 = s4[3];
  a[0] = x0.x; a[1] = x0.y; a[2] = x0.z; a[3] = x0.w; a[4] = x1.x; a[5] = x1.y; a[6] = x1.z; a[7] = x1.w;
  b[0] = x2.x; b[1] = x2.y; b[2] = x2.z; b[3] = x2.w; b[4] = x3.x; b[5] = x3.y; b[6] = x3.z; b[7] = x3.w;
  p254_hash_pair(a, b, d);
}

__global__ __launch_bounds__(kThreads) void p254_fold_kernel(uint32_t* io, uint64_t in_off, uint64_t out_off,
                                                           uint64_t n) {
  uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (i >= n) return;
  uint32_t d[8];
  p254_node(io + (in_off + 2 * i) * 8, d);
  store_digest(io + (out_off + i) * 8, d);
}

// ---- SHA-256 ------------------------------------------------------------------
__constant__ static const uint32_t kK256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_rotateright32(x, n); }
// three-way XOR as one v_bitop3_b32 (gfx950; truth table 0x96 is symmetric in its inputs):
// LLVM otherwise emits two v_xor_b32 after the three v_alignbit of every Σ/σ function
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// Ch and Maj as one v_bitop3_b32 each (truth-table index = src0*4 + src1*2 + src2)
__device__ __forceinline__ uint32_t sha_ch(uint32_t e, uint32_t f, uint32_t g) {
  return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);  // e ? f : g
}
__device__ __forceinline__ uint32_t sha_maj(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);  // majority
}

// FIPS 180-4 compression; w[] holds the 16 big-endian message words.
__device__ __forceinline__ void sha_compress(uint32_t* s, uint32_t* w) {
  uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
      uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
    uint32_t ch = sha_ch(e, f, g);
    uint32_t t1 = h + S1 + ch + kK256[i] + wi;
    uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
    uint32_t mj = sha_maj(a, b, c);
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
  }
  s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
}

__device__ __forceinline__ void sha_init(uint32_t* s) {
  s[0] = 0x6a09e667; s[1] = 0xbb67ae85; s[2] = 0x3c6ef372; s[3] = 0xa54ff53a;
  s[4] = 0x510e527f; s[5] = 0x9b05688c; s[6] = 0x1f83d9ab; s[7] = 0x5be0cd19;
}

// Digest words are the big-endian digest bytes in memory order: bswap each state word.
template <bool FIRST, bool LAST>
__global__ __launch_bounds__(kThreads) void sha_rows_kernel(uint32_t* out, uint32_t* state,
                                                          const uint32_t* __restrict__ m, uint64_t rows,
                                                          uint32_t cols, ZeroSub z) {
  uint64_t row = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (row >= rows) return;
  uint32_t s[8], w[16], nxt[16];
  if (FIRST) {
    sha_init(s);
  } else {
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = state[row * 8 + i];
  }
  // the next block's loads are in flight during the current compression
  auto load = [&](uint32_t col) {
#pragma unroll
    for (int i = 0; i < 16; i++) nxt[i] = (col + i < cols) ? m[uint64_t(col + i) * rows + row] : 0u;
  };
  if (cols) load(0);
  if (FIRST && LAST && cols <= 16 && z.on) {  // one block: a zero row hashes to Z_0
    uint32_t any = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) any |= cols ? nxt[i] : 0u;
    if (wave_all(any == 0)) {
      store_digest(out + row * 8, z.out);
      return;
    }
  }
  for (uint32_t col = 0; col < cols; col += 16) {
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = __builtin_bswap32(nxt[i]);
    if (col + 16 < cols) load(col + 16);
    sha_compress(s, w);
  }
  if (!LAST) {
    store_digest(state + row * 8, s);
    return;
  }
  uint32_t d[8];
#pragma unroll
  for (int i = 0; i < 8; i++) d[i] = __builtin_bswap32(s[i]);
  store_digest(out + row * 8, d);
}

__global__ __launch_bounds__(kThreads) void sha_fold_kernel(uint32_t* io, uint64_t in_off, uint64_t out_off,
                                                          uint64_t n, ZeroSub z) {
  uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (i >= n) return;
  const uint4* src4 = reinterpret_cast<const uint4*>(io + (in_off + 2 * i) * 8);
  const uint4 a = src4[0], b = src4[1], c = src4[2], e = src4[3];
  if (z.on && wave_all(eq_digest(a, b, z.in) && eq_digest(c, e, z.in))) {
    store_digest(io + (out_off + i) * 8, z.out);
    return;
  }
  const uint32_t src[16] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, e.x, e.y, e.z, e.w};
  uint32_t s[8], w[16];
  sha_init(s);
#pragma unroll
  for (int k = 0; k < 16; k++) w[k] = __builtin_bswap32(src[k]);
  sha_compress(s, w);
  uint32_t d[8];
#pragma unroll
  for (int k = 0; k < 8; k++) d[k] = __builtin_bswap32(s[k]);
  store_digest(io + (out_off + i) * 8, d);
}

// Poseidon2 tree top in one workgroup of 1024 lanes: layers above quad_max nodes one lane
// per node, smaller layers one quad per node (poseidon2_mix_quad: a quarter of the
// permutation's dependent instructions per lane, so a layer's latency is about a quarter)
constexpr uint32_t kTopThreads = 1024;
// zt (or null): the zero-subtree chain, zt + 8k = Z_k, with Z_k0 the top layer's children
__global__ __launch_bounds__(kTopThreads) void p2_fold_top_kernel(uint32_t* io, uint32_t top_layer_size,
                                                                 uint32_t quad_max, const uint32_t* zt,
                                                                 uint32_t k0) {
  for (uint32_t out = top_layer_size, lvl = k0; out >= 1; out >>= 1, lvl++) {
    const uint32_t* zin = zt ? zt + 8 * lvl : nullptr;
    if (out > quad_max) {
      for (uint32_t i = threadIdx.x; i < out; i += kTopThreads) {
        const uint32_t* src = io + (uint64_t(2 * out) + 2 * i) * 8;
        uint32_t c[24];
#pragma unroll
        for (int k = 0; k < 16; k++) c[k] = src[k];
        if (zin) {
          uint32_t x = 0;
#pragma unroll
          for (int w = 0; w < 16; w++) x |= c[w] ^ zin[w & 7];
          if (wave_all(x == 0)) {
            store_digest(io + (uint64_t(out) + i) * 8, zin + 8);
            continue;
          }
        }
#pragma unroll
        for (int k = 16; k < 24; k++) c[k] = 0;
        poseidon2_mix(c);
        store_digest(io + (uint64_t(out) + i) * 8, c);
      }
    } else {
      // whole quads per iteration (kTopThreads is a multiple of 4)
      for (uint32_t t = threadIdx.x; t < 4 * out; t += kTopThreads) {
        const uint32_t i = t >> 2, q = t & 3;
        const uint32_t* src = io + (uint64_t(2 * out) + 2 * i) * 8;
        uint32_t c[6];
#pragma unroll
        for (int j = 0; j < 4; j++) c[j] = src[4 * j + q];
        uint32_t* dst = io + (uint64_t(out) + i) * 8;
        if (zin && wave_all(quad_zero(c, zin, q))) {
          dst[q] = sel4(zin + 8, q);
          dst[4 + q] = sel4(zin + 12, q);
          continue;
        }
        c[4] = c[5] = 0;
        poseidon2_mix_quad(c);
        dst[q] = c[0];
        dst[4 + q] = c[1];
      }
    }
    __threadfence_block();
    __syncthreads();
  }
}

// SHA-256 / Poseidon254 tree top inside one workgroup: layers with <= 512 nodes, all
// hashed by 256 lanes with a workgroup barrier between layers (same-CU visibility).
template <int SUITE>
__global__ __launch_bounds__(kThreads) void fold_top_kernel(uint32_t* io, uint32_t top_layer_size, const uint32_t* zt,
                                                          uint32_t k0) {
  for (uint32_t out = top_layer_size, lvl = k0; out >= 1; out >>= 1, lvl++) {
    const uint32_t* zin = zt ? zt + 8 * lvl : nullptr;
    for (uint32_t i = threadIdx.x; i < out; i += kThreads) {
      const uint32_t* src = io + (uint64_t(2 * out) + 2 * i) * 8;
      uint32_t d[8];
      if (zin) {
        uint32_t x = 0;
#pragma unroll
        for (int w = 0; w < 16; w++) x |= src[w] ^ zin[w & 7];
        if (wave_all(x == 0)) {
          store_digest(io + (uint64_t(out) + i) * 8, zin + 8);
          continue;
        }
      }
      if (SUITE == 2) {
        p254_node(src, d);
      } else {
        uint32_t s[8], w[16];
        sha_init(s);
#pragma unroll
        for (int k = 0; k < 16; k++) w[k] = __builtin_bswap32(src[k]);
        sha_compress(s, w);
#pragma unroll
        for (int k = 0; k < 8; k++) d[k] = __builtin_bswap32(s[k]);
      }
      store_digest(io + (uint64_t(out) + i) * 8, d);
    }
    __threadfence_block();
    __syncthreads();
  }
}

}  // namespace

// Z_0 .. Z_levels for rows of `cols` columns ((levels + 1) * 8 words, cached): Z_0 is
// hash_rows of an all-zero row (the suite's unpadded row hash, transcript.h hash_elems),
// Z_{k+1} the pair hash of (Z_k, Z_k). Suites 0 (Poseidon2) and 1 (SHA-256).
static const std::vector<uint32_t>& zero_chain(int suite, size_t cols, size_t levels) {
  static std::mutex mu;
  static std::map<std::tuple<int, size_t, size_t>, std::vector<uint32_t>> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto& v = cache[{suite, cols, levels}];
  if (v.empty()) {
    const std::vector<uint32_t> zeros(cols, 0u);
    Digest d = hash_elems(suite, zeros.data(), cols);
    v.assign(d.w, d.w + 8);
    for (size_t k = 0; k < levels; k++) {
      Digest a;
      memcpy(a.w, &v[8 * k], 32);
      if (suite == 0) {
        uint32_t c[24] = {0};
        for (int i = 0; i < 8; i++) c[i] = c[8 + i] = a.w[i];
        poseidon2_mix(c);
        memcpy(d.w, c, 32);
      } else {
        d = sha::hash_pair(a, a);
      }
      v.insert(v.end(), d.w, d.w + 8);
    }
  }
  return v;
}

static ZeroSub zero_off() {
  ZeroSub z{};
  return z;
}

// R0_P2_ZERO=0 turns the zero-subtree path off (same-box A/B)
static bool zero_enabled() {
  static const bool v = [] {
    const char* e = getenv("R0_P2_ZERO");
    return !e || strtoul(e, nullptr, 10) != 0;
  }();
  return v;
}

// the leaf constant for one-block rows (the row kernels check zero rows only then)
static ZeroSub zero_rows(int suite, size_t cols) {
  ZeroSub z{};
  if (suite > 1 || cols > 16 || !zero_enabled()) return z;
  const auto& ch = zero_chain(suite, cols, 0);
  for (int i = 0; i < 8; i++) z.out[i] = ch[i];
  z.on = 1;
  return z;
}

// Trees built call by call (the per-op ABI: r0hip_hash_rows into nodes[rows .. 2 rows), then
// r0hip_hash_fold per layer, as MerkleTreeProver::new drives the HAL, prove/merkle.rs:54-81):
// hash_rows notes the heap its leaf range may belong to (base = out - 8 rows words), and
// hash_fold on that base takes the layer's height from the note, so those layers get the
// zero-subtree path too. A stale or unrelated note only changes the hit rate: a node whose
// children are both Z_k is Z_{k+1} in any tree.
namespace {
struct HeapNote {
  int suite;
  size_t rows, cols;
};
std::mutex g_note_mu;
std::map<uintptr_t, HeapNote> g_notes;
}  // namespace
static void note_heap(int suite, const uint32_t* leaves, size_t rows, size_t cols) {
  if (suite > 1 || rows < 2 || (rows & (rows - 1)) != 0) return;
  const uintptr_t base = uintptr_t(leaves) - uintptr_t(rows) * 32;
  std::lock_guard<std::mutex> lk(g_note_mu);
  if (g_notes.size() >= 256) g_notes.clear();
  g_notes[base] = HeapNote{suite, rows, cols};
}
static ZeroSub noted_layer(int suite, const uint32_t* io, size_t input_size) {
  ZeroSub z{};
  if (suite > 1 || input_size < 2 || !zero_enabled()) return z;
  HeapNote n;
  {
    std::lock_guard<std::mutex> lk(g_note_mu);
    auto it = g_notes.find(uintptr_t(io));
    if (it == g_notes.end()) return z;
    n = it->second;
  }
  if (n.suite != suite || input_size > n.rows || n.rows % input_size != 0) return z;
  size_t k = 0, levels = 0;
  while ((input_size << k) < n.rows) k++;
  while ((size_t(1) << levels) < n.rows) levels++;
  if ((input_size << k) != n.rows) return z;
  const auto& ch = zero_chain(suite, n.cols, levels);
  for (int i = 0; i < 8; i++) z.in[i] = ch[8 * k + i], z.out[i] = ch[8 * (k + 1) + i];
  z.on = 1;
  return z;
}

void hash_rows(hipStream_t s, int suite, uint32_t* out, const uint32_t* matrix, size_t rows, size_t cols) {
  if (rows == 0) return;
  note_heap(suite, out, rows, cols);
  R0_REQUIRE(cols < (1ull << 31), "hash_rows: too many columns");
  R0_REQUIRE(suite >= 0 && suite <= 2, "hash_rows: unknown hash suite");
  // Poseidon2 permutation = 1356 modmul (8x24 S-boxes x4, 21 partial S-boxes x4, 21x24 diagonal)
  const double perms = double(rows) * (cols ? (cols + 15) / 16 : 1);
  static const char* names[3] = {"hash_rows_poseidon2", "hash_rows_sha256", "hash_rows_poseidon254"};
  KScope ks(names[suite], double(rows) * (cols * 4 + 32),
            suite == 0 ? perms * kP2Modmuls : 0);
  const dim3 grid(div_up(rows, kThreads)), block(kThreads);
  if (suite == 0)
    hipLaunchKernelGGL((p2_rows_kernel<true, true>), grid, block, 0, s, out, nullptr, matrix, uint64_t(rows),
                       uint32_t(cols), zero_rows(suite, cols));
  else if (suite == 1)
    hipLaunchKernelGGL((sha_rows_kernel<true, true>), grid, block, 0, s, out, nullptr, matrix, uint64_t(rows),
                       uint32_t(cols), zero_rows(suite, cols));
  else
    hipLaunchKernelGGL(p254_rows_kernel, grid, block, 0, s, out, matrix, uint64_t(rows), uint32_t(cols));
  HIP_OK(hipGetLastError());
}

template <bool FIRST, bool LAST>
static void launch_rows_range(hipStream_t s, int suite, uint32_t* out, uint32_t* state, const uint32_t* chunk,
                              size_t rows, size_t cols) {
  const dim3 grid(div_up(rows, kThreads)), block(kThreads);
  if (suite == 0)
    hipLaunchKernelGGL((p2_rows_kernel<FIRST, LAST>), grid, block, 0, s, out, state, chunk, uint64_t(rows),
                       uint32_t(cols), FIRST && LAST ? zero_rows(suite, cols) : zero_off());
  else
    hipLaunchKernelGGL((sha_rows_kernel<FIRST, LAST>), grid, block, 0, s, out, state, chunk, uint64_t(rows),
                       uint32_t(cols), FIRST && LAST ? zero_rows(suite, cols) : zero_off());
  HIP_OK(hipGetLastError());
}

void hash_rows_range(hipStream_t s, int suite, uint32_t* out, uint32_t* state, const uint32_t* chunk, size_t rows,
                     size_t cols, bool first, bool last) {
  if (rows == 0) return;
  R0_REQUIRE(suite == 0 || suite == 1, "hash_rows_range: Poseidon2 and SHA-256 only");
  R0_REQUIRE(last || (cols > 0 && cols % 16 == 0), "hash_rows_range: a range before the last needs 16k columns");
  R0_REQUIRE(cols > 0 || (first && last), "hash_rows_range: empty range");
  R0_REQUIRE((first && last) || state, "hash_rows_range: state buffer is NULL");
  static const char* names[2] = {"hash_rows_poseidon2", "hash_rows_sha256"};
  const double perms = double(rows) * ((cols + 15) / 16);
  KScope ks(names[suite], double(rows) * (cols * 4 + 32), suite == 0 ? perms * kP2Modmuls : 0);
  if (first && last) launch_rows_range<true, true>(s, suite, out, state, chunk, rows, cols);
  else if (first) launch_rows_range<true, false>(s, suite, out, state, chunk, rows, cols);
  else if (last) launch_rows_range<false, true>(s, suite, out, state, chunk, rows, cols);
  else launch_rows_range<false, false>(s, suite, out, state, chunk, rows, cols);
}

// Poseidon2 layers up to this many nodes hash one quad per node: below it one lane per
// node leaves SIMDs idle (<= 1 wave each), so the quad's 3x shorter latency wins.
// R0_P2_QUAD_MAX overrides it (tools/micro/fold_latency.py measures the crossover).
static size_t env_size(const char* name, size_t dflt) {
  const char* e = getenv(name);
  return e ? size_t(strtoull(e, nullptr, 10)) : dflt;
}
static size_t quad_fold_max() {
  static const size_t v = env_size("R0_P2_QUAD_MAX", 32768);
  return v;
}
// tree tops (one workgroup): quads for layers up to this size (R0_P2_TOP_QUAD_MAX)
static uint32_t quad_top_max() {
  static const uint32_t v = uint32_t(env_size("R0_P2_TOP_QUAD_MAX", 128));
  return v;
}

// wide Poseidon2 layers two nodes per lane (R0_P2_FOLD_TWO=0: one)
static bool fold_two() {
  static const bool v = env_size("R0_P2_FOLD_TWO", 1) != 0;
  return v;
}

// z: the zero-subtree pair of this layer (merkle_layers), or off (a standalone fold)
static void hash_fold_z(hipStream_t s, int suite, uint32_t* io, size_t input_size, size_t output_size,
                        const ZeroSub& z) {
  if (output_size == 0) return;
  R0_REQUIRE(input_size == 2 * output_size, "hash_fold: input_size != 2*output_size");
  R0_REQUIRE(suite >= 0 && suite <= 2, "hash_fold: unknown hash suite");
  const dim3 grid(div_up(output_size, kThreads)), block(kThreads);
  const uint64_t in = input_size, out = output_size;
  if (suite == 0 && output_size <= quad_fold_max())
    hipLaunchKernelGGL(p2_fold_quad_kernel, dim3(div_up(4 * output_size, kThreads)), block, 0, s, io, in, out, out,
                       z);
  else if (suite == 0 && fold_two())
    hipLaunchKernelGGL(p2_fold2_kernel, dim3(div_up((output_size + 1) / 2, kThreads)), block, 0, s, io, in, out, out,
                       z);
  else if (suite == 0)
    hipLaunchKernelGGL(p2_fold_kernel, grid, block, 0, s, io, in, out, out, z);
  else if (suite == 1)
    hipLaunchKernelGGL(sha_fold_kernel, grid, block, 0, s, io, in, out, out, z);
  else
    hipLaunchKernelGGL(p254_fold_kernel, grid, block, 0, s, io, in, out, out);
  HIP_OK(hipGetLastError());
}

void hash_fold(hipStream_t s, int suite, uint32_t* io, size_t input_size, size_t output_size) {
  hash_fold_z(s, suite, io, input_size, output_size, noted_layer(suite, io, input_size));
}

// MerkleTreeProver::new (risc0/zkp/src/prove/merkle.rs:54-81): leaves, then every layer.
void merkle_tree(hipStream_t s, int suite, uint32_t* nodes, const uint32_t* matrix, size_t rows, size_t cols) {
  hash_rows(s, suite, nodes + rows * 8, matrix, rows, cols);
  merkle_layers(s, suite, nodes, rows, cols);
}

// Poseidon2 tree tops start at this many nodes (R0_P2_TOP_NODES, a power of two <= 512): the
// layers above it are separate multi-CU launches (quad kernels, ~11 us each), the ones from it
// to the root one workgroup of quads. The one-workgroup top took 114 us from 512 nodes (the 512-
// and 256-node layers one lane per node, two waves per SIMD), 63 us from 64 (`profiles/r4m_*`).
// Measured and rejected: every layer of <= 32768 nodes plus the root in one dataflow launch
// (the second child to arrive hashes the parent, agent-scope release/acquire around a per-
// parent counter): 419 us per tree against 140 us, the L2 write-back and invalidate of each
// release/acquire costing more than the launches they save (`profiles/r4n_merkle_tree_ab.txt`).
static size_t p2_top_nodes() {
  static const size_t v = env_size("R0_P2_TOP_NODES", 64);
  return v;
}

void merkle_layers(hipStream_t s, int suite, uint32_t* nodes, size_t rows, size_t cols) {
  static const char* names[3] = {"merkle_fold_poseidon2", "merkle_fold_sha256", "merkle_fold_poseidon254"};
  KScope ks(names[suite], double(rows) * 32 * 1.5, suite == 0 ? double(rows - 1) * kP2Modmuls : 0);
  size_t layer = rows / 2;
  const size_t top = suite == 0 ? std::min<size_t>(512, p2_top_nodes()) : 512;
  // zero-subtree chain of this tree (Poseidon2 or SHA-256 with a known column count): the children of
  // the layer of `out` nodes are at level log2(rows / (2 out))
  size_t levels = 0;
  while ((size_t(1) << levels) < rows) levels++;
  const bool zon = suite <= 1 && cols != SIZE_MAX && rows >= 2 && zero_enabled();
  const std::vector<uint32_t>* chain = zon ? &zero_chain(suite, cols, levels) : nullptr;
  size_t k = 0;
  for (; layer > top; layer /= 2, k++) {
    ZeroSub z = zero_off();
    if (chain) {
      for (int i = 0; i < 8; i++) z.in[i] = (*chain)[8 * k + i], z.out[i] = (*chain)[8 * (k + 1) + i];
      z.on = 1;
    }
    hash_fold_z(s, suite, nodes, 2 * layer, layer, z);
  }
  if (layer >= 1) {
    const dim3 grid(1), block(kThreads);
    const uint32_t* zt = nullptr;
    if (chain)
      zt = dev_table("zero" + std::to_string(suite) + "_" + std::to_string(cols) + "_" + std::to_string(levels),
                     [=] { return *chain; });
    if (suite == 0) hipLaunchKernelGGL(p2_fold_top_kernel, grid, dim3(kTopThreads), 0, s, nodes, uint32_t(layer),
                                    quad_top_max(), zt, uint32_t(k));
    else if (suite == 1)
      hipLaunchKernelGGL(fold_top_kernel<1>, grid, block, 0, s, nodes, uint32_t(layer), zt, uint32_t(k));
    else hipLaunchKernelGGL(fold_top_kernel<2>, grid, block, 0, s, nodes, uint32_t(layer), nullptr, 0u);
    HIP_OK(hipGetLastError());
  }
}

}  // namespace r0
