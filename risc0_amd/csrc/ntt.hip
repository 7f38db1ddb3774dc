// Batched BabyBear NTTs for CDNA4 (gfx950): forward evaluate with expansion,
// inverse interpolate with fused 1/n and zk_shift, bit-reversal and zk_shift.
//
// Semantics are the reference CPU HAL's (risc0/zkp/src/core/ntt.rs:232-342,
// risc0/zkp/src/hal/cpu.rs:305-408): evaluate takes bit-reversed coefficients to
// natural-order evaluations, interpolate takes natural evaluations to
// bit-reversed coefficients times 1/n. Results are exact, so any factorisation
// gives bit-identical words.
//
// Layout: `count` polynomials of 2^L words each, back to back (column-major
// trace). One launch per *pass* covers every polynomial; a pass runs the
// butterfly stages of index bits [a, a+b) for groups of 2^b elements staged in
// LDS. With the DIT identity
//   X[t'*2^a + low] = sum_t w_{2^b}^{t' * rev_b(t)} * (w_{2^(a+b)}^{low * rev_b(t)} * x[t])
// each pass is a local size-2^b DIT after one twiddle multiply per element (and
// the transpose of that for the inverse). Pass 0 (a = 0) reads contiguous rows;
// upper passes read 2^c adjacent columns per workgroup so every global access is
// a >=64-byte contiguous run. A po2=20 evaluate (L = 22) is two passes (13 + 9 bits): one read
// of the coefficients and one read+write of the 4x domain through HBM.
#include "runtime.h"

#include <map>
#include <mutex>

namespace r0 {

namespace {

constexpr int kThreads = 256;

struct PassArgs {
  uint32_t* out;
  const uint32_t* in;       // expand source (first forward pass) or == out
  const uint32_t* local_tw; // [2^(s-1) + k] = w_{2^s}^k, s = 1..b (fwd or rev roots)
  const uint32_t* sc_lo;    // w_{2^(a+b)}^e = sc_hi[e >> sc_split] * sc_lo[e & mask]
  const uint32_t* sc_hi;
  const uint32_t* post_t;   // last inverse pass: per-t factor (norm * 3^{rev_b(t)*2^(L-b)})
  const uint32_t* post_hi;  // last inverse pass: per-row factor 3^{rev_{L-b}(row)} (or null)
  uint64_t groups;          // total groups of 2^b elements over the whole batch
  uint32_t L, a, b, c, eb;  // eb: expand bits (first forward pass only)
  uint32_t sc_split;
};

// LDS placement. Row passes (a == 0) keep each row contiguous with one pad word
// per 8 so strided butterfly reads spread over the banks; column passes store
// [t][j] with the 2^c (= 32) adjacent columns of a row in consecutive words.
template <bool COLS>
__device__ __forceinline__ uint32_t lidx(uint32_t j, uint32_t t, uint32_t b, uint32_t c) {
  if (COLS) return (t << c) + j;
  return j * ((1u << b) + (1u << b >> 3)) + t + (t >> 3);
}

// One stage group of 1..3 radix-2 stages [s0, s0+NST) done in registers: each lane
// owns blocks of 2^NST elements t_base + m*h (h = 2^(s0-1)), so the group costs one
// LDS read and one write per element instead of NST.
template <bool INV, bool COLS, int NST>
__device__ __forceinline__ void stage_group(uint32_t* lds, const uint32_t* __restrict__ tw, uint32_t s0,
                                            uint32_t b, uint32_t c) {
  constexpr uint32_t M = 1u << NST;
  const uint32_t h = 1u << (s0 - 1);
  const uint32_t nrb = 1u << (b - NST);  // blocks per column/row
  const uint32_t nblk = nrb << c;
  for (uint32_t blk = threadIdx.x; blk < nblk; blk += kThreads) {
    uint32_t j, r;
    if (COLS) {
      j = blk & ((1u << c) - 1);
      r = blk >> c;
    } else {
      j = blk / nrb;
      r = blk & (nrb - 1);
    }
    const uint32_t k = r & (h - 1);
    const uint32_t tb = ((r >> (s0 - 1)) << (s0 - 1 + NST)) | k;
    uint32_t v[M];
#pragma unroll
    for (uint32_t m = 0; m < M; m++) v[m] = lds[lidx<COLS>(j, tb + m * h, b, c)];
    if (!INV) {
#pragma unroll
      for (uint32_t st = 0; st < NST; st++) {
        const uint32_t half = 1u << st, hs = h << st;
#pragma unroll
        for (uint32_t m = 0; m < M; m++) {
          if (m & half) continue;
          uint32_t w = tw[hs + k + (m & (half - 1)) * h];
          uint32_t x = v[m], y = fp_mul(v[m + half], w);
          v[m] = fp_add(x, y);
          v[m + half] = fp_sub(x, y);
        }
      }
    } else {
#pragma unroll
      for (int st = NST - 1; st >= 0; st--) {
        const uint32_t half = 1u << st, hs = h << st;
#pragma unroll
        for (uint32_t m = 0; m < M; m++) {
          if (m & half) continue;
          uint32_t w = tw[hs + k + (m & (half - 1)) * h];
          uint32_t x = v[m], y = v[m + half];
          v[m] = fp_add(x, y);
          v[m + half] = fp_mul(fp_sub(x, y), w);
        }
      }
    }
#pragma unroll
    for (uint32_t m = 0; m < M; m++) lds[lidx<COLS>(j, tb + m * h, b, c)] = v[m];
  }
  __syncthreads();
}

template <bool INV, bool COLS>
__device__ __forceinline__ void stages(uint32_t* lds, const uint32_t* __restrict__ tw, uint32_t first,
                                       uint32_t last, uint32_t b, uint32_t c) {
  // stages [first, last] inclusive, ascending for DIT, descending for DIF
  if (!INV) {
    uint32_t s = first;
    while (s <= last) {
      uint32_t n = last - s + 1;
      if (n >= 3) {
        stage_group<INV, COLS, 3>(lds, tw, s, b, c);
        s += 3;
      } else if (n == 2) {
        stage_group<INV, COLS, 2>(lds, tw, s, b, c);
        s += 2;
      } else {
        stage_group<INV, COLS, 1>(lds, tw, s, b, c);
        s += 1;
      }
    }
  } else {
    int s = int(last);
    while (s >= int(first)) {
      int n = s - int(first) + 1;
      if (n >= 3) {
        stage_group<INV, COLS, 3>(lds, tw, uint32_t(s - 2), b, c);
        s -= 3;
      } else if (n == 2) {
        stage_group<INV, COLS, 2>(lds, tw, uint32_t(s - 1), b, c);
        s -= 2;
      } else {
        stage_group<INV, COLS, 1>(lds, tw, uint32_t(s), b, c);
        s -= 1;
      }
    }
  }
}

template <bool INV, bool EXPAND, bool LAST, bool COLS>
__global__ __launch_bounds__(kThreads) void ntt_pass_kernel(PassArgs p) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t tid = threadIdx.x;
  const uint32_t nb = 1u << p.b;
  const uint32_t C = 1u << p.c;
  const uint32_t total = nb << p.c;
  const uint32_t bmask = nb - 1;
  const uint64_t wg = blockIdx.x;
  uint64_t g_hi = 0;
  uint32_t low0 = 0;
  if (COLS) {
    uint32_t lowblocks = 1u << (p.a - p.c);
    low0 = uint32_t(wg % lowblocks) << p.c;
    g_hi = wg / lowblocks;
  }
  // ---- load (forward column passes pre-scale by w_{2^(a+b)}^{low * rev_b(t)}) ----
  for (uint32_t idx = tid; idx < total; idx += kThreads) {
    uint32_t t, j;
    uint64_t e;
    bool ok = true;
    if (!COLS) {
      t = idx & bmask;
      j = idx >> p.b;
      uint64_t g = (wg << p.c) + j;
      ok = g < p.groups;
      e = (g << p.b) + t;
    } else {
      j = idx & (C - 1);
      t = idx >> p.c;
      e = (g_hi << (p.a + p.b)) + (uint64_t(t) << p.a) + low0 + j;
    }
    uint32_t v = 0;
    if (ok) {
      if (EXPAND) v = p.in[e >> p.eb];
      else v = p.out[e];
      if (!INV && COLS) {
        uint32_t ex = (low0 + j) * bitrev_n(t, p.b);
        v = fp_mul(v, fp_mul(p.sc_hi[ex >> p.sc_split], p.sc_lo[ex & ((1u << p.sc_split) - 1)]));
      }
    }
    lds[lidx<COLS>(j, t, p.b, p.c)] = v;
  }
  __syncthreads();
  if (!INV) stages<false, COLS>(lds, p.local_tw, 1 + (EXPAND ? p.eb : 0), p.b, p.b, p.c);
  else stages<true, COLS>(lds, p.local_tw, 1, p.b, p.b, p.c);
  // ---- store (inverse column passes post-scale; last inverse pass normalises) ----
  for (uint32_t idx = tid; idx < total; idx += kThreads) {
    uint32_t t, j;
    uint64_t e;
    if (!COLS) {
      t = idx & bmask;
      j = idx >> p.b;
      uint64_t g = (wg << p.c) + j;
      if (g >= p.groups) continue;
      e = (g << p.b) + t;
    } else {
      j = idx & (C - 1);
      t = idx >> p.c;
      e = (g_hi << (p.a + p.b)) + (uint64_t(t) << p.a) + low0 + j;
    }
    uint32_t v = lds[lidx<COLS>(j, t, p.b, p.c)];
    if (INV && COLS) {
      uint32_t ex = (low0 + j) * bitrev_n(t, p.b);
      v = fp_mul(v, fp_mul(p.sc_hi[ex >> p.sc_split], p.sc_lo[ex & ((1u << p.sc_split) - 1)]));
    }
    if (LAST) {
      v = fp_mul(v, p.post_t[t]);
      if (p.post_hi) {
        uint64_t g = (wg << p.c) + j;
        uint32_t row = uint32_t(g & ((uint64_t(1) << (p.L - p.b)) - 1));
        v = fp_mul(v, p.post_hi[row]);
      }
    }
    p.out[e] = v;
  }
}

// ---- bit reversal -----------------------------------------------------------
// Rows of 2^L: i = (hi:k | mid:m | lo:k) -> rev(i) = (rev_k(lo) | rev_m(mid) | rev_k(hi)).
// A workgroup swaps the 2^k x 2^k tiles of mid and rev_m(mid) through LDS, so
// both the reads (lo contiguous) and the writes (rev_k(hi) contiguous) coalesce.
__global__ __launch_bounds__(kThreads) void bit_reverse_tiles(uint32_t* io, uint32_t L, uint32_t k) {
  __shared__ uint32_t ta[32 * 33];
  __shared__ uint32_t tb[32 * 33];
  const uint32_t m = L - 2 * k;
  const uint32_t nmid = 1u << m;
  const uint32_t mid = blockIdx.x % nmid;
  const uint64_t row = blockIdx.x / nmid;
  const uint32_t rmid = bitrev_n(mid, m);
  if (mid > rmid) return;
  const uint32_t K = 1u << k;
  uint32_t* base = io + (row << L);
  for (uint32_t i = threadIdx.x; i < K * K; i += kThreads) {
    uint32_t hi = i >> k, lo = i & (K - 1);
    ta[hi * 33 + lo] = base[(uint64_t(hi) << (m + k)) + (uint64_t(mid) << k) + lo];
    tb[hi * 33 + lo] = base[(uint64_t(hi) << (m + k)) + (uint64_t(rmid) << k) + lo];
  }
  __syncthreads();
  // dest (hi', rmid or mid, lo') takes source (hi = rev(lo'), ., lo = rev(hi'))
  for (uint32_t i = threadIdx.x; i < K * K; i += kThreads) {
    uint32_t hi2 = i >> k, lo2 = i & (K - 1);
    uint32_t shi = bitrev_n(lo2, k), slo = bitrev_n(hi2, k);
    base[(uint64_t(hi2) << (m + k)) + (uint64_t(rmid) << k) + lo2] = ta[shi * 33 + slo];
    if (rmid != mid) base[(uint64_t(hi2) << (m + k)) + (uint64_t(mid) << k) + lo2] = tb[shi * 33 + slo];
  }
}

// Small rows (L < 2): nothing; rows with L <= 10 handled by the tile kernel with k = L/2.

// ---- zk_shift: io[i] *= 3^{rev_L(i mod 2^L)} -------------------------------------
// cpu.rs:395-408. 3^{rev(i)} = A[rev_h(lo)] * B[rev_{L-h}(hi)], i = hi*2^h + lo.
__global__ __launch_bounds__(kThreads) void zk_shift_kernel(uint32_t* io, uint64_t n, uint32_t L, uint32_t h,
                                                          const uint32_t* A, const uint32_t* B) {
  uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (i >= n) return;
  uint32_t pos = uint32_t(i & ((uint64_t(1) << L) - 1));
  uint32_t lo = pos & ((1u << h) - 1), hi = pos >> h;
  io[i] = fp_mul(io[i], fp_mul(A[bitrev_n(lo, h)], B[bitrev_n(hi, L - h)]));
}

// ---- host-side table generation ---------------------------------------------
uint32_t root(bool inv, uint32_t s) { return fp_encode(inv ? kRouRev[s] : kRouFwd[s]); }

const uint32_t* local_tw_table(bool inv, uint32_t b) {
  return dev_table(std::string("ltw") + (inv ? "r" : "f") + std::to_string(b), [=] {
    std::vector<uint32_t> t(size_t(1) << b, 0);
    for (uint32_t s = 1; s <= b; s++) {
      uint32_t h = 1u << (s - 1), w = root(inv, s), cur = kOne;
      for (uint32_t k = 0; k < h; k++) {
        t[h + k] = cur;
        cur = fp_mul(cur, w);
      }
    }
    return t;
  });
}

// powers of w_{2^m}: split into lo (2^split) and hi (2^(m-split)) tables
void scale_tables(bool inv, uint32_t m, const uint32_t** lo, const uint32_t** hi, uint32_t* split) {
  uint32_t sp = (m + 1) / 2;
  *split = sp;
  std::string key = std::string("sc") + (inv ? "r" : "f") + std::to_string(m);
  *lo = dev_table(key + "lo", [=] {
    std::vector<uint32_t> t(size_t(1) << sp);
    uint32_t w = root(inv, m), cur = kOne;
    for (auto& x : t) {
      x = cur;
      cur = fp_mul(cur, w);
    }
    return t;
  });
  *hi = dev_table(key + "hi", [=] {
    std::vector<uint32_t> t(size_t(1) << (m - sp));
    uint32_t w = fp_pow(root(inv, m), uint64_t(1) << sp), cur = kOne;
    for (auto& x : t) {
      x = cur;
      cur = fp_mul(cur, w);
    }
    return t;
  });
}

// Pass plan over index bits: the row pass (a = 0) takes up to 13 bits (32 KiB rows
// in LDS); the remaining bits go to column passes of at most 9 bits over 32
// adjacent columns (128-byte global segments, 64 KiB of LDS per workgroup).
std::vector<std::pair<uint32_t, uint32_t>> plan(uint32_t L) {
  std::vector<std::pair<uint32_t, uint32_t>> v;
  uint32_t first = L < 13 ? L : 13;
  v.push_back({0, first});
  uint32_t rest = L - first;
  if (rest) {
    uint32_t np = (rest + 8) / 9;
    uint32_t a = first;
    for (uint32_t i = 0; i < np; i++) {
      uint32_t b = rest / np + (i < rest % np ? 1 : 0);
      v.push_back({a, b});
      a += b;
    }
  }
  return v;
}

template <bool INV, bool EXPAND, bool LAST, bool COLS>
void launch_pass(hipStream_t s, PassArgs p) {
  size_t lds = COLS ? (size_t(4) << (p.b + p.c)) : size_t(4) * ((size_t(1) << p.b) + (size_t(1) << p.b >> 3)) << p.c;
  uint64_t nwg;
  if (!COLS) nwg = (p.groups + (uint64_t(1) << p.c) - 1) >> p.c;
  else nwg = p.groups >> p.c;  // groups = count * 2^(L-b); each wg takes 2^c adjacent columns
  R0_REQUIRE(nwg < (1ull << 31), "ntt grid too large");
  hipLaunchKernelGGL((ntt_pass_kernel<INV, EXPAND, LAST, COLS>), dim3(unsigned(nwg)), dim3(kThreads), lds, s, p);
  HIP_OK(hipGetLastError());
}

void fill_pass(PassArgs& p, bool inv, uint32_t L, uint32_t a, uint32_t b, size_t count) {
  p.L = L;
  p.a = a;
  p.b = b;
  p.groups = uint64_t(count) << (L - b);
  if (a == 0) {
    // rows per workgroup so a workgroup holds >= 2048 elements
    p.c = b >= 11 ? 0 : 11 - b;
  } else {
    p.c = a < 5 ? a : 5;
  }
  p.local_tw = local_tw_table(inv, b);
  p.sc_lo = p.sc_hi = nullptr;
  p.sc_split = 0;
  if (a > 0) scale_tables(inv, a + b, &p.sc_lo, &p.sc_hi, &p.sc_split);
}

}  // namespace

void ntt_evaluate(hipStream_t s, uint32_t* out, const uint32_t* in, size_t count, uint32_t L,
                  uint32_t eb) {
  if (count == 0) return;
  KScope ks("ntt_evaluate", double(count) * 4 * ((size_t(1) << L) + (size_t(1) << (L - eb))),
            double(count) * double(size_t(1) << L) / 2 * (L - eb));  // one modmul per butterfly
  R0_REQUIRE(in != out || eb == 0, "expand_into_evaluate needs distinct buffers");
  if (L == 0) {
    HIP_OK(hipMemcpyAsync(out, in, count * 4, hipMemcpyDeviceToDevice, s));
    return;
  }
  auto pl = plan(L);
  R0_REQUIRE(eb <= pl[0].second, "expand_bits larger than the first NTT pass");
  for (size_t i = 0; i < pl.size(); i++) {
    PassArgs p{};
    p.out = out;
    p.in = in;
    p.eb = eb;
    fill_pass(p, false, L, pl[i].first, pl[i].second, count);
    if (i == 0) launch_pass<false, true, false, false>(s, p);
    else launch_pass<false, false, false, true>(s, p);
  }
}

void ntt_interpolate(hipStream_t s, uint32_t* io, size_t count, uint32_t L, bool zk) {
  if (count == 0 || L == 0) return;  // size-1 transform (and 3^0 shift) is the identity
  KScope ks("ntt_interpolate", double(count) * 8 * (size_t(1) << L), double(count) * double(size_t(1) << L) / 2 * L);
  auto pl = plan(L);
  for (size_t i = pl.size(); i-- > 0;) {
    PassArgs p{};
    p.out = io;
    p.in = io;
    fill_pass(p, true, L, pl[i].first, pl[i].second, count);
    if (i == 0) {
      uint32_t b = pl[0].second;
      // post factor for element t of a row: norm * 3^{rev_b(t) * 2^(L-b)} (zk) ; rows: 3^{rev_{L-b}(row)}
      std::string key = "post" + std::to_string(L) + "_" + std::to_string(b) + (zk ? "z" : "n");
      p.post_t = dev_table(key, [=] {
        std::vector<uint32_t> t(size_t(1) << b);
        uint32_t norm = fp_inv(fp_encode(uint32_t(1u << L)));  // L <= 26 < 31
        uint32_t g = fp_pow(fp_encode(3), uint64_t(1) << (L - b));
        for (uint32_t i2 = 0; i2 < t.size(); i2++)
          t[i2] = zk ? fp_mul(norm, fp_pow(g, bitrev_n(i2, b))) : norm;
        return t;
      });
      p.post_hi = nullptr;
      if (zk && L > b) {
        p.post_hi = dev_table("posthi" + std::to_string(L - b), [=] {
          uint32_t r = L - b;
          std::vector<uint32_t> t(size_t(1) << r);
          for (uint32_t i2 = 0; i2 < t.size(); i2++) t[i2] = fp_pow(fp_encode(3), bitrev_n(i2, r));
          return t;
        });
      }
      launch_pass<true, false, true, false>(s, p);
    } else {
      launch_pass<true, false, false, true>(s, p);
    }
  }
}

void bit_reverse(hipStream_t s, uint32_t* io, size_t count, uint32_t L) {
  if (count == 0 || L < 2) return;
  KScope ks("bit_reverse", double(count) * 8 * (size_t(1) << L));
  uint32_t k = L / 2 < 5 ? L / 2 : 5;
  uint64_t nwg = uint64_t(count) << (L - 2 * k);
  R0_REQUIRE(nwg < (1ull << 31), "bit_reverse grid too large");
  hipLaunchKernelGGL(bit_reverse_tiles, dim3(unsigned(nwg)), dim3(kThreads), 0, s, io, L, k);
  HIP_OK(hipGetLastError());
}

void zk_shift(hipStream_t s, uint32_t* io, size_t count, uint32_t L) {
  uint64_t n = uint64_t(count) << L;
  if (n == 0) return;
  KScope ks("zk_shift", double(n) * 8);
  uint32_t h = L / 2;
  const uint32_t* A = dev_table("zkA" + std::to_string(L), [=] {
    std::vector<uint32_t> t(size_t(1) << h);
    uint32_t g = fp_pow(fp_encode(3), uint64_t(1) << (L - h)), cur = kOne;
    for (auto& x : t) {
      x = cur;
      cur = fp_mul(cur, g);
    }
    return t;
  });
  const uint32_t* B = dev_table("zkB" + std::to_string(L - h), [=] {
    std::vector<uint32_t> t(size_t(1) << (L - h));
    uint32_t cur = kOne, g = fp_encode(3);
    for (auto& x : t) {
      x = cur;
      cur = fp_mul(cur, g);
    }
    return t;
  });
  hipLaunchKernelGGL(zk_shift_kernel, dim3(div_up(n, kThreads)), dim3(kThreads), 0, s, io, n, L, h, A, B);
  HIP_OK(hipGetLastError());
}

}  // namespace r0
