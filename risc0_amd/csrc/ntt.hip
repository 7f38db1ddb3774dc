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
  const uint32_t* in;       // source: the caller's buffer for the first pass, == out after
  const uint32_t* local_tw; // [2^(s-1) + k] = w_{2^s}^k, s = 1..B (fwd or rev roots)
  const uint32_t* sc_lo;    // w_{2^(a+B)}^e = sc_hi[e >> sc_split] * sc_lo[e & mask]
  const uint32_t* sc_hi;
  const uint32_t* post_t;   // last inverse pass: per-t factor (norm * 3^{rev_B(t)*2^(L-B)})
  const uint32_t* post_hi;  // last inverse pass: per-row factor 3^{rev_{L-B}(row)} (or null)
  uint64_t groups;          // total groups of 2^B elements over the whole batch
  uint32_t L, a, eb;        // eb: expand bits (first forward pass only)
  uint32_t sc_split;
};

// Pass shapes are compile-time (B index bits per pass, 2^C rows or columns per
// workgroup), so every LDS index below is shifts and masks of constants.
//
// LDS placement. Row passes (a == 0) keep each row contiguous with one pad word per
// 8 so strided butterfly reads spread over the banks; column passes store [t][j]
// with the 2^C (= 32) adjacent columns of a row in consecutive words.
template <bool COLS, int B, int C>
__device__ __forceinline__ uint32_t lidx(uint32_t j, uint32_t t) {
  if (COLS) return (t << C) + j;
  return j * ((1u << B) + (1u << B >> 3)) + t + (t >> 3);
}
template <bool COLS, int B, int C>
constexpr uint32_t lds_words() {
  return COLS ? (1u << (B + C)) : ((1u << B) + (1u << B >> 3)) << C;
}

// One group of NST (1..3) radix-2 stages [S0, S0+NST) in registers: a lane owns blocks
// of 2^NST elements t_base + m*h (h = 2^(S0-1)), so a group costs one LDS read and
// write per element instead of NST. Twiddles come from the LDS copy of the table. S0 is a
// template parameter, so h and every shift below are constants.
template <bool INV, bool COLS, int B, int C, int NST, int FROM_EB, int NT, int S0>
__device__ __forceinline__ void stage_group(uint32_t* lds, const uint32_t* tw, const uint32_t* csrc) {
  if constexpr (NST > B) return;  // never reached; keeps the shifts below well-formed
  constexpr uint32_t M = 1u << NST;
  constexpr uint32_t h = 1u << (S0 - 1);
  constexpr uint32_t nrb = 1u << (B >= NST ? B - NST : 0);  // blocks per column/row
  constexpr uint32_t nblk = nrb << C;
  // Row layout t + (t >> 3): the elements t_base + m*h sit at constant offsets from
  // t_base's word when h is a multiple of 8 (m*h*9/8) or the whole block lies in one
  // 8-word run (h*M <= 8: t_base is aligned to h*M up to k < h, so t_base mod 8 +
  // (M-1)*h < 8); column layout (t << C) + j always.
  constexpr bool LIN = COLS || h % 8 == 0 || h * M <= 8;
  constexpr uint32_t step = COLS ? (h << C) : (h % 8 == 0 ? h + h / 8 : h);
#pragma unroll
  for (uint32_t it = 0; it < (nblk + NT - 1) / NT; it++) {
    const uint32_t blk = it * NT + threadIdx.x;
    if (nblk % NT != 0 && blk >= nblk) break;
    uint32_t j, r;
    if (COLS) {
      j = blk & ((1u << C) - 1);
      r = blk >> C;
    } else {
      j = blk >> (B >= NST ? B - NST : 0);
      r = blk & (nrb - 1);
    }
    const uint32_t k = r & (h - 1);
    const uint32_t tb = ((r >> (S0 - 1)) << (S0 - 1 + NST)) | k;
    const uint32_t base = lidx<COLS, B, C>(j, tb);
    uint32_t v[M];
#pragma unroll
    for (uint32_t m = 0; m < M; m++) {
      if (FROM_EB) v[m] = csrc[(j << (B - FROM_EB)) + ((tb + m * h) >> FROM_EB)];  // replicated input
      else v[m] = lds[LIN ? base + m * step : lidx<COLS, B, C>(j, tb + m * h)];
    }
    if (!INV) {
#pragma unroll
      for (uint32_t st = 0; st < NST; st++) {
        const uint32_t half = 1u << st, hs = h << st;
#pragma unroll
        for (uint32_t m = 0; m < M; m++) {
          if (m & half) continue;
          // a group that starts at stage 1 has k = 0, so its twiddle w_{2^s}^0 = 1 wherever
          // m & (half - 1) == 0 (all of stage 1, half of stage 2, a quarter of stage 3):
          // no multiply, the staged words being canonical already
          uint32_t x = v[m], y = v[m + half];
          if (!(S0 == 1 && (m & (half - 1)) == 0)) y = fp_mul(y, tw[hs + k + (m & (half - 1)) * h]);
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
          uint32_t x = v[m], y = v[m + half];
          v[m] = fp_add(x, y);
          v[m + half] = fp_sub(x, y);
          if (!(S0 == 1 && (m & (half - 1)) == 0)) v[m + half] = fp_mul(v[m + half], tw[hs + k + (m & (half - 1)) * h]);
        }
      }
    }
#pragma unroll
    for (uint32_t m = 0; m < M; m++) lds[LIN ? base + m * step : lidx<COLS, B, C>(j, tb + m * h)] = v[m];
  }
  __syncthreads();
}

// Stages per register group: n remaining stages in groups of at most MAXR (row passes
// R0_NTT_MAXR_ROW, column passes R0_NTT_MAXR_COL), sizes balanced, the larger ones first.
#ifndef R0_NTT_MAXR_ROW
#define R0_NTT_MAXR_ROW 3
#endif
#ifndef R0_NTT_MAXR_COL
#define R0_NTT_MAXR_COL 3
#endif
template <bool COLS>
constexpr int group_stages(int n) {
  const int maxr = COLS ? R0_NTT_MAXR_COL : R0_NTT_MAXR_ROW;
  const int g = (n + maxr - 1) / maxr;
  return (n + g - 1) / g;
}

// DIT stages [S, B] ascending, larger groups first; the first group of an expanding pass
// (S == EB + 1) reads the compact (unreplicated) input. Compile-time recursion, so each
// group's first stage is a constant.
template <bool COLS, int B, int C, int EB, int NT, int S>
__device__ __forceinline__ void fwd_stages(uint32_t* lds, const uint32_t* tw, const uint32_t* csrc) {
  if constexpr (S <= B) {
    constexpr int n = B - S + 1;
    constexpr int NST = group_stages<COLS>(n);
    constexpr int FROM = (S == EB + 1 && EB > 0) ? EB : 0;
    stage_group<false, COLS, B, C, NST, FROM, NT, S>(lds, tw, csrc);
    fwd_stages<COLS, B, C, EB, NT, S + NST>(lds, tw, csrc);
  }
}

// DIF stages [1, S] descending, larger groups first
template <bool COLS, int B, int C, int NT, int S>
__device__ __forceinline__ void inv_stages(uint32_t* lds, const uint32_t* tw) {
  if constexpr (S >= 1) {
    constexpr int NST = group_stages<COLS>(S);
    stage_group<true, COLS, B, C, NST, 0, NT, S - NST + 1>(lds, tw, nullptr);
    inv_stages<COLS, B, C, NT, S - NST>(lds, tw);
  }
}

// stages [EB+1, B] ascending (DIT) or [1, B] descending (DIF)
template <bool INV, bool COLS, int B, int C, int EB = 0, int NT = kThreads>
__device__ __forceinline__ void stages(uint32_t* lds, const uint32_t* tw, const uint32_t* csrc = nullptr) {
  if constexpr (!INV) fwd_stages<COLS, B, C, EB, NT, EB + 1>(lds, tw, csrc);
  else inv_stages<COLS, B, C, NT, B>(lds, tw);
}


// Column passes (2^C columns, B >= 8 - C): lane (j = tid mod 2^C, t0 = tid >> C)
// owns rows t = R*i + t0 with R = 256 >> C, so rev_B(t) = rev_r(t0)*2^(B-r) +
// rev_{B-r}(i) (r = log R) and its twiddles are base * c^k, k = rev_{B-r}(i) < E, with
// c = w_{2^(a+B)}^(low0+j) and base = c^(rev_r(t0)*2^(B-r)): E running products
// (8 independent chains) replace two table loads and a multiply per element.
template <int B, int C>
struct ColTwiddles {
  static constexpr uint32_t LR = 8 - C;  // log2 rows per i
  static constexpr uint32_t E = 1u << (B - LR);
  static constexpr uint32_t S = E < 8 ? E : 8;
  // f(i, w) for every i < E with w = base * c^k, k = rev_{B-LR}(i), walking k in order: S
  // running products advance by c^S, so only S twiddles are live at a time (a table of all E
  // held 32 more VGPRs per lane in the B = 9 column pass: 165 VGPRs, 3 waves per SIMD)
  template <typename F>
  __device__ __forceinline__ static void apply(const PassArgs& p, uint32_t ex, uint32_t t0, F&& f) {
    const uint32_t c = fp_mul(p.sc_hi[ex >> p.sc_split], p.sc_lo[ex & ((1u << p.sc_split) - 1)]);
    uint32_t cur[S];
    cur[0] = fp_pow(c, uint64_t(bitrev_n(t0, LR)) << (B - LR));
#pragma unroll
    for (uint32_t k = 1; k < S; k++) cur[k] = fp_mul(cur[k - 1], c);
    uint32_t step = c;
#pragma unroll
    for (uint32_t k = 1; k < S; k <<= 1) step = fp_mul(step, step);  // c^S
#pragma unroll
    for (uint32_t k0 = 0; k0 < E; k0 += S) {
#pragma unroll
      for (uint32_t s = 0; s < S; s++) {
        f(bitrev_n(k0 + s, B - LR), cur[s]);
        if (k0 + S < E) cur[s] = fp_mul(cur[s], step);
      }
    }
  }
};

// Column passes with 2^C < 32 columns cover half an L2 line per workgroup. Consecutive
// block ids land on consecutive XCDs, so the block -> column-group map pairs blocks
// b and b+8 (same XCD, dispatched together) on the two halves of each 128-B line.
template <int C>
__device__ __forceinline__ uint64_t col_block(uint64_t b) {
  if constexpr (C >= 5) return b;
  constexpr uint64_t H = uint64_t(1) << (C < 5 ? 5 - C : 0);  // workgroups per 128-B line
  const uint64_t grp = b / (8 * H), r = b % (8 * H);
  return grp * (8 * H) + (r % 8) * H + r / 8;
}

template <bool INV, bool EXPAND, bool LAST, bool COLS, int B, int C, int EB, int NT>
__global__ __launch_bounds__(NT) void ntt_pass_kernel(PassArgs p) {
  static_assert(!COLS || NT == kThreads, "column passes assume 256 lanes (ColTwiddles)");
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* tw = lds + lds_words<COLS, B, C>();
  const uint32_t tid = threadIdx.x;
  constexpr uint32_t nb = 1u << B;
  constexpr uint32_t total = nb << C;
  const uint64_t wg = COLS ? col_block<C>(blockIdx.x) : uint64_t(blockIdx.x);
  // stage twiddles -> LDS (entries 1 .. 2^B - 1)
#pragma unroll
  for (uint32_t i = 0; i < (nb + NT - 1) / NT; i++) {
    uint32_t q = i * NT + tid;
    if (q < nb) tw[q] = p.local_tw[q];
  }
  uint64_t g_hi = 0;
  uint32_t low0 = 0;
  if (COLS) {
    const uint32_t lowblocks = 1u << (p.a - C);
    low0 = uint32_t(wg & (lowblocks - 1)) << C;
    g_hi = wg >> (p.a - C);
  }
  // ---- load: every global load of the workgroup is issued before the first LDS
  // write (E words per lane in registers), so each lane has E loads in flight ----
  uint32_t* compact = tw + nb;  // expand passes: the 2^(B+C-EB) distinct input words
  if constexpr (!COLS) {
    // rows [wg*2^C, +2^C): a contiguous run of 2^(B+C-EB) source words (expand: each
    // stands for 2^EB replicated slots, which the first stage group reads in place)
    constexpr uint32_t NIN = total >> EB;
    constexpr uint32_t EIN = (NIN + NT - 1) / NT;
    const uint32_t* src = p.in;
    const uint64_t base = wg << (B + C - EB);
    const uint64_t limit = p.groups << (B - EB);
    uint32_t r[EIN];
#pragma unroll
    for (uint32_t i = 0; i < EIN; i++) {
      const uint32_t q = i * NT + tid;
      r[i] = 0;
      if ((NIN % NT == 0 || q < NIN) && base + q < limit) r[i] = src[base + q];
    }
#pragma unroll
    for (uint32_t i = 0; i < EIN; i++) {
      const uint32_t q = i * NT + tid;
      if (NIN % NT != 0 && q >= NIN) continue;
      if (EB == 0) lds[lidx<COLS, B, C>(q >> B, q & (nb - 1))] = r[i];
      else if (EB >= B) {
#pragma unroll
        for (uint32_t rep = 0; rep < (1u << EB); rep++) {
          const uint32_t el = (q << EB) + rep;
          lds[lidx<COLS, B, C>(el >> B, el & (nb - 1))] = r[i];
        }
      } else compact[q] = r[i];
    }
  } else if constexpr (B < 8 - C) {
    // tiny column passes: plain mapping, table twiddles
    constexpr uint32_t E = (total + NT - 1) / NT;
#pragma unroll
    for (uint32_t i = 0; i < E; i++) {
      const uint32_t idx = i * NT + tid;
      if (total % NT != 0 && idx >= total) continue;
      const uint32_t j = idx & ((1u << C) - 1), t = idx >> C;
      uint32_t v = p.in[(g_hi << (p.a + B)) + (uint64_t(t) << p.a) + low0 + j];
      if (!INV) {
        const uint32_t ex = (low0 + j) * bitrev_n(t, B);
        v = fp_mul(v, fp_mul(p.sc_hi[ex >> p.sc_split], p.sc_lo[ex & ((1u << p.sc_split) - 1)]));
      }
      lds[lidx<COLS, B, C>(j, t)] = v;
    }
  } else {
    // 2^C adjacent columns x 2^B rows of stride 2^a. Lane (j, r0) owns the rows t with
    // rev_B(t) = u = r0*E + i, i < E, so its forward pre-scale factors
    // w_{2^(a+B)}^{(low0+j)*u} are one running product (c^i) — no table loads.
    constexpr uint32_t E = total / NT;
    constexpr uint32_t R = NT >> C;  // rows per i
    const uint32_t j = tid & ((1u << C) - 1), t0 = tid >> C;
    // a uniform base and 32-bit byte offsets (a pass spans 2^(a+B) <= 2^L words): saddr-form
    // loads, one VGPR of offset per load instead of a 64-bit address pair
    const char* cbase = reinterpret_cast<const char*>(p.in + (g_hi << (p.a + B)) + low0);
    const uint32_t off0 = ((t0 << p.a) + j) * 4u, ostep = (R << p.a) * 4u;
    uint32_t r[E];
#pragma unroll
    for (uint32_t i = 0; i < E; i++) r[i] = *reinterpret_cast<const uint32_t*>(cbase + (off0 + i * ostep));
    if (!INV) ColTwiddles<B, C>::apply(p, low0 + j, t0, [&](uint32_t i, uint32_t w) { r[i] = fp_mul(r[i], w); });
#pragma unroll
    for (uint32_t i = 0; i < E; i++) lds[lidx<COLS, B, C>(j, R * i + t0)] = r[i];
  }
  __syncthreads();
  if (!INV) stages<false, COLS, B, C, (EB < B ? EB : 0), NT>(lds, tw, compact);
  else stages<true, COLS, B, C, 0, NT>(lds, tw);
  // ---- store (inverse column passes post-scale; last inverse pass normalises) ----
  if constexpr (COLS && B >= 8 - C) {
    constexpr uint32_t E = total / NT;
    constexpr uint32_t R = NT >> C;
    const uint32_t j = tid & ((1u << C) - 1), t0 = tid >> C;
    char* obase = reinterpret_cast<char*>(p.out + (g_hi << (p.a + B)) + low0);
    const uint32_t off0 = ((t0 << p.a) + j) * 4u, ostep = (R << p.a) * 4u;
    auto put = [&](uint32_t i, uint32_t v) { *reinterpret_cast<uint32_t*>(obase + (off0 + i * ostep)) = v; };
    if (INV) {
      ColTwiddles<B, C>::apply(p, low0 + j, t0, [&](uint32_t i, uint32_t w) {
        put(i, fp_mul(lds[lidx<COLS, B, C>(j, R * i + t0)], w));
      });
    } else {
#pragma unroll
      for (uint32_t i = 0; i < E; i++) put(i, lds[lidx<COLS, B, C>(j, R * i + t0)]);
    }
    return;
  }
#pragma unroll 4
  for (uint32_t idx = tid; idx < total; idx += NT) {
    uint32_t t, j;
    uint64_t e;
    if (!COLS) {
      t = idx & (nb - 1);
      j = idx >> B;
      const uint64_t g = (wg << C) + j;
      if (g >= p.groups) continue;
      e = (g << B) + t;
    } else {
      j = idx & ((1u << C) - 1);
      t = idx >> C;
      e = (g_hi << (p.a + B)) + (uint64_t(t) << p.a) + low0 + j;
    }
    uint32_t v = lds[lidx<COLS, B, C>(j, t)];
    if (INV && COLS) {
      const uint32_t ex = (low0 + j) * bitrev_n(t, B);
      v = fp_mul(v, fp_mul(p.sc_hi[ex >> p.sc_split], p.sc_lo[ex & ((1u << p.sc_split) - 1)]));
    }
    if (LAST) {
      v = fp_mul(v, p.post_t[t]);
      if (p.post_hi) {
        const uint64_t g = (wg << C) + j;
        const uint32_t row = uint32_t(g & ((uint64_t(1) << (p.L - B)) - 1));
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
// T = uint32_t for Fp rows, uint4 for rows of FpExt (AoS, 16-byte elements).
template <typename T>
__global__ __launch_bounds__(kThreads) void bit_reverse_tiles(T* io, uint32_t L, uint32_t k) {
  __shared__ T ta[32 * 33];
  __shared__ T tb[32 * 33];
  const uint32_t m = L - 2 * k;
  const uint32_t nmid = 1u << m;
  const uint32_t mid = blockIdx.x % nmid;
  const uint64_t row = blockIdx.x / nmid;
  const uint32_t rmid = bitrev_n(mid, m);
  if (mid > rmid) return;
  const uint32_t K = 1u << k;
  T* base = io + (row << L);
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
  for (uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kThreads) {
    uint32_t pos = uint32_t(i & ((uint64_t(1) << L) - 1));
    uint32_t lo = pos & ((1u << h) - 1), hi = pos >> h;
    io[i] = fp_mul(io[i], fp_mul(A[bitrev_n(lo, h)], B[bitrev_n(hi, L - h)]));
  }
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

// columns per workgroup of a column pass (log2): 16 columns (32 KiB of LDS at B = 9,
// four workgroups per CU; see col_block for the L2-line pairing) for the deep passes,
// 32 columns below B = 8 where LDS does not limit occupancy (measured: B = 9 forward
// 3.47 -> 2.32 ms with 16 columns; B = 7 inverse 0.45 -> 0.52 ms, so it keeps 32)
constexpr int col_c(int B) { return B >= 8 ? 4 : 5; }

// rows per workgroup of a row pass: enough rows that a workgroup holds >= 2048 words
constexpr int row_c(int B) { return B >= 11 ? 0 : 11 - B; }

template <bool INV, bool EXPAND, bool LAST, bool COLS, int B, int EB>
void launch_pass_be(hipStream_t s, const PassArgs& p) {
  constexpr int C = COLS ? col_c(B) : row_c(B);
  if (COLS) R0_REQUIRE(p.a >= 5, "column pass needs >= 32 columns");
  const size_t lds =
      4 * (size_t(lds_words<COLS, B, C>()) + (size_t(1) << B) + (EB > 0 && EB < B ? (size_t(1) << (B + C - EB)) : 0));
  uint64_t nwg = COLS ? (p.groups >> C) : ((p.groups + (uint64_t(1) << C) - 1) >> C);
  R0_REQUIRE(nwg < (1ull << 31), "ntt grid too large");
  // 13-bit row passes hold ~74 KB of LDS (data + stage twiddles), so only two workgroups
  // fit a CU: 1024 lanes per workgroup (forward and inverse) multiply the waves that hide
  // their loads (forward 512 -> 1024 lanes: 2219 -> 2148 us per pass, profiles/r3m_ntt_*)
  constexpr int NT = (!COLS && B >= 13) ? 1024 : kThreads;
  hipLaunchKernelGGL((ntt_pass_kernel<INV, EXPAND, LAST, COLS, B, C, EB, NT>), dim3(unsigned(nwg)), dim3(NT), lds,
                     s, p);
  HIP_OK(hipGetLastError());
}

template <bool INV, bool EXPAND, bool LAST, bool COLS, int B>
void launch_pass_b(hipStream_t s, const PassArgs& p) {
  if (!EXPAND || p.eb == 0) return launch_pass_be<INV, EXPAND, LAST, COLS, B, 0>(s, p);
  if constexpr (EXPAND && !COLS) {
    if (p.eb == 1 && B >= 1) return launch_pass_be<INV, EXPAND, LAST, COLS, B, (B >= 1 ? 1 : 0)>(s, p);
    if (p.eb == 2 && B >= 2) return launch_pass_be<INV, EXPAND, LAST, COLS, B, (B >= 2 ? 2 : 0)>(s, p);
    if (p.eb == 3 && B >= 3) return launch_pass_be<INV, EXPAND, LAST, COLS, B, (B >= 3 ? 3 : 0)>(s, p);
  }
  R0_REQUIRE(false, "unsupported expand_bits for this NTT pass");
}

template <bool INV, bool EXPAND, bool LAST, bool COLS>
void launch_pass(hipStream_t s, const PassArgs& p, uint32_t b) {
  switch (b) {
#define R0_CASE(X) \
  case X: return launch_pass_b<INV, EXPAND, LAST, COLS, X>(s, p);
    R0_CASE(1) R0_CASE(2) R0_CASE(3) R0_CASE(4) R0_CASE(5) R0_CASE(6) R0_CASE(7) R0_CASE(8) R0_CASE(9)
#undef R0_CASE
    default: break;
  }
  if (!COLS) {
    switch (b) {
      case 10: return launch_pass_b<INV, EXPAND, LAST, false, 10>(s, p);
      case 11: return launch_pass_b<INV, EXPAND, LAST, false, 11>(s, p);
      case 12: return launch_pass_b<INV, EXPAND, LAST, false, 12>(s, p);
      case 13: return launch_pass_b<INV, EXPAND, LAST, false, 13>(s, p);
      default: break;
    }
  }
  R0_REQUIRE(false, "unsupported NTT pass size");
}

void fill_pass(PassArgs& p, bool inv, uint32_t L, uint32_t a, uint32_t b, size_t count) {
  p.L = L;
  p.a = a;
  p.groups = uint64_t(count) << (L - b);
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
    p.in = i == 0 ? in : out;
    p.eb = eb;
    fill_pass(p, false, L, pl[i].first, pl[i].second, count);
    if (i == 0) launch_pass<false, true, false, false>(s, p, pl[i].second);
    else launch_pass<false, false, false, true>(s, p, pl[i].second);
  }
}

void ntt_interpolate(hipStream_t s, uint32_t* io, size_t count, uint32_t L, bool zk) {
  ntt_interpolate_from(s, io, io, count, L, zk);
}

// io = interpolate(src): the first pass reads `src` (e.g. the witness) directly, so an
// out-of-place transform costs no extra copy
void ntt_interpolate_from(hipStream_t s, uint32_t* io, const uint32_t* src, size_t count, uint32_t L, bool zk) {
  if (count == 0) return;
  if (L == 0) {  // size-1 transform (and 3^0 shift) is the identity
    if (src != io) HIP_OK(hipMemcpyAsync(io, src, count * 4, hipMemcpyDeviceToDevice, s));
    return;
  }
  KScope ks("ntt_interpolate", double(count) * 8 * (size_t(1) << L), double(count) * double(size_t(1) << L) / 2 * L);
  auto pl = plan(L);
  for (size_t i = pl.size(); i-- > 0;) {
    PassArgs p{};
    p.out = io;
    p.in = i == pl.size() - 1 ? src : io;
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
      launch_pass<true, false, true, false>(s, p, b);
    } else {
      launch_pass<true, false, false, true>(s, p, pl[i].second);
    }
  }
}

template <typename T>
static void launch_bit_reverse(hipStream_t s, T* io, size_t count, uint32_t L) {
  KScope ks("bit_reverse", double(count) * 2 * sizeof(T) * (size_t(1) << L));
  uint32_t k = L / 2 < 5 ? L / 2 : 5;
  uint64_t nwg = uint64_t(count) << (L - 2 * k);
  R0_REQUIRE(nwg < (1ull << 31), "bit_reverse grid too large");
  hipLaunchKernelGGL(bit_reverse_tiles<T>, dim3(unsigned(nwg)), dim3(kThreads), 0, s, io, L, k);
  HIP_OK(hipGetLastError());
}

void bit_reverse(hipStream_t s, uint32_t* io, size_t count, uint32_t L) {
  if (count == 0 || L < 2) return;
  launch_bit_reverse(s, io, count, L);
}

void bit_reverse_ext(hipStream_t s, uint32_t* io, size_t count, uint32_t L) {
  if (count == 0 || L < 2) return;
  launch_bit_reverse(s, reinterpret_cast<uint4*>(io), count, L);
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
  hipLaunchKernelGGL(zk_shift_kernel, dim3(grid_stride(n, kThreads)), dim3(kThreads), 0, s, io, n, L, h, A, B);
  HIP_OK(hipGetLastError());
}

}  // namespace r0
