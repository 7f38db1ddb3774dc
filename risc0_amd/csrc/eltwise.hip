// Element-wise and polynomial HAL kernels for CDNA4: mix_poly_coeffs,
// batch_evaluate_any, fri_fold, eltwise_{add,copy,zeroize,sum_extelem},
// gather_sample, scatter, copy_elem_slice, prefix_products and the parallel
// synthetic division behind combos_divide. Semantics follow
// risc0/zkp/src/hal/cpu.rs (line refs on each kernel). All HBM-bound except
// evaluate_any/poly_divide, which are integer-VALU bound.
#include "runtime.h"

#include <map>

#include <algorithm>

namespace r0 {
namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ FpExt ld_fe(const uint32_t* p) {
  uint4 v = *reinterpret_cast<const uint4*>(p);
  return FpExt{{v.x, v.y, v.z, v.w}};
}
__device__ __forceinline__ void st_fe(uint32_t* p, FpExt a) {
  *reinterpret_cast<uint4*>(p) = make_uint4(a.c[0], a.c[1], a.c[2], a.c[3]);
}

// ---- element-wise ---------------------------------------------------------------
__global__ void add_kernel(uint32_t* o, const uint32_t* a, const uint32_t* b, uint64_t n) {
  for (uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kThreads)
    o[i] = fp_add(a[i], b[i]);
}
// cpu.rs:518-522: INVALID (0xffffffff) -> 0
__global__ void zeroize_kernel(uint32_t* io, uint64_t n) {
  for (uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kThreads)
    if (io[i] == 0xffffffffu) io[i] = 0;
}
// synthetic witness words (uniform canonical BabyBear values): a
// splitmix64 counter hash of (seed, index), reduced mod p — for benches and tests at sizes
// whose host generation and upload would dominate
__global__ void fill_uniform_kernel(uint32_t* o, uint64_t n, uint64_t seed) {
  for (uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x; i < n; i += uint64_t(gridDim.x) * kThreads) {
    uint64_t z = seed + (i + 1) * 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    z ^= z >> 31;
    o[i] = uint32_t(z % kP);
  }
}
// cpu.rs:475-500: out[k*count + idx] = (sum_i in[i*count + idx])[k]
__global__ void sum_extelem_kernel(uint32_t* out, const uint32_t* in, uint64_t count, uint32_t to_add) {
  uint64_t idx = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (idx >= count) return;
  FpExt s = fe_zero();
  for (uint32_t i = 0; i < to_add; i++) s = fe_add(s, ld_fe(in + (i * count + idx) * 4));
#pragma unroll
  for (int k = 0; k < 4; k++) out[k * count + idx] = s.c[k];
}
// cpu.rs:524-553 (FRI_FOLD = 16, rev_i = bit_rev over 4 bits)
__global__ void fri_fold_kernel(uint32_t* out, const uint32_t* in, FpExt mix, uint64_t count) {
  uint64_t idx = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (idx >= count) return;
  FpExt tot = fe_zero(), cur = fe_one();
#pragma unroll
  for (uint32_t i = 0; i < 16; i++) {
    uint64_t rev_idx = uint64_t(bitrev_n(i, 4)) * count + idx;
    FpExt f;
#pragma unroll
    for (int k = 0; k < 4; k++) f.c[k] = in[k * count * 16 + rev_idx];
    tot = fe_add(tot, fe_mul(cur, f));
    cur = fe_mul(cur, mix);
  }
#pragma unroll
  for (int k = 0; k < 4; k++) out[k * count + idx] = tot.c[k];
}
// cpu.rs:583-596
__global__ void gather_kernel(uint32_t* dst, const uint32_t* src, uint64_t idx, uint64_t size, uint64_t stride) {
  uint64_t g = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (g < size) dst[g] = src[g * stride + idx];
}
// cpu.rs:598-615: one lane per cycle walks its CSR slice
// offsets at or past `limit` (the buffer's words) are skipped, and no row reads entries past
// index[cycles] (the arrays' length): a resident injector the host has not checked can neither
// write outside the buffer nor read past its own arrays
__global__ void scatter_kernel(uint32_t* into, const uint32_t* index, const uint32_t* offsets,
                               const uint32_t* values, uint64_t cycles, uint64_t limit) {
  uint64_t c = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (c >= cycles) return;
  const uint32_t end = min(index[c + 1], index[cycles]);
  for (uint32_t i = index[c]; i < end; i++)
    if (offsets[i] < limit) into[offsets[i]] = values[i];
}
// cpu.rs:617-635
__global__ void copy_slice_kernel(uint32_t* into, const uint32_t* from, uint64_t rows, uint64_t cols,
                                  uint64_t from_offset, uint64_t from_stride, uint64_t into_offset,
                                  uint64_t into_stride) {
  for (uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x; i < rows * cols;
       i += uint64_t(gridDim.x) * kThreads) {
    uint64_t r = i / cols, c = i % cols;
    into[into_offset + r * into_stride + c] = from[from_offset + r * from_stride + c];
  }
}

// ---- mix_poly_coeffs (cpu.rs:410-455) ---------------------------------------------
// out[combo*count + idx] += sum_{i: combos[i]==combo} mix_start*mix^i * in[i*count + idx]
// The host sorts the input rows by combo (rows[], with their mix powers in the same
// order, and one segment per combo). One lane per idx streams its segment's rows with
// coalesced loads, four in flight, into four unreduced u64 sums (one v_mad_u64_u32 per
// product limb, folded every 3 products below 2^64), then one REDC per limb and one add
// into the combo's FpExt: per product 4 multiply-adds instead of a canonical FpExt*Fp
// multiply and add (32 instructions).
__global__ __launch_bounds__(kThreads) void mix_kernel(uint32_t* out, const uint32_t* __restrict__ in,
                                                      const uint32_t* __restrict__ rows,
                                                      const uint32_t* __restrict__ pows,  // FpExt per sorted row
                                                      const uint32_t* __restrict__ seg,   // nseg + 1 bounds
                                                      const uint32_t* __restrict__ seg_combo, uint32_t nseg,
                                                      uint64_t count) {
  const uint64_t idx = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (idx >= count) return;
  for (uint32_t sg = 0; sg < nseg; sg++) {
    const uint32_t b = seg[sg], e = seg[sg + 1];
    uint64_t a[4] = {0, 0, 0, 0};
    uint32_t since_fold = 0;  // products added since the sums were last folded (< 2^58)
    for (uint32_t j = b; j < e; j += 4) {
      uint32_t v[4];
#pragma unroll
      for (int u = 0; u < 4; u++) v[u] = j + u < e ? in[uint64_t(rows[j + u]) * count + idx] : 0u;
#pragma unroll
      for (int u = 0; u < 4; u++) {
        if (since_fold == 3) {  // 2^58 + 3 p^2 < 2^64; one more product could pass it
#pragma unroll
          for (int k = 0; k < 4; k++) a[k] = fold64(a[k]);
          since_fold = 0;
        }
        const uint32_t* pw = pows + 4 * uint64_t(j + u < e ? j + u : b);
#pragma unroll
        for (int k = 0; k < 4; k++) a[k] += uint64_t(v[u]) * pw[k];
        since_fold++;
      }
    }
    uint32_t* o = out + (uint64_t(seg_combo[sg]) * count + idx) * 4;
    FpExt r;
#pragma unroll
    for (int k = 0; k < 4; k++) r.c[k] = mont_reduce(fold64(a[k]));
    st_fe(o, fe_add(ld_fe(o), r));
  }
}

// ---- batch_evaluate_any (cpu.rs:362-393) -----------------------------------------
// out[k] = sum_i coeffs[which[k]][i] * xs[k]^i. Evaluations of the same polynomial
// are grouped (a trace column has one tap per `back`), so each coefficient is read
// once per group. A workgroup reads a 16384-coefficient chunk of one polynomial; each of
// its waves owns 4096 of them and works alone (no workgroup barrier per evaluation).
// The wave reads its piece with fully coalesced 1 KB uint4 loads, so lane l holds the
// coefficients at 256 q + 4 l + r (q < 16, r < 4); per evaluation x it forms
// sum c x^(256 q + r) as four unreduced u64 dot products against the wave's copy of that
// 64-entry table in LDS (4 v_mad_u64_u32 per coefficient, folded every 4), scales by
// x^(4 l), and the wave adds its lanes with xor shuffles. A last kernel combines the
// 4096-coefficient pieces by Horner in x^4096.
// Bit-reversed rows (the inverse NTT's order, L >= 12 bits): stored position
// j = piece*4096 + 256 q + 4 l + r holds coefficient rev_L(j) = rev_2(r) 2^(L-2) +
// rev_6(l) 2^(L-8) + rev_4(q) 2^(L-12) + rev_(L-12)(piece), so the same kernel runs with
// the table x^(rev_2(r) 2^(L-2) + rev_4(q) 2^(L-12)), the lane scale x^(rev_6(l) 2^(L-8)),
// and the pieces are summed with weights x^rev_(L-12)(piece) instead of by Horner.
constexpr int kEvLane = 64;                     // coefficients per lane
constexpr int kEvWave = 64 * kEvLane;           // 4096 per wave
constexpr int kEvChunk = kThreads * kEvLane;    // 16384 per workgroup
constexpr int kEvTab = kEvLane + 64 + 1;        // x^(256 q + r), x^(4 l) l < 64, x^4096

__global__ __launch_bounds__(kThreads) void eval_tables_kernel(const uint32_t* __restrict__ xs, uint32_t evals,
                                                             uint32_t* tab, uint32_t L, bool bitrev) {
  const uint64_t id = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (id >= uint64_t(evals) * kEvTab) return;
  const uint32_t k = uint32_t(id / kEvTab), e = uint32_t(id % kEvTab);
  const FpExt x = ld_fe(xs + 4 * k);
  uint64_t pw;
  if (!bitrev)
    pw = e < kEvLane ? 256 * (e >> 2) + (e & 3) : (e < kEvLane + 64 ? 4 * (e - kEvLane) : kEvWave);
  else if (e < kEvLane)
    pw = (uint64_t(bitrev_n(e & 3, 2)) << (L - 2)) + (uint64_t(bitrev_n(e >> 2, 4)) << (L - 12));
  else if (e < kEvLane + 64)
    pw = uint64_t(bitrev_n(e - kEvLane, 6)) << (L - 8);
  else
    pw = 0;  // no Horner step
  st_fe(tab + (uint64_t(k) * kEvTab + e) * 4, fe_pow(x, pw));
}

__device__ __forceinline__ FpExt shfl_xor4(const FpExt& a, int m) {
  FpExt r;
#pragma unroll
  for (int i = 0; i < 4; i++) r.c[i] = __shfl_xor(a.c[i], m, 64);
  return r;
}

__global__ __launch_bounds__(kThreads) void eval_chunk_kernel(const uint32_t* __restrict__ coeffs, uint64_t n,
                                                            const uint32_t* __restrict__ gpoly,
                                                            const uint32_t* __restrict__ gbegin,
                                                            const uint32_t* __restrict__ geval,
                                                            const uint32_t* __restrict__ tab, uint32_t* partial,
                                                            uint32_t npieces) {
  __shared__ FpExt xp[kThreads / 64][kEvLane];  // one x^0..63 table per wave
  const uint32_t g = blockIdx.y, chunk = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t piece = chunk * (kThreads / 64) + wave;
  const uint32_t* poly = coeffs + uint64_t(gpoly[g]) * n;
  const uint64_t start = uint64_t(piece) * kEvWave;
  uint32_t c[kEvLane];  // c[4 q + r] = coefficient start + 256 q + 4 lane + r
  if (start + kEvWave <= n) {
    const uint4* src = reinterpret_cast<const uint4*>(poly + start);
#pragma unroll
    for (int q = 0; q < kEvLane / 4; q++) {
      const uint4 v = src[q * 64 + lane];
      c[4 * q] = v.x;
      c[4 * q + 1] = v.y;
      c[4 * q + 2] = v.z;
      c[4 * q + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < kEvLane; j++) {
      const uint64_t i = start + 256 * (j >> 2) + 4 * lane + (j & 3);
      c[j] = i < n ? poly[i] : 0u;
    }
  }
  FpExt* t = xp[wave];
  for (uint32_t q = gbegin[g]; q < gbegin[g + 1]; q++) {
    const uint32_t k = geval[q];
    const uint32_t* tk = tab + uint64_t(k) * kEvTab * 4;
    // the wave's previous readers of t are done (one wave, LDS ops in order): rewrite it
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    t[lane] = ld_fe(tk + 4 * lane);
    const FpExt scale = ld_fe(tk + 4 * (kEvLane + lane));
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    uint64_t acc[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < kEvLane; j++) {
      const FpExt w = t[j];
#pragma unroll
      for (int i = 0; i < 4; i++) acc[i] += uint64_t(c[j]) * w.c[i];
      if (j % 4 == 3) {
#pragma unroll
        for (int i = 0; i < 4; i++) acc[i] = fold64(acc[i]);
        // keep the table reads next to their products: hoisted, the 64 ds_read_b128
        // results took 256 VGPRs and spilled to scratch
        asm volatile("" ::: "memory");
      }
    }
    FpExt a{{mont_reduce(acc[0]), mont_reduce(acc[1]), mont_reduce(acc[2]), mont_reduce(acc[3])}};
    a = fe_mul(a, scale);
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) a = fe_add(a, shfl_xor4(a, m));
    if (lane == 0) st_fe(partial + (uint64_t(k) * npieces + piece) * 4, a);
    __builtin_amdgcn_wave_barrier();
  }
}

// one wave per evaluation: lane l runs Horner over pieces l, l + 64, ... in y^64 (y = x^4096),
// then the wave adds S_l * y^l. Bit-reversed rows: lane l adds piece c times x^rev_P(c)
// (P = L - 12) for c = l, l + 64, ...
__global__ __launch_bounds__(kThreads) void eval_any_reduce(const uint32_t* partial, uint32_t npieces,
                                                          const uint32_t* tab, uint32_t* out, uint32_t evals,
                                                          const uint32_t* xs, uint32_t L, bool bitrev) {
  const uint32_t k = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (k >= evals) return;  // whole waves leave together
  const uint32_t* pk = partial + uint64_t(k) * npieces * 4;
  if (bitrev) {
    const FpExt x = ld_fe(xs + 4 * k);
    FpExt s = fe_zero();
    for (uint32_t c = lane; c < npieces; c += 64)
      s = fe_add(s, fe_mul(ld_fe(pk + uint64_t(c) * 4), fe_pow(x, bitrev_n(c, L - 12))));
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s = fe_add(s, shfl_xor4(s, m));
    if (lane == 0) st_fe(out + uint64_t(k) * 4, s);
    return;
  }
  const FpExt y = ld_fe(tab + (uint64_t(k) * kEvTab + kEvTab - 1) * 4);  // x^4096
  FpExt y64 = y;
#pragma unroll
  for (int i = 0; i < 6; i++) y64 = fe_mul(y64, y64);
  FpExt s = fe_zero();
  if (lane < npieces) {
    uint32_t c = lane + ((npieces - 1 - lane) / 64) * 64;  // the lane's last piece
    for (;; c -= 64) {
      s = fe_add(fe_mul(s, y64), ld_fe(pk + uint64_t(c) * 4));
      if (c < 64) break;
    }
  }
  s = fe_mul(s, fe_pow(y, lane));
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s = fe_add(s, shfl_xor4(s, m));
  if (lane == 0) st_fe(out + uint64_t(k) * 4, s);
}

// ---- prefix products (cpu.rs:637-642), serial by definition --------------------------
__global__ void prefix_products_kernel(uint32_t* io, uint64_t n) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  FpExt prev = ld_fe(io);
  for (uint64_t i = 1; i < n; i++) {
    prev = fe_mul(ld_fe(io + 4 * i), prev);
    st_fe(io + 4 * i, prev);
  }
}

// ---- synthetic division (core/poly.rs:81-89) -----------------------------------------
// p(x) = q(x) (x - z) + r. Going down from the top, cur_i = z*cur_{i+1} + p_i and
// p_i <- cur_{i+1}. A lane owning 16 coefficients maps an incoming carry c to
// Z*c + L (Z = z^16, L = its local sum), an affine map; composing maps is
// associative, so the row is solved as a two-level scan:
//   div_local  : each lane computes L
//   div_block  : each 256-lane workgroup scans its maps (Hillis-Steele in LDS),
//                keeps per-lane "maps of the lanes above me" and its block map
//   div_top    : one workgroup per row scans the block maps from the top and
//                produces each block's carry-in and the remainder cur_0
//   div_apply  : each lane rewrites its 16 quotients from its carry-in
// All rows of one division round run in the same launches (grid.y = row).
constexpr int kDivPer = 16;

struct DivRow {
  uint32_t* p;     // row base (FpExt AoS)
  FpExt z;
  uint32_t* rem;   // where the remainder goes (FpExt)
};

__global__ __launch_bounds__(kThreads) void div_local_kernel(const DivRow* rows, uint32_t nlanes, uint32_t* lanev) {
  const DivRow r = rows[blockIdx.y];
  uint32_t lane = blockIdx.x * kThreads + threadIdx.x;
  if (lane >= nlanes) return;
  const uint32_t* p = r.p + uint64_t(lane) * kDivPer * 4;
  FpExt cur = fe_zero();
#pragma unroll
  for (int i = kDivPer - 1; i >= 0; i--) cur = fe_add(fe_mul(r.z, cur), ld_fe(p + 4 * i));
  st_fe(lanev + (uint64_t(blockIdx.y) * nlanes + lane) * 4, cur);
}

// in: lanev = L per lane. out: lanev = v_{t+1}, lanem = m_{t+1} (maps of lanes above
// t inside the block), blockv/blockm = whole-block map.
__global__ __launch_bounds__(kThreads) void div_block_kernel(const DivRow* rows, uint32_t nlanes, uint32_t* lanev,
                                                            uint32_t* lanem, uint32_t* blockv, uint32_t* blockm) {
  __shared__ FpExt vals[kThreads + 1];
  __shared__ FpExt mul[kThreads + 1];
  const uint32_t row = blockIdx.y, tid = threadIdx.x, nblocks = gridDim.x;
  const uint32_t lane = blockIdx.x * kThreads + tid;
  const FpExt Z = fe_pow(rows[row].z, kDivPer);
  uint32_t* lv = lanev + (uint64_t(row) * nlanes) * 4;
  vals[tid] = lane < nlanes ? ld_fe(lv + uint64_t(lane) * 4) : fe_zero();
  mul[tid] = lane < nlanes ? Z : fe_one();
  if (tid == 0) {
    vals[kThreads] = fe_zero();
    mul[kThreads] = fe_one();
  }
  __syncthreads();
  for (uint32_t off = 1; off < kThreads; off <<= 1) {
    FpExt v = vals[tid], m = mul[tid];
    if (tid + off < kThreads) {
      v = fe_add(v, fe_mul(m, vals[tid + off]));
      m = fe_mul(m, mul[tid + off]);
    }
    __syncthreads();
    vals[tid] = v;
    mul[tid] = m;
    __syncthreads();
  }
  if (lane < nlanes) {
    st_fe(lv + uint64_t(lane) * 4, vals[tid + 1]);
    st_fe(lanem + (uint64_t(row) * nlanes + lane) * 4, mul[tid + 1]);
  }
  if (tid == 0) {
    st_fe(blockv + (uint64_t(row) * nblocks + blockIdx.x) * 4, vals[0]);
    st_fe(blockm + (uint64_t(row) * nblocks + blockIdx.x) * 4, mul[0]);
  }
}

// blockv <- carry into the top lane of each block; the row's remainder = cur_0.
__global__ __launch_bounds__(kThreads) void div_top_kernel(const DivRow* rows, uint32_t nblocks, uint32_t* blockv,
                                                          const uint32_t* blockm) {
  __shared__ FpExt vals[kThreads + 1];
  __shared__ FpExt mul[kThreads + 1];
  const uint32_t row = blockIdx.x, tid = threadIdx.x;
  uint32_t* bv = blockv + uint64_t(row) * nblocks * 4;
  const uint32_t* bm = blockm + uint64_t(row) * nblocks * 4;
  FpExt carry = fe_zero();
  uint32_t nseg = (nblocks + kThreads - 1) / kThreads;
  for (int seg = int(nseg) - 1; seg >= 0; seg--) {
    uint32_t b = uint32_t(seg) * kThreads + tid;
    vals[tid] = b < nblocks ? ld_fe(bv + uint64_t(b) * 4) : fe_zero();
    mul[tid] = b < nblocks ? ld_fe(bm + uint64_t(b) * 4) : fe_one();
    if (tid == 0) {
      vals[kThreads] = fe_zero();
      mul[kThreads] = fe_one();
    }
    __syncthreads();
    for (uint32_t off = 1; off < kThreads; off <<= 1) {
      FpExt v = vals[tid], m = mul[tid];
      if (tid + off < kThreads) {
        v = fe_add(v, fe_mul(m, vals[tid + off]));
        m = fe_mul(m, mul[tid + off]);
      }
      __syncthreads();
      vals[tid] = v;
      mul[tid] = m;
      __syncthreads();
    }
    FpExt cin = fe_add(vals[tid + 1], fe_mul(mul[tid + 1], carry));
    FpExt total = fe_add(vals[0], fe_mul(mul[0], carry));
    __syncthreads();
    if (b < nblocks) st_fe(bv + uint64_t(b) * 4, cin);
    carry = total;
  }
  if (tid == 0) st_fe(rows[row].rem, carry);
}

__global__ __launch_bounds__(kThreads) void div_apply_kernel(const DivRow* rows, uint32_t nlanes, const uint32_t* lanev,
                                                            const uint32_t* lanem, const uint32_t* blockv) {
  const DivRow r = rows[blockIdx.y];
  const uint32_t lane = blockIdx.x * kThreads + threadIdx.x;
  if (lane >= nlanes) return;
  const uint64_t li = uint64_t(blockIdx.y) * nlanes + lane;
  FpExt bc = ld_fe(blockv + (uint64_t(blockIdx.y) * gridDim.x + blockIdx.x) * 4);
  FpExt cur = fe_add(ld_fe(lanev + li * 4), fe_mul(ld_fe(lanem + li * 4), bc));
  uint32_t* p = r.p + uint64_t(lane) * kDivPer * 4;
#pragma unroll
  for (int i = kDivPer - 1; i >= 0; i--) {
    FpExt pi = ld_fe(p + 4 * i);
    st_fe(p + 4 * i, cur);
    cur = fe_add(fe_mul(r.z, cur), pi);
  }
}

// rows whose length is not a multiple of 16: one lane per row, serial
__global__ void div_serial_kernel(const DivRow* rows, uint64_t n, uint32_t nrows) {
  uint32_t row = blockIdx.x * kThreads + threadIdx.x;
  if (row >= nrows) return;
  const DivRow r = rows[row];
  FpExt cur = fe_zero();
  for (uint64_t i = n; i-- > 0;) {
    FpExt pi = ld_fe(r.p + 4 * i);
    st_fe(r.p + 4 * i, cur);
    cur = fe_add(fe_mul(r.z, cur), pi);
  }
  st_fe(r.rem, cur);
}

// combos_prepare tail (hal/mod.rs:212-233): combos[r*cycles + i] -= deltas[r*width + i]
__global__ void combos_sub_kernel(uint32_t* combos, const uint32_t* deltas, uint32_t rows, uint32_t width,
                                  uint64_t cycles) {
  uint32_t t = blockIdx.x * kThreads + threadIdx.x;
  if (t >= rows * width) return;
  uint32_t r = t / width, i = t % width;
  if (i >= cycles) return;
  uint32_t* p = combos + (uint64_t(r) * cycles + i) * 4;
  st_fe(p, fe_sub(ld_fe(p), ld_fe(deltas + uint64_t(t) * 4)));
}

// Query openings: dst[i] = bases[base_id[i]][offsets[i]]
__global__ void gather_words_kernel(uint32_t* dst, const uint32_t* const* bases, const uint32_t* base_id,
                                    const uint64_t* offsets, uint64_t n) {
  uint64_t i = uint64_t(blockIdx.x) * kThreads + threadIdx.x;
  if (i < n) dst[i] = bases[base_id[i]][offsets[i]];
}

}  // namespace

void eltwise_add(hipStream_t s, uint32_t* out, const uint32_t* a, const uint32_t* b, size_t n) {
  if (!n) return;
  hipLaunchKernelGGL(add_kernel, dim3(grid_stride(n, kThreads)), dim3(kThreads), 0, s, out, a, b, uint64_t(n));
  HIP_OK(hipGetLastError());
}
void eltwise_copy(hipStream_t s, uint32_t* out, const uint32_t* in, size_t n) {
  if (!n || out == in) return;
  HIP_OK(hipMemcpyAsync(out, in, n * 4, hipMemcpyDeviceToDevice, s));
}
void eltwise_zeroize(hipStream_t s, uint32_t* io, size_t n) {
  if (!n) return;
  hipLaunchKernelGGL(zeroize_kernel, dim3(grid_stride(n, kThreads)), dim3(kThreads), 0, s, io, uint64_t(n));
  HIP_OK(hipGetLastError());
}
void fill_uniform(hipStream_t s, uint32_t* out, size_t n, uint64_t seed) {
  if (!n) return;
  hipLaunchKernelGGL(fill_uniform_kernel, dim3(grid_stride(n, kThreads)), dim3(kThreads), 0, s, out, uint64_t(n), seed);
  HIP_OK(hipGetLastError());
}
void eltwise_sum_extelem(hipStream_t s, uint32_t* out, const uint32_t* in, size_t count, size_t to_add) {
  if (!count) return;
  KScope ks("eltwise_sum_extelem", double(count) * 16 * (to_add + 1));
  hipLaunchKernelGGL(sum_extelem_kernel, dim3(div_up(count, kThreads)), dim3(kThreads), 0, s, out, in,
                     uint64_t(count), uint32_t(to_add));
  HIP_OK(hipGetLastError());
}
void fri_fold(hipStream_t s, uint32_t* out, const uint32_t* in, FpExt mix, size_t count) {
  if (!count) return;
  KScope ks("fri_fold", double(count) * (16 * 16 + 16));
  hipLaunchKernelGGL(fri_fold_kernel, dim3(div_up(count, kThreads)), dim3(kThreads), 0, s, out, in, mix,
                     uint64_t(count));
  HIP_OK(hipGetLastError());
}
void gather_sample(hipStream_t s, uint32_t* dst, const uint32_t* src, size_t idx, size_t size, size_t stride) {
  if (!size) return;
  hipLaunchKernelGGL(gather_kernel, dim3(div_up(size, kThreads)), dim3(kThreads), 0, s, dst, src, uint64_t(idx),
                     uint64_t(size), uint64_t(stride));
  HIP_OK(hipGetLastError());
}
void scatter(hipStream_t s, uint32_t* into, const uint32_t* index, const uint32_t* offsets, const uint32_t* values,
             size_t cycles, uint64_t limit) {
  if (!cycles) return;
  hipLaunchKernelGGL(scatter_kernel, dim3(div_up(cycles, kThreads)), dim3(kThreads), 0, s, into, index, offsets,
                     values, uint64_t(cycles), limit);
  HIP_OK(hipGetLastError());
}
void copy_elem_slice(hipStream_t s, uint32_t* into, const uint32_t* from, size_t rows, size_t cols,
                     size_t from_offset, size_t from_stride, size_t into_offset, size_t into_stride) {
  if (!rows || !cols) return;
  hipLaunchKernelGGL(copy_slice_kernel, dim3(grid_stride(rows * cols, kThreads)), dim3(kThreads), 0, s, into, from,
                     uint64_t(rows), uint64_t(cols), uint64_t(from_offset), uint64_t(from_stride),
                     uint64_t(into_offset), uint64_t(into_stride));
  HIP_OK(hipGetLastError());
}
void prefix_products(hipStream_t s, uint32_t* io, size_t n) {
  if (n < 2) return;
  hipLaunchKernelGGL(prefix_products_kernel, dim3(1), dim3(64), 0, s, io, uint64_t(n));
  HIP_OK(hipGetLastError());
}

void mix_poly_coeffs(hipStream_t s, uint32_t* out, const uint32_t* in, const uint32_t* combos_dev,
                     const std::vector<uint32_t>& combos_host, FpExt mix_start, FpExt mix, size_t input_size,
                     size_t count) {
  if (!count || !input_size) return;
  uint32_t used = 0, maxc = 0;
  for (uint32_t c : combos_host) used |= 1u << (c & 31);
  KScope ks("mix_poly_coeffs", double(count) * (input_size * 4 + 32.0 * __builtin_popcount(used)));
  used = 0;
  for (uint32_t c : combos_host) {
    R0_REQUIRE(c < 32, "mix_poly_coeffs: combo id too large");
    used |= 1u << c;
    maxc = std::max(maxc, c);
  }
  // rows sorted by combo id (stable), their mix powers mix_start * mix^i in that order
  std::vector<uint32_t> rows, pows, seg{0}, seg_combo;
  std::vector<FpExt> pw(input_size);
  FpExt cur = mix_start;
  for (size_t i = 0; i < input_size; i++) {
    pw[i] = cur;
    cur = fe_mul(cur, mix);
  }
  for (uint32_t k = 0; k <= maxc; k++) {
    if (!(used >> k & 1)) continue;
    for (size_t i = 0; i < input_size; i++) {
      if (combos_host[i] != k) continue;
      rows.push_back(uint32_t(i));
      for (int w = 0; w < 4; w++) pows.push_back(pw[i].c[w]);
    }
    seg.push_back(uint32_t(rows.size()));
    seg_combo.push_back(k);
  }
  (void)combos_dev;  // the device copy of the ids is the ABI's; the sorted tables replace it
  uint32_t* d_rows = static_cast<uint32_t*>(scratch(rows.size() * 4, kSlotMixRows));
  uint32_t* d_pows = static_cast<uint32_t*>(scratch(pows.size() * 4, kSlotMixPows));
  uint32_t* d_seg = static_cast<uint32_t*>(scratch(seg.size() * 4, kSlotMixSeg));
  uint32_t* d_seg_combo = static_cast<uint32_t*>(scratch(seg_combo.size() * 4, kSlotMixSegCombo));
  upload_async(d_rows, rows.data(), rows.size() * 4);
  upload_async(d_pows, pows.data(), pows.size() * 4);
  upload_async(d_seg, seg.data(), seg.size() * 4);
  upload_async(d_seg_combo, seg_combo.data(), seg_combo.size() * 4);
  hipLaunchKernelGGL(mix_kernel, dim3(div_up(count, kThreads)), dim3(kThreads), 0, s, out, in, d_rows, d_pows,
                     d_seg, d_seg_combo, uint32_t(seg_combo.size()), uint64_t(count));
  HIP_OK(hipGetLastError());
}

void batch_evaluate_any_host(hipStream_t s, const uint32_t* coeffs, size_t poly_count, uint32_t log_n,
                             const std::vector<uint32_t>& which, const uint32_t* xs, uint32_t* out, bool bitrev) {
  const size_t eval_count = which.size();
  if (!eval_count) return;
  R0_REQUIRE(!bitrev || log_n >= kEvalBitrevMinLog, "batch_evaluate_any: bit-reversed rows need log_n >= 12");
  const uint64_t n = uint64_t(1) << log_n;
  const uint32_t nchunks = uint32_t((n + kEvChunk - 1) / kEvChunk);
  const uint32_t npieces = nchunks * (kThreads / 64);  // 4096-coefficient pieces, one per wave
  // group evaluations by polynomial
  std::map<uint32_t, std::vector<uint32_t>> groups;
  for (size_t k = 0; k < eval_count; k++) {
    R0_REQUIRE(which[k] < poly_count, "batch_evaluate_any: which out of range");
    groups[which[k]].push_back(uint32_t(k));
  }
  std::vector<uint32_t> gpoly, gbegin{0}, geval;
  for (auto& kv : groups) {
    gpoly.push_back(kv.first);
    geval.insert(geval.end(), kv.second.begin(), kv.second.end());
    gbegin.push_back(uint32_t(geval.size()));
  }
  // one read of each evaluated polynomial; per coefficient and evaluation 4 products
  KScope ks("batch_evaluate_any", double(groups.size()) * n * 4, double(eval_count) * n * 4);
  R0_REQUIRE(groups.size() < 65536, "batch_evaluate_any: too many polynomials");
  uint32_t* d_gpoly = static_cast<uint32_t*>(scratch(gpoly.size() * 4, kSlotEvalPoly));
  uint32_t* d_gbegin = static_cast<uint32_t*>(scratch(gbegin.size() * 4, kSlotEvalBegin));
  uint32_t* d_geval = static_cast<uint32_t*>(scratch(geval.size() * 4, kSlotEvalIdx));
  upload_async(d_gpoly, gpoly.data(), gpoly.size() * 4);
  upload_async(d_gbegin, gbegin.data(), gbegin.size() * 4);
  upload_async(d_geval, geval.data(), geval.size() * 4);
  uint32_t* tab = static_cast<uint32_t*>(scratch(eval_count * kEvTab * 16, kSlotEvalTable));
  uint32_t* partial = static_cast<uint32_t*>(scratch(eval_count * npieces * 16, kSlotEvalPartial));
  hipLaunchKernelGGL(eval_tables_kernel, dim3(div_up(eval_count * kEvTab, kThreads)), dim3(kThreads), 0, s, xs,
                     uint32_t(eval_count), tab, log_n, bitrev);
  HIP_OK(hipGetLastError());
  hipLaunchKernelGGL(eval_chunk_kernel, dim3(nchunks, unsigned(groups.size())), dim3(kThreads), 0, s, coeffs, n,
                     d_gpoly, d_gbegin, d_geval, tab, partial, npieces);
  HIP_OK(hipGetLastError());
  hipLaunchKernelGGL(eval_any_reduce, dim3(div_up(eval_count, kThreads / 64)), dim3(kThreads), 0, s, partial, npieces,
                     tab, out, uint32_t(eval_count), xs, log_n, bitrev);
  HIP_OK(hipGetLastError());
}

void batch_evaluate_any(hipStream_t s, const uint32_t* coeffs, size_t poly_count, uint32_t log_n,
                        const uint32_t* which, const uint32_t* xs, uint32_t* out, size_t eval_count) {
  if (!eval_count) return;
  std::vector<uint32_t> h(eval_count);
  HIP_OK(hipMemcpyAsync(h.data(), which, eval_count * 4, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  batch_evaluate_any_host(s, coeffs, poly_count, log_n, h, xs, out);
}

void poly_divide_rows(hipStream_t s, uint32_t* io, size_t n, const std::vector<std::vector<FpExt>>& zs,
                      uint32_t* rem_dev) {
  size_t rows = zs.size();
  size_t maxz = 0;
  for (auto& v : zs) maxz = std::max(maxz, v.size());
  if (!rows || !maxz || !n) return;
  size_t ndiv = 0;
  for (auto& v : zs) ndiv += v.size();
  KScope ks("poly_divide", double(ndiv) * n * 32);
  // round k divides every row that has a k-th z (the rows' z lists run in order)
  for (size_t k = 0; k < maxz; k++) {
    // each row's remainder goes straight to its place in rem_dev (row-major, maxz per row)
    std::vector<DivRow> rs;
    for (size_t r = 0; r < rows; r++)
      if (k < zs[r].size()) rs.push_back(DivRow{io + uint64_t(r) * n * 4, zs[r][k], rem_dev + (uint64_t(r) * maxz + k) * 4});
    uint32_t nr = uint32_t(rs.size());
    DivRow* drows = static_cast<DivRow*>(scratch(rs.size() * sizeof(DivRow), k % 2 ? kSlotDivRowsAlt : kSlotDivRows));
    upload_async(drows, rs.data(), rs.size() * sizeof(DivRow));
    if (n % kDivPer != 0) {
      hipLaunchKernelGGL(div_serial_kernel, dim3(div_up(nr, kThreads)), dim3(kThreads), 0, s, drows, uint64_t(n), nr);
      HIP_OK(hipGetLastError());
    } else {
      uint32_t nlanes = uint32_t(n / kDivPer);
      uint32_t nblocks = div_up(nlanes, kThreads);
      uint32_t* lanev = static_cast<uint32_t*>(scratch(size_t(nr) * nlanes * 16, kSlotDivLaneV));
      uint32_t* lanem = static_cast<uint32_t*>(scratch(size_t(nr) * nlanes * 16, kSlotDivLaneM));
      uint32_t* blockv = static_cast<uint32_t*>(scratch(size_t(nr) * nblocks * 16, kSlotDivBlockV));
      uint32_t* blockm = static_cast<uint32_t*>(scratch(size_t(nr) * nblocks * 16, kSlotDivBlockM));
      hipLaunchKernelGGL(div_local_kernel, dim3(nblocks, nr), dim3(kThreads), 0, s, drows, nlanes, lanev);
      HIP_OK(hipGetLastError());
      hipLaunchKernelGGL(div_block_kernel, dim3(nblocks, nr), dim3(kThreads), 0, s, drows, nlanes, lanev, lanem,
                         blockv, blockm);
      HIP_OK(hipGetLastError());
      hipLaunchKernelGGL(div_top_kernel, dim3(nr), dim3(kThreads), 0, s, drows, nblocks, blockv, blockm);
      HIP_OK(hipGetLastError());
      hipLaunchKernelGGL(div_apply_kernel, dim3(nblocks, nr), dim3(kThreads), 0, s, drows, nlanes, lanev, lanem,
                         blockv);
      HIP_OK(hipGetLastError());
    }
  }
}

void combos_sub(hipStream_t s, uint32_t* combos, const uint32_t* deltas, size_t rows, size_t width,
                size_t cycles) {
  if (!rows || !width) return;
  hipLaunchKernelGGL(combos_sub_kernel, dim3(div_up(rows * width, kThreads)), dim3(kThreads), 0, s, combos, deltas,
                     uint32_t(rows), uint32_t(width), uint64_t(cycles));
  HIP_OK(hipGetLastError());
}

void gather_words(hipStream_t s, uint32_t* dst, const uint32_t* const* bases, const uint32_t* base_id,
                  const uint64_t* offsets, size_t n) {
  if (!n) return;
  hipLaunchKernelGGL(gather_words_kernel, dim3(div_up(n, kThreads)), dim3(kThreads), 0, s, dst, bases, base_id,
                     offsets, uint64_t(n));
  HIP_OK(hipGetLastError());
}

}  // namespace r0
