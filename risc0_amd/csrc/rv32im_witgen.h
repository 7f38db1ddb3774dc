// Shared by the generated rv32im witness-generation kernels (tools/gen_rv32im_witgen.py ->
// gen/rvwitgen/*.hip) and their driver (rv32im_witgen.hip): the preflight records, the
// argument block, the reference's checked buffers and its externs on the device
// (rv32im-sys/kernels/cxx/ffi.cpp:84-228, buffers.h, tables.h).
#pragma once
#include "bb31.h"
#include "runtime.h"

namespace r0 {
namespace rvwg {

constexpr uint32_t kThreads = 256;  // po2 20 loop guest: 0.78 -> 0.64 ms vs 128 (profiles/r4thr_witgen_threads_ab.txt)
constexpr uint32_t kInvalid = 0xFFFFFFFFu;  // Fp::invalid()
constexpr uint32_t kMajors = 13;            // Top's instruction mux (majorOnehot)
constexpr uint32_t kDataCols = 211;         // the rv32im data group (REGCOUNT_DATA)
constexpr uint32_t kNoSlot = 0x3FFF, kInjectedCol = 0x4000;  // rv32im_witgen_slot_table() entries

// rv32im-sys/kernels/cxx/preflight.h:21-41 (RawPreflightCycle / RawMemoryTransaction)
struct PreflightCycle {
  uint32_t state;
  uint32_t pc;
  uint8_t major;
  uint8_t minor;
  uint8_t machine_mode;
  uint8_t padding;
  uint32_t user_cycle;
  uint32_t txn_idx;
  uint32_t paging_idx;
  uint32_t bigint_idx;
  uint32_t diff_count[2];
};
static_assert(sizeof(PreflightCycle) == 36, "RawPreflightCycle layout");

struct MemoryTxn {
  uint32_t addr;
  uint32_t cycle;
  uint32_t word;
  uint32_t prev_cycle;
  uint32_t prev_word;
};
static_assert(sizeof(MemoryTxn) == 20, "RawMemoryTransaction layout");

// error codes (err[0]); err[1] is the cycle, err[2] a detail (column, index)
constexpr uint32_t kErrEqz = 0x10000u;  // + the EQZ message index (gen/rvwitgen messages)
constexpr uint32_t kErrUnset = 0x20001u;         // checked read of Fp::invalid() (buffers.h:45-52)
constexpr uint32_t kErrInconsistent = 0x20002u;  // checked set of another value (buffers.h:30-43)
constexpr uint32_t kErrUnreachable = 0x20003u;   // "Reached unreachable mux arm"
constexpr uint32_t kErrTxnCycle = 0x20004u;      // ffi.cpp:96-99
constexpr uint32_t kErrTxnAddr = 0x20005u;       // ffi.cpp:101-104
constexpr uint32_t kErrTxnRange = 0x20006u;      // a transaction past the trace's
constexpr uint32_t kErrLookupTable = 0x20007u;   // tables.h:40-42, 57-59
constexpr uint32_t kErrLookupIndex = 0x20008u;   // tables.h:43-46
constexpr uint32_t kErrBigint = 0x20009u;        // bigIntExtern past the trace's bytes
constexpr uint32_t kErrDiffCount = 0x2000Au;     // getDiffCount past the trace's cycles
constexpr uint32_t kErrMajor = 0x2000Bu;         // a cycle's major outside the 13 instruction arms
// an injector entry of row r whose offset lies in another row (the reference's Injector::set
// writes only its own row, witgen/mod.rs:352-377; the init pass writes a row per lane)
constexpr uint32_t kErrInjectorRow = 0x2000Cu;

struct Args {
  uint32_t* data;    // DATA x rows, column-major (MutableBufObj over Buffer<checked>)
  uint32_t* global;  // the global vector (GlobalBufObj over Buffer<checked>)
  uint32_t rows;     // a power of two
  uint32_t ncycles;  // preflight cycles (lastCycle)
  const PreflightCycle* cycles;
  const MemoryTxn* txns;
  uint32_t n_txns;
  const uint8_t* bigint;
  uint32_t n_bigint;
  uint32_t* u8;   // LookupTables::tableU8 (256 counters)
  uint32_t* u16;  // LookupTables::tableU16 (65536 counters)
  uint32_t* err;  // [code, cycle, detail]
};

// Fp::asUInt32 / Fp(uint32_t)
__device__ __forceinline__ uint32_t to_u32(uint32_t x) { return mont_reduce(x); }
__device__ __forceinline__ uint32_t from_u32(uint32_t v) { return fp_mul(v % kP, kR2); }

__device__ __forceinline__ void fail(const Args& A, uint32_t code, uint32_t cycle, uint32_t detail = 0) {
  if (atomicCAS(A.err, 0u, code) == 0u) {
    A.err[1] = cycle;
    A.err[2] = detail;
  }
}

// A lane's first failed check, in program order, kept in two registers without a branch;
// the kernel reports it once, at its end (fail). The reference throws at the first failure;
// later values of a failed cycle are garbage here, but the call fails with that first error.
struct Err {
  uint32_t code, detail;
  bool pin;  // a per-kernel constant (see note)
};
__device__ __forceinline__ void note(Err& e, bool bad, uint32_t code, uint32_t detail = 0u) {
  const bool first = bad && e.code == 0u;
  e.code = first ? code : e.code;
  e.detail = first ? detail : e.detail;
  // pin: both selects stay at this point. Unpinned, the scheduler sinks every `detail` select
  // to the kernel's end (nothing reads it earlier) and keeps each check's 64-bit lane mask live
  // until then: SGPR spills into VGPR lanes, 188 instead of 76 VGPRs for arm 4, 2.5 KB of
  // scratch per lane for the SHA-256 arm. Pinned, the other arms lose their freedom to hoist
  // loads and run slower (tools/gen_rv32im_witgen.py PIN_NOTES, profiles/r4s_*).
  if (e.pin) asm volatile("" : "+v"(e.code), "+v"(e.detail));
}

// Buffer::get with checked = true. `view` is A.data, or for the injected columns a read-only
// alias the generated kernels declare __restrict__ (see tools/gen_rv32im_witgen.py, Path)
__device__ __forceinline__ uint32_t ld(const Args& A, Err& err, const uint32_t* view, uint32_t col, uint32_t row,
                                       uint32_t cycle) {
  const uint32_t v = view[uint64_t(col) * A.rows + row];
  note(err, v == kInvalid, kErrUnset, col);
  return v;
}

// A load of an injected cell again, near a far use of its first (checked) load: the opaque row
// keeps the compiler from merging the two, so the value need not stay live in between
__device__ __forceinline__ uint32_t reld(const Args& A, const uint32_t* view, uint32_t col, uint32_t row) {
  asm volatile("" : "+v"(row));
  return view[uint64_t(col) * A.rows + row];
}

// The arm kernels keep this cycle's own row values in a compact, slot-major buffer of their
// bin (cb[slot * n + i], lane i = the cycle's place in the bin's list: one coalesced store per
// column for a wavefront), with a bit per slot in the lane's mask words sm0.. (stored after the
// slots, cb[(nslots + w) * n + i]): a slot is read only if its bit is set, so the buffer needs
// no INVALID fill. rv32im_witgen.hip's merge writes the values into the column-major data
// group afterwards, whole lines at a time. (Writing the data group from the arm kernels
// directly cost ≈3.7 GB of partial-line writes per po2=20 segment: a line of a column holds
// 32 consecutive cycles of every arm.)
//
// a store whose cell the generator knows to be INVALID (set by no injector and by no earlier
// store of this cycle): the checked set cannot fail
__device__ __forceinline__ void stc(uint32_t* cb, uint32_t n, uint32_t i, uint32_t slot, uint32_t v, uint32_t& smw,
                                    uint32_t bit) {
  cb[size_t(slot) * n + i] = v;
  smw |= bit;
}

// the row's value of a column stored earlier on some path of this cycle: its slot (checked get)
__device__ __forceinline__ uint32_t ldc(const Args& A, Err& err, const uint32_t* cb, uint32_t n, uint32_t i,
                                        uint32_t slot, uint32_t col, uint32_t cycle, uint32_t smw, uint32_t bit) {
  const uint32_t v = (smw & bit) ? cb[size_t(slot) * n + i] : kInvalid;
  note(err, v == kInvalid, kErrUnset, col);
  return v;
}

// checked set of an injected column: the old value is the injector's (data, read-only view)
__device__ __forceinline__ void st_inj(const Args& A, Err& err, const uint32_t* view, uint32_t* cb, uint32_t n,
                                       uint32_t i, uint32_t slot, uint32_t col, uint32_t cycle, uint32_t v,
                                       uint32_t& smw, uint32_t bit) {
  const uint32_t old = view[uint64_t(col) * A.rows + cycle];
  note(err, old != kInvalid && old != v, kErrInconsistent, col);
  cb[size_t(slot) * n + i] = v;
  smw |= bit;
}

// checked set of a column some earlier path of this cycle may have stored
__device__ __forceinline__ void st_maybe(const Args& A, Err& err, uint32_t* cb, uint32_t n, uint32_t i, uint32_t slot,
                                         uint32_t col, uint32_t cycle, uint32_t v, uint32_t& smw, uint32_t bit) {
  uint32_t* p = cb + size_t(slot) * n + i;
  const uint32_t old = (smw & bit) ? *p : kInvalid;
  note(err, old != kInvalid && old != v, kErrInconsistent, col);
  *p = v;
  smw |= bit;
}

__device__ __forceinline__ uint32_t gld(const Args& A, Err& err, uint32_t idx, uint32_t cycle) {
  const uint32_t v = A.global[idx];
  note(err, v == kInvalid, kErrUnset, 0x10000u + idx);
  return v;
}

__device__ __forceinline__ void gst(const Args& A, Err& err, uint32_t idx, uint32_t cycle, uint32_t v) {
  const uint32_t old = A.global[idx];
  note(err, old != kInvalid && old != v, kErrInconsistent, 0x10000u + idx);
  A.global[idx] = v;
}

// extern_getMemoryTxn (ffi.cpp:84-113): the cycle's next transaction. A.txns always holds at
// least one record (rv32im_witgen_dev points it at a zero record when the trace has none), so
// a cursor past the end reads record 0 and reports the overrun.
__device__ __forceinline__ void txn(const Args& A, Err& err, const MemoryTxn* txs, uint32_t cycle, uint32_t& cur,
                                    uint32_t addr_w, uint32_t& prev_cycle, uint32_t& prev_lo, uint32_t& prev_hi,
                                    uint32_t& lo, uint32_t& hi) {
  const bool oob = cur >= A.n_txns;
  note(err, oob, kErrTxnRange, cur);
  const MemoryTxn t = txs[oob ? 0u : cur];
  cur++;
  note(err, t.cycle / 2 != cycle, kErrTxnCycle, t.cycle);
  note(err, t.addr != to_u32(addr_w), kErrTxnAddr, t.addr);
  prev_cycle = from_u32(t.prev_cycle);
  prev_lo = from_u32(t.prev_word & 0xFFFFu);
  prev_hi = from_u32(t.prev_word >> 16);
  lo = from_u32(t.word & 0xFFFFu);
  hi = from_u32(t.word >> 16);
}

// extern_hostReadPrepare / extern_hostWrite (ffi.cpp:201-212): the word of the cycle's next
// transaction, without advancing
__device__ __forceinline__ uint32_t host_word(const Args& A, Err& err, const MemoryTxn* txs, uint32_t cycle,
                                              uint32_t cur) {
  const bool oob = cur >= A.n_txns;
  note(err, oob, kErrTxnRange, cur);
  return from_u32(txs[oob ? 0u : cur].word);
}

// The workgroup's lookup counts in LDS, added to the device tables once at the kernel's end:
// the u8 table whole (256 counters), the u16 table through a small open-addressing table of
// (index, count) slots. A few u16 indices take most lookups (index 0: 43% of the shift/divide
// arm's 19 lookups per cycle on the bench guest), and device atomics on one address serialise
// (≈14 ns each), so the counts are summed per workgroup first; an index that finds no slot
// within kU16Probe probes goes to the device table directly.
constexpr uint32_t kU16Slots = 1024, kU16Probe = 4, kEmpty = 0xFFFFFFFFu;
struct LdsTables {
  uint32_t* h8;    // [256]
  uint32_t* keys;  // [kU16Slots], kEmpty when free
  uint32_t* cnt;   // [kU16Slots]
};

__device__ __forceinline__ void lds_tables_init(const LdsTables& T) {
  for (uint32_t t = threadIdx.x; t < 256u; t += kThreads) T.h8[t] = 0u;
  for (uint32_t t = threadIdx.x; t < kU16Slots; t += kThreads) {
    T.keys[t] = kEmpty;
    T.cnt[t] = 0u;
  }
  __syncthreads();
}

__device__ __forceinline__ void lds_tables_flush(const Args& A, const LdsTables& T) {
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < 256u; t += kThreads)
    if (T.h8[t]) atomicAdd(A.u8 + t, T.h8[t]);
  for (uint32_t t = threadIdx.x; t < kU16Slots; t += kThreads)
    if (T.keys[t] != kEmpty) atomicAdd(A.u16 + T.keys[t], T.cnt[t]);
}

__device__ __forceinline__ void u16_count(const Args& A, const LdsTables& T, uint32_t index) {
  const uint32_t h = (index * 2654435761u) >> 22;  // 10-bit multiplicative hash
#pragma unroll
  for (uint32_t p = 0; p < kU16Probe; p++) {
    const uint32_t slot = (h + p) & (kU16Slots - 1);
    const uint32_t k = atomicCAS(T.keys + slot, kEmpty, index);
    if (k == kEmpty || k == index) {
      atomicAdd(T.cnt + slot, 1u);
      return;
    }
  }
  atomicAdd(A.u16 + index, 1u);
}

// LookupTables::lookupDelta (tables.h:33-53; the count argument is not used there either)
__device__ __forceinline__ void lookup_delta(const Args& A, Err& err, uint32_t cycle, uint32_t table_w,
                                             uint32_t index_w, const LdsTables& T) {
  const uint32_t table = to_u32(table_w), index = to_u32(index_w);
  if (table == 0u) return;
  const bool bad_t = table != 8u && table != 16u;
  const bool bad_i = !bad_t && index >= (1u << table);
  note(err, bad_t, kErrLookupTable, table);
  note(err, bad_i, kErrLookupIndex, index);
  if (bad_t || bad_i) return;
  if (table == 8u)
    atomicAdd(T.h8 + index, 1u);
  else
    u16_count(A, T, index);
}

// LookupTables::lookupCurrent (tables.h:55-66)
__device__ __forceinline__ uint32_t lookup_current(const Args& A, Err& err, uint32_t cycle, uint32_t table_w,
                                                   uint32_t index_w) {
  const uint32_t table = to_u32(table_w), index = to_u32(index_w);
  const bool bad_t = table != 8u && table != 16u;
  const bool bad_i = !bad_t && index >= (1u << table);
  note(err, bad_t, kErrLookupTable, index);
  note(err, bad_i, kErrLookupIndex, index);
  const uint32_t* tab = table == 8u ? A.u8 : A.u16;
  return from_u32(__hip_atomic_load(tab + (bad_t || bad_i ? 0u : index), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// extern_getDiffCount (ffi.cpp:141-145)
__device__ __forceinline__ uint32_t diff_count(const Args& A, Err& err, uint32_t cycle, uint32_t c_w) {
  const uint32_t c = to_u32(c_w);
  const bool bad = c / 2 >= A.ncycles;
  note(err, bad, kErrDiffCount, c);
  return from_u32(A.cycles[bad ? 0u : c / 2].diff_count[c % 2]);
}

// divide_rv32im + extern_divide (ffi.cpp:54-82, 177-188)
__device__ __forceinline__ void divide(uint32_t nl, uint32_t nh, uint32_t dl, uint32_t dh, uint32_t sign_w, uint32_t& q0,
                                       uint32_t& q1, uint32_t& r0, uint32_t& r1) {
  uint32_t numer = to_u32(nl) | (to_u32(nh) << 16);
  uint32_t denom = to_u32(dl) | (to_u32(dh) << 16);
  const uint32_t sign = to_u32(sign_w);
  const uint32_t ones = sign == 2u;
  const bool neg_n = sign && int32_t(numer) < 0;
  const bool neg_d = sign == 1u && int32_t(denom) < 0;
  if (neg_n) numer = -numer - ones;
  if (neg_d) denom = -denom - ones;
  uint32_t quot, rem;
  if (denom == 0u) {
    quot = 0xFFFFFFFFu;
    rem = numer;
  } else {
    quot = numer / denom;
    rem = numer % denom;
  }
  const uint32_t qneg = uint32_t(neg_n ^ neg_d) - uint32_t(denom == 0u) * uint32_t(neg_n);
  if (qneg) quot = -quot - ones;
  if (neg_n) rem = -rem - ones;
  q0 = from_u32(quot & 0xFFFFu);
  q1 = from_u32(quot >> 16);
  r0 = from_u32(rem & 0xFFFFu);
  r1 = from_u32(rem >> 16);
}

// extern_bigIntExtern (ffi.cpp:221-228); A.bigint always holds at least one byte (as A.txns)
__device__ __forceinline__ uint32_t bigint_byte(const Args& A, Err& err, uint32_t cycle, uint32_t i) {
  const uint32_t k = A.cycles[cycle].bigint_idx + i;
  const bool bad = k >= A.n_bigint;
  note(err, bad, kErrBigint, k);
  return from_u32(A.bigint[bad ? 0u : k]);
}

}  // namespace rvwg

// the generated kernels: step_Top specialised to instruction arm `major` over a list of cycles
void rv32im_witgen_major(uint32_t major, hipStream_t s, const rvwg::Args& A, const uint32_t* list, uint32_t n,
                         uint32_t* cb);
// each arm's compact slot of every data column ([13][211]: low 14 bits the slot, kNoSlot if the
// arm never stores the column; kInjectedCol if the injector sets it on the arm's rows) and the
// arms' slot counts
const int16_t* rv32im_witgen_slot_table();
uint32_t rv32im_witgen_nslots(uint32_t major);
// EQZ messages of the generated code (steps.cpp locations), by index
const char* rv32im_witgen_message(uint32_t k);
// the driver (rv32im_witgen.hip): both phases over cycles [0, last_cycle) with the preflight
// arrays resident on the device; synchronises, throws on a failed check
// zeroize (the prover's path): the data group is the prover's own, INVALID in the injected
// columns but the injector's words (rv32im_prover_groups_fill + rv32im_prover_inject; its other
// words are never read), and the merge writes 0 for INVALID words (eltwise_zeroize fused, as
// hal_generate_witness does right after stepExec, witgen/mod.rs:166-169). extra_err: the inject
// pass's record (4 words): a failure there is raised; word 3 set (an entry outside its row's
// injected columns) calls reinit, which must leave the group as the reference prepares it (all
// INVALID, the injector scattered in), and the merge then reads every column back.
void rv32im_witgen_dev(hipStream_t s, uint32_t mode, uint32_t* data, uint32_t* global, size_t rows,
                       const rvwg::PreflightCycle* d_cycles, const rvwg::MemoryTxn* d_txns, size_t n_txns,
                       const uint8_t* d_bigint, size_t n_bigint, uint32_t table_split, uint32_t last_cycle,
                       bool zeroize = false, const uint32_t* extra_err = nullptr,
                       const std::function<void()>& reinit = {});
// The prover's groups before witness generation (replacing the INVALID fills of
// WitnessGenerator::new and ::accum, witgen/mod.rs:135-170, 178-186, and the injector's scatter).
// fill, one pass over the rows with no input (queued before the trace lands): data INVALID in
// the injected columns — the only ones any arm or the prover-mode merge reads back (every other
// data word is written by the merge) —; code 0; accum INVALID in the machine columns the
// accumulation's phase 3 adds to, 0 elsewhere: its zeroize then has nothing left to change
// (AccumStep::zeroed; every row is stepped).
void rv32im_prover_groups_fill(hipStream_t s, uint32_t* data, uint32_t* code, uint32_t* accum, size_t rows,
                               size_t accum_cols);
// inject: the injector's entries (offsets at or past `limit` skipped, reads clamped to
// index[inj_rows]), one lane per row; an entry in another row records kErrInjectorRow in err, an
// entry in a column its row's arm (the cycle's major) does not take from the injector sets err[3]
// (err: 4 words, zeroed by the caller; rv32im_witgen_dev's extra_err).
void rv32im_prover_inject(hipStream_t s, uint32_t* data, size_t rows, const uint32_t* index, const uint32_t* offsets,
                          const uint32_t* values, size_t inj_rows, uint64_t limit, const rvwg::PreflightCycle* d_cycles,
                          uint32_t* err);
// the same from host preflight arrays (uploaded first), as RawPreflightTrace hands them over
void rv32im_witgen(hipStream_t s, uint32_t mode, uint32_t* data, uint32_t* global, size_t rows,
                   const rvwg::PreflightCycle* h_cycles, const rvwg::MemoryTxn* h_txns, size_t n_txns,
                   const uint8_t* h_bigint, size_t n_bigint, uint32_t table_split, uint32_t last_cycle,
                   bool zeroize = false, const uint32_t* extra_err = nullptr,
                   const std::function<void()>& reinit = {});
// the host preflight cycles uploaded into this thread's witgen scratch (what rv32im_witgen does
// first), for callers that need them on the device before witness generation
const rvwg::PreflightCycle* rv32im_upload_cycles(const rvwg::PreflightCycle* h_cycles, size_t n);

}  // namespace r0
