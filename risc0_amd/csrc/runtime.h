// Host-side runtime shared by the C ABI (api.cpp), the segment prover
// (prover.cpp) and the kernel launchers: error plumbing, the per-process HIP
// stream, cached constant tables in HBM, and the launcher declarations.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

#include "bb31.h"

struct r0hip_bigint_back;  // include/r0hip.h

#define HIP_OK(expr)                                                                          \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess)                                                                     \
      throw std::runtime_error(std::string(#expr) + " failed: " + hipGetErrorString(e_) +     \
                               " (" + __FILE__ + ":" + std::to_string(__LINE__) + ")");      \
  } while (0)

#define R0_REQUIRE(cond, msg)                                             \
  do {                                                                    \
    if (!(cond)) throw std::runtime_error(std::string("r0hip: ") + (msg)); \
  } while (0)

namespace r0 {

// Per-process stream on the current device (created by r0hip_init / lazily).
hipStream_t stream();
void ensure_init();
// One process-wide stream for copies that run beside every thread's work
// (r0hip_memcpy_d2h_start).
hipStream_t copy_stream();
// [p, p + bytes) lies inside one live r0hip_host_alloc block
bool host_pinned(const void* p, size_t bytes);

// Constant tables kept resident in HBM for the life of the process, keyed by a
// string; `gen` runs on the host once per key.
const uint32_t* dev_table(const std::string& key, const std::function<std::vector<uint32_t>()>& gen);

// Per-thread scratch slots. A slot is one buffer reused across calls in stream order (a
// later use on the thread's stream runs after every earlier kernel that read it); two
// buffers that are live at the same time need two slots. Every slot id is named here.
enum ScratchSlot : int {
  kSlotDefault = 0,
  // batch_evaluate_any (eltwise.hip)
  kSlotEvalPartial = 2,
  kSlotEvalPoly = 9,
  kSlotEvalBegin = 10,
  kSlotEvalIdx = 11,
  kSlotEvalTable = 12,
  // poly_divide_rows (eltwise.hip): row tables alternate between two slots per batch
  kSlotDivRows = 3,
  kSlotDivRowsAlt = 103,
  kSlotDivRem = 4,
  kSlotDivLaneV = 5,
  kSlotDivLaneM = 6,
  kSlotDivBlockV = 7,
  kSlotDivBlockM = 8,
  // eval_check (prover.cpp)
  kSlotEcPolyMix = 20,
  kSlotEcVinv = 21,
  kSlotEcAcc = 22,
  kSlotEcMatFp = 23,
  kSlotEcMatExt = 24,
  kSlotEcPolyMixNb = 25,
  kSlotEcColPtr = 26,
  kSlotEcUniform = 27,
  // prover uploads (prover.cpp): evaluation points per group (3 groups), check points,
  // mix_poly_coeffs row lists, combos deltas, query gather tables
  kSlotTapXs = 33,  // .. 35
  kSlotCheckXs = 37,
  kSlotMixWhich = 38,
  kSlotMixWhichCheck = 39,
  kSlotCombosDeltas = 44,
  kSlotQueryBases = 45,
  kSlotQueryIds = 46,
  kSlotQueryOffs = 47,
  // mix_poly_coeffs (eltwise.hip)
  kSlotMixRows = 40,
  kSlotMixPows = 41,
  kSlotMixSeg = 42,
  kSlotMixSegCombo = 43,
  // per-op ABI (api.cpp)
  kSlotApiMixWhich = 50,
  kSlotApiDeltas = 51,
  kSlotApiRem = 52,
  kSlotApiRems = 53,
  kSlotApiGather = 54,
  // accumulation (recursion_accum.hip, accum.hip, bigint.cpp)
  kSlotRecAccVals = 60,
  kSlotRecAccProds = 61,
  kSlotAccTileSums = 62,
  kSlotBigIntRows = 63,
  kSlotBigIntStates = 64,
  // recursion witness generation (recursion_witgen.hip): the uploaded preflight trace, the
  // exec runs, each cycle's first IOP value, hipcub temporary storage
  kSlotWitgenWom = 70,
  kSlotWitgenIops = 71,
  kSlotWitgenRuns = 72,
  kSlotWitgenIopIdx = 73,
  kSlotWitgenTemp = 74,
  kSlotWitgenRunKey = 88,  // .. 91: run keys and indices, sorted
  kSlotWitgenRunTemp = 92,
  // rv32im witness generation (rv32im_witgen.hip): the uploaded preflight trace, the cycle
  // lists per instruction arm, the lookup tables and the error record
  kSlotRvwgCycles = 75,
  kSlotRvwgTxns = 76,
  kSlotRvwgBigint = 77,
  kSlotRvwgLists = 78,
  kSlotRvwgTables = 79,
  kSlotRvwgKeys = 83,
  kSlotRvwgSortTemp = 84,
  kSlotRvwgCompact = 85,
  kSlotRvwgSlotTable = 86,
  // r0hip_prove_segment_trace (api.cpp): the injector's index, offsets and values
  kSlotRvInjIndex = 80,
  kSlotRvInjOffsets = 81,
  kSlotRvInjValues = 82,
  kSlotRvInitErr = 87,
};

// Scratch buffer reused across calls (grown on demand; stream-ordered use only).
void* scratch(size_t bytes, int slot = kSlotDefault);
// After an error: wait for whatever this thread already queued on its stream (ignoring the
// status), so no buffer is reused or handed to another thread while kernels still use it.
// Only a thread that has a stream drains; it never creates one.
void drain_after_error() noexcept;
// At the end of every entry point, with this thread's stream drained: hand the thread's idle
// pool and scratch blocks to the shared lists, where any thread's next request finds them (as
// an exiting worker thread's are handed over). A caller's thread — one that proves and
// returns, or the calling thread of r0hip_prove_segments, which runs a prover itself — then
// keeps no device memory between calls.
void release_thread_memory() noexcept;

// Stream-ordered host->device upload through a pinned bump arena, so the caller's
// host data may die immediately. The arena is recycled by stage_reset() (call only
// when the stream is idle). Exception: a source of 64 KiB or more inside a live
// r0hip_host_alloc block is copied to the device directly, with no staging, so it must
// stay valid until the copy has run. Rule for every entry point that takes host arrays:
// drain this thread's stream (or stage_reset) before returning to the caller.
void upload_async(void* d_dst, const void* h_src, size_t bytes);
void stage_reset();
// Device-to-host copy in stream order, complete on return (this thread's stream is drained):
// small copies into pageable memory bounce through the page-locked arena.
void download(void* h_dst, const void* d_src, size_t bytes);
// The same host-to-device (small pageable sources bounce through the arena), complete on return.
void upload(void* d_dst, const void* h_src, size_t bytes);

// Optional kernel-level timing (HIP events on the library stream around each
// launcher), with the launcher's algorithmic HBM bytes and modmul-equivalent count
// (field multiplications of the restated algorithm) for roofline reporting.
struct KScope {
  KScope(const char* name, double alg_bytes, double alg_modmuls = 0);
  ~KScope();
  int idx = -1;
};
void ktimer_enable(bool on);
std::string ktimer_report();  // "name=total_ms:calls:alg_bytes:alg_modmuls;..." (synchronises)

// Device-memory accounting, the reference HAL's MemoryTracker (zkp/src/hal/mod.rs:292-317):
// `live` = bytes of the buffers handed out (pooled DevBufs and per-thread scratch), `reserved`
// = bytes held from hipMalloc (live + free pool blocks + constant tables), their peaks since
// the last reset, and the number of hipMalloc calls the library has made.
struct MemStats {
  uint64_t live, peak_live, reserved, peak_reserved, mallocs;
};
MemStats mem_stats();
void mem_reset_peak();

// A named host range for rocprofv3 --marker-trace (roctx), the reference's scope! spans
// (core/src/perf.rs:40-72; prover.rs, fri.rs, merkle.rs use the same names). Like the
// reference's, a range covers the host work of a phase: the device work it queues runs
// asynchronously on the thread's stream and shows up in the kernel trace.
struct Span {
  explicit Span(const char* name);
  ~Span();
  Span(const Span&) = delete;
  Span& operator=(const Span&) = delete;
};

// Witness groups that may still be uploading when a proof starts (the segment pipeline),
// copied in column chunks of chunk_cols(g): wait(g, col_end, s) returns once columns
// [0, col_end) of group g (0 code, 1 data, 2 accum, 3 global) have their copies queued,
// with stream s made to wait for those copies on the device.
struct UploadGate {
  virtual void wait(int group, size_t col_end, hipStream_t s) const = 0;
  virtual size_t chunk_cols(int group) const = 0;
 protected:
  ~UploadGate() = default;
};

// Workgroups for a 1-D launch of a lanes at b per workgroup. An AQL dispatch counts
// work-items in 32 bits, so a grid of 2^32 or more lanes cannot launch; such sizes go
// through grid_stride() instead.
inline unsigned div_up(size_t a, size_t b) {
  const size_t g = (a + b - 1) / b;
  R0_REQUIRE(g * b < (size_t(1) << 32), "1-D launch of " + std::to_string(a) + " lanes exceeds the 32-bit grid");
  return unsigned(g);
}
// Grid for element-wise kernels that stride over n elements (for (i = gid; i < n; i += lanes)):
// at most 2^20 workgroups (every CU stays busy), never above the 32-bit grid.
inline unsigned grid_stride(size_t n, size_t b) {
  const size_t g = (n + b - 1) / b;
  return unsigned(g < (size_t(1) << 20) ? g : (size_t(1) << 20));
}

// ---- launchers (all asynchronous on `s`) -----------------------------------
// NTT family (ntt.hip). Sizes are log2 of the per-polynomial length.
void ntt_evaluate(hipStream_t s, uint32_t* out, const uint32_t* in, size_t count, uint32_t log_out,
                  uint32_t expand_bits);
void ntt_interpolate(hipStream_t s, uint32_t* io, size_t count, uint32_t log_n, bool zk_shift);
void ntt_interpolate_from(hipStream_t s, uint32_t* io, const uint32_t* src, size_t count, uint32_t log_n,
                          bool zk_shift);
void bit_reverse(hipStream_t s, uint32_t* io, size_t count, uint32_t log_n);
// the same permutation on rows of 2^log_n FpExt elements (AoS, 4 words each)
void bit_reverse_ext(hipStream_t s, uint32_t* io, size_t count, uint32_t log_n);
void zk_shift(hipStream_t s, uint32_t* io, size_t count, uint32_t log_n);

// Hashes (hash.hip). suite: 0 = poseidon2, 1 = sha-256, 2 = poseidon254.
void hash_rows(hipStream_t s, int suite, uint32_t* out, const uint32_t* matrix, size_t rows, size_t cols);
// Row hashes over a matrix that arrives in column ranges: `cols` columns starting at
// `chunk` (column-major, `rows` per column), continuing the per-row sponge held in `state`
// (8 words per row) unless `first`; the `last` range writes the digests to `out`. Every
// range but the last must hold a multiple of 16 columns. Poseidon2 and SHA-256 only.
void hash_rows_range(hipStream_t s, int suite, uint32_t* out, uint32_t* state, const uint32_t* chunk, size_t rows,
                     size_t cols, bool first, bool last);
void hash_fold(hipStream_t s, int suite, uint32_t* io, size_t input_size, size_t output_size);
// Full merkle tree: nodes[rows..2rows) = leaves, hashes every layer up to the root.
void merkle_tree(hipStream_t s, int suite, uint32_t* nodes, const uint32_t* matrix, size_t rows, size_t cols);
// The layers above leaves already in nodes[rows..2rows). `cols` (the matrix's column count,
// SIZE_MAX if unknown) lets Poseidon2 and SHA-256 layers skip zero subtrees (hash.hip, ZeroSub).
void merkle_layers(hipStream_t s, int suite, uint32_t* nodes, size_t rows, size_t cols = SIZE_MAX);

// Element-wise and polynomial kernels (eltwise.hip).
void eltwise_add(hipStream_t s, uint32_t* out, const uint32_t* a, const uint32_t* b, size_t n);
void eltwise_copy(hipStream_t s, uint32_t* out, const uint32_t* in, size_t n);
void eltwise_zeroize(hipStream_t s, uint32_t* io, size_t n);
void fill_uniform(hipStream_t s, uint32_t* out, size_t n, uint64_t seed);
void rv32im_accum_finalize(hipStream_t s, uint32_t* accum, size_t rows, size_t cols, size_t split, size_t last);
void rv32im_accum(hipStream_t s, const uint32_t* data, uint32_t* accum, const uint32_t* global,
                  const uint32_t* mix, size_t rows, size_t cols, size_t last);
// The accumulation a segment prover runs between the mix draw and the accum commit
// (rv32im prove/witgen/mod.rs:178-221, recursion prove/witgen.rs:138-177): `accum` holds the
// group as the witness generator left it (INVALID words, plus the recursion ZK noise rows);
// the circuit's accumulation fills it for `work_cycles` cycles, then INVALID words become 0.
struct AccumStep {
  uint32_t* accum;
  size_t work_cycles;
  bool fill_invalid = false;  // the buffer is reused: fill it with INVALID words first
  // rv32im: the trace's Back::BigInt records, whose accumulator states are injected with the
  // final mix before the step (witgen/mod.rs:178-205)
  const r0hip_bigint_back* bigint = nullptr;
  size_t n_bigint = 0;
  // the group starts as rv32im_prover_groups_init leaves it (0 where the reference's INVALID
  // would be zeroized, INVALID where phase 3 adds to it), with every row stepped: the zeroize
  // after the accumulation would change nothing and is skipped
  bool zeroed = false;
};
// BigIntAccum::step over the records (byte_poly.rs:403-470): 12 words per record (poly, term,
// total), in record order; throws on an invalid EqZero as the reference does
std::vector<uint32_t> rv32im_bigint_accum_states(const uint32_t* mix, const r0hip_bigint_back* backs, size_t n,
                                                 size_t rows);
// the states scattered into accum columns 0..11 of each record's row (witgen/mod.rs:187-205)
void rv32im_bigint_inject(hipStream_t s, uint32_t* accum, size_t rows, const uint32_t* mix,
                          const r0hip_bigint_back* backs, size_t n);
void bigint_scatter(hipStream_t s, uint32_t* accum, size_t rows, const uint32_t* d_rows, const uint32_t* d_states,
                    size_t n);
// recursion circuit accumulation (recursion_accum.hip): compute, prefix product, verify
void recursion_accum(hipStream_t s, const uint32_t* ctrl, const uint32_t* global, const uint32_t* data,
                     const uint32_t* mix, uint32_t* accum, size_t steps, size_t cycles);
// recursion circuit witness generation (recursion_witgen.hip; risc0_circuit_recursion_cpu_witgen,
// recursion-sys/kernels/cxx/ffi.cpp:191-205): data (INVALID-filled) and global written from the
// control group and the preflight trace (WOM and IOP values 4 words each, cycles {iopIdx,
// isParSafe}); synchronises, throws on a failed check
void recursion_witgen(hipStream_t s, const uint32_t* ctrl, uint32_t* data, uint32_t* global, size_t total_cycles,
                      const uint32_t* h_wom, size_t n_wom, const uint32_t* h_cycles, size_t ncycles,
                      const uint32_t* h_iops, size_t n_iops);
void eltwise_sum_extelem(hipStream_t s, uint32_t* out, const uint32_t* in, size_t count, size_t to_add);
void fri_fold(hipStream_t s, uint32_t* out, const uint32_t* in, FpExt mix, size_t count);
void gather_sample(hipStream_t s, uint32_t* dst, const uint32_t* src, size_t idx, size_t size, size_t stride);
void mix_poly_coeffs(hipStream_t s, uint32_t* out, const uint32_t* in, const uint32_t* combos_dev,
                     const std::vector<uint32_t>& combos_host, FpExt mix_start, FpExt mix,
                     size_t input_size, size_t count);
void batch_evaluate_any(hipStream_t s, const uint32_t* coeffs, size_t poly_count, uint32_t log_n,
                        const uint32_t* which, const uint32_t* xs, uint32_t* out, size_t eval_count);
// the same with `which` on the host (groups evaluations by polynomial without a D2H)
// bitrev: the coefficient rows are stored in bit-reversed order (row[j] = coefficient
// rev_{log_n}(j), as the inverse NTT leaves them); needs log_n >= kEvalBitrevMinLog
void batch_evaluate_any_host(hipStream_t s, const uint32_t* coeffs, size_t poly_count, uint32_t log_n,
                             const std::vector<uint32_t>& which, const uint32_t* xs, uint32_t* out,
                             bool bitrev = false);
constexpr uint32_t kEvalBitrevMinLog = 12;
void scatter(hipStream_t s, uint32_t* into, const uint32_t* index, const uint32_t* offsets,
             const uint32_t* values, size_t cycles, uint64_t limit = ~uint64_t(0));
void copy_elem_slice(hipStream_t s, uint32_t* into, const uint32_t* from, size_t rows, size_t cols,
                     size_t from_offset, size_t from_stride, size_t into_offset, size_t into_stride);
void prefix_products(hipStream_t s, uint32_t* io, size_t n);
// In-place synthetic division of `nrows` FpExt polys of length n (row r at io + r*n*4)
// by (x - z_k) for each of its z's, in order. zs/zbegin: flattened per-row lists.
// The remainders (must be zero) are written to rem_dev[row*maxz + k].
void poly_divide_rows(hipStream_t s, uint32_t* io, size_t n, const std::vector<std::vector<FpExt>>& zs,
                      uint32_t* rem_dev);

}  // namespace r0
