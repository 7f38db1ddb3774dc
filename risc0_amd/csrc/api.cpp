// C ABI (include/r0hip.h): the symbols a Rust `HipHal` binds in place of the
// reference's risc0_zkp_cuda_* / sppark_* / cust calls. Each entry point runs its
// kernels on the library stream and returns only when they have finished
// (risc0/sys/kernels/zkp/cuda/cuda.h:77-100 semantics); errors come back as a
// malloc'd string (risc0/sys/src/lib.rs:53-75 convention).
#include "../../include/r0hip.h"

#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <functional>
#include <memory>
#include <stdexcept>
#include <vector>

#include "circuit.h"
#include "devmem.h"
#include "runtime.h"
#include "rv32im_witgen.h"

namespace r0 {
void combos_sub(hipStream_t s, uint32_t* combos, const uint32_t* deltas, size_t rows, size_t width,
                size_t cycles);
void run_eval_check(const CircuitDef& c, uint32_t* check, const uint32_t* const* groups, const uint32_t* mix,
                    const uint32_t* global, FpExt poly_mix, size_t po2, const uint32_t* h_mix = nullptr,
                    const uint32_t* h_global = nullptr);
std::vector<uint32_t> prove_segment(const CircuitDef& c, int suite, uint32_t po2, const uint32_t* code,
                                    const uint32_t* data, const uint32_t* accum, uint32_t* global,
                                    bool write_version, uint32_t version, std::vector<uint32_t>* mix_out,
                                    const UploadGate* uploads = nullptr, const AccumStep* acc = nullptr);
std::string last_profile();
}  // namespace r0

using namespace r0;

namespace {
// The call's work is complete on return, and the calling thread's idle device memory goes back
// to the shared pool (release_thread_memory), so a caller's thread holds none between calls.
template <typename F>
const char* wrap(F f) {
  try {
    f();
    HIP_OK(hipStreamSynchronize(stream()));
  } catch (const std::exception& e) {
    drain_after_error();
    release_thread_memory();
    return strdup(e.what());
  } catch (...) {
    drain_after_error();
    release_thread_memory();
    return strdup("r0hip: unknown error");
  }
  release_thread_memory();
  return nullptr;
}
// host-only entry points: no stream, no device
template <typename F>
const char* wrap_nosync(F f) {
  try {
    f();
  } catch (const std::exception& e) {
    return strdup(e.what());
  }
  return nullptr;
}
uint32_t lg(size_t n, const char* what) {
  uint32_t r = 0;
  while ((size_t(1) << r) < n) r++;
  if ((size_t(1) << r) != n) throw std::runtime_error(std::string("r0hip: ") + what + " is not a power of two");
  return r;
}
FpExt fe(const uint32_t* w) { return FpExt{{w[0], w[1], w[2], w[3]}}; }
}  // namespace

extern "C" {

const char* r0hip_init(int device_ordinal) {
  return wrap([&] {
    set_device(device_ordinal);
    // warm the module (loads every code object once)
    (void)stream();
  });
}

const char* r0hip_device_info(char* name, size_t name_cap, uint64_t* total_mem) {
  return wrap([&] {
    ensure_init();
    int dev = 0;
    HIP_OK(hipGetDevice(&dev));
    hipDeviceProp_t p;
    HIP_OK(hipGetDeviceProperties(&p, dev));
    if (name && name_cap) {
      strncpy(name, p.gcnArchName, name_cap - 1);
      name[name_cap - 1] = 0;
    }
    if (total_mem) *total_mem = p.totalGlobalMem;
  });
}

const char* r0hip_alloc(void** d_ptr, size_t bytes) {
  return wrap([&] { *d_ptr = dev_alloc(bytes); });
}
const char* r0hip_free(void* d_ptr) {
  return wrap([&] { dev_free(d_ptr); });
}
const char* r0hip_memset32(void* d_dst, uint32_t value, size_t count) {
  return wrap([&] { HIP_OK(hipMemsetD32Async(d_dst, int(value), count, stream())); });
}
const char* r0hip_memcpy_h2d(void* d_dst, const void* h_src, size_t bytes) {
  return wrap([&] { upload(d_dst, h_src, bytes); });
}
const char* r0hip_memcpy_d2h(void* h_dst, const void* d_src, size_t bytes) {
  return wrap([&] { download(h_dst, d_src, bytes); });
}
const char* r0hip_memcpy_d2d(void* d_dst, const void* d_src, size_t bytes) {
  return wrap([&] { HIP_OK(hipMemcpyAsync(d_dst, d_src, bytes, hipMemcpyDeviceToDevice, stream())); });
}
const char* r0hip_host_alloc(void** h_ptr, size_t bytes) {
  return wrap([&] { *h_ptr = host_alloc(bytes); });
}
const char* r0hip_host_free(void* h_ptr) {
  return wrap([&] { host_free(h_ptr); });
}
const char* r0hip_synchronize(void) {
  return wrap([] {});
}

namespace {
struct PendingCopy {  // r0hip_memcpy_d2h_start's handle: the copy's completion on the copy stream
  hipEvent_t ev = nullptr;
  ~PendingCopy() {
    if (ev) (void)hipEventDestroy(ev);
  }
};
}  // namespace

const char* r0hip_memcpy_d2h_start(void* h_dst, const void* d_src, size_t bytes, void** h_copy) {
  return wrap([&] {
    R0_REQUIRE(h_copy, "r0hip_memcpy_d2h_start: h_copy is NULL");
    *h_copy = nullptr;
    if (!bytes) return;
    R0_REQUIRE(h_dst && d_src, "r0hip_memcpy_d2h_start: null pointer");
    if (!host_pinned(h_dst, bytes)) {  // pageable: copied now, as r0hip_memcpy_d2h
      download(h_dst, d_src, bytes);
      return;
    }
    auto pc = std::make_unique<PendingCopy>();
    HIP_OK(hipEventCreateWithFlags(&pc->ev, hipEventDisableTiming));
    const hipStream_t cs = copy_stream();
    HIP_OK(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, cs));
    HIP_OK(hipEventRecord(pc->ev, cs));
    *h_copy = pc.release();
  });
}
const char* r0hip_copy_finish(void* h_copy, int block, int* done) {
  return wrap_nosync([&] {
    int fin = 1;
    if (h_copy) {
      auto* pc = static_cast<PendingCopy*>(h_copy);
      const hipError_t e = block ? hipEventSynchronize(pc->ev) : hipEventQuery(pc->ev);
      if (e == hipErrorNotReady) {
        fin = 0;
      } else {
        delete pc;  // the handle is spent either way
        HIP_OK(e);
      }
    }
    if (done) *done = fin;
  });
}
void r0hip_free_error(const char* err) { free(const_cast<char*>(err)); }

const char* r0hip_batch_expand_into_evaluate_ntt(uint32_t* d_out, const uint32_t* d_in, size_t count, uint32_t lg_out,
                                                 uint32_t expand_bits) {
  return wrap([&] {
    R0_REQUIRE(lg_out >= expand_bits && lg_out <= 27, "bad NTT size");
    ntt_evaluate(stream(), d_out, d_in, count, lg_out, expand_bits);
  });
}
const char* r0hip_batch_interpolate_ntt(uint32_t* d_io, size_t count, uint32_t lg_size) {
  return wrap([&] {
    R0_REQUIRE(lg_size <= 27, "bad NTT size");
    ntt_interpolate(stream(), d_io, count, lg_size, false);
  });
}
const char* r0hip_zk_shift(uint32_t* d_io, size_t count, uint32_t lg_size) {
  return wrap([&] { zk_shift(stream(), d_io, count, lg_size); });
}
const char* r0hip_batch_bit_reverse(uint32_t* d_io, size_t count, uint32_t lg_size) {
  return wrap([&] { bit_reverse(stream(), d_io, count, lg_size); });
}

const char* r0hip_batch_evaluate_any(uint32_t* d_out, const uint32_t* d_coeffs, size_t poly_count,
                                     uint32_t lg_poly_size, const uint32_t* d_which, const uint32_t* d_xs,
                                     size_t eval_count) {
  return wrap([&] { batch_evaluate_any(stream(), d_coeffs, poly_count, lg_poly_size, d_which, d_xs, d_out, eval_count); });
}

const char* r0hip_mix_poly_coeffs(uint32_t* d_out, const uint32_t* d_in, const uint32_t* h_combos,
                                  const uint32_t* h_mix_start, const uint32_t* h_mix, size_t input_size,
                                  size_t count) {
  return wrap([&] {
    std::vector<uint32_t> combos(h_combos, h_combos + input_size);
    uint32_t* d = static_cast<uint32_t*>(scratch(input_size * 4 + 16, kSlotApiMixWhich));
    upload_async(d, combos.data(), input_size * 4);
    mix_poly_coeffs(stream(), d_out, d_in, d, combos, fe(h_mix_start), fe(h_mix), input_size, count);
  });
}

const char* r0hip_fri_fold(uint32_t* d_out, const uint32_t* d_in, const uint32_t* h_mix, size_t count) {
  return wrap([&] { fri_fold(stream(), d_out, d_in, fe(h_mix), count); });
}

const char* r0hip_combos_prepare(uint32_t* d_combos, const uint32_t* h_coeff_u, size_t combo_count, size_t cycles,
                                 const uint32_t* h_reg_sizes, const uint32_t* h_reg_combo_ids, size_t reg_count,
                                 const uint32_t* h_mix) {
  return wrap([&] {
    size_t width = 1;
    for (size_t r = 0; r < reg_count; r++) width = std::max<size_t>(width, h_reg_sizes[r]);
    std::vector<FpExt> deltas((combo_count + 1) * width, fe_zero());
    FpExt cur = fe_one(), mix = fe(h_mix);
    size_t pos = 0;
    for (size_t r = 0; r < reg_count; r++) {
      for (size_t i = 0; i < h_reg_sizes[r]; i++) {
        FpExt& d = deltas[h_reg_combo_ids[r] * width + i];
        d = fe_add(d, fe_mul(cur, fe(h_coeff_u + 4 * (pos + i))));
      }
      cur = fe_mul(cur, mix);
      pos += h_reg_sizes[r];
    }
    for (size_t i = 0; i < 16; i++) {
      FpExt& d = deltas[combo_count * width];
      d = fe_add(d, fe_mul(cur, fe(h_coeff_u + 4 * pos)));
      pos++;
      cur = fe_mul(cur, mix);
    }
    uint32_t* dd = static_cast<uint32_t*>(scratch(deltas.size() * 16, kSlotApiDeltas));
    upload_async(dd, deltas.data(), deltas.size() * 16);
    combos_sub(stream(), d_combos, dd, combo_count + 1, width, cycles);
  });
}

const char* r0hip_poly_divide(uint32_t* d_poly, size_t size, uint32_t* h_remainder, const uint32_t* h_z) {
  return wrap([&] {
    std::vector<std::vector<FpExt>> zs{{fe(h_z)}};
    uint32_t* rem = static_cast<uint32_t*>(scratch(16, kSlotApiRem));
    poly_divide_rows(stream(), d_poly, size, zs, rem);
    HIP_OK(hipMemcpyAsync(h_remainder, rem, 16, hipMemcpyDeviceToHost, stream()));
  });
}

const char* r0hip_combos_divide(uint32_t* d_combos, size_t nchunks, const uint32_t* h_pows, const uint32_t* h_begin,
                                size_t cycles, int64_t* bad_chunk) {
  return wrap([&] {
    std::vector<std::vector<FpExt>> zs(nchunks);
    size_t maxz = 0;
    for (size_t i = 0; i < nchunks; i++) {
      for (uint32_t k = h_begin[i]; k < h_begin[i + 1]; k++) zs[i].push_back(fe(h_pows + 4 * k));
      maxz = std::max(maxz, zs[i].size());
    }
    std::vector<uint32_t> h(nchunks * std::max<size_t>(maxz, 1) * 4, 0);
    uint32_t* rem = static_cast<uint32_t*>(scratch(h.size() * 4 + 16, kSlotApiRems));
    HIP_OK(hipMemsetAsync(rem, 0, h.size() * 4, stream()));
    poly_divide_rows(stream(), d_combos, cycles, zs, rem);
    HIP_OK(hipMemcpyAsync(h.data(), rem, h.size() * 4, hipMemcpyDeviceToHost, stream()));
    HIP_OK(hipStreamSynchronize(stream()));
    *bad_chunk = -1;
    for (size_t i = 0; i < h.size(); i++)
      if (h[i]) {
        *bad_chunk = int64_t(i / (std::max<size_t>(maxz, 1) * 4));
        break;
      }
  });
}

const char* r0hip_eltwise_add_elem(uint32_t* d_out, const uint32_t* d_a, const uint32_t* d_b, size_t count) {
  return wrap([&] { eltwise_add(stream(), d_out, d_a, d_b, count); });
}
const char* r0hip_eltwise_copy_elem(uint32_t* d_out, const uint32_t* d_in, size_t count) {
  return wrap([&] { eltwise_copy(stream(), d_out, d_in, count); });
}
const char* r0hip_eltwise_zeroize_elem(uint32_t* d_io, size_t count) {
  return wrap([&] { eltwise_zeroize(stream(), d_io, count); });
}
const char* r0hip_eltwise_sum_extelem(uint32_t* d_out, const uint32_t* d_in, size_t to_add, size_t count) {
  return wrap([&] { eltwise_sum_extelem(stream(), d_out, d_in, count, to_add); });
}
const char* r0hip_eltwise_copy_elem_slice(uint32_t* d_into, const uint32_t* d_from, size_t from_rows,
                                          size_t from_cols, size_t from_offset, size_t from_stride,
                                          size_t into_offset, size_t into_stride) {
  return wrap([&] {
    copy_elem_slice(stream(), d_into, d_from, from_rows, from_cols, from_offset, from_stride, into_offset,
                    into_stride);
  });
}
const char* r0hip_gather_sample(uint32_t* d_dst, const uint32_t* d_src, size_t idx, size_t size, size_t stride) {
  return wrap([&] { gather_sample(stream(), d_dst, d_src, idx, size, stride); });
}
const char* r0hip_gather_sample_host(uint32_t* h_dst, const uint32_t* d_src, size_t idx, size_t size,
                                     size_t stride) {
  return wrap([&] {
    if (!size) return;
    R0_REQUIRE(h_dst && d_src, "gather_sample_host: null pointer");
    uint32_t* d = static_cast<uint32_t*>(scratch(size * 4, kSlotApiGather));
    gather_sample(stream(), d, d_src, idx, size, stride);
    download(h_dst, d, size * 4);
  });
}
const char* r0hip_scatter(uint32_t* d_into, const uint32_t* d_index, const uint32_t* d_offsets,
                          const uint32_t* d_values, size_t cycles) {
  return wrap([&] { scatter(stream(), d_into, d_index, d_offsets, d_values, cycles); });
}
const char* r0hip_prefix_products(uint32_t* d_io, size_t count) {
  return wrap([&] { prefix_products(stream(), d_io, count); });
}
const char* r0hip_rv32im_accum_finalize(uint32_t* d_accum, size_t rows, size_t cols, size_t last_cycle) {
  // kUserAccumSplit = kLayout_TopAccum.columns[0].col (rv32im-sys/kernels/cxx/ffi.cpp:52,
  // layout.cpp.inc:6993-6999): the first machine accumulator column
  return wrap([&] { rv32im_accum_finalize(stream(), d_accum, rows, cols, 23, last_cycle); });
}
const char* r0hip_rv32im_accum(const uint32_t* d_data, uint32_t* d_accum, const uint32_t* d_global,
                               const uint32_t* d_mix, size_t rows, size_t cols, size_t last_cycle) {
  return wrap([&] { rv32im_accum(stream(), d_data, d_accum, d_global, d_mix, rows, cols, last_cycle); });
}
const char* r0hip_rv32im_bigint_accum_states(const uint32_t* h_mix, const r0hip_bigint_back* h_backs, size_t n,
                                             size_t rows, uint32_t* h_states) {
  return wrap_nosync([&] {
    R0_REQUIRE(h_mix && (n == 0 || (h_backs && h_states)), "r0hip_rv32im_bigint_accum_states: null argument");
    const std::vector<uint32_t> st = rv32im_bigint_accum_states(h_mix, h_backs, n, rows);
    if (n) memcpy(h_states, st.data(), st.size() * 4);
  });
}
const char* r0hip_rv32im_bigint_accum_inject(uint32_t* d_accum, size_t rows, const uint32_t* h_mix,
                                             const r0hip_bigint_back* h_backs, size_t n) {
  return wrap([&] {
    R0_REQUIRE(d_accum && h_mix, "r0hip_rv32im_bigint_accum_inject: null argument");
    stage_reset();
    rv32im_bigint_inject(stream(), d_accum, rows, h_mix, h_backs, n);
  });
}
const char* r0hip_recursion_accum(const uint32_t* d_ctrl, const uint32_t* d_global, const uint32_t* d_data,
                                  const uint32_t* d_mix, uint32_t* d_accum, size_t work_cycles,
                                  size_t total_cycles) {
  return wrap([&] {
    R0_REQUIRE(d_ctrl && d_global && d_data && d_mix && d_accum, "r0hip_recursion_accum: null argument");
    recursion_accum(stream(), d_ctrl, d_global, d_data, d_mix, d_accum, work_cycles, total_cycles);
  });
}
const char* r0hip_rv32im_witgen(uint32_t mode, const r0hip_raw_exec_buffers* buffers,
                                const r0hip_raw_preflight_trace* preflight, uint32_t cycles) {
  return wrap([&] {
    R0_REQUIRE(buffers && preflight && buffers->global.buf && buffers->data.buf, "r0hip_rv32im_witgen: null argument");
    const CircuitDef* c = find_circuit("rv32im");
    R0_REQUIRE(buffers->data.cols == c->group_size(2) && buffers->global.cols == c->output_size &&
                   buffers->global.rows == 1,
               "r0hip_rv32im_witgen: buffers are not the rv32im data group and global vector");
    R0_REQUIRE(cycles == buffers->data.rows, "r0hip_rv32im_witgen: cycles must equal the data group's rows");
    // the reference's witness generator takes Buffer<checked = true> (witgen/mod.rs:150) and
    // these kernels always run the checked stores and reads
    R0_REQUIRE(buffers->data.checked && buffers->global.checked,
               "r0hip_rv32im_witgen: unchecked buffers are not supported (the reference passes checked = true)");
    stage_reset();
    rv32im_witgen(stream(), mode, buffers->data.buf, buffers->global.buf, buffers->data.rows,
                  static_cast<const rvwg::PreflightCycle*>(preflight->cycles),
                  static_cast<const rvwg::MemoryTxn*>(preflight->txns), preflight->txns_len, preflight->bigint_bytes,
                  preflight->bigint_bytes_len, preflight->table_split_cycle, cycles);
  });
}

}  // extern "C"

namespace r0 {

void check_injector(const uint32_t* index, size_t rows, const uint32_t* offsets, const uint32_t* values,
                    size_t limit, size_t seg_rows);

// SegmentProverImpl::prove_core from a preflight (circuit/rv32im/src/prove/hal/mod.rs:143-224):
// WitnessGenerator::hal_generate_witness (witgen/mod.rs:135-176: globals, code and data
// INVALID, the injector scattered into data, stepExec, zeroize), then the prove core with the
// version word 2 and WitnessGenerator::accum on the device. `resident`: the global vector,
// the injector and the preflight arrays are device pointers; otherwise host pointers.
// inputs_ready (resident only): called with the stream after the groups' fill (which reads no
// input) and before the first read of the inputs (the segment pipeline makes the stream wait for
// their upload there, so the fill runs while the trace still uploads).
std::vector<uint32_t> prove_trace(int suite, uint32_t po2, uint32_t mode, const uint32_t* global_in,
                                  const uint32_t* inj_index, size_t inj_rows, const uint32_t* inj_offsets,
                                  const uint32_t* inj_values, const r0hip_raw_preflight_trace* pf,
                                  const r0hip_bigint_back* h_bigint, size_t n_bigint, bool resident,
                                  std::vector<uint32_t>* mix, const std::function<void(hipStream_t)>& inputs_ready) {
  const CircuitDef* c = find_circuit("rv32im");
  R0_REQUIRE(global_in && inj_index && pf && pf->cycles, "r0hip_prove_segment_trace: null argument");
  R0_REQUIRE(po2 >= 2 && po2 <= 24, "r0hip_prove_segment_trace: po2 out of range");
  R0_REQUIRE(n_bigint == 0 || h_bigint, "r0hip_prove_segment_trace: h_bigint is NULL with n_bigint > 0");
  const size_t n = size_t(1) << po2;
  R0_REQUIRE(inj_rows <= n, "r0hip_prove_segment_trace: injector longer than the segment");
  const size_t data_cols = c->group_size(2);
  hipStream_t s = stream();
  stage_reset();
  Span span("prove_segment_trace");
  DevBuf code(c->group_size(1) * n), data(data_cols * n), global(c->output_size), accum(c->group_size(0) * n);
  // the groups as WitnessGenerator::new / ::accum allocate them (INVALID), already zeroized where
  // nothing reads INVALID (rv32im_prover_groups_fill), then the injector (rv32im_prover_inject)
  rv32im_prover_groups_fill(s, data.p, code.p, accum.p, n, c->group_size(0));
  const uint32_t *idx = inj_index, *off = inj_offsets, *val = inj_values;
  const rvwg::PreflightCycle* cyc = static_cast<const rvwg::PreflightCycle*>(pf->cycles);
  const rvwg::MemoryTxn* txn = static_cast<const rvwg::MemoryTxn*>(pf->txns);
  const uint8_t* big = pf->bigint_bytes;
  if (resident) {
    if (inputs_ready) inputs_ready(s);
    HIP_OK(hipMemcpyAsync(global.p, global_in, global.words * 4, hipMemcpyDeviceToDevice, s));
  } else {
    R0_REQUIRE((pf->txns_len == 0 || pf->txns) && (pf->bigint_bytes_len == 0 || pf->bigint_bytes),
               "r0hip_prove_segment_trace: null trace array with a nonzero count");
    check_injector(inj_index, inj_rows, inj_offsets, inj_values, data_cols * n, n);
    const size_t n_inj = inj_index[inj_rows];
    upload_async(global.p, global_in, global.words * 4);
    auto* d_idx = static_cast<uint32_t*>(scratch((inj_rows + 1) * 4, kSlotRvInjIndex));
    auto* d_off = static_cast<uint32_t*>(scratch(n_inj * 4 + 4, kSlotRvInjOffsets));
    auto* d_val = static_cast<uint32_t*>(scratch(n_inj * 4 + 4, kSlotRvInjValues));
    upload_async(d_idx, inj_index, (inj_rows + 1) * 4);
    upload_async(d_off, inj_offsets, n_inj * 4);
    upload_async(d_val, inj_values, n_inj * 4);
    idx = d_idx, off = d_off, val = d_val;
    cyc = rv32im_upload_cycles(cyc, n);
    auto* d_txn = static_cast<rvwg::MemoryTxn*>(scratch(size_t(pf->txns_len) * sizeof(rvwg::MemoryTxn) + 16, kSlotRvwgTxns));
    auto* d_big = static_cast<uint8_t*>(scratch(size_t(pf->bigint_bytes_len) + 16, kSlotRvwgBigint));
    upload_async(d_txn, pf->txns, size_t(pf->txns_len) * sizeof(rvwg::MemoryTxn));
    upload_async(d_big, pf->bigint_bytes, pf->bigint_bytes_len);
    txn = pf->txns_len ? d_txn : nullptr;
    big = pf->bigint_bytes_len ? d_big : nullptr;
  }
  auto* ierr = static_cast<uint32_t*>(scratch(16, kSlotRvInitErr));
  HIP_OK(hipMemsetD32Async(ierr, 0u, 4, s));
  rv32im_prover_inject(s, data.p, n, idx, off, val, inj_rows, data.words, cyc, ierr);
  {
    Span w("witgen");
    // an injector entry outside its row's injected columns: the group as the reference prepares
    // it (hal_generate_witness, witgen/mod.rs:146-162), every word INVALID and the injector scattered
    auto reinit = [&] {
      HIP_OK(hipMemsetD32Async(data.p, 0xFFFFFFFFu, data.words, s));
      scatter(s, data.p, idx, off, val, inj_rows, data.words);
    };
    rv32im_witgen_dev(s, mode, data.p, global.p, n, cyc, txn, pf->txns_len, big, pf->bigint_bytes_len,
                      pf->table_split_cycle, uint32_t(n), true, ierr, reinit);
  }
  eltwise_zeroize(s, global.p, global.words);  // the data group was zeroized by the witgen merge
  AccumStep acc{accum.p, n, false, h_bigint, n_bigint};
  acc.zeroed = true;
  return prove_segment(*c, suite, po2, code.p, data.p, nullptr, global.p, true, 2, mix, nullptr, &acc);
}

// The host injector (Injector, witgen/mod.rs:329-378) before it is uploaded: a CSR index that
// never decreases (entries of row c are [index[c], index[c + 1])), offsets inside the data group
// and in the entry's own row (col * seg_rows + c: Injector::set writes only its row). O(rows +
// entries); the resident path's inject pass bounds its reads and writes and reports other rows.
void check_injector(const uint32_t* index, size_t rows, const uint32_t* offsets, const uint32_t* values,
                    size_t limit, size_t seg_rows) {
  for (size_t c = 0; c < rows; c++)
    R0_REQUIRE(index[c] <= index[c + 1], "r0hip_prove_segment_trace: injector index decreases at row " +
                                             std::to_string(c));
  const size_t n_inj = index[rows];
  R0_REQUIRE(n_inj == 0 || (offsets && values), "r0hip_prove_segment_trace: null injector arrays");
  for (size_t c = 0; c < rows; c++)
    for (size_t i = index[c]; i < index[c + 1]; i++) {
      R0_REQUIRE(offsets[i] < limit, "r0hip_prove_segment_trace: injector offset outside the data group");
      R0_REQUIRE(offsets[i] % seg_rows == c, "r0hip_prove_segment_trace: injector entry of row " + std::to_string(c) +
                                                 " sets word " + std::to_string(offsets[i]) +
                                                 " of another row (Injector::set writes its own row)");
    }
}

}  // namespace r0

namespace {

void seal_out(const std::vector<uint32_t>& seal, const std::vector<uint32_t>& mix, uint32_t* h_seal, size_t seal_cap,
              size_t* seal_len, uint32_t* h_mix_out) {
  if (seal_len) *seal_len = seal.size();
  if (h_mix_out) memcpy(h_mix_out, mix.data(), mix.size() * 4);
  if (h_seal) {
    R0_REQUIRE(seal.size() <= seal_cap, "seal buffer too small");
    memcpy(h_seal, seal.data(), seal.size() * 4);
  }
}

}  // namespace

extern "C" {

const char* r0hip_prove_segment_trace(int suite, uint32_t po2, uint32_t mode, const uint32_t* h_global,
                                      const uint32_t* h_inj_index, size_t inj_rows, const uint32_t* h_inj_offsets,
                                      const uint32_t* h_inj_values, const r0hip_raw_preflight_trace* preflight,
                                      const r0hip_bigint_back* h_bigint, size_t n_bigint, uint32_t* h_seal,
                                      size_t seal_cap, size_t* seal_len, uint32_t* h_mix_out) {
  return wrap([&] {
    std::vector<uint32_t> mix;
    auto seal = prove_trace(suite, po2, mode, h_global, h_inj_index, inj_rows, h_inj_offsets, h_inj_values, preflight,
                            h_bigint, n_bigint, false, &mix, {});
    seal_out(seal, mix, h_seal, seal_cap, seal_len, h_mix_out);
  });
}

const char* r0hip_prove_segment_trace_resident(int suite, uint32_t po2, uint32_t mode, const uint32_t* d_global,
                                               const uint32_t* d_inj_index, size_t inj_rows,
                                               const uint32_t* d_inj_offsets, const uint32_t* d_inj_values,
                                               const r0hip_raw_preflight_trace* d_preflight,
                                               const r0hip_bigint_back* h_bigint, size_t n_bigint, uint32_t* h_seal,
                                               size_t seal_cap, size_t* seal_len, uint32_t* h_mix_out) {
  return wrap([&] {
    std::vector<uint32_t> mix;
    auto seal = prove_trace(suite, po2, mode, d_global, d_inj_index, inj_rows, d_inj_offsets, d_inj_values,
                            d_preflight, h_bigint, n_bigint, true, &mix, {});
    seal_out(seal, mix, h_seal, seal_cap, seal_len, h_mix_out);
  });
}

const char* r0hip_recursion_witgen(const uint32_t* d_ctrl, uint32_t* d_data, uint32_t* d_global, size_t total_cycles,
                                   const uint32_t* h_wom, size_t n_wom, const uint32_t* h_cycles, size_t n_cycles,
                                   const uint32_t* h_iops, size_t n_iops) {
  return wrap([&] {
    R0_REQUIRE(d_ctrl && d_data && d_global, "r0hip_recursion_witgen: null argument");
    stage_reset();
    recursion_witgen(stream(), d_ctrl, d_data, d_global, total_cycles, h_wom, n_wom, h_cycles, n_cycles, h_iops,
                     n_iops);
  });
}

const char* r0hip_prove_recursion(int suite, uint32_t po2, const uint32_t* d_ctrl, const uint32_t* h_wom, size_t n_wom,
                                  const uint32_t* h_cycles, size_t n_cycles, const uint32_t* h_iops, size_t n_iops,
                                  uint64_t noise_seed, uint32_t* h_seal, size_t seal_cap, size_t* seal_len,
                                  uint32_t* h_mix_out) {
  return wrap([&] {
    const CircuitDef* c = find_circuit("recursion");
    R0_REQUIRE(c && d_ctrl, "r0hip_prove_recursion: null argument");
    R0_REQUIRE(po2 >= 11 && po2 <= 24, "r0hip_prove_recursion: po2 out of range (ZK rows need po2 >= 11)");
    constexpr size_t kZk = 1024;  // risc0_zkp::ZK_CYCLES (zkp/src/lib.rs:42)
    const size_t n = size_t(1) << po2;
    R0_REQUIRE(n_cycles <= n - kZk, "r0hip_prove_recursion: program longer than 2^po2 - ZK_CYCLES rows");
    const size_t data_cols = c->group_size(2), accum_cols = c->group_size(0);
    hipStream_t s = stream();
    stage_reset();
    // WitnessGenerator::new (circuit/recursion/src/prove/witgen.rs:44-133)
    DevBuf data(data_cols * n), global(c->output_size), accum(accum_cols * n), noise(std::max(data_cols, accum_cols) * kZk);
    HIP_OK(hipMemsetD32Async(data.p, 0xFFFFFFFFu, data.words, s));
    HIP_OK(hipMemsetD32Async(global.p, 0xFFFFFFFFu, global.words, s));
    recursion_witgen(s, d_ctrl, data.p, global.p, n, h_wom, n_wom, h_cycles, n_cycles, h_iops, n_iops);
    // ZK noise in the last ZK_CYCLES data rows (witgen.rs:101-116: eltwise_copy_elem_slice
    // from a data_size x ZK_CYCLES noise matrix), here per-cell values of r0hip_fill_uniform
    fill_uniform(s, noise.p, data_cols * kZk, noise_seed);
    copy_elem_slice(s, data.p, noise.p, data_cols, kZk, 0, kZk, n - kZk, n);
    eltwise_zeroize(s, data.p, data.words);
    // WitnessGenerator::accum (witgen.rs:134-177): INVALID plus noise rows, then the
    // accumulation inside the proof; prove (prove/mod.rs:160-230)
    HIP_OK(hipMemsetD32Async(accum.p, 0xFFFFFFFFu, accum.words, s));
    fill_uniform(s, noise.p, accum_cols * kZk, noise_seed + 1);
    copy_elem_slice(s, accum.p, noise.p, accum_cols, kZk, 0, kZk, n - kZk, n);
    std::vector<uint32_t> mix;
    const AccumStep acc{accum.p, n_cycles};
    std::vector<uint32_t> seal =
        prove_segment(*c, suite, po2, d_ctrl, data.p, nullptr, global.p, false, 0, &mix, nullptr, &acc);
    if (seal_len) *seal_len = seal.size();
    if (h_mix_out) memcpy(h_mix_out, mix.data(), mix.size() * 4);
    if (h_seal) {
      R0_REQUIRE(seal.size() <= seal_cap, "seal buffer too small");
      memcpy(h_seal, seal.data(), seal.size() * 4);
    }
  });
}

const char* r0hip_fill_uniform(uint32_t* d_out, size_t count, uint64_t seed) {
  return wrap([&] { fill_uniform(stream(), d_out, count, seed); });
}

const char* r0hip_hash_rows(int suite, uint32_t* d_out, const uint32_t* d_matrix, size_t rows, size_t cols) {
  return wrap([&] {
    R0_REQUIRE(suite >= 0 && suite <= 2, "unknown hash suite");
    hash_rows(stream(), suite, d_out, d_matrix, rows, cols);
  });
}
const char* r0hip_hash_fold(int suite, uint32_t* d_io, size_t input_size, size_t output_size) {
  return wrap([&] {
    R0_REQUIRE(suite >= 0 && suite <= 2, "unknown hash suite");
    hash_fold(stream(), suite, d_io, input_size, output_size);
  });
}
const char* r0hip_merkle_tree(int suite, uint32_t* d_nodes, const uint32_t* d_matrix, size_t rows, size_t cols) {
  return wrap([&] {
    R0_REQUIRE(suite >= 0 && suite <= 2, "unknown hash suite");
    R0_REQUIRE(rows > 0 && (rows & (rows - 1)) == 0, "merkle_tree: rows must be a power of two");
    merkle_tree(stream(), suite, d_nodes, d_matrix, rows, cols);
  });
}

const char* r0hip_eval_check(const char* circuit, uint32_t* d_check, const uint32_t* const* d_groups,
                             const uint32_t* d_mix, const uint32_t* d_global, const uint32_t* h_poly_mix,
                             uint32_t po2) {
  return wrap([&] {
    const CircuitDef* c = find_circuit(circuit ? circuit : "");
    R0_REQUIRE(c, std::string("unknown circuit ") + (circuit ? circuit : "(null)"));
    R0_REQUIRE(d_check && d_groups && h_poly_mix, "eval_check: null argument");
    for (int g = 0; g < 3; g++) R0_REQUIRE(d_groups[g], "eval_check: null register group");
    stage_reset();
    run_eval_check(*c, d_check, d_groups, d_mix, d_global, fe(h_poly_mix), po2);
  });
}

const char* r0hip_prove_segment(const char* circuit, int suite, uint32_t po2, const uint32_t* d_code,
                                const uint32_t* d_data, const uint32_t* d_accum, uint32_t* d_global,
                                int write_version, uint32_t version, uint32_t* h_seal, size_t seal_cap,
                                size_t* seal_len, uint32_t* h_mix_out) {
  return wrap([&] {
    const CircuitDef* c = find_circuit(circuit ? circuit : "");
    R0_REQUIRE(c, std::string("unknown circuit ") + (circuit ? circuit : "(null)"));
    std::vector<uint32_t> mix;
    std::vector<uint32_t> seal = prove_segment(*c, suite, po2, d_code, d_data, d_accum, d_global, write_version != 0,
                                               version, &mix);
    if (seal_len) *seal_len = seal.size();
    if (h_mix_out) memcpy(h_mix_out, mix.data(), mix.size() * 4);
    if (h_seal) {
      R0_REQUIRE(seal.size() <= seal_cap, "seal buffer too small");
      memcpy(h_seal, seal.data(), seal.size() * 4);
    }
  });
}

const char* r0hip_prove_segment_accum(const char* circuit, int suite, uint32_t po2, const uint32_t* d_code,
                                      const uint32_t* d_data, uint32_t* d_accum, size_t work_cycles,
                                      const r0hip_bigint_back* h_bigint, size_t n_bigint, uint32_t* d_global,
                                      int write_version, uint32_t version, uint32_t* h_seal, size_t seal_cap,
                                      size_t* seal_len, uint32_t* h_mix_out) {
  return wrap([&] {
    const CircuitDef* c = find_circuit(circuit ? circuit : "");
    R0_REQUIRE(c, std::string("unknown circuit ") + (circuit ? circuit : "(null)"));
    R0_REQUIRE(n_bigint == 0 || h_bigint, "prove_segment_accum: h_bigint is NULL with n_bigint > 0");
    std::vector<uint32_t> mix;
    const AccumStep acc{d_accum, work_cycles, false, h_bigint, n_bigint};
    std::vector<uint32_t> seal = prove_segment(*c, suite, po2, d_code, d_data, nullptr, d_global, write_version != 0,
                                               version, &mix, nullptr, &acc);
    if (seal_len) *seal_len = seal.size();
    if (h_mix_out) memcpy(h_mix_out, mix.data(), mix.size() * 4);
    if (h_seal) {
      R0_REQUIRE(seal.size() <= seal_cap, "seal buffer too small");
      memcpy(h_seal, seal.data(), seal.size() * 4);
    }
  });
}

const char* r0hip_set_kernel_timing(int on) {
  return wrap([&] { ktimer_enable(on != 0); });
}

const char* r0hip_kernel_times(char* buf, size_t cap) {
  return wrap([&] {
    std::string p = ktimer_report();
    if (buf && cap) {
      strncpy(buf, p.c_str(), cap - 1);
      buf[cap - 1] = 0;
    }
  });
}

const char* r0hip_last_profile(char* buf, size_t cap) {
  return wrap([&] {
    std::string p = last_profile();
    if (buf && cap) {
      strncpy(buf, p.c_str(), cap - 1);
      buf[cap - 1] = 0;
    }
  });
}

// MemoryTracker (zkp/src/hal/mod.rs:292-317): out[0..5) = live bytes, peak live bytes,
// reserved bytes, peak reserved bytes, hipMalloc calls so far. Host-only, never fails.
const char* r0hip_mem_stats(uint64_t* out) {
  return wrap_nosync([&] {
    R0_REQUIRE(out != nullptr, "r0hip_mem_stats: null output");
    const MemStats m = mem_stats();
    out[0] = m.live;
    out[1] = m.peak_live;
    out[2] = m.reserved;
    out[3] = m.peak_reserved;
    out[4] = m.mallocs;
  });
}

const char* r0hip_mem_reset_peak(void) {
  return wrap_nosync([&] { mem_reset_peak(); });
}

const char* r0hip_trim(void) {
  return wrap([&] {
    dev_trim();
    host_trim();
  });
}

}  // extern "C"
