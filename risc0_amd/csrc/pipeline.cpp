// Segment pipeline: many segments through one GPU with the witness upload of the next
// segment overlapped with the proofs in flight — the queue r0vm's GPU worker keeps
// (GPU_QUEUE_DEPTH=2, risc0/r0vm/src/actors/worker.rs:75-76) and the per-segment loop of
// the zkvm prover (risc0/zkvm/src/host/server/prove/prover_impl.rs:84-94), native here.
//
// One uploader thread copies a job's witness groups from host memory (page-locked for
// full PCIe rate) into a free device buffer set on its own stream, recording an event per
// group; `in_flight` prover threads each take a set as soon as its copies are queued, run
// the whole-segment prover on their own stream (which waits on each group's event just
// before that group's first use)
// (runtime.cpp gives every host thread its own stream, pool and staging), write the
// seal, and hand the set back. in_flight + 1 sets circulate, so an upload is always
// running ahead while the GPU proves. Each job reports its own error.
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <chrono>
#include <deque>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/r0hip.h"
#include "circuit.h"
#include "devmem.h"
#include "runtime.h"

namespace r0 {
std::vector<uint32_t> prove_segment(const CircuitDef& c, int suite, uint32_t po2, const uint32_t* code,
                                    const uint32_t* data, const uint32_t* accum, uint32_t* global,
                                    bool write_version, uint32_t version, std::vector<uint32_t>* mix_out,
                                    const UploadGate* uploads, const AccumStep* acc = nullptr);
// api.cpp: rv32im prove_core from a preflight trace, and the host check of an injector
std::vector<uint32_t> prove_trace(int suite, uint32_t po2, uint32_t mode, const uint32_t* global_in,
                                  const uint32_t* inj_index, size_t inj_rows, const uint32_t* inj_offsets,
                                  const uint32_t* inj_values, const r0hip_raw_preflight_trace* pf,
                                  const r0hip_bigint_back* h_bigint, size_t n_bigint, bool resident,
                                  std::vector<uint32_t>* mix, const std::function<void(hipStream_t)>& inputs_ready);
void check_injector(const uint32_t* index, size_t rows, const uint32_t* offsets, const uint32_t* values,
                    size_t limit, size_t seg_rows);

namespace {

// Columns per upload chunk: a multiple of 16, so the prover can hash a group's rows range by
// range as the chunks land (hash_rows_range); ~200 MB per chunk at po2=20.
constexpr size_t kChunkCols = 48;

// A device buffer set and its upload state. hipMemcpyAsync from page-locked memory returns
// only when a large copy is done, so the set is handed to a prover before its copies are
// queued: the prover blocks in wait() until the uploader has queued the chunks it needs and
// recorded the last one's event, then its stream waits on that event.
struct BufSet final : UploadGate {
  DevBuf g[4];                     // code, data, accum, global
  size_t cols[4] = {1, 1, 1, 1};   // columns per group (global: one)
  size_t col_words[4] = {0, 0, 0, 0};
  std::vector<hipEvent_t> ev[4];   // per chunk, recorded on the uploader stream
  size_t job = 0;
  mutable std::mutex mu;
  mutable std::condition_variable cv;
  size_t queued[4] = {0, 0, 0, 0};  // chunks queued per group (all of them after an upload error)
  size_t chunks(int grp) const { return (cols[grp] + kChunkCols - 1) / kChunkCols; }
  size_t chunk_cols(int) const override { return kChunkCols; }
  void mark(int grp, size_t n) {
    {
      std::lock_guard<std::mutex> lk(mu);
      queued[grp] = n;
    }
    cv.notify_all();
  }
  void mark_all() {
    {
      std::lock_guard<std::mutex> lk(mu);
      for (int i = 0; i < 4; i++) queued[i] = chunks(i);
    }
    cv.notify_all();
  }
  void wait(int grp, size_t col_end, hipStream_t s) const override {
    const size_t need = (std::min(col_end, cols[grp]) + kChunkCols - 1) / kChunkCols;
    if (need == 0) return;
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return queued[grp] >= need; });
    }
    // one stream carries every copy in order: the last needed chunk's event covers the rest
    HIP_OK(hipStreamWaitEvent(s, ev[grp][need - 1], 0));
  }
};

// a bounded queue of set indices
struct Queue {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<long> q;
  void put(long v) {
    {
      std::lock_guard<std::mutex> lk(mu);
      q.push_back(v);
    }
    cv.notify_one();
  }
  long get() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return !q.empty(); });
    long v = q.front();
    q.pop_front();
    return v;
  }
};

// k provers: k - 1 threads and the calling thread, whose stream the process already holds, so
// a call keeps k + 1 streams busy (the uploader's and the provers') and the runtime's default 4
// hardware queues give each its own for k <= 3 (a shared queue runs its streams' kernels in
// order). R0_PIPE_CALLER_PROVES=0: k prover threads (the calling thread only waits).
template <typename F>
void run_provers(size_t k, F& prover) {
  static const bool caller = [] {
    const char* e = getenv("R0_PIPE_CALLER_PROVES");
    return !e || strtoul(e, nullptr, 10) != 0;
  }();
  std::vector<std::thread> threads;
  for (size_t t = caller ? 1 : 0; t < k; t++) threads.emplace_back(prover);
  if (caller) prover();  // returns at its stop token; never throws (errors are per job)
  for (auto& t : threads) t.join();
}

char* dup_msg(const char* m) {
  size_t n = strlen(m) + 1;
  char* p = static_cast<char*>(malloc(n));
  if (p) memcpy(p, m, n);
  return p;
}

// A device trace set: one job's preflight trace, injector and global vector, and the event
// that marks their upload on the uploader's stream. `landed`: the uploader has queued every
// copy and recorded the event, or failed (the job then carries the error).
struct TraceSet {
  DevBuf glob, index, offsets, values, cycles, txns, bigint;
  hipEvent_t ev = nullptr;
  size_t job = 0;
  std::mutex mu;
  std::condition_variable cv;
  bool landed = false;
  void mark() {
    {
      std::lock_guard<std::mutex> lk(mu);
      landed = true;
    }
    cv.notify_all();
  }
  void wait_landed() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return landed; });
  }
};

// Trace jobs: the uploader copies job i's trace into a free trace set and hands the set to a
// prover at once; the prover allocates its witness groups and queues their fill (which reads no
// input), then waits on the host until the uploader has queued the set's copies and makes its
// stream wait for the set's event before the injector pass (prove_trace's inputs_ready), so the
// copies of one segment overlap the proofs of the others. k + 1 sets, sized once for the largest
// job.
// verify: each finished seal is checked by r0hip_verify_seal (the validity equation included) on
// a host thread of its own while the GPU proves the next segments, as ProverImpl::
// prove_segment_core verifies a receipt before it returns it (zkvm/src/host/server/prove/
// prover_impl.rs:262-280); a seal that fails fails its job.
const char* prove_trace_jobs(int suite, uint32_t po2, r0hip_trace_job* jobs, size_t njobs, size_t k, bool verify) {
  constexpr size_t kCycleWords = 9, kTxnWords = 5, kGlobalWords = 90;  // RawPreflightCycle 36 B, txn 20 B
  const size_t n = size_t(1) << po2;
  const size_t data_words = size_t(211) * n;
  size_t cap_inj = 1, cap_txn = 1, cap_big = 4;
  for (size_t i = 0; i < njobs; i++) {
    const r0hip_trace_input* t = &jobs[i].trace;
    if (t->h_inj_index && t->inj_rows <= n) cap_inj = std::max<size_t>(cap_inj, t->h_inj_index[t->inj_rows]);
    cap_txn = std::max<size_t>(cap_txn, t->preflight.txns_len);
    cap_big = std::max<size_t>(cap_big, t->preflight.bigint_bytes_len);
  }
  std::vector<TraceSet> sets(k + 1);
  struct Events {
    std::vector<TraceSet>& sets;
    ~Events() {
      for (auto& s : sets)
        if (s.ev) (void)hipEventDestroy(s.ev);
    }
  } events{sets};
  for (auto& s : sets) {
    s.glob = DevBuf(kGlobalWords);
    s.index = DevBuf(n + 1);
    s.offsets = DevBuf(cap_inj);
    s.values = DevBuf(cap_inj);
    s.cycles = DevBuf(n * kCycleWords);
    s.txns = DevBuf(cap_txn * kTxnWords);
    s.bigint = DevBuf((cap_big + 3) / 4);
    HIP_OK(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming));
  }
  HIP_OK(hipDeviceSynchronize());  // allocations complete before other streams use them
  Queue free_q, ready_q;
  for (size_t s = 0; s < sets.size(); s++) free_q.put(long(s));

  std::thread uploader([&] {
    for (size_t i = 0; i < njobs; i++) {
      long s = free_q.get();
      TraceSet& b = sets[s];
      {
        std::lock_guard<std::mutex> lk(b.mu);
        b.job = i;
        b.landed = false;
      }
      ready_q.put(s);  // the prover fills its groups while the trace uploads
      try {
        ensure_init();
        const r0hip_trace_input& t = jobs[i].trace;
        const r0hip_raw_preflight_trace& pf = t.preflight;
        R0_REQUIRE(t.h_global && t.h_inj_index && pf.cycles, "trace job: null argument");
        R0_REQUIRE(t.inj_rows <= n, "trace job: injector longer than the segment");
        R0_REQUIRE((pf.txns_len == 0 || pf.txns) && (pf.bigint_bytes_len == 0 || pf.bigint_bytes),
                   "trace job: null trace array with a nonzero count");
        R0_REQUIRE(jobs[i].n_bigint == 0 || jobs[i].h_bigint, "trace job: h_bigint is NULL with n_bigint > 0");
        check_injector(t.h_inj_index, t.inj_rows, t.h_inj_offsets, t.h_inj_values, data_words, n);
        const size_t n_inj = t.h_inj_index[t.inj_rows];
        stage_reset();  // the previous job's staged copies have landed: the arena is free
        upload_async(b.glob.p, t.h_global, kGlobalWords * 4);
        upload_async(b.index.p, t.h_inj_index, (t.inj_rows + 1) * 4);
        upload_async(b.offsets.p, t.h_inj_offsets, n_inj * 4);
        upload_async(b.values.p, t.h_inj_values, n_inj * 4);
        upload_async(b.cycles.p, pf.cycles, n * kCycleWords * 4);
        upload_async(b.txns.p, pf.txns, size_t(pf.txns_len) * kTxnWords * 4);
        upload_async(b.bigint.p, pf.bigint_bytes, pf.bigint_bytes_len);
        HIP_OK(hipEventRecord(b.ev, stream()));
      } catch (const std::exception& e) {
        {
          std::lock_guard<std::mutex> lk(b.mu);
          if (!jobs[i].error) jobs[i].error = dup_msg(e.what());
        }
        drain_after_error();
      }
      b.mark();
    }
    // every copy done before the call returns: the caller may free its host buffers then
    drain_after_error();
    for (size_t t = 0; t < k; t++) ready_q.put(-1);
  });

  // the receipt check: finished seals queue here (job index and seal) for the verifier thread
  std::mutex vmu;
  std::condition_variable vcv;
  std::deque<std::pair<long, std::vector<uint32_t>>> vq;
  std::thread verifier;
  if (verify)
    verifier = std::thread([&] {
      for (;;) {
        std::pair<long, std::vector<uint32_t>> item;
        {
          std::unique_lock<std::mutex> lk(vmu);
          vcv.wait(lk, [&] { return !vq.empty(); });
          item = std::move(vq.front());
          vq.pop_front();
        }
        if (item.first < 0) return;
        r0hip_trace_job& j = jobs[item.first];
        const auto t0 = std::chrono::steady_clock::now();
        uint32_t got = 0;
        const char* err = r0hip_verify_seal("rv32im", suite, item.second.data(), item.second.size(), nullptr, 0,
                                            nullptr, &got);
        j.verify_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (!err && got != po2) err = dup_msg("the seal is of another segment size");
        std::lock_guard<std::mutex> lk(vmu);
        if (err) {
          if (!j.error) j.error = dup_msg((std::string("receipt verification failed: ") + err).c_str());
          free(const_cast<char*>(err));
        } else {
          j.verified = 1;
        }
      }
    });
  auto to_verifier = [&](long job, std::vector<uint32_t> seal) {
    {
      std::lock_guard<std::mutex> lk(vmu);
      vq.emplace_back(job, std::move(seal));
    }
    vcv.notify_one();
  };

  const long corrupt_job = [] {
    const char* e = getenv("R0HIP_TESTING_CORRUPT_SEAL_JOB");
    return e ? strtol(e, nullptr, 10) : -1L;
  }();
  auto prover = [&] {
    for (;;) {
      long s = ready_q.get();
      if (s < 0) return;
      TraceSet& b = sets[s];
      const long job = long(b.job);
      r0hip_trace_job& j = jobs[job];
      const r0hip_trace_input& tr = j.trace;
      const auto t0 = std::chrono::steady_clock::now();
      try {
        ensure_init();
        r0hip_raw_preflight_trace pf = tr.preflight;  // the set's device copies
        pf.cycles = b.cycles.p;
        pf.txns = pf.txns_len ? b.txns.p : nullptr;
        pf.bigint_bytes = pf.bigint_bytes_len ? reinterpret_cast<const uint8_t*>(b.bigint.p) : nullptr;
        std::vector<uint32_t> mix;
        std::vector<uint32_t> seal = prove_trace(
            suite, po2, tr.mode, b.glob.p, b.index.p, tr.inj_rows, b.offsets.p, b.values.p, &pf, j.h_bigint,
            j.n_bigint, true, &mix, [&](hipStream_t st) {
              b.wait_landed();
              {
                std::lock_guard<std::mutex> lk(b.mu);
                if (j.error) throw std::runtime_error(j.error);
              }
              HIP_OK(hipStreamWaitEvent(st, b.ev, 0));
            });
        HIP_OK(hipStreamSynchronize(stream()));
        j.prove_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        j.seal_len = seal.size();
        if (j.h_mix_out) memcpy(j.h_mix_out, mix.data(), mix.size() * 4);
        // TESTING ONLY (tests/test_rv32im_witgen_gpu.py): R0HIP_TESTING_CORRUPT_SEAL_JOB=i flips a
        // bit of job i's first Merkle root word, so its receipt check must fail that job alone
        if (job == corrupt_job && seal.size() > 92) seal[92] ^= 1u;
        R0_REQUIRE(!j.h_seal || seal.size() <= j.seal_cap, "seal buffer too small");
        if (j.h_seal) memcpy(j.h_seal, seal.data(), seal.size() * 4);
        if (verify) to_verifier(job, std::move(seal));
      } catch (const std::exception& e) {
        {
          std::lock_guard<std::mutex> lk(b.mu);
          if (!j.error) j.error = dup_msg(e.what());
        }
        drain_after_error();  // kernels queued before the throw may still read this set
      }
      b.wait_landed();  // the uploader is done with this job before the set is refilled
      free_q.put(s);
    }
  };
  run_provers(k, prover);
  uploader.join();
  if (verify) {
    to_verifier(-1, {});
    verifier.join();
  }
  for (size_t i = 0; i < njobs; i++)
    if (jobs[i].error) return dup_msg((std::string("segment ") + std::to_string(i) + ": " + jobs[i].error).c_str());
  return nullptr;
}

}  // namespace
}  // namespace r0

using namespace r0;

namespace {
const char* prove_segments_impl(const char* circuit, int suite, uint32_t po2, int write_version, uint32_t version,
                                r0hip_segment_job* jobs, size_t njobs, uint32_t in_flight) {
  try {
    const CircuitDef* c = find_circuit(circuit ? circuit : "");
    R0_REQUIRE(c, std::string("unknown circuit ") + (circuit ? circuit : "(null)"));
    R0_REQUIRE(suite >= 0 && suite <= 2, "unknown hash suite");
    R0_REQUIRE(po2 >= 1 && po2 <= 24, "po2 out of range");
    R0_REQUIRE(njobs == 0 || jobs, "jobs is NULL");
    ensure_init();
    if (njobs == 0) return nullptr;
    const size_t k = std::max<size_t>(1, std::min<size_t>(in_flight ? in_flight : 2, njobs));
    for (size_t i = 0; i < njobs; i++) {
      jobs[i].error = nullptr;
      jobs[i].seal_len = 0;
    }
    const bool device_accum_ok = std::string(c->name) == "rv32im";
    const size_t n = size_t(1) << po2;
    // group_sizes: accum 0, code 1, data 2 (the reference's register-group order)
    const size_t words[4] = {c->group_sizes[1] * n, c->group_sizes[2] * n, c->group_sizes[0] * n, c->output_size};
    std::vector<BufSet> sets(k + 1);
    struct Events {  // destroyed on every exit path
      std::vector<BufSet>& sets;
      ~Events() {
        for (auto& s : sets)
          for (auto& v : s.ev)
            for (auto e : v)
              if (e) (void)hipEventDestroy(e);
      }
    } events{sets};
    const size_t gcols[4] = {c->group_sizes[1], c->group_sizes[2], c->group_sizes[0], 1};
    for (auto& s : sets)
      for (int g = 0; g < 4; g++) {
        s.g[g] = DevBuf(words[g]);
        s.cols[g] = std::max<size_t>(1, gcols[g]);
        s.col_words[g] = g == 3 ? words[3] : n;
        s.ev[g].assign(s.chunks(g), nullptr);
        for (auto& e : s.ev[g]) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      }
    HIP_OK(hipDeviceSynchronize());  // allocations complete before other streams use them
    for (size_t i = 0; i < njobs; i++) {
      jobs[i].error = nullptr;
      jobs[i].seal_len = 0;
    }

    Queue free_q, ready_q;
    for (size_t s = 0; s < sets.size(); s++) free_q.put(long(s));

    std::thread uploader([&] {
      for (size_t i = 0; i < njobs; i++) {
        long s = free_q.get();
        BufSet& b = sets[s];
        b.job = i;
        {
          std::lock_guard<std::mutex> lk(b.mu);
          for (auto& q : b.queued) q = 0;  // the set is free: no prover waits on it
        }
        const uint32_t* src[4] = {jobs[i].h_code, jobs[i].h_data, jobs[i].h_accum, jobs[i].h_global};
        // rv32im without an accum group: the prover accumulates on the device
        const bool dev_accum = !src[2] && device_accum_ok;
        bool null_group = false;
        for (int g = 0; g < 4; g++) null_group |= !src[g] && !(g == 2 && dev_accum);
        if (null_group) jobs[i].error = dup_msg("witness group pointer is NULL");  // before the hand-over
        else if (jobs[i].n_bigint && (!dev_accum || !jobs[i].h_bigint))
          // the states need the mix drawn inside the proof: only a device accumulation takes them
          jobs[i].error = dup_msg("BigInt backs given without a device accumulation (h_accum must be NULL, rv32im)");
        null_group |= jobs[i].error != nullptr;
        ready_q.put(s);  // a prover may start now; it waits per group (BufSet::wait)
        if (null_group) {
          b.mark_all();
          continue;
        }
        try {
          ensure_init();
          // in the order the prover first touches them (globals, code, data, accum), each in
          // column chunks, so a segment's commits run while its later columns still upload
          for (int g : {3, 0, 1, 2}) {
            if (g == 2 && dev_accum) {
              b.mark(g, b.chunks(g));  // nothing to upload; the prover never waits on it
              continue;
            }
            for (size_t k = 0; k < b.chunks(g); k++) {
              const size_t c0 = k * kChunkCols, cc = std::min(kChunkCols, b.cols[g] - c0);
              HIP_OK(hipMemcpyAsync(b.g[g].p + c0 * b.col_words[g], src[g] + c0 * b.col_words[g],
                                    cc * b.col_words[g] * 4, hipMemcpyHostToDevice, stream()));
              HIP_OK(hipEventRecord(b.ev[g][k], stream()));
              b.mark(g, k + 1);
            }
          }
        } catch (const std::exception& e) {
          {
            std::lock_guard<std::mutex> lk(b.mu);
            if (!jobs[i].error) jobs[i].error = dup_msg(e.what());
          }
          // the job's earlier chunks may still be copying: no prover waits on them now, and
          // the set goes back to the free queue once the prover sees the error
          drain_after_error();
          b.mark_all();  // release a waiting prover; the job reports the error
        }
      }
      // every copy done before the call can return: a prover that failed early never waited
      // on its job's events, and the caller may free its host buffers once we return (free
      // on the success path, where every event was waited on)
      drain_after_error();
      for (size_t t = 0; t < k; t++) ready_q.put(-1);  // one stop token per prover
    });

    auto prover = [&] {
      for (;;) {
        long s = ready_q.get();
        if (s < 0) return;
        BufSet& b = sets[s];
        r0hip_segment_job& j = jobs[b.job];
        // j.error is written by the uploader under b.mu while this job's copies are queued
        auto failed = [&] {
          std::lock_guard<std::mutex> lk(b.mu);
          return j.error != nullptr;
        };
        if (!failed()) {
          try {
            ensure_init();
            std::vector<uint32_t> mix;
            const bool dev_accum = !j.h_accum;  // (rv32im only: checked by the uploader)
            const AccumStep acc{b.g[2].p, n, true, j.h_bigint, j.n_bigint};
            std::vector<uint32_t> seal =
                prove_segment(*c, suite, po2, b.g[0].p, b.g[1].p, dev_accum ? nullptr : b.g[2].p, b.g[3].p,
                              write_version != 0, version, &mix, &b, dev_accum ? &acc : nullptr);
            HIP_OK(hipStreamSynchronize(stream()));
            if (!failed()) {  // an upload error leaves the proof meaningless: drop it
              j.seal_len = seal.size();
              if (j.h_mix_out) memcpy(j.h_mix_out, mix.data(), mix.size() * 4);
              R0_REQUIRE(!j.h_seal || seal.size() <= j.seal_cap, "seal buffer too small");
              if (j.h_seal) memcpy(j.h_seal, seal.data(), seal.size() * 4);
            }
          } catch (const std::exception& e) {
            {
              std::lock_guard<std::mutex> lk(b.mu);
              if (!j.error) j.error = dup_msg(e.what());
            }
            // kernels queued before the throw may still read this buffer set: drain
            // them before the uploader refills it
            drain_after_error();
          }
        }
        free_q.put(s);
      }
    };
    run_provers(k, prover);
    uploader.join();
    for (size_t i = 0; i < njobs; i++)
      if (jobs[i].error) return dup_msg((std::string("segment ") + std::to_string(i) + ": " + jobs[i].error).c_str());
    return nullptr;
  } catch (const std::exception& e) {
    return dup_msg(e.what());
  } catch (...) {
    return dup_msg("r0hip: unknown error");
  }
}
}  // namespace

extern "C" const char* r0hip_prove_segments(const char* circuit, int suite, uint32_t po2, int write_version,
                                            uint32_t version, r0hip_segment_job* jobs, size_t njobs,
                                            uint32_t in_flight) {
  const char* err = prove_segments_impl(circuit, suite, po2, write_version, version, jobs, njobs, in_flight);
  // the buffer sets are freed; the calling thread (one of the provers) keeps no device memory
  drain_after_error();
  release_thread_memory();
  return err;
}

extern "C" const char* r0hip_prove_trace_segments(int suite, uint32_t po2, r0hip_trace_job* jobs, size_t njobs,
                                                  uint32_t in_flight, int verify) {
  const char* err = nullptr;
  try {
    R0_REQUIRE(suite >= 0 && suite <= 2, "unknown hash suite");
    R0_REQUIRE(po2 >= 2 && po2 <= 24, "po2 out of range");
    R0_REQUIRE(njobs == 0 || jobs, "jobs is NULL");
    ensure_init();
    for (size_t i = 0; i < njobs; i++) {
      jobs[i].error = nullptr;
      jobs[i].seal_len = 0;
      jobs[i].verified = 0;
      jobs[i].verify_ms = 0;
      jobs[i].prove_ms = 0;
    }
    if (njobs) {
      const size_t k = std::max<size_t>(1, std::min<size_t>(in_flight ? in_flight : 2, njobs));
      err = prove_trace_jobs(suite, po2, jobs, njobs, k, verify != 0);
    }
  } catch (const std::exception& e) {
    err = dup_msg(e.what());
  } catch (...) {
    err = dup_msg("r0hip: unknown error");
  }
  // the trace sets are freed; the calling thread (one of the provers) keeps no device memory
  drain_after_error();
  release_thread_memory();
  return err;
}
