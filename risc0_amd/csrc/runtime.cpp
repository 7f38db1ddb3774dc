// HIP runtime state. Process-wide: device selection and cached constant tables.
// Per host thread: the thread's ordered stream, its size-keyed device-buffer pool,
// growable scratch and pinned upload arena — so several host threads can each run
// whole segment proofs concurrently on one GPU (segments in flight), and a block
// freed on one stream is only ever reused on that same stream.
#include "runtime.h"

#include <algorithm>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <tuple>
#include <mutex>
#include <thread>
#include <unordered_map>

#include <atomic>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "devmem.h"

namespace r0 {

namespace {
std::mutex g_mu;
int g_device = -1;
bool g_device_fixed = false;
std::unordered_map<std::string, uint32_t*> g_tables;
std::unordered_map<void*, size_t> g_live;  // every pooled allocation -> bytes
struct Scratch {
  void* p = nullptr;
  size_t bytes = 0;
};
struct Stage {
  uint8_t* base = nullptr;
  size_t cap = 0, used = 0;
};
// blocks left by exited threads (their stream was drained), reusable by anyone: pool
// blocks by size, scratch blocks by (slot, size) — kept apart so a new thread's scratch
// never takes the block its own dev_alloc of the same phase is about to need
std::multimap<size_t, void*> g_orphans;
std::map<int, std::multimap<size_t, void*>> g_scratch_orphans;
std::thread::id g_main_thread;
std::vector<hipStream_t> g_free_streams;  // streams of exited threads (drained)
std::vector<Stage> g_free_stages;         // their pinned upload arenas
// MemStats counters (see mem_stats)
std::atomic<uint64_t> g_mem_live{0}, g_peak_live{0}, g_reserved{0}, g_peak_reserved{0}, g_mallocs{0};

struct ThreadCtx {
  hipStream_t stream = nullptr;
  std::map<int, Scratch> scratch;
  std::multimap<size_t, void*> pool;  // free blocks by size, last used on `stream`
  Stage stage;
  std::vector<uint8_t*> stage_old;
  // the idle pool and scratch blocks to the shared lists (caller holds g_mu; stream drained)
  void hand_back_memory() {
    for (auto& kv : pool) g_orphans.emplace(kv.first, kv.second);
    for (auto& kv : scratch)
      if (kv.second.p) {
        g_scratch_orphans[kv.first].emplace(kv.second.bytes, kv.second.p);
        g_mem_live.fetch_sub(kv.second.bytes, std::memory_order_relaxed);
      }
    pool.clear();
    scratch.clear();
  }
  ~ThreadCtx() {
    // A worker thread hands its stream and memory over when it exits — no HIP calls
    // here (thread-exit destructors run after tools' per-thread state is gone). Every
    // API call drains its stream before returning, so the blocks are idle. The main
    // thread's context dies in process teardown and is left alone.
    if (!stream || std::this_thread::get_id() == g_main_thread) return;
    std::lock_guard<std::mutex> lk(g_mu);
    hand_back_memory();
    g_free_streams.push_back(stream);
    if (stage.base) g_free_stages.push_back(Stage{stage.base, stage.cap, 0});
    // superseded arenas in stage_old are left allocated (rare: only after growth)
  }
};
thread_local ThreadCtx t_ctx;

// ---- accounting (MemStats) ----
void raise_peak(std::atomic<uint64_t>& peak, uint64_t v) {
  uint64_t cur = peak.load(std::memory_order_relaxed);
  while (v > cur && !peak.compare_exchange_weak(cur, v, std::memory_order_relaxed)) {
  }
}
void live_add(uint64_t b) { raise_peak(g_peak_live, g_mem_live.fetch_add(b, std::memory_order_relaxed) + b); }
void live_sub(uint64_t b) { g_mem_live.fetch_sub(b, std::memory_order_relaxed); }
// every device allocation of the library goes through these two
// R0HIP_TRACE_MALLOC=1: every device allocation to stderr with its scratch slot (-1: the
// block pool or a table), for finding allocations in a steady state
const bool g_trace_malloc = std::getenv("R0HIP_TRACE_MALLOC") != nullptr;

hipError_t counted_malloc(void** p, size_t bytes, int slot = -1) {
  const hipError_t e = hipMalloc(p, bytes);
  if (g_trace_malloc) std::fprintf(stderr, "r0hip malloc %zu bytes slot %d -> %d\n", bytes, slot, int(e));
  if (e == hipSuccess) {
    g_mallocs.fetch_add(1, std::memory_order_relaxed);
    raise_peak(g_peak_reserved, g_reserved.fetch_add(bytes, std::memory_order_relaxed) + bytes);
  }
  return e;
}
void counted_free(void* p, size_t bytes) {
  if (hipFree(p) == hipSuccess) g_reserved.fetch_sub(bytes, std::memory_order_relaxed);
}
}  // namespace

MemStats mem_stats() {
  return MemStats{g_mem_live.load(), g_peak_live.load(), g_reserved.load(), g_peak_reserved.load(), g_mallocs.load()};
}
void mem_reset_peak() {
  g_peak_live.store(g_mem_live.load());
  g_peak_reserved.store(g_reserved.load());
}

Span::Span(const char* name) { roctxRangePushA(name); }
Span::~Span() { roctxRangePop(); }

void ensure_init() {
  if (t_ctx.stream) return;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_device < 0) {
      int n = 0;
      HIP_OK(hipGetDeviceCount(&n));
      R0_REQUIRE(n > 0, "no HIP device visible");
      g_device = 0;
    }
    if (!g_device_fixed) g_main_thread = std::this_thread::get_id();
    g_device_fixed = true;
  }
  HIP_OK(hipSetDevice(g_device));  // the current device is per host thread
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_free_streams.empty()) {
      t_ctx.stream = g_free_streams.back();
      g_free_streams.pop_back();
    }
    if (!g_free_stages.empty()) {
      t_ctx.stage = g_free_stages.back();
      g_free_stages.pop_back();
    }
  }
  if (!t_ctx.stream) HIP_OK(hipStreamCreateWithFlags(&t_ctx.stream, hipStreamNonBlocking));
}

void set_device(int ordinal) {
  {
    std::lock_guard<std::mutex> lk(g_mu);
    R0_REQUIRE(!g_device_fixed || ordinal == g_device, "r0hip already initialised on another device");
    g_device = ordinal;
  }
  ensure_init();
}

hipStream_t stream() {
  ensure_init();
  return t_ctx.stream;
}

hipStream_t copy_stream() {
  ensure_init();
  static hipStream_t s = [] {
    hipStream_t c = nullptr;
    HIP_OK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
    return c;
  }();
  return s;
}

void drain_after_error() noexcept {
  if (t_ctx.stream) (void)hipStreamSynchronize(t_ctx.stream);
}

void release_thread_memory() noexcept {
  if (!t_ctx.stream) return;
  std::lock_guard<std::mutex> lk(g_mu);
  t_ctx.hand_back_memory();
}

const uint32_t* dev_table(const std::string& key, const std::function<std::vector<uint32_t>()>& gen) {
  ensure_init();
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_tables.find(key);
    if (it != g_tables.end()) return it->second;
  }
  std::vector<uint32_t> host = gen();
  uint32_t* d = nullptr;
  HIP_OK(counted_malloc(reinterpret_cast<void**>(&d), host.size() * 4));
  HIP_OK(hipMemcpy(d, host.data(), host.size() * 4, hipMemcpyHostToDevice));
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_tables.find(key);
  if (it != g_tables.end()) {
    counted_free(d, host.size() * 4);
    return it->second;
  }
  g_tables[key] = d;
  return d;
}

void* scratch(size_t bytes, int slot) {
  ensure_init();
  Scratch& s = t_ctx.scratch[slot];
  if (s.bytes < bytes) {
    if (s.p) {
      // the last user of the old block must be done; the block goes back to the slot's
      // orphans (some slots hold data-dependent sizes, e.g. upload vectors, so a thread that
      // took another thread's smaller leftover grows here; freeing it would make the next
      // thread hipMalloc again). dev_trim releases orphans under memory pressure.
      HIP_OK(hipStreamSynchronize(t_ctx.stream));
      std::lock_guard<std::mutex> lk(g_mu);
      g_scratch_orphans[slot].emplace(s.bytes, s.p);
      live_sub(s.bytes);
    }
    size_t want = bytes < 4096 ? 4096 : bytes + bytes / 4;
    s.p = nullptr;
    {
      // a block left by an exited thread (bench and pipeline threads come and go; each
      // new one would otherwise hipMalloc its eval_check scratch again, GBs at po2 >= 20)
      std::lock_guard<std::mutex> lk(g_mu);
      auto& orph = g_scratch_orphans[slot];
      auto ot = orph.find(want);  // the size this request allocates itself, else the best fit
      if (ot == orph.end()) ot = orph.lower_bound(bytes);
      // at most 8x the block this request would allocate: a po2=10 proof must not pin a
      // po2=24 block (it would stay live and count in mem_stats), while a slot whose proof
      // asks small first and then grows (eval_check's, 5.6x between its two requests) still
      // finds the block another thread grew
      if (ot != orph.end() && ot->first <= 8 * want) {
        s.p = ot->second;
        want = ot->first;
        orph.erase(ot);
      }
    }
    if (!s.p && counted_malloc(&s.p, want, slot) != hipSuccess) {
      dev_trim();
      HIP_OK(counted_malloc(&s.p, want, slot));
    }
    s.bytes = want;
    live_add(want);
  }
  return s.p;
}

// ---- pinned staging for async uploads (per thread) ---------------------------

namespace {
// `bytes` of this thread's page-locked arena (a new, larger arena when it is full; the old one
// stays alive for copies still queued from it until stage_reset)
uint8_t* stage_take(size_t bytes) {
  Stage& st = t_ctx.stage;
  size_t need = (bytes + 255) & ~size_t(255);
  if (st.used + need > st.cap) {
    if (st.base) t_ctx.stage_old.push_back(st.base);
    size_t cap = std::max<size_t>(size_t(64) << 20, need * 2);
    void* p = nullptr;
    HIP_OK(hipHostMalloc(&p, cap, hipHostMallocDefault));
    st.base = static_cast<uint8_t*>(p);
    st.cap = cap;
    st.used = 0;
  }
  uint8_t* h = st.base + st.used;
  st.used += need;
  return h;
}
}  // namespace

void upload_async(void* d_dst, const void* h_src, size_t bytes) {
  if (!bytes) return;
  ensure_init();
  // source inside a live r0hip_host_alloc block: already page-locked, copy it directly (the
  // callers keep their sources alive until the stream has drained: every entry point that
  // takes host arrays returns only after its work is done)
  if (bytes >= (size_t(64) << 10) && host_pinned(h_src, bytes)) {
    HIP_OK(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, t_ctx.stream));
    return;
  }
  uint8_t* h = stage_take(bytes);
  memcpy(h, h_src, bytes);
  HIP_OK(hipMemcpyAsync(d_dst, h, bytes, hipMemcpyHostToDevice, t_ctx.stream));
}

void upload(void* d_dst, const void* h_src, size_t bytes) {
  ensure_init();
  hipStream_t s = t_ctx.stream;
  if (!bytes || bytes > (size_t(256) << 10) || host_pinned(h_src, bytes)) {
    HIP_OK(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, s));
    HIP_OK(hipStreamSynchronize(s));
    return;
  }
  Stage& st = t_ctx.stage;
  const uint8_t* base = st.base;
  const size_t mark = st.used;
  uint8_t* h = stage_take(bytes);
  memcpy(h, h_src, bytes);
  HIP_OK(hipMemcpyAsync(d_dst, h, bytes, hipMemcpyHostToDevice, s));
  HIP_OK(hipStreamSynchronize(s));
  if (st.base == base) st.used = mark;
}

void download(void* h_dst, const void* d_src, size_t bytes) {
  ensure_init();
  hipStream_t s = t_ctx.stream;
  // a small copy into pageable memory takes the runtime's staged path, about twice as long as a
  // copy into page-locked memory followed by a host memcpy (25 against 13 us for 32 B,
  // profiles/r6d_small_d2h.txt); larger or pinned destinations are copied directly
  if (!bytes || bytes > (size_t(256) << 10) || host_pinned(h_dst, bytes)) {
    HIP_OK(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    return;
  }
  Stage& st = t_ctx.stage;
  const uint8_t* base = st.base;
  const size_t mark = st.used;
  uint8_t* h = stage_take(bytes);
  HIP_OK(hipMemcpyAsync(h, d_src, bytes, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  memcpy(h_dst, h, bytes);
  if (st.base == base) st.used = mark;  // the bounce space is free again (same arena)
}

void stage_reset() {
  if (t_ctx.stream) HIP_OK(hipStreamSynchronize(t_ctx.stream));
  for (auto* p : t_ctx.stage_old) (void)hipHostFree(p);
  t_ctx.stage_old.clear();
  t_ctx.stage.used = 0;
}

// ---- kernel timing -----------------------------------------------------------
namespace {
struct KRec {
  std::string name;
  double bytes, mm;
  hipEvent_t a, b;
};
bool g_kt_on = false;
std::vector<KRec> g_kt;
}  // namespace

void ktimer_enable(bool on) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_kt_on = on;
}

KScope::KScope(const char* name, double bytes, double mm) {
  if (!g_kt_on) return;
  KRec r{name, bytes, mm, nullptr, nullptr};
  HIP_OK(hipEventCreate(&r.a));
  HIP_OK(hipEventCreate(&r.b));
  HIP_OK(hipEventRecord(r.a, stream()));
  std::lock_guard<std::mutex> lk(g_mu);
  idx = int(g_kt.size());
  g_kt.push_back(r);
}

KScope::~KScope() {
  if (idx < 0) return;
  hipEvent_t b;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    b = g_kt[idx].b;
  }
  (void)hipEventRecord(b, stream());
}

std::string ktimer_report() {
  HIP_OK(hipStreamSynchronize(stream()));
  std::lock_guard<std::mutex> lk(g_mu);
  std::map<std::string, std::tuple<double, int, double, double>> agg;
  for (auto& r : g_kt) {
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, r.a, r.b));
    auto& t = agg[r.name];
    std::get<0>(t) += ms;
    std::get<1>(t) += 1;
    std::get<2>(t) += r.bytes;
    std::get<3>(t) += r.mm;
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  g_kt.clear();
  std::string out;
  for (auto& kv : agg) {
    char buf[256];
    snprintf(buf, sizeof(buf), "%s=%.6f:%d:%.0f:%.0f;", kv.first.c_str(), std::get<0>(kv.second),
             std::get<1>(kv.second), std::get<2>(kv.second), std::get<3>(kv.second));
    out += buf;
  }
  return out;
}

// ---- pooled device buffers ---------------------------------------------------
void* dev_alloc(size_t bytes) {
  ensure_init();
  if (bytes == 0) bytes = 16;
  bytes = (bytes + 255) & ~size_t(255);
  {
    // best fit, exact or up to 25% larger, as for the orphans below: a block taken from the
    // orphans at its own (larger) size comes back here under that size, and an exact-size
    // lookup would then miss it and allocate again in a steady state
    // an exact size first, then the best fit up to 25% larger: a request that takes a larger
    // block than it needs can leave another thread's request for that size without one (the
    // threads of a batch race for the blocks exited threads left)
    auto it = t_ctx.pool.find(bytes);
    if (it == t_ctx.pool.end()) it = t_ctx.pool.lower_bound(bytes);
    if (it != t_ctx.pool.end() && it->first <= bytes + bytes / 4) {
      void* p = it->second;
      const size_t have = it->first;
      t_ctx.pool.erase(it);
      live_add(have);
      std::lock_guard<std::mutex> lk(g_mu);
      g_live[p] = have;
      return p;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    auto ot = g_orphans.find(bytes);  // exact, else up to 25% larger
    if (ot == g_orphans.end()) ot = g_orphans.lower_bound(bytes);
    if (ot != g_orphans.end() && ot->first <= bytes + bytes / 4) {
      void* p = ot->second;
      g_live[p] = ot->first;
      live_add(ot->first);
      g_orphans.erase(ot);
      return p;
    }
  }
  void* p = nullptr;
  hipError_t e = counted_malloc(&p, bytes);
  if (e != hipSuccess) {
    // release pooled blocks and retry once
    dev_trim();
    HIP_OK(counted_malloc(&p, bytes));
  }
  live_add(bytes);
  std::lock_guard<std::mutex> lk(g_mu);
  g_live[p] = bytes;
  return p;
}

void dev_free(void* p) {
  if (!p) return;
  size_t bytes;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_live.find(p);
    if (it == g_live.end()) return;
    bytes = it->second;
    g_live.erase(it);
  }
  live_sub(bytes);
  t_ctx.pool.emplace(bytes, p);  // reused only by this thread, i.e. on this stream
}

// ---- page-locked host memory (r0hip_host_alloc / r0hip_host_free) ----------------
// Freed blocks stay page-locked in a size-keyed list for the next request instead of going
// back through hipHostFree. Unpinning host memory is not free for the device: after the
// bench's end-to-end leg released its 2.2 GB of pinned witness buffers, every later proof
// in the process ran 10-15 ms slower (a kernel early in each proof ran 20-30x longer while
// the other stream's kernels could not start), and keeping those buffers
// pinned removed the slowdown. r0hip_trim releases the list.
namespace {
std::mutex g_host_mu;
std::multimap<size_t, void*> g_host_free;
std::map<void*, size_t> g_host_size;
std::set<void*> g_host_idle;  // the blocks now on g_host_free (a second free must not list one twice)
}  // namespace

void* host_alloc(size_t bytes) {
  if (bytes == 0) bytes = 1;
  {
    std::lock_guard<std::mutex> lk(g_host_mu);
    auto it = g_host_free.lower_bound(bytes);
    if (it != g_host_free.end() && it->first <= 2 * bytes) {
      void* p = it->second;
      g_host_free.erase(it);
      g_host_idle.erase(p);
      return p;
    }
  }
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
    host_trim();  // pinned memory is a system resource: give back the idle blocks, retry once
    HIP_OK(hipHostMalloc(&p, bytes, hipHostMallocDefault));
  }
  std::lock_guard<std::mutex> lk(g_host_mu);
  g_host_size[p] = bytes;
  return p;
}

// [p, p + bytes) lies inside one live (not freed) r0hip_host_alloc block
bool host_pinned(const void* p, size_t bytes) {
  std::lock_guard<std::mutex> lk(g_host_mu);
  auto it = g_host_size.upper_bound(const_cast<void*>(p));
  if (it == g_host_size.begin()) return false;
  --it;
  const auto* base = static_cast<const uint8_t*>(it->first);
  const auto* q = static_cast<const uint8_t*>(p);
  return q >= base && q + bytes <= base + it->second && !g_host_idle.count(it->first);
}

void host_free(void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_host_mu);
  auto it = g_host_size.find(p);
  R0_REQUIRE(it != g_host_size.end(), "r0hip_host_free: pointer was not returned by r0hip_host_alloc");
  R0_REQUIRE(g_host_idle.insert(p).second, "r0hip_host_free: block is already free (double free)");
  g_host_free.emplace(it->second, p);
}

void host_trim() {
  std::vector<void*> release;
  {
    std::lock_guard<std::mutex> lk(g_host_mu);
    for (auto& kv : g_host_free) {
      release.push_back(kv.second);
      g_host_size.erase(kv.second);
    }
    g_host_free.clear();
    g_host_idle.clear();
  }
  for (void* p : release) (void)hipHostFree(p);
}

void dev_trim() {
  if (t_ctx.stream) HIP_OK(hipStreamSynchronize(t_ctx.stream));
  for (auto& kv : t_ctx.pool) counted_free(kv.second, kv.first);
  t_ctx.pool.clear();
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& kv : g_orphans) counted_free(kv.second, kv.first);
  g_orphans.clear();
  for (auto& sl : g_scratch_orphans)
    for (auto& kv : sl.second) counted_free(kv.second, kv.first);
  g_scratch_orphans.clear();
}

}  // namespace r0
