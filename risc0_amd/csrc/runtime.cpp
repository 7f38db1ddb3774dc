// Process-wide HIP runtime state: device selection, the single ordered stream,
// a size-keyed device-buffer pool, cached constant tables and growable scratch.
#include "runtime.h"

#include <algorithm>
#include <cstring>
#include <cstdio>
#include <map>
#include <tuple>
#include <mutex>
#include <unordered_map>

#include "devmem.h"

namespace r0 {

namespace {
std::mutex g_mu;
hipStream_t g_stream = nullptr;
int g_device = -1;
std::unordered_map<std::string, uint32_t*> g_tables;
struct Scratch {
  void* p = nullptr;
  size_t bytes = 0;
};
std::map<int, Scratch> g_scratch;
std::multimap<size_t, void*> g_pool;  // free blocks by size
std::unordered_map<void*, size_t> g_live;
}  // namespace

void ensure_init() {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_stream) return;
  if (g_device < 0) {
    int n = 0;
    HIP_OK(hipGetDeviceCount(&n));
    R0_REQUIRE(n > 0, "no HIP device visible");
    g_device = 0;
  }
  HIP_OK(hipSetDevice(g_device));
  HIP_OK(hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking));
}

void set_device(int ordinal) {
  {
    std::lock_guard<std::mutex> lk(g_mu);
    R0_REQUIRE(!g_stream || ordinal == g_device, "r0hip already initialised on another device");
    g_device = ordinal;
  }
  ensure_init();
}

hipStream_t stream() {
  ensure_init();
  return g_stream;
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
  HIP_OK(hipMalloc(&d, host.size() * 4));
  HIP_OK(hipMemcpy(d, host.data(), host.size() * 4, hipMemcpyHostToDevice));
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_tables.find(key);
  if (it != g_tables.end()) {
    (void)hipFree(d);
    return it->second;
  }
  g_tables[key] = d;
  return d;
}

void* scratch(size_t bytes, int slot) {
  ensure_init();
  std::lock_guard<std::mutex> lk(g_mu);
  Scratch& s = g_scratch[slot];
  if (s.bytes < bytes) {
    if (s.p) {
      HIP_OK(hipStreamSynchronize(g_stream));  // last user of the old block must be done
      HIP_OK(hipFree(s.p));
    }
    size_t want = bytes < 4096 ? 4096 : bytes + bytes / 4;
    HIP_OK(hipMalloc(&s.p, want));
    s.bytes = want;
  }
  return s.p;
}

// ---- pinned staging for async uploads ---------------------------------------
namespace {
struct Stage {
  uint8_t* base = nullptr;
  size_t cap = 0, used = 0;
};
Stage g_stage;
std::vector<uint8_t*> g_stage_old;
}  // namespace

void upload_async(void* d_dst, const void* h_src, size_t bytes) {
  if (!bytes) return;
  ensure_init();
  std::lock_guard<std::mutex> lk(g_mu);
  size_t need = (bytes + 255) & ~size_t(255);
  if (g_stage.used + need > g_stage.cap) {
    // keep the old arena alive (queued copies may still read it) until stage_reset
    if (g_stage.base) g_stage_old.push_back(g_stage.base);
    size_t cap = std::max<size_t>(size_t(64) << 20, need * 2);
    void* p = nullptr;
    HIP_OK(hipHostMalloc(&p, cap, hipHostMallocDefault));
    g_stage.base = static_cast<uint8_t*>(p);
    g_stage.cap = cap;
    g_stage.used = 0;
  }
  uint8_t* h = g_stage.base + g_stage.used;
  g_stage.used += need;
  memcpy(h, h_src, bytes);
  HIP_OK(hipMemcpyAsync(d_dst, h, bytes, hipMemcpyHostToDevice, g_stream));
}

void stage_reset() {
  if (g_stream) HIP_OK(hipStreamSynchronize(g_stream));
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto* p : g_stage_old) (void)hipHostFree(p);
  g_stage_old.clear();
  g_stage.used = 0;
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
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_pool.find(bytes);
    if (it != g_pool.end()) {
      void* p = it->second;
      g_pool.erase(it);
      g_live[p] = bytes;
      return p;
    }
  }
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, bytes);
  if (e != hipSuccess) {
    // release pooled blocks and retry once
    dev_trim();
    HIP_OK(hipMalloc(&p, bytes));
  }
  std::lock_guard<std::mutex> lk(g_mu);
  g_live[p] = bytes;
  return p;
}

void dev_free(void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_live.find(p);
  if (it == g_live.end()) return;
  g_pool.emplace(it->second, p);
  g_live.erase(it);
}

void dev_trim() {
  if (g_stream) HIP_OK(hipStreamSynchronize(g_stream));
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& kv : g_pool) (void)hipFree(kv.second);
  g_pool.clear();
}

}  // namespace r0
