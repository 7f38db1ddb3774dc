// Device buffers for the host driver: pooled allocations (the bench proves the
// same shapes back to back, so blocks are recycled by exact size instead of
// paying hipMalloc/hipFree per segment) and a small RAII owner.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace r0 {

void* dev_alloc(size_t bytes);
void dev_free(void* p);
void dev_trim();  // return pooled blocks to the driver
// page-locked host buffers (r0hip_host_alloc): freed blocks are kept pinned for reuse,
// host_trim() returns the idle ones to the driver
void* host_alloc(size_t bytes);
void host_free(void* p);
void host_trim();
void set_device(int ordinal);

// RAII buffer of u32 words.
struct DevBuf {
  uint32_t* p = nullptr;
  size_t words = 0;
  DevBuf() = default;
  explicit DevBuf(size_t w) : p(static_cast<uint32_t*>(dev_alloc(w * 4))), words(w) {}
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), words(o.words) {
    o.p = nullptr;
    o.words = 0;
  }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) {
      dev_free(p);
      p = o.p;
      words = o.words;
      o.p = nullptr;
      o.words = 0;
    }
    return *this;
  }
  ~DevBuf() { dev_free(p); }
};

}  // namespace r0
