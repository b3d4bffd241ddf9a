// device.h — RAII device memory over the C-ABI, and loud error mapping.
#pragma once

#include <cstddef>
#include <stdexcept>
#include <string>
#include <utility>

#include "openr_gpu.h"

namespace openr_amd {

// Every C-ABI failure becomes an exception: the product has no CPU path to
// fall back to, so a missing device or an unsupported input must be loud.
inline void ogsCheck(int rc, const char* what) {
  if (rc == OGS_OK) return;
  std::string msg = std::string(what) + " failed (" + std::to_string(rc) +
      "): " + ogs_last_error();
  if (rc == OGS_E_UNSUPPORTED) throw std::domain_error(msg);
  if (rc == OGS_E_INVALID) throw std::invalid_argument(msg);
  throw std::runtime_error(msg);
}

class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  explicit DeviceBuffer(size_t bytes) { resize(bytes); }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  DeviceBuffer(DeviceBuffer&& o) noexcept { swap(o); }
  DeviceBuffer& operator=(DeviceBuffer&& o) noexcept {
    swap(o);
    return *this;
  }
  ~DeviceBuffer() {
    if (owned_) ogs_free(ptr_);
  }

  // non-owning view of `bytes` at `base` (a span of a packed block that
  // outlives it); growing past the span re-homes it into its own allocation
  void view(void* base, size_t bytes) {
    if (owned_) ogs_free(ptr_);
    ptr_ = base;
    cap_ = size_ = bytes;
    owned_ = false;
  }

  size_t capacity() const { return cap_; }
  void resize(size_t bytes) {  // grow-only, contents kept within capacity()
    if (bytes <= cap_) {
      size_ = bytes;
      return;
    }
    if (owned_) ogs_free(ptr_);
    ptr_ = nullptr;
    cap_ = size_ = 0;
    owned_ = true;
    ogsCheck(ogs_malloc(&ptr_, bytes), "ogs_malloc");
    cap_ = size_ = bytes;
  }
  template <typename T>
  void upload(const T* host, size_t count, void* stream = nullptr) {
    if (count == 0) {  // keep a valid (never read) allocation
      resize(16);
      return;
    }
    resize(count * sizeof(T));
    ogsCheck(ogs_memcpy_h2d(ptr_, host, count * sizeof(T), stream),
             "ogs_memcpy_h2d");
  }
  template <typename T>
  void download(T* host, size_t count, void* stream = nullptr) const {
    ogsCheck(ogs_memcpy_d2h(host, ptr_, count * sizeof(T), stream),
             "ogs_memcpy_d2h");
  }
  void* get() const { return ptr_; }
  template <typename T>
  T* as() const {
    return static_cast<T*>(ptr_);
  }
  size_t size() const { return size_; }

 private:
  void swap(DeviceBuffer& o) noexcept {
    std::swap(ptr_, o.ptr_);
    std::swap(size_, o.size_);
    std::swap(cap_, o.cap_);
    std::swap(owned_, o.owned_);
  }
  void* ptr_{nullptr};
  size_t size_{0}, cap_{0};
  bool owned_{true};
};

// Process-wide cache of page-locked blocks: page-locking is a syscall +
// page-table update (tens of microseconds), a solver's staging blocks are
// recycled instead. Owners synchronise their transfers before release.
void* pinnedAcquire(size_t bytes, size_t* cap);
void pinnedRelease(void* p, size_t cap);

// Page-locked host block (grow-only, contents not preserved): the staging
// side of one-transfer H2D / D2H round trips.
class PinnedBuffer {
 public:
  PinnedBuffer() = default;
  PinnedBuffer(const PinnedBuffer&) = delete;
  PinnedBuffer& operator=(const PinnedBuffer&) = delete;
  ~PinnedBuffer() { pinnedRelease(ptr_, cap_); }
  void resize(size_t bytes) {
    if (bytes <= cap_) return;
    pinnedRelease(ptr_, cap_);
    ptr_ = nullptr;
    cap_ = 0;
    ptr_ = pinnedAcquire(bytes, &cap_);
  }
  template <typename T>
  T* at(size_t byteOffset) const {
    return reinterpret_cast<T*>(static_cast<char*>(ptr_) + byteOffset);
  }
  void* get() const { return ptr_; }

 private:
  void* ptr_{nullptr};
  size_t cap_{0};
};

// byte offset `off` into a device block
template <typename T>
inline T* devAt(const DeviceBuffer& b, size_t off) {
  return reinterpret_cast<T*>(static_cast<char*>(b.get()) + off);
}

}  // namespace openr_amd
