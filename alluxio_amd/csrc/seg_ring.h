// Persistent descriptor ring for batched_copy_kernel launches.
//
// A launch reads its CopySeg descriptors from device memory.  Allocating them per call (hipMalloc
// + hipFree, which can synchronize the whole device) was the old pattern; instead every owner
// keeps kSlots pinned-host / device descriptor buffers and an event per buffer.  A buffer is
// reused only after the event recorded behind its previous launch has completed, so launches
// stay asynchronous and any number of streams may use the ring concurrently.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "kernels.h"

namespace amdx {

class SegRing {
 public:
  static constexpr int kSlots = 8;
  static constexpr size_t kSegs = 8192;

  SegRing() = default;
  ~SegRing() { release(); }
  SegRing(const SegRing&) = delete;
  SegRing& operator=(const SegRing&) = delete;

  void init() {
    if (host_) return;
    check(hipHostMalloc((void**)&host_, sizeof(CopySeg) * kSlots * kSegs, hipHostMallocDefault), "hipHostMalloc");
    check(hipMalloc((void**)&dev_, sizeof(CopySeg) * kSlots * kSegs), "hipMalloc");
    for (int i = 0; i < kSlots; ++i) check(hipEventCreateWithFlags(&ev_[i], hipEventDisableTiming), "event");
  }

  void release() {
    for (int i = 0; i < kSlots; ++i)
      if (ev_[i]) {
        hipEventSynchronize(ev_[i]);
        hipEventDestroy(ev_[i]);
        ev_[i] = nullptr;
      }
    if (host_) hipHostFree(host_);
    if (dev_) hipFree(dev_);
    host_ = nullptr;
    dev_ = nullptr;
  }

  // Launch copies for `segs` (chunk0 is recomputed) on `stream`; returns without waiting.
  hipError_t launch(const std::vector<CopySeg>& segs, hipStream_t stream) {
    std::lock_guard<std::mutex> g(mu_);
    size_t base = 0;
    while (base < segs.size()) {
      const size_t cnt = std::min(segs.size() - base, kSegs);
      const int slot = pos_;
      pos_ = (pos_ + 1) % kSlots;
      hipError_t e = hipEventSynchronize(ev_[slot]);
      if (e != hipSuccess) return e;
      CopySeg* h = host_ + (size_t)slot * kSegs;
      CopySeg* d = dev_ + (size_t)slot * kSegs;
      uint64_t chunks = 0;
      for (size_t i = 0; i < cnt; ++i) {
        h[i] = segs[base + i];
        h[i].chunk0 = chunks;
        chunks += (h[i].bytes + kCopyChunk - 1) / kCopyChunk;
      }
      if ((e = hipMemcpyAsync(d, h, sizeof(CopySeg) * cnt, hipMemcpyHostToDevice, stream)) != hipSuccess) return e;
      if ((e = launch_batched_copy(d, (int)cnt, chunks, stream)) != hipSuccess) return e;
      if ((e = hipEventRecord(ev_[slot], stream)) != hipSuccess) return e;
      base += cnt;
    }
    return hipSuccess;
  }

 private:
  static void check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("SegRing ") + what + ": " + hipGetErrorString(e));
  }
  CopySeg* host_ = nullptr;
  CopySeg* dev_ = nullptr;
  hipEvent_t ev_[kSlots] = {};
  int pos_ = 0;
  std::mutex mu_;
};

}  // namespace amdx
