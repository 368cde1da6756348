#include "ipc.h"

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <thread>

namespace amdx {
namespace {

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

struct Mapped {
  uint64_t base;
  int refs;
};

std::mutex g_mu;
std::map<std::string, Mapped> g_by_handle;   // handle bytes -> mapping
std::map<uint64_t, std::string> g_by_base;

}  // namespace

IpcExport ipc_export(uint64_t ptr) {
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  check(hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(ptr)),
        "hipMemGetAddressRange");
  hipIpcMemHandle_t h;
  check(hipIpcGetMemHandle(&h, base), "hipIpcGetMemHandle");
  IpcExport out;
  out.handle.assign(reinterpret_cast<const char*>(&h), sizeof(h));
  out.offset = ptr - reinterpret_cast<uint64_t>(base);
  out.alloc_bytes = size;
  return out;
}

uint64_t ipc_open(const std::string& handle, int device) {
  if (handle.size() != sizeof(hipIpcMemHandle_t))
    throw std::runtime_error("ipc_open: bad handle size");
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_by_handle.find(handle);
  if (it != g_by_handle.end()) {
    it->second.refs++;
    return it->second.base;
  }
  int prev = 0;
  check(hipGetDevice(&prev), "hipGetDevice");
  check(hipSetDevice(device), "hipSetDevice");
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.data(), sizeof(h));
  void* p = nullptr;
  hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
  (void)hipSetDevice(prev);
  check(e, "hipIpcOpenMemHandle");
  uint64_t base = reinterpret_cast<uint64_t>(p);
  g_by_handle[handle] = Mapped{base, 1};
  g_by_base[base] = handle;
  return base;
}

namespace {
std::map<std::string, bool> g_poisoned;   // handles whose open timed out (not retried)
}

uint64_t ipc_open_bounded(const std::string& handle, int device, int timeout_ms) {
  if (handle.size() != sizeof(hipIpcMemHandle_t))
    throw std::runtime_error("ipc_open: bad handle size");
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_by_handle.find(handle);
    if (it != g_by_handle.end()) {
      it->second.refs++;
      return it->second.base;
    }
    if (g_poisoned.count(handle)) throw IpcTimeout("hipIpcOpenMemHandle of this arena timed out before");
  }
  struct Pending {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false, abandoned = false;
    hipError_t err = hipSuccess;
    void* ptr = nullptr;
  };
  auto pd = std::make_shared<Pending>();
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.data(), sizeof(h));
  // test hook: ALLUXIO_AMD_IPC_OPEN_DELAY_MS stalls the open like a stuck import would
  const char* dly = std::getenv("ALLUXIO_AMD_IPC_OPEN_DELAY_MS");
  const int delay_ms = dly ? std::atoi(dly) : 0;
  std::thread([pd, h, device, delay_ms] {
    if (delay_ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(delay_ms));
    void* p = nullptr;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
    bool late;
    {
      std::lock_guard<std::mutex> g(pd->mu);
      pd->done = true;
      pd->err = e;
      pd->ptr = p;
      late = pd->abandoned;
    }
    pd->cv.notify_all();
    if (late && e == hipSuccess) (void)hipIpcCloseMemHandle(p);   // nobody took it
  }).detach();
  std::unique_lock<std::mutex> lk(pd->mu);
  if (!pd->cv.wait_for(lk, std::chrono::milliseconds(std::max(1, timeout_ms)), [&] { return pd->done; })) {
    pd->abandoned = true;
    lk.unlock();
    std::lock_guard<std::mutex> g(g_mu);
    g_poisoned[handle] = true;
    throw IpcTimeout("hipIpcOpenMemHandle did not return within " + std::to_string(timeout_ms) + " ms");
  }
  const hipError_t e = pd->err;
  void* p = pd->ptr;
  lk.unlock();
  check(e, "hipIpcOpenMemHandle");
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_by_handle.find(handle);
  if (it != g_by_handle.end()) {   // opened concurrently by another caller: keep one mapping
    (void)hipIpcCloseMemHandle(p);
    it->second.refs++;
    return it->second.base;
  }
  const uint64_t base = reinterpret_cast<uint64_t>(p);
  g_by_handle[handle] = Mapped{base, 1};
  g_by_base[base] = handle;
  return base;
}

uint64_t device_arena_alloc(uint64_t bytes, int device) {
  int prev = 0;
  check(hipGetDevice(&prev), "hipGetDevice");
  check(hipSetDevice(device), "hipSetDevice");
  void* p = nullptr;
  const hipError_t e = hipMalloc(&p, (size_t)std::max<uint64_t>(bytes, 1));
  (void)hipSetDevice(prev);
  check(e, "hipMalloc of the HBM arena");
  return reinterpret_cast<uint64_t>(p);
}

void device_arena_free(uint64_t ptr, int device) {
  if (!ptr) return;
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) return;
  (void)hipSetDevice(device);
  (void)hipFree(reinterpret_cast<void*>(ptr));
  (void)hipSetDevice(prev);
}

void ipc_close(uint64_t base) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_by_base.find(base);
  if (it == g_by_base.end()) return;
  auto& m = g_by_handle[it->second];
  if (--m.refs > 0) return;
  (void)hipIpcCloseMemHandle(reinterpret_cast<void*>(base));
  g_by_handle.erase(it->second);
  g_by_base.erase(it);
}

int can_access_peer(int device, int peer) {
  int ok = 0;
  check(hipDeviceCanAccessPeer(&ok, device, peer), "hipDeviceCanAccessPeer");
  return ok;
}

bool enable_peer_access(int device, int peer) {
  if (device == peer) return true;
  if (!can_access_peer(device, peer)) return false;
  int prev = 0;
  check(hipGetDevice(&prev), "hipGetDevice");
  check(hipSetDevice(device), "hipSetDevice");
  hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
  (void)hipSetDevice(prev);
  if (e == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();
    return true;
  }
  check(e, "hipDeviceEnablePeerAccess");
  return true;
}

}  // namespace amdx
