#include "ipc.h"

#include <hip/hip_runtime.h>

#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>

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
