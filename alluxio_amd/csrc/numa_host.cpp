// Pinned host memory on the GPU's NUMA node (see numa_host.h).
#include "numa_host.h"

#include <hip/hip_runtime.h>

#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>

namespace amdx {

namespace {
constexpr int kMpolDefault = 0, kMpolPreferred = 1;
constexpr unsigned long kMaxNode = 1024;
}  // namespace

int gpu_numa_node(int device) {
  static std::mutex mu;
  static std::map<int, int> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(device);
  if (it != cache.end()) return it->second;
  int node = -1;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) == hipSuccess) {
    std::string id(bus);
    for (char& c : id) c = (char)std::tolower((unsigned char)c);
    std::ifstream f("/sys/bus/pci/devices/" + id + "/numa_node");
    if (f) f >> node;
  }
  cache[device] = node;
  return node;
}

void* pinned_alloc_near(size_t bytes, int device) {
  const int node = gpu_numa_node(device);
  void* p = nullptr;
  if (node < 0) {
    return hipHostMalloc(&p, bytes, hipHostMallocDefault) == hipSuccess ? p : nullptr;
  }
  // this thread's policy -> preferred(node) for the allocation (and its first touch), then back
  int old_mode = kMpolDefault;
  unsigned long old_mask[kMaxNode / (8 * sizeof(unsigned long))] = {0};
  const bool saved = syscall(SYS_get_mempolicy, &old_mode, old_mask, kMaxNode, nullptr, 0) == 0;
  unsigned long mask[kMaxNode / (8 * sizeof(unsigned long))] = {0};
  mask[node / (8 * sizeof(unsigned long))] |= 1ul << (node % (8 * sizeof(unsigned long)));
  const bool set = syscall(SYS_set_mempolicy, kMpolPreferred, mask, kMaxNode) == 0;
  hipError_t e = hipHostMalloc(&p, bytes, set ? hipHostMallocNumaUser : hipHostMallocDefault);
  if (e == hipSuccess && set) std::memset(p, 0, bytes < 4096 ? bytes : 4096);   // first touch on the node
  if (set) {
    if (saved) (void)syscall(SYS_set_mempolicy, old_mode, old_mode == kMpolDefault ? nullptr : old_mask, kMaxNode);
    else (void)syscall(SYS_set_mempolicy, kMpolDefault, nullptr, kMaxNode);
  }
  if (e != hipSuccess) {
    p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) p = nullptr;
  }
  return p;
}

std::string process_placement() {
  cpu_set_t set;
  CPU_ZERO(&set);
  std::ostringstream o;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) {
    int first = -1, prev = -2, count = 0;
    std::string ranges;
    auto flush = [&] {
      if (first < 0) return;
      if (!ranges.empty()) ranges += ",";
      ranges += prev == first ? std::to_string(first) : std::to_string(first) + "-" + std::to_string(prev);
    };
    for (int c = 0; c < CPU_SETSIZE; ++c) {
      if (!CPU_ISSET(c, &set)) continue;
      ++count;
      if (c != prev + 1) {
        flush();
        first = c;
      }
      prev = c;
    }
    flush();
    o << "cpus " << ranges << " (" << count << ")";
  }
  unsigned cpu = 0, node = 0;
  if (syscall(SYS_getcpu, &cpu, &node, nullptr) == 0) o << ", running on cpu " << cpu << " node " << node;
  return o.str();
}

}  // namespace amdx
