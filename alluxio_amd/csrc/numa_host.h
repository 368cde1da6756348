// Pinned host memory on the GPU's NUMA node.
//
// The D2H / H2D staging buffers of the data path (the worker's data-server staging and cold-read
// slots, the client's chunk buffers) are DMA targets of one GPU; on a multi-socket MI355X node a
// buffer on the far socket crosses the inter-socket link on every copy.  hipHostMalloc's default
// placement follows the allocating thread, which for a pool is whichever thread asked first.
// pinned_alloc_near() places the buffer on the node of `device` (its PCI function's numa_node in
// sysfs) with a preferred-node memory policy around hipHostMalloc(hipHostMallocNumaUser).
#pragma once
#include <cstddef>
#include <string>

namespace amdx {

// NUMA node of HIP device `device` (-1 when unknown: one node, no sysfs, no device).
int gpu_numa_node(int device);
// Pinned host memory preferring `device`'s NUMA node; nullptr on failure.  Free with hipHostFree.
void* pinned_alloc_near(size_t bytes, int device);
// "node <n>, cpus <list>" of the calling process (diagnostics for the bench rows).
std::string process_placement();

}  // namespace amdx
