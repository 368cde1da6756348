// HIP IPC export/import of HBM arenas and peer-access setup (MI355X short-circuit data plane).
//
// The reference's short-circuit read hands a same-node client the block *file path* to mmap
// (core/server/worker/.../grpc/ShortCircuitBlockReadHandler.java); here the worker hands out a
// HIP IPC handle of the HBM arena allocation plus the block's page list, and the client process
// maps the arena once and gathers pages with its own copy kernel (over xGMI when the client
// sits on another GPU of the node).
#pragma once
#include <cstdint>
#include <string>

namespace amdx {

struct IpcExport {
  std::string handle;   // raw hipIpcMemHandle_t bytes
  uint64_t offset;      // byte offset of `ptr` inside the exported allocation
  uint64_t alloc_bytes; // size of the whole allocation
};

// Export the allocation containing device pointer `ptr` (throws std::runtime_error on failure).
IpcExport ipc_export(uint64_t ptr);
// Map an exported allocation into this process on `device`; returns the allocation base.
// Maps are reference counted per handle so repeated opens are cheap.
uint64_t ipc_open(const std::string& handle, int device);
// Drop one reference; unmaps when the count reaches zero.
void ipc_close(uint64_t base);
// Enable peer access device -> peer (idempotent); returns false if the pair cannot peer.
bool enable_peer_access(int device, int peer);
int can_access_peer(int device, int peer);

}  // namespace amdx
