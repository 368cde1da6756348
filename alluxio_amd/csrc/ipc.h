// HIP IPC export/import of HBM arenas and peer-access setup (MI355X short-circuit data plane).
//
// The reference's short-circuit read hands a same-node client the block *file path* to mmap
// (core/server/worker/.../grpc/ShortCircuitBlockReadHandler.java); here the worker hands out a
// HIP IPC handle of the HBM arena allocation plus the block's page list, and the client process
// maps the arena once and gathers pages with its own copy kernel (over xGMI when the client
// sits on another GPU of the node).
#pragma once
#include <cstdint>
#include <stdexcept>
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
// ipc_open with a deadline: the open runs on a helper thread and a call that has not returned
// after `timeout_ms` fails with IpcTimeout (the helper keeps waiting and closes the mapping if it
// ever arrives; the handle is not tried again in this process).  The caller then takes another
// path to the bytes (the worker's gRPC data port).
struct IpcTimeout : std::runtime_error {
  using std::runtime_error::runtime_error;
};
uint64_t ipc_open_bounded(const std::string& handle, int device, int timeout_ms);
// Drop one reference; unmaps when the count reaches zero.
void ipc_close(uint64_t base);
// The worker's HBM arena: one plain hipMalloc owned by the caller (not the framework's caching
// allocator, whose pooled segments export as a different -- larger -- allocation than the arena).
uint64_t device_arena_alloc(uint64_t bytes, int device);
void device_arena_free(uint64_t ptr, int device);
// Enable peer access device -> peer (idempotent); returns false if the pair cannot peer.
bool enable_peer_access(int device, int peer);
int can_access_peer(int device, int peer);

}  // namespace amdx
