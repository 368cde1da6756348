// Native block data server of a worker: gRPC ReadBlock streams answered on the I/O threads of the
// HTTP/2 front end (frame_rpc.cpp) straight from the tiered block store.
//
// Reference: core/server/worker/src/main/java/alluxio/worker/grpc/GrpcDataServer.java:50-198 (the
// Netty data server), BlockReadHandler.java:111-152 (lock the block, hand out chunks of the block
// reader) and AbstractReadHandler.java (chunked streaming with the offset_received flow-control
// window), core/common/src/main/java/alluxio/grpc/ReadResponseMarshaller.java:38-80 (the chunk goes
// out as a hand-built protobuf header followed by the raw buffer).
//
// MI355X design: a call for a block held by the store is read-locked for its lifetime and streamed
// chunk by chunk: an HBM chunk is DMA'd (D2H, one stream per I/O thread) into a pinned staging
// buffer, a DRAM / file-tier chunk is copied straight from the arena or file into the outgoing
// HTTP/2 frame.  The next chunk is produced only while the client's unacknowledged bytes stay
// below the window (ReadRequest.offset_received acks).  Calls the store cannot serve alone (UFS
// read-through, promote, a block still being written or moved) go to the Python servicer through
// the front end's streaming bridge, so the port serves the whole BlockWorker service.
#pragma once
#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>

#include "block_store.h"
#include "frame_rpc.h"

namespace amdx {

struct DataServerStats {
  std::atomic<uint64_t> streams{0};      // calls served natively
  std::atomic<uint64_t> declined{0};     // calls handed to Python
  std::atomic<uint64_t> bytes{0};        // block bytes sent natively
  std::atomic<uint64_t> domain_bytes{0}; // of which to Unix-domain-socket (same-node) clients
  std::atomic<uint64_t> chunks{0};
  std::atomic<uint64_t> staged_bytes{0}; // of which D2H-staged from HBM
  std::atomic<uint64_t> write_streams{0};  // WriteBlock calls served natively
  std::atomic<uint64_t> write_declined{0}; // WriteBlock calls handed to Python (UFS / fallback)
  std::atomic<uint64_t> write_bytes{0};    // block bytes written natively
  std::atomic<uint64_t> ufs_write_streams{0};  // UFS_FILE writes into a local UFS served natively
  std::atomic<uint64_t> ufs_write_bytes{0};
};

// Mounts whose UFS is a local directory, so a UFS_FILE WriteBlock can be written by the I/O
// thread with plain file calls.  The worker registers a mount once its Python side has resolved
// it to the local UFS (worker/block_worker.py); other mounts (S3, HDFS, ...) stay in Python.
class LocalUfsRoots {
 public:
  void set(int64_t mount_id, const std::string& root);
  void remove(int64_t mount_id);
  size_t size() const;
  // The local path of `ufs_path` ("file:///x" or "/x") if mount `mount_id` is registered and the
  // path lies inside its root without "." / ".." components.
  bool resolve(int64_t mount_id, const std::string& ufs_path, std::string* local) const;

 private:
  mutable std::mutex mu_;
  std::unordered_map<int64_t, std::string> roots_;
};

// Serve `method` (the ReadBlock path's index) of `srv` from `store`.  `max_chunk` caps a client's
// chunk_size, `window` is the un-acked byte limit per call.
void serve_block_reads(FrameRpcServer& srv, uint32_t method, BlockStore* store, uint64_t max_chunk,
                       uint64_t window, std::shared_ptr<DataServerStats> stats);

// Serve `method` (WriteBlock) of `srv` into `store` for ALLUXIO_BLOCK writes: the block is created
// on the first message, chunk messages are written into it on the I/O thread (HBM: through a
// pinned staging buffer and an async H2D on the thread's stream), flush commands are answered
// with the offset; at the client's half-close the commit -- CRC, master report -- runs in Python
// as the internal unary `commit_method` (NativeWriteCommitRequest) whose reply ends the call.
// UFS_FILE writes under a mount of `ufs_roots` (may be null) are written natively too: a temp
// file beside the target, renamed over it at the half-close (reference UfsFileWriteHandler.java
// with the local UFS's AtomicFileOutputStream).  Other UFS_FILE and UFS_FALLBACK_BLOCK writes go
// to the Python servicer.
void serve_block_writes(FrameRpcServer& srv, uint32_t method, uint32_t commit_method, BlockStore* store,
                        uint64_t stage_bytes, std::shared_ptr<DataServerStats> stats,
                        std::shared_ptr<LocalUfsRoots> ufs_roots = nullptr);

}  // namespace amdx
