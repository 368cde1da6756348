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
// UFS_FILE / UFS_FALLBACK_BLOCK writes go to the Python servicer.
void serve_block_writes(FrameRpcServer& srv, uint32_t method, uint32_t commit_method, BlockStore* store,
                        uint64_t stage_bytes, std::shared_ptr<DataServerStats> stats);

}  // namespace amdx
