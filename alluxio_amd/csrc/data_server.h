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
// chunk by chunk: an HBM chunk is DMA'd (D2H, one stream per I/O thread) into one of two pinned
// staging buffers while the previous chunk is being sent, a DRAM / file-tier chunk is copied
// straight from the arena or file into the outgoing HTTP/2 frame.  The next chunk is produced only
// while the client's unacknowledged bytes stay below the window (ReadRequest.offset_received acks).
// A cold block of a registered local or S3 mount is read through natively (see serve_block_reads).
// Calls the store cannot serve alone (promote, a block still being written or moved, a UFS the I/O
// threads cannot reach) go to the Python servicer through the front end's streaming bridge, so the
// port serves the whole BlockWorker service.
#pragma once
#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>

#include "block_store.h"
#include "frame_rpc.h"
#include "http_blob.h"
#include "sigv4.h"

namespace amdx {

// The store a server's streams and background tasks share: a cold reader or an AppendBlock task
// that outlives its call (or the server) keeps the store alive until it is done.
using StoreRef = std::shared_ptr<BlockStore>;

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
  std::atomic<uint64_t> write_evict_waits{0};  // WriteBlock creates that evicted on a pool thread
  std::atomic<uint64_t> ufs_write_streams{0};  // UFS_FILE writes into a local UFS served natively
  std::atomic<uint64_t> ufs_write_bytes{0};
  std::atomic<uint64_t> cold_streams{0};     // UFS read-through / uncached UFS reads served natively
  std::atomic<uint64_t> cold_cached{0};      // of which cached the whole block (committed)
  std::atomic<uint64_t> cold_aborted{0};     // read-throughs abandoned (cancel, error): temp block aborted
  std::atomic<uint64_t> cold_bytes{0};       // bytes read from the UFS by those streams
  std::atomic<int64_t> cold_active{0};       // background UFS readers still running
  std::atomic<int64_t> store_tasks{0};       // AppendBlock copies queued or running (they use the store)
  std::atomic<uint64_t> ufs_tee_bytes{0};     // CACHE_THROUGH bytes the UFS stream copied from the store
  std::atomic<uint64_t> zero_copy_frames{0}; // HTTP/2 DATA frames sent straight from staging (no copy)
  std::atomic<uint64_t> prefetched{0};       // HBM chunks whose D2H was issued ahead of the send
  std::atomic<uint64_t> promoted{0};         // CACHE_PROMOTE reads whose block moved to tier 0 natively
  std::atomic<uint64_t> commits{0};          // blocks committed by the native committer
  std::atomic<uint64_t> commit_batches{0};   // master reports (one internal call each) they took
  std::atomic<uint64_t> commit_failures{0};  // blocks whose commit failed (removed / aborted)
  std::atomic<uint64_t> crc_streamed{0};     // blocks whose CRCs were computed on the write stream
  // where the cold readers' time goes (ns summed over reads): queued for a pool thread, setting up
  // (mount resolve, temp block create), until the first slot could be sent, inside UFS reads,
  // waiting for the stream to free a slot (consumer-bound), waiting for a slot's H2D
  std::atomic<uint64_t> cold_queue_ns{0}, cold_setup_ns{0}, cold_first_ns{0}, cold_read_ns{0},
      cold_slot_wait_ns{0}, cold_dma_wait_ns{0};
  // parts of the above: device / stream setup before the first read, slot buffer + event set-up,
  // the first UFS read alone
  std::atomic<uint64_t> cold_device_ns{0}, cold_slot_alloc_ns{0}, cold_first_read_ns{0};
  std::atomic<uint64_t> cold_readahead_bytes{0};   // next-block bytes read ahead by finished read-throughs
  std::atomic<uint64_t> cold_readahead_hits{0};    // UFS reads of cold streams served by those bytes
  std::atomic<bool> stopping{false};               // the worker stops: background UFS reads give up
  // The send side of ReadBlock streams, [0] cached (HBM staging) and [1] cold: streams finished,
  // ns from the call's start to its last byte and to its first, and the gaps in which the stream
  // had nothing to send -- the client's ack window was full, or the next bytes were not there yet
  // (cold: the slot not read; cached: the staging D2H not done).
  struct SendTiming {
    std::atomic<uint64_t> streams{0}, life_ns{0}, first_ns{0}, window_stalls{0}, window_ns{0}, data_stalls{0},
        data_ns{0};
  };
  SendTiming send[2];
};

// One block handed to the committer: the temp block of a finished WriteBlock (or of a complete
// cold read-through), the event after its last device work, its CRCs once they land.
struct CommitTicket {
  int64_t session = 0, block = 0;
  uint64_t length = 0;
  bool pin = false;
  bool ufs_read = false;            // a cold read-through's block (no client waits for it)
  bool hold = false;                // CACHE_THROUGH tee: held for the UFS stream's AppendBlock
  hipEvent_t done = nullptr;        // H2D copies + CRC kernel + CRC D2H of the block (may be null)
  uint32_t* crc_host = nullptr;     // pinned: `crc_pages` per-page CRC32Cs, valid once `done` fired
  uint32_t* crc_dev = nullptr;      // device scratch the CRCs were computed in (returned to the pool)
  size_t crc_words = 0, crc_pages = 0;
  uint64_t crc_page = 0;
  bool crc_sync = false;            // no streamed CRCs: the committer computes them (checksum())
  // result
  std::mutex mu;
  bool finished = false;
  int status = 0;
  std::string msg;
  std::function<void()> wake;       // the waiting stream's waker (null once it is gone)
  ~CommitTicket();
};

// Native block commit of a worker (reference BlockWriteHandler.java:124-149 ->
// DefaultBlockWorker.commitBlock:274-306 -> BlockMaster commitBlock): a thread that takes the
// blocks WriteBlock streams (and cold read-throughs) hand it, waits for each block's device work
// and streamed CRCs, commits it in the store, and reports everything it committed since the last
// report to the master in ONE internal call (`method`, NativeCommitBatch: Python stores the CRCs
// and sends one CommitBlocks RPC, retried for alluxio.user.rpc.retry.max.duration).  A report is
// in flight at most once: blocks that finish meanwhile form the next batch (group commit).  The
// streams answer their clients only once the store commit and the master's ack are both in; a
// block the master could not be told about is removed again and its stream fails UNAVAILABLE.
class BlockCommitter {
 public:
  using Caller = std::function<void(uint32_t, std::string,
                                    std::function<void(int, const std::string&, const std::string&)>)>;
  BlockCommitter(StoreRef store, uint32_t method, bool crc_device, bool crc_host,
                 std::shared_ptr<DataServerStats> stats);
  ~BlockCommitter();
  // The server's internal caller (FrameRpcServer::internal_caller); set on first use.
  void set_caller(Caller c);
  bool has_caller();
  void submit(std::shared_ptr<CommitTicket> t);
  bool crc_device() const { return crc_device_; }
  bool crc_host() const { return crc_host_; }
  // A device CRC buffer (dev + pinned host) of at least `words` words for a ticket, or false.
  bool take_crc_buffer(size_t words, CommitTicket* t);

 private:
  struct State;
  static void run(std::shared_ptr<State> st);
  std::shared_ptr<State> st_;
  bool crc_device_, crc_host_;
};

// An S3-compatible object mount the native data path reads from (plain-HTTP endpoint).
struct S3Mount {
  std::string host;
  int port = 80;
  std::string bucket;
  S3Credentials cred;
  int parallel = 8;            // concurrent sub-range GETs of one read
  uint64_t part = 4u << 20;    // minimum sub-range
  uint64_t upload_part = 64u << 20;   // multipart upload part of a UFS_FILE write
  int upload_inflight = 4;            // part buffers of one write (bounded memory)
  HttpOptions http;                   // timeouts / retries (alluxio.underfs.s3.*)
  std::shared_ptr<HttpRangeReader> reader;
};

// Mounts the I/O threads can reach without Python: local directories (a UFS_FILE WriteBlock is
// written with plain file calls, a cold ReadBlock preads the file) and S3-compatible buckets (a
// cold ReadBlock issues signed ranged GETs).  The worker registers a mount once its Python side
// has resolved it (worker/block_worker.py note_ufs_mount); other mounts (HDFS, ...) stay in Python.
class UfsMounts {
 public:
  void set(int64_t mount_id, const std::string& root);
  void set_s3(int64_t mount_id, const std::string& host, int port, const std::string& bucket,
              const std::string& access_key, const std::string& secret_key, const std::string& region,
              int parallel, uint64_t part, uint64_t upload_part = 64u << 20, int upload_inflight = 4,
              const HttpOptions& http = HttpOptions());
  void remove(int64_t mount_id);
  size_t size() const;
  // Mounts the worker resolved and found the I/O threads cannot reach (HDFS, HTTPS S3, ...): their
  // cold reads go straight to Python.
  void mark_python(int64_t mount_id);
  bool is_python(int64_t mount_id) const;
  // The local path of `ufs_path` ("file:///x" or "/x") if mount `mount_id` is a registered local
  // directory and the path lies inside its root without "." / ".." components.
  bool resolve(int64_t mount_id, const std::string& ufs_path, std::string* local) const;
  // The object mount and key of `ufs_path` ("s3://bucket/key") if `mount_id` is a registered
  // S3 mount of that bucket.
  bool resolve_s3(int64_t mount_id, const std::string& ufs_path, std::shared_ptr<const S3Mount>* m,
                  std::string* key) const;

 private:
  mutable std::mutex mu_;
  std::unordered_map<int64_t, std::string> roots_;
  std::unordered_map<int64_t, std::shared_ptr<const S3Mount>> s3_;
  std::unordered_map<int64_t, bool> python_;
};
using LocalUfsRoots = UfsMounts;

// Cold-read settings of serve_block_reads.
struct ColdReadConfig {
  uint64_t slot_bytes = 8u << 20;   // one UFS read / H2D copy
  int depth = 3;                    // slots per stream (reads run this far ahead of the sends)
  int max_active = 256;             // concurrent background UFS readers; more go to Python
  uint32_t commit_method = UINT32_MAX;   // internal NativeWriteCommit (caches are committed in Python)
  // internal ResolveUfsMount: a cold read of a mount the data server does not know yet asks the
  // worker to resolve it (GetUfsInfo from the master, reference WorkerUfsManager.java:56-65) on the
  // reader's pool thread, then reads natively -- no first read of a mount goes through Python
  uint32_t resolve_method = UINT32_MAX;
  uint32_t read_range_method = UINT32_MAX;   // internal ReadUfsRange (a resolved mount that is Python's)
  // a whole-block read-through reads the file's next block's first two reads ahead once its own
  // reads are done (alluxio.worker.data.server.native.ufs.readahead.enabled)
  bool readahead = true;
  // UFS reads of a read-through before its temp block is created (0: one per slot;
  // alluxio.worker.data.server.native.ufs.create.after.reads)
  int create_after_reads = 2;
};

// Serve `method` (the ReadBlock path's index) of `srv` from `store`.  `max_chunk` caps a client's
// chunk_size, `window` is the un-acked byte limit per call.
// With `mounts`, a read of a block the store does not hold that carries open_ufs_block_options of a
// registered mount is served natively too (reference BlockReadHandler.java:159-235 openUfsBlock,
// UnderFileSystemBlockReader.java:205-274): a background thread reads the UFS into pinned slots,
// each slot is copied into a fresh temp block (async H2D for HBM) and streamed to the client as
// soon as it lands; at the end the block is committed through `cold.commit_method` in Python (CRC,
// master report) before the call ends.  A partial, offset or no_cache read streams the range
// without caching; a cancelled or failed read-through aborts the temp block.
void serve_block_reads(FrameRpcServer& srv, uint32_t method, StoreRef store, uint64_t max_chunk,
                       uint64_t window, std::shared_ptr<DataServerStats> stats,
                       std::shared_ptr<UfsMounts> mounts = nullptr, ColdReadConfig cold = ColdReadConfig(),
                       std::shared_ptr<BlockCommitter> committer = nullptr);

// Serve `method` (WriteBlock) of `srv` into `store` for ALLUXIO_BLOCK writes: the block is created
// on the first message, chunk messages are written into it on the I/O thread (HBM: through a
// pinned staging buffer and an async H2D on the thread's stream), flush commands are answered
// with the offset; at the client's half-close the commit -- CRC, master report -- runs in Python
// as the internal unary `commit_method` (NativeWriteCommitRequest) whose reply ends the call.
// UFS_FILE writes under a local mount of `ufs_roots` (may be null) are written natively too: a temp
// file beside the target, renamed over it at the half-close (reference UfsFileWriteHandler.java
// with the local UFS's AtomicFileOutputStream); under an S3 mount they become a multipart upload
// whose parts go out on upload threads while the client streams (S3ALowLevelOutputStream), with
// the request window held back while every part buffer is in flight.  Other UFS_FILE and
// UFS_FALLBACK_BLOCK writes go to the Python servicer.
// With `committer`, the commit runs natively (BlockCommitter) instead of as `commit_method` in Python.
void serve_block_writes(FrameRpcServer& srv, uint32_t method, uint32_t commit_method, StoreRef store,
                        uint64_t stage_bytes, std::shared_ptr<DataServerStats> stats,
                        std::shared_ptr<UfsMounts> ufs_roots = nullptr,
                        std::shared_ptr<BlockCommitter> committer = nullptr);

// Deletes the local file `path`: its name goes now, the freeing of its pages later.  Unlinking a
// large file costs its page-cache and extent teardown inline (~20 ms for 256 MiB on ext4), and a
// master Remove would wait for it.  A file of at least `defer_bytes` is opened, unlinked (only the
// directory entry goes while the descriptor holds the inode), and its descriptor is closed on a
// background "ufs-reclaim" thread, where the last reference frees it.  Smaller files, or any
// that cannot be opened, are unlinked directly.  With more than `max_pending` descriptors
// waiting, the close runs inline.  Returns 0 or the errno of the unlink.
int unlink_deferred(const std::string& path, uint64_t defer_bytes = 8u << 20, size_t max_pending = 256);
// Descriptors closed by the reclaim thread so far, and those still waiting.
uint64_t reclaimed_files();
size_t reclaim_pending();

}  // namespace amdx
