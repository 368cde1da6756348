// Host-reader data path of the client: where one block's bytes come from, and the chunk-buffered
// input stream that turns many small read(buf) calls into a few large refills.
//
// Reference: core/client/fs/src/main/java/alluxio/client/block/stream/LocalFileDataReader.java:58-70
// (short-circuit: map the block, hand out chunks of up to 8 MB; a read(buf) is a copy out of the
// mapping), GrpcDataReader.java (the ReadBlock stream with offset_received acks), BlockInStream
// and AlluxioFileInStream.java:66-434 (block switching).  StressWorkerBench's reader loop
// (stress/shell/.../StressWorkerBench.java:251-276) is 4 KiB read(buf) calls on these streams.
//
// MI355X design: a HIP-IPC short-circuit block lives in another process's HBM arena, so a chunk
// (1 MiB default) is DMA'd D2H into a pinned buffer of the stream by one hipMemcpyAsync per page
// run, and every read(buf) inside it is a memcpy; a shared DRAM arena is read in place; a remote
// block arrives over a native gRPC (HTTP/2) ReadBlock call whose DATA frames are parsed straight
// into the destination.  No device tensor, Python bytes object or GIL is involved per read.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <atomic>
#include <memory>
#include <string>
#include <vector>

#include "block_store.h"

namespace amdx {

class BlockSource {
 public:
  explicit BlockSource(uint64_t length) : length_(length) {}
  virtual ~BlockSource() = default;
  // Copies block bytes [off, off + n) into host memory at dst.  Blocking; called without the GIL
  // unless needs_gil().  Throws std::runtime_error / StoreError.
  virtual void read(uint64_t off, uint64_t n, uint8_t* dst) = 0;
  // Reads straight into the caller's buffer are as cheap as refilling the chunk buffer (host
  // arenas: a memcpy; network streams: the frames are parsed into the destination).
  virtual bool direct() const { return false; }
  virtual bool needs_gil() const { return false; }
  // A read mostly waits on a socket (true) rather than on a DMA or a memcpy: prefetches of such
  // sources run on a pool that grows with the streams, DMA ones on a small fixed pool (hundreds
  // of threads issuing D2H copies at once contend inside the HIP runtime).
  virtual bool waits_on_network() const { return false; }
  // Begins delivering the block from offset 0 before the first read() (a network source sends
  // its request now, so the bytes are on their way while the reader finishes the previous block).
  virtual void start() {}
  virtual void close() {}
  uint64_t length() const { return length_; }

 protected:
  uint64_t length_;
};

// A block in an HBM arena mapped into this process (HIP IPC of a same-node worker, or the arena of
// an in-process worker): chunks are DMA'd into pinned host memory.
class DeviceArenaSource : public BlockSource {
 public:
  DeviceArenaSource(uint64_t base, std::vector<int64_t> pages, uint64_t page_size, uint64_t length, int device);
  void read(uint64_t off, uint64_t n, uint8_t* dst) override;

 private:
  uint64_t base_;
  std::vector<int64_t> pages_;
  uint64_t page_size_;
  int device_;
};

// A block in host memory (a shared DRAM arena mapped from another worker process).
class HostArenaSource : public BlockSource {
 public:
  HostArenaSource(uint64_t base, std::vector<int64_t> pages, uint64_t page_size, uint64_t length);
  void read(uint64_t off, uint64_t n, uint8_t* dst) override;
  bool direct() const override { return true; }

 private:
  uint64_t base_;
  std::vector<int64_t> pages_;
  uint64_t page_size_;
};

// A block of a worker in this process, read through its store (the caller holds the block lock).
class StoreSource : public BlockSource {
 public:
  StoreSource(BlockStore* store, int64_t block_id, uint64_t length, bool device_tier);
  void read(uint64_t off, uint64_t n, uint8_t* dst) override;
  bool direct() const override { return !device_; }
  // bytes served so far (the worker's BytesReadAlluxio for in-process readers)
  uint64_t bytes() const { return bytes_.load(std::memory_order_relaxed); }

 private:
  BlockStore* store_;
  int64_t block_;
  bool device_;
  std::atomic<uint64_t> bytes_{0};
};

// A block streamed from a worker's data port over gRPC: ReadBlock on HTTP/2 (h2c, prior
// knowledge) with ReadRequest.offset_received acks, spoken directly with libnghttp2.  Works
// against the native data server and any stock gRPC server of the BlockWorker service.
class GrpcBlockSource : public BlockSource {
 public:
  struct Options {
    std::string host;
    int port = 0;
    std::string unix_path;           // the worker's domain socket (same node): used instead of TCP
    int64_t block_id = 0;
    uint64_t chunk = 1u << 20;       // ReadRequest.chunk_size
    std::string ufs_options;         // serialized OpenUfsBlockOptions ("" = none)
    bool promote = false;
    std::string channel_id, user;    // call headers (SASL channel / NOSASL user)
    int timeout_ms = 60000;
  };
  GrpcBlockSource(Options o, uint64_t length);
  ~GrpcBlockSource() override;
  void read(uint64_t off, uint64_t n, uint8_t* dst) override;
  bool direct() const override { return true; }
  bool waits_on_network() const override { return true; }
  void start() override;
  void close() override;
  struct Conn;

 private:
  void open(uint64_t off);
  void maybe_ack(uint64_t offset);
  Options o_;
  std::unique_ptr<Conn> c_;
};

// Writes into the pages of a temp block of a same-node worker's arena mapped into this process
// (short-circuit write; worker OpenDeviceWrite / CommitDeviceWrite).  HBM: the caller's bytes are
// copied into two alternating pinned staging buffers and DMA'd H2D page run by page run, the
// memcpy of piece i+1 overlapping the DMA of piece i; shared DRAM: memcpy into the pages.
class ArenaSink {
 public:
  ArenaSink(uint64_t base, std::vector<int64_t> pages, uint64_t page_size, uint64_t capacity, int device, bool host_arena);
  ~ArenaSink();
  void write(uint64_t off, const uint8_t* src, uint64_t n);
  uint64_t length() const { return length_; }    // end of the furthest byte written

 private:
  uint64_t base_;
  std::vector<int64_t> pages_;
  uint64_t page_size_, capacity_;
  int device_;
  bool host_;
  uint64_t length_ = 0;
  static constexpr uint64_t kStage = 4u << 20;
  uint8_t* stage_[2] = {nullptr, nullptr};
  bool pinned_[2] = {false, false};
  hipEvent_t ev_[2] = {nullptr, nullptr};
};

// A block written to a worker's data port: WriteBlock over HTTP/2 spoken directly with libnghttp2
// (command, then WriteRequest{chunk} messages framed around the caller's bytes -- copied once, into
// the HTTP/2 frames --, half-close, final WriteResponse).  The native data server writes the
// chunks into the block on its I/O threads (csrc/data_server.cpp); any gRPC BlockWorker works.
class GrpcBlockSink {
 public:
  struct Options {
    std::string host;
    int port = 0;
    std::string unix_path;
    int64_t block_id = 0;
    int tier = 0;
    std::string medium;
    uint64_t reserve = 1u << 20;
    bool pin = false;
    uint64_t chunk = 1u << 20;       // bytes per WriteRequest message
    std::string channel_id, user;
    int timeout_ms = 60000;
    // A serialized WriteRequestCommand sent instead of the ALLUXIO_BLOCK one built from the
    // fields above (e.g. a UFS_FILE write to the worker's UFS).
    std::string command;
  };
  explicit GrpcBlockSink(Options o);
  ~GrpcBlockSink();
  // Streams n bytes; returns once they are in the socket (flow control permitting).
  void write(const uint8_t* p, uint64_t n);
  // UFS_FILE streams: the next `length` bytes of the file are block `block_id`, which the same
  // worker already holds (CACHE_THROUGH tee: the worker copies them from its store).
  void append_block(int64_t block_id, uint64_t length);
  // Half-closes and waits for the worker's commit; returns the committed length.  `hold_for_append`:
  // the worker keeps the committed block locked until the file's UFS stream appends it (CACHE_THROUGH
  // tee), so it cannot be evicted in between.
  uint64_t commit(bool hold_for_append = false);
  void cancel();
  uint64_t written() const { return written_; }
  struct Conn;

 private:
  void wait_drained();
  Options o_;
  std::unique_ptr<Conn> c_;
  uint64_t written_ = 0;
};

// Block bytes [off, off + n) of `src` into device memory at dptr: chunks land in two alternating
// pinned buffers, each DMA'd H2D while the next chunk is being received (a GPU consumer of a
// remote worker's block).
void source_read_to_device(BlockSource& src, uint64_t off, uint64_t n, uint8_t* dptr, int device);

// Pinned (device-mapped) host buffer for a chunk buffer (pooled by size; malloc without a GPU).
uint8_t* host_buffer_alloc(uint64_t n, bool* pinned);
// Gives a buffer of host_buffer_alloc(n) back (pinned ones to the pool).
void host_buffer_release(uint8_t* p, uint64_t n, bool pinned);

// Sequential reader over a file's blocks with two chunk buffers: read(buf) calls inside the
// current chunk are a memcpy; while they drain it, the next chunk of the block is prefetched into
// the other buffer by a shared pool of native threads, so a reader thread reaching the end of a
// chunk normally just swaps buffers (no I/O wait, and no GIL release on the Python side).  The
// owner (bindings) supplies sources per block index and holds the GIL rules.
class HostInStream {
 public:
  HostInStream(uint64_t length, uint64_t block_size, uint64_t chunk, bool prefetch = true);
  ~HostInStream();
  inline bool fast(uint8_t* dst, uint64_t n) {
    if (pos_ >= buf_lo_ && pos_ + n <= buf_hi_) {
      std::memcpy(dst, buf_ + (pos_ - buf_lo_), n);
      pos_ += n;
      bytes_ += n;
      return true;
    }
    return false;
  }
  // The prefetched chunk is complete and holds pos(): make it current (no waiting, no I/O).
  bool try_swap();
  // Copies up to n bytes at pos() that the current chunk (or a completed prefetch) already
  // holds, within the current block; 0 when I/O is needed.  Never blocks.
  uint64_t copy_buffered(uint8_t* dst, uint64_t n);
  // Copies up to n bytes at pos() from the current block's source (which must cover pos());
  // returns the bytes copied (> 0).  Called without the GIL unless the source needs it.
  uint64_t read_block_part(uint8_t* dst, uint64_t n);
  void set_source(int64_t idx, std::shared_ptr<BlockSource> src);
  void drop_source();
  void invalidate() { buf_lo_ = buf_hi_ = 0; }
  int64_t block_index() const { return cur_idx_; }
  BlockSource* source() const { return cur_.get(); }
  uint64_t pos() const { return pos_; }
  void seek(uint64_t p) { pos_ = p > length_ ? length_ : p; }
  uint64_t length() const { return length_; }
  uint64_t block_size() const { return block_size_; }
  uint64_t bytes() const { return bytes_; }
  uint64_t refills() const { return refills_; }
  uint64_t prefetch_hits() const { return pf_hits_; }

 private:
  struct Prefetch;
  void schedule_prefetch();
  void cancel_prefetch();                 // waits for an in-flight prefetch, forgets it
  void make_current(int i, uint64_t lo, uint64_t hi);
  uint64_t length_, block_size_, chunk_;
  bool prefetch_;
  uint64_t pos_ = 0;
  uint8_t* bufs_[2] = {nullptr, nullptr};
  bool pinned_[2] = {false, false};
  int cur_buf_ = 0;
  uint8_t* buf_ = nullptr;             // bufs_[cur_buf_]
  uint64_t buf_lo_ = 0, buf_hi_ = 0;   // file offsets held by buf_
  int64_t cur_idx_ = -1;
  uint64_t cur_start_ = 0;
  std::shared_ptr<BlockSource> cur_;
  std::shared_ptr<Prefetch> pf_;       // in flight / completed prefetch into bufs_[1 - cur_buf_]
  uint64_t bytes_ = 0, refills_ = 0, pf_hits_ = 0;
};

// Cap on the threads of each prefetch pool (0 = defaults: 64 for network sources, 16 for DMA /
// memcpy sources).  The pools add threads on demand up to the cap.
void set_prefetch_threads(int n);

}  // namespace amdx
