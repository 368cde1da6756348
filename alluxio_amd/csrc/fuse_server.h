// Native /dev/fuse request loop with a C++ fast path for the read side of the namespace.
//
// Reference: integration/fuse/src/main/java/alluxio/fuse/AlluxioFuseFileSystem.java:535-641
// (getattr / open / read / release through jnr-fuse).  A Python FUSE loop pays a GIL acquisition
// and an interpreter dispatch per kernel request -- about 5.5 requests per small file read
// (LOOKUP, OPEN, READ, FLUSH, RELEASE).  Here C++ threads own the /dev/fuse fd and answer, without
// Python:
//   * LOOKUP / GETATTR from an attribute cache (entries pushed by the Python op layer: the fuse_attr
//     bytes, a TTL, the Alluxio file id and the file's blocks);
//   * OPEN (read-only) of a completed file whose blocks are all cached in the co-located worker's
//     store: the blocks are read-locked in the BlockStore and the handle gets the page list;
//   * READ on such a handle: memcpy from the DRAM arena (hipMemcpy D2H from an HBM arena);
//   * FLUSH / RELEASE of such a handle (RELEASE drops the block locks), FORGET, INTERRUPT.
// Everything else (mutations, attribute misses, files not cached locally) is queued for Python
// handler threads (poll/reply), which use the same node table through this object.
//
// Page-cache coherence: FOPEN_KEEP_CACHE is set on a native open only when the node's
// Alluxio file id is the one it had at its previous open (Alluxio files are write-once; a path
// deleted and re-created gets a new file id, so its stale kernel pages are dropped).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace amdx {

class BlockStore;

struct FuseRequest {
  uint64_t unique;
  uint32_t opcode;
  uint64_t nodeid;
  uint32_t uid, gid, pid;
  std::string body;      // bytes after fuse_in_header
};

class FuseServer {
 public:
  // `store` (may be null): the co-located worker's block store for native opens; `session`: the
  // lock session id native opens use.  keep_cache: 0 never, 1 always, 2 when the file id is unchanged.
  FuseServer(int fd, int threads, BlockStore* store, int64_t session, int keep_cache);
  ~FuseServer();
  void start();
  void stop();
  // Python slow path: up to max_n queued requests (GIL released while waiting).
  std::vector<FuseRequest> poll(int max_n, int timeout_ms);
  void reply(uint64_t unique, int err, const std::string& payload);

  // ---- node table (shared with the Python op layer) ------------------------------------------
  uint64_t node_of(const std::string& path);       // allocates
  std::string path_of(uint64_t nodeid, bool* ok);
  void forget_path(const std::string& path);
  void moved(const std::string& from, const std::string& to);

  // ---- attribute cache -------------------------------------------------------------------------
  // attr = struct fuse_attr (88 bytes; its ino field is rewritten per node), ttl in ms (0: do
  // not cache), entry/attr valid seconds reported to the kernel; blocks/lens: the file's blocks
  // (empty for directories) for native opens when `complete`.
  void put_attr(const std::string& path, const std::string& attr, int64_t ttl_ms, uint32_t valid_s,
                int64_t file_id, bool complete, const std::vector<int64_t>& blocks,
                const std::vector<int64_t>& lens);
  // Cache every entry of serialized ListStatus replies (alluxio.grpc.file.ListStatusPResponse
  // chunks) in one call: fuse_attr built natively from the decoded columns; Alluxio paths lose the
  // `strip` prefix (the mount's root).  Completed files get file_ttl_s, directories dir_ttl_s,
  // files still being written are skipped.  Returns the number cached.
  size_t cache_listing(const std::vector<std::string>& chunks, const std::string& strip, uint32_t uid, uint32_t gid,
                       uint32_t file_ttl_s, uint32_t dir_ttl_s);
  // LOOKUP reply payload (fuse_entry_out) for a cached path (allocating its node id).
  bool entry_reply(const std::string& path, std::string& out);
  void invalidate(const std::string& path, bool subtree);   // the path (and everything below it)
  void clear_attrs();

  // Kernel page cache policy of an open of `nodeid` (file id) -- shared by native and python
  // opens so both see the node's previous file id.
  bool keep_open(uint64_t nodeid, int64_t file_id);
  // Read-only mount that negotiated FUSE_NO_OPEN_SUPPORT: answer OPEN with ENOSYS (zero-message
  // opens) and serve fh-0 READs by pinning the blocks per request.
  void set_no_open(bool v) { no_open_.store(v); }
  // The kernel accepted FUSE_PASSTHROUGH: opens of single-block files held in a file dir (tmpfs
  // tier) get FOPEN_PASSTHROUGH with the block file as backing file -- reads never reach us.
  void set_passthrough(bool v) { passthrough_.store(v); }
  uint64_t passthrough_opens() const { return passthrough_opens_.load(); }
  // A shared DRAM arena (memfd `fd` mapped at `base`): READ replies splice its pages.  Before start().
  void add_arena(uint64_t base, uint64_t size, int fd);
  bool alive() const { return running_.load() && !dead_.load(); }
  // per opcode: native counts [0,64), python counts [64,128), native service ns [128,192)
  std::vector<uint64_t> stats();
  uint64_t native_opens() const { return native_opens_.load(); }
  uint64_t native_reads() const { return native_reads_.load(); }
  uint64_t fallback_opens() const { return fallback_opens_.load(); }

  // ---- write-behind of sequential writes (write handles the Python side registers) ----------
  // WRITE requests of a registered handle at its next offset are answered on the reader thread
  // and gathered into batches of kWriteBatchBytes, queued to Python as one request of opcode
  // kOpWriteBatch (body: fh u64, file offset u64, data) -- one Python call per batch instead of
  // one per 128 KiB request.  At most one batch per handle is queued or being applied at a time
  // (the next waits: bounded memory, in-order application by any Python thread).  FLUSH /
  // RELEASE / FSYNC of the handle queue its pending bytes first; Python waits for them
  // (wait_batches) before completing the file, and reports each batch back (batch_done).
  static constexpr uint32_t kOpWriteBatch = 4096;
  static constexpr size_t kWriteBatchBytes = 8u << 20;
  void register_write_handle(uint64_t fh, uint64_t offset);
  void unregister_write_handle(uint64_t fh);
  void batch_done(uint64_t fh, int err);
  int wait_batches(uint64_t fh, int timeout_ms);   // first error of the handle's batches (0: none)
  uint64_t write_batches() const { return write_batches_.load(); }

 private:
  struct WriteBehind {
    uint64_t next = 0;      // file offset the next sequential WRITE must carry
    uint64_t buf_off = 0;   // file offset of buf[0]
    std::string buf;
    int outstanding = 0;    // batches queued to / being applied by Python
    int err = 0;
    uint64_t nodeid = 0;
    uint32_t uid = 0, gid = 0, pid = 0;
  };
  std::mutex wb_mu_;
  std::condition_variable wb_cv_;
  std::unordered_map<uint64_t, WriteBehind> wb_;
  std::atomic<uint64_t> write_batches_{0};
  // queues the handle's pending bytes as a batch (wb_mu_ held in `lk`; waits for the previous one)
  void queue_batch(std::unique_lock<std::mutex>& lk, uint64_t fh, WriteBehind& w);
  bool write_behind(const char* req, size_t n);   // true: the WRITE was taken
  void flush_handle(uint64_t fh);                  // before a FLUSH / RELEASE / FSYNC goes to Python

  struct Attr {
    std::string raw;                 // fuse_attr
    int64_t expires_ms;
    uint32_t valid_s;
    int64_t file_id;
    bool complete;
    std::vector<int64_t> blocks, lens;
  };
  struct Seg {
    uint64_t file_off, len, src;     // file offset, bytes, source address
    bool device;
  };
  struct Handle {
    std::vector<int64_t> locks;
    std::vector<Seg> segs;
    uint64_t size = 0;
    int32_t backing = 0;             // FUSE passthrough backing id (reads bypass this server)
  };
  void loop(int idx);
  bool fast(const char* req, size_t n, std::string& out);   // true: answered (out = reply)
  void send(uint64_t unique, int err, const char* payload, size_t n);
  bool lookup_attr(const std::string& path, Attr& a);
  bool native_open(uint64_t nodeid, const std::string& path, uint32_t flags, uint64_t* fh, uint32_t* open_flags,
                   int32_t* backing);
  int32_t passthrough_backing(const Attr& a);
  void release_handle(uint64_t fh);
  bool pin(const Attr& a, uint64_t lo, uint64_t hi, Handle& h);
  bool splice_reply(const void* hdr, const std::vector<Seg>& segs);
  struct Arena {
    uint64_t base, size;
    int fd;
  };
  std::vector<Arena> arenas_;
  static thread_local int tl_pipe_[2];
  void unpin(Handle& h);

  int fd_;
  int nthreads_;
  BlockStore* store_;
  int64_t session_;
  int keep_cache_;
  std::atomic<bool> running_{false};
  std::atomic<bool> dead_{false};
  std::atomic<bool> no_open_{false};
  std::atomic<bool> passthrough_{false};
  std::atomic<uint64_t> passthrough_opens_{0};                  // a reader saw the connection end
  std::vector<std::thread> threads_;

  std::mutex qmu_;
  std::condition_variable qcv_;
  std::deque<FuseRequest> queue_;

  std::mutex nmu_;
  std::unordered_map<uint64_t, std::string> paths_;
  std::unordered_map<std::string, uint64_t> ids_;
  std::unordered_map<uint64_t, int64_t> last_open_fid_;
  uint64_t next_id_ = 2;

  std::mutex amu_;
  std::map<std::string, Attr> attrs_;             // ordered: subtree invalidation is a range

  std::mutex hmu_;
  std::unordered_map<uint64_t, Handle> handles_;
  uint64_t next_fh_ = 1;

  std::atomic<uint64_t> native_ops_[64];
  std::atomic<uint64_t> python_ops_[64];
  std::atomic<uint64_t> native_ns_[64];
  std::atomic<uint64_t> native_opens_{0}, native_reads_{0}, fallback_opens_{0};
};

}  // namespace amdx
