// Native block data server (see data_server.h).
#include "data_server.h"

#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <mutex>
#include <string>
#include <vector>

#include "h2_abi.h"

namespace amdx {

namespace {

// Pinned staging buffers for HBM chunks (hipHostMalloc is far too slow to call per stream).
class StagingPool {
 public:
  StagingPool(uint64_t size, bool pinned) : size_(size), pinned_(pinned) {}
  ~StagingPool() {
    for (void* p : free_) release(p);
  }
  uint8_t* get() {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!free_.empty()) {
        void* p = free_.back();
        free_.pop_back();
        return static_cast<uint8_t*>(p);
      }
    }
    void* p = nullptr;
    if (pinned_) {
      if (hipHostMalloc(&p, size_, hipHostMallocDefault) != hipSuccess) p = nullptr;
    }
    if (!p) p = std::malloc(size_);
    if (!p) throw StoreError(kErrOutOfSpace, "data server: cannot allocate a staging buffer");
    std::lock_guard<std::mutex> g(mu_);
    if (pinned_) pinned_set_.push_back(p);
    return static_cast<uint8_t*>(p);
  }
  void put(uint8_t* p) {
    std::lock_guard<std::mutex> g(mu_);
    if (free_.size() < 512) {
      free_.push_back(p);
      return;
    }
    release(p);
  }
  uint64_t size() const { return size_; }

 private:
  void release(void* p) {
    bool was_pinned = false;
    for (auto it = pinned_set_.begin(); it != pinned_set_.end(); ++it)
      if (*it == p) {
        was_pinned = true;
        pinned_set_.erase(it);
        break;
      }
    if (was_pinned) (void)hipHostFree(p);
    else std::free(p);
  }
  uint64_t size_;
  bool pinned_;
  std::mutex mu_;
  std::vector<void*> free_;
  std::vector<void*> pinned_set_;
};

// One D2H stream per I/O thread: staging copies of different connections never queue behind
// each other on a shared stream.
hipStream_t thread_stream(BlockStore* store) {
  thread_local hipStream_t st = nullptr;
  thread_local BlockStore* owner = nullptr;
  if (owner != store) {
    store->use_device();
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) st = nullptr;
    owner = store;
  }
  return st;
}

struct ReadRequestMsg {
  int64_t block_id = 0;
  int64_t offset = 0;
  int64_t length = 0;
  bool promote = false;
  int64_t chunk_size = 0;
  bool has_ufs = false;
  bool has_ack = false;
  int64_t offset_received = 0;
};

// ReadRequest (proto/defs/block.py): block_id=1 offset=2 length=3 promote=4 chunk_size=5
// open_ufs_block_options=6 offset_received=7 position_short=8.
bool parse_read_request(const char* data, size_t n, ReadRequestMsg* r) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(data);
  size_t i = 0;
  while (i < n) {
    uint64_t key;
    if (!h2::get_varint(p, n, &i, &key)) return false;
    const uint32_t field = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
    if (wt == 0) {
      uint64_t v;
      if (!h2::get_varint(p, n, &i, &v)) return false;
      switch (field) {
        case 1: r->block_id = (int64_t)v; break;
        case 2: r->offset = (int64_t)v; break;
        case 3: r->length = (int64_t)v; break;
        case 4: r->promote = v != 0; break;
        case 5: r->chunk_size = (int64_t)v; break;
        case 7: r->has_ack = true; r->offset_received = (int64_t)v; break;
        default: break;
      }
    } else if (wt == 2) {
      uint64_t len;
      if (!h2::get_varint(p, n, &i, &len) || len > n - i) return false;
      if (field == 6) r->has_ufs = true;
      i += (size_t)len;
    } else if (wt == 1) {
      if (n - i < 8) return false;
      i += 8;
    } else if (wt == 5) {
      if (n - i < 4) return false;
      i += 4;
    } else {
      return false;
    }
  }
  return true;
}

class BlockReadStream : public NativeStream {
 public:
  BlockReadStream(BlockStore* store, int64_t session, int64_t lock_id, int64_t block_id, uint64_t pos, uint64_t end,
                  uint64_t chunk, uint64_t window, bool device, bool unix_peer, std::shared_ptr<StagingPool> pool,
                  std::shared_ptr<DataServerStats> stats)
      : store_(store), session_(session), lock_(lock_id), block_(block_id), pos_(pos), acked_(pos), end_(end),
        chunk_(chunk), window_(window), device_(device), unix_(unix_peer), pool_(std::move(pool)), stats_(std::move(stats)) {}

  ~BlockReadStream() override {
    if (stage_) pool_->put(stage_);
    try {
      store_->unlock(lock_);
      store_->cleanup_session(session_);
    } catch (...) {
    }
  }

  void on_message(const char* p, size_t n) override {
    ReadRequestMsg r;
    if (parse_read_request(p, n, &r) && r.has_ack && (uint64_t)r.offset_received > acked_)
      acked_ = (uint64_t)r.offset_received;
  }

  ssize_t produce(uint8_t* dst, size_t max, bool* eof, int* status, std::string* msg) override {
    size_t w = 0;
    try {
      while (w < max) {
        if (hdr_off_ < hdr_.size()) {   // gRPC prefix + protobuf header of the current chunk
          const size_t n = std::min(max - w, hdr_.size() - hdr_off_);
          std::memcpy(dst + w, hdr_.data() + hdr_off_, n);
          hdr_off_ += n;
          w += n;
          continue;
        }
        if (left_ > 0) {                // chunk bytes
          const size_t n = (size_t)std::min<uint64_t>(max - w, left_);
          if (device_) {
            std::memcpy(dst + w, stage_ + stage_off_, n);
            stage_off_ += n;
          } else {                      // DRAM arena / file tier: straight into the frame
            std::vector<ReadReq> rq{ReadReq{block_, data_pos_, n, reinterpret_cast<uint64_t>(dst + w),
                                            (int)MemKind::kHost}};
            store_->read_batch(rq, 0, false);   // host copies: nothing to wait for on a stream
            data_pos_ += n;
          }
          left_ -= n;
          w += n;
          stats_->bytes.fetch_add(n, std::memory_order_relaxed);
          if (unix_) stats_->domain_bytes.fetch_add(n, std::memory_order_relaxed);
          continue;
        }
        if (pos_ >= end_) {
          *eof = true;
          break;
        }
        if (pos_ - acked_ >= window_) break;   // wait for offset_received
        next_chunk();
      }
    } catch (const std::exception& e) {
      *status = 13;   // INTERNAL
      *msg = std::string("reading block ") + std::to_string(block_) + ": " + e.what();
      return -1;
    }
    return (ssize_t)w;
  }

 private:
  void next_chunk() {
    const uint64_t n = std::min(chunk_, end_ - pos_);
    hdr_ = h2::read_response_prefix(n);
    hdr_off_ = 0;
    left_ = n;
    data_pos_ = pos_;
    if (device_) {
      if (!stage_) stage_ = pool_->get();
      std::vector<ReadReq> rq{ReadReq{block_, pos_, n, reinterpret_cast<uint64_t>(stage_), (int)MemKind::kHost}};
      store_->read_batch(rq, reinterpret_cast<uint64_t>(thread_stream(store_)), true);
      stage_off_ = 0;
      stats_->staged_bytes.fetch_add(n, std::memory_order_relaxed);
    }
    pos_ += n;
    stats_->chunks.fetch_add(1, std::memory_order_relaxed);
  }

  BlockStore* store_;
  int64_t session_, lock_, block_;
  uint64_t pos_, acked_, end_, chunk_, window_;
  bool device_, unix_;
  std::shared_ptr<StagingPool> pool_;
  std::shared_ptr<DataServerStats> stats_;
  std::string hdr_;
  size_t hdr_off_ = 0;
  uint64_t left_ = 0, data_pos_ = 0;
  uint8_t* stage_ = nullptr;
  uint64_t stage_off_ = 0;
};

std::atomic<int64_t> g_session{(int64_t)1 << 62};   // above the Python range (utils/ids.py)

// ---- WriteBlock ---------------------------------------------------------------------------------
// WriteRequestCommand (proto/defs/block.py): type=1 id=2 offset=3 tier=4 flush=5
// create_ufs_file_options=6 create_ufs_block_options=7 medium_type=8 pin_on_create=9
// space_to_reserve=10.  WriteRequest: command=1 chunk=2 (Chunk: data=1).
// CreateUfsFileOptions (proto/defs/common.py): ufs_path=1 owner=2 group=3 mode=4 mount_id=5 acl=6.
struct WriteCmd {
  int64_t type = 0, id = 0, offset = 0, tier = 0, reserve = 0;
  bool has_tier = false, flush = false, pin = false, has_ufs = false, has_ufs_file = false;
  std::string medium;
  std::string ufs_path;
  int64_t ufs_mode = 0, ufs_mount = 0;
};

bool skip_field(const uint8_t* p, size_t n, size_t* i, uint32_t wt) {
  if (wt == 0) {
    uint64_t v;
    return h2::get_varint(p, n, i, &v);
  }
  if (wt == 2) {
    uint64_t len;
    if (!h2::get_varint(p, n, i, &len) || len > n - *i) return false;
    *i += (size_t)len;
    return true;
  }
  if (wt == 1 && n - *i >= 8) { *i += 8; return true; }
  if (wt == 5 && n - *i >= 4) { *i += 4; return true; }
  return false;
}

bool parse_ufs_file_options(const uint8_t* p, size_t n, WriteCmd* c) {
  size_t i = 0;
  while (i < n) {
    uint64_t key;
    if (!h2::get_varint(p, n, &i, &key)) return false;
    const uint32_t field = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
    if (wt == 0 && (field == 4 || field == 5)) {
      uint64_t v;
      if (!h2::get_varint(p, n, &i, &v)) return false;
      if (field == 4) c->ufs_mode = (int64_t)(int32_t)v;
      else c->ufs_mount = (int64_t)v;
    } else if (wt == 2 && field == 1) {
      uint64_t len;
      if (!h2::get_varint(p, n, &i, &len) || len > n - i) return false;
      c->ufs_path.assign(reinterpret_cast<const char*>(p + i), (size_t)len);
      i += (size_t)len;
    } else if (!skip_field(p, n, &i, wt)) {
      return false;
    }
  }
  return true;
}

bool parse_write_command(const uint8_t* p, size_t n, WriteCmd* c) {
  size_t i = 0;
  while (i < n) {
    uint64_t key;
    if (!h2::get_varint(p, n, &i, &key)) return false;
    const uint32_t field = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
    if (wt == 0) {
      uint64_t v;
      if (!h2::get_varint(p, n, &i, &v)) return false;
      switch (field) {
        case 1: c->type = (int64_t)v; break;
        case 2: c->id = (int64_t)v; break;
        case 3: c->offset = (int64_t)v; break;
        case 4: c->tier = (int64_t)(int32_t)v; c->has_tier = true; break;
        case 5: c->flush = v != 0; break;
        case 9: c->pin = v != 0; break;
        case 10: c->reserve = (int64_t)v; break;
        default: break;
      }
    } else if (wt == 2) {
      uint64_t len;
      if (!h2::get_varint(p, n, &i, &len) || len > n - i) return false;
      if (field == 6 || field == 7) c->has_ufs = true;
      if (field == 6) {
        c->has_ufs_file = true;
        if (!parse_ufs_file_options(p + i, (size_t)len, c)) return false;
      }
      if (field == 8) c->medium.assign(reinterpret_cast<const char*>(p + i), (size_t)len);
      i += (size_t)len;
    } else if (!skip_field(p, n, &i, wt)) {
      return false;
    }
  }
  return true;
}

// Splits one WriteRequest into its command (if any) and its chunk bytes (pointer into `data`).
bool parse_write_request(const char* data, size_t n, WriteCmd* cmd, bool* has_cmd, const uint8_t** chunk,
                         size_t* chunk_len) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(data);
  size_t i = 0;
  *has_cmd = false;
  *chunk = nullptr;
  *chunk_len = 0;
  while (i < n) {
    uint64_t key;
    if (!h2::get_varint(p, n, &i, &key)) return false;
    const uint32_t field = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
    if (wt == 2 && (field == 1 || field == 2)) {
      uint64_t len;
      if (!h2::get_varint(p, n, &i, &len) || len > n - i) return false;
      if (field == 1) {
        *has_cmd = true;
        if (!parse_write_command(p + i, (size_t)len, cmd)) return false;
      } else {                                    // Chunk{data=1}
        size_t j = i;
        const size_t end = i + (size_t)len;
        while (j < end) {
          uint64_t k2;
          if (!h2::get_varint(p, end, &j, &k2)) return false;
          if ((k2 >> 3) == 1 && (k2 & 7) == 2) {
            uint64_t l2;
            if (!h2::get_varint(p, end, &j, &l2) || l2 > end - j) return false;
            *chunk = p + j;
            *chunk_len = (size_t)l2;
            j += (size_t)l2;
          } else if (!skip_field(p, end, &j, (uint32_t)(k2 & 7))) {
            return false;
          }
        }
      }
      i += (size_t)len;
    } else if (!skip_field(p, n, &i, wt)) {
      return false;
    }
  }
  return true;
}

int grpc_status_of(const StoreError& e) {
  switch (e.code) {
    case kErrNotFound: return 5;          // NOT_FOUND
    case kErrAlreadyExists: return 6;     // ALREADY_EXISTS
    case kErrOutOfSpace: return 8;        // RESOURCE_EXHAUSTED
    case kErrInvalidArgument: return 3;   // INVALID_ARGUMENT
    case kErrInvalidState: return 9;      // FAILED_PRECONDITION
    case kErrTimeout: return 4;           // DEADLINE_EXCEEDED
    default: return 13;                   // INTERNAL
  }
}

std::string write_response_frame(uint64_t offset) {
  std::string m;
  if (offset) {
    h2::put_varint(m, (1u << 3) | 0);
    h2::put_varint(m, offset);
  }
  std::string f;
  f.push_back('\0');
  h2::put_be32(f, (uint32_t)m.size());
  f += m;
  return f;
}

// Response side shared by the write streams: queued WriteResponse frames, then EOF or a failure.
class WriteStreamBase : public NativeStream {
 public:
  ssize_t produce(uint8_t* dst, size_t max, bool* eof, int* status, std::string* msg) override {
    if (err_) {
      *status = err_status_;
      *msg = err_msg_;
      return -1;
    }
    const size_t n = std::min(max, out_.size() - out_off_);
    std::memcpy(dst, out_.data() + out_off_, n);
    out_off_ += n;
    if (out_off_ == out_.size()) {
      out_.clear();
      out_off_ = 0;
      if (done_) *eof = true;
    }
    return (ssize_t)n;
  }

 protected:
  void fail(int status, const std::string& msg) {
    if (err_) return;
    err_ = true;
    err_status_ = status;
    err_msg_ = msg;
  }

  std::string out_;
  size_t out_off_ = 0;
  bool ended_ = false, done_ = false, err_ = false;
  int err_status_ = 0;
  std::string err_msg_;
};

class BlockWriteStream : public WriteStreamBase {
 public:
  BlockWriteStream(BlockStore* store, int64_t session, int64_t block_id, uint64_t pos, bool pin, bool device,
                   uint32_t commit_method, std::shared_ptr<StagingPool> pool, std::shared_ptr<DataServerStats> stats)
      : store_(store), session_(session), block_(block_id), pos_(pos), pin_(pin), device_(device),
        commit_(commit_method), pool_(std::move(pool)), stats_(std::move(stats)) {}

  ~BlockWriteStream() override {
    if (stage_) pool_->put(stage_);
    try {
      store_->cleanup_session(session_);     // aborts the temp block unless Python committed it
    } catch (...) {
    }
  }

  void on_message(const char* p, size_t n) override {
    if (err_ || ended_) return;
    WriteCmd cmd;
    bool has_cmd;
    const uint8_t* chunk;
    size_t len;
    if (!parse_write_request(p, n, &cmd, &has_cmd, &chunk, &len)) {
      fail(3, "malformed WriteRequest");
      return;
    }
    try {
      if (len) write(chunk, len);
    } catch (const StoreError& e) {
      fail(grpc_status_of(e), std::string("writing block ") + std::to_string(block_) + ": " + e.what());
      return;
    } catch (const std::exception& e) {
      fail(13, std::string("writing block ") + std::to_string(block_) + ": " + e.what());
      return;
    }
    if (has_cmd && cmd.flush) out_ += write_response_frame(pos_);
  }

  bool on_end(uint32_t* method, std::string* payload) override {
    ended_ = true;
    if (err_) return false;
    // NativeWriteCommitRequest: session_id=1 block_id=2 length=3 pin=4
    std::string m;
    h2::put_varint(m, (1u << 3));
    h2::put_varint(m, (uint64_t)session_);
    h2::put_varint(m, (2u << 3));
    h2::put_varint(m, (uint64_t)block_);
    h2::put_varint(m, (3u << 3));
    h2::put_varint(m, pos_);
    if (pin_) {
      h2::put_varint(m, (4u << 3));
      h2::put_varint(m, 1);
    }
    *method = commit_;
    *payload = std::move(m);
    return true;
  }

  void on_reply(int status, const std::string& msg, const std::string& payload) override {
    if (status != 0) {
      fail(status, msg);
      return;
    }
    out_.push_back('\0');
    h2::put_be32(out_, (uint32_t)payload.size());
    out_ += payload;
    done_ = true;
  }

 private:
  void write(const uint8_t* p, size_t n) {
    if (!device_) {       // host arena / file dir: straight from the HTTP/2 receive buffer
      store_->write(session_, block_, pos_, reinterpret_cast<uint64_t>(p), n, (int)MemKind::kHost, 0, true);
    } else {              // HBM: through pinned staging, so the H2D is a DMA and not a pageable copy
      if (!stage_) stage_ = pool_->get();
      hipStream_t st = thread_stream(store_);
      size_t done = 0;
      while (done < n) {
        const size_t k = (size_t)std::min<uint64_t>(n - done, pool_->size());
        std::memcpy(stage_, p + done, k);
        store_->write(session_, block_, pos_ + done, reinterpret_cast<uint64_t>(stage_), k, (int)MemKind::kHost,
                      reinterpret_cast<uint64_t>(st), true);
        done += k;
      }
    }
    pos_ += n;
    stats_->write_bytes.fetch_add(n, std::memory_order_relaxed);
  }

  BlockStore* store_;
  int64_t session_, block_;
  uint64_t pos_;
  bool pin_, device_;
  uint32_t commit_;
  std::shared_ptr<StagingPool> pool_;
  std::shared_ptr<DataServerStats> stats_;
  uint8_t* stage_ = nullptr;
};

int grpc_status_of_errno(int e) {
  switch (e) {
    case ENOSPC:
    case EDQUOT: return 8;                    // RESOURCE_EXHAUSTED
    case EACCES:
    case EPERM:
    case EROFS: return 7;                     // PERMISSION_DENIED
    case EEXIST: return 6;                    // ALREADY_EXISTS
    case ENOENT:
    case ENOTDIR: return 5;                   // NOT_FOUND
    default: return 13;                       // INTERNAL
  }
}

// mkdir -p of the directories above `path` (os.makedirs(parent, exist_ok=True) of the local UFS).
bool make_parents(const std::string& path, int* err) {
  for (size_t i = path.find('/', 1); i != std::string::npos; i = path.find('/', i + 1)) {
    const std::string dir = path.substr(0, i);
    if (::mkdir(dir.c_str(), 0777) != 0 && errno != EEXIST) {
      *err = errno;
      return false;
    }
  }
  return true;
}

// UFS_FILE WriteBlock into a local-directory UFS: chunks are written to a temp file beside the
// target on the I/O thread; the half-close sets the mode and renames it over the target (the
// local UFS's atomic create, underfs/local.py _AtomicWriter).  A failed or cancelled call
// removes the temp file and leaves the target untouched.
class UfsFileWriteStream : public WriteStreamBase {
 public:
  UfsFileWriteStream(const std::string& path, int mode, std::shared_ptr<DataServerStats> stats)
      : path_(path), mode_(mode), stats_(std::move(stats)) {}

  // Creates the parents and the temp file; false with *status / *msg set on failure.
  bool open(int* status, std::string* msg) {
    int e = 0;
    if (!make_parents(path_, &e)) {
      *status = grpc_status_of_errno(e);
      *msg = "creating the parent of " + path_ + ": " + std::strerror(e);
      return false;
    }
    thread_local std::mt19937_64 rng(std::random_device{}());
    char tag[17];
    std::snprintf(tag, sizeof(tag), "%08x", (unsigned)(rng() & 0xffffffffu));
    tmp_ = path_ + ".alluxio." + tag + ".tmp";
    fd_ = ::open(tmp_.c_str(), O_WRONLY | O_CREAT | O_EXCL | O_CLOEXEC, 0666);
    if (fd_ < 0) {
      e = errno;
      *status = grpc_status_of_errno(e);
      *msg = "creating " + tmp_ + ": " + std::strerror(e);
      return false;
    }
    return true;
  }

  ~UfsFileWriteStream() override {
    if (fd_ >= 0) ::close(fd_);
    if (!committed_ && !tmp_.empty()) ::unlink(tmp_.c_str());
  }

  void on_message(const char* p, size_t n) override {
    if (err_ || ended_) return;
    WriteCmd cmd;
    bool has_cmd;
    const uint8_t* chunk;
    size_t len;
    if (!parse_write_request(p, n, &cmd, &has_cmd, &chunk, &len)) {
      fail(3, "malformed WriteRequest");
      return;
    }
    size_t done = 0;
    while (done < len) {
      const ssize_t w = ::write(fd_, chunk + done, len - done);
      if (w < 0) {
        if (errno == EINTR) continue;
        const int e = errno;
        fail(grpc_status_of_errno(e), "writing " + path_ + ": " + std::strerror(e));
        return;
      }
      done += (size_t)w;
    }
    pos_ += len;
    stats_->ufs_write_bytes.fetch_add(len, std::memory_order_relaxed);
    if (has_cmd && cmd.flush) out_ += write_response_frame(pos_);
  }

  bool on_end(uint32_t*, std::string*) override {
    ended_ = true;
    if (err_) return false;
    const int fd = fd_;
    fd_ = -1;
    int e = 0;
    if (::fchmod(fd, (mode_t)mode_) != 0) e = errno;
    if (::close(fd) != 0 && !e) e = errno;
    if (!e && ::rename(tmp_.c_str(), path_.c_str()) != 0) e = errno;
    if (e) {
      fail(grpc_status_of_errno(e), "completing " + path_ + ": " + std::strerror(e));
      return false;
    }
    committed_ = true;
    out_ += write_response_frame(pos_);
    done_ = true;
    return false;
  }

 private:
  std::string path_, tmp_;
  int mode_;
  int fd_ = -1;
  uint64_t pos_ = 0;
  bool committed_ = false;
  std::shared_ptr<DataServerStats> stats_;
};

}  // namespace

namespace {
std::string strip_file_scheme(const std::string& p) { return p.compare(0, 7, "file://") == 0 ? p.substr(7) : p; }
}  // namespace

void LocalUfsRoots::set(int64_t mount_id, const std::string& root) {
  std::string r = strip_file_scheme(root);
  while (!r.empty() && r.back() == '/') r.pop_back();     // "/" -> "" (every absolute path)
  std::lock_guard<std::mutex> g(mu_);
  roots_[mount_id] = r;
}

void LocalUfsRoots::remove(int64_t mount_id) {
  std::lock_guard<std::mutex> g(mu_);
  roots_.erase(mount_id);
}

size_t LocalUfsRoots::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return roots_.size();
}

bool LocalUfsRoots::resolve(int64_t mount_id, const std::string& ufs_path, std::string* local) const {
  std::string root;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = roots_.find(mount_id);
    if (it == roots_.end()) return false;
    root = it->second;
  }
  const std::string p = strip_file_scheme(ufs_path);
  if (p.size() < 2 || p[0] != '/') return false;
  for (size_t i = 1; i <= p.size();) {                     // no empty, "." or ".." component
    size_t j = p.find('/', i);
    if (j == std::string::npos) j = p.size();
    const size_t n = j - i;
    if (n == 0 || (n == 1 && p[i] == '.') || (n == 2 && p[i] == '.' && p[i + 1] == '.')) return false;
    i = j + 1;
  }
  if (p.size() <= root.size() + 1 || p.compare(0, root.size(), root) != 0 || p[root.size()] != '/') return false;
  *local = p;
  return true;
}

void serve_block_reads(FrameRpcServer& srv, uint32_t method, BlockStore* store, uint64_t max_chunk, uint64_t window,
                       std::shared_ptr<DataServerStats> stats) {
  if (max_chunk == 0) max_chunk = 2u << 20;
  if (window == 0) window = 4u << 20;
  auto pool = std::make_shared<StagingPool>(max_chunk, store->has_device());
  FrameRpcServer* s = &srv;
  srv.set_native_stream(method, [=](const std::string& first, const std::string& cid, const std::string& user,
                                    bool unix_peer, int* status, std::string* msg) -> std::unique_ptr<NativeStream> {
    (void)user;
    ReadRequestMsg r;
    if (!parse_read_request(first.data(), first.size(), &r)) {
      *status = 3;   // INVALID_ARGUMENT
      *msg = "malformed ReadRequest";
      return nullptr;
    }
    if (s->require_channel_auth() && (cid.empty() || !s->channel_user(cid, nullptr))) {
      *status = 16;  // UNAUTHENTICATED
      *msg = cid.empty() ? "channel is not authenticated (no channel-id)"
                         : "channel " + cid + " is not authenticated";
      return nullptr;
    }
    // UFS read-through, promotion and locks that would wait: the Python servicer
    if (r.has_ufs || r.promote || r.offset < 0) {
      stats->declined.fetch_add(1, std::memory_order_relaxed);
      return nullptr;
    }
    const int64_t session = g_session.fetch_add(1);
    int64_t lock = -1;
    try {
      lock = store->lock_block(session, r.block_id, false, 0);
    } catch (const StoreError& e) {
      lock = -1;   // not (yet) committed here
    }
    if (lock < 0) {
      stats->declined.fetch_add(1, std::memory_order_relaxed);
      return nullptr;
    }
    try {
      const BlockInfoOut info = store->block_info(r.block_id);
      const uint64_t off = (uint64_t)r.offset;
      if (off > info.length) {
        store->unlock(lock);
        *status = 11;  // OUT_OF_RANGE
        *msg = "offset " + std::to_string(off) + " beyond block " + std::to_string(r.block_id) + " of " +
               std::to_string(info.length) + " bytes";
        return nullptr;
      }
      const uint64_t end = r.length > 0 ? std::min<uint64_t>(info.length, off + (uint64_t)r.length) : info.length;
      const uint64_t chunk = r.chunk_size > 0 ? std::min<uint64_t>((uint64_t)r.chunk_size, max_chunk) : std::min<uint64_t>(1u << 20, max_chunk);
      const bool device = store->dir_spec(info.dir).kind == DirKind::kDevice;
      store->access_block(session, r.block_id);
      stats->streams.fetch_add(1, std::memory_order_relaxed);
      return std::unique_ptr<NativeStream>(new BlockReadStream(store, session, lock, r.block_id, off, end, chunk,
                                                               window, device, unix_peer, pool, stats));
    } catch (const std::exception& e) {
      try {
        store->unlock(lock);
      } catch (...) {
      }
      *status = 13;
      *msg = e.what();
      return nullptr;
    }
  });
}

void serve_block_writes(FrameRpcServer& srv, uint32_t method, uint32_t commit_method, BlockStore* store,
                        uint64_t stage_bytes, std::shared_ptr<DataServerStats> stats,
                        std::shared_ptr<LocalUfsRoots> ufs_roots) {
  if (stage_bytes == 0) stage_bytes = 4u << 20;
  auto pool = std::make_shared<StagingPool>(stage_bytes, store->has_device());
  FrameRpcServer* s = &srv;
  srv.set_native_stream(method, [=](const std::string& first, const std::string& cid, const std::string& user,
                                    bool unix_peer, int* status, std::string* msg) -> std::unique_ptr<NativeStream> {
    (void)user;
    (void)unix_peer;
    WriteCmd cmd;
    bool has_cmd;
    const uint8_t* chunk;
    size_t len;
    if (!parse_write_request(first.data(), first.size(), &cmd, &has_cmd, &chunk, &len) || !has_cmd) {
      *status = 3;
      *msg = "WriteBlock stream must start with a command";
      return nullptr;
    }
    if (s->require_channel_auth() && (cid.empty() || !s->channel_user(cid, nullptr))) {
      *status = 16;
      *msg = cid.empty() ? "channel is not authenticated (no channel-id)" : "channel " + cid + " is not authenticated";
      return nullptr;
    }
    std::string local;
    if (cmd.type == 1 && cmd.has_ufs_file && ufs_roots && ufs_roots->resolve(cmd.ufs_mount, cmd.ufs_path, &local)) {
      auto us = std::unique_ptr<UfsFileWriteStream>(
          new UfsFileWriteStream(local, cmd.ufs_mode > 0 ? (int)(cmd.ufs_mode & 07777) : 0644, stats));
      if (!us->open(status, msg)) return nullptr;
      stats->ufs_write_streams.fetch_add(1, std::memory_order_relaxed);
      if (len) us->on_message(first.data(), first.size());
      return us;
    }
    if (cmd.type != 0 || cmd.has_ufs || cmd.offset < 0) {   // other UFS_FILE / UFS_FALLBACK_BLOCK: Python
      stats->write_declined.fetch_add(1, std::memory_order_relaxed);
      return nullptr;
    }
    const int64_t session = g_session.fetch_add(1);
    const uint64_t reserve = cmd.reserve > 0 ? (uint64_t)cmd.reserve : (1u << 20);
    try {
      const int dir = store->create_block(session, cmd.id, cmd.medium.empty() ? (cmd.has_tier ? (int)cmd.tier : 0) : -1,
                                          cmd.medium, reserve, true, cmd.pin);
      const bool device = store->dir_spec(dir).kind == DirKind::kDevice;
      auto ws = std::unique_ptr<BlockWriteStream>(new BlockWriteStream(store, session, cmd.id, (uint64_t)cmd.offset,
                                                                       cmd.pin, device, commit_method, pool, stats));
      stats->write_streams.fetch_add(1, std::memory_order_relaxed);
      if (len) ws->on_message(first.data(), first.size());   // a command that carries data too
      return ws;
    } catch (const StoreError& e) {
      try {
        store->cleanup_session(session);
      } catch (...) {
      }
      *status = grpc_status_of(e);
      *msg = e.what();
      return nullptr;
    }
  });
}

}  // namespace amdx
