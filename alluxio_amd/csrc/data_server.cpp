// Native block data server (see data_server.h).
#include "data_server.h"

#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <condition_variable>
#include <deque>
#include <map>
#include <pthread.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "h2_abi.h"
#include "numa_host.h"

namespace amdx {

namespace {

// Pinned staging buffers for HBM chunks (hipHostMalloc is far too slow to call per stream).
class StagingPool {
 public:
  StagingPool(uint64_t size, bool pinned, int device = 0) : size_(size), pinned_(pinned), device_(device) {}
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
    if (pinned_) p = pinned_alloc_near(size_, device_);   // on the GPU's NUMA node
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
  int device_;
  std::mutex mu_;
  std::vector<void*> free_;
  std::vector<void*> pinned_set_;
};

// One D2H stream per I/O thread (and device): staging copies of different connections never
// queue behind each other on a shared stream.
hipStream_t thread_stream(const StoreRef& store) {
  store->use_device();
  return thread_stream_on(store->device());
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
  std::string ufs_opts;   // serialized OpenUfsBlockOptions
};

// OpenUfsBlockOptions (proto/defs/common.py): ufs_path=1 offset_in_file=2 block_size=3
// maxUfsReadConcurrency=4 mountId=5 no_cache=6 user=7 block_in_ufs_tier=8.
struct UfsOpts {
  std::string ufs_path;
  int64_t offset_in_file = 0, block_size = 0, mount_id = 0;
  bool no_cache = false, block_in_ufs_tier = false;
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
      if (field == 6) {
        r->has_ufs = true;
        r->ufs_opts.assign(data + i, (size_t)len);
      }
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

// Optional per-chunk timeline of HBM ReadBlock streams (ALLUXIO_READ_TRACE=<file>, read once):
// when each chunk's D2H was issued, when it ran on the GPU (timing events against a base event
// recorded with the host clock), how long the I/O thread waited for it, and when its bytes were
// handed to the socket.  Evidence that chunk k+1's DMA runs while chunk k is being sent.
struct ReadTraceRec {
  uint64_t pos, len;
  int64_t issue_ns = 0, gpu_start_ns = 0, gpu_end_ns = 0, ready_ns = 0, wait_ns = 0, send_first_ns = 0,
          send_last_ns = 0;
};

class ReadTraceSink {
 public:
  static ReadTraceSink& get() {
    static ReadTraceSink* s = new ReadTraceSink();
    return *s;
  }
  bool on() const { return !path_.empty(); }
  void write(int64_t block, const std::vector<ReadTraceRec>& recs) {
    if (recs.empty()) return;
    std::lock_guard<std::mutex> g(mu_);
    if (written_ > 200000) return;
    FILE* f = std::fopen(path_.c_str(), "a");
    if (!f) return;
    for (const auto& r : recs) {
      std::fprintf(f,
                   "{\"block\": %lld, \"pos\": %llu, \"len\": %llu, \"issue_ns\": %lld, \"gpu_start_ns\": %lld, "
                   "\"gpu_end_ns\": %lld, \"ready_ns\": %lld, \"wait_ns\": %lld, \"send_first_ns\": %lld, "
                   "\"send_last_ns\": %lld}\n",
                   (long long)block, (unsigned long long)r.pos, (unsigned long long)r.len, (long long)r.issue_ns,
                   (long long)r.gpu_start_ns, (long long)r.gpu_end_ns, (long long)r.ready_ns, (long long)r.wait_ns,
                   (long long)r.send_first_ns, (long long)r.send_last_ns);
      ++written_;
    }
    std::fclose(f);
  }

 private:
  ReadTraceSink() {
    const char* p = std::getenv("ALLUXIO_READ_TRACE");
    if (p) path_ = p;
  }
  std::string path_;
  std::mutex mu_;
  uint64_t written_ = 0;
};

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// Send-side timing of one ReadBlock stream (DataServerStats::SendTiming): the gaps between a call
// of produce that stopped for want of window or data and the next call.
class SendClock {
 public:
  explicit SendClock(DataServerStats::SendTiming* t) : t_(t), t0_(now_ns()) {}
  void resume() {                 // produce entered: close the open gap
    if (!kind_) return;
    const uint64_t d = (uint64_t)(now_ns() - since_);
    (kind_ == 1 ? t_->window_ns : t_->data_ns).fetch_add(d, std::memory_order_relaxed);
    kind_ = 0;
  }
  void stall(int kind) {          // 1 window full, 2 next bytes not there
    kind_ = kind;
    since_ = now_ns();
    (kind == 1 ? t_->window_stalls : t_->data_stalls).fetch_add(1, std::memory_order_relaxed);
  }
  void add_data_wait(int64_t ns) { t_->data_ns.fetch_add((uint64_t)ns, std::memory_order_relaxed); }
  void sent() {
    if (first_) return;
    first_ = true;
    t_->first_ns.fetch_add((uint64_t)(now_ns() - t0_), std::memory_order_relaxed);
  }
  void done() {
    if (done_) return;
    done_ = true;
    t_->streams.fetch_add(1, std::memory_order_relaxed);
    t_->life_ns.fetch_add((uint64_t)(now_ns() - t0_), std::memory_order_relaxed);
  }

 private:
  DataServerStats::SendTiming* t_;
  int64_t t0_, since_ = 0;
  int kind_ = 0;
  bool first_ = false, done_ = false;
};

class BlockReadStream : public NativeStream {
 public:
  BlockReadStream(StoreRef store, int64_t session, int64_t lock_id, int64_t block_id, uint64_t pos, uint64_t end,
                  uint64_t chunk, uint64_t window, bool device, bool unix_peer, std::shared_ptr<StagingPool> pool,
                  std::shared_ptr<DataServerStats> stats)
      : store_(std::move(store)), session_(session), lock_(lock_id), block_(block_id), pos_(pos), acked_(pos), end_(end),
        chunk_(chunk), window_(window), device_(device), unix_(unix_peer), pool_(std::move(pool)), stats_(std::move(stats)),
        clock_(&stats_->send[0]) {}

  ~BlockReadStream() override {
    for (int k = 0; k < 2; ++k) {
      if (!slot_[k].buf) continue;
      if (slot_[k].inflight) (void)hipEventSynchronize(slot_[k].ev);   // no DMA into a pooled buffer
      if (slot_[k].ev) (void)hipEventDestroy(slot_[k].ev);
      if (slot_[k].t0) (void)hipEventDestroy(slot_[k].t0);
      pool_->put(slot_[k].buf);
    }
    if (!trace_.empty()) {
      ReadTraceSink::get().write(block_, trace_);
    }
    if (base_ev_) (void)hipEventDestroy(base_ev_);
    try {
      store_->unlock(lock_);
      store_->cleanup_session(session_);
    } catch (...) {
    }
  }

  void on_message(const char* p, size_t n) override {
    ReadRequestMsg r;
    // acks only move forward and never past what was sent (an ack beyond it would wrap the
    // unsigned window test below and stall the call with its read lock held)
    if (parse_read_request(p, n, &r) && r.has_ack && (uint64_t)r.offset_received > acked_)
      acked_ = std::min<uint64_t>((uint64_t)r.offset_received, pos_);
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
            std::memcpy(dst + w, slot_[cur_].buf + stage_off_, n);
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

  // HBM blocks: the chunk's gRPC/protobuf prefix and the bytes in the staging slot go to the
  // socket as they are (no copy into the HTTP/2 frame buffer).  A DATA frame never crosses a chunk
  // boundary: moving to the next chunk re-stages the slot the previous chunk sat in.
  ssize_t produce_spans(size_t max, ByteSpan* spans, int max_spans, int* nspans, bool* eof, int* status,
                        std::string* msg) override {
    if (!device_ || max_spans < 2) return -2;
    clock_.resume();
    size_t w = 0;
    int ns = 0;
    try {
      while (w < max && ns < max_spans) {
        if (hdr_off_ < hdr_.size()) {
          const size_t n = std::min(max - w, hdr_.size() - hdr_off_);
          spans[ns++] = ByteSpan{reinterpret_cast<const uint8_t*>(hdr_.data()) + hdr_off_, n};
          hdr_off_ += n;
          w += n;
          continue;
        }
        if (left_ > 0) {
          const size_t n = (size_t)std::min<uint64_t>(max - w, left_);
          spans[ns++] = ByteSpan{slot_[cur_].buf + stage_off_, n};
          if (tracing_ && cur_rec_ >= 0) {
            const int64_t t = now_ns();
            if (!trace_[cur_rec_].send_first_ns) trace_[cur_rec_].send_first_ns = t;
            trace_[cur_rec_].send_last_ns = t;
          }
          stage_off_ += n;
          left_ -= n;
          w += n;
          stats_->bytes.fetch_add(n, std::memory_order_relaxed);
          if (unix_) stats_->domain_bytes.fetch_add(n, std::memory_order_relaxed);
          continue;
        }
        if (w > 0) break;                      // this frame ends with the chunk
        if (pos_ >= end_) {
          *eof = true;
          clock_.done();
          break;
        }
        if (pos_ - acked_ >= window_) {        // wait for offset_received
          clock_.stall(1);
          break;
        }
        next_chunk();
      }
    } catch (const std::exception& e) {
      *status = 13;
      *msg = std::string("reading block ") + std::to_string(block_) + ": " + e.what();
      return -1;
    }
    if (w > 0) clock_.sent();
    *nspans = ns;
    if (w > 0) stats_->zero_copy_frames.fetch_add(1, std::memory_order_relaxed);
    return (ssize_t)w;
  }

 private:
  // Double-buffered D2H staging: chunk k is copied out of the slot its DMA landed in while the DMA
  // of chunk k+1 runs into the other slot (reference AbstractReadHandler.java:336-439 DataReader
  // runs ahead of the sender the same way, up to the window).
  struct Slot {
    uint8_t* buf = nullptr;
    hipEvent_t ev = nullptr;
    hipEvent_t t0 = nullptr;          // tracing: recorded before the copy (timing events)
    uint64_t pos = 0, len = 0;
    bool inflight = false, valid = false;
    int rec = -1;                     // tracing: index into trace_
  };

  void stage(int k, uint64_t pos, uint64_t n) {
    Slot& s = slot_[k];
    if (!s.buf) {
      s.buf = pool_->get();
      if (hipEventCreateWithFlags(&s.ev, tracing_ ? hipEventDefault : hipEventDisableTiming) != hipSuccess)
        s.ev = nullptr;
      if (tracing_ && hipEventCreate(&s.t0) != hipSuccess) s.t0 = nullptr;
    }
    std::vector<ReadReq> rq{ReadReq{block_, pos, n, reinterpret_cast<uint64_t>(s.buf), (int)MemKind::kHost}};
    hipStream_t st = thread_stream(store_);
    if (tracing_) {
      if (!base_ev_ && hipEventCreate(&base_ev_) == hipSuccess) {
        (void)hipEventRecord(base_ev_, st);
        (void)hipEventSynchronize(base_ev_);
        base_ns_ = now_ns();
      }
      ReadTraceRec r;
      r.pos = pos;
      r.len = n;
      r.issue_ns = now_ns();
      trace_.push_back(r);
      s.rec = (int)trace_.size() - 1;
      if (s.t0) (void)hipEventRecord(s.t0, st);
    }
    store_->read_batch(rq, reinterpret_cast<uint64_t>(st), s.ev == nullptr);
    s.inflight = s.ev != nullptr && hipEventRecord(s.ev, st) == hipSuccess;
    if (s.ev && !s.inflight) (void)hipStreamSynchronize(st);
    s.pos = pos;
    s.len = n;
    s.valid = true;
    stats_->staged_bytes.fetch_add(n, std::memory_order_relaxed);
  }

  void next_chunk() {
    const uint64_t n = std::min(chunk_, end_ - pos_);
    hdr_ = h2::read_response_prefix(n);
    hdr_off_ = 0;
    left_ = n;
    data_pos_ = pos_;
    if (device_) {
      const int k = cur_ ^ 1;                      // the slot chunk k was (pre)staged into
      if (!(slot_[k].valid && slot_[k].pos == pos_ && slot_[k].len == n)) stage(k, pos_, n);
      const int64_t w0 = now_ns();
      if (slot_[k].inflight) {
        // normally long done: it ran during the last send
        if (hipEventSynchronize(slot_[k].ev) != hipSuccess) throw std::runtime_error("D2H staging copy failed");
        slot_[k].inflight = false;
        clock_.add_data_wait(now_ns() - w0);
      }
      if (tracing_ && slot_[k].rec >= 0) {
        ReadTraceRec& r = trace_[slot_[k].rec];
        r.ready_ns = now_ns();
        r.wait_ns = r.ready_ns - w0;
        float ms = 0.f;
        if (base_ev_ && slot_[k].t0 && hipEventElapsedTime(&ms, base_ev_, slot_[k].t0) == hipSuccess)
          r.gpu_start_ns = base_ns_ + (int64_t)(ms * 1e6);
        if (base_ev_ && hipEventElapsedTime(&ms, base_ev_, slot_[k].ev) == hipSuccess)
          r.gpu_end_ns = base_ns_ + (int64_t)(ms * 1e6);
        cur_rec_ = slot_[k].rec;
      }
      cur_ = k;
      stage_off_ = 0;
      const uint64_t nx = pos_ + n;                // prefetch chunk k+1 into the slot just released
      if (nx < end_) {
        stage(cur_ ^ 1, nx, std::min(chunk_, end_ - nx));
        stats_->prefetched.fetch_add(1, std::memory_order_relaxed);
      }
    }
    pos_ += n;
    stats_->chunks.fetch_add(1, std::memory_order_relaxed);
  }

  StoreRef store_;
  int64_t session_, lock_, block_;
  uint64_t pos_, acked_, end_, chunk_, window_;
  bool device_, unix_;
  std::shared_ptr<StagingPool> pool_;
  std::shared_ptr<DataServerStats> stats_;
  std::string hdr_;
  size_t hdr_off_ = 0;
  uint64_t left_ = 0, data_pos_ = 0;
  Slot slot_[2];
  int cur_ = 1;
  uint64_t stage_off_ = 0;
  const bool tracing_ = ReadTraceSink::get().on();
  std::vector<ReadTraceRec> trace_;
  int cur_rec_ = -1;
  hipEvent_t base_ev_ = nullptr;
  int64_t base_ns_ = 0;
  SendClock clock_;
};

std::atomic<int64_t> g_session{(int64_t)1 << 62};   // above the Python range (utils/ids.py)

// ---- cold reads: UFS -> pinned slots -> (temp block) + client ---------------------------------

bool parse_ufs_opts(const std::string& b, UfsOpts* o) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(b.data());
  const size_t n = b.size();
  size_t i = 0;
  while (i < n) {
    uint64_t key;
    if (!h2::get_varint(p, n, &i, &key)) return false;
    const uint32_t field = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
    if (wt == 0) {
      uint64_t v;
      if (!h2::get_varint(p, n, &i, &v)) return false;
      switch (field) {
        case 2: o->offset_in_file = (int64_t)v; break;
        case 3: o->block_size = (int64_t)v; break;
        case 5: o->mount_id = (int64_t)v; break;
        case 6: o->no_cache = v != 0; break;
        case 8: o->block_in_ufs_tier = v != 0; break;
        default: break;
      }
    } else if (wt == 2) {
      uint64_t len;
      if (!h2::get_varint(p, n, &i, &len) || len > n - i) return false;
      if (field == 1) o->ufs_path.assign(b.data() + i, (size_t)len);
      i += (size_t)len;
    } else if (wt == 1 && n - i >= 8) {
      i += 8;
    } else if (wt == 5 && n - i >= 4) {
      i += 4;
    } else {
      return false;
    }
  }
  return true;
}

// A byte range source of one UFS file.
class UfsReader {
 public:
  virtual ~UfsReader() = default;
  // Exactly n bytes at `off` of the file into dst; false with *err set (and status()) otherwise.
  virtual bool read(uint64_t off, uint64_t n, uint8_t* dst, std::string* err) = 0;
  // gRPC status of the last failure: UNAVAILABLE for a UFS that timed out or dropped the
  // connection after its retries, NOT_FOUND, CANCELLED, INTERNAL otherwise.
  int status() const { return status_; }
  // Polled by a read under way (an S3 GET looks at it every ~100 ms): set when the call is gone.
  const std::atomic<bool>* cancel = nullptr;

 protected:
  int status_ = 13;
};

// Helper threads for the parallel sub-range preads of local cold reads (immortal pool).
class PreadPool {
 public:
  static PreadPool& get() {
    static PreadPool* p = new PreadPool(8);
    return *p;
  }
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }

 private:
  explicit PreadPool(int n) {
    for (int i = 0; i < n; ++i)
      std::thread([this] {
        pthread_setname_np(pthread_self(), "ufs-pread");
        for (;;) {
          std::function<void()> f;
          {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return !q_.empty(); });
            f = std::move(q_.front());
            q_.pop_front();
          }
          f();
        }
      }).detach();
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
};

class LocalFileReader : public UfsReader {
 public:
  // A slot of at least 2 * kPart bytes is read as up to kParts sub-ranges at once: one pread copies
  // page-cache pages at ~8 GB/s on one core, below what one cold stream can send.
  static constexpr uint64_t kPart = 2ull << 20;
  static constexpr int kParts = 4;
  explicit LocalFileReader(int fd) : fd_(fd) {}
  ~LocalFileReader() override { ::close(fd_); }
  bool read(uint64_t off, uint64_t n, uint8_t* dst, std::string* err) override {
    const int parts = (int)std::min<uint64_t>(kParts, n / kPart);
    if (parts <= 1) return read_range(off, n, dst, err, &status_);
    const uint64_t each = (n + parts - 1) / parts;
    struct Shared {
      std::mutex mu;
      std::condition_variable cv;
      int left = 0;
      bool ok = true;
      std::string err;
      int status = 13;
    };
    auto sh = std::make_shared<Shared>();
    sh->left = parts - 1;
    for (int i = 1; i < parts; ++i) {
      const uint64_t a = (uint64_t)i * each, k = std::min(each, n - a);
      const int fd = fd_;
      PreadPool::get().submit([sh, fd, off, a, k, dst] {
        std::string e;
        int st = 13;
        const bool ok = read_range_fd(fd, off + a, k, dst + a, &e, &st);
        std::lock_guard<std::mutex> g(sh->mu);
        if (!ok && sh->ok) {
          sh->ok = false;
          sh->err = e;
          sh->status = st;
        }
        if (--sh->left == 0) sh->cv.notify_all();
      });
    }
    std::string e0;
    int st0 = 13;
    const bool ok0 = read_range(off, std::min(each, n), dst, &e0, &st0);
    std::unique_lock<std::mutex> lk(sh->mu);
    sh->cv.wait(lk, [&] { return sh->left == 0; });   // every helper is done with dst
    if (!ok0) {
      *err = e0;
      status_ = st0;
      return false;
    }
    if (!sh->ok) {
      *err = sh->err;
      status_ = sh->status;
      return false;
    }
    return true;
  }

 private:
  bool read_range(uint64_t off, uint64_t n, uint8_t* dst, std::string* err, int* st) {
    return read_range_fd(fd_, off, n, dst, err, st);
  }
  static bool read_range_fd(int fd, uint64_t off, uint64_t n, uint8_t* dst, std::string* err, int* st) {
    uint64_t done = 0;
    while (done < n) {
      const ssize_t r = ::pread(fd, dst + done, (size_t)(n - done), (off_t)(off + done));
      if (r < 0 && errno == EINTR) continue;
      if (r <= 0) {
        *err = r == 0 ? "unexpected end of the UFS file at " + std::to_string(off + done)
                      : std::string("pread: ") + std::strerror(errno);
        *st = r == 0 ? 11 : 13;          // OUT_OF_RANGE / INTERNAL
        return false;
      }
      done += (uint64_t)r;
    }
    return true;
  }
  int fd_;
};

class S3ObjectReader : public UfsReader {
 public:
  S3ObjectReader(std::shared_ptr<const S3Mount> m, std::string key) : m_(std::move(m)), key_(std::move(key)) {}
  bool read(uint64_t off, uint64_t n, uint8_t* dst, std::string* err) override {
    static const std::string kEmptySha = "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855";
    const std::string path = "/" + m_->bucket + "/" + key_;
    const std::string head = s3_header_lines(m_->cred, "GET", path, "", kEmptySha);
    const int64_t got = m_->reader->get_into(uri_encode_path(path), head, off, n, reinterpret_cast<uint64_t>(dst),
                                             m_->parallel, m_->part, cancel);
    if (got == (int64_t)n) return true;
    std::string why;
    if (got == -404) {
      why = "not found";
      status_ = 5;
    } else if (got == kHttpTimeout) {
      why = "timed out (socket " + std::to_string(m_->http.socket_timeout_ms) + " ms, request " +
            std::to_string(m_->http.request_timeout_ms) + " ms)";
      status_ = 14;
    } else if (got == kHttpCancelled) {
      why = "cancelled";
      status_ = 1;
    } else if (got == kHttpTransportError) {
      why = "connection failed after " + std::to_string(m_->http.max_retries) + " retries";
      status_ = 14;
    } else {
      why = "HTTP " + std::to_string(-got);
      status_ = HttpRangeReader::retryable(got) ? 14 : 13;
    }
    *err = "S3 GET " + path + " [" + std::to_string(off) + ", +" + std::to_string(n) + ") " + why;
    return false;
  }

 private:
  std::shared_ptr<const S3Mount> m_;
  std::string key_;
};

// A UFS the I/O threads cannot reach (HDFS, HTTPS S3, ...), read through the worker's Python UFS
// by internal ReadUfsRange calls from the reader's pool thread: only the first cold read of such a
// mount takes it (later ones go to the Python servicer directly, UfsMounts::is_python).
class PythonRangeReader : public UfsReader {
 public:
  PythonRangeReader(BlockCommitter::Caller caller, uint32_t method, int64_t mount_id, std::string path)
      : caller_(std::move(caller)), method_(method), mount_(mount_id), path_(std::move(path)) {}
  bool read(uint64_t off, uint64_t n, uint8_t* dst, std::string* err) override {
    uint64_t done = 0;
    while (done < n) {
      if (cancel && cancel->load(std::memory_order_relaxed)) {
        status_ = 1;
        *err = "cancelled";
        return false;
      }
      const uint64_t k = std::min<uint64_t>(n - done, 8u << 20);
      // ReadUfsRangeRequest: mount_id=1 ufs_path=2 offset=3 length=4
      std::string m;
      h2::put_varint(m, (1u << 3));
      h2::put_varint(m, (uint64_t)mount_);
      h2::put_varint(m, (2u << 3) | 2);
      h2::put_varint(m, path_.size());
      m += path_;
      h2::put_varint(m, (3u << 3));
      h2::put_varint(m, off + done);
      h2::put_varint(m, (4u << 3));
      h2::put_varint(m, k);
      struct Reply {
        std::mutex mu;
        std::condition_variable cv;
        bool got = false;
        int status = 0;
        std::string msg, payload;
      };
      auto rep = std::make_shared<Reply>();
      caller_(method_, std::move(m), [rep](int s, const std::string& msg, const std::string& payload) {
        std::lock_guard<std::mutex> g(rep->mu);
        rep->got = true;
        rep->status = s;
        rep->msg = msg;
        rep->payload = payload;
        rep->cv.notify_all();
      });
      std::unique_lock<std::mutex> lk(rep->mu);
      if (!rep->cv.wait_for(lk, std::chrono::minutes(5), [&] { return rep->got; })) {
        status_ = 14;
        *err = "reading the UFS through the worker timed out";
        return false;
      }
      if (rep->status) {
        status_ = rep->status;
        *err = rep->msg;
        return false;
      }
      // ReadUfsRangeResponse: data=1 (bytes)
      const uint8_t* p = reinterpret_cast<const uint8_t*>(rep->payload.data());
      const size_t pn = rep->payload.size();
      size_t i = 0;
      uint64_t got = 0;
      while (i < pn) {
        uint64_t key, len;
        if (!h2::get_varint(p, pn, &i, &key)) break;
        if ((key >> 3) == 1 && (key & 7) == 2 && h2::get_varint(p, pn, &i, &len) && len <= pn - i) {
          got = std::min<uint64_t>(len, k);
          std::memcpy(dst + done, p + i, (size_t)got);
          i += (size_t)len;
        } else {
          break;
        }
      }
      if (got != k) {
        status_ = 11;
        *err = "unexpected end of the UFS file at " + std::to_string(off + done + got);
        return false;
      }
      done += k;
    }
    return true;
  }

 private:
  BlockCommitter::Caller caller_;
  uint32_t method_;
  int64_t mount_;
  std::string path_;
};

// The UFS reads of a cold stream: the first covers `first` bytes (one chunk, so the first bytes
// go out after one small read instead of a whole slot), every later one a slot.  Read i lands
// in slot i % depth; this is the read holding stream-relative offset `rel`.
inline size_t cold_read_index(uint64_t rel, uint64_t first, uint64_t slot) {
  return rel < first ? 0 : 1 + (size_t)((rel - first) / slot);
}

// Completed HIP events of finished cold streams, per device, for the next streams' slots:
// hipEventCreate contends with the copies of concurrent streams (0.4 ms per stream with four).
class EventPool {
 public:
  static EventPool& get() {
    static EventPool* p = new EventPool();   // immortal: its events live as long as the process
    return *p;
  }
  // An event of the current device (`device`), or null.
  hipEvent_t take(int device) {
    {
      std::lock_guard<std::mutex> g(mu_);
      auto& v = free_[device];
      if (!v.empty()) {
        hipEvent_t e = v.back();
        v.pop_back();
        return e;
      }
    }
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
    return e;
  }
  // A completed event back (destroyed beyond 256 kept per device).
  void put(int device, hipEvent_t e) {
    {
      std::lock_guard<std::mutex> g(mu_);
      auto& v = free_[device];
      if (v.size() < 256) {
        v.push_back(e);
        return;
      }
    }
    (void)hipEventDestroy(e);
  }

 private:
  std::mutex mu_;
  std::map<int, std::vector<hipEvent_t>> free_;
};

// State shared by a cold stream (I/O threads) and its background reader thread.
struct ColdState {
  struct Slot {
    uint8_t* buf = nullptr;
    hipEvent_t ev = nullptr;
    uint64_t off = 0, len = 0;    // block offsets of the bytes it holds
    bool ready = false;           // filled (and its H2D queued): the stream may send it
    bool dma = false;             // an H2D out of it may still run
  };
  std::mutex mu;
  std::condition_variable cv;
  std::vector<Slot> slots;
  bool cancelled = false, read_done = false, failed = false, job_exited = false, caching = false;
  bool handed_off = false;      // the cached block went to the commit: its session is not ours
  std::atomic<bool> cancel_flag{false};   // `cancelled`, for a UFS read under way to poll
  int err_status = 13;          // gRPC status of the failure (UNAVAILABLE: the UFS timed out / dropped)
  std::string err;
  std::function<void()> wake;
  std::shared_ptr<StagingPool> pool;
  int device = -1;              // of the slots' events (the reader synchronized them before exiting)
  ~ColdState() {
    for (auto& sl : slots) {
      if (sl.ev) EventPool::get().put(device, sl.ev);
      if (sl.buf) pool->put(sl.buf);
    }
  }
};

// Next-block read-ahead of the native cold path.  A whole-block read-through that reached the end
// of its block reads the first two UFS reads of the file's next block (one chunk, then a slot) into
// pinned buffers of its slot pool once its own reads are done; the next block's cold stream adopts
// them as its first two slots, so its first bytes go out without waiting on the UFS.  One client
// stream reads one block at a time, so without it every block of a sequential cold read pays the
// UFS latency before its first byte (profiles/r6_cold_read.md).  Pieces are matched by (block id,
// mount, path, file offset, length) -- a file rewritten under the same path has new block ids, so
// its reads never see the old bytes -- expire after kTtl and are bounded to kMaxPieces per server.
class ColdReadAhead {
 public:
  static constexpr size_t kMaxPieces = 32;
  static constexpr std::chrono::milliseconds kTtl{5000};
  ~ColdReadAhead() {
    for (auto& p : pieces_) p.pool->put(p.buf);
  }
  void put(int64_t block, const std::string& key, std::shared_ptr<StagingPool> pool, uint64_t off, uint64_t len,
           uint8_t* buf) {
    std::vector<Piece> drop;
    {
      std::lock_guard<std::mutex> g(mu_);
      expire_locked(&drop);
      if (pieces_.size() >= kMaxPieces) {
        drop.push_back(pieces_.front());
        pieces_.pop_front();
      }
      pieces_.push_back({block, key, std::move(pool), off, len, buf, std::chrono::steady_clock::now()});
    }
    for (auto& p : drop) p.pool->put(p.buf);
  }
  // The buffer holding exactly [off, off + len) of block `block` of `key` from `pool`, now the
  // caller's, or null.
  uint8_t* take(int64_t block, const std::string& key, const StagingPool* pool, uint64_t off, uint64_t len) {
    std::vector<Piece> drop;
    uint8_t* got = nullptr;
    {
      std::lock_guard<std::mutex> g(mu_);
      expire_locked(&drop);
      for (auto it = pieces_.begin(); it != pieces_.end(); ++it)
        if (it->block == block && it->off == off && it->len == len && it->pool.get() == pool && it->key == key) {
          got = it->buf;
          pieces_.erase(it);
          break;
        }
    }
    for (auto& p : drop) p.pool->put(p.buf);
    return got;
  }
  // Blocks with a cold stream under way: a stream never reads ahead a block another stream reads
  // (a client reading several blocks at once opens the next one before the current one ends).
  void begin(int64_t block) {
    std::lock_guard<std::mutex> g(mu_);
    ++active_[block];
  }
  void end(int64_t block) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = active_.find(block);
    if (it != active_.end() && --it->second <= 0) active_.erase(it);
  }
  bool active(int64_t block) {
    std::lock_guard<std::mutex> g(mu_);
    return active_.count(block) != 0;
  }

 private:
  struct Piece {
    int64_t block;
    std::string key;
    std::shared_ptr<StagingPool> pool;
    uint64_t off, len;
    uint8_t* buf;
    std::chrono::steady_clock::time_point at;
  };
  void expire_locked(std::vector<Piece>* drop) {
    const auto now = std::chrono::steady_clock::now();
    while (!pieces_.empty() && now - pieces_.front().at > kTtl) {
      drop->push_back(pieces_.front());
      pieces_.pop_front();
    }
  }
  std::mutex mu_;
  std::deque<Piece> pieces_;
  std::unordered_map<int64_t, int> active_;
};

struct ColdJob {
  StoreRef store;
  int64_t session, block;
  uint64_t start, end, block_len, file_off, slot_bytes;
  uint64_t first_bytes = 0;     // the first read (<= slot_bytes; 0 = a whole slot)
  size_t create_after = 2;      // reads before the temp block is created (capped at the slot count)
  bool want_cache;
  std::unique_ptr<UfsReader> reader;
  std::shared_ptr<ColdState> st;
  std::shared_ptr<DataServerStats> stats;
  std::function<void(uint32_t, std::string)> post;   // internal requests to Python (the commit)
  uint32_t commit_method = UINT32_MAX;
  std::shared_ptr<BlockCommitter> committer;         // native commit (instead of `post`) when set
  // A mount the data server did not know at the call's start: resolves it (blocking internal call
  // to the worker) and opens the reader; false with *status / *err when it cannot be read natively.
  std::function<bool(std::unique_ptr<UfsReader>*, int*, std::string*)> resolve;
  std::chrono::steady_clock::time_point queued_at = std::chrono::steady_clock::now();
  std::shared_ptr<ColdReadAhead> readahead;   // null: no next-block read-ahead (its stream registry too)
  std::string ra_key;                         // "<mount id>:<ufs path>"
  bool ra_next = false;                       // a whole-block read-through: read the next block ahead

  void wake() {
    std::function<void()> w;
    {
      std::lock_guard<std::mutex> g(st->mu);
      w = st->wake;
    }
    if (w) w();
  }

  // Runs on its own thread: UFS reads (and the H2D copies into the temp block) run ahead of the
  // sends by up to `depth` slots; a slot is reused once the stream has sent it and its H2D is done.
  void run() {
    using clk = std::chrono::steady_clock;
    auto ns_since = [](clk::time_point t) {
      return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t).count();
    };
    const auto t_run = clk::now();
    stats->cold_queue_ns.fetch_add(
        (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t_run - queued_at).count(),
        std::memory_order_relaxed);
    bool caching = false;
    hipStream_t hs = nullptr;
    std::string err;
    bool ok = true;
    uint64_t ingested = start;
    int err_status = 13;
    uint64_t read_ns = 0, slot_wait_ns = 0, dma_wait_ns = 0;
    if (!reader && resolve && !resolve(&reader, &err_status, &err)) reader.reset();
    if (!reader) {                    // unresolvable mount: fail the stream, drop the session
      if (err.empty()) err = "the UFS of this block cannot be read natively";
      {
        std::lock_guard<std::mutex> g(st->mu);
        st->failed = true;
        st->err = err;
        st->err_status = err_status;
        st->read_done = true;
        st->job_exited = true;
      }
      try {
        store->cleanup_session(session);
      } catch (...) {
      }
      if (readahead) readahead->end(block);
      stats->cold_active.fetch_sub(1, std::memory_order_relaxed);
      wake();
      return;
    }
    reader->cancel = &st->cancel_flag;
    try {
      if (store->has_device()) {
        store->use_device();
        hs = thread_stream_on(store->device());   // the pool thread's stream (never one per read)
        st->device = store->device();
      }
      // The temp block is created once the first `create_after` reads are on their way to the
      // client (default two: one chunk, then a slot): the create -- page allocation, maybe
      // eviction; ~3 ms with four cold streams at once -- runs while they go out instead of
      // before them; their bytes go into the block after it.
      bool create_pending = want_cache;
      const size_t create_at = std::max<size_t>(1, std::min(create_after, st->slots.size()));
      struct Unstored {
        ColdState::Slot* sl;
        uint64_t off, n;
      };
      std::vector<Unstored> unstored;
      stats->cold_device_ns.fetch_add(ns_since(t_run), std::memory_order_relaxed);
      stats->cold_setup_ns.fetch_add(ns_since(t_run), std::memory_order_relaxed);
      const size_t depth = st->slots.size();
      const uint64_t first = first_bytes ? std::min(first_bytes, slot_bytes) : slot_bytes;
      size_t idx = 0;
      for (uint64_t off = start, n = 0; off < end; off += n, ++idx) {
        n = std::min(idx == 0 ? first : slot_bytes, end - off);
        ColdState::Slot* sl;
        {
          const auto tw = clk::now();
          std::unique_lock<std::mutex> lk(st->mu);
          sl = &st->slots[idx % depth];
          st->cv.wait(lk, [&] { return st->cancelled || !sl->ready; });
          slot_wait_ns += ns_since(tw);
          if (st->cancelled) break;
        }
        if (sl->dma) {   // the H2D of the bytes this slot held `depth` reads ago
          const auto td = clk::now();
          if (hipEventSynchronize(sl->ev) != hipSuccess) throw std::runtime_error("H2D into the block failed");
          dma_wait_ns += ns_since(td);
          sl->dma = false;
        }
        // the previous block's stream may have read this one's first two reads ahead
        const auto ta = clk::now();
        uint8_t* pre = readahead && idx < 2 ? readahead->take(block, ra_key, st->pool.get(), file_off + off, n) : nullptr;
        if (!sl->buf) {
          sl->buf = pre ? pre : st->pool->get();
          if (hs) sl->ev = EventPool::get().take(st->device);
        }
        stats->cold_slot_alloc_ns.fetch_add(ns_since(ta), std::memory_order_relaxed);
        const auto tr = clk::now();
        if (pre) {
          if (sl->buf != pre) {
            std::memcpy(sl->buf, pre, n);
            st->pool->put(pre);
          }
          stats->cold_readahead_hits.fetch_add(1, std::memory_order_relaxed);
        } else if (!reader->read(file_off + off, n, sl->buf, &err)) {
          ok = false;
          err_status = reader->status();
          break;
        }
        read_ns += ns_since(tr);
        if (idx == 0) stats->cold_first_read_ns.fetch_add(ns_since(tr), std::memory_order_relaxed);
        stats->cold_bytes.fetch_add(n, std::memory_order_relaxed);
        // a slot's bytes into the temp block (async H2D on this thread's stream; the slot is
        // refilled only after its event, `depth` reads from now)
        auto ingest = [&](ColdState::Slot* s, uint64_t o, uint64_t k) {
          const bool async = hs && s->ev;
          store->write(session, block, o, reinterpret_cast<uint64_t>(s->buf), k, (int)MemKind::kHost,
                       reinterpret_cast<uint64_t>(hs), !async);
          if (async) {
            if (hipEventRecord(s->ev, hs) != hipSuccess) throw std::runtime_error("hipEventRecord failed");
            s->dma = true;
          }
        };
        if (caching) ingest(sl, off, n);
        else if (create_pending) unstored.push_back({sl, off, n});
        {
          std::lock_guard<std::mutex> g(st->mu);
          sl->off = off;
          sl->len = n;
          sl->ready = true;
        }
        if (idx == 0) stats->cold_first_ns.fetch_add(ns_since(t_run), std::memory_order_relaxed);
        ingested = off + n;
        wake();
        // after `create_at` reads (or the last one), before any slot comes round again: the
        // sender only reads the slots, the reader refills them later
        if (create_pending && (idx + 1 >= create_at || off + n >= end || unstored.size() >= depth)) {
          create_pending = false;
          const auto tc = clk::now();
          try {   // may evict (the I/O thread never waits for space: this thread does)
            store->create_block(session, block, 0, "", std::max<uint64_t>(block_len, 1), true, false);
            caching = true;
          } catch (const StoreError&) {
            caching = false;      // another reader caches it, or no space: stream without caching
          }
          {
            std::lock_guard<std::mutex> g(st->mu);
            st->caching = caching;
          }
          if (caching)
            for (const auto& u : unstored) ingest(u.sl, u.off, u.n);
          unstored.clear();
          stats->cold_setup_ns.fetch_add(ns_since(tc), std::memory_order_relaxed);
        }
      }
    } catch (const std::exception& e) {
      ok = false;
      err = e.what();
    }
    stats->cold_read_ns.fetch_add(read_ns, std::memory_order_relaxed);
    stats->cold_slot_wait_ns.fetch_add(slot_wait_ns, std::memory_order_relaxed);
    stats->cold_dma_wait_ns.fetch_add(dma_wait_ns, std::memory_order_relaxed);
    if (hs) {
      if (hipStreamSynchronize(hs) != hipSuccess && ok) {   // every H2D is done before commit / abort
        ok = false;
        err = "H2D into the block failed";
      }
    }
    // UnderFileSystemBlockReader.close: a block read through to its end is committed -- also when
    // the client went away after the last byte -- anything less is aborted
    const bool complete = ok && ingested >= end;
    const bool commit = caching && complete && ((post && commit_method != UINT32_MAX) || committer);
    bool cancelled;
    {
      std::lock_guard<std::mutex> g(st->mu);
      for (auto& sl : st->slots) sl.dma = false;
      if (!ok) {
        st->failed = true;
        st->err = err;
        st->err_status = err_status;
      }
      st->read_done = true;
      st->job_exited = true;
      st->handed_off = commit;
      cancelled = st->cancelled;
    }
    if (commit && committer) {
      // the native committer commits it and reports it with the next batch (no client waits)
      auto t = std::make_shared<CommitTicket>();
      t->session = session;
      t->block = block;
      t->length = block_len;
      t->ufs_read = true;
      t->crc_sync = store->has_device() ? committer->crc_device() : committer->crc_host();
      committer->submit(t);
      stats->cold_cached.fetch_add(1, std::memory_order_relaxed);
    } else if (commit) {
      // NativeWriteCommitRequest: session_id=1 block_id=2 length=3 pin=4 ufs_read=5; Python
      // commits (CRC, master report) and drops the session, whether or not the call still exists
      std::string m;
      h2::put_varint(m, (1u << 3));
      h2::put_varint(m, (uint64_t)session);
      h2::put_varint(m, (2u << 3));
      h2::put_varint(m, (uint64_t)block);
      h2::put_varint(m, (3u << 3));
      h2::put_varint(m, block_len);
      h2::put_varint(m, (5u << 3));
      h2::put_varint(m, 1);
      post(commit_method, std::move(m));
      stats->cold_cached.fetch_add(1, std::memory_order_relaxed);
    } else if (caching || cancelled || !ok) {
      if (caching) stats->cold_aborted.fetch_add(1, std::memory_order_relaxed);
      try {
        store->cleanup_session(session);   // drops the temp block of an incomplete read-through
      } catch (...) {
      }
    }
    if (!cancelled) wake();   // the stream may end now: the read-ahead below is off its path
    if (readahead) {
      readahead->end(block);
      // a client that went away after the last byte still read the block sequentially to its end
      if (ra_next && complete) read_ahead_next();
    }
    stats->cold_active.fetch_sub(1, std::memory_order_relaxed);
  }

  // The next block's first two reads (see ColdReadAhead), unless the store has that block.  A
  // read past the end of the file (this was its last block) fails and leaves nothing.
  void read_ahead_next() {
    const int64_t next = block + 1;   // BlockId: container << 24 | sequence, the file's next block
    try {
      if (readahead->active(next) || store->has_block(next) || store->has_temp_block(next)) return;
    } catch (...) {
      return;
    }
    const uint64_t base = file_off + block_len;
    const uint64_t first = first_bytes ? std::min(first_bytes, slot_bytes) : slot_bytes;
    const uint64_t sizes[2] = {first, slot_bytes};
    uint64_t off = base;
    // not the stream's cancel flag (the stream ends, and sets it, while these reads run): the data
    // server's, set when the worker stops (a GET under way stops within ~100 ms)
    reader->cancel = &stats->stopping;
    for (int i = 0; i < 2; ++i) {
      uint8_t* buf = st->pool->get();
      std::string err;
      if (!reader->read(off, sizes[i], buf, &err)) {
        st->pool->put(buf);
        reader->cancel = nullptr;
        return;
      }
      stats->cold_readahead_bytes.fetch_add(sizes[i], std::memory_order_relaxed);
      readahead->put(next, ra_key, st->pool, off, sizes[i], buf);
      off += sizes[i];
    }
    reader->cancel = nullptr;
  }
};

// Threads of the native cold reads, shared by every data server of the process: a thread is
// spawned only while every one is busy, up to the largest ufs.read.max.active any server asked for
// (make_cold_stream admits at most that many reads per server); idle threads wait for the next
// read, so a read costs no thread creation and no HIP stream (each thread keeps its own).
class ColdPool {
 public:
  static ColdPool& get() {
    static ColdPool* p = new ColdPool();   // immortal, like its threads
    return *p;
  }
  bool submit(std::function<void()> f, int max_threads) {
    std::lock_guard<std::mutex> g(mu_);
    q_.push_back(std::move(f));
    if (q_.size() > idle_ && threads_ < std::max(1, max_threads)) {
      try {
        std::thread([this] { loop(); }).detach();
        ++threads_;
      } catch (...) {
        if (threads_ == 0) {
          q_.pop_back();
          return false;
        }
      }
    }
    cv_.notify_one();
    return true;
  }
  int threads() {
    std::lock_guard<std::mutex> g(mu_);
    return threads_;
  }

 private:
  void loop() {
    pthread_setname_np(pthread_self(), "ufs-cold-read");
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        ++idle_;
        cv_.wait(lk, [&] { return !q_.empty(); });
        --idle_;
        f = std::move(q_.front());
        q_.pop_front();
      }
      try {
        f();
      } catch (...) {
      }
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  size_t idle_ = 0;
  int threads_ = 0;
};

class ColdReadStream : public NativeStream {
 public:
  ColdReadStream(StoreRef store, int64_t session, int64_t block_id, uint64_t pos, uint64_t end, uint64_t chunk,
                 uint64_t window, uint64_t slot_bytes, uint64_t first_bytes, bool unix_peer,
                 std::shared_ptr<ColdState> st, std::shared_ptr<DataServerStats> stats)
      : store_(store), session_(session), block_(block_id), start_(pos), pos_(pos), acked_(pos), end_(end),
        chunk_(chunk), window_(window), slot_bytes_(slot_bytes),
        first_(first_bytes ? std::min(first_bytes, slot_bytes) : slot_bytes), unix_(unix_peer), st_(std::move(st)),
        stats_(std::move(stats)), clock_(&stats_->send[1]) {}

  ~ColdReadStream() override {
    bool exited, handed_off;
    {
      std::lock_guard<std::mutex> g(st_->mu);
      st_->cancelled = true;
      st_->cancel_flag.store(true, std::memory_order_relaxed);   // a GET under way stops within ~100 ms
      st_->wake = nullptr;
      exited = st_->job_exited;
      handed_off = st_->handed_off;
    }
    st_->cv.notify_all();
    // a running reader cleans up itself once it sees the cancel; a block handed to the commit is
    // Python's; otherwise the (exited) reader's session goes here
    if (exited && !handed_off) {
      try {
        store_->cleanup_session(session_);
      } catch (...) {
      }
    }
  }

  void set_waker(std::function<void()> w) override {
    std::lock_guard<std::mutex> g(st_->mu);
    st_->wake = std::move(w);
  }

  void on_message(const char* p, size_t n) override {
    ReadRequestMsg r;
    if (parse_read_request(p, n, &r) && r.has_ack && (uint64_t)r.offset_received > acked_)
      acked_ = std::min<uint64_t>((uint64_t)r.offset_received, pos_);
  }

  ssize_t produce(uint8_t* dst, size_t max, bool* eof, int* status, std::string* msg) override {
    size_t w = 0;
    while (w < max) {
      if (hdr_off_ < hdr_.size()) {
        const size_t n = std::min(max - w, hdr_.size() - hdr_off_);
        std::memcpy(dst + w, hdr_.data() + hdr_off_, n);
        hdr_off_ += n;
        w += n;
        continue;
      }
      if (left_ > 0) {
        const size_t n = (size_t)std::min<uint64_t>(max - w, left_);
        std::memcpy(dst + w, src_, n);
        src_ += n;
        left_ -= n;
        w += n;
        stats_->bytes.fetch_add(n, std::memory_order_relaxed);
        if (unix_) stats_->domain_bytes.fetch_add(n, std::memory_order_relaxed);
        if (left_ == 0 && pos_ >= slot_end_) release_slot();
        continue;
      }
      if (pos_ >= end_) {            // every byte sent (the reader commits the cache by itself)
        *eof = true;
        break;
      }
      if (pos_ - acked_ >= window_) break;       // wait for offset_received
      // the slot holding pos_
      const size_t depth = st_->slots.size();
      const size_t idx = cold_read_index(pos_ - start_, first_, slot_bytes_);
      ColdState::Slot* sl = &st_->slots[idx % depth];
      bool ready, failed;
      int fail_status;
      std::string err;
      {
        std::lock_guard<std::mutex> g(st_->mu);
        ready = sl->ready && sl->off <= pos_ && pos_ < sl->off + sl->len;
        failed = st_->failed;
        fail_status = st_->err_status;
        err = st_->err;
      }
      if (!ready) {
        if (failed) {
          *status = fail_status;
          *msg = "UFS read of block " + std::to_string(block_) + ": " + err;
          return w ? (ssize_t)w : -1;
        }
        break;                                   // the reader wakes this call when it lands
      }
      const uint64_t n = std::min(chunk_, std::min(sl->off + sl->len, end_) - pos_);
      hdr_ = h2::read_response_prefix(n);
      hdr_off_ = 0;
      left_ = n;
      src_ = sl->buf + (pos_ - sl->off);
      slot_end_ = sl->off + sl->len;
      cur_slot_ = sl;
      pos_ += n;
      stats_->chunks.fetch_add(1, std::memory_order_relaxed);
    }
    return (ssize_t)w;
  }

  // Zero-copy sends (as the cached path's BlockReadStream): the chunk's prefix and its bytes in the
  // pinned UFS slot go to the socket as they are.  A DATA frame never crosses a chunk boundary, and
  // a slot whose last byte went out is handed back to the reader only at the next call, once the
  // server has written the spans.
  ssize_t produce_spans(size_t max, ByteSpan* spans, int max_spans, int* nspans, bool* eof, int* status,
                        std::string* msg) override {
    if (max_spans < 2) return -2;
    clock_.resume();
    if (release_pending_) {
      release_pending_ = false;
      release_slot();
    }
    size_t w = 0;
    int ns = 0;
    while (w < max && ns < max_spans) {
      if (hdr_off_ < hdr_.size()) {
        const size_t n = std::min(max - w, hdr_.size() - hdr_off_);
        spans[ns++] = ByteSpan{reinterpret_cast<const uint8_t*>(hdr_.data()) + hdr_off_, n};
        hdr_off_ += n;
        w += n;
        continue;
      }
      if (left_ > 0) {
        const size_t n = (size_t)std::min<uint64_t>(max - w, left_);
        spans[ns++] = ByteSpan{src_, n};
        src_ += n;
        left_ -= n;
        w += n;
        stats_->bytes.fetch_add(n, std::memory_order_relaxed);
        if (unix_) stats_->domain_bytes.fetch_add(n, std::memory_order_relaxed);
        if (left_ == 0 && pos_ >= slot_end_) release_pending_ = true;
        continue;
      }
      if (w > 0) break;                          // this frame ends with the chunk
      if (pos_ >= end_) {
        *eof = true;
        clock_.done();
        break;
      }
      if (pos_ - acked_ >= window_) {
        clock_.stall(1);
        break;
      }
      const int r = select_chunk(status, msg);
      if (r < 0) return -1;
      if (r == 0) {
        clock_.stall(2);
        break;
      }
    }
    if (w > 0) clock_.sent();
    *nspans = ns;
    if (w > 0) stats_->zero_copy_frames.fetch_add(1, std::memory_order_relaxed);
    return (ssize_t)w;
  }

 private:
  // Makes the next chunk at pos_ current: 1 = done, 0 = its slot has not landed yet, -1 = the UFS
  // read failed (*status / *msg set).
  int select_chunk(int* status, std::string* msg) {
    const size_t depth = st_->slots.size();
    const size_t idx = cold_read_index(pos_ - start_, first_, slot_bytes_);
    ColdState::Slot* sl = &st_->slots[idx % depth];
    bool ready, failed;
    int fail_status;
    std::string err;
    {
      std::lock_guard<std::mutex> g(st_->mu);
      ready = sl->ready && sl->off <= pos_ && pos_ < sl->off + sl->len;
      failed = st_->failed;
      fail_status = st_->err_status;
      err = st_->err;
    }
    if (!ready) {
      if (failed) {
        *status = fail_status;
        *msg = "UFS read of block " + std::to_string(block_) + ": " + err;
        return -1;
      }
      return 0;
    }
    const uint64_t n = std::min(chunk_, std::min(sl->off + sl->len, end_) - pos_);
    hdr_ = h2::read_response_prefix(n);
    hdr_off_ = 0;
    left_ = n;
    src_ = sl->buf + (pos_ - sl->off);
    slot_end_ = sl->off + sl->len;
    cur_slot_ = sl;
    pos_ += n;
    stats_->chunks.fetch_add(1, std::memory_order_relaxed);
    return 1;
  }

  void release_slot() {
    {
      std::lock_guard<std::mutex> g(st_->mu);
      if (cur_slot_) cur_slot_->ready = false;
    }
    cur_slot_ = nullptr;
    st_->cv.notify_all();
  }
  bool release_pending_ = false;

  StoreRef store_;
  int64_t session_, block_;
  uint64_t start_, pos_, acked_, end_, chunk_, window_, slot_bytes_, first_;
  bool unix_;
  std::shared_ptr<ColdState> st_;
  std::shared_ptr<DataServerStats> stats_;
  std::string hdr_;
  size_t hdr_off_ = 0;
  uint64_t left_ = 0, slot_end_ = 0;
  const uint8_t* src_ = nullptr;
  ColdState::Slot* cur_slot_ = nullptr;
  SendClock clock_;
};

// ---- WriteBlock ---------------------------------------------------------------------------------
// WriteRequestCommand (proto/defs/block.py): type=1 id=2 offset=3 tier=4 flush=5
// create_ufs_file_options=6 create_ufs_block_options=7 medium_type=8 pin_on_create=9
// space_to_reserve=10.  WriteRequest: command=1 chunk=2 (Chunk: data=1).
// CreateUfsFileOptions (proto/defs/common.py): ufs_path=1 owner=2 group=3 mode=4 mount_id=5 acl=6.
struct WriteCmd {
  int64_t type = 0, id = 0, offset = 0, tier = 0, reserve = 0;
  bool has_tier = false, flush = false, pin = false, has_ufs = false, has_ufs_file = false;
  bool hold = false;                  // hold_for_append=20: keep the block locked for an AppendBlock
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
        case 20: c->hold = v != 0; break;
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
                         size_t* chunk_len, int64_t* append_id = nullptr, uint64_t* append_len = nullptr) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(data);
  size_t i = 0;
  *has_cmd = false;
  *chunk = nullptr;
  *chunk_len = 0;
  if (append_id) *append_id = -1;
  while (i < n) {
    uint64_t key;
    if (!h2::get_varint(p, n, &i, &key)) return false;
    const uint32_t field = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
    if (wt == 2 && field == 20 && append_id) {       // AppendBlock{block_id=1, length=2}
      uint64_t len;
      if (!h2::get_varint(p, n, &i, &len) || len > n - i) return false;
      size_t j = i;
      const size_t end = i + (size_t)len;
      uint64_t id = 0, ln = 0;
      while (j < end) {
        uint64_t k2, v;
        if (!h2::get_varint(p, end, &j, &k2)) return false;
        if ((k2 & 7) != 0) {
          if (!skip_field(p, end, &j, (uint32_t)(k2 & 7))) return false;
          continue;
        }
        if (!h2::get_varint(p, end, &j, &v)) return false;
        if ((k2 >> 3) == 1) id = v;
        else if ((k2 >> 3) == 2) ln = v;
      }
      *append_id = (int64_t)id;
      *append_len = ln;
      i = end;
      continue;
    }
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

// A block whose creation needs eviction: created on a pool thread (the I/O thread never waits for
// space) while the stream queues what arrives, its receive window held back past kMaxBacklog.
struct PendingCreate {
  std::mutex mu;
  bool done = false, cancelled = false;
  int status = 0;
  std::string msg;
  int dir = -1;
  std::function<void()> wake;
};

class BlockWriteStream : public WriteStreamBase {
 public:
  static constexpr uint64_t kMaxBacklog = 8ull << 20;

  BlockWriteStream(StoreRef store, int64_t session, int64_t block_id, uint64_t pos, bool pin, bool device,
                   uint32_t commit_method, std::shared_ptr<StagingPool> pool, std::shared_ptr<DataServerStats> stats,
                   std::shared_ptr<BlockCommitter> committer = nullptr, std::shared_ptr<PendingCreate> pending = nullptr)
      : store_(std::move(store)), session_(session), block_(block_id), start_(pos), pos_(pos), pin_(pin),
        device_(device), commit_(commit_method), pool_(std::move(pool)), stats_(std::move(stats)),
        committer_(std::move(committer)), pc_(std::move(pending)) {}

  ~BlockWriteStream() override {
    drain();                                 // no DMA may still target the block's pages
    for (auto& sl : slot_) {
      if (sl.ev) (void)hipEventDestroy(sl.ev);
      if (sl.buf) pool_->put(sl.buf);
    }
    if (pc_) {
      std::lock_guard<std::mutex> g(pc_->mu);
      pc_->wake = nullptr;
      if (!pc_->done) {                      // the create task drops the block it makes
        pc_->cancelled = true;
        return;
      }
    }
    if (ticket_) {                           // the committer owns the session now
      std::lock_guard<std::mutex> g(ticket_->mu);
      ticket_->wake = nullptr;
      return;
    }
    try {
      store_->cleanup_session(session_);     // aborts the temp block unless Python committed it
    } catch (...) {
    }
  }

  void set_waker(std::function<void()> w) override {
    waker_ = w;
    if (pc_) {
      bool done;
      {
        std::lock_guard<std::mutex> g(pc_->mu);
        pc_->wake = w;
        done = pc_->done;
      }
      if (done && w) w();
    }
  }

  bool accepting() override { return !pc_ || backlog_bytes_ < kMaxBacklog; }

  bool take_post(uint32_t* method, std::string* payload) override {
    if (!post_ready_) return false;
    post_ready_ = false;
    *method = post_method_;
    *payload = std::move(post_payload_);
    return true;
  }

  ssize_t produce(uint8_t* dst, size_t max, bool* eof, int* status, std::string* msg) override {
    if (pc_) settle_create();
    if (ticket_ && !done_ && !err_) {        // the native commit: answer once it is through
      bool fin;
      int st;
      std::string m;
      {
        std::lock_guard<std::mutex> g(ticket_->mu);
        fin = ticket_->finished;
        st = ticket_->status;
        m = ticket_->msg;
      }
      if (fin) {
        if (st) fail(st, m);
        else {
          out_ += write_response_frame(pos_);
          done_ = true;
        }
      }
    }
    return WriteStreamBase::produce(dst, max, eof, status, msg);
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
    if (pc_) {                               // the block is still being created: queue in order
      Queued q;
      q.data.assign(reinterpret_cast<const char*>(chunk), len);
      q.flush = has_cmd && cmd.flush;
      backlog_bytes_ += len;
      backlog_.push_back(std::move(q));
      if (has_cmd && cmd.hold) hold_ = true;
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
    if (has_cmd && cmd.hold) hold_ = true;
  }

  bool on_end(uint32_t* method, std::string* payload) override {
    ended_ = true;
    if (err_) return false;
    if (pc_) {                               // finished once the block exists (settle_create)
      end_seen_ = true;
      return false;
    }
    return finish(method, payload);
  }

  // The half-close's commit: native (committer) or the internal Python call {*method, *payload}.
  bool finish(uint32_t* method, std::string* payload) {
    if (committer_ && committer_->has_caller()) {
      try {
        hand_to_committer();
        return false;                        // produce() answers when the ticket is through
      } catch (const std::exception& e) {
        ticket_.reset();                     // nothing was submitted: commit through Python below
      }
    }
    if (!drain()) {                          // every H2D landed before the commit reads the block
      fail(13, "writing block " + std::to_string(block_) + ": H2D staging copy failed");
      return false;
    }
    // NativeWriteCommitRequest: session_id=1 block_id=2 length=3 pin=4 hold_for_append=6
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
    if (hold_) {
      h2::put_varint(m, (6u << 3));
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
  // The pool thread's create finished: write what queued up, then carry on as a normal stream.
  void settle_create() {
    {
      std::lock_guard<std::mutex> g(pc_->mu);
      if (!pc_->done) return;
      if (pc_->status) {
        if (!err_) fail(pc_->status, "creating block " + std::to_string(block_) + ": " + pc_->msg);
        pc_.reset();
        backlog_.clear();
        return;
      }
      device_ = store_->dir_spec(pc_->dir).kind == DirKind::kDevice;
    }
    pc_.reset();
    while (!backlog_.empty() && !err_) {
      Queued& q = backlog_.front();
      try {
        if (!q.data.empty()) write(reinterpret_cast<const uint8_t*>(q.data.data()), q.data.size());
      } catch (const StoreError& e) {
        fail(grpc_status_of(e), std::string("writing block ") + std::to_string(block_) + ": " + e.what());
      } catch (const std::exception& e) {
        fail(13, std::string("writing block ") + std::to_string(block_) + ": " + e.what());
      }
      if (q.flush && !err_) out_ += write_response_frame(pos_);
      backlog_.pop_front();
    }
    backlog_.clear();
    backlog_bytes_ = 0;
    if (waker_) waker_();                    // the client's window opens again
    if (end_seen_ && !err_) post_ready_ = finish(&post_method_, &post_payload_);
  }

  struct Queued {
    std::string data;
    bool flush = false;
  };

  void write(const uint8_t* p, size_t n) {
    if (!device_) {       // host arena / file dir: straight from the HTTP/2 receive buffer
      store_->write(session_, block_, pos_, reinterpret_cast<uint64_t>(p), n, (int)MemKind::kHost, 0, true);
    } else {
      // HBM: through two pinned staging slots, so the H2D is a DMA and not a pageable copy, and the
      // I/O thread does not wait for it -- the DMA of chunk k runs while chunk k+1 is received
      // and copied into the other slot; a slot is waited for only when it comes round again
      hipStream_t st = thread_stream(store_);
      size_t done = 0;
      while (done < n) {
        Slot& sl = slot_[cur_];
        if (!sl.buf) {
          sl.buf = pool_->get();
          if (hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming) != hipSuccess) sl.ev = nullptr;
        }
        if (sl.inflight) {
          if (hipEventSynchronize(sl.ev) != hipSuccess) throw std::runtime_error("H2D staging copy failed");
          sl.inflight = false;
        }
        const size_t k = (size_t)std::min<uint64_t>(n - done, pool_->size());
        std::memcpy(sl.buf, p + done, k);
        store_->write(session_, block_, pos_ + done, reinterpret_cast<uint64_t>(sl.buf), k, (int)MemKind::kHost,
                      reinterpret_cast<uint64_t>(st), sl.ev == nullptr);
        sl.inflight = sl.ev != nullptr && hipEventRecord(sl.ev, st) == hipSuccess;
        if (sl.ev && !sl.inflight) (void)hipStreamSynchronize(st);
        cur_ ^= 1;
        done += k;
      }
    }
    pos_ += n;
    stats_->write_bytes.fetch_add(n, std::memory_order_relaxed);
  }

  // The half-close of a native commit: HBM blocks get their per-page CRC32C computed on this I/O
  // thread's stream right behind the last H2D (no host pass over the bytes, no wait here), then an
  // event closes the block's device work; the committer thread takes it from there.
  void hand_to_committer() {
    auto t = std::make_shared<CommitTicket>();
    t->session = session_;
    t->block = block_;
    t->length = pos_;
    t->pin = pin_;
    t->hold = hold_;
    t->wake = waker_;
    if (device_) {
      hipStream_t st = thread_stream(store_);
      if (committer_->crc_device() && start_ == 0 && pos_ > 0) {
        const DirSpec ds = store_->dir_spec(store_->block_info(block_).dir);
        const size_t words = BlockStore::checksum_async_words(pos_, ds.page_size);
        if (words && committer_->take_crc_buffer(words, t.get())) {
          t->crc_pages = store_->checksum_async(block_, st, t->crc_dev, t->crc_words, t->crc_host, &t->crc_page);
          if (!t->crc_pages) t->crc_sync = true;
        } else {
          t->crc_sync = true;
        }
      } else if (committer_->crc_device()) {
        t->crc_sync = pos_ > 0;              // a resumed write: the committer checksums the whole block
      }
      if (hipEventCreateWithFlags(&t->done, hipEventDisableTiming) != hipSuccess) {
        t->done = nullptr;
        (void)hipStreamSynchronize(st);
      } else if (hipEventRecord(t->done, st) != hipSuccess) {
        (void)hipStreamSynchronize(st);
      }
    } else if (committer_->crc_host() && pos_ > 0) {
      t->crc_sync = true;                    // host blocks: the committer computes them
    }
    ticket_ = t;
    committer_->submit(t);
  }

  // Waits for the staging copies still in flight; false if one failed.
  bool drain() {
    bool ok = true;
    for (auto& sl : slot_) {
      if (!sl.inflight) continue;
      if (hipEventSynchronize(sl.ev) != hipSuccess) ok = false;
      sl.inflight = false;
    }
    return ok;
  }

  struct Slot {
    uint8_t* buf = nullptr;
    hipEvent_t ev = nullptr;
    bool inflight = false;
  };
  Slot slot_[2];
  int cur_ = 0;

  StoreRef store_;
  int64_t session_, block_;
  uint64_t start_, pos_;
  bool pin_, device_;
  uint32_t commit_;
  std::shared_ptr<StagingPool> pool_;
  std::shared_ptr<DataServerStats> stats_;
  std::shared_ptr<BlockCommitter> committer_;
  std::shared_ptr<CommitTicket> ticket_;
  std::function<void()> waker_;
  bool hold_ = false;
  std::shared_ptr<PendingCreate> pc_;
  std::deque<Queued> backlog_;
  uint64_t backlog_bytes_ = 0;
  bool end_seen_ = false, post_ready_ = false;
  uint32_t post_method_ = 0;
  std::string post_payload_;
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

// Threads for local-UFS file I/O of UFS_FILE write streams (immortal, like the upload pool): the
// I/O thread only queues chunks; mkdir, open, write(2), chmod and rename run here, so a slow or
// throttled disk never stalls the other streams multiplexed on that I/O thread.
class FilePool {
 public:
  static FilePool& get() {
    // one thread per concurrently written file up to 16 (ALLUXIO_UFS_FILE_THREADS overrides):
    // a CACHE_THROUGH tee append holds its thread for a whole block's D2H + write(2)
    static FilePool* p = [] {
      const char* e = std::getenv("ALLUXIO_UFS_FILE_THREADS");
      const int n = e ? std::atoi(e) : 16;
      return new FilePool(n > 0 ? std::min(n, 256) : 16);
    }();
    return *p;
  }
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }

 private:
  explicit FilePool(int n) {
    for (int i = 0; i < n; ++i)
      std::thread([this] {
        pthread_setname_np(pthread_self(), "ufs-file");
        for (;;) {
          std::function<void()> f;
          {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return !q_.empty(); });
            f = std::move(q_.front());
            q_.pop_front();
          }
          try {
            f();
          } catch (...) {
          }
        }
      }).detach();
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
};

// Pinned 8 MiB pieces for AppendBlock copies, shared by every stream of the process (per device):
// a small CACHE_THROUGH file must not pay a pinned allocation of its own.
constexpr uint64_t kTeePiece = 8ull << 20;
StagingPool& tee_pieces(int device) {
  static std::mutex mu;
  static std::map<int, StagingPool*> pools;      // immortal, like the pool threads that use them
  std::lock_guard<std::mutex> g(mu);
  StagingPool*& p = pools[device];
  if (!p) p = new StagingPool(kTeePiece, true, device);
  return *p;
}

struct TeePieces {                 // n pieces borrowed from tee_pieces() for one block copy
  StagingPool& pool;
  uint8_t* b[2] = {nullptr, nullptr};
  TeePieces(int device, int n) : pool(tee_pieces(device)) {
    for (int i = 0; i < n; ++i) b[i] = pool.get();
  }
  ~TeePieces() {
    for (uint8_t* p : b)
      if (p) pool.put(p);
  }
  TeePieces(const TeePieces&) = delete;
  TeePieces& operator=(const TeePieces&) = delete;
};

// State of one local UFS file write shared by its stream (I/O thread) and its pool tasks: one task
// at a time drains the chunk queue in order.
struct LocalFileJob {
  // Pool tasks writing one file at once: each takes the next queued item and pwrite()s it at its
  // own file offset, so a CACHE_THROUGH tee's block appends (D2H + write) and a THROUGH stream's
  // chunks use several cores instead of one sequential writer.
  static constexpr int kParallel = 4;
  std::string path, tmp;
  int mode = 0644;
  int fd = -1;
  std::mutex mu;
  // An appended block is split into pieces of kAppendPiece that the tasks may copy in parallel.
  // Buffered writes to one file serialize on its inode lock (pwrite of 512 MiB to one ext4 file
  // from 1/2/4/8 threads: 2.55/2.81/2.78/2.58 GB/s), so small pieces only add tasks contending for
  // that lock -- 16 MiB pieces cut 16-file CACHE_THROUGH from 20 to 15 GB/s.  Pieces are whole
  // blocks: parallel tasks overlap one block's D2H with another's write, nothing finer.
  static constexpr uint64_t kAppendPiece = 1ull << 30;
  struct Item {
    std::string data;                 // received bytes, or
    int64_t block = -1;               // [boff, boff + len) of a block this worker holds (CACHE_THROUGH tee)
    uint64_t boff = 0;
    uint64_t len = 0;
    uint64_t off = 0;                 // file offset
  };
  std::map<int64_t, int> pieces_left;   // appended block -> pieces not yet copied (its hold goes at 0)
  std::deque<Item> chunks;
  uint64_t queued = 0, written = 0;   // bytes; `written` is the contiguous prefix on disk
  std::map<uint64_t, uint64_t> done_ranges;   // completed [off, end) past `written`
  StoreRef store;                     // source of appended blocks
  int64_t session = 0;

  ~LocalFileJob() {
    for (const Item& it : chunks)      // appends never run (failed / cancelled file)
      if (it.block >= 0 && stats) stats->store_tasks.fetch_sub(1, std::memory_order_relaxed);
    if (store)
      for (const auto& kv : pieces_left)
        if (kv.second > 0) store->release_hold(kv.first);
  }

  // A piece of block `id` is done (copied or failed): the block's append hold goes with its last.
  void piece_done_locked(int64_t id) {
    auto it = pieces_left.find(id);
    if (it == pieces_left.end()) return;
    if (--it->second <= 0) {
      pieces_left.erase(it);
      if (store) store->release_hold(id);
    }
  }
  int active = 0, inflight = 0;       // pool tasks running / items being written
  bool opening = false, opened = false, failed = false, cancelled = false;
  bool end = false, finishing = false, finished = false, cleaned = false;
  int err_status = 0;
  std::string err;
  std::function<void()> wake;
  std::shared_ptr<DataServerStats> stats;

  void poke() {
    std::function<void()> w;
    {
      std::lock_guard<std::mutex> g(mu);
      w = wake;
    }
    if (w) w();
  }

  void fail_locked(int e, const std::string& what) {
    if (failed) return;
    failed = true;
    err_status = grpc_status_of_errno(e);
    err = what + ": " + std::strerror(e);
  }

  // [off, off + n) is on disk: advance the contiguous prefix.
  void complete_locked(uint64_t off, uint64_t n) {
    if (n == 0) return;
    done_ranges[off] = off + n;
    for (auto it = done_ranges.begin(); it != done_ranges.end() && it->first == written;
         it = done_ranges.erase(it))
      written = it->second;
  }

  // Tasks to add for what is queued (called with mu held); the caller submits that many drains.
  int want_tasks_locked() const {
    if (failed || cancelled) return active == 0 ? 1 : 0;     // one to clean up
    int work = (int)chunks.size() + ((!opened && !opening) ? 1 : 0) + ((end && !finishing && !finished) ? 1 : 0);
    if (!opened) work = std::min(work, 1);                    // one opens, the rest follow
    return std::max(0, std::min(kParallel - active, work - (active - inflight)));
  }

  // Creates the parents and the temp file beside the target.
  bool open_file() {
    int e = 0;
    if (!make_parents(path, &e)) {
      std::lock_guard<std::mutex> g(mu);
      fail_locked(e, "creating the parent of " + path);
      return false;
    }
    thread_local std::mt19937_64 rng(std::random_device{}());
    char tag[17];
    std::snprintf(tag, sizeof(tag), "%08x", (unsigned)(rng() & 0xffffffffu));
    const std::string t = path + ".alluxio." + tag + ".tmp";
    const int f = ::open(t.c_str(), O_WRONLY | O_CREAT | O_EXCL | O_CLOEXEC, 0666);
    std::lock_guard<std::mutex> g(mu);
    if (f < 0) {
      fail_locked(errno, "creating " + t);
      return false;
    }
    fd = f;
    tmp = t;
    opened = true;
    return true;
  }

  void cleanup() {   // failed / cancelled: drop the temp file, leave the target untouched
    if (cleaned) return;
    cleaned = true;
    if (fd >= 0) ::close(fd);
    fd = -1;
    if (!tmp.empty()) ::unlink(tmp.c_str());
  }

  static int pwrite_all(int fd, const uint8_t* p, uint64_t n, uint64_t off) {
    uint64_t done = 0;
    while (done < n) {
      const ssize_t w = ::pwrite(fd, p + done, (size_t)(n - done), (off_t)(off + done));
      if (w < 0) {
        if (errno == EINTR) continue;
        return errno;
      }
      done += (uint64_t)w;
    }
    return 0;
  }

  // Appends block `id` ([0, n) of it) from the store at file offset `at`: read-locked, copied out
  // in 8 MiB pieces through two pinned buffers on this pool thread's own stream, so the DMA of
  // piece k+1 runs while piece k is written to the file (and never waits behind the store's
  // internal stream).
  int append_block(int64_t id, uint64_t boff, uint64_t n, uint64_t at, std::string* what) {
    if (!store) {
      *what = "no block store for an appended block";
      return EINVAL;
    }
    int64_t lock = -1;
    try {
      lock = store->lock_block(session, id, false, 30000);
    } catch (const std::exception& e) {
      *what = std::string("appending block ") + std::to_string(id) + ": " + e.what();
      return ENOENT;
    }
    if (lock < 0) {
      *what = "appending block " + std::to_string(id) + ": lock timed out";
      return ETIMEDOUT;
    }
    constexpr uint64_t kPiece = kTeePiece;
    const bool dev = store->has_device();
    std::unique_ptr<TeePieces> pieces_buf;      // declared before the stream sync that frees them
    hipStream_t st = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    int e = 0;
    try {
      pieces_buf.reset(new TeePieces(store->device(), 2));
      if (dev) {
        // this pool thread's stream on the device: the copy never waits behind the store's
        // internal stream, and pool threads do not create a stream per block
        store->use_device();
        st = thread_stream_on(store->device());
        for (auto& x : ev)
          if (hipEventCreateWithFlags(&x, hipEventDisableTiming) != hipSuccess)
            throw std::runtime_error("hipEventCreate failed");
      }
      const uint64_t pieces = (n + kPiece - 1) / kPiece;
      auto issue = [&](uint64_t i) {
        const uint64_t off = i * kPiece, k = std::min(kPiece, n - off);
        uint8_t* b = pieces_buf->b[i & 1];
        std::vector<ReadReq> rq{ReadReq{id, boff + off, k, reinterpret_cast<uint64_t>(b), (int)MemKind::kHost}};
        store->read_batch(rq, reinterpret_cast<uint64_t>(st), !dev);
        if (dev && hipEventRecord(ev[i & 1], st) != hipSuccess) throw std::runtime_error("hipEventRecord failed");
      };
      if (pieces) issue(0);
      for (uint64_t i = 0; i < pieces && !e; ++i) {
        if (i + 1 < pieces) issue(i + 1);            // its buffer's previous piece is written
        if (dev && hipEventSynchronize(ev[i & 1]) != hipSuccess) throw std::runtime_error("D2H of an appended piece failed");
        const uint64_t k = std::min(kPiece, n - i * kPiece);
        e = pwrite_all(fd, pieces_buf->b[i & 1], k, at + i * kPiece);
        if (e) *what = "writing " + path;
      }
      if (dev && hipStreamSynchronize(st) != hipSuccess)   // nothing in flight into the pieces on return
        throw std::runtime_error("D2H of an appended piece failed");
    } catch (const std::exception& x) {
      e = EIO;
      *what = std::string("appending block ") + std::to_string(id) + ": " + x.what();
      if (st) (void)hipStreamSynchronize(st);
    }
    for (auto x : ev)
      if (x) (void)hipEventDestroy(x);
    try {
      store->unlock(lock);
    } catch (...) {
    }
    return e;
  }

  // Starts the pool tasks the queue wants (never holds mu across the submit).
  static void kick(const std::shared_ptr<LocalFileJob>& j) {
    int n;
    {
      std::lock_guard<std::mutex> g(j->mu);
      n = j->want_tasks_locked();
      j->active += n;
    }
    for (int i = 0; i < n; ++i) FilePool::get().submit([j] { LocalFileJob::drain(j); });
  }

  // One pool task: open (once), write queued items at their offsets, and -- the last one, when the
  // stream ended and every item is on disk -- chmod + rename.  A failed / cancelled file is
  // cleaned up by the last task to leave.
  static void drain(std::shared_ptr<LocalFileJob> j) {
    for (;;) {
      Item it;
      bool have = false, do_open = false, do_end = false;
      {
        std::lock_guard<std::mutex> g(j->mu);
        if (j->failed || j->cancelled) {
          if (--j->active == 0) j->cleanup();
          break;
        }
        if (!j->opened) {
          if (j->opening) {               // another task opens; it starts the others after
            --j->active;
            break;
          }
          j->opening = do_open = true;
        } else if (!j->chunks.empty()) {
          it = std::move(j->chunks.front());
          j->chunks.pop_front();
          ++j->inflight;
          have = true;
        } else if (j->end && j->inflight == 0 && !j->finishing && !j->finished) {
          j->finishing = do_end = true;
        } else {
          --j->active;
          break;
        }
      }
      if (do_open) {
        j->open_file();
        {
          std::lock_guard<std::mutex> g(j->mu);
          j->opening = false;
        }
        kick(j);                          // the other tasks the queue wants
        continue;
      }
      if (have && it.block >= 0) {
        std::string what;
        const int e = j->append_block(it.block, it.boff, it.len, it.off, &what);
        j->stats->store_tasks.fetch_sub(1, std::memory_order_relaxed);
        std::lock_guard<std::mutex> g(j->mu);
        --j->inflight;
        j->piece_done_locked(it.block);
        if (e) {
          if (!j->failed) {
            j->failed = true;
            j->err_status = grpc_status_of_errno(e);
            j->err = what + ": " + std::strerror(e);
          }
        } else {
          j->complete_locked(it.off, it.len);
          j->stats->ufs_write_bytes.fetch_add(it.len, std::memory_order_relaxed);
          j->stats->ufs_tee_bytes.fetch_add(it.len, std::memory_order_relaxed);
        }
      } else if (have) {
        const std::string& c = it.data;
        const int e = pwrite_all(j->fd, reinterpret_cast<const uint8_t*>(c.data()), c.size(), it.off);
        std::lock_guard<std::mutex> g(j->mu);
        --j->inflight;
        if (e) {
          j->fail_locked(e, "writing " + j->path);
        } else {
          j->complete_locked(it.off, c.size());
          j->stats->ufs_write_bytes.fetch_add(c.size(), std::memory_order_relaxed);
        }
      } else if (do_end) {
        int e = 0;
        if (::fchmod(j->fd, (mode_t)j->mode) != 0) e = errno;
        if (::close(j->fd) != 0 && !e) e = errno;
        j->fd = -1;
        if (!e && ::rename(j->tmp.c_str(), j->path.c_str()) != 0) e = errno;
        std::lock_guard<std::mutex> g(j->mu);
        if (e) j->fail_locked(e, "completing " + j->path);
        else j->finished = true;
      }
      j->poke();
    }
    j->poke();
  }
};

// UFS_FILE WriteBlock into a local-directory UFS: chunks go to a temp file beside the target (the
// local UFS's atomic create, underfs/local.py _AtomicWriter), written by FilePool tasks; the
// half-close sets the mode and renames it over the target.  A failed or cancelled call removes the
// temp file and leaves the target untouched.  At most kMaxQueued bytes wait for the disk: beyond
// that the stream stops accepting and the client's request window is held back.
class UfsFileWriteStream : public WriteStreamBase {
 public:
  static constexpr uint64_t kMaxQueued = 32ull << 20;

  UfsFileWriteStream(const std::string& path, int mode, std::shared_ptr<DataServerStats> stats,
                     StoreRef store = nullptr)
      : j_(std::make_shared<LocalFileJob>()) {
    j_->path = path;
    j_->mode = mode;
    j_->stats = std::move(stats);
    j_->store = store;
    j_->session = g_session.fetch_add(1);
  }

  // Queues the open (parents + temp file) on the file pool; errors surface on the stream.
  bool open(int*, std::string*) {
    kick();
    return true;
  }

  ~UfsFileWriteStream() override {
    {
      std::lock_guard<std::mutex> g(j_->mu);
      j_->wake = nullptr;
      if (!j_->finished) j_->cancelled = true;
    }
    LocalFileJob::kick(j_);          // with no task running, one closes + unlinks the temp file
  }

  void set_waker(std::function<void()> w) override {
    std::lock_guard<std::mutex> g(j_->mu);
    j_->wake = std::move(w);
  }

  bool accepting() override {
    std::lock_guard<std::mutex> g(j_->mu);
    return j_->queued - j_->written < kMaxQueued || j_->failed;
  }

  void on_message(const char* p, size_t n) override {
    if (err_ || ended_) return;
    WriteCmd cmd;
    bool has_cmd;
    const uint8_t* chunk;
    size_t len;
    int64_t append_id = -1;
    uint64_t append_len = 0;
    if (!parse_write_request(p, n, &cmd, &has_cmd, &chunk, &len, &append_id, &append_len)) {
      fail(3, "malformed WriteRequest");
      return;
    }
    if (append_id >= 0) {              // CACHE_THROUGH tee: the next bytes are a block we hold
      {
        std::lock_guard<std::mutex> g(j_->mu);
        int pieces = 0;
        for (uint64_t b = 0; b < append_len || (append_len == 0 && b == 0); b += LocalFileJob::kAppendPiece) {
          LocalFileJob::Item it;
          it.block = append_id;
          it.boff = b;
          it.len = std::min<uint64_t>(LocalFileJob::kAppendPiece, append_len - b);
          it.off = j_->queued + b;
          j_->chunks.push_back(std::move(it));
          j_->stats->store_tasks.fetch_add(1, std::memory_order_relaxed);
          ++pieces;
          if (append_len == 0) break;
        }
        j_->pieces_left[append_id] += pieces;
        j_->queued += append_len;
      }
      kick();
      pos_ += append_len;
    }
    if (len) {
      {
        std::lock_guard<std::mutex> g(j_->mu);
        LocalFileJob::Item it;
        it.data.assign(reinterpret_cast<const char*>(chunk), len);
        it.off = j_->queued;
        j_->chunks.push_back(std::move(it));
        j_->queued += len;
      }
      kick();
    }
    pos_ += len;
    if (has_cmd && cmd.flush) flushes_.push_back(pos_);   // acked once written
    emit();
  }

  bool on_end(uint32_t*, std::string*) override {
    ended_ = true;
    if (err_) return false;
    {
      std::lock_guard<std::mutex> g(j_->mu);
      j_->end = true;
    }
    kick();
    return false;
  }

  ssize_t produce(uint8_t* dst, size_t max, bool* eof, int* status, std::string* msg) override {
    emit();
    return WriteStreamBase::produce(dst, max, eof, status, msg);
  }

 private:
  void kick() { LocalFileJob::kick(j_); }

  // Flush acks for written data, the failure, or the final frame once the file is in place.
  void emit() {
    std::lock_guard<std::mutex> g(j_->mu);
    if (j_->failed) {
      if (!err_) fail(j_->err_status, j_->err);
      return;
    }
    while (!flushes_.empty() && flushes_.front() <= j_->written) {
      out_ += write_response_frame(flushes_.front());
      flushes_.pop_front();
    }
    if (j_->finished && !done_) {
      out_ += write_response_frame(pos_);
      done_ = true;
    }
  }

  std::shared_ptr<LocalFileJob> j_;
  uint64_t pos_ = 0;
  std::deque<uint64_t> flushes_;
};


// ---- UFS_FILE writes into an S3 mount: streamed multipart upload -------------------------------

// Upload threads shared by every S3 write stream (immortal: a stuck HTTP call never blocks exit).
class UploadPool {
 public:
  static UploadPool& get() {
    static UploadPool* p = new UploadPool(16);
    return *p;
  }
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }

 private:
  explicit UploadPool(int n) {
    for (int i = 0; i < n; ++i)
      std::thread([this] {
        pthread_setname_np(pthread_self(), "s3-upload");
        for (;;) {
          std::function<void()> f;
          {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return !q_.empty(); });
            f = std::move(q_.front());
            q_.pop_front();
          }
          try {
            f();
          } catch (...) {
          }
        }
      }).detach();
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
};

std::string xml_tag(const std::string& x, const std::string& tag) {
  const std::string a = "<" + tag + ">", b = "</" + tag + ">";
  const size_t i = x.find(a);
  if (i == std::string::npos) return "";
  const size_t j = x.find(b, i + a.size());
  return j == std::string::npos ? "" : x.substr(i + a.size(), j - i - a.size());
}

std::string query_escape(const std::string& v) {   // RFC 3986, '/' escaped too (SigV4 query)
  std::string e = uri_encode_path(v), o;
  for (char c : e) {
    if (c == '/') o += "%2F";
    else o.push_back(c);
  }
  return o;
}

// State of one multipart upload shared by its stream (I/O thread) and its upload tasks.
struct S3Upload {
  std::shared_ptr<const S3Mount> m;
  std::string path;                 // "/bucket/key"
  std::mutex mu;
  std::condition_variable cv;
  std::string upload_id;
  bool init_started = false, init_done = false;
  std::map<int, std::string> etags;
  int inflight = 0;                 // part uploads queued or running
  std::vector<uint8_t*> free_bufs;
  int allocated = 0;
  bool failed = false, cancelled = false, finishing = false, finished = false;
  std::string err;
  std::function<void()> wake;
  std::shared_ptr<DataServerStats> stats;
  uint64_t part = 0;                // part size
  int max_bufs = 0;                 // part buffers in flight at most (+1 being filled)
  // The part being filled.  Owned by the stream's I/O thread, or by an AppendBlock task while
  // `appending` (the I/O thread then only queues what arrives).
  uint8_t* cur = nullptr;
  uint64_t fill = 0;
  int parts = 0;
  bool appending = false;

  ~S3Upload() {
    for (uint8_t* b : free_bufs) std::free(b);
    if (cur) std::free(cur);
  }

  // A free part buffer, a new one while under max_bufs, else null -- or, with `wait`, blocks until
  // an upload returns one (null when the upload failed or was cancelled meanwhile).
  uint8_t* take_buf(bool wait) {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      if (!free_bufs.empty()) {
        uint8_t* b = free_bufs.back();
        free_bufs.pop_back();
        return b;
      }
      if (allocated < max_bufs) {
        uint8_t* b = static_cast<uint8_t*>(std::malloc(part));
        if (b) ++allocated;
        return b;
      }
      if (!wait || failed || cancelled) return nullptr;
      cv.wait(lk);
    }
  }

  static void submit_cur(const std::shared_ptr<S3Upload>& u) {
    uint8_t* b = u->cur;
    const uint64_t n = u->fill;
    u->cur = nullptr;
    u->fill = 0;
    const int num = ++u->parts;
    {
      std::lock_guard<std::mutex> g(u->mu);
      ++u->inflight;
    }
    auto uu = u;
    UploadPool::get().submit([uu, num, b, n] { S3Upload::upload_part(uu, num, b, n); });
  }

  // Copies into part buffers, submitting each full one; returns the bytes taken (fewer when every
  // buffer is in flight and `wait` is off, or when the upload failed / was cancelled).
  static size_t fill_parts(const std::shared_ptr<S3Upload>& u, const uint8_t* p, size_t n, bool wait) {
    size_t done = 0;
    while (done < n) {
      if (!u->cur) {
        u->cur = u->take_buf(wait);
        u->fill = 0;
        if (!u->cur) break;
      }
      const size_t k = (size_t)std::min<uint64_t>(n - done, u->part - u->fill);
      std::memcpy(u->cur + u->fill, p + done, k);
      u->fill += k;
      done += k;
      if (u->fill == u->part) submit_cur(u);
    }
    return done;
  }

  // AppendBlock on a pool thread: block `id` ([0, n)) of the worker's store goes into the parts,
  // read-locked and copied out in 8 MiB pieces through a pinned bounce buffer.  Clears `appending`
  // and wakes the stream when done; a failure fails the upload (aborted like any other).
  static void append_block(std::shared_ptr<S3Upload> u, StoreRef store, int64_t session, int64_t id, uint64_t n) {
    std::string e;
    int64_t lock = -1;
    try {
      lock = store->lock_block(session, id, false, 30000);
      if (lock < 0) e = "appending block " + std::to_string(id) + ": lock timed out";
      else store->release_hold(id);
    } catch (const std::exception& x) {
      e = std::string("appending block ") + std::to_string(id) + ": " + x.what();
    }
    if (e.empty()) {
      constexpr uint64_t kPiece = kTeePiece;
      std::unique_ptr<TeePieces> piece;
      hipStream_t own = nullptr;
      try {
        piece.reset(new TeePieces(store->device(), 1));
        uint8_t* bounce = piece->b[0];
        if (store->has_device()) {
          store->use_device();
          own = thread_stream_on(store->device());
        }
        const uint64_t st = reinterpret_cast<uint64_t>(own);
        for (uint64_t off = 0; off < n;) {
          {
            std::lock_guard<std::mutex> g(u->mu);
            if (u->failed || u->cancelled) break;
          }
          const uint64_t k = std::min(kPiece, n - off);
          std::vector<ReadReq> rq{ReadReq{id, off, k, reinterpret_cast<uint64_t>(bounce), (int)MemKind::kHost}};
          store->read_batch(rq, st, true);
          if (fill_parts(u, bounce, (size_t)k, true) < k) break;      // failed / cancelled meanwhile
          u->stats->ufs_tee_bytes.fetch_add(k, std::memory_order_relaxed);
          off += k;
        }
      } catch (const std::exception& x) {
        e = std::string("appending block ") + std::to_string(id) + ": " + x.what();
      }
      if (own) (void)hipStreamSynchronize(own);   // nothing in flight into the piece
      piece.reset();
      try {
        store->unlock(lock);
      } catch (...) {
      }
    }
    bool abort_now;
    {
      std::lock_guard<std::mutex> g(u->mu);
      u->appending = false;
      if (!e.empty() && !u->failed) {
        u->failed = true;
        u->err = e;
      }
      abort_now = (u->failed || u->cancelled) && u->inflight == 0 && !u->finished;
    }
    u->cv.notify_all();
    if (abort_now) finish(u);
    u->poke();
    u->stats->store_tasks.fetch_sub(1, std::memory_order_relaxed);   // the store is not used past here
  }

  // One S3 call (retried inside the reader on 5xx / SlowDown / resets / timeouts).  Part and object
  // PUTs stop early once the stream is cancelled; Complete / Abort always run to their end.
  int send(const std::string& method, const std::string& query, const uint8_t* body, uint64_t n, std::string* resp,
           std::string* etag, const std::string& payload_hash = "UNSIGNED-PAYLOAD", bool cancellable = false) {
    const std::string head = s3_header_lines(m->cred, method, path, query, payload_hash);
    const std::string target = uri_encode_path(path) + (query.empty() ? "" : "?" + query);
    return m->reader->request(method, target, head, body, n, resp, etag, cancellable ? &abort_flag : nullptr);
  }
  std::atomic<bool> abort_flag{false};   // set with `cancelled`
  int err_status = 13;                   // gRPC status of `err`

  void poke() {
    std::function<void()> w;
    {
      std::lock_guard<std::mutex> g(mu);
      w = wake;
    }
    if (w) w();
  }

  // CreateMultipartUpload, once (the first part's task runs it; the others wait).
  bool ensure_init(std::string* e) {
    std::unique_lock<std::mutex> lk(mu);
    if (!init_started) {
      init_started = true;
      lk.unlock();
      std::string resp;
      const int code = send("POST", "uploads=", nullptr, 0, &resp, nullptr);
      const std::string id = code == 200 ? xml_tag(resp, "UploadId") : "";
      lk.lock();
      if (id.empty() && !failed) {
        failed = true;
        err = "CreateMultipartUpload of " + path + " failed: " + std::to_string(code);
      }
      upload_id = id;
      init_done = true;
      cv.notify_all();
    }
    cv.wait(lk, [&] { return init_done; });
    if (upload_id.empty()) {
      *e = err;
      return false;
    }
    return true;
  }

  // Runs on an upload thread: UploadPart `num` out of `buf` (returned to the free list).
  static void upload_part(std::shared_ptr<S3Upload> u, int num, uint8_t* buf, uint64_t n) {
    std::string e, etag;
    bool skip;
    {
      std::lock_guard<std::mutex> g(u->mu);
      skip = u->cancelled || u->failed;
    }
    bool ok = skip ? false : u->ensure_init(&e);
    if (ok) {
      const std::string q = "partNumber=" + std::to_string(num) + "&uploadId=" + query_escape(u->upload_id);
      const int code = u->send("PUT", q, buf, n, nullptr, &etag, "UNSIGNED-PAYLOAD", true);
      ok = code == 200 || code == 204;
      if (!ok) {
        e = "UploadPart " + std::to_string(num) + " of " + u->path + " failed after retries: " + std::to_string(code);
        if (HttpRangeReader::retryable(code)) {
          std::lock_guard<std::mutex> g(u->mu);
          u->err_status = 14;   // UNAVAILABLE: the store kept failing / timing out
        }
      }
      else u->stats->ufs_write_bytes.fetch_add(n, std::memory_order_relaxed);
    }
    bool last;
    {
      std::lock_guard<std::mutex> g(u->mu);
      if (ok) u->etags[num] = etag;
      else if (!skip && !u->failed) {
        u->failed = true;
        u->err = e;
      }
      u->free_bufs.push_back(buf);
      last = --u->inflight == 0 && (u->finishing || u->cancelled || u->failed) && !u->appending;
    }
    u->cv.notify_all();                // an AppendBlock task may wait for this buffer
    if (last) finish(u);
    u->poke();
  }

  // After the last part: CompleteMultipartUpload, or AbortMultipartUpload on failure / cancel.
  static void finish(std::shared_ptr<S3Upload> u) {
    bool abort;
    std::string id;
    {
      std::lock_guard<std::mutex> g(u->mu);
      if (u->finished) return;
      abort = u->failed || u->cancelled;
      id = u->upload_id;
      if (!abort && !u->finishing) return;
    }
    std::string e;
    if (abort) {
      if (!id.empty()) u->send("DELETE", "uploadId=" + query_escape(id), nullptr, 0, nullptr, nullptr);
    } else {
      std::string body = "<CompleteMultipartUpload>";
      {
        std::lock_guard<std::mutex> g(u->mu);
        for (const auto& kv : u->etags)
          body += "<Part><PartNumber>" + std::to_string(kv.first) + "</PartNumber><ETag>" + kv.second +
                  "</ETag></Part>";
      }
      body += "</CompleteMultipartUpload>";
      std::string resp;
      const int code = u->send("POST", "uploadId=" + query_escape(id), reinterpret_cast<const uint8_t*>(body.data()),
                               body.size(), &resp, nullptr, sha256_hex(body.data(), body.size()));
      if (code != 200 || resp.find("<Error>") != std::string::npos) {
        e = "CompleteMultipartUpload of " + u->path + " failed: " + std::to_string(code);
        u->send("DELETE", "uploadId=" + query_escape(id), nullptr, 0, nullptr, nullptr);
      }
    }
    {
      std::lock_guard<std::mutex> g(u->mu);
      if (!e.empty() && !u->failed) {
        u->failed = true;
        u->err = e;
      }
      u->finished = true;
    }
    u->poke();
  }
};

class S3UfsWriteStream : public WriteStreamBase {
 public:
  S3UfsWriteStream(std::shared_ptr<const S3Mount> m, const std::string& key, std::shared_ptr<DataServerStats> stats,
                   StoreRef store)
      : u_(std::make_shared<S3Upload>()), store_(store), session_(g_session.fetch_add(1)) {
    u_->part = m->upload_part;
    u_->max_bufs = m->upload_inflight + 1;
    u_->m = std::move(m);
    u_->path = "/" + u_->m->bucket + "/" + key;
    u_->stats = std::move(stats);
  }

  ~S3UfsWriteStream() override {
    for (const Pending& p : pending_)  // appends that never ran
      if (p.block >= 0 && store_) store_->release_hold(p.block);
    bool idle;
    {
      std::lock_guard<std::mutex> g(u_->mu);
      u_->wake = nullptr;
      if (!u_->finished && !(u_->finishing && !u_->failed)) {   // abandoned: abort
        u_->cancelled = true;
        u_->abort_flag.store(true, std::memory_order_relaxed);
      }
      idle = u_->inflight == 0 && !u_->appending;
    }
    u_->cv.notify_all();               // an AppendBlock task waiting for a buffer stops
    if (idle && u_->cancelled) {
      auto u = u_;
      UploadPool::get().submit([u] { S3Upload::finish(u); });
    }
  }

  void set_waker(std::function<void()> w) override {
    std::lock_guard<std::mutex> g(u_->mu);
    u_->wake = std::move(w);
  }

  bool accepting() override {
    drain_pending();
    return pending_.empty() && !busy();
  }

  void on_message(const char* p, size_t n) override {
    if (err_ || ended_) return;
    WriteCmd cmd;
    bool has_cmd;
    const uint8_t* chunk;
    size_t len;
    int64_t append_id = -1;
    uint64_t append_len = 0;
    if (!parse_write_request(p, n, &cmd, &has_cmd, &chunk, &len, &append_id, &append_len)) {
      fail(3, "malformed WriteRequest");
      return;
    }
    if (append_id >= 0) {              // the next bytes are a block of this worker's store
      if (!store_) {
        fail(12, "AppendBlock needs the worker's block store");
        return;
      }
      pending_.push_back(Pending{std::string(), append_id, append_len});
      pos_ += append_len;
      drain_pending();
    }
    if (len) {
      if (pending_.empty() && !busy()) {
        const size_t took = S3Upload::fill_parts(u_, chunk, len, false);
        if (took < len) pending_.push_back(Pending{std::string(reinterpret_cast<const char*>(chunk + took), len - took)});
      } else {
        pending_.push_back(Pending{std::string(reinterpret_cast<const char*>(chunk), len)});
      }
      pos_ += len;
    }
    if (has_cmd && cmd.flush) out_ += write_response_frame(pos_);   // S3 has nothing to flush
  }

  bool on_end(uint32_t*, std::string*) override {
    ended_ = true;
    if (err_) return false;
    end_pending_ = true;
    try_finish();
    return false;
  }

  ssize_t produce(uint8_t* dst, size_t max, bool* eof, int* status, std::string* msg) override {
    drain_pending();
    if (end_pending_) try_finish();
    {
      std::lock_guard<std::mutex> g(u_->mu);
      if (u_->failed && !err_) fail(u_->err_status, u_->err);
      else if (u_->finished && !done_ && !err_ && submitted_end_) {
        out_ += write_response_frame(pos_);
        done_ = true;
      }
    }
    return WriteStreamBase::produce(dst, max, eof, status, msg);
  }

 private:
  // What arrived while the parts could not take it, in file order: received bytes, or a block
  // to append (AppendBlock).
  struct Pending {
    std::string data;
    int64_t block = -1;
    uint64_t len = 0;
  };

  bool busy() {
    std::lock_guard<std::mutex> g(u_->mu);
    return u_->appending;
  }

  // Feeds queued items to the parts in order; an AppendBlock hands the parts to a pool task and
  // stops here until that task is done (it wakes the stream).
  void drain_pending() {
    while (!pending_.empty()) {
      if (busy()) return;
      Pending& f = pending_.front();
      if (f.block >= 0) {
        {
          std::lock_guard<std::mutex> g(u_->mu);
          u_->appending = true;
        }
        auto u = u_;
        StoreRef st = store_;
        const int64_t ses = session_, id = f.block;
        const uint64_t n = f.len;
        pending_.pop_front();
        u->stats->store_tasks.fetch_add(1, std::memory_order_relaxed);
        FilePool::get().submit([u, st, ses, id, n] { S3Upload::append_block(u, st, ses, id, n); });
        return;
      }
      const size_t took = S3Upload::fill_parts(u_, reinterpret_cast<const uint8_t*>(f.data.data()), f.data.size(), false);
      if (took < f.data.size()) {
        f.data.erase(0, took);
        return;
      }
      pending_.pop_front();
    }
  }

  void try_finish() {
    if (!pending_.empty() || busy() || submitted_end_) return;
    submitted_end_ = true;
    end_pending_ = false;
    if (u_->parts == 0) {              // smaller than a part: one PutObject
      uint8_t* b = u_->cur;
      const uint64_t n = u_->fill;
      u_->cur = nullptr;
      {
        std::lock_guard<std::mutex> g(u_->mu);
        ++u_->inflight;
        u_->init_started = u_->init_done = true;
      }
      auto u = u_;
      UploadPool::get().submit([u, b, n] {
        std::string e;
        const int code = u->send("PUT", "", b, n, nullptr, nullptr, "UNSIGNED-PAYLOAD", true);
        if (code == 200 || code == 204) u->stats->ufs_write_bytes.fetch_add(n, std::memory_order_relaxed);
        std::lock_guard<std::mutex> g(u->mu);
        if (code != 200 && code != 204 && !u->failed) {
          u->failed = true;
          u->err = "PutObject " + u->path + " failed: " + std::to_string(code);
        }
        if (b) u->free_bufs.push_back(b);
        --u->inflight;
        u->finished = true;
        u->cv.notify_all();
        auto w = u->wake;
        if (w) w();
      });
      return;
    }
    if (u_->fill) S3Upload::submit_cur(u_);
    bool idle;
    {
      std::lock_guard<std::mutex> g(u_->mu);
      u_->finishing = true;
      idle = u_->inflight == 0;
    }
    if (idle) {
      auto u = u_;
      UploadPool::get().submit([u] { S3Upload::finish(u); });
    }
  }

  std::shared_ptr<S3Upload> u_;
  StoreRef store_;
  int64_t session_;
  uint64_t pos_ = 0;
  std::deque<Pending> pending_;
  bool end_pending_ = false, submitted_end_ = false;
};

}  // namespace

// ---- deferred reclaim of deleted UFS files ------------------------------------------------------
namespace {

class Reclaimer {
 public:
  static Reclaimer& get() {
    static Reclaimer* r = new Reclaimer();   // immortal, like its thread
    return *r;
  }
  // Threads freeing files at once: 16 CACHE_THROUGH writers delete ~70 files of 256 MiB a second
  // (~20 ms of teardown each), more than one thread keeps up with -- a backlog of deleted pages
  // would push the writers into direct reclaim.
  static constexpr int kMaxThreads = 4;
  // false: too many waiting (the caller closes inline)
  bool push(int fd, size_t max_pending) {
    std::lock_guard<std::mutex> g(mu_);
    if (q_.size() >= max_pending) return false;
    q_.push_back(fd);
    if ((int)q_.size() > idle_ && threads_ < kMaxThreads) {
      try {
        std::thread([this] { loop(); }).detach();
        ++threads_;
      } catch (...) {
        if (threads_ == 0) {
          q_.pop_back();
          return false;
        }
      }
    }
    cv_.notify_one();
    return true;
  }
  uint64_t done() const { return done_.load(std::memory_order_relaxed); }
  size_t pending() {
    std::lock_guard<std::mutex> g(mu_);
    return q_.size() + (size_t)busy_;
  }

 private:
  void loop() {
    pthread_setname_np(pthread_self(), "ufs-reclaim");
    for (;;) {
      int fd;
      {
        std::unique_lock<std::mutex> lk(mu_);
        ++idle_;
        cv_.wait(lk, [&] { return !q_.empty(); });
        --idle_;
        fd = q_.front();
        q_.pop_front();
        ++busy_;
      }
      ::close(fd);                 // the last reference: the inode and its pages go here
      done_.fetch_add(1, std::memory_order_relaxed);
      std::lock_guard<std::mutex> g(mu_);
      --busy_;
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<int> q_;
  int threads_ = 0, idle_ = 0, busy_ = 0;
  std::atomic<uint64_t> done_{0};
};

}  // namespace

int unlink_deferred(const std::string& path, uint64_t defer_bytes, size_t max_pending) {
  const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC | O_NOFOLLOW | O_NONBLOCK);
  struct stat sb;
  if (fd < 0 || ::fstat(fd, &sb) != 0 || !S_ISREG(sb.st_mode) || (uint64_t)sb.st_size < defer_bytes) {
    if (fd >= 0) ::close(fd);
    return ::unlink(path.c_str()) == 0 ? 0 : errno;
  }
  if (::unlink(path.c_str()) != 0) {
    const int e = errno;
    ::close(fd);
    return e;
  }
  if (!Reclaimer::get().push(fd, max_pending)) ::close(fd);
  return 0;
}

uint64_t reclaimed_files() { return Reclaimer::get().done(); }
size_t reclaim_pending() { return Reclaimer::get().pending(); }


namespace {
std::string strip_file_scheme(const std::string& p) { return p.compare(0, 7, "file://") == 0 ? p.substr(7) : p; }
}  // namespace

void UfsMounts::set(int64_t mount_id, const std::string& root) {
  std::string r = strip_file_scheme(root);
  while (!r.empty() && r.back() == '/') r.pop_back();     // "/" -> "" (every absolute path)
  std::lock_guard<std::mutex> g(mu_);
  roots_[mount_id] = r;
}

void UfsMounts::remove(int64_t mount_id) {
  std::lock_guard<std::mutex> g(mu_);
  roots_.erase(mount_id);
  s3_.erase(mount_id);
  python_.erase(mount_id);
}

void UfsMounts::set_s3(int64_t mount_id, const std::string& host, int port, const std::string& bucket,
                       const std::string& access_key, const std::string& secret_key, const std::string& region,
                       int parallel, uint64_t part, uint64_t upload_part, int upload_inflight,
                       const HttpOptions& http) {
  auto m = std::make_shared<S3Mount>();
  m->http = http;
  m->upload_part = std::max<uint64_t>(upload_part, 64u << 10);
  m->upload_inflight = std::max(1, upload_inflight);
  m->host = host;
  m->port = port;
  m->bucket = bucket;
  m->cred.host_header = port == 80 ? host : host + ":" + std::to_string(port);
  m->cred.access_key = access_key;
  m->cred.secret_key = secret_key;
  m->cred.region = region.empty() ? "us-east-1" : region;
  m->parallel = std::max(1, parallel);
  m->part = std::max<uint64_t>(part, 64u << 10);
  m->reader = std::make_shared<HttpRangeReader>(host, port, 2 * m->parallel, m->http);
  std::lock_guard<std::mutex> g(mu_);
  s3_[mount_id] = std::move(m);
}

bool UfsMounts::resolve_s3(int64_t mount_id, const std::string& ufs_path, std::shared_ptr<const S3Mount>* m,
                           std::string* key) const {
  std::shared_ptr<const S3Mount> mount;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = s3_.find(mount_id);
    if (it == s3_.end()) return false;
    mount = it->second;
  }
  const size_t sch = ufs_path.find("://");
  if (sch == std::string::npos) return false;
  const std::string rest = ufs_path.substr(sch + 3);      // bucket/key
  const size_t slash = rest.find('/');
  if (rest.substr(0, slash) != mount->bucket) return false;
  std::string k = slash == std::string::npos ? std::string() : rest.substr(slash + 1);
  size_t lead = 0;
  while (lead < k.size() && k[lead] == '/') ++lead;
  k.erase(0, lead);
  if (k.empty()) return false;
  *m = std::move(mount);
  *key = std::move(k);
  return true;
}

void UfsMounts::mark_python(int64_t mount_id) {
  std::lock_guard<std::mutex> g(mu_);
  python_[mount_id] = true;
}

bool UfsMounts::is_python(int64_t mount_id) const {
  std::lock_guard<std::mutex> g(mu_);
  return python_.count(mount_id) != 0;
}

size_t UfsMounts::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return roots_.size() + s3_.size();
}

bool UfsMounts::resolve(int64_t mount_id, const std::string& ufs_path, std::string* local) const {
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

namespace {

// The reader of `o`'s file when its mount is registered: 1 = *reader set, 0 = mount not registered
// (or the path is outside it), -1 = the file cannot be opened (*status / *msg set).
int open_ufs_reader(const UfsMounts& mounts, const UfsOpts& o, std::unique_ptr<UfsReader>* reader, int* status,
                    std::string* msg) {
  std::string local, key;
  std::shared_ptr<const S3Mount> s3;
  if (mounts.resolve(o.mount_id, o.ufs_path, &local)) {
    const int fd = ::open(local.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) {
      const int e = errno;
      *status = grpc_status_of_errno(e);
      *msg = "opening " + o.ufs_path + ": " + std::strerror(e);
      return -1;
    }
    reader->reset(new LocalFileReader(fd));
    return 1;
  }
  if (mounts.resolve_s3(o.mount_id, o.ufs_path, &s3, &key)) {
    reader->reset(new S3ObjectReader(std::move(s3), std::move(key)));
    return 1;
  }
  return 0;
}

// A native cold stream for `r` (the block is not in the store), or nullptr to hand the call to
// Python (mount not registered, UFS-tier block, too many readers).
std::unique_ptr<NativeStream> make_cold_stream(const ReadRequestMsg& r, const StoreRef& store, uint64_t max_chunk,
                                               uint64_t window, bool unix_peer, const ColdReadConfig& cfg,
                                               const std::shared_ptr<UfsMounts>& mounts,
                                               const std::shared_ptr<StagingPool>& slot_pool,
                                               const std::shared_ptr<DataServerStats>& stats,
                                               std::function<void(uint32_t, std::string)> post, int* status,
                                               std::string* msg,
                                               const std::shared_ptr<BlockCommitter>& committer = nullptr,
                                               BlockCommitter::Caller caller = nullptr,
                                               const std::shared_ptr<ColdReadAhead>& readahead = nullptr) {
  UfsOpts o;
  if (!mounts || !parse_ufs_opts(r.ufs_opts, &o) || o.ufs_path.empty() || o.block_in_ufs_tier || o.block_size <= 0)
    return nullptr;
  const uint64_t block_len = (uint64_t)o.block_size;
  const uint64_t off = (uint64_t)std::max<int64_t>(0, r.offset);
  if (off > block_len) {
    *status = 11;
    *msg = "offset " + std::to_string(off) + " beyond block " + std::to_string(r.block_id) + " of " +
           std::to_string(block_len) + " bytes";
    return nullptr;
  }
  const uint64_t end = r.length > 0 ? std::min<uint64_t>(block_len, off + (uint64_t)r.length) : block_len;
  std::unique_ptr<UfsReader> reader;
  std::function<bool(std::unique_ptr<UfsReader>*, int*, std::string*)> resolve;
  const int opened = open_ufs_reader(*mounts, o, &reader, status, msg);
  if (opened < 0) return nullptr;
  if (opened == 0) {
    // not registered yet: a plain local or S3 path of a mount not known to be Python's is resolved
    // on the reader's pool thread (ResolveUfsMount) and then read natively
    const std::string& p = o.ufs_path;
    const bool plausible = p[0] == '/' || p.compare(0, 7, "file://") == 0 || p.compare(0, 5, "s3://") == 0 ||
                           p.compare(0, 6, "s3a://") == 0;
    if (!plausible || cfg.resolve_method == UINT32_MAX || !caller || mounts->is_python(o.mount_id)) return nullptr;
    auto ms = mounts;
    const uint32_t method = cfg.resolve_method, range_method = cfg.read_range_method;
    resolve = [ms, o, method, range_method, caller](std::unique_ptr<UfsReader>* out, int* st,
                                                    std::string* err) -> bool {
      // ResolveUfsMountRequest: mount_id=1 ufs_path=2
      std::string m;
      h2::put_varint(m, (1u << 3));
      h2::put_varint(m, (uint64_t)o.mount_id);
      h2::put_varint(m, (2u << 3) | 2);
      h2::put_varint(m, o.ufs_path.size());
      m += o.ufs_path;
      struct Reply {
        std::mutex mu;
        std::condition_variable cv;
        bool got = false;
        int status = 0;
        std::string msg;
      };
      auto rep = std::make_shared<Reply>();
      caller(method, std::move(m), [rep](int s, const std::string& msg, const std::string&) {
        std::lock_guard<std::mutex> g(rep->mu);
        rep->got = true;
        rep->status = s;
        rep->msg = msg;
        rep->cv.notify_all();
      });
      {
        std::unique_lock<std::mutex> lk(rep->mu);
        if (!rep->cv.wait_for(lk, std::chrono::seconds(60), [&] { return rep->got; })) {
          *st = 14;
          *err = "resolving the UFS of mount " + std::to_string(o.mount_id) + " timed out";
          return false;
        }
      }
      if (rep->status) {
        *st = rep->status == 5 ? 5 : 14;
        *err = "resolving the UFS of mount " + std::to_string(o.mount_id) + ": " + rep->msg;
        return false;
      }
      const int r = open_ufs_reader(*ms, o, out, st, err);
      if (r == 0) {                          // resolved, but not something the I/O threads reach
        ms->mark_python(o.mount_id);         // its later cold reads go to the Python servicer
        if (range_method == UINT32_MAX) {
          *st = 14;
          *err = "the UFS of mount " + std::to_string(o.mount_id) + " is served by the worker's Python data path";
          return false;
        }
        out->reset(new PythonRangeReader(caller, range_method, o.mount_id, o.ufs_path));
        return true;
      }
      return r > 0;
    };
  }
  if (stats->cold_active.fetch_add(1, std::memory_order_relaxed) >= cfg.max_active) {
    stats->cold_active.fetch_sub(1, std::memory_order_relaxed);
    return nullptr;
  }
  // UnderFileSystemBlockReader caches only a whole-block sequential read; anything else streams
  const bool cache = !o.no_cache && off == 0 && end == block_len &&
                     (cfg.commit_method != UINT32_MAX || committer) && !store->has_temp_block(r.block_id);
  auto st = std::make_shared<ColdState>();
  st->pool = slot_pool;
  st->slots.resize((size_t)std::max(2, cfg.depth));
  auto job = std::make_shared<ColdJob>();
  job->store = store;
  job->session = g_session.fetch_add(1);
  job->block = r.block_id;
  job->start = off;
  job->end = end;
  job->block_len = block_len;
  job->file_off = (uint64_t)std::max<int64_t>(0, o.offset_in_file);
  job->slot_bytes = slot_pool->size();
  job->want_cache = cache;
  job->create_after = cfg.create_after_reads > 0 ? (size_t)cfg.create_after_reads : st->slots.size();
  job->reader = std::move(reader);
  job->st = st;
  job->stats = stats;
  job->post = std::move(post);
  job->commit_method = cfg.commit_method;
  job->committer = committer;
  job->resolve = std::move(resolve);
  if (readahead) {
    job->readahead = readahead;
    job->ra_key = std::to_string(o.mount_id) + ":" + o.ufs_path;
    job->ra_next = cache;     // a whole-block read-through: a sequential reader's next block follows
  }
  const uint64_t chunk =
      r.chunk_size > 0 ? std::min<uint64_t>((uint64_t)r.chunk_size, max_chunk) : std::min<uint64_t>(1u << 20, max_chunk);
  job->first_bytes = std::min<uint64_t>(chunk, job->slot_bytes);   // the first chunk goes after one small read
  std::unique_ptr<NativeStream> ns(new ColdReadStream(store, job->session, r.block_id, off, end, chunk, window,
                                                      slot_pool->size(), job->first_bytes, unix_peer, st, stats));
  stats->cold_streams.fetch_add(1, std::memory_order_relaxed);
  if (readahead) readahead->begin(r.block_id);
  if (!ColdPool::get().submit([job] { job->run(); }, cfg.max_active)) {
    if (readahead) readahead->end(r.block_id);
    stats->cold_active.fetch_sub(1, std::memory_order_relaxed);
    *status = 8;
    *msg = "cannot start a UFS reader thread";
    return nullptr;
  }
  return ns;
}

}  // namespace

// ---- native block commit ------------------------------------------------------------------------

// How long an append hold keeps a CACHE_THROUGH block from eviction when no AppendBlock comes.
constexpr int64_t kAppendHoldMs = 120000;

CommitTicket::~CommitTicket() {
  if (done) (void)hipEventDestroy(done);
}

struct BlockCommitter::State {
  StoreRef store;
  uint32_t method = UINT32_MAX;
  std::shared_ptr<DataServerStats> stats;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::shared_ptr<CommitTicket>> q;
  bool stop = false;
  Caller caller;
  struct CrcBuf {
    uint32_t* dev = nullptr;
    uint32_t* host = nullptr;
    size_t words = 0;
  };
  std::vector<CrcBuf> free_crc;       // device + pinned CRC buffers, reused across tickets
  ~State() {
    for (auto& b : free_crc) {
      if (b.dev) (void)hipFree(b.dev);
      if (b.host) (void)hipHostFree(b.host);
    }
  }
};

BlockCommitter::BlockCommitter(StoreRef store, uint32_t method, bool crc_device, bool crc_host,
                               std::shared_ptr<DataServerStats> stats)
    : st_(std::make_shared<State>()), crc_device_(crc_device), crc_host_(crc_host) {
  st_->store = std::move(store);
  st_->method = method;
  st_->stats = std::move(stats);
  auto st = st_;
  // detached: it holds the state (and so the store) until its queue is drained after the stop
  std::thread([st] { BlockCommitter::run(st); }).detach();
}

BlockCommitter::~BlockCommitter() {
  {
    std::lock_guard<std::mutex> g(st_->mu);
    st_->stop = true;
  }
  st_->cv.notify_all();
}

void BlockCommitter::set_caller(Caller c) {
  std::lock_guard<std::mutex> g(st_->mu);
  if (!st_->caller) st_->caller = std::move(c);
}

bool BlockCommitter::has_caller() {
  std::lock_guard<std::mutex> g(st_->mu);
  return (bool)st_->caller;
}

void BlockCommitter::submit(std::shared_ptr<CommitTicket> t) {
  {
    std::lock_guard<std::mutex> g(st_->mu);
    st_->q.push_back(std::move(t));
  }
  st_->cv.notify_one();
}

bool BlockCommitter::take_crc_buffer(size_t words, CommitTicket* t) {
  State::CrcBuf b;
  {
    std::lock_guard<std::mutex> g(st_->mu);
    for (size_t i = 0; i < st_->free_crc.size(); ++i)
      if (st_->free_crc[i].words >= words) {
        b = st_->free_crc[i];
        st_->free_crc.erase(st_->free_crc.begin() + (long)i);
        break;
      }
  }
  if (!b.dev) {
    words = std::max<size_t>(words, 4096);   // one size fits the usual blocks: buffers get reused
    st_->store->use_device();
    if (hipMalloc((void**)&b.dev, words * sizeof(uint32_t)) != hipSuccess) return false;
    if (hipHostMalloc((void**)&b.host, words * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess) {
      (void)hipFree(b.dev);
      return false;
    }
    b.words = words;
  }
  t->crc_dev = b.dev;
  t->crc_host = b.host;
  t->crc_words = b.words;
  return true;
}

namespace {
void put_key_varint(std::string& m, uint32_t field, uint64_t v) {
  h2::put_varint(m, (uint64_t)field << 3);
  h2::put_varint(m, v);
}

// NativeCommitBatchResponse (proto/defs/block.py): failed=1:i64* message=2:str
void parse_commit_reply(const std::string& b, std::vector<int64_t>* failed, std::string* msg) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(b.data());
  const size_t n = b.size();
  size_t i = 0;
  while (i < n) {
    uint64_t key;
    if (!h2::get_varint(p, n, &i, &key)) return;
    const uint32_t field = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
    if (field == 1 && wt == 0) {
      uint64_t v;
      if (!h2::get_varint(p, n, &i, &v)) return;
      failed->push_back((int64_t)v);
    } else if (field == 1 && wt == 2) {            // packed
      uint64_t len;
      if (!h2::get_varint(p, n, &i, &len) || len > n - i) return;
      const size_t end = i + (size_t)len;
      while (i < end) {
        uint64_t v;
        if (!h2::get_varint(p, end, &i, &v)) return;
        failed->push_back((int64_t)v);
      }
    } else if (field == 2 && wt == 2) {
      uint64_t len;
      if (!h2::get_varint(p, n, &i, &len) || len > n - i) return;
      msg->assign(b.data() + i, (size_t)len);
      i += (size_t)len;
    } else if (!skip_field(p, n, &i, wt)) {
      return;
    }
  }
}
}  // namespace

void BlockCommitter::run(std::shared_ptr<State> st) {
  pthread_setname_np(pthread_self(), "block-commit");
  const StoreRef& store = st->store;
  if (store->has_device()) store->use_device();
  for (;;) {
    std::vector<std::shared_ptr<CommitTicket>> batch;
    Caller caller;
    {
      std::unique_lock<std::mutex> lk(st->mu);
      st->cv.wait(lk, [&] { return st->stop || !st->q.empty(); });
      if (st->q.empty()) break;                   // stopped and drained
      while (!st->q.empty() && batch.size() < 1024) {
        batch.push_back(std::move(st->q.front()));
        st->q.pop_front();
      }
      caller = st->caller;
    }
    struct Item {
      std::shared_ptr<CommitTicket> t;
      int status = 0;
      std::string msg;
      int64_t lock = -1;
      std::string crc;                            // little-endian u32 per page
      uint64_t piece = 0;
    };
    std::vector<Item> items(batch.size());
    // 1) the device work of every block (H2D, CRC kernel, CRC D2H), then the store commit
    for (size_t i = 0; i < batch.size(); ++i) {
      Item& it = items[i];
      it.t = batch[i];
      CommitTicket& t = *it.t;
      if (t.done && hipEventSynchronize(t.done) != hipSuccess) {
        it.status = 13;
        it.msg = "writing block " + std::to_string(t.block) + ": a device copy into the block failed";
      }
      if (!it.status && t.crc_pages && t.crc_host) {
        it.crc.assign(reinterpret_cast<const char*>(t.crc_host), t.crc_pages * sizeof(uint32_t));
        it.piece = t.crc_page;
        st->stats->crc_streamed.fetch_add(1, std::memory_order_relaxed);
      }
      if (t.crc_dev) {                            // the buffer goes back to the pool
        std::lock_guard<std::mutex> g(st->mu);
        st->free_crc.push_back(State::CrcBuf{t.crc_dev, t.crc_host, t.crc_words});
        t.crc_dev = nullptr;
        t.crc_host = nullptr;
      }
      if (it.status) continue;
      try {
        if (t.crc_sync) {                         // no streamed CRCs: compute them here
          int dir = -1;
          uint64_t ps = 0, base = 0;
          store->block_pages(t.block, &dir, &ps, &base);
          const std::vector<uint32_t> c = store->checksum(t.block, 0);
          it.crc.assign(reinterpret_cast<const char*>(c.data()), c.size() * sizeof(uint32_t));
          it.piece = store->dir_spec(dir).kind == DirKind::kFile ? (2ull << 20) : ps;
        }
        store->commit_block(t.session, t.block, t.pin);
        // held until the master knows (DefaultBlockWorker.commitBlockLocked): never evicted between
        it.lock = store->lock_block(t.session, t.block, false, 0);
      } catch (const StoreError& e) {
        it.status = grpc_status_of(e);
        it.msg = "committing block " + std::to_string(t.block) + ": " + e.what();
      } catch (const std::exception& e) {
        it.status = 13;
        it.msg = "committing block " + std::to_string(t.block) + ": " + e.what();
      }
    }
    // 2) one master report for every block committed above
    std::string req;
    size_t ncommitted = 0;
    for (const Item& it : items) {
      if (it.status) continue;
      ++ncommitted;
      put_key_varint(req, 1, (uint64_t)it.t->block);
      put_key_varint(req, 2, it.t->length);
      put_key_varint(req, 3, it.piece);
      h2::put_varint(req, (4u << 3) | 2);
      h2::put_varint(req, it.crc.size());
      req += it.crc;
      put_key_varint(req, 5, it.t->ufs_read ? 1 : 0);
    }
    int rstatus = 0;
    std::string rmsg;
    std::vector<int64_t> failed;
    if (ncommitted) {
      if (!caller) {
        rstatus = 14;
        rmsg = "the data server cannot reach its worker process";
      } else {
        struct Reply {
          std::mutex mu;
          std::condition_variable cv;
          bool got = false;
          int status = 0;
          std::string msg, payload;
        };
        auto rep = std::make_shared<Reply>();
        caller(st->method, std::move(req), [rep](int status, const std::string& msg, const std::string& payload) {
          std::lock_guard<std::mutex> g(rep->mu);
          rep->got = true;
          rep->status = status;
          rep->msg = msg;
          rep->payload = payload;
          rep->cv.notify_all();
        });
        std::unique_lock<std::mutex> lk(rep->mu);
        if (!rep->cv.wait_for(lk, std::chrono::minutes(10), [&] { return rep->got; })) {
          rstatus = 4;
          rmsg = "the worker did not answer the block commit report in 10 minutes";
        } else {
          rstatus = rep->status;
          rmsg = rep->msg;
          if (!rstatus) parse_commit_reply(rep->payload, &failed, &rmsg);
        }
      }
      st->stats->commit_batches.fetch_add(1, std::memory_order_relaxed);
    }
    // 3) finish: a block the master does not know about does not stay
    for (Item& it : items) {
      CommitTicket& t = *it.t;
      if (!it.status && (rstatus || std::find(failed.begin(), failed.end(), t.block) != failed.end())) {
        it.status = rstatus ? (rstatus == 4 ? 4 : 14) : 14;
        it.msg = "block " + std::to_string(t.block) + " committed locally but the master was not told: " +
                 (rmsg.empty() ? std::string("report failed") : rmsg);
      }
      if (!it.status && t.hold) store->hold_block(t.block, kAppendHoldMs);   // before our lock goes
      try {
        if (it.lock >= 0) store->unlock(it.lock);
      } catch (...) {
      }
      if (it.status && it.lock >= 0) {
        try {
          store->remove_block(t.session, t.block);
        } catch (...) {
        }
      }
      try {
        store->cleanup_session(t.session);       // aborts a temp block that never got committed
      } catch (...) {
      }
      if (it.status) st->stats->commit_failures.fetch_add(1, std::memory_order_relaxed);
      else st->stats->commits.fetch_add(1, std::memory_order_relaxed);
      std::function<void()> w;
      {
        std::lock_guard<std::mutex> g(t.mu);
        t.finished = true;
        t.status = it.status;
        t.msg = it.msg;
        w = t.wake;
      }
      if (w) w();
    }
  }
}

namespace {

// The stream of a block the store holds: locked (no wait) for the call's lifetime; nullptr with
// *status == 0 when it is not (yet) committed here, with *status != 0 on a bad request.
std::unique_ptr<BlockReadStream> open_block_stream(const ReadRequestMsg& r, const StoreRef& store, uint64_t max_chunk,
                                                   uint64_t window, bool unix_peer,
                                                   const std::shared_ptr<StagingPool>& pool,
                                                   const std::shared_ptr<DataServerStats>& stats, int* status,
                                                   std::string* msg) {
  const int64_t session = g_session.fetch_add(1);
  int64_t lock = -1;
  try {
    lock = store->lock_block(session, r.block_id, false, 0);
  } catch (const StoreError& e) {
    lock = -1;   // not (yet) committed here
  }
  if (lock < 0) return nullptr;
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
    const uint64_t chunk = r.chunk_size > 0 ? std::min<uint64_t>((uint64_t)r.chunk_size, max_chunk)
                                            : std::min<uint64_t>(1u << 20, max_chunk);
    const bool device = store->dir_spec(info.dir).kind == DirKind::kDevice;
    store->access_block(session, r.block_id);
    stats->streams.fetch_add(1, std::memory_order_relaxed);
    return std::unique_ptr<BlockReadStream>(new BlockReadStream(store, session, lock, r.block_id, off, end, chunk,
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
}

// ReadBlock with promote = true (CACHE_PROMOTE) of a block below the top tier: the block moves to
// tier 0 first -- on a pool thread, with the batched copy kernel for device tiers -- and is then
// streamed from there; a failed move (no room, locked by a reader) streams it where it is
// (reference BlockReadHandler.openBlock:159-175 moves, logs a failure and reads).
class PromoteReadStream : public NativeStream {
 public:
  struct Move {
    std::mutex mu;
    bool done = false;
    std::function<void()> wake;
  };
  PromoteReadStream(ReadRequestMsg r, StoreRef store, uint64_t max_chunk, uint64_t window, bool unix_peer,
                    std::shared_ptr<StagingPool> pool, std::shared_ptr<DataServerStats> stats, std::shared_ptr<Move> mv)
      : r_(std::move(r)), store_(std::move(store)), max_chunk_(max_chunk), window_(window), unix_(unix_peer),
        pool_(std::move(pool)), stats_(std::move(stats)), mv_(std::move(mv)) {}
  ~PromoteReadStream() override {
    std::lock_guard<std::mutex> g(mv_->mu);
    mv_->wake = nullptr;
  }
  void set_waker(std::function<void()> w) override {
    waker_ = w;
    bool done;
    {
      std::lock_guard<std::mutex> g(mv_->mu);
      mv_->wake = w;
      done = mv_->done;
    }
    if (done && w) w();
  }
  void on_message(const char* p, size_t n) override {
    if (inner_) inner_->on_message(p, n);
  }
  ssize_t produce(uint8_t* dst, size_t max, bool* eof, int* status, std::string* msg) override {
    if (!ready(status, msg)) return *status ? -1 : 0;
    return inner_->produce(dst, max, eof, status, msg);
  }
  ssize_t produce_spans(size_t max, ByteSpan* spans, int max_spans, int* nspans, bool* eof, int* status,
                        std::string* msg) override {
    if (!inner_) return -2;
    return inner_->produce_spans(max, spans, max_spans, nspans, eof, status, msg);
  }

 private:
  bool ready(int* status, std::string* msg) {
    if (inner_) return true;
    {
      std::lock_guard<std::mutex> g(mv_->mu);
      if (!mv_->done) return false;
    }
    int st = 0;
    std::string m;
    inner_ = open_block_stream(r_, store_, max_chunk_, window_, unix_, pool_, stats_, &st, &m);
    if (!inner_) {
      *status = st ? st : 5;
      *msg = st ? m : "block " + std::to_string(r_.block_id) + " does not exist on this worker";
      return false;
    }
    if (waker_) inner_->set_waker(waker_);
    return true;
  }
  ReadRequestMsg r_;
  StoreRef store_;
  uint64_t max_chunk_, window_;
  bool unix_;
  std::shared_ptr<StagingPool> pool_;
  std::shared_ptr<DataServerStats> stats_;
  std::shared_ptr<Move> mv_;
  std::unique_ptr<BlockReadStream> inner_;
  std::function<void()> waker_;
};

}  // namespace

void serve_block_reads(FrameRpcServer& srv, uint32_t method, StoreRef store, uint64_t max_chunk, uint64_t window,
                       std::shared_ptr<DataServerStats> stats, std::shared_ptr<UfsMounts> mounts, ColdReadConfig cold,
                       std::shared_ptr<BlockCommitter> committer) {
  if (max_chunk == 0) max_chunk = 2u << 20;
  if (window == 0) window = 4u << 20;
  if (cold.slot_bytes == 0) cold.slot_bytes = 8u << 20;
  auto pool = std::make_shared<StagingPool>(max_chunk, store->has_device(), store->device());
  auto slot_pool = std::make_shared<StagingPool>(cold.slot_bytes, store->has_device(), store->device());
  auto readahead = cold.readahead ? std::make_shared<ColdReadAhead>() : nullptr;
  FrameRpcServer* s = &srv;
  srv.set_native_stream(method, [=](const std::string& first, const std::string& cid, const std::string& user,
                                    bool unix_peer, int* status, std::string* msg) -> std::unique_ptr<NativeStream> {
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
    if (r.offset < 0) {
      stats->declined.fetch_add(1, std::memory_order_relaxed);
      return nullptr;
    }
    if (r.promote) {
      bool below_top = false;
      try {
        below_top = store->has_block(r.block_id) && store->block_info(r.block_id).tier > 0;
      } catch (...) {
      }
      if (below_top) {
        auto mv = std::make_shared<PromoteReadStream::Move>();
        const int64_t session = g_session.fetch_add(1), id = r.block_id;
        auto st = store;
        auto sts = stats;
        if (ColdPool::get().submit([st, sts, session, id, mv] {
              try {
                st->move_block(session, id, 0, "", true);
                sts->promoted.fetch_add(1, std::memory_order_relaxed);
              } catch (...) {              // no room / locked / gone: read it where it is
              }
              try {
                st->cleanup_session(session);
              } catch (...) {
              }
              std::function<void()> w;
              {
                std::lock_guard<std::mutex> g(mv->mu);
                mv->done = true;
                w = mv->wake;
              }
              if (w) w();
            }, 64))
          return std::unique_ptr<NativeStream>(
              new PromoteReadStream(r, store, max_chunk, window, unix_peer, pool, stats, mv));
      }
    }
    auto bs = open_block_stream(r, store, max_chunk, window, unix_peer, pool, stats, status, msg);
    if (bs) return bs;
    if (*status != 0) return nullptr;
    if (r.has_ufs) {     // a cold block: read it through from the UFS (BlockReadHandler.openUfsBlock)
      if (committer && !committer->has_caller()) committer->set_caller(s->internal_caller(cid, user));
      auto cs = make_cold_stream(r, store, max_chunk, window, unix_peer, cold, mounts, slot_pool, stats,
                                 s->internal_poster(cid, user), status, msg, committer,
                                 cold.resolve_method != UINT32_MAX ? s->internal_caller(cid, user) : nullptr,
                                 readahead);
      if (cs || *status != 0) return cs;
    }
    stats->declined.fetch_add(1, std::memory_order_relaxed);
    return nullptr;
  });
}

void serve_block_writes(FrameRpcServer& srv, uint32_t method, uint32_t commit_method, StoreRef store,
                        uint64_t stage_bytes, std::shared_ptr<DataServerStats> stats,
                        std::shared_ptr<UfsMounts> ufs_roots, std::shared_ptr<BlockCommitter> committer) {
  if (stage_bytes == 0) stage_bytes = 4u << 20;
  auto pool = std::make_shared<StagingPool>(stage_bytes, store->has_device(), store->device());
  FrameRpcServer* s = &srv;
  srv.set_native_stream(method, [=](const std::string& first, const std::string& cid, const std::string& user,
                                    bool unix_peer, int* status, std::string* msg) -> std::unique_ptr<NativeStream> {
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
    std::string local, key;
    std::shared_ptr<const S3Mount> s3;
    if (cmd.type == 1 && cmd.has_ufs_file && ufs_roots && ufs_roots->resolve_s3(cmd.ufs_mount, cmd.ufs_path, &s3, &key)) {
      auto ws = std::unique_ptr<S3UfsWriteStream>(new S3UfsWriteStream(std::move(s3), key, stats, store));
      stats->ufs_write_streams.fetch_add(1, std::memory_order_relaxed);
      if (len) ws->on_message(first.data(), first.size());
      return ws;
    }
    if (cmd.type == 1 && cmd.has_ufs_file && ufs_roots && ufs_roots->resolve(cmd.ufs_mount, cmd.ufs_path, &local)) {
      auto us = std::unique_ptr<UfsFileWriteStream>(
          new UfsFileWriteStream(local, cmd.ufs_mode > 0 ? (int)(cmd.ufs_mode & 07777) : 0644, stats, store));
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
      // evict = false: the I/O thread never waits for space (eviction can block on locks and run
      // demotion copies); a write that needs eviction goes to the Python servicer, which may wait
      int dir;
      const int tier = cmd.medium.empty() ? (cmd.has_tier ? (int)cmd.tier : 0) : -1;
      try {
        dir = store->create_block(session, cmd.id, tier, cmd.medium, reserve, false, cmd.pin);
      } catch (const StoreError& e) {
        if (e.code != kErrOutOfSpace) throw;
        // no space without evicting: the eviction runs on a pool thread while this stream queues
        // what arrives (the I/O thread never waits for space, and nothing goes to Python)
        auto pc = std::make_shared<PendingCreate>();
        const WriteCmd c = cmd;
        auto ok = ColdPool::get().submit([store, session, c, tier, reserve, pc] {
          int d = -1, st = 0;
          std::string m;
          try {
            d = store->create_block(session, c.id, tier, c.medium, reserve, true, c.pin);
          } catch (const StoreError& e) {
            st = grpc_status_of(e);
            m = e.what();
          } catch (const std::exception& e) {
            st = 13;
            m = e.what();
          }
          std::function<void()> w;
          bool cancelled;
          {
            std::lock_guard<std::mutex> g(pc->mu);
            pc->done = true;
            pc->status = st;
            pc->msg = m;
            pc->dir = d;
            cancelled = pc->cancelled;
            w = pc->wake;
          }
          if (cancelled) {
            try {
              store->cleanup_session(session);
            } catch (...) {
            }
          } else if (w) {
            w();
          }
        }, 64);
        if (!ok) {
          try {
            store->cleanup_session(session);
          } catch (...) {
          }
          stats->write_declined.fetch_add(1, std::memory_order_relaxed);
          return nullptr;
        }
        if (committer && !committer->has_caller()) committer->set_caller(s->internal_caller(cid, user));
        auto ws = std::unique_ptr<BlockWriteStream>(new BlockWriteStream(
            store, session, cmd.id, (uint64_t)cmd.offset, cmd.pin, false, commit_method, pool, stats, committer, pc));
        stats->write_streams.fetch_add(1, std::memory_order_relaxed);
        stats->write_evict_waits.fetch_add(1, std::memory_order_relaxed);
        if (len) ws->on_message(first.data(), first.size());
        return ws;
      }
      const bool device = store->dir_spec(dir).kind == DirKind::kDevice;
      if (committer && !committer->has_caller()) committer->set_caller(s->internal_caller(cid, user));
      auto ws = std::unique_ptr<BlockWriteStream>(new BlockWriteStream(store, session, cmd.id, (uint64_t)cmd.offset,
                                                                       cmd.pin, device, commit_method, pool, stats,
                                                                       committer));
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
