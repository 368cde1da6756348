// Host-reader block sources and the chunk-buffered input stream (see block_source.h).
#include "block_source.h"
#include "numa_host.h"

#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <pthread.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <cstdlib>
#include <functional>
#include <map>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "h2_abi.h"

namespace amdx {

namespace {

// ---- pinned chunk buffers: pooled per size (hipHostMalloc costs far more than a refill) -------
std::mutex g_buf_mu;
std::multimap<uint64_t, uint8_t*> g_buf_free;   // size -> pinned buffer
size_t g_buf_free_bytes = 0;
constexpr size_t kBufPoolCap = 1ull << 30;

bool have_device() {
  static const bool yes = [] {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess && n > 0;
  }();
  return yes;
}

// D2H copies of host readers: a few non-blocking streams per device shared round-robin by the
// reading threads, each thread waiting on its own event (not on the whole stream).
struct DevCtx {
  std::vector<hipStream_t> streams;
};
hipStream_t reader_stream(int device) {
  static std::mutex mu;
  static std::map<int, DevCtx> ctx;
  thread_local int last_dev = -1;
  thread_local size_t slot = std::hash<std::thread::id>{}(std::this_thread::get_id());
  if (last_dev != device) {
    if (hipSetDevice(device) != hipSuccess) throw StoreError(kErrHip, "hipSetDevice failed");
    last_dev = device;
  }
  std::lock_guard<std::mutex> g(mu);
  DevCtx& c = ctx[device];
  if (c.streams.empty()) {
    // ALLUXIO_READER_STREAMS: streams per device (default 8; a process maps them onto at most
    // GPU_MAX_HW_QUEUES hardware queues)
    static const int nstreams = [] {
      const char* e = getenv("ALLUXIO_READER_STREAMS");
      const int v = e ? atoi(e) : 8;
      return v < 1 ? 1 : (v > 64 ? 64 : v);
    }();
    for (int i = 0; i < nstreams; ++i) {
      hipStream_t s = nullptr;
      if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
        throw StoreError(kErrHip, "hipStreamCreate failed");
      c.streams.push_back(s);
    }
  }
  return c.streams[slot % c.streams.size()];
}

void wait_stream(hipStream_t st) {
  thread_local hipEvent_t ev = nullptr;
  thread_local int ev_dev = -1;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (!ev || ev_dev != dev) {
    if (ev) (void)hipEventDestroy(ev);
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventBlockingSync) != hipSuccess)
      throw StoreError(kErrHip, "hipEventCreate failed");
    ev_dev = dev;
  }
  hipError_t e = hipEventRecord(ev, st);
  if (e == hipSuccess) e = hipEventSynchronize(ev);
  if (e != hipSuccess) throw StoreError(kErrHip, std::string("D2H copy failed: ") + hipGetErrorString(e));
}

// Copy segments of a paged block: (page-run address, bytes) for [off, off + n).
template <class Fn>
void for_page_runs(uint64_t base, const std::vector<int64_t>& pages, uint64_t ps, uint64_t off, uint64_t n, Fn fn) {
  uint64_t done = 0;
  while (done < n) {
    const uint64_t pos = off + done;
    const size_t pi = (size_t)(pos / ps);
    if (pi >= pages.size()) throw StoreError(kErrInvalidArgument, "read beyond the block's pages");
    size_t pj = pi + 1;
    while (pj < pages.size() && pages[pj] == pages[pj - 1] + 1) ++pj;
    const uint64_t in_page = pos % ps;
    const uint64_t take = std::min<uint64_t>((uint64_t)(pj - pi) * ps - in_page, n - done);
    fn(base + (uint64_t)pages[pi] * ps + in_page, done, take);
    done += take;
  }
}

}  // namespace

uint8_t* host_buffer_alloc(uint64_t n, bool* pinned) {
  {
    std::lock_guard<std::mutex> g(g_buf_mu);
    auto it = g_buf_free.find(n);
    if (it != g_buf_free.end()) {
      uint8_t* p = it->second;
      g_buf_free.erase(it);
      g_buf_free_bytes -= n;
      *pinned = true;
      return p;
    }
  }
  void* p = nullptr;
  if (have_device()) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    p = pinned_alloc_near(n, dev);          // on the NUMA node of the device that DMAs into it
    if (p) {
      *pinned = true;
      return static_cast<uint8_t*>(p);
    }
  }
  *pinned = false;
  p = std::malloc(n ? n : 1);
  if (!p) throw StoreError(kErrOutOfSpace, "cannot allocate a read buffer");
  return static_cast<uint8_t*>(p);
}

void host_buffer_release(uint8_t* p, uint64_t n, bool pinned) {
  if (!p) return;
  if (pinned) {
    {
      std::lock_guard<std::mutex> g(g_buf_mu);
      if (g_buf_free_bytes + n <= kBufPoolCap) {
        g_buf_free.emplace(n, p);
        g_buf_free_bytes += n;
        return;
      }
    }
    (void)hipHostFree(p);
    return;
  }
  std::free(p);
}

// ---- DeviceArenaSource ------------------------------------------------------------------------
DeviceArenaSource::DeviceArenaSource(uint64_t base, std::vector<int64_t> pages, uint64_t page_size, uint64_t length,
                                     int device)
    : BlockSource(length), base_(base), pages_(std::move(pages)), page_size_(page_size), device_(device) {
  if (page_size_ == 0) throw StoreError(kErrInvalidArgument, "page size must be > 0");
  if (length_ > (uint64_t)pages_.size() * page_size_) throw StoreError(kErrInvalidArgument, "block longer than its pages");
}

void DeviceArenaSource::read(uint64_t off, uint64_t n, uint8_t* dst) {
  if (off + n > length_) throw StoreError(kErrInvalidArgument, "read beyond the block");
  hipStream_t st = reader_stream(device_);
  for_page_runs(base_, pages_, page_size_, off, n, [&](uint64_t src, uint64_t at, uint64_t take) {
    const hipError_t e = hipMemcpyAsync(dst + at, reinterpret_cast<const void*>(src), take, hipMemcpyDeviceToHost, st);
    if (e != hipSuccess) throw StoreError(kErrHip, std::string("hipMemcpyAsync D2H: ") + hipGetErrorString(e));
  });
  wait_stream(st);
}

// ---- ArenaSink ----------------------------------------------------------------------------------
ArenaSink::ArenaSink(uint64_t base, std::vector<int64_t> pages, uint64_t page_size, uint64_t capacity, int device,
                     bool host_arena)
    : base_(base), pages_(std::move(pages)), page_size_(page_size), capacity_(capacity), device_(device),
      host_(host_arena) {
  if (page_size_ == 0) throw StoreError(kErrInvalidArgument, "page size must be > 0");
  if (capacity_ > (uint64_t)pages_.size() * page_size_)
    throw StoreError(kErrInvalidArgument, "write capacity beyond the block's pages");
  if (!host_) {
    for (int i = 0; i < 2; ++i) {
      stage_[i] = host_buffer_alloc(kStage, &pinned_[i]);
      if (hipEventCreateWithFlags(&ev_[i], hipEventDisableTiming | hipEventBlockingSync) != hipSuccess)
        throw StoreError(kErrHip, "hipEventCreate failed");
    }
  }
}

ArenaSink::~ArenaSink() {
  for (int i = 0; i < 2; ++i) {
    if (ev_[i]) {
      (void)hipEventSynchronize(ev_[i]);
      (void)hipEventDestroy(ev_[i]);
    }
    if (stage_[i]) host_buffer_release(stage_[i], kStage, pinned_[i]);
  }
}

void ArenaSink::write(uint64_t off, const uint8_t* src, uint64_t n) {
  if (off + n > capacity_) throw StoreError(kErrOutOfSpace, "write beyond the reserved block");
  if (host_) {
    for_page_runs(base_, pages_, page_size_, off, n, [&](uint64_t dst, uint64_t at, uint64_t take) {
      std::memcpy(reinterpret_cast<void*>(dst), src + at, take);
    });
  } else {
    hipStream_t st = reader_stream(device_);
    uint64_t done = 0;
    int k = 0;
    while (done < n) {
      const uint64_t take = std::min<uint64_t>(kStage, n - done);
      // the buffer's previous DMA must be done before it is overwritten
      if (hipEventSynchronize(ev_[k]) != hipSuccess) throw StoreError(kErrHip, "hipEventSynchronize failed");
      std::memcpy(stage_[k], src + done, take);
      const uint8_t* sp = stage_[k];
      for_page_runs(base_, pages_, page_size_, off + done, take, [&](uint64_t dst, uint64_t at, uint64_t t) {
        const hipError_t e = hipMemcpyAsync(reinterpret_cast<void*>(dst), sp + at, t, hipMemcpyHostToDevice, st);
        if (e != hipSuccess) throw StoreError(kErrHip, std::string("hipMemcpyAsync H2D: ") + hipGetErrorString(e));
      });
      if (hipEventRecord(ev_[k], st) != hipSuccess) throw StoreError(kErrHip, "hipEventRecord failed");
      done += take;
      k ^= 1;
    }
    wait_stream(st);
  }
  length_ = std::max(length_, off + n);
}

// ---- reads into device memory ------------------------------------------------------------------
void source_read_to_device(BlockSource& src, uint64_t off, uint64_t n, uint8_t* dptr, int device) {
  constexpr uint64_t kStage = 4u << 20;
  struct Buf {
    uint8_t* p = nullptr;
    bool pinned = false;
    hipEvent_t ev = nullptr;
  } b[2];
  struct Cleanup {
    Buf* b;
    ~Cleanup() {
      for (int i = 0; i < 2; ++i) {
        if (b[i].ev) {
          (void)hipEventSynchronize(b[i].ev);
          (void)hipEventDestroy(b[i].ev);
        }
        if (b[i].p) host_buffer_release(b[i].p, kStage, b[i].pinned);
      }
    }
  } cleanup{b};
  hipStream_t st = reader_stream(device);
  for (int i = 0; i < 2; ++i) {
    b[i].p = host_buffer_alloc(kStage, &b[i].pinned);
    if (hipEventCreateWithFlags(&b[i].ev, hipEventDisableTiming | hipEventBlockingSync) != hipSuccess)
      throw StoreError(kErrHip, "hipEventCreate failed");
  }
  uint64_t done = 0;
  int k = 0;
  while (done < n) {
    const uint64_t take = std::min<uint64_t>(kStage, n - done);
    if (hipEventSynchronize(b[k].ev) != hipSuccess) throw StoreError(kErrHip, "hipEventSynchronize failed");
    src.read(off + done, take, b[k].p);            // network / arena bytes into pinned memory
    const hipError_t e = hipMemcpyAsync(dptr + done, b[k].p, take, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) throw StoreError(kErrHip, std::string("hipMemcpyAsync H2D: ") + hipGetErrorString(e));
    if (hipEventRecord(b[k].ev, st) != hipSuccess) throw StoreError(kErrHip, "hipEventRecord failed");
    done += take;
    k ^= 1;
  }
  wait_stream(st);
}

// ---- HostArenaSource --------------------------------------------------------------------------
HostArenaSource::HostArenaSource(uint64_t base, std::vector<int64_t> pages, uint64_t page_size, uint64_t length)
    : BlockSource(length), base_(base), pages_(std::move(pages)), page_size_(page_size) {
  if (page_size_ == 0) throw StoreError(kErrInvalidArgument, "page size must be > 0");
  if (length_ > (uint64_t)pages_.size() * page_size_) throw StoreError(kErrInvalidArgument, "block longer than its pages");
}

void HostArenaSource::read(uint64_t off, uint64_t n, uint8_t* dst) {
  if (off + n > length_) throw StoreError(kErrInvalidArgument, "read beyond the block");
  for_page_runs(base_, pages_, page_size_, off, n, [&](uint64_t src, uint64_t at, uint64_t take) {
    std::memcpy(dst + at, reinterpret_cast<const void*>(src), take);
  });
}

// ---- StoreSource ------------------------------------------------------------------------------
StoreSource::StoreSource(BlockStore* store, int64_t block_id, uint64_t length, bool device_tier)
    : BlockSource(length), store_(store), block_(block_id), device_(device_tier) {}

void StoreSource::read(uint64_t off, uint64_t n, uint8_t* dst) {
  std::vector<ReadReq> rq{ReadReq{block_, off, n, reinterpret_cast<uint64_t>(dst), (int)MemKind::kHost}};
  if (!device_) {
    store_->read_batch(rq, 0, false);
  } else {
    hipStream_t st = reader_stream(store_->device());
    store_->read_batch(rq, reinterpret_cast<uint64_t>(st), false);
    wait_stream(st);
  }
  bytes_.fetch_add(n, std::memory_order_relaxed);
}

// ---- GrpcBlockSource: ReadBlock over HTTP/2 ---------------------------------------------------
struct GrpcBlockSource::Conn {
  int fd = -1;
  void* ng = nullptr;
  int32_t sid = -1;
  std::string authority;
  // request body (first ReadRequest, then offset_received acks)
  std::string outq;
  size_t outq_off = 0;
  // response parsing: gRPC prefix -> ReadResponse{chunk{data}} -> data bytes
  int state = 0;                  // 0 prefix, 1 message header, 2 data, 3 skip, 4 slow (whole message)
  uint8_t pfx[5];
  size_t pfx_n = 0;
  uint64_t msg_left = 0, data_left = 0;
  std::string mh;                 // message header bytes / slow-path message
  // destination of parsed data
  uint8_t* dst = nullptr;
  uint64_t need = 0;
  std::string spill;              // parsed bytes beyond the current request
  size_t spill_off = 0;
  uint64_t pos = 0;               // block offset of the next byte handed out
  uint64_t acked = 0;
  uint64_t ack_every = 1u << 20;
  bool closed = false, headers_ok = false;
  int grpc_status = -1;
  std::string grpc_msg;
  uint32_t close_code = 0;
  std::string inbuf;
  // Raw HTTP/2 frame boundaries of the server->client byte stream, tracked alongside nghttp2 so
  // the chunk bytes of our DATA frames can be received straight into the caller's buffer (one
  // copy, the kernel's) instead of into inbuf and then memcpy'd.  nghttp2 still parses every byte
  // (flow control, headers, trailers): it is handed the same bytes where they landed.
  uint8_t fh[9];
  size_t fh_n = 0;
  uint64_t frame_left = 0;
  bool in_payload = false, our_data = false;
  uint64_t direct_bytes = 0;

  ~Conn() {
    if (ng) h2::lib().session_del(ng);
    if (fd >= 0) ::close(fd);
  }

  void track(const uint8_t* p, size_t n) {
    while (n) {
      if (!in_payload) {
        const size_t t = std::min(n, 9 - fh_n);
        std::memcpy(fh + fh_n, p, t);
        fh_n += t;
        p += t;
        n -= t;
        if (fh_n < 9) break;
        fh_n = 0;
        frame_left = ((uint64_t)fh[0] << 16) | ((uint64_t)fh[1] << 8) | fh[2];
        const int32_t id = (int32_t)((((uint32_t)fh[5] & 0x7f) << 24) | ((uint32_t)fh[6] << 16) |
                                     ((uint32_t)fh[7] << 8) | fh[8]);
        our_data = fh[3] == h2::kTypeData && id == sid && !(fh[4] & 0x08);   // not PADDED
        in_payload = frame_left > 0;
      } else {
        const size_t t = (size_t)std::min<uint64_t>(n, frame_left);
        frame_left -= t;
        p += t;
        n -= t;
        if (!frame_left) in_payload = false;
      }
    }
  }

  void deliver(const uint8_t* p, size_t n) {
    const size_t take = (size_t)std::min<uint64_t>(n, need);
    if (take) {
      if (p != dst) std::memcpy(dst, p, take);   // == dst: received there directly
      dst += take;
      need -= take;
    }
    if (take < n) {
      if (spill_off == spill.size()) {
        spill.clear();
        spill_off = 0;
      }
      spill.append(reinterpret_cast<const char*>(p) + take, n - take);
    }
  }

  // Generic decode of one whole ReadResponse (any field order / extra fields).
  bool slow_message(const std::string& m) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(m.data());
    size_t i = 0, n = m.size();
    while (i < n) {
      uint64_t key, len;
      if (!h2::get_varint(p, n, &i, &key)) return false;
      if ((key & 7) != 2) {
        uint64_t v;
        if ((key & 7) != 0 || !h2::get_varint(p, n, &i, &v)) return false;
        continue;
      }
      if (!h2::get_varint(p, n, &i, &len) || len > n - i) return false;
      if ((key >> 3) == 1) {   // chunk
        size_t j = i, end = i + (size_t)len;
        while (j < end) {
          uint64_t k2, l2;
          if (!h2::get_varint(p, end, &j, &k2)) return false;
          if ((k2 & 7) != 2) {
            uint64_t v;
            if ((k2 & 7) != 0 || !h2::get_varint(p, end, &j, &v)) return false;
            continue;
          }
          if (!h2::get_varint(p, end, &j, &l2) || l2 > end - j) return false;
          if ((k2 >> 3) == 1) deliver(p + j, (size_t)l2);
          j += (size_t)l2;
        }
      }
      i += (size_t)len;
    }
    return true;
  }

  // Feeds DATA bytes of the response; false on a malformed stream.
  bool feed(const uint8_t* p, size_t n) {
    while (n) {
      switch (state) {
        case 0: {
          const size_t t = std::min(n, 5 - pfx_n);
          std::memcpy(pfx + pfx_n, p, t);
          pfx_n += t;
          p += t;
          n -= t;
          if (pfx_n < 5) break;
          pfx_n = 0;
          if (pfx[0] != 0) return false;   // compressed: never requested
          msg_left = ((uint64_t)pfx[1] << 24) | ((uint64_t)pfx[2] << 16) | ((uint64_t)pfx[3] << 8) | pfx[4];
          mh.clear();
          state = msg_left ? 1 : 0;
          break;
        }
        case 1: {   // "0A <len> 0A <len>": collect until both varints parse
          mh.push_back((char)*p++);
          --n;
          --msg_left;
          const uint8_t* q = reinterpret_cast<const uint8_t*>(mh.data());
          if (q[0] != 0x0A) {                       // not the fast layout: whole message
            state = msg_left ? 4 : 0;
            if (!msg_left && !slow_message(mh)) return false;
            break;
          }
          size_t i = 1;
          uint64_t l1, l2;
          if (!h2::get_varint(q, mh.size(), &i, &l1)) {
            if (mh.size() > 12 || !msg_left) return false;
            break;
          }
          if (l1 == 0 && msg_left == 0) {            // empty chunk
            state = 0;
            break;
          }
          if (i == mh.size()) {
            if (!msg_left) return false;
            break;
          }
          if (q[i] != 0x0A || l1 != msg_left + (mh.size() - i)) {   // extra fields: slow path
            state = msg_left ? 4 : 0;
            if (!msg_left && !slow_message(mh)) return false;
            break;
          }
          size_t j = i + 1;
          if (!h2::get_varint(q, mh.size(), &j, &l2)) {
            if (mh.size() > 24 || !msg_left) return false;
            break;
          }
          if (l2 != msg_left) {
            state = msg_left ? 4 : 0;
            if (!msg_left && !slow_message(mh)) return false;
            break;
          }
          data_left = l2;
          state = data_left ? 2 : 0;
          break;
        }
        case 2: {
          const size_t t = (size_t)std::min<uint64_t>(n, data_left);
          deliver(p, t);
          p += t;
          n -= t;
          data_left -= t;
          msg_left -= t;
          if (!data_left) state = 0;
          break;
        }
        case 4: {
          const size_t t = (size_t)std::min<uint64_t>(n, msg_left);
          mh.append(reinterpret_cast<const char*>(p), t);
          p += t;
          n -= t;
          msg_left -= t;
          if (!msg_left) {
            if (!slow_message(mh)) return false;
            state = 0;
          }
          break;
        }
        default:
          return false;
      }
    }
    return true;
  }

  static int on_header(void*, const void* frame, const uint8_t* name, size_t namelen, const uint8_t* value,
                       size_t valuelen, uint8_t, void* ud) {
    Conn& c = *static_cast<Conn*>(ud);
    const h2::FrameHd* hd = static_cast<const h2::FrameHd*>(frame);
    if (hd->stream_id != c.sid) return 0;
    const std::string n(reinterpret_cast<const char*>(name), namelen);
    const std::string v(reinterpret_cast<const char*>(value), valuelen);
    if (n == ":status") c.headers_ok = v == "200";
    else if (n == "grpc-status") c.grpc_status = std::atoi(v.c_str());
    else if (n == "grpc-message") c.grpc_msg = v;
    return 0;
  }
  static int on_data(void*, uint8_t, int32_t sid, const uint8_t* data, size_t len, void* ud) {
    Conn& c = *static_cast<Conn*>(ud);
    if (sid != c.sid) return 0;
    if (!c.feed(data, len)) return h2::kErrCallbackFailure;
    return 0;
  }
  // END_STREAM from the worker (trailers / trailers-only error): the response is complete even
  // though this side never half-closes the request stream.
  static int on_frame(void*, const void* frame, void* ud) {
    Conn& c = *static_cast<Conn*>(ud);
    const h2::FrameHd* hd = static_cast<const h2::FrameHd*>(frame);
    if (hd->stream_id == c.sid && (hd->type == h2::kTypeData || hd->type == h2::kTypeHeaders) &&
        (hd->flags & h2::kFlagEndStream))
      c.closed = true;
    return 0;
  }
  static int on_close(void*, int32_t sid, uint32_t code, void* ud) {
    Conn& c = *static_cast<Conn*>(ud);
    if (sid == c.sid) {
      c.closed = true;
      c.close_code = code;
    }
    return 0;
  }
  static ssize_t read_req(void*, int32_t, uint8_t* buf, size_t length, uint32_t*, h2::DataSource*, void* ud) {
    Conn& c = *static_cast<Conn*>(ud);
    const size_t n = std::min(length, c.outq.size() - c.outq_off);
    if (!n) return h2::kErrDeferred;
    std::memcpy(buf, c.outq.data() + c.outq_off, n);
    c.outq_off += n;
    if (c.outq_off == c.outq.size()) {
      c.outq.clear();
      c.outq_off = 0;
    }
    return (ssize_t)n;
  }
  static void* callbacks() {
    static void* cbs = [] {
      const h2::Lib& g = h2::lib();
      void* cb = nullptr;
      if (!g.ok || g.callbacks_new(&cb) != 0) return (void*)nullptr;
      g.set_on_header(cb, &Conn::on_header);
      g.set_on_data_chunk_recv(cb, &Conn::on_data);
      g.set_on_stream_close(cb, &Conn::on_close);
      g.set_on_frame_recv(cb, &Conn::on_frame);
      g.set_read_length(cb, &h2::read_length);
      return cb;
    }();
    return cbs;
  }

  void send_pending(int timeout_ms) {
    const h2::Lib& g = h2::lib();
    for (;;) {
      const uint8_t* d = nullptr;
      const ssize_t n = g.mem_send(ng, &d);
      if (n < 0) throw std::runtime_error("gRPC client: HTTP/2 framing error");
      if (n == 0) return;
      size_t off = 0;
      while (off < (size_t)n) {
        const ssize_t w = ::send(fd, d + off, (size_t)n - off, MSG_NOSIGNAL);
        if (w > 0) {
          off += (size_t)w;
          continue;
        }
        if (w < 0 && errno == EINTR) continue;
        if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
          pollfd pf{fd, POLLOUT, 0};
          if (::poll(&pf, 1, timeout_ms) <= 0) throw std::runtime_error("gRPC client: send timed out");
          continue;
        }
        throw std::runtime_error("gRPC client: connection lost while sending");
      }
    }
  }

  // One socket read + parse; false on timeout.  Chunk bytes the caller is waiting for are received
  // into its buffer directly; everything else (frame headers, message headers, control frames,
  // read-ahead) goes through inbuf, read no further than the next point where that can start.
  bool pump(int timeout_ms) {
    if (inbuf.size() < (1u << 20)) inbuf.resize(1u << 20);
    uint8_t* target = reinterpret_cast<uint8_t*>(&inbuf[0]);
    size_t want = inbuf.size();
    if (!in_payload) {
      want = 9 - fh_n;                                   // the next frame header
    } else if (our_data && state == 2 && need > 0) {
      target = dst;                                      // chunk bytes: straight into place
      want = (size_t)std::min<uint64_t>(std::min<uint64_t>(frame_left, data_left), need);
    } else if (our_data && need > 0) {
      want = (size_t)std::min<uint64_t>(frame_left, 16);  // gRPC prefix + ReadResponse header
    } else {
      want = (size_t)std::min<uint64_t>(frame_left, inbuf.size());
    }
    // bytes usually wait in the socket already: poll only when a non-blocking receive finds none
    ssize_t got = ::recv(fd, target, want, MSG_DONTWAIT);
    if (got < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      pollfd pf{fd, POLLIN, 0};
      const int r = ::poll(&pf, 1, timeout_ms);
      if (r == 0) return false;
      if (r < 0 && errno != EINTR) throw std::runtime_error("gRPC client: poll failed");
      got = ::recv(fd, target, want, MSG_DONTWAIT);
    }
    if (got == 0) throw std::runtime_error("gRPC client: connection closed by the worker");
    if (got < 0) {
      if (errno == EINTR || errno == EAGAIN) return true;
      throw std::runtime_error("gRPC client: connection lost");
    }
    if (target != reinterpret_cast<uint8_t*>(&inbuf[0])) direct_bytes += (uint64_t)got;
    track(target, (size_t)got);
    const ssize_t rc = h2::lib().mem_recv(ng, target, (size_t)got);
    if (rc < 0) throw std::runtime_error("gRPC client: malformed ReadBlock response stream");
    return true;
  }
};

namespace {

void put_field_varint(std::string& s, uint32_t field, uint64_t v) {
  h2::put_varint(s, (uint64_t)(field << 3));
  h2::put_varint(s, v);
}

int connect_tcp(const std::string& host, int port, int timeout_ms) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  const std::string h = host == "localhost" ? "127.0.0.1" : host;
  if (::getaddrinfo(h.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("gRPC client: cannot resolve " + host);
  const int fd = ::socket(res->ai_family, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
  if (fd < 0) {
    ::freeaddrinfo(res);
    throw std::runtime_error("gRPC client: socket() failed");
  }
  int rc = ::connect(fd, res->ai_addr, res->ai_addrlen);
  ::freeaddrinfo(res);
  if (rc != 0 && errno == EINPROGRESS) {
    pollfd pf{fd, POLLOUT, 0};
    rc = ::poll(&pf, 1, timeout_ms) == 1 ? 0 : -1;
    int err = 0;
    socklen_t el = sizeof(err);
    if (rc == 0 && (::getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &el) != 0 || err != 0)) rc = -1;
  }
  if (rc != 0) {
    ::close(fd);
    throw std::runtime_error("gRPC client: connect to " + host + ":" + std::to_string(port) + " failed");
  }
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  return fd;
}

int connect_unix(const std::string& path, int timeout_ms) {
  sockaddr_un ua{};
  ua.sun_family = AF_UNIX;
  if (path.size() >= sizeof(ua.sun_path)) throw std::runtime_error("gRPC client: unix socket path too long");
  std::memcpy(ua.sun_path, path.c_str(), path.size() + 1);
  const int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) throw std::runtime_error("gRPC client: socket() failed");
  timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
  ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  int sb = 8 << 20;            // uploads: a Unix stream's in-flight bytes count against the sender
  ::setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sb, sizeof(sb));
  if (::connect(fd, (sockaddr*)&ua, sizeof(ua)) != 0) {
    ::close(fd);
    throw std::runtime_error("gRPC client: connect to unix:" + path + " failed");
  }
  return fd;
}

}  // namespace

GrpcBlockSource::GrpcBlockSource(Options o, uint64_t length) : BlockSource(length), o_(std::move(o)) {
  if (!Conn::callbacks()) throw std::runtime_error("gRPC client: libnghttp2 is not available");
  open(0);
}

GrpcBlockSource::~GrpcBlockSource() { close(); }

void GrpcBlockSource::close() { c_.reset(); }

void GrpcBlockSource::open(uint64_t off) {
  c_.reset();
  auto c = std::make_unique<Conn>();
  const h2::Lib& g = h2::lib();
  c->fd = o_.unix_path.empty() ? connect_tcp(o_.host, o_.port, o_.timeout_ms) : connect_unix(o_.unix_path, o_.timeout_ms);
  if (g.client_new2(&c->ng, Conn::callbacks(), c.get(), nullptr) != 0) throw std::runtime_error("gRPC client: session");
  const h2::SettingsEntry iv[] = {{h2::kSettingsEnablePush, 0},
                                  {h2::kSettingsInitialWindowSize, 16u << 20},
                                  {h2::kSettingsMaxFrameSize, h2::kMaxFramePayload}};
  g.submit_settings(c->ng, 0, iv, 3);
  g.set_local_window_size(c->ng, 0, 0, 64 << 20);
  // first ReadRequest: block_id=1 offset=2 length=3 promote=4 chunk_size=5 open_ufs_block_options=6
  std::string req;
  put_field_varint(req, 1, (uint64_t)o_.block_id);
  if (off) put_field_varint(req, 2, off);
  put_field_varint(req, 3, length_ - off);
  if (o_.promote) put_field_varint(req, 4, 1);
  put_field_varint(req, 5, o_.chunk);
  if (!o_.ufs_options.empty()) {
    h2::put_varint(req, (6u << 3) | 2);
    h2::put_varint(req, o_.ufs_options.size());
    req += o_.ufs_options;
  }
  c->outq.push_back('\0');
  h2::put_be32(c->outq, (uint32_t)req.size());
  c->outq += req;
  c->authority = o_.host + ":" + std::to_string(o_.port);
  std::vector<h2::Nv> nva = {h2::nv(":method", "POST"), h2::nv(":scheme", "http"),
                             h2::nv(":path", "/alluxio.grpc.block.BlockWorker/ReadBlock"),
                             h2::nv(":authority", c->authority), h2::nv("content-type", "application/grpc"),
                             h2::nv("te", "trailers")};
  if (!o_.channel_id.empty()) nva.push_back(h2::nv("channel-id", o_.channel_id));
  if (!o_.user.empty()) nva.push_back(h2::nv("alluxio-user", o_.user));
  h2::DataProvider dp;
  dp.source.ptr = c.get();
  dp.read_callback = &Conn::read_req;
  c->sid = g.submit_request(c->ng, nullptr, nva.data(), nva.size(), &dp, nullptr);
  if (c->sid < 0) throw std::runtime_error("gRPC client: cannot submit ReadBlock");
  c->pos = off;
  c->acked = off;
  c->ack_every = std::max<uint64_t>(o_.chunk, 64u << 10);
  c->send_pending(o_.timeout_ms);
  c_ = std::move(c);
}

void GrpcBlockSource::start() {
  if (!c_) open(0);
}

void GrpcBlockSource::read(uint64_t off, uint64_t n, uint8_t* dst) {
  if (off + n > length_) throw StoreError(kErrInvalidArgument, "read beyond the block");
  if (!c_ || off != c_->pos) open(off);   // positioned / backward read: a new call at `off`
  Conn& c = *c_;
  uint64_t got = 0;
  if (c.spill_off < c.spill.size()) {
    got = std::min<uint64_t>(n, c.spill.size() - c.spill_off);
    std::memcpy(dst, c.spill.data() + c.spill_off, got);
    c.spill_off += got;
  }
  c.dst = dst + got;
  c.need = n - got;
  while (c.need > 0) {
    if (c.closed) {
      if (c.grpc_status > 0)
        throw StoreError(c.grpc_status == 5 ? kErrNotFound : kErrIo,
                         "ReadBlock of block " + std::to_string(o_.block_id) + " failed (gRPC status " +
                             std::to_string(c.grpc_status) + "): " + c.grpc_msg);
      throw StoreError(kErrIo, "ReadBlock stream of block " + std::to_string(o_.block_id) + " ended after " +
                                   std::to_string(c.pos + (n - c.need)) + " of " + std::to_string(length_) + " bytes");
    }
    if (!c.pump(o_.timeout_ms))
      throw StoreError(kErrTimeout, "ReadBlock of block " + std::to_string(o_.block_id) + " timed out");
    // offset_received of what this call already took: a read longer than the server's window
    // keeps the stream moving
    maybe_ack(c.pos + (n - c.need));
    c.send_pending(o_.timeout_ms);     // acks, WINDOW_UPDATEs
  }
  c.dst = nullptr;
  c.pos += n;
  maybe_ack(c.pos);
  c.send_pending(o_.timeout_ms);
}

void GrpcBlockSource::maybe_ack(uint64_t offset) {
  Conn& c = *c_;
  if (c.closed || offset < c.acked + c.ack_every) return;
  std::string ack;
  put_field_varint(ack, 7, offset);
  c.outq.push_back('\0');
  h2::put_be32(c.outq, (uint32_t)ack.size());
  c.outq += ack;
  c.acked = offset;
  h2::lib().resume_data(c.ng, c.sid);
}

// ---- GrpcBlockSink: WriteBlock over HTTP/2 -----------------------------------------------------
struct GrpcBlockSink::Conn {
  struct Seg {
    std::string hdr;               // gRPC prefix + WriteRequest/Chunk headers (or a whole message)
    const uint8_t* data = nullptr; // caller bytes (valid until write() returns)
    size_t len = 0;
    size_t off = 0;                // over hdr then data
  };
  int fd = -1;
  void* ng = nullptr;
  int32_t sid = -1;
  std::string authority;
  std::deque<Seg> q;
  bool closing = false, closed = false, headers_ok = false;
  int grpc_status = -1;
  std::string grpc_msg;
  std::string resp;                // response DATA (WriteResponse messages)
  std::string inbuf;

  ~Conn() {
    if (ng) h2::lib().session_del(ng);
    if (fd >= 0) ::close(fd);
  }
  static int on_header(void*, const void* frame, const uint8_t* name, size_t namelen, const uint8_t* value,
                       size_t valuelen, uint8_t, void* ud) {
    Conn& c = *static_cast<Conn*>(ud);
    const h2::FrameHd* hd = static_cast<const h2::FrameHd*>(frame);
    if (hd->stream_id != c.sid) return 0;
    const std::string n(reinterpret_cast<const char*>(name), namelen);
    const std::string v(reinterpret_cast<const char*>(value), valuelen);
    if (n == ":status") c.headers_ok = v == "200";
    else if (n == "grpc-status") c.grpc_status = std::atoi(v.c_str());
    else if (n == "grpc-message") c.grpc_msg = v;
    return 0;
  }
  static int on_data(void*, uint8_t, int32_t sid, const uint8_t* data, size_t len, void* ud) {
    Conn& c = *static_cast<Conn*>(ud);
    if (sid == c.sid && c.resp.size() < (1u << 20)) c.resp.append(reinterpret_cast<const char*>(data), len);
    return 0;
  }
  static int on_frame(void*, const void* frame, void* ud) {
    Conn& c = *static_cast<Conn*>(ud);
    const h2::FrameHd* hd = static_cast<const h2::FrameHd*>(frame);
    if (hd->stream_id == c.sid && (hd->type == h2::kTypeData || hd->type == h2::kTypeHeaders) &&
        (hd->flags & h2::kFlagEndStream))
      c.closed = true;
    return 0;
  }
  static int on_close(void*, int32_t sid, uint32_t, void* ud) {
    Conn& c = *static_cast<Conn*>(ud);
    if (sid == c.sid) c.closed = true;
    return 0;
  }
  static ssize_t read_req(void*, int32_t, uint8_t* buf, size_t length, uint32_t* flags, h2::DataSource*, void* ud) {
    Conn& c = *static_cast<Conn*>(ud);
    size_t w = 0;
    while (w < length && !c.q.empty()) {
      Seg& s = c.q.front();
      if (s.off < s.hdr.size()) {
        const size_t n = std::min(length - w, s.hdr.size() - s.off);
        std::memcpy(buf + w, s.hdr.data() + s.off, n);
        s.off += n;
        w += n;
        continue;
      }
      const size_t d = s.off - s.hdr.size();
      const size_t n = std::min(length - w, s.len - d);
      if (n) std::memcpy(buf + w, s.data + d, n);
      s.off += n;
      w += n;
      if (s.off == s.hdr.size() + s.len) c.q.pop_front();
    }
    if (c.q.empty() && c.closing) {
      *flags |= h2::kDataEof;      // END_STREAM: the request stream is complete
      return (ssize_t)w;
    }
    return w ? (ssize_t)w : h2::kErrDeferred;
  }
  static void* callbacks() {
    static void* cbs = [] {
      const h2::Lib& g = h2::lib();
      void* cb = nullptr;
      if (!g.ok || g.callbacks_new(&cb) != 0) return (void*)nullptr;
      g.set_on_header(cb, &Conn::on_header);
      g.set_on_data_chunk_recv(cb, &Conn::on_data);
      g.set_on_stream_close(cb, &Conn::on_close);
      g.set_on_frame_recv(cb, &Conn::on_frame);
      g.set_read_length(cb, &h2::read_length);
      return cb;
    }();
    return cbs;
  }
  void send_pending(int timeout_ms) {
    const h2::Lib& g = h2::lib();
    for (;;) {
      const uint8_t* d = nullptr;
      const ssize_t n = g.mem_send(ng, &d);
      if (n < 0) throw std::runtime_error("gRPC client: HTTP/2 framing error");
      if (n == 0) return;
      size_t off = 0;
      while (off < (size_t)n) {
        const ssize_t w = ::send(fd, d + off, (size_t)n - off, MSG_NOSIGNAL);
        if (w > 0) {
          off += (size_t)w;
          continue;
        }
        if (w < 0 && errno == EINTR) continue;
        if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
          pollfd pf{fd, POLLOUT, 0};
          if (::poll(&pf, 1, timeout_ms) <= 0) throw std::runtime_error("gRPC client: send timed out");
          continue;
        }
        throw std::runtime_error("gRPC client: connection lost while sending");
      }
    }
  }
  bool pump(int timeout_ms) {
    pollfd pf{fd, POLLIN, 0};
    const int r = ::poll(&pf, 1, timeout_ms);
    if (r == 0) return false;
    if (r < 0 && errno != EINTR) throw std::runtime_error("gRPC client: poll failed");
    if (inbuf.size() < (256u << 10)) inbuf.resize(256u << 10);
    const ssize_t got = ::recv(fd, &inbuf[0], inbuf.size(), 0);
    if (got == 0) throw std::runtime_error("gRPC client: connection closed by the worker");
    if (got < 0) {
      if (errno == EINTR || errno == EAGAIN) return true;
      throw std::runtime_error("gRPC client: connection lost");
    }
    if (h2::lib().mem_recv(ng, reinterpret_cast<const uint8_t*>(inbuf.data()), (size_t)got) < 0)
      throw std::runtime_error("gRPC client: malformed WriteBlock response stream");
    return true;
  }
};

namespace {
int store_code_of(int grpc_status) {
  switch (grpc_status) {
    case 5: return kErrNotFound;
    case 6: return kErrAlreadyExists;
    case 8: return kErrOutOfSpace;
    case 3: return kErrInvalidArgument;
    case 9: return kErrInvalidState;
    case 4: return kErrTimeout;
    default: return kErrIo;
  }
}
}  // namespace

GrpcBlockSink::GrpcBlockSink(Options o) : o_(std::move(o)) {
  if (!Conn::callbacks()) throw std::runtime_error("gRPC client: libnghttp2 is not available");
  auto c = std::make_unique<Conn>();
  const h2::Lib& g = h2::lib();
  c->fd = o_.unix_path.empty() ? connect_tcp(o_.host, o_.port, o_.timeout_ms) : connect_unix(o_.unix_path, o_.timeout_ms);
  if (g.client_new2(&c->ng, Conn::callbacks(), c.get(), nullptr) != 0) throw std::runtime_error("gRPC client: session");
  const h2::SettingsEntry iv[] = {{h2::kSettingsEnablePush, 0},
                                  {h2::kSettingsInitialWindowSize, 1u << 20},
                                  {h2::kSettingsMaxFrameSize, h2::kMaxFramePayload}};
  g.submit_settings(c->ng, 0, iv, 3);
  // WriteRequest{command{type=0 id tier pin space_to_reserve medium_type}}
  std::string cmd = o_.command;
  if (cmd.empty()) {
    put_field_varint(cmd, 1, 0);
    put_field_varint(cmd, 2, (uint64_t)o_.block_id);
    put_field_varint(cmd, 4, (uint64_t)(uint32_t)o_.tier);
    if (!o_.medium.empty()) {
      h2::put_varint(cmd, (8u << 3) | 2);
      h2::put_varint(cmd, o_.medium.size());
      cmd += o_.medium;
    }
    if (o_.pin) put_field_varint(cmd, 9, 1);
    put_field_varint(cmd, 10, o_.reserve);
  }
  std::string req;
  h2::put_varint(req, (1u << 3) | 2);
  h2::put_varint(req, cmd.size());
  req += cmd;
  Conn::Seg first;
  first.hdr.push_back('\0');
  h2::put_be32(first.hdr, (uint32_t)req.size());
  first.hdr += req;
  c->q.push_back(std::move(first));
  c->authority = o_.host + ":" + std::to_string(o_.port);
  std::vector<h2::Nv> nva = {h2::nv(":method", "POST"), h2::nv(":scheme", "http"),
                             h2::nv(":path", "/alluxio.grpc.block.BlockWorker/WriteBlock"),
                             h2::nv(":authority", c->authority), h2::nv("content-type", "application/grpc"),
                             h2::nv("te", "trailers")};
  if (!o_.channel_id.empty()) nva.push_back(h2::nv("channel-id", o_.channel_id));
  if (!o_.user.empty()) nva.push_back(h2::nv("alluxio-user", o_.user));
  h2::DataProvider dp;
  dp.source.ptr = c.get();
  dp.read_callback = &Conn::read_req;
  c->sid = g.submit_request(c->ng, nullptr, nva.data(), nva.size(), &dp, nullptr);
  if (c->sid < 0) throw std::runtime_error("gRPC client: cannot submit WriteBlock");
  c_ = std::move(c);
  wait_drained();
}

GrpcBlockSink::~GrpcBlockSink() {
  if (c_ && !c_->closed) cancel();
}

void GrpcBlockSink::wait_drained() {
  Conn& c = *c_;
  h2::lib().resume_data(c.ng, c.sid);
  c.send_pending(o_.timeout_ms);
  while (!c.q.empty()) {
    if (c.closed) break;                 // the worker failed the call early
    if (!c.pump(o_.timeout_ms))
      throw StoreError(kErrTimeout, "WriteBlock of block " + std::to_string(o_.block_id) + " timed out");
    h2::lib().resume_data(c.ng, c.sid);  // WINDOW_UPDATEs reopen the send window
    c.send_pending(o_.timeout_ms);
  }
  if (c.closed && c.grpc_status > 0) {
    c.q.clear();
    throw StoreError(store_code_of(c.grpc_status), "WriteBlock of block " + std::to_string(o_.block_id) +
                                                       " failed (gRPC status " + std::to_string(c.grpc_status) +
                                                       "): " + c.grpc_msg);
  }
}

void GrpcBlockSink::write(const uint8_t* p, uint64_t n) {
  if (!c_ || c_->closing) throw StoreError(kErrInvalidState, "write after commit/cancel");
  Conn& c = *c_;
  uint64_t off = 0;
  while (off < n) {
    const size_t k = (size_t)std::min<uint64_t>(o_.chunk, n - off);
    // WriteRequest{chunk(2){data(1)}}
    std::string inner;
    h2::put_varint(inner, (1u << 3) | 2);
    h2::put_varint(inner, k);
    std::string outer;
    h2::put_varint(outer, (2u << 3) | 2);
    h2::put_varint(outer, inner.size() + k);
    Conn::Seg s;
    s.hdr.push_back('\0');
    h2::put_be32(s.hdr, (uint32_t)(outer.size() + inner.size() + k));
    s.hdr += outer;
    s.hdr += inner;
    s.data = p + off;
    s.len = k;
    c.q.push_back(std::move(s));
    off += k;
  }
  wait_drained();                        // the caller's bytes are in HTTP/2 frames from here on
  written_ += n;
}

void GrpcBlockSink::append_block(int64_t block_id, uint64_t length) {
  if (!c_ || c_->closing) throw StoreError(kErrInvalidState, "append after commit/cancel");
  // WriteRequest{append_block(20){block_id(1), length(2)}}
  std::string inner;
  h2::put_varint(inner, (1u << 3));
  h2::put_varint(inner, (uint64_t)block_id);
  h2::put_varint(inner, (2u << 3));
  h2::put_varint(inner, length);
  std::string msg;
  h2::put_varint(msg, (20u << 3) | 2);
  h2::put_varint(msg, inner.size());
  msg += inner;
  Conn::Seg s;
  s.hdr.push_back('\0');
  h2::put_be32(s.hdr, (uint32_t)msg.size());
  s.hdr += msg;
  c_->q.push_back(std::move(s));
  wait_drained();
  written_ += length;
}

uint64_t GrpcBlockSink::commit(bool hold_for_append) {
  if (!c_) throw StoreError(kErrInvalidState, "commit after cancel");
  Conn& c = *c_;
  if (hold_for_append) {
    // WriteRequest{command(1){hold_for_append(20)=true}} ahead of the half-close
    std::string inner, msg;
    h2::put_varint(inner, (20u << 3));
    h2::put_varint(inner, 1);
    h2::put_varint(msg, (1u << 3) | 2);
    h2::put_varint(msg, inner.size());
    msg += inner;
    Conn::Seg s;
    s.hdr.push_back('\0');
    h2::put_be32(s.hdr, (uint32_t)msg.size());
    s.hdr += msg;
    c.q.push_back(std::move(s));
  }
  c.closing = true;
  wait_drained();
  while (!c.closed) {
    if (!c.pump(o_.timeout_ms))
      throw StoreError(kErrTimeout, "commit of block " + std::to_string(o_.block_id) + " timed out");
    c.send_pending(o_.timeout_ms);
  }
  if (c.grpc_status != 0)
    throw StoreError(store_code_of(c.grpc_status), "WriteBlock of block " + std::to_string(o_.block_id) +
                                                       " failed (gRPC status " + std::to_string(c.grpc_status) +
                                                       "): " + c.grpc_msg);
  const uint64_t n = written_;
  c_.reset();
  return n;
}

void GrpcBlockSink::cancel() {
  if (!c_) return;
  Conn& c = *c_;
  try {
    h2::lib().submit_rst_stream(c.ng, 0, c.sid, 8 /*CANCEL*/);
    c.send_pending(1000);
  } catch (...) {
  }
  c_.reset();
}

// ---- prefetch pool ------------------------------------------------------------------------------
namespace {

class PrefetchPool {
 public:
  // Two pools: prefetches of network sources (threads mostly blocked in recv) and of DMA / memcpy
  // sources (threads issuing copies: more than a few dozen only contend).
  static PrefetchPool& get(bool network = false) {
    static PrefetchPool* net = new PrefetchPool(kNetworkCap);   // never destroyed: threads outlive statics
    static PrefetchPool* dma = new PrefetchPool(kDmaCap);
    return network ? *net : *dma;
  }
  // A thread is added whenever a prefetch would otherwise queue behind busy ones, up to the cap:
  // each stream has at most one prefetch in flight, so the network pool grows with the streams
  // reading at once (64 reader threads of one client process get 64 concurrent chunk reads, not
  // 16), and idle threads serve the next ones.
  void submit(std::function<void()> fn) {
    std::function<void()> here;
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(std::move(fn));
      const int cap = want_ > 0 ? want_ : cap_;
      if ((int)q_.size() > idle_ && threads_ < cap) {
        try {
          std::thread([this] { run(); }).detach();
          ++threads_;
        } catch (...) {
          // the queued prefetch runs on an existing thread; with none, the caller runs it
          if (threads_ == 0) {
            here = std::move(q_.back());
            q_.pop_back();
          }
        }
      }
    }
    if (here) {
      here();
      return;
    }
    cv_.notify_one();
  }
  void set_threads(int n) {
    std::lock_guard<std::mutex> g(mu_);
    want_ = n;
  }

 private:
  // measured on one MI355X box, 4 KiB readers of one client process: a 16-thread pool held gRPC
  // at ~22-26 GB/s from 64 readers on; with a pool growing to 256, IPC readers fell from 46 to
  // 11-16 GB/s at 64-256 threads (the D2H copies contend), while gRPC gained
  static constexpr int kNetworkCap = 64, kDmaCap = 16;
  explicit PrefetchPool(int cap) : cap_(cap) {}
  const int cap_;
  void run() {
    pthread_setname_np(pthread_self(), "chunk-prefetch");
    for (;;) {
      std::function<void()> fn;
      {
        std::unique_lock<std::mutex> lk(mu_);
        ++idle_;
        cv_.wait(lk, [&] { return !q_.empty(); });
        --idle_;
        fn = std::move(q_.front());
        q_.pop_front();
      }
      fn();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  int threads_ = 0, idle_ = 0;
  int want_ = 0;
};

}  // namespace

void set_prefetch_threads(int n) {
  PrefetchPool::get(false).set_threads(n);
  PrefetchPool::get(true).set_threads(n);
}

// One chunk read ahead: [lo, hi) of the file into `buf`, by a pool thread.
struct HostInStream::Prefetch {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  int err_code = 0;
  std::string err;
  uint64_t lo = 0, hi = 0;
  int buf = 0;
  void finish(int code, std::string msg) {
    std::lock_guard<std::mutex> g(mu);
    err_code = code;
    err = std::move(msg);
    done = true;
    cv.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return done; });
  }
  bool ready() {
    std::lock_guard<std::mutex> g(mu);
    return done;
  }
};

// ---- HostInStream -----------------------------------------------------------------------------
HostInStream::HostInStream(uint64_t length, uint64_t block_size, uint64_t chunk, bool prefetch)
    : length_(length), block_size_(block_size ? block_size : (64ull << 20)), chunk_(chunk ? chunk : (1u << 20)),
      prefetch_(prefetch) {}

HostInStream::~HostInStream() {
  drop_source();
  for (int i = 0; i < 2; ++i) host_buffer_release(bufs_[i], chunk_, pinned_[i]);
}

void HostInStream::cancel_prefetch() {
  if (!pf_) return;
  pf_->wait();
  pf_.reset();
}

void HostInStream::set_source(int64_t idx, std::shared_ptr<BlockSource> src) {
  drop_source();
  cur_idx_ = idx;
  cur_start_ = (uint64_t)idx * block_size_;
  cur_ = std::move(src);
}

void HostInStream::drop_source() {
  cancel_prefetch();
  if (cur_) cur_->close();
  cur_.reset();
  cur_idx_ = -1;
  buf_lo_ = buf_hi_ = 0;
}

void HostInStream::make_current(int i, uint64_t lo, uint64_t hi) {
  cur_buf_ = i;
  buf_ = bufs_[i];
  buf_lo_ = lo;
  buf_hi_ = hi;
}

// Reads the chunk after the current one (same block) into the other buffer on a pool thread.
void HostInStream::schedule_prefetch() {
  if (!prefetch_ || !cur_ || cur_->needs_gil() || pf_) return;
  const uint64_t block_end = cur_start_ + cur_->length();
  if (buf_hi_ >= block_end || buf_hi_ <= buf_lo_) return;
  const int nb = 1 - cur_buf_;
  if (!bufs_[nb]) bufs_[nb] = host_buffer_alloc(chunk_, &pinned_[nb]);
  auto p = std::make_shared<Prefetch>();
  p->lo = buf_hi_;
  p->hi = std::min(buf_hi_ + chunk_, block_end);
  p->buf = nb;
  std::shared_ptr<BlockSource> src = cur_;
  uint8_t* dst = bufs_[nb];
  const uint64_t off = p->lo - cur_start_, n = p->hi - p->lo;
  pf_ = p;
  PrefetchPool::get(src->waits_on_network()).submit([p, src, dst, off, n] {
    try {
      src->read(off, n, dst);
      p->finish(0, std::string());
    } catch (const StoreError& e) {
      p->finish(e.code, e.what());
    } catch (const std::exception& e) {
      p->finish(kErrIo, e.what());
    }
  });
}

bool HostInStream::try_swap() {
  if (!pf_ || pos_ < pf_->lo || pos_ >= pf_->hi || !pf_->ready()) return false;
  if (pf_->err_code) return false;          // the synchronous path reports (or retries) it
  std::shared_ptr<Prefetch> p = std::move(pf_);
  make_current(p->buf, p->lo, p->hi);
  ++refills_;
  ++pf_hits_;
  schedule_prefetch();
  return true;
}

uint64_t HostInStream::copy_buffered(uint8_t* dst, uint64_t n) {
  if (!cur_) return 0;
  if (!(pos_ >= buf_lo_ && pos_ < buf_hi_) && !try_swap()) return 0;
  const uint64_t t = std::min(n, buf_hi_ - pos_);
  std::memcpy(dst, buf_ + (pos_ - buf_lo_), t);
  pos_ += t;
  bytes_ += t;
  return t;
}

uint64_t HostInStream::read_block_part(uint8_t* dst, uint64_t n) {
  if (!cur_) throw StoreError(kErrInvalidState, "no block source for the read position");
  const uint64_t off = pos_ - cur_start_;
  const uint64_t blen = cur_->length();
  if (off >= blen) throw StoreError(kErrInvalidState, "block " + std::to_string(cur_idx_) + " is shorter than expected");
  n = std::min(n, blen - off);
  if (pos_ >= buf_lo_ && pos_ < buf_hi_) {   // the tail of the buffered chunk first
    const uint64_t t = std::min(n, buf_hi_ - pos_);
    std::memcpy(dst, buf_ + (pos_ - buf_lo_), t);
    pos_ += t;
    bytes_ += t;
    return t;
  }
  if (pf_) {
    const bool covers = pos_ >= pf_->lo && pos_ < pf_->hi;
    pf_->wait();                              // the source is ours again after this
    if (covers && !pf_->err_code) {
      std::shared_ptr<Prefetch> p = std::move(pf_);
      make_current(p->buf, p->lo, p->hi);
      ++refills_;
      ++pf_hits_;
      schedule_prefetch();
      const uint64_t t = std::min(n, buf_hi_ - pos_);
      std::memcpy(dst, buf_ + (pos_ - buf_lo_), t);
      pos_ += t;
      bytes_ += t;
      return t;
    }
    pf_.reset();                              // a seek elsewhere, or a failed read: redo it here
  }
  if (cur_->direct() && n >= chunk_) {
    cur_->read(off, n, dst);   // big reads: no bounce through the chunk buffer
    pos_ += n;
    bytes_ += n;
    return n;
  }
  if (!bufs_[cur_buf_]) bufs_[cur_buf_] = host_buffer_alloc(chunk_, &pinned_[cur_buf_]);
  buf_ = bufs_[cur_buf_];
  const uint64_t fill = std::min(chunk_, blen - off);
  buf_lo_ = buf_hi_ = 0;
  cur_->read(off, fill, buf_);
  ++refills_;
  make_current(cur_buf_, pos_, pos_ + fill);
  schedule_prefetch();
  const uint64_t t = std::min(n, fill);
  std::memcpy(dst, buf_, t);
  pos_ += t;
  bytes_ += t;
  return t;
}

}  // namespace amdx
