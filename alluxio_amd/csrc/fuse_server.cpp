// Native /dev/fuse request loop (see fuse_server.h).
#include "fuse_server.h"

#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <poll.h>
#include <pthread.h>
#include <sys/ioctl.h>
#include <sys/stat.h>
#include <sys/uio.h>
#include <unistd.h>

#include <chrono>
#include <cstring>

#include "block_store.h"
#include "meta_codec.h"

namespace amdx {

namespace {

// linux/fuse.h (protocol 7.x) wire structs used on the fast path
struct InHeader {
  uint32_t len, opcode;
  uint64_t unique, nodeid;
  uint32_t uid, gid, pid, padding;
};
struct OutHeader {
  uint32_t len;
  int32_t error;
  uint64_t unique;
};
struct EntryHead {
  uint64_t nodeid, generation, entry_valid, attr_valid;
  uint32_t entry_valid_nsec, attr_valid_nsec;
};
struct AttrOutHead {
  uint64_t attr_valid;
  uint32_t attr_valid_nsec, dummy;
};
struct OpenIn {
  uint32_t flags, unused;
};
struct OpenOut {
  uint64_t fh;
  uint32_t open_flags;
  int32_t backing_id;          // protocol 7.40 (was padding)
};
struct BackingMap {            // FUSE_DEV_IOC_BACKING_OPEN argument (protocol 7.40)
  int32_t fd;
  uint32_t flags;
  uint64_t padding;
};
constexpr unsigned long kIocBackingOpen = _IOW(229, 1, BackingMap);
constexpr unsigned long kIocBackingClose = _IOW(229, 2, uint32_t);
constexpr uint32_t kFopenPassthrough = 1u << 7;
struct ReadIn {
  uint64_t fh, offset;
  uint32_t size, read_flags;
  uint64_t lock_owner;
  uint32_t flags, padding;
};
struct ReleaseIn {
  uint64_t fh;
  uint32_t flags, release_flags;
  uint64_t lock_owner;
};
struct FlushIn {
  uint64_t fh;
  uint32_t unused, padding;
  uint64_t lock_owner;
};
constexpr size_t kAttrBytes = 88;
constexpr uint32_t kLookup = 1, kForget = 2, kGetattr = 3, kOpen = 14, kRead = 15, kWrite = 16, kRelease = 18,
                   kFsync = 20, kFlush = 25, kInterrupt = 36, kIoctl = 39, kBatchForget = 42;
constexpr uint32_t kFopenKeepCache = 1u << 1;
constexpr uint32_t kFopenNoFlush = 1u << 5;       // read-only native handle: close() sends no FLUSH
constexpr uint64_t kNativeFh = 1ull << 62;
constexpr size_t kBufSize = (1u << 20) + 4096 * 2;      // a 1 MiB WRITE (max_pages 256) + headers
constexpr size_t kPipeSize = ((128u << 10) + 4096 * 2) * 2; // splice of READ replies (<= 128 KiB)

int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

std::string child_path(const std::string& parent, const char* name) {
  std::string p = parent;
  if (p.empty() || p.back() != '/') p.push_back('/');
  p.append(name);
  return p;
}

}  // namespace

FuseServer::FuseServer(int fd, int threads, BlockStore* store, int64_t session, int keep_cache)
    : fd_(fd), nthreads_(threads < 1 ? 1 : threads), store_(store), session_(session), keep_cache_(keep_cache) {
  for (int i = 0; i < 64; ++i) {
    native_ops_[i] = 0;
    python_ops_[i] = 0;
    native_ns_[i] = 0;
  }
  paths_[1] = "/";
  ids_["/"] = 1;
}

FuseServer::~FuseServer() {
  stop();
  std::lock_guard<std::mutex> g(hmu_);
  if (store_) {
    for (auto& kv : handles_)
      for (int64_t l : kv.second.locks) {
        try { store_->unlock(l); } catch (...) {}
      }
  }
  handles_.clear();
}

void FuseServer::start() {
  if (!threads_.empty()) return;
  if (fd_ >= 0) fcntl(fd_, F_SETFL, fcntl(fd_, F_GETFL) | O_NONBLOCK);
  running_.store(true);
  for (int i = 0; i < nthreads_; ++i) threads_.emplace_back([this, i] { loop(i); });
}

void FuseServer::stop() {
  running_.store(false);
  qcv_.notify_all();
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
}

// ---- node table ---------------------------------------------------------------------------------
uint64_t FuseServer::node_of(const std::string& path) {
  std::lock_guard<std::mutex> g(nmu_);
  auto it = ids_.find(path);
  if (it != ids_.end()) return it->second;
  const uint64_t id = next_id_++;
  ids_[path] = id;
  paths_[id] = path;
  return id;
}

std::string FuseServer::path_of(uint64_t nodeid, bool* ok) {
  std::lock_guard<std::mutex> g(nmu_);
  auto it = paths_.find(nodeid);
  *ok = it != paths_.end();
  return *ok ? it->second : std::string();
}

void FuseServer::forget_path(const std::string& path) {
  std::lock_guard<std::mutex> g(nmu_);
  auto it = ids_.find(path);
  if (it == ids_.end()) return;
  if (it->second != 1) {
    paths_.erase(it->second);
    last_open_fid_.erase(it->second);
  }
  ids_.erase(it);
}

void FuseServer::moved(const std::string& from, const std::string& to) {
  std::lock_guard<std::mutex> g(nmu_);
  std::string pre = from;
  if (pre.empty() || pre.back() != '/') pre.push_back('/');
  std::vector<std::pair<std::string, uint64_t>> hit;
  for (auto& kv : ids_)
    if (kv.first == from || kv.first.compare(0, pre.size(), pre) == 0) hit.emplace_back(kv.first, kv.second);
  for (auto& h : hit) {
    ids_.erase(h.first);
    const std::string np = to + h.first.substr(from.size());
    ids_[np] = h.second;
    paths_[h.second] = np;
  }
}

// ---- attribute cache --------------------------------------------------------------------------
void FuseServer::put_attr(const std::string& path, const std::string& attr, int64_t ttl_ms, uint32_t valid_s,
                          int64_t file_id, bool complete, const std::vector<int64_t>& blocks,
                          const std::vector<int64_t>& lens) {
  if (attr.size() != kAttrBytes || ttl_ms <= 0) return;
  Attr a{attr, now_ms() + ttl_ms, valid_s, file_id, complete, blocks, lens};
  std::lock_guard<std::mutex> g(amu_);
  attrs_[path] = std::move(a);
}

size_t FuseServer::cache_listing(const std::vector<std::string>& chunks, const std::string& strip, uint32_t uid,
                                 uint32_t gid, uint32_t file_ttl_s, uint32_t dir_ttl_s) {
  FileInfoColumns c;
  decode_file_infos(chunks, c);
  const int64_t now = now_ms();
  std::string pre = strip;
  while (!pre.empty() && pre.back() == '/') pre.pop_back();
  size_t n = 0;
  std::vector<std::pair<std::string, Attr>> batch;
  batch.reserve(c.ids.size());
  for (size_t i = 0; i < c.ids.size(); ++i) {
    const bool dir = c.folder[i] != 0;
    if (!dir && !c.completed[i]) continue;       // size still changing: never cached
    std::string path = c.paths[i];
    if (!pre.empty()) {
      if (path.compare(0, pre.size(), pre) != 0 || (path.size() > pre.size() && path[pre.size()] != '/')) continue;
      path = path.size() == pre.size() ? std::string("/") : path.substr(pre.size());
    }
    struct {
      uint64_t ino, size, blocks, atime, mtime, ctime;
      uint32_t atimensec, mtimensec, ctimensec, mode, nlink, uid, gid, rdev, blksize, flags;
    } fa{};
    static_assert(sizeof(fa) == kAttrBytes, "fuse_attr layout");
    const uint64_t size = (uint64_t)c.lengths[i];
    const int64_t mt = c.mtimes[i], at = c.atimes[i] ? c.atimes[i] : c.mtimes[i];
    fa.size = size;
    fa.blocks = (size + 511) / 512;
    fa.atime = (uint64_t)(at / 1000);
    fa.atimensec = (uint32_t)((at % 1000) * 1000000);
    fa.mtime = fa.ctime = (uint64_t)(mt / 1000);
    fa.mtimensec = fa.ctimensec = (uint32_t)((mt % 1000) * 1000000);
    fa.mode = (dir ? 0040000u : 0100000u) | ((uint32_t)c.modes[i] & 07777u);
    fa.nlink = dir ? 2 : 1;
    fa.uid = uid;
    fa.gid = gid;
    const int64_t bs = c.block_sizes[i];
    fa.blksize = bs > 0 ? (uint32_t)std::min<int64_t>(bs, 1 << 30) : 4096;
    Attr a;
    a.raw.assign(reinterpret_cast<const char*>(&fa), kAttrBytes);
    a.valid_s = dir ? dir_ttl_s : file_ttl_s;
    a.expires_ms = now + (int64_t)a.valid_s * 1000;
    a.file_id = c.ids[i];
    a.complete = !dir;
    if (!dir && c.nblocks[i] > 0 && bs > 0) {
      a.blocks.resize((size_t)c.nblocks[i]);
      a.lens.resize((size_t)c.nblocks[i]);
      for (int64_t b = 0; b < c.nblocks[i]; ++b) {
        a.blocks[(size_t)b] = c.first_blocks[i] + b;        // a file's blocks: consecutive ids of its container
        a.lens[(size_t)b] = std::min<int64_t>(bs, (int64_t)size - b * bs);
      }
    }
    if (a.valid_s == 0) continue;
    batch.emplace_back(std::move(path), std::move(a));
    ++n;
  }
  std::lock_guard<std::mutex> g(amu_);
  for (auto& kv : batch) attrs_[std::move(kv.first)] = std::move(kv.second);
  return n;
}

bool FuseServer::entry_reply(const std::string& path, std::string& out) {
  Attr a;
  if (!lookup_attr(path, a)) return false;
  const uint64_t nid = node_of(path);
  out.resize(sizeof(EntryHead) + kAttrBytes);
  EntryHead e{nid, 0, a.valid_s, a.valid_s, 0, 0};
  std::memcpy(&out[0], &e, sizeof(e));
  std::memcpy(&out[sizeof(e)], a.raw.data(), kAttrBytes);
  std::memcpy(&out[sizeof(e)], &nid, 8);            // fuse_attr.ino
  return true;
}

void FuseServer::invalidate(const std::string& path, bool subtree) {
  std::string pre = path;
  if (pre.empty() || pre.back() != '/') pre.push_back('/');
  std::lock_guard<std::mutex> g(amu_);
  attrs_.erase(path);
  if (!subtree) return;
  auto it = attrs_.lower_bound(pre);
  while (it != attrs_.end() && it->first.compare(0, pre.size(), pre) == 0) it = attrs_.erase(it);
}

void FuseServer::clear_attrs() {
  std::lock_guard<std::mutex> g(amu_);
  attrs_.clear();
}

bool FuseServer::lookup_attr(const std::string& path, Attr& a) {
  std::lock_guard<std::mutex> g(amu_);
  auto it = attrs_.find(path);
  if (it == attrs_.end()) return false;
  if (it->second.expires_ms < now_ms()) {
    attrs_.erase(it);
    return false;
  }
  a = it->second;
  return true;
}

std::vector<uint64_t> FuseServer::stats() {
  std::vector<uint64_t> v(192);
  for (int i = 0; i < 64; ++i) {
    v[i] = native_ops_[i].load();
    v[64 + i] = python_ops_[i].load();
    v[128 + i] = native_ns_[i].load();
  }
  return v;
}

// ---- write-behind -------------------------------------------------------------------------------
void FuseServer::register_write_handle(uint64_t fh, uint64_t offset) {
  std::lock_guard<std::mutex> g(wb_mu_);
  WriteBehind& w = wb_[fh];
  w.next = w.buf_off = offset;
}

void FuseServer::unregister_write_handle(uint64_t fh) {
  std::unique_lock<std::mutex> lk(wb_mu_);
  wb_cv_.wait_for(lk, std::chrono::seconds(60), [&] {
    auto it = wb_.find(fh);
    return it == wb_.end() || it->second.outstanding == 0;
  });
  wb_.erase(fh);
  wb_cv_.notify_all();
}

void FuseServer::batch_done(uint64_t fh, int err) {
  std::lock_guard<std::mutex> g(wb_mu_);
  auto it = wb_.find(fh);
  if (it != wb_.end()) {
    if (it->second.outstanding > 0) --it->second.outstanding;
    if (err && !it->second.err) it->second.err = err;
  }
  wb_cv_.notify_all();
}

int FuseServer::wait_batches(uint64_t fh, int timeout_ms) {
  std::unique_lock<std::mutex> lk(wb_mu_);
  auto it = wb_.find(fh);
  if (it == wb_.end()) return 0;
  if (!it->second.buf.empty()) queue_batch(lk, fh, it->second);    // a FLUSH that raced the WRITEs
  const bool done = wb_cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] {
    auto j = wb_.find(fh);
    return j == wb_.end() || j->second.outstanding == 0;
  });
  it = wb_.find(fh);
  if (!done) return ETIMEDOUT;
  return it == wb_.end() ? 0 : it->second.err;
}

void FuseServer::queue_batch(std::unique_lock<std::mutex>& lk, uint64_t fh, WriteBehind& w) {
  // one batch per handle in flight: the next waits for Python to apply the previous one
  wb_cv_.wait(lk, [&] { return w.outstanding == 0 || !alive(); });
  if (w.buf.empty()) return;
  FuseRequest r{0, kOpWriteBatch, w.nodeid, w.uid, w.gid, w.pid, std::string()};
  r.body.reserve(16 + w.buf.size());
  r.body.append(reinterpret_cast<const char*>(&fh), 8);
  r.body.append(reinterpret_cast<const char*>(&w.buf_off), 8);
  r.body += w.buf;
  w.buf.clear();
  w.buf_off = w.next;
  ++w.outstanding;
  write_batches_.fetch_add(1, std::memory_order_relaxed);
  {
    std::lock_guard<std::mutex> g(qmu_);
    queue_.push_back(std::move(r));
  }
  qcv_.notify_one();
}

bool FuseServer::write_behind(const char* req, size_t n) {
  const InHeader* ih = reinterpret_cast<const InHeader*>(req);
  const char* body = req + sizeof(InHeader);
  const size_t blen = n - sizeof(InHeader);
  if (blen < 40) return false;
  uint64_t fh, off;
  uint32_t size;
  std::memcpy(&fh, body, 8);
  std::memcpy(&off, body + 8, 8);
  std::memcpy(&size, body + 16, 4);
  if (blen < 40 + (size_t)size) return false;
  std::unique_lock<std::mutex> lk(wb_mu_);
  auto it = wb_.find(fh);
  if (it == wb_.end()) return false;
  WriteBehind& w = it->second;
  if (w.err) return false;                              // Python reports the error
  if (off + size <= w.next && off < w.next) {
    // re-send of a range already taken (a kernel quirk the Python path also tolerates)
  } else if (off != w.next) {
    if (!w.buf.empty()) queue_batch(lk, fh, w);         // what came before goes first
    return false;
  } else {
    if (w.buf.empty()) w.buf_off = off;
    w.nodeid = ih->nodeid;
    w.uid = ih->uid;
    w.gid = ih->gid;
    w.pid = ih->pid;
    w.buf.append(body + 40, size);
    w.next += size;
    if (w.buf.size() >= kWriteBatchBytes) queue_batch(lk, fh, w);
  }
  lk.unlock();
  const uint32_t out[2] = {size, 0};                    // fuse_write_out
  send(ih->unique, 0, reinterpret_cast<const char*>(out), sizeof(out));
  return true;
}

void FuseServer::flush_handle(uint64_t fh) {
  std::unique_lock<std::mutex> lk(wb_mu_);
  auto it = wb_.find(fh);
  if (it != wb_.end() && !it->second.buf.empty()) queue_batch(lk, fh, it->second);
}

// ---- python slow path ---------------------------------------------------------------------------
std::vector<FuseRequest> FuseServer::poll(int max_n, int timeout_ms) {
  std::unique_lock<std::mutex> lk(qmu_);
  if (queue_.empty() && alive())
    qcv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return !queue_.empty() || !alive(); });
  std::vector<FuseRequest> out;
  while (!queue_.empty() && (int)out.size() < max_n) {
    out.push_back(std::move(queue_.front()));
    queue_.pop_front();
  }
  return out;
}

void FuseServer::send(uint64_t unique, int err, const char* payload, size_t n) {
  OutHeader h{(uint32_t)(sizeof(OutHeader) + (err ? 0 : n)), -err, unique};
  iovec iov[2] = {{&h, sizeof(h)}, {const_cast<char*>(payload), err ? 0 : n}};
  // ENOENT: the request was interrupted and already answered; EBADF/ENODEV: unmounted
  (void)!writev(fd_, iov, (err || n == 0) ? 1 : 2);
}

void FuseServer::reply(uint64_t unique, int err, const std::string& payload) {
  send(unique, err, payload.data(), payload.size());
}

// ---- native opens -----------------------------------------------------------------------------
// Read-locks the blocks of a cached file that overlap [lo, hi) and lists their arena pages as
// file-offset segments.  False (nothing held) when a block is missing, busy or file-backed.
bool FuseServer::pin(const Attr& a, uint64_t lo, uint64_t hi, Handle& h) {
  uint64_t size;
  std::memcpy(&size, a.raw.data() + 8, 8);                        // fuse_attr.size
  h.size = size;
  uint64_t off = 0;
  bool ok = true;
  for (size_t i = 0; i < a.blocks.size() && ok; off += (uint64_t)a.lens[i], ++i) {
    const uint64_t blen = (uint64_t)a.lens[i];
    if (off + blen <= lo || off >= hi) continue;
    int64_t lock = -1;
    try {
      // non-waiting: a block being written/evicted goes to the python path instead
      lock = store_->lock_block(session_, a.blocks[i], false, 0);
    } catch (...) {
      lock = -1;
    }
    if (lock < 0) {
      ok = false;
      break;
    }
    h.locks.push_back(lock);
    try {
      int dir = -1;
      uint64_t ps = 0, base = 0;
      std::vector<int64_t> pages = store_->block_pages(a.blocks[i], &dir, &ps, &base);
      const DirSpec spec = store_->dir_spec(dir);
      if (spec.kind == DirKind::kFile || ps == 0 || pages.size() * ps < blen) {
        ok = false;
        break;
      }
      const bool dev = spec.kind == DirKind::kDevice;
      for (uint64_t done = 0; done < blen;) {
        const uint64_t pi = done / ps, po = done % ps;
        const uint64_t n = std::min<uint64_t>(ps - po, blen - done);
        const uint64_t src = base + (uint64_t)pages[pi] * ps + po;
        if (!h.segs.empty()) {                    // merge physically contiguous pages
          Seg& last = h.segs.back();
          if (last.src + last.len == src && last.file_off + last.len == off + done && last.device == dev) {
            last.len += n;
            done += n;
            continue;
          }
        }
        h.segs.push_back(Seg{off + done, n, src, dev});
        done += n;
      }
    } catch (...) {
      ok = false;
    }
  }
  if (!ok || (hi >= size && off < size)) {
    unpin(h);
    return false;
  }
  return true;
}

void FuseServer::unpin(Handle& h) {
  for (int64_t l : h.locks) {
    try { store_->unlock(l); } catch (...) {}
  }
  h.locks.clear();
  h.segs.clear();
}

int32_t FuseServer::passthrough_backing(const Attr& a) {
  if (!passthrough_.load() || a.blocks.size() != 1) return 0;
  std::string file;
  try {
    file = store_->committed_file(a.blocks[0]);
  } catch (...) {
    return 0;
  }
  if (file.empty()) return 0;
  const int fd = ::open(file.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return 0;                                           // evicted meanwhile
  struct stat st;
  int32_t id = 0;
  if (fstat(fd, &st) == 0 && (uint64_t)st.st_size >= (uint64_t)a.lens[0]) {
    BackingMap m{fd, 0, 0};
    const int r = ioctl(fd_, kIocBackingOpen, &m);
    if (r > 0) id = r;
  }
  ::close(fd);                                                    // the backing id holds the file
  return id;
}

bool FuseServer::native_open(uint64_t nodeid, const std::string& path, uint32_t flags, uint64_t* fh,
                             uint32_t* open_flags, int32_t* backing) {
  if (!store_ || (flags & 3) != 0) return false;                 // O_RDONLY only
  Attr a;
  if (!lookup_attr(path, a) || !a.complete || a.file_id == 0 || a.blocks.size() != a.lens.size()) return false;
  Handle h;
  uint32_t of = kFopenNoFlush;
  h.backing = passthrough_backing(a);
  if (h.backing > 0) {
    std::memcpy(&h.size, a.raw.data() + 8, 8);
    of |= kFopenPassthrough;
    passthrough_opens_++;
  } else if (!pin(a, 0, ~0ull, h)) {
    return false;
  }
  *backing = h.backing;
  try { store_->access_blocks(a.blocks); } catch (...) {}
  // passthrough opens take only PASSTHROUGH|DIRECT_IO|PARALLEL_DIRECT_WRITES|NOFLUSH (else EIO);
  // their reads use the backing file's page cache, not the FUSE inode's
  if (keep_open(nodeid, a.file_id) && h.backing <= 0) of |= kFopenKeepCache;
  {
    std::lock_guard<std::mutex> g(hmu_);
    const uint64_t id = kNativeFh | next_fh_++;
    handles_.emplace(id, std::move(h));
    *fh = id;
  }
  *open_flags = of;
  return true;
}

thread_local int FuseServer::tl_pipe_[2] = {-1, -1};

void FuseServer::add_arena(uint64_t base, uint64_t size, int fd) {
  if (running_.load()) return;                    // readers set their pipes up at start
  arenas_.push_back(Arena{base, size, fd});
}

bool FuseServer::splice_reply(const void* hdr, const std::vector<Seg>& segs) {
  if (tl_pipe_[1] < 0 || segs.empty()) return false;
  // every segment must lie in a registered shared arena (memfd): splice reads its page cache
  std::vector<std::pair<int, loff_t>> src(segs.size());
  for (size_t i = 0; i < segs.size(); ++i) {
    bool found = false;
    for (const Arena& a : arenas_)
      if (segs[i].src >= a.base && segs[i].src + segs[i].len <= a.base + a.size) {
        src[i] = {a.fd, (loff_t)(segs[i].src - a.base)};
        found = true;
        break;
      }
    if (!found) return false;
  }
  size_t total = sizeof(OutHeader);
  if (write(tl_pipe_[1], hdr, sizeof(OutHeader)) != (ssize_t)sizeof(OutHeader)) return false;
  bool ok = true;
  for (size_t i = 0; i < segs.size() && ok; ++i) {
    loff_t off = src[i].second;
    uint64_t left = segs[i].len;
    while (left > 0) {
      const ssize_t n = splice(src[i].first, &off, tl_pipe_[1], nullptr, left, 0);
      if (n <= 0) {
        ok = false;
        break;
      }
      left -= (uint64_t)n;
      total += (size_t)n;
    }
  }
  if (ok) {
    // the whole message in one splice: /dev/fuse takes one request reply per write
    const ssize_t n = splice(tl_pipe_[0], nullptr, fd_, nullptr, total, 0);
    if (n == (ssize_t)total) return true;
    if (n > 0) return true;                       // consumed (an interrupted request): nothing to redo
  }
  // drain whatever is left in the pipe so the next reply starts clean, then let writev answer
  char sink[4096];
  int fl = fcntl(tl_pipe_[0], F_GETFL);
  fcntl(tl_pipe_[0], F_SETFL, fl | O_NONBLOCK);
  while (read(tl_pipe_[0], sink, sizeof(sink)) > 0) {
  }
  fcntl(tl_pipe_[0], F_SETFL, fl);
  return false;
}

bool FuseServer::keep_open(uint64_t nodeid, int64_t file_id) {
  if (keep_cache_ == 1) return true;
  if (keep_cache_ != 2 || file_id == 0) return false;
  // the kernel inode's cached pages can only be of a file this node held before: keep them
  // unless that was another file id (the path was replaced under the same node)
  std::lock_guard<std::mutex> g(nmu_);
  auto it = last_open_fid_.find(nodeid);
  const bool keep = it == last_open_fid_.end() || it->second == file_id;
  last_open_fid_[nodeid] = file_id;
  return keep;
}

void FuseServer::release_handle(uint64_t fh) {
  Handle h;
  {
    std::lock_guard<std::mutex> g(hmu_);
    auto it = handles_.find(fh);
    if (it == handles_.end()) return;
    h = std::move(it->second);
    handles_.erase(it);
  }
  if (h.backing > 0) {
    uint32_t id = (uint32_t)h.backing;
    (void)ioctl(fd_, kIocBackingClose, &id);
  }
  unpin(h);
}

// ---- fast path --------------------------------------------------------------------------------
// Returns true when the request was fully handled (reply sent or none due).
bool FuseServer::fast(const char* req, size_t n, std::string& scratch) {
  const InHeader* ih = reinterpret_cast<const InHeader*>(req);
  const char* body = req + sizeof(InHeader);
  const size_t blen = n - sizeof(InHeader);
  const uint32_t op = ih->opcode;
  auto count = [&] { if (op < 64) native_ops_[op]++; };
  switch (op) {
    case kForget:
    case kBatchForget:
    case kInterrupt:
      count();
      return true;                                  // no reply; node ids stay valid
    case kIoctl:                                    // isatty() probes of open(): "not a terminal"
      count();
      send(ih->unique, ENOTTY, nullptr, 0);
      return true;
    case kWrite:
      if (!write_behind(req, n)) return false;
      count();
      return true;
    case kLookup: {
      if (blen == 0 || body[blen - 1] != '\0') return false;
      bool ok;
      const std::string parent = path_of(ih->nodeid, &ok);
      if (!ok) return false;
      const std::string path = child_path(parent, body);
      if (!entry_reply(path, scratch)) return false;
      count();
      send(ih->unique, 0, scratch.data(), scratch.size());
      return true;
    }
    case kGetattr: {
      bool ok;
      const std::string path = path_of(ih->nodeid, &ok);
      if (!ok) return false;
      Attr a;
      if (!lookup_attr(path, a)) return false;
      char out[sizeof(AttrOutHead) + kAttrBytes];
      AttrOutHead h{a.valid_s, 0, 0};
      std::memcpy(out, &h, sizeof(h));
      std::memcpy(out + sizeof(h), a.raw.data(), kAttrBytes);
      const uint64_t nid = ih->nodeid;
      std::memcpy(out + sizeof(h), &nid, 8);
      count();
      send(ih->unique, 0, out, sizeof(out));
      return true;
    }
    case kOpen: {
      if (blen < sizeof(OpenIn)) return false;
      const OpenIn* oi = reinterpret_cast<const OpenIn*>(body);
      bool ok;
      const std::string path = path_of(ih->nodeid, &ok);
      if (!ok) return false;
      if (no_open_.load() && (oi->flags & 3) == 0) {
        // read-only mount with FUSE_NO_OPEN_SUPPORT: ENOSYS switches the kernel to zero-message
        // opens (no OPEN/RELEASE round trips from here on; READs carry fh 0 and pin per request)
        count();
        send(ih->unique, ENOSYS, nullptr, 0);
        return true;
      }
      uint64_t fh = 0;
      uint32_t of = 0;
      int32_t backing = 0;
      if (!native_open(ih->nodeid, path, oi->flags, &fh, &of, &backing)) {
        if ((oi->flags & 3) == 0) fallback_opens_++;
        return false;
      }
      native_opens_++;
      OpenOut o{fh, of, backing};
      count();
      send(ih->unique, 0, reinterpret_cast<const char*>(&o), sizeof(o));
      return true;
    }
    case kRead: {
      if (blen < 24) return false;
      const ReadIn* ri = reinterpret_cast<const ReadIn*>(body);
      std::vector<Seg> segs;
      Handle tmp;                                   // zero-message open: blocks pinned per READ
      const bool transient = ri->fh == 0 && no_open_.load() && store_;
      if (transient) {
        bool ok;
        const std::string path = path_of(ih->nodeid, &ok);
        Attr a;
        if (!ok || !lookup_attr(path, a) || !a.complete || a.blocks.size() != a.lens.size()) return false;
        if (!pin(a, ri->offset, ri->offset + ri->size, tmp)) return false;
        if (ri->offset == 0) {
          try { store_->access_blocks(a.blocks); } catch (...) {}
        }
        const uint64_t lo = ri->offset, hi = std::min<uint64_t>(tmp.size, ri->offset + ri->size);
        for (const Seg& s : tmp.segs) {
          if (s.file_off + s.len <= lo || s.file_off >= hi) continue;
          const uint64_t x = std::max(lo, s.file_off), y = std::min(hi, s.file_off + s.len);
          segs.push_back(Seg{x, y - x, s.src + (x - s.file_off), s.device});
        }
      } else {
        if (!(ri->fh & kNativeFh)) return false;
        std::lock_guard<std::mutex> g(hmu_);
        auto it = handles_.find(ri->fh);
        if (it == handles_.end()) {
          send(ih->unique, EBADF, nullptr, 0);
          count();
          return true;
        }
        const uint64_t lo = ri->offset, hi = std::min<uint64_t>(it->second.size, ri->offset + ri->size);
        for (const Seg& s : it->second.segs) {
          if (s.file_off + s.len <= lo || s.file_off >= hi) continue;
          const uint64_t x = std::max(lo, s.file_off), y = std::min(hi, s.file_off + s.len);
          segs.push_back(Seg{x, y - x, s.src + (x - s.file_off), s.device});
        }
      }
      // the handle's (or this request's) block locks keep every page in place during the copy
      uint64_t total = 0;
      for (const Seg& s : segs) total += s.len;
      OutHeader h{(uint32_t)(sizeof(OutHeader) + total), 0, ih->unique};
      bool any_dev = false;
      for (const Seg& s : segs) any_dev |= s.device;
      bool failed = false;
      const auto tw = std::chrono::steady_clock::now();
      if (!any_dev && splice_reply(&h, segs)) {
        // shared DRAM arena: its pages spliced into the reply (no user-page pinning per 4 KiB)
      } else if (!any_dev && segs.size() < 15) {    // DRAM arena: zero-copy gather into the reply
        iovec iov[16];
        iov[0] = {&h, sizeof(h)};
        for (size_t i = 0; i < segs.size(); ++i) iov[i + 1] = {reinterpret_cast<void*>(segs[i].src), segs[i].len};
        (void)!writev(fd_, iov, (int)segs.size() + 1);
      } else {
        scratch.resize(sizeof(OutHeader) + total);
        std::memcpy(&scratch[0], &h, sizeof(h));
        char* dst = &scratch[sizeof(OutHeader)];
        for (const Seg& s : segs) {
          if (s.device) {
            if (hipMemcpy(dst, reinterpret_cast<const void*>(s.src), s.len, hipMemcpyDeviceToHost) != hipSuccess) {
              failed = true;
              break;
            }
          } else {
            std::memcpy(dst, reinterpret_cast<const void*>(s.src), s.len);
          }
          dst += s.len;
        }
        if (failed) send(ih->unique, EIO, nullptr, 0);
        else (void)!write(fd_, scratch.data(), scratch.size());
      }
      native_ns_[63] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                            std::chrono::steady_clock::now() - tw).count();   // reply time (stats()[191])
      if (transient) unpin(tmp);
      native_reads_++;
      count();
      return true;
    }
    case kFlush: {
      if (blen < sizeof(FlushIn)) return false;
      const FlushIn* fi = reinterpret_cast<const FlushIn*>(body);
      if (fi->fh == 0 && no_open_.load()) {
        // read-only mount: nothing to flush, and ENOSYS stops FLUSH requests for good
        count();
        send(ih->unique, ENOSYS, nullptr, 0);
        return true;
      }
      if (!(fi->fh & kNativeFh)) return false;
      count();
      send(ih->unique, 0, nullptr, 0);
      return true;
    }
    case kRelease: {
      if (blen < sizeof(ReleaseIn)) return false;
      const ReleaseIn* ri = reinterpret_cast<const ReleaseIn*>(body);
      if (!(ri->fh & kNativeFh)) return false;
      release_handle(ri->fh);
      count();
      send(ih->unique, 0, nullptr, 0);
      return true;
    }
    default:
      return false;
  }
}

void FuseServer::loop(int idx) {
  {
    char name[16];
    snprintf(name, sizeof(name), "fuse-rd-%d", idx);
    pthread_setname_np(pthread_self(), name);
  }
  std::vector<char> buf(kBufSize);
  std::string scratch;
  tl_pipe_[0] = tl_pipe_[1] = -1;
  int pfd[2];
  if (!arenas_.empty() && !getenv("ALLUXIO_FUSE_NO_SPLICE") && pipe2(pfd, O_CLOEXEC) == 0) {
    if (fcntl(pfd[1], F_SETPIPE_SZ, (int)kPipeSize) >= (int)(kPipeSize / 2)) {
      tl_pipe_[0] = pfd[0];
      tl_pipe_[1] = pfd[1];
    } else {
      close(pfd[0]);
      close(pfd[1]);
    }
  }
  while (running_.load() && !dead_.load()) {
    // the fd is non-blocking: take a queued request at once, sleep in poll() only when none is
    // queued (a busy mount skips one syscall per request).  Spinning instead of sleeping was
    // measured slower: the readers compete with the application for CPUs.
    ssize_t n = ::read(fd_, buf.data(), buf.size());
    if (n < 0 && errno == EAGAIN) {
      pollfd p{fd_, POLLIN, 0};
      const int pr = ::poll(&p, 1, 200);
      if (pr < 0 && errno != EINTR) break;
      if (pr > 0 && (p.revents & (POLLERR | POLLHUP | POLLNVAL))) break;
      continue;
    }
    if (n < 0) {
      if (errno == EINTR || errno == ENOENT) continue;
      break;                                        // ENODEV / EBADF: unmounted
    }
    if ((size_t)n < sizeof(InHeader)) continue;
    try {
      const auto t0 = std::chrono::steady_clock::now();
      if (fast(buf.data(), (size_t)n, scratch)) {
        const uint32_t op = reinterpret_cast<const InHeader*>(buf.data())->opcode;
        if (op < 64)
          native_ns_[op] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                std::chrono::steady_clock::now() - t0).count();
        continue;
      }
    } catch (...) {
      // fall through to the python path
    }
    const InHeader* ih = reinterpret_cast<const InHeader*>(buf.data());
    if ((ih->opcode == kFlush || ih->opcode == kRelease || ih->opcode == kFsync) &&
        (size_t)n >= sizeof(InHeader) + 8) {
      uint64_t fh;                                  // the handle's buffered writes go first
      std::memcpy(&fh, buf.data() + sizeof(InHeader), 8);
      flush_handle(fh);
    }
    if (ih->opcode < 64) python_ops_[ih->opcode]++;
    FuseRequest r{ih->unique, ih->opcode, ih->nodeid, ih->uid, ih->gid, ih->pid,
                  std::string(buf.data() + sizeof(InHeader), (size_t)n - sizeof(InHeader))};
    {
      std::lock_guard<std::mutex> g(qmu_);
      queue_.push_back(std::move(r));
    }
    qcv_.notify_one();
  }
  if (tl_pipe_[0] >= 0) {
    close(tl_pipe_[0]);
    close(tl_pipe_[1]);
  }
  dead_.store(true);                                // the connection is gone: wake the python side
  wb_cv_.notify_all();
  qcv_.notify_all();
}

}  // namespace amdx
