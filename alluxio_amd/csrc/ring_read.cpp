#include "ring_read.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>

#include "kernels.h"

namespace amdx {

#define RR_HIP(expr)                                                                           \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess)                                                                      \
      throw StoreError(kErrHip, std::string("HIP error: ") + hipGetErrorString(_e) + " at " #expr); \
  } while (0)

RingReadSession::RingReadSession(BlockStore* store, int64_t session, const std::vector<int64_t>& block_ids,
                                 const std::vector<uint64_t>& block_lens, uint64_t dst_base,
                                 uint64_t stream_stride, uint64_t buf_bytes, uint32_t depth, uint32_t streams,
                                 int dst_kind, const std::vector<uint64_t>& start_offsets)
    : store_(store), session_(session), blocks_(block_ids), buf_(buf_bytes), stride_(stream_stride),
      dst_(dst_base), depth_(depth), streams_(streams), kind_(dst_kind) {
  if (block_ids.size() != block_lens.size() || block_ids.empty())
    throw StoreError(kErrInvalidArgument, "ring read: bad block list");
  for (uint64_t l : block_lens) file_len_ += l;
  check_shape();
  // lock every block (read) and build the file page table
  try {
    for (size_t b = 0; b < blocks_.size(); ++b) {
      locks_.push_back(store_->lock_block(session_, blocks_[b], false, -1));
      int dir = -1;
      uint64_t ps = 0, base = 0;
      std::vector<int64_t> pages = store_->block_pages(blocks_[b], &dir, &ps, &base);
      const DirSpec spec = store_->dir_spec(dir);
      if (spec.kind == DirKind::kFile) throw StoreError(kErrInvalidArgument, "ring read: block in a file tier");
      if (dir_ < 0) {
        dir_ = dir;
        page_size_ = ps;
        arena_ = base;
        if (ps & (ps - 1)) throw StoreError(kErrInvalidArgument, "ring read: page size must be a power of two");
        while ((1ull << page_shift_) < ps) ++page_shift_;
      } else if (dir != dir_) {
        throw StoreError(kErrInvalidArgument, "ring read: blocks span several dirs");
      }
      const uint64_t np = (block_lens[b] + ps - 1) / ps;
      if (b + 1 < blocks_.size() && block_lens[b] % ps != 0)
        throw StoreError(kErrInvalidArgument, "ring read: block size must be a multiple of the page size");
      if (pages.size() < np) throw StoreError(kErrInvalidState, "ring read: block shorter than its length");
      ftab_.insert(ftab_.end(), pages.begin(), pages.begin() + np);
    }
    on_device_ = store_->has_device();
    finish_init(start_offsets);
  } catch (...) {
    for (int64_t l : locks_) store_->unlock(l);
    locks_.clear();
    throw;
  }
}

RingReadSession::RingReadSession(uint64_t arena_base, const std::vector<int64_t>& file_pages, uint64_t page_size,
                                 uint64_t file_len, int device, uint64_t dst_base, uint64_t stream_stride,
                                 uint64_t buf_bytes, uint32_t depth, uint32_t streams, int dst_kind,
                                 const std::vector<uint64_t>& start_offsets)
    : store_(nullptr), session_(0), file_len_(file_len), buf_(buf_bytes), stride_(stream_stride), dst_(dst_base),
      depth_(depth), streams_(streams), kind_(dst_kind), on_device_(device >= 0), device_(device),
      page_size_(page_size), arena_(arena_base), ftab_(file_pages) {
  check_shape();
  if (page_size_ == 0 || (page_size_ & (page_size_ - 1)))
    throw StoreError(kErrInvalidArgument, "ring read: page size must be a power of two");
  while ((1ull << page_shift_) < page_size_) ++page_shift_;
  if (ftab_.size() < (file_len_ + page_size_ - 1) / page_size_)
    throw StoreError(kErrInvalidArgument, "ring read: page table shorter than the file");
  finish_init(start_offsets);
}

void RingReadSession::check_shape() {
  if (buf_ == 0 || depth_ == 0 || streams_ == 0 || streams_ > kSeqReadMaxStreams)
    throw StoreError(kErrInvalidArgument, "ring read: bad buffer/depth/stream count");
  if (stride_ < (uint64_t)depth_ * buf_) throw StoreError(kErrInvalidArgument, "ring read: stride too small");
  if (file_len_ == 0) throw StoreError(kErrInvalidArgument, "ring read: empty file");
  const uint64_t calls = (file_len_ + buf_ - 1) / buf_;
  if (calls + 1 >= (1ull << 32)) throw StoreError(kErrInvalidArgument, "ring read: too many calls per pass");
  cycle_ = (uint32_t)(calls + 1);
}

void RingReadSession::set_device() const {
  if (store_) store_->use_device();
  else if (device_ >= 0) RR_HIP(hipSetDevice(device_));
}

void RingReadSession::finish_init(const std::vector<uint64_t>& start_offsets) {
  c_init_.assign(streams_, 0);
  for (uint32_t s = 0; s < streams_ && s < start_offsets.size(); ++s) {
    if (start_offsets[s] % buf_) throw StoreError(kErrInvalidArgument, "ring read: start offsets must be buffer aligned");
    c_init_[s] = std::min<uint64_t>(start_offsets[s] / buf_, cycle_ - 1);
  }
  // streams that start at distinct calls read distinct bytes each step (lockstep streams re-read
  // the same depth*buf window): the kernel's cache policy keys on this footprint
  std::vector<uint64_t> starts(c_init_);
  std::sort(starts.begin(), starts.end());
  const uint64_t distinct = (uint64_t)(std::unique(starts.begin(), starts.end()) - starts.begin());
  footprint_ = std::min<uint64_t>(file_len_, distinct * depth_ * buf_);
  if (on_device_) {
    if (buf_ & 15 || stride_ & 15 || dst_ & 15)
      throw StoreError(kErrInvalidArgument, "ring read: buffer size, stride and ring base must be 16-byte aligned");
    set_device();
    RR_HIP(hipMalloc((void**)&d_ftab_, ftab_.size() * sizeof(int64_t)));
    RR_HIP(hipMalloc((void**)&d_cinit_, c_init_.size() * sizeof(uint64_t)));
    RR_HIP(hipMemcpy(d_ftab_, ftab_.data(), ftab_.size() * sizeof(int64_t), hipMemcpyHostToDevice));
    RR_HIP(hipMemcpy(d_cinit_, c_init_.data(), c_init_.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
  }
}

RingReadSession::~RingReadSession() {
  try {
    close();
  } catch (...) {
  }
}

void RingReadSession::close() {
  if (closed_) return;
  closed_ = true;
  if (d_ftab_) (void)hipFree(d_ftab_);
  if (d_cinit_) (void)hipFree(d_cinit_);
  d_ftab_ = nullptr;
  d_cinit_ = nullptr;
  for (int64_t l : locks_) {
    try {
      if (store_) store_->unlock(l);
    } catch (...) {
    }
  }
  locks_.clear();
}

uint64_t RingReadSession::bytes_before(uint64_t g) const {
  const uint64_t passes = g / cycle_, rem = g % cycle_;
  return passes * file_len_ + std::min<uint64_t>(rem * buf_, file_len_);
}

uint64_t RingReadSession::step(uint64_t stream, uint64_t* eofs) {
  if (closed_) throw StoreError(kErrInvalidState, "ring read session closed");
  const uint64_t base = calls_per_stream_;
  if (on_device_) {
    set_device();
    SeqReadArgs a;
    a.arena = reinterpret_cast<const uint8_t*>(arena_);
    a.ftab = d_ftab_;
    a.c_init = d_cinit_;
    a.dst = reinterpret_cast<uint8_t*>(dst_);
    a.stream_stride = stride_;
    a.file_len = file_len_;
    a.buf = buf_;
    a.launch_base = base;
    a.cycle = cycle_;
    a.streams = streams_;
    a.depth = depth_;
    a.page_shift = page_shift_;
    a.footprint = footprint_;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    RR_HIP(launch_seq_read(a, st));
    if (kind_ == (int)MemKind::kHost) RR_HIP(hipStreamSynchronize(st));
  } else {
    // CPU-only build/test path: same schedule with memcpy from the host arena
    for (uint32_t s = 0; s < streams_; ++s)
      for (uint32_t k = 0; k < depth_; ++k) {
        auto [off, len] = std::pair<uint64_t, uint64_t>(0, 0);
        const uint64_t c = (c_init_[s] + base + k) % cycle_;
        if (c == cycle_ - 1) continue;
        off = c * buf_;
        len = std::min(buf_, file_len_ - off);
        uint8_t* d = reinterpret_cast<uint8_t*>(dst_ + s * stride_ + (uint64_t)k * buf_);
        uint64_t done = 0;
        while (done < len) {
          const uint64_t fo = off + done;
          const uint64_t po = fo & (page_size_ - 1);
          const uint64_t take = std::min(len - done, page_size_ - po);
          std::memcpy(d + done,
                      reinterpret_cast<const uint8_t*>(arena_ + ((uint64_t)ftab_[fo >> page_shift_] << page_shift_) + po),
                      take);
          done += take;
        }
      }
  }
  uint64_t bytes = 0, eof = 0;
  for (uint32_t s = 0; s < streams_; ++s) {
    const uint64_t g0 = c_init_[s] + base, g1 = g0 + depth_;
    bytes += bytes_before(g1) - bytes_before(g0);
    eof += g1 / cycle_ - g0 / cycle_;
  }
  calls_per_stream_ += depth_;
  total_ += bytes;
  reopens_ += eof;
  if (store_) store_->access_blocks(blocks_);
  if (eofs) *eofs = eof;
  return bytes;
}

uint64_t RingReadSession::position(uint32_t s) const {
  const uint64_t c = (c_init_.at(s) + calls_per_stream_) % cycle_;
  return std::min<uint64_t>(c * buf_, file_len_);
}

std::pair<uint64_t, uint64_t> RingReadSession::last_call(uint32_t s, uint32_t k) const {
  if (calls_per_stream_ < depth_) return {0, 0};
  const uint64_t c = (c_init_.at(s) + calls_per_stream_ - depth_ + k) % cycle_;
  if (c == cycle_ - 1) return {file_len_, 0};
  const uint64_t off = c * buf_;
  return {off, std::min(buf_, file_len_ - off)};
}

}  // namespace amdx
