#include "block_store.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <thread>
#include <chrono>
#include <cmath>
#include <cstring>
#include <sstream>

#include "cpu_codecs.h"
#include "trace.h"

namespace amdx {

#define HIP_OK(expr)                                                                       \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess)                                                                  \
      throw StoreError(kErrHip, std::string("HIP error: ") + hipGetErrorString(_e) + " at " \
                                    + #expr);                                              \
  } while (0)

static inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

uint64_t StorageDir::available() const {
  if (!healthy) return 0;
  if (spec.kind == DirKind::kFile) {
    const uint64_t cap = spec.capacity > spec.reserved ? spec.capacity - spec.reserved : 0;
    return file_used >= cap ? 0 : cap - file_used;
  }
  return free_pages > reserved_pages ? (uint64_t)(free_pages - reserved_pages) * spec.page_size : 0;
}

uint64_t StorageDir::mgmt_available() const {
  if (!healthy) return 0;
  if (spec.kind == DirKind::kFile) return file_used >= spec.capacity ? 0 : spec.capacity - file_used;
  return (uint64_t)free_pages * spec.page_size;
}

// User-visible capacity: the reserved space is management headroom, not capacity.
uint64_t StorageDir::capacity() const {
  if (spec.kind == DirKind::kFile) return spec.capacity > spec.reserved ? spec.capacity - spec.reserved : 0;
  return (uint64_t)(num_pages - reserved_pages) * spec.page_size;
}

// -------------------------------------------------------------------------------------------
BlockStore::BlockStore(const std::vector<DirSpec>& dirs, int annotator, int alloc_policy,
                       float lrfu_step, float lrfu_attenuation, int device)
    : annotator_(static_cast<Annotator>(annotator)),
      alloc_policy_(static_cast<AllocPolicy>(alloc_policy)),
      lrfu_step_(lrfu_step),
      lrfu_att_(lrfu_attenuation),
      device_(device) {
  int max_tier = 0;
  for (size_t i = 0; i < dirs.size(); ++i) {
    auto d = std::make_unique<StorageDir>();
    d->spec = dirs[i];
    d->index = (int)i;
    if (d->spec.kind != DirKind::kFile) {
      if (d->spec.page_size == 0) throw StoreError(kErrInvalidArgument, "page size must be > 0");
      if (d->spec.base == 0 && d->spec.capacity >= d->spec.page_size)
        throw StoreError(kErrInvalidArgument, "arena dir " + std::to_string(i) + " has no base address");
      d->num_pages = (int64_t)(d->spec.capacity / d->spec.page_size);
      d->reserved_pages = std::min<int64_t>(d->num_pages, (int64_t)ceil_div(d->spec.reserved, d->spec.page_size));
      d->free_bits.assign(ceil_div((uint64_t)d->num_pages, 64), 0);
      for (int64_t p = 0; p < d->num_pages; ++p) d->free_bits[p >> 6] |= 1ull << (p & 63);
      d->free_pages = d->num_pages;
      if (d->spec.kind == DirKind::kDevice) has_device_ = true;
    } else {
      ::mkdir(d->spec.path.c_str(), 0755);
      ::mkdir((d->spec.path + "/.tmp_blocks").c_str(), 0755);
    }
    max_tier = std::max(max_tier, d->spec.tier);
    dirs_.push_back(std::move(d));
  }
  rr_index_.assign(max_tier + 1, 0);
  dir_ev_bytes_.assign(dirs_.size(), 0);
  if (has_device_) {
    set_device();
    HIP_OK(hipStreamCreateWithFlags(&internal_stream_, hipStreamNonBlocking));
    for (int i = 0; i < 2; ++i) HIP_OK(hipEventCreateWithFlags(&upd_ev_[i], hipEventDisableTiming));
    HIP_OK(hipHostMalloc((void**)&h_ctl_, sizeof(EvictCtl), hipHostMallocDefault));
    HIP_OK(hipMalloc((void**)&d_ctl_, sizeof(EvictCtl)));
    HIP_OK(hipHostMalloc((void**)&h_claimed_, sizeof(uint32_t), hipHostMallocDefault));
    HIP_OK(hipMalloc((void**)&d_claimed_, sizeof(uint32_t)));
    HIP_OK(hipHostMalloc((void**)&host_ring_, sizeof(CopySeg) * kRing * kRingSegs, hipHostMallocDefault));
    HIP_OK(hipMalloc((void**)&dev_ring_, sizeof(CopySeg) * kRing * kRingSegs));
    for (int i = 0; i < kRing; ++i) HIP_OK(hipEventCreateWithFlags(&ring_ev_[i], hipEventDisableTiming));
    for (auto& d : dirs_) {
      if (d->spec.kind != DirKind::kDevice || d->free_bits.empty()) continue;
      HIP_OK(hipMalloc((void**)&d->mag_bits, d->free_bits.size() * 8));
      HIP_OK(hipMemset(d->mag_bits, 0, d->free_bits.size() * 8));
    }
    const char* mk = std::getenv("ALLUXIO_MOVE_COPY_KERNEL");
    const bool mapped_moves = !(mk && mk[0] == '0');
    for (auto& d : dirs_) {
      if (!mapped_moves || d->spec.kind != DirKind::kHost || !d->spec.base || !d->spec.capacity) continue;
      void* dp = nullptr;
      if (hipHostGetDevicePointer(&dp, reinterpret_cast<void*>(d->spec.base), 0) == hipSuccess && dp)
        d->dev_base = reinterpret_cast<uint64_t>(dp);
      else
        (void)hipGetLastError();      // not registered: tier moves use runtime copies
    }
  }
}

namespace {
std::atomic<uint64_t> g_thread_streams{0};

struct ThreadStreams {
  std::vector<std::pair<int, hipStream_t>> by_device;
  ~ThreadStreams() {
    for (auto& kv : by_device) (void)hipStreamDestroy(kv.second);
  }
};
}  // namespace

hipStream_t thread_stream_on(int device) {
  thread_local ThreadStreams tl;
  for (auto& kv : tl.by_device)
    if (kv.first == device) return kv.second;
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (prev != device) HIP_OK(hipSetDevice(device));
  hipStream_t st = nullptr;
  const hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  if (prev != device && prev >= 0) (void)hipSetDevice(prev);
  HIP_OK(e);
  tl.by_device.emplace_back(device, st);
  g_thread_streams.fetch_add(1, std::memory_order_relaxed);
  return st;
}

uint64_t thread_streams_created() { return g_thread_streams.load(std::memory_order_relaxed); }

hipStream_t BlockStore::move_stream() {
  // this thread's stream on the store's device: concurrent evictions move in parallel and never
  // queue behind the page-claim / eviction-select kernels on internal_stream_; keyed by device
  // (not store), so a thread that serves many stores keeps one stream per device
  set_device();
  return thread_stream_on(device_);
}

BlockStore::~BlockStore() {
  if (has_device_) {
    hipSetDevice(device_);
    for (int i = 0; i < kRing; ++i)
      if (ring_ev_[i]) hipEventDestroy(ring_ev_[i]);
    if (host_ring_) hipHostFree(host_ring_);
    if (dev_ring_) hipFree(dev_ring_);
    if (ingest_dev_) hipFree(ingest_dev_);
    for (int i = 0; i < 2; ++i) {
      if (upd_ev_[i]) hipEventDestroy(upd_ev_[i]);
      if (h_upd_[i]) hipHostFree(h_upd_[i]);
    }
    for (void* p : {(void*)d_crf_, (void*)d_last_, (void*)d_fbytes_, (void*)d_dir_, (void*)d_keys_,
                    (void*)d_excl_, (void*)d_ctl_, (void*)d_upd_, (void*)d_bits_, (void*)d_partial_,
                    (void*)d_claimed_})
      if (p) hipFree(p);
    for (void* p : {(void*)h_excl_, (void*)h_ctl_, (void*)h_out_, (void*)h_pages_, (void*)h_claimed_})
      if (p) hipHostFree(p);
    if (crc_dev_) hipFree(crc_dev_);
    for (auto& d : dirs_) {
      if (d->mag_bits) hipFree(d->mag_bits);
      if (d->mag_upd) hipFree(d->mag_upd);
      // the HBM arena lives exactly as long as the store that hands out its pages
      if (d->spec.owns_base && d->spec.kind == DirKind::kDevice && d->spec.base) {
        (void)hipDeviceSynchronize();
        (void)hipFree(reinterpret_cast<void*>(d->spec.base));
      }
    }
    for (ClaimScratch* cp : {&claim_[0], &claim_[1], &claim_one_}) {
      ClaimScratch& c = *cp;
      for (void* p : {(void*)c.items_d, (void*)c.pages_d, (void*)c.got_d})
        if (p) hipFree(p);
      for (void* p : {(void*)c.items_h, (void*)c.pages_h, (void*)c.got_h})
        if (p) hipHostFree(p);
    }
    if (internal_stream_) hipStreamDestroy(internal_stream_);
  }
}

void BlockStore::set_device() const {
  if (has_device_) {
    // hipSetDevice takes a runtime lock that concurrent copies hold (1.5 ms per cold read with four
    // streams at once, profiles/r6_cold_read.md); the current device is a thread-local read
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur == device_) return;
    hipError_t e = hipSetDevice(device_);
    if (e != hipSuccess) throw StoreError(kErrHip, std::string("hipSetDevice: ") + hipGetErrorString(e));
  }
}

hipStream_t BlockStore::stream_or_default(uint64_t s) const {
  return s ? reinterpret_cast<hipStream_t>(s) : internal_stream_;
}

// -------------------------------------------------------------------------------------------
// metadata helpers
BlockMeta* BlockStore::find(int64_t id) {
  auto it = blocks_.find(id);
  return it == blocks_.end() ? nullptr : &it->second;
}

BlockMeta& BlockStore::get_committed(int64_t id) {
  BlockMeta* b = find(id);
  if (!b || b->temp) throw StoreError(kErrNotFound, "block " + std::to_string(id) + " does not exist");
  return *b;
}

bool BlockStore::dir_matches(const StorageDir& d, int tier, const std::string& medium) const {
  if (!d.healthy) return false;
  if (tier >= 0 && d.spec.tier != tier) return false;
  if (!medium.empty() && d.spec.medium != medium) return false;
  return true;
}

uint32_t BlockStore::alloc_slot() {
  if (!free_slots_.empty()) {
    const uint32_t s = free_slots_.back();
    free_slots_.pop_back();
    return s;
  }
  crf_.push_back(0.f);
  last_.push_back(0);
  slot_block_.push_back(0);
  slot_dir_.push_back(-1);
  slot_fb_.push_back(0);
  dirty_flag_.push_back(0);
  return (uint32_t)(crf_.size() - 1);
}

void BlockStore::mark_dirty(uint32_t slot) {
  if (!device_evict_active() || dirty_flag_[slot]) return;
  dirty_flag_[slot] = 1;
  dirty_.push_back(slot);
  if (dirty_.size() >= 65536) flush_annotations_locked();   // bound the host queue (async)
}

void BlockStore::touch_slot(uint32_t slot) {
  const uint64_t now = ++clock_;
  if (annotator_ == Annotator::kLRFU) {
    const double age = (double)(now - last_[slot]);
    crf_[slot] = (float)(crf_[slot] * std::pow(1.0 / lrfu_att_, age * lrfu_step_) + 1.0);
  }
  last_[slot] = now;
  mark_dirty(slot);
}

// Page-rounded footprint: what evicting the block gives back to its dir.
uint64_t BlockStore::footprint(const BlockMeta& b) const {
  const StorageDir& d = *dirs_[b.dir];
  if (d.spec.kind == DirKind::kFile) return std::max(b.length, b.reserved);
  return (uint64_t)b.pages.size() * d.spec.page_size;
}

// Static evictability (committed, not pinned) and footprint of a slot changed; `live` = false
// when the block is going away.  Keeps dir_ev_bytes_ and the device mirror current.
void BlockStore::note_state(const BlockMeta& b, bool live) {
  int32_t nd = -1;
  uint64_t nf = 0;
  if (live && !b.temp && !b.pinned_on_create) {
    const int64_t file_id = (int64_t)(((uint64_t)b.id & ~0xFFFFFFull) | 0xFFFFFFull);
    if (pinned_files_.find(file_id) == pinned_files_.end()) {
      nd = b.dir;
      nf = footprint(b);
    }
  }
  const uint32_t s = b.slot;
  if (slot_dir_[s] >= 0) dir_ev_bytes_[slot_dir_[s]] -= std::min(dir_ev_bytes_[slot_dir_[s]], slot_fb_[s]);
  if (nd >= 0) dir_ev_bytes_[nd] += nf;
  slot_dir_[s] = nd;
  slot_fb_[s] = nf;
  mark_dirty(s);
}

bool BlockStore::evictable(const BlockMeta& b) const {
  if (b.temp || b.readers > 0 || b.writer || b.evicting || b.pinned_on_create) return false;
  // file id = container id with the max 24-bit sequence number (reference BlockId.getFileId)
  const int64_t file_id = (int64_t)(((uint64_t)b.id & ~0xFFFFFFull) | 0xFFFFFFull);
  return pinned_files_.find(file_id) == pinned_files_.end();
}

void BlockStore::emit(int kind, const BlockMeta& b) {
  const auto& d = dirs_[b.dir]->spec;
  events_.push_back(Event{kind, b.id, d.tier_alias, d.medium});
}

void BlockStore::file_path(const StorageDir& d, int64_t id, std::string& out) const {
  out = d.spec.path + "/" + std::to_string(id);
}

// -------------------------------------------------------------------------------------------
// page allocation
static bool bit_free(const std::vector<uint64_t>& bits, int64_t p) { return (bits[p >> 6] >> (p & 63)) & 1; }
static void bit_take(std::vector<uint64_t>& bits, int64_t p) { bits[p >> 6] &= ~(1ull << (p & 63)); }
static void bit_give(std::vector<uint64_t>& bits, int64_t p) { bits[p >> 6] |= 1ull << (p & 63); }

// First run of `n` free pages (returns -1 if none).
static int64_t find_run(const std::vector<uint64_t>& bits, int64_t num_pages, int64_t n) {
  int64_t run = 0, start = 0;
  for (int64_t w = 0; w < (int64_t)bits.size(); ++w) {
    const uint64_t word = bits[w];
    if (word == 0) { run = 0; continue; }
    if (word == ~0ull && (w + 1) * 64 <= num_pages) {
      if (run == 0) start = w * 64;
      run += 64;
      if (run >= n) return start;
      continue;
    }
    for (int b = 0; b < 64; ++b) {
      const int64_t p = w * 64 + b;
      if (p >= num_pages) break;
      if ((word >> b) & 1) {
        if (run == 0) start = p;
        if (++run >= n) return start;
      } else {
        run = 0;
      }
    }
  }
  return -1;
}

bool BlockStore::grow_pages(StorageDir& d, BlockMeta& b, uint64_t new_reserved, bool use_reserved) {
  if (d.spec.kind == DirKind::kFile) {
    const uint64_t add = new_reserved > b.reserved ? new_reserved - b.reserved : 0;
    if (add > (use_reserved ? d.mgmt_available() : d.available())) return false;
    d.file_used += add;
    b.reserved = std::max(b.reserved, new_reserved);
    return true;
  }
  const int64_t want = (int64_t)ceil_div(new_reserved, d.spec.page_size);
  int64_t need = want - (int64_t)b.pages.size();
  if (need <= 0) {
    b.reserved = std::max(b.reserved, new_reserved);
    return true;
  }
  if (need > d.free_pages - (use_reserved ? 0 : d.reserved_pages)) return false;
  // 1) extend the block's current run in place
  if (!b.pages.empty()) {
    int64_t p = b.pages.back() + 1;
    while (need > 0 && p < d.num_pages && bit_free(d.free_bits, p)) {
      bit_take(d.free_bits, p);
      b.pages.push_back(p++);
      --d.free_pages;
      --need;
    }
  }
  // 2) a fresh contiguous run
  if (need > 0) {
    const int64_t s = find_run(d.free_bits, d.num_pages, need);
    if (s >= 0) {
      for (int64_t p = s; p < s + need; ++p) {
        bit_take(d.free_bits, p);
        b.pages.push_back(p);
      }
      d.free_pages -= need;
      need = 0;
    }
  }
  // 3) scattered pages (the device magazine handed back first when the host pool runs dry)
  for (int pass = 0; pass < 2 && need > 0; ++pass) {
    if (pass == 1) {
      if (d.mag_pages <= 0 || !d.mag_bits) break;
      mag_drain(d);
    }
    for (int64_t w = 0; need > 0 && w < (int64_t)d.free_bits.size(); ++w) {
      uint64_t word = d.free_bits[w];
      while (word && need > 0) {
        const int b0 = __builtin_ctzll(word);
        const int64_t p = w * 64 + b0;
        if (p >= d.num_pages) break;
        bit_take(d.free_bits, p);
        b.pages.push_back(p);
        --d.free_pages;
        --need;
        word &= word - 1;
      }
    }
  }
  b.reserved = std::max(b.reserved, new_reserved);
  return need == 0;
}

// ---- K7 device magazine -----------------------------------------------------------------------
// Moves >= want free pages (whole host bitmap words at a time: no per-page host work) into the
// device bitmap (done when this returns).
void BlockStore::mag_refill(StorageDir& d, int64_t want) {
  if (!d.mag_bits || want <= 0) return;
  const int64_t nwords = (int64_t)d.free_bits.size();
  std::vector<uint64_t> upd;
  int64_t moved = 0;
  const int64_t start = d.mag_cursor;
  for (int64_t k = 0; k < nwords && moved < want; ++k) {
    const int64_t w = (start + k) % nwords;
    uint64_t word = d.free_bits[w];
    if (!word) continue;
    if ((w + 1) * 64 > d.num_pages) {             // tail word: only real pages
      const int64_t valid = d.num_pages - w * 64;
      word &= valid >= 64 ? ~0ull : ((1ull << valid) - 1);
      if (!word) continue;
    }
    d.free_bits[w] &= ~word;
    if (d.mag_lo < 0) d.mag_lo = w;
    upd.push_back((uint64_t)w);
    upd.push_back(word);
    moved += __builtin_popcountll(word);
    d.mag_cursor = (w + 1) % nwords;
  }
  if (upd.empty()) return;
  const size_t n = upd.size() / 2;
  if (d.mag_upd_cap < upd.size()) {
    if (d.mag_upd) hipFree(d.mag_upd);
    d.mag_upd = nullptr;
    const size_t cap = std::max<size_t>(upd.size(), 1024);
    HIP_OK(hipMalloc((void**)&d.mag_upd, cap * 8));
    d.mag_upd_cap = cap;
  }
  // on the internal stream, completed before returning: the (pageable) update list is consumed
  // and any stream claiming afterwards sees the pages
  HIP_OK(hipMemcpyAsync(d.mag_upd, upd.data(), upd.size() * 8, hipMemcpyHostToDevice, internal_stream_));
  HIP_OK(launch_mag_fill(d.mag_bits, (uint32_t)nwords, d.mag_upd, (uint32_t)n, internal_stream_));
  HIP_OK(hipStreamSynchronize(internal_stream_));
  d.mag_pages += moved;
  ++stats_.mag_refills;
  stats_.mag_refill_pages += moved;
}

// Words holding the magazine's bits: the arc [mag_lo, mag_cursor) refills filled since the last
// drain (the whole bitmap once the cursor wrapped onto it); (0, 0) = the whole bitmap.
std::pair<uint32_t, uint32_t> BlockStore::mag_window(const StorageDir& d) const {
  const int64_t nwords = (int64_t)d.free_bits.size();
  if (d.mag_lo < 0 || nwords == 0) return {0u, 0u};
  const int64_t len = ((d.mag_cursor - d.mag_lo) % nwords + nwords) % nwords;
  if (len == 0) return {0u, 0u};
  return {(uint32_t)d.mag_lo, (uint32_t)len};
}

// Hands every page left in the magazine back to the host pool (atomic exchange per word, so a
// claim running concurrently on another stream still owns exactly the bits it won).
int64_t BlockStore::mag_drain(StorageDir& d) {
  if (!d.mag_bits) return 0;
  const uint32_t nwords = (uint32_t)d.free_bits.size();
  uint64_t* dout = nullptr;
  HIP_OK(hipMalloc((void**)&dout, (size_t)nwords * 8));
  std::vector<uint64_t> out(nwords);
  hipError_t e = launch_mag_drain(d.mag_bits, nwords, dout, internal_stream_);
  if (e == hipSuccess) e = hipMemcpyAsync(out.data(), dout, (size_t)nwords * 8, hipMemcpyDeviceToHost, internal_stream_);
  if (e == hipSuccess) e = hipStreamSynchronize(internal_stream_);
  hipFree(dout);
  if (e != hipSuccess) throw StoreError(kErrHip, std::string("magazine drain: ") + hipGetErrorString(e));
  int64_t back = 0;
  for (uint32_t w = 0; w < nwords; ++w) {
    d.free_bits[w] |= out[w];
    back += __builtin_popcountll(out[w]);
  }
  d.mag_pages -= back;
  d.mag_lo = -1;
  ++stats_.mag_drains;
  stats_.mag_drain_pages += back;
  return back;
}

void BlockStore::release_storage(BlockMeta& b) {
  StorageDir& d = *dirs_[b.dir];
  if (d.spec.kind == DirKind::kFile) {
    d.file_used -= std::min(d.file_used, b.reserved);
    std::string p;
    if (b.temp) {
      p = d.spec.path + "/.tmp_blocks/" + std::to_string(b.session) + "-" + std::to_string(b.id);
    } else {
      file_path(d, b.id, p);
    }
    ::unlink(p.c_str());
  } else {
    for (int64_t p : b.pages) bit_give(d.free_bits, p);
    d.free_pages += (int64_t)b.pages.size();
    b.pages.clear();
  }
  if (!b.temp) d.committed_bytes -= std::min(d.committed_bytes, b.length);
  b.reserved = 0;
}

int BlockStore::allocate_dir(int tier, const std::string& medium, uint64_t bytes, bool use_reserved) {
  auto avail = [&](const StorageDir& d) { return use_reserved ? d.mgmt_available() : d.available(); };
  // tier < 0: top-down over tiers, first tier with a fitting dir wins (MaxFreeAllocator anyTier)
  int max_tier = (int)rr_index_.size() - 1;
  const int t0 = tier < 0 ? 0 : tier, t1 = tier < 0 ? max_tier : tier;
  for (int t = t0; t <= t1; ++t) {
    std::vector<int> cands;
    for (auto& d : dirs_)
      if (dir_matches(*d, t, medium)) cands.push_back(d->index);
    if (cands.empty()) continue;
    int pick = -1;
    if (alloc_policy_ == AllocPolicy::kGreedy) {
      for (int c : cands)
        if (avail(*dirs_[c]) >= bytes) { pick = c; break; }
    } else if (alloc_policy_ == AllocPolicy::kRoundRobin) {
      const int n = (int)cands.size();
      for (int k = 0; k < n; ++k) {
        const int c = cands[(rr_index_[t] + k) % n];
        if (avail(*dirs_[c]) >= bytes) {
          pick = c;
          rr_index_[t] = (rr_index_[t] + k + 1) % n;
          break;
        }
      }
    } else {
      uint64_t best = 0;
      for (int c : cands) {
        const uint64_t a = avail(*dirs_[c]);
        if (a >= bytes && (pick < 0 || a > best)) { pick = c; best = a; }
      }
    }
    if (pick >= 0) return pick;
  }
  return -1;
}

// -------------------------------------------------------------------------------------------
// lifecycle
int BlockStore::create_block(int64_t session, int64_t block_id, int tier, const std::string& medium,
                             uint64_t initial, bool evict, bool pin) {
  std::unique_lock<std::mutex> lk(mu_);
  if (blocks_.count(block_id))
    throw StoreError(kErrAlreadyExists, "block " + std::to_string(block_id) + " already exists");
  int d = allocate_dir(tier, medium, initial);
  if (d < 0 && evict) {
    free_space_locked(lk, session, initial, tier, -1, medium, free_ahead_);
    if (blocks_.count(block_id))   // created by another thread while the store was unlocked
      throw StoreError(kErrAlreadyExists, "block " + std::to_string(block_id) + " already exists");
    d = allocate_dir(tier, medium, initial);
  }
  if (d < 0)
    throw StoreError(kErrOutOfSpace, "no space for " + std::to_string(initial) + " bytes in tier " +
                                         std::to_string(tier));
  BlockMeta b;
  b.id = block_id;
  b.dir = d;
  b.temp = true;
  b.session = session;
  b.pinned_on_create = pin;
  if (!grow_pages(*dirs_[d], b, std::max<uint64_t>(initial, 1))) {
    release_storage(b);
    throw StoreError(kErrOutOfSpace, "allocation raced for block " + std::to_string(block_id));
  }
  b.slot = alloc_slot();
  b.seq = ++create_seq_;
  slot_block_[b.slot] = block_id;
  crf_[b.slot] = 0.f;
  last_[b.slot] = clock_.load();
  note_state(b, true);   // temp: not evictable yet; resets the slot's device annotations
  if (dirs_[d]->spec.kind == DirKind::kFile) {
    const std::string p = dirs_[d]->spec.path + "/.tmp_blocks/" + std::to_string(session) + "-" +
                          std::to_string(block_id);
    int fd = ::open(p.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
    if (fd < 0) throw StoreError(kErrIo, "cannot create " + p);
    ::close(fd);
  }
  blocks_.emplace(block_id, std::move(b));
  session_temps_[session].insert(block_id);
  return d;
}

void BlockStore::request_space(int64_t session, int64_t block_id, uint64_t additional) {
  std::unique_lock<std::mutex> lk(mu_);
  BlockMeta* b = find(block_id);
  if (!b || !b->temp) throw StoreError(kErrNotFound, "temp block " + std::to_string(block_id) + " not found");
  if (b->session != session) throw StoreError(kErrInvalidState, "temp block owned by another session");
  StorageDir& d = *dirs_[b->dir];
  const uint64_t target = b->reserved + additional;
  if (grow_pages(d, *b, target)) return;
  free_space_locked(lk, session, additional, d.spec.tier, b->dir, "", free_ahead_);
  b = find(block_id);
  if (!b || !grow_pages(*dirs_[b->dir], *b, target))
    throw StoreError(kErrOutOfSpace, "cannot reserve " + std::to_string(additional) + " more bytes");
}

std::vector<int64_t> BlockStore::external_write(int64_t session, int64_t block_id, uint64_t offset,
                                                uint64_t len) {
  std::unique_lock<std::mutex> lk(mu_);
  BlockMeta* b = find(block_id);
  if (!b || !b->temp) throw StoreError(kErrNotFound, "temp block " + std::to_string(block_id) + " not found");
  if (b->session != session) throw StoreError(kErrInvalidState, "temp block owned by another session");
  if (dirs_[b->dir]->spec.kind == DirKind::kFile)
    throw StoreError(kErrInvalidArgument, "external writes need a memory (HBM/DRAM) dir");
  if (offset + len > b->reserved) {
    const uint64_t add = offset + len - b->reserved;
    lk.unlock();
    request_space(session, block_id, add);
    lk.lock();
    b = find(block_id);
    if (!b || !b->temp) throw StoreError(kErrNotFound, "temp block vanished during reserve");
  }
  b->length = std::max(b->length, offset + len);
  return b->pages;
}

void BlockStore::write(int64_t session, int64_t block_id, uint64_t offset, uint64_t src, uint64_t len,
                       int src_kind, uint64_t stream, bool sync) {
  TraceRange trace_("BlockStore.write");
  if (len == 0) return;
  set_device();
  std::vector<CopySeg> dev_segs;
  hipStream_t st = stream_or_default(stream);
  BlockMeta snapshot;
  {
    std::unique_lock<std::mutex> lk(mu_);
    BlockMeta* b = find(block_id);
    if (!b || !b->temp) throw StoreError(kErrNotFound, "temp block " + std::to_string(block_id) + " not found");
    if (b->session != session) throw StoreError(kErrInvalidState, "temp block owned by another session");
    if (offset + len > b->reserved) {
      const uint64_t add = offset + len - b->reserved;
      lk.unlock();
      request_space(session, block_id, add);
      lk.lock();
      b = find(block_id);
      if (!b || !b->temp) throw StoreError(kErrNotFound, "temp block vanished during write");
    }
    b->length = std::max(b->length, offset + len);
    snapshot = *b;
  }
  plan_block_range(snapshot, offset, len, src, src_kind, /*to_block=*/true, dev_segs, st);
  if (!dev_segs.empty()) copy_segments(dev_segs, st);
  if (sync && has_device_) HIP_OK(hipStreamSynchronize(st));
}

void BlockStore::commit_block(int64_t session, int64_t block_id, bool pin) {
  std::unique_lock<std::mutex> lk(mu_);
  BlockMeta* b = find(block_id);
  if (!b || !b->temp) throw StoreError(kErrNotFound, "temp block " + std::to_string(block_id) + " not found");
  if (b->session != session) throw StoreError(kErrInvalidState, "temp block owned by another session");
  StorageDir& d = *dirs_[b->dir];
  // return over-reserved pages
  if (d.spec.kind != DirKind::kFile) {
    const size_t keep = (size_t)ceil_div(std::max<uint64_t>(b->length, 1), d.spec.page_size);
    while (b->pages.size() > keep) {
      bit_give(d.free_bits, b->pages.back());
      b->pages.pop_back();
      ++d.free_pages;
    }
    b->reserved = b->pages.size() * d.spec.page_size;
  } else {
    const std::string tmp = d.spec.path + "/.tmp_blocks/" + std::to_string(session) + "-" + std::to_string(block_id);
    std::string fin;
    file_path(d, block_id, fin);
    if (::rename(tmp.c_str(), fin.c_str()) != 0) throw StoreError(kErrIo, "rename failed for " + tmp);
    d.file_used -= std::min(d.file_used, b->reserved);
    b->reserved = b->length;
    d.file_used += b->reserved;
  }
  b->temp = false;
  b->pinned_on_create = b->pinned_on_create || pin;
  d.committed_bytes += b->length;
  session_temps_[session].erase(block_id);
  note_state(*b, true);
  touch_slot(b->slot);
  emit(0, *b);
}

void BlockStore::abort_block(int64_t session, int64_t block_id) {
  std::unique_lock<std::mutex> lk(mu_);
  BlockMeta* b = find(block_id);
  if (!b || !b->temp) throw StoreError(kErrNotFound, "temp block " + std::to_string(block_id) + " not found");
  if (b->session != session) throw StoreError(kErrInvalidState, "temp block owned by another session");
  note_state(*b, false);
  release_storage(*b);
  free_slots_.push_back(b->slot);
  session_temps_[session].erase(block_id);
  blocks_.erase(block_id);
}

void BlockStore::remove_locked(BlockMeta& b, bool emit_event) {
  if (emit_event) emit(1, b);
  note_state(b, false);
  release_storage(b);
  free_slots_.push_back(b.slot);
  crf_[b.slot] = 0.f;
  blocks_.erase(b.id);
}

void BlockStore::remove_block(int64_t session, int64_t block_id) {
  {
    // an explicit removal (free, delete, a failed commit) outranks append holds, which only keep
    // the block from eviction: the AppendBlock that wanted it then fails NOT_FOUND
    std::lock_guard<std::mutex> g(holds_mu_);
    auto it = holds_.find(block_id);
    if (it != holds_.end()) {
      for (auto& h : it->second) {
        try {
          unlock(h.first);
        } catch (...) {
        }
      }
      holds_.erase(it);
    }
  }
  std::unique_lock<std::mutex> lk(mu_);
  BlockMeta* b = find(block_id);
  if (!b) throw StoreError(kErrNotFound, "block " + std::to_string(block_id) + " does not exist");
  if (b->temp) throw StoreError(kErrInvalidState, "cannot remove temp block " + std::to_string(block_id));
  // wait for readers/writers held by *other* sessions (reference: removeBlock takes a write lock)
  auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(30);
  while (true) {
    b = find(block_id);
    if (!b) throw StoreError(kErrNotFound, "block " + std::to_string(block_id) + " does not exist");
    if (b->readers == 0 && !b->writer) break;
    if (lock_cv_.wait_until(lk, deadline) == std::cv_status::timeout)
      throw StoreError(kErrTimeout, "timed out waiting to remove locked block " + std::to_string(block_id));
  }
  remove_locked(*b, true);
  lock_cv_.notify_all();
}

int BlockStore::move_block(int64_t session, int64_t block_id, int dst_tier, const std::string& medium,
                           bool evict) {
  set_device();
  std::unique_lock<std::mutex> lk(mu_);
  BlockMeta* b = find(block_id);
  if (!b || b->temp) throw StoreError(kErrNotFound, "block " + std::to_string(block_id) + " does not exist");
  if (b->writer || b->readers > 0) throw StoreError(kErrInvalidState, "block is locked");
  if (dir_matches(*dirs_[b->dir], dst_tier, medium)) return b->dir;
  const uint64_t len = b->length;
  int d = allocate_dir(dst_tier, medium, std::max<uint64_t>(len, 1));
  if (d < 0 && evict) {
    b->evicting = true;  // never pick the block being moved as its own victim
    evicting_ids_.insert(block_id);
    try {
      free_space_locked(lk, session, len, dst_tier, -1, medium);
    } catch (...) {
      evicting_ids_.erase(block_id);
      b = find(block_id);
      if (b) b->evicting = false;
      throw;
    }
    evicting_ids_.erase(block_id);
    b = find(block_id);
    if (b) b->evicting = false;
    d = allocate_dir(dst_tier, medium, std::max<uint64_t>(len, 1));
  }
  if (!b) throw StoreError(kErrNotFound, "block vanished during move");
  if (d < 0) throw StoreError(kErrOutOfSpace, "no space in destination tier for move");
  BlockMeta nb;
  nb.id = block_id;
  nb.dir = d;
  nb.temp = false;
  nb.length = len;
  if (!grow_pages(*dirs_[d], nb, std::max<uint64_t>(len, 1))) throw StoreError(kErrOutOfSpace, "move allocation failed");
  b->writer = true;  // hold the block while copying
  BlockMeta src_snap = *b;
  lk.unlock();
  hipStream_t st = has_device_ ? move_stream() : internal_stream_;
  std::vector<CopySeg> dev_segs;
  try {
    copy_block_storage(src_snap, nb, dev_segs, st);
    if (!dev_segs.empty()) copy_segments(dev_segs, st);
    if (has_device_) HIP_OK(hipStreamSynchronize(st));
  } catch (...) {
    lk.lock();
    release_storage(nb);
    BlockMeta* bb = find(block_id);
    if (bb) bb->writer = false;
    lock_cv_.notify_all();
    throw;
  }
  lk.lock();
  b = find(block_id);
  // swap storage
  BlockMeta old = *b;
  old.temp = false;
  release_storage(old);
  b->dir = d;
  b->pages = nb.pages;
  b->reserved = nb.reserved;
  b->writer = false;
  note_state(*b, true);
  dirs_[d]->committed_bytes += len;
  emit(2, *b);
  lock_cv_.notify_all();
  return d;
}

// Bytes of a committed block (src_snap) into freshly allocated storage nb.  Arena->arena pieces
// are queued on `st` (HBM<->HBM pieces appended to dev_segs for one batched-copy launch, DMA
// pieces issued async); file endpoints go through a host bounce buffer synchronously.
void BlockStore::copy_block_storage(const BlockMeta& src_snap, const BlockMeta& nb, std::vector<CopySeg>& dev_segs,
                                    hipStream_t st) {
  const StorageDir& sd = *dirs_[src_snap.dir];
  const StorageDir& dd = *dirs_[nb.dir];
  const uint64_t len = src_snap.length;
  const bool dst_dev = dd.spec.kind == DirKind::kDevice;
  if (sd.spec.kind != DirKind::kFile && dd.spec.kind != DirKind::kFile) {
    // arena -> arena: walk destination page runs, reading the source range into each
    uint64_t off = 0;
    size_t i = 0;
    while (off < len) {
      const int64_t p0 = nb.pages[i];
      size_t j = i + 1;
      while (j < nb.pages.size() && nb.pages[j] == nb.pages[j - 1] + 1) ++j;
      const uint64_t run = std::min<uint64_t>((j - i) * dd.spec.page_size, len - off);
      const uint64_t dst_addr = dd.spec.base + (uint64_t)p0 * dd.spec.page_size;
      const uint64_t dst_mapped = (!dst_dev && dd.dev_base) ? dd.dev_base + (uint64_t)p0 * dd.spec.page_size : 0;
      plan_block_range(src_snap, off, run, dst_addr, dst_dev ? (int)MemKind::kDevice : (int)MemKind::kHost, false,
                       dev_segs, st, dst_mapped, true);
      off += run;
      i = j;
    }
    return;
  }
  // via a host bounce buffer (file tiers)
  std::vector<uint8_t> bounce(len);
  std::vector<CopySeg> none;
  plan_block_range(src_snap, 0, len, (uint64_t)bounce.data(), (int)MemKind::kHost, false, none, st);
  if (has_device_) HIP_OK(hipStreamSynchronize(st));
  if (dd.spec.kind == DirKind::kFile) {
    std::string fin;
    file_path(dd, nb.id, fin);
    int fd = ::open(fin.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
    if (fd < 0) throw StoreError(kErrIo, "cannot create " + fin);
    ssize_t w = ::pwrite(fd, bounce.data(), len, 0);
    ::close(fd);
    if (w != (ssize_t)len) throw StoreError(kErrIo, "short write to " + fin);
  } else {
    plan_block_range(nb, 0, len, (uint64_t)bounce.data(), (int)MemKind::kHost, true, none, st);
    if (has_device_) HIP_OK(hipStreamSynchronize(st));
  }
}

int BlockStore::lower_tier(int tier) const {
  int best = -1;
  for (auto& d : dirs_)
    if (d->spec.tier > tier && d->healthy && (best < 0 || d->spec.tier < best)) best = d->spec.tier;
  return best;
}

std::vector<int64_t> BlockStore::move_blocks(int64_t session, const std::vector<int64_t>& ids, int dst_tier,
                                             const std::string& medium, bool evict, bool use_reserved) {
  TraceRange trace_("BlockStore.move_blocks");
  set_device();
  std::unique_lock<std::mutex> lk(mu_);
  return move_blocks_locked(lk, session, ids, dst_tier, medium, evict, use_reserved);
}

std::vector<int64_t> BlockStore::move_blocks_locked(std::unique_lock<std::mutex>& lk, int64_t session,
                                                    const std::vector<int64_t>& ids, int dst_tier,
                                                    const std::string& medium, bool evict, bool use_reserved) {
  std::vector<int64_t> cand;
  uint64_t need = 0;
  for (int64_t id : ids) {
    BlockMeta* b = find(id);
    if (!b || b->temp || b->writer || b->readers > 0 || b->evicting) continue;
    if (dir_matches(*dirs_[b->dir], dst_tier, medium)) continue;
    cand.push_back(id);
    need += std::max<uint64_t>(b->length, 1);
  }
  if (cand.empty()) return {};
  // movers are held: never victims of the eviction below, not lockable meanwhile
  for (int64_t id : cand) {
    find(id)->evicting = true;
    evicting_ids_.insert(id);
  }
  auto release_hold = [&] {
    for (int64_t id : cand) {
      evicting_ids_.erase(id);
      BlockMeta* b = find(id);
      if (b) b->evicting = false;
    }
  };
  if (evict) {
    try {
      free_space_locked(lk, session, need, dst_tier, -1, medium);
    } catch (const StoreError&) {
      // best effort: move what fits
    }
  }
  struct Job {
    BlockMeta snap;
    BlockMeta nb;
  };
  std::vector<Job> jobs;
  for (int64_t id : cand) {
    BlockMeta* b = find(id);
    if (!b || b->readers > 0 || b->writer) continue;
    const uint64_t len = b->length;
    const int d = allocate_dir(dst_tier, medium, std::max<uint64_t>(len, 1), use_reserved);
    if (d < 0) break;
    Job j;
    j.nb.id = id;
    j.nb.dir = d;
    j.nb.temp = false;
    j.nb.length = len;
    if (!grow_pages(*dirs_[d], j.nb, std::max<uint64_t>(len, 1), use_reserved)) {
      release_storage(j.nb);
      break;
    }
    b->writer = true;   // hold the block while copying
    j.snap = *b;
    jobs.push_back(std::move(j));
  }
  release_hold();
  if (jobs.empty()) {
    lock_cv_.notify_all();
    return {};
  }
  lk.unlock();
  hipStream_t st = internal_stream_;
  std::vector<CopySeg> dev_segs;
  std::exception_ptr err;
  try {
    for (auto& j : jobs) copy_block_storage(j.snap, j.nb, dev_segs, st);
    if (!dev_segs.empty()) copy_segments(dev_segs, st);
    if (has_device_) HIP_OK(hipStreamSynchronize(st));   // one sync for the whole batch
  } catch (...) {
    err = std::current_exception();
  }
  lk.lock();
  std::vector<int64_t> moved;
  for (auto& j : jobs) {
    BlockMeta* b = find(j.nb.id);
    if (err || !b) {
      release_storage(j.nb);
      if (b) b->writer = false;
      continue;
    }
    BlockMeta old = *b;
    old.temp = false;
    release_storage(old);
    b->dir = j.nb.dir;
    b->pages = j.nb.pages;
    b->reserved = j.nb.reserved;
    b->writer = false;
    note_state(*b, true);
    dirs_[j.nb.dir]->committed_bytes += b->length;
    emit(2, *b);
    moved.push_back(b->id);
  }
  lock_cv_.notify_all();
  ++stats_.batched_moves;
  stats_.batched_move_blocks += moved.size();
  if (err) std::rethrow_exception(err);
  return moved;
}

// -------------------------------------------------------------------------------------------
// locks
int64_t BlockStore::lock_block(int64_t session, int64_t block_id, bool write, int64_t timeout_ms) {
  std::unique_lock<std::mutex> lk(mu_);
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms < 0 ? 0 : timeout_ms);
  while (true) {
    BlockMeta* b = find(block_id);
    if (!b || b->temp) throw StoreError(kErrNotFound, "block " + std::to_string(block_id) + " does not exist");
    const bool ok = write ? (b->readers == 0 && !b->writer) : !b->writer;
    if (ok && !b->evicting) {
      if (write) b->writer = true; else ++b->readers;
      const int64_t id = next_lock_++;
      locks_[id] = LockRec{block_id, session, write};
      session_locks_[session].insert(id);
      return id;
    }
    if (timeout_ms < 0) {
      lock_cv_.wait(lk);
    } else if (lock_cv_.wait_until(lk, deadline) == std::cv_status::timeout) {
      return -1;
    }
  }
}

namespace {
constexpr int64_t kHoldSession = INT64_MAX - 7;   // owner of append holds (no client uses it)
int64_t steady_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
}  // namespace

void BlockStore::sweep_holds_locked(int64_t now) {
  for (auto it = holds_.begin(); it != holds_.end();) {
    auto& v = it->second;
    for (size_t i = 0; i < v.size();) {
      if (v[i].second <= now) {
        try {
          unlock(v[i].first);
        } catch (...) {
        }
        v.erase(v.begin() + (long)i);
      } else {
        ++i;
      }
    }
    it = v.empty() ? holds_.erase(it) : std::next(it);
  }
}

bool BlockStore::hold_block(int64_t block_id, int64_t ttl_ms) {
  int64_t lock;
  try {
    lock = lock_block(kHoldSession, block_id, false, 0);
  } catch (const StoreError&) {
    return false;
  }
  if (lock < 0) return false;
  const int64_t now = steady_ns();
  std::lock_guard<std::mutex> g(holds_mu_);
  sweep_holds_locked(now);
  holds_[block_id].emplace_back(lock, now + std::max<int64_t>(ttl_ms, 1) * 1000000LL);
  return true;
}

bool BlockStore::release_hold(int64_t block_id) {
  std::lock_guard<std::mutex> g(holds_mu_);
  bool released = false;
  auto it = holds_.find(block_id);
  if (it != holds_.end() && !it->second.empty()) {
    try {
      unlock(it->second.front().first);
    } catch (...) {
    }
    it->second.erase(it->second.begin());
    if (it->second.empty()) holds_.erase(it);
    released = true;
  }
  sweep_holds_locked(steady_ns());
  return released;
}

size_t BlockStore::holds() {
  std::lock_guard<std::mutex> g(holds_mu_);
  size_t n = 0;
  for (auto& kv : holds_) n += kv.second.size();
  return n;
}

void BlockStore::unlock(int64_t lock_id) {
  std::unique_lock<std::mutex> lk(mu_);
  auto it = locks_.find(lock_id);
  if (it == locks_.end()) throw StoreError(kErrNotFound, "lock " + std::to_string(lock_id) + " not held");
  BlockMeta* b = find(it->second.block);
  if (b) {
    if (it->second.write) b->writer = false; else if (b->readers > 0) --b->readers;
  }
  auto sit = session_locks_.find(it->second.session);
  if (sit != session_locks_.end()) {
    sit->second.erase(lock_id);
    if (sit->second.empty()) session_locks_.erase(sit);
  }
  locks_.erase(it);
  lock_cv_.notify_all();
}

void BlockStore::cleanup_session(int64_t session) {
  std::vector<int64_t> lock_ids, temps;
  {
    std::unique_lock<std::mutex> lk(mu_);
    auto sit = session_locks_.find(session);
    if (sit != session_locks_.end()) lock_ids.assign(sit->second.begin(), sit->second.end());
    auto tit = session_temps_.find(session);
    if (tit != session_temps_.end()) temps.assign(tit->second.begin(), tit->second.end());
  }
  for (int64_t l : lock_ids) {
    try { unlock(l); } catch (const StoreError&) {}
  }
  for (int64_t t : temps) {
    try { abort_block(session, t); } catch (const StoreError&) {}
  }
  std::unique_lock<std::mutex> lk(mu_);
  session_temps_.erase(session);
}

void BlockStore::access_block(int64_t session, int64_t block_id) {
  (void)session;
  std::unique_lock<std::mutex> lk(mu_);
  BlockMeta* b = find(block_id);
  if (!b) throw StoreError(kErrNotFound, "block " + std::to_string(block_id) + " does not exist");
  touch_slot(b->slot);
}

void BlockStore::access_blocks(const std::vector<int64_t>& ids) {
  std::unique_lock<std::mutex> lk(mu_);
  for (int64_t id : ids) {
    BlockMeta* b = find(id);
    if (b) touch_slot(b->slot);
  }
}

void BlockStore::set_pinned_files(const std::vector<int64_t>& file_ids) {
  std::unique_lock<std::mutex> lk(mu_);
  pinned_files_.clear();
  pinned_files_.insert(file_ids.begin(), file_ids.end());
  for (auto& kv : blocks_)
    if (!kv.second.temp) note_state(kv.second, true);
}

// -------------------------------------------------------------------------------------------
// data plane
void BlockStore::plan_block_range(const BlockMeta& b, uint64_t offset, uint64_t len, uint64_t ext,
                                  int ext_kind, bool to_block, std::vector<CopySeg>& dev_segs,
                                  hipStream_t stream, uint64_t ext_mapped, bool mapped_kernel) {
  const StorageDir& d = *dirs_[b.dir];
  const bool ext_dev = ext_kind == (int)MemKind::kDevice;
  if (d.spec.kind == DirKind::kFile) {
    std::string p;
    if (b.temp) p = d.spec.path + "/.tmp_blocks/" + std::to_string(b.session) + "-" + std::to_string(b.id);
    else file_path(d, b.id, p);
    int fd = ::open(p.c_str(), to_block ? O_WRONLY : O_RDONLY);
    if (fd < 0) throw StoreError(kErrIo, "cannot open block file " + p);
    std::vector<uint8_t> bounce;
    uint8_t* host = reinterpret_cast<uint8_t*>(ext);
    if (ext_dev) {
      bounce.resize(len);
      host = bounce.data();
      if (to_block) {
        hipError_t e = hipMemcpy(host, reinterpret_cast<void*>(ext), len, hipMemcpyDeviceToHost);
        if (e != hipSuccess) { ::close(fd); HIP_OK(e); }
      }
    }
    uint64_t done = 0;
    while (done < len) {
      ssize_t r = to_block ? ::pwrite(fd, host + done, len - done, offset + done)
                           : ::pread(fd, host + done, len - done, offset + done);
      if (r <= 0) { ::close(fd); throw StoreError(kErrIo, "block file I/O failed on " + p); }
      done += (uint64_t)r;
    }
    ::close(fd);
    if (ext_dev && !to_block) HIP_OK(hipMemcpy(reinterpret_cast<void*>(ext), host, len, hipMemcpyHostToDevice));
    return;
  }
  const uint64_t ps = d.spec.page_size;
  const bool arena_dev = d.spec.kind == DirKind::kDevice;
  uint64_t pos = offset, done = 0;
  while (done < len) {
    const size_t pi = (size_t)(pos / ps);
    if (pi >= b.pages.size()) throw StoreError(kErrInvalidArgument, "range beyond block reservation");
    uint64_t in_page = pos % ps;
    // merge physically contiguous pages into one segment
    size_t pj = pi + 1;
    while (pj < b.pages.size() && b.pages[pj] == b.pages[pj - 1] + 1) ++pj;
    const uint64_t run_bytes = (uint64_t)(pj - pi) * ps - in_page;
    const uint64_t n = std::min(run_bytes, len - done);
    const uint64_t arena_addr = d.spec.base + (uint64_t)b.pages[pi] * ps + in_page;
    const uint64_t ext_addr = ext + done;
    const uint64_t src = to_block ? ext_addr : arena_addr;
    const uint64_t dst = to_block ? arena_addr : ext_addr;
    // device-visible addresses of both ends (0 = not reachable by a kernel)
    const uint64_t arena_k = arena_dev ? arena_addr : (d.dev_base ? d.dev_base + (arena_addr - d.spec.base) : 0);
    const uint64_t ext_k = ext_dev ? ext_addr : (ext_mapped ? ext_mapped + done : 0);
    if (arena_dev && ext_dev) {
      dev_segs.push_back(CopySeg{src, dst, n, 0});
    } else if (mapped_kernel && arena_dev != ext_dev && arena_k && ext_k) {
      // HBM <-> GPU-mapped host arena (tier moves): one batched copy kernel for the whole move
      dev_segs.push_back(CopySeg{to_block ? ext_k : arena_k, to_block ? arena_k : ext_k, n, 0});
    } else if (!arena_dev && !ext_dev) {
      std::memcpy(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), n);
    } else {
      const hipMemcpyKind kind = to_block ? (arena_dev ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost)
                                          : (arena_dev ? hipMemcpyDeviceToHost : hipMemcpyHostToDevice);
      HIP_OK(hipMemcpyAsync(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), n, kind, stream));
    }
    pos += n;
    done += n;
  }
}

void BlockStore::copy_segments(std::vector<CopySeg>& segs, hipStream_t stream) {
  std::lock_guard<std::mutex> g(ring_mu_);
  size_t base = 0;
  while (base < segs.size()) {
    const size_t cnt = std::min<size_t>(segs.size() - base, kRingSegs);
    const int slot = ring_pos_;
    ring_pos_ = (ring_pos_ + 1) % kRing;
    HIP_OK(hipEventSynchronize(ring_ev_[slot]));
    CopySeg* h = host_ring_ + (size_t)slot * kRingSegs;
    CopySeg* dv = dev_ring_ + (size_t)slot * kRingSegs;
    uint64_t chunks = 0;
    for (size_t i = 0; i < cnt; ++i) {
      h[i] = segs[base + i];
      h[i].chunk0 = chunks;
      chunks += ceil_div(h[i].bytes, kCopyChunk);
    }
    HIP_OK(hipMemcpyAsync(dv, h, sizeof(CopySeg) * cnt, hipMemcpyHostToDevice, stream));
    HIP_OK(launch_batched_copy(dv, (int)cnt, chunks, stream));
    HIP_OK(hipEventRecord(ring_ev_[slot], stream));
    base += cnt;
  }
  segs.clear();
}

void BlockStore::read_batch(const std::vector<ReadReq>& reqs, uint64_t stream, bool sync) {
  TraceRange trace_("BlockStore.read_batch");
  set_device();
  hipStream_t st = stream_or_default(stream);
  std::vector<CopySeg> dev_segs;
  dev_segs.reserve(reqs.size() * 2);
  // Snapshot the (small) page lists under the lock; callers hold block read locks, so the
  // pages cannot be released while the copies are in flight.
  std::vector<BlockMeta> snaps;
  snaps.reserve(reqs.size());
  {
    std::unique_lock<std::mutex> lk(mu_);
    for (const auto& r : reqs) {
      BlockMeta* b = find(r.block_id);
      if (!b) throw StoreError(kErrNotFound, "block " + std::to_string(r.block_id) + " does not exist");
      if (r.offset + r.length > b->length)
        throw StoreError(kErrInvalidArgument, "read [" + std::to_string(r.offset) + ", +" +
                                                  std::to_string(r.length) + ") beyond block length " +
                                                  std::to_string(b->length));
      snaps.push_back(*b);
    }
  }
  for (size_t i = 0; i < reqs.size(); ++i)
    plan_block_range(snaps[i], reqs[i].offset, reqs[i].length, reqs[i].dst, reqs[i].dst_kind, false,
                     dev_segs, st);
  if (!dev_segs.empty()) copy_segments(dev_segs, st);
  if (sync && has_device_) HIP_OK(hipStreamSynchronize(st));
}

std::vector<uint32_t> BlockStore::checksum(int64_t block_id, uint64_t piece_bytes) {
  TraceRange trace_("BlockStore.checksum");
  set_device();
  BlockMeta snap;
  {
    std::unique_lock<std::mutex> lk(mu_);
    BlockMeta* b = find(block_id);
    if (!b) throw StoreError(kErrNotFound, "block " + std::to_string(block_id) + " does not exist");
    snap = *b;
  }
  const StorageDir& d = *dirs_[snap.dir];
  const uint64_t ps = d.spec.kind == DirKind::kFile ? (piece_bytes ? piece_bytes : (2ull << 20)) : d.spec.page_size;
  if (piece_bytes == 0) piece_bytes = ps;
  if (d.spec.kind != DirKind::kFile && ps % piece_bytes != 0)
    throw StoreError(kErrInvalidArgument, "piece size must divide the page size");
  const uint64_t len = snap.length;
  std::vector<uint32_t> out(len ? ceil_div(len, piece_bytes) : 0);
  if (len == 0) return out;
  if (d.spec.kind != DirKind::kDevice) {
    std::vector<uint8_t> buf(len);
    std::vector<CopySeg> none;
    plan_block_range(snap, 0, len, (uint64_t)buf.data(), (int)MemKind::kHost, false, none, internal_stream_);
    for (size_t i = 0; i < out.size(); ++i) {
      const uint64_t o = i * piece_bytes;
      out[i] = crc32c_sw(buf.data() + o, std::min(piece_bytes, len - o));
    }
    return out;
  }
  std::lock_guard<std::mutex> g(ev_mu_);
  const size_t need = out.size() + crc32c_scratch_words(len, piece_bytes) + 64;
  if (crc_cap_ < need) {
    if (crc_dev_) hipFree(crc_dev_);
    crc_dev_ = nullptr;
    HIP_OK(hipMalloc((void**)&crc_dev_, need * sizeof(uint32_t)));
    crc_cap_ = need;
  }
  // contiguous page runs, each a whole number of pieces
  uint64_t off = 0;
  size_t i = 0, piece_idx = 0;
  while (off < len) {
    size_t j = i + 1;
    while (j < snap.pages.size() && snap.pages[j] == snap.pages[j - 1] + 1) ++j;
    const uint64_t run = std::min<uint64_t>((j - i) * ps, len - off);
    const uint8_t* base = reinterpret_cast<const uint8_t*>(d.spec.base + (uint64_t)snap.pages[i] * ps);
    const uint64_t np = ceil_div(run, piece_bytes);
    uint32_t* scratch = crc_dev_ + out.size();
    HIP_OK(launch_crc32c_pieces(base, run, piece_bytes, crc_dev_ + piece_idx, scratch,
                                crc_cap_ - out.size(), internal_stream_));
    piece_idx += np;
    off += run;
    i = j;
  }
  HIP_OK(hipMemcpyAsync(out.data(), crc_dev_, out.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, internal_stream_));
  HIP_OK(hipStreamSynchronize(internal_stream_));
  return out;
}

size_t BlockStore::checksum_async_words(uint64_t length, uint64_t page_size) {
  if (!length || !page_size) return 0;
  const uint64_t np = ceil_div(length, page_size);
  // out | scratch of either launch form | the page index array (int64, 2 words each, aligned)
  const uint64_t scratch = std::max<uint64_t>(crc32c_scratch_words(length, page_size),
                                              crc32c_pages_scratch_words(length, page_size));
  return (size_t)(np + scratch + 2 + 2 * np + 64);
}

size_t BlockStore::checksum_async(int64_t block_id, hipStream_t stream, uint32_t* dev_buf, size_t dev_words,
                                  uint32_t* host_out, uint64_t* page_size_out) {
  BlockMeta snap;
  {
    std::unique_lock<std::mutex> lk(mu_);
    BlockMeta* b = find(block_id);
    if (!b) throw StoreError(kErrNotFound, "block " + std::to_string(block_id) + " does not exist");
    snap = *b;
  }
  const StorageDir& d = *dirs_[snap.dir];
  if (d.spec.kind != DirKind::kDevice || !snap.length) return 0;
  const uint64_t ps = d.spec.page_size, len = snap.length;
  const size_t np = (size_t)ceil_div(len, ps);
  if (dev_words < checksum_async_words(len, ps)) return 0;
  set_device();
  // One launch over the block's scattered pages: the page index array goes through the caller's
  // pinned buffer (same size as dev_buf, words [np, ...) are free until the CRCs land in [0, np))
  // into dev_buf behind the scratch.
  {
    const uint64_t scratch = std::max<uint64_t>(crc32c_scratch_words(len, ps), crc32c_pages_scratch_words(len, ps));
    const size_t idx_word = (size_t)((np + scratch + 1) & ~1ull);     // 8-byte aligned
    if (idx_word + 2 * np <= dev_words && snap.pages.size() >= np) {
      int64_t* host_idx = reinterpret_cast<int64_t*>(host_out + idx_word);
      for (size_t k = 0; k < np; ++k) host_idx[k] = snap.pages[k];
      int64_t* dev_idx = reinterpret_cast<int64_t*>(dev_buf + idx_word);
      HIP_OK(hipMemcpyAsync(dev_idx, host_idx, np * sizeof(int64_t), hipMemcpyHostToDevice, stream));
      const hipError_t e = launch_crc32c_pages(reinterpret_cast<const uint8_t*>(d.spec.base), dev_idx, len, ps,
                                               dev_buf, dev_buf + np, scratch, stream);
      if (e == hipSuccess) {
        HIP_OK(hipMemcpyAsync(host_out, dev_buf, np * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        if (page_size_out) *page_size_out = ps;
        return np;
      }
      if (e != hipErrorNotSupported) HIP_OK(e);
    }
  }
  uint64_t off = 0;
  size_t i = 0, piece_idx = 0;
  while (off < len) {                      // contiguous page runs, one launch each
    size_t j = i + 1;
    while (j < snap.pages.size() && snap.pages[j] == snap.pages[j - 1] + 1) ++j;
    const uint64_t run = std::min<uint64_t>((j - i) * ps, len - off);
    const uint8_t* base = reinterpret_cast<const uint8_t*>(d.spec.base + (uint64_t)snap.pages[i] * ps);
    HIP_OK(launch_crc32c_pieces(base, run, ps, dev_buf + piece_idx, dev_buf + np, dev_words - np, stream));
    piece_idx += (size_t)ceil_div(run, ps);
    off += run;
    i = j;
  }
  HIP_OK(hipMemcpyAsync(host_out, dev_buf, np * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
  if (page_size_out) *page_size_out = ps;
  return np;
}

std::vector<std::pair<uint64_t, std::vector<uint32_t>>> BlockStore::checksum_blocks(
    const std::vector<int64_t>& ids, bool device_only) {
  TraceRange trace_("BlockStore.checksum_blocks");
  set_device();
  std::vector<std::pair<uint64_t, std::vector<uint32_t>>> out(ids.size());
  std::vector<uint64_t> ptrs;
  std::vector<uint32_t> lens;
  std::vector<std::pair<size_t, size_t>> where;   // (index into ids, first piece) of gathered blocks
  std::vector<size_t> slow;
  {
    std::unique_lock<std::mutex> lk(mu_);
    for (size_t i = 0; i < ids.size(); ++i) {
      BlockMeta* b = find(ids[i]);
      if (!b) continue;
      const StorageDir& d = *dirs_[b->dir];
      if (d.spec.kind != DirKind::kDevice || d.spec.page_size > crc32c_gather_max_piece()) {
        if (!device_only || d.spec.kind == DirKind::kDevice) slow.push_back(i);
        continue;
      }
      where.emplace_back(i, ptrs.size());
      const uint64_t ps = d.spec.page_size;
      for (uint64_t off = 0, k = 0; off < b->length; off += ps, ++k) {
        ptrs.push_back(d.spec.base + (uint64_t)b->pages[k] * ps);
        lens.push_back((uint32_t)std::min(ps, b->length - off));
      }
      out[i].first = ps;
      out[i].second.resize(ceil_div(b->length, ps));
    }
  }
  if (!ptrs.empty()) {
    std::lock_guard<std::mutex> g(ev_mu_);
    const size_t n = ptrs.size();
    // device scratch: pointers (2 words each), lengths, results
    const size_t need = 4 * n + 64;
    if (crc_cap_ < need) {
      if (crc_dev_) hipFree(crc_dev_);
      crc_dev_ = nullptr;
      HIP_OK(hipMalloc((void**)&crc_dev_, need * sizeof(uint32_t)));
      crc_cap_ = need;
    }
    uint64_t* dptr = reinterpret_cast<uint64_t*>(crc_dev_);
    uint32_t* dlen = crc_dev_ + 2 * n;
    uint32_t* dout = crc_dev_ + 3 * n;
    HIP_OK(hipMemcpyAsync(dptr, ptrs.data(), n * sizeof(uint64_t), hipMemcpyHostToDevice, internal_stream_));
    HIP_OK(hipMemcpyAsync(dlen, lens.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice, internal_stream_));
    HIP_OK(launch_crc32c_gather(dptr, dlen, n, dout, internal_stream_));
    std::vector<uint32_t> res(n);
    HIP_OK(hipMemcpyAsync(res.data(), dout, n * sizeof(uint32_t), hipMemcpyDeviceToHost, internal_stream_));
    HIP_OK(hipStreamSynchronize(internal_stream_));
    for (auto& [i, first] : where)
      std::copy(res.begin() + first, res.begin() + first + out[i].second.size(), out[i].second.begin());
  }
  for (size_t i : slow) {
    try {
      out[i].second = checksum(ids[i], 0);
      std::lock_guard<std::mutex> lk(mu_);
      BlockMeta* b = find(ids[i]);
      if (b) {
        const StorageDir& d = *dirs_[b->dir];
        out[i].first = d.spec.kind == DirKind::kFile ? (2ull << 20) : d.spec.page_size;
      }
    } catch (const StoreError&) {
      out[i] = {0, {}};   // removed meanwhile
    }
  }
  return out;
}

void BlockStore::fill_pattern(int64_t session, int64_t block_id, uint64_t length, uint64_t seed) {
  set_device();
  BlockMeta snap;
  {
    std::unique_lock<std::mutex> lk(mu_);
    BlockMeta* b = find(block_id);
    if (!b || !b->temp || b->session != session) throw StoreError(kErrNotFound, "temp block not found");
    if (length > b->reserved) {
      lk.unlock();
      request_space(session, block_id, length - b->reserved);
      lk.lock();
      b = find(block_id);
    }
    b->length = std::max(b->length, length);
    snap = *b;
  }
  const StorageDir& d = *dirs_[snap.dir];
  if (d.spec.kind != DirKind::kDevice) throw StoreError(kErrInvalidArgument, "fill_pattern needs a device dir");
  uint64_t off = 0;
  size_t i = 0;
  const uint64_t ps = d.spec.page_size;
  while (off < length) {
    size_t j = i + 1;
    while (j < snap.pages.size() && snap.pages[j] == snap.pages[j - 1] + 1) ++j;
    const uint64_t run = std::min<uint64_t>((j - i) * ps, length - off);
    uint8_t* base = reinterpret_cast<uint8_t*>(d.spec.base + (uint64_t)snap.pages[i] * ps);
    HIP_OK(launch_fill_pattern(base, run, seed, off >> 3, internal_stream_));
    off += run;
    i = j;
  }
  HIP_OK(hipStreamSynchronize(internal_stream_));
}

// -------------------------------------------------------------------------------------------
// eviction
EvictState BlockStore::dev_state(uint64_t now) const {
  EvictState st;
  st.crf = d_crf_;
  st.last = d_last_;
  st.fbytes = d_fbytes_;
  st.dir = d_dir_;
  st.n = (uint32_t)crf_.size();
  st.now = now;
  st.step = lrfu_step_;
  st.log2_inv_att = (float)std::log2(1.0 / (double)lrfu_att_);
  st.policy = annotator_ == Annotator::kLRFU ? 1 : 0;
  st.dir_mask = 0;
  st.unit = 0;
  st.invert = 0;
  return st;
}

// The annotator key of a slot from the host mirror (identical formula to the device key).
uint32_t BlockStore::host_key(uint32_t s, uint64_t now) const {
  const uint64_t age = now > last_[s] ? now - last_[s] : 0;
  uint32_t key;
  if (annotator_ == Annotator::kLRU) {
    key = 0xFFFFFFFEu - (uint32_t)std::min<uint64_t>(age, 0xFFFFFFFEull);
  } else {
    float crf = crf_[s] * std::pow(1.0f / lrfu_att_, (float)age * lrfu_step_);
    if (!(crf >= 0.f)) crf = 0.f;
    std::memcpy(&key, &crf, 4);
  }
  return key >= 0xFFFFFFFEu ? 0xFFFFFFFDu : key;
}

// Grow the slot-indexed device arrays to hold `n` slots (doubling).  Called under mu_; takes
// ev_mu_ so no selection is reading the old arrays.  Growth is logarithmic in the slot count.
void BlockStore::ensure_dev_slots_locked(size_t n) {
  if (n <= dev_slots_ && dev_synced_) return;
  std::lock_guard<std::mutex> g(ev_mu_);
  set_device();
  if (n > dev_slots_) {
    size_t cap = std::max<size_t>({n, dev_slots_ * 2, 16384});
    cap = (cap + 31) / 32 * 32;
    float* crf;
    uint64_t *last, *fb;
    int32_t* dir;
    uint32_t *keys, *excl, *hexcl, *hout, *hout_dev;
    HIP_OK(hipMalloc((void**)&crf, cap * 4));
    HIP_OK(hipMalloc((void**)&last, cap * 8));
    HIP_OK(hipMalloc((void**)&fb, cap * 8));
    HIP_OK(hipMalloc((void**)&dir, cap * 4));
    HIP_OK(hipMalloc((void**)&keys, cap * 4));
    HIP_OK(hipMalloc((void**)&excl, cap / 8));
    HIP_OK(hipHostMalloc((void**)&hexcl, cap / 8, hipHostMallocDefault));
    HIP_OK(hipHostMalloc((void**)&hout, cap * 4, hipHostMallocMapped));
    HIP_OK(hipHostGetDevicePointer((void**)&hout_dev, hout, 0));
    std::memset(hexcl, 0, cap / 8);
    HIP_OK(hipMemsetAsync(dir, 0xFF, cap * 4, internal_stream_));   // -1: no evictable block
    HIP_OK(hipMemsetAsync(fb, 0, cap * 8, internal_stream_));
    if (dev_slots_) {
      HIP_OK(hipMemcpyAsync(crf, d_crf_, dev_slots_ * 4, hipMemcpyDeviceToDevice, internal_stream_));
      HIP_OK(hipMemcpyAsync(last, d_last_, dev_slots_ * 8, hipMemcpyDeviceToDevice, internal_stream_));
      HIP_OK(hipMemcpyAsync(fb, d_fbytes_, dev_slots_ * 8, hipMemcpyDeviceToDevice, internal_stream_));
      HIP_OK(hipMemcpyAsync(dir, d_dir_, dev_slots_ * 4, hipMemcpyDeviceToDevice, internal_stream_));
    }
    HIP_OK(hipStreamSynchronize(internal_stream_));
    for (void* p : {(void*)d_crf_, (void*)d_last_, (void*)d_fbytes_, (void*)d_dir_, (void*)d_keys_, (void*)d_excl_})
      if (p) hipFree(p);
    for (void* p : {(void*)h_excl_, (void*)h_out_})
      if (p) hipHostFree(p);
    d_crf_ = crf;
    d_last_ = last;
    d_fbytes_ = fb;
    d_dir_ = dir;
    d_keys_ = keys;
    d_excl_ = excl;
    h_excl_ = hexcl;
    h_out_ = hout;
    h_out_dev_ = hout_dev;
    dev_slots_ = cap;
  }
  if (!dev_synced_) {
    // (re)publish every slot's mirror: first use, or device eviction switched back on
    dev_synced_ = true;
    for (uint32_t s = 0; s < (uint32_t)crf_.size(); ++s)
      if (!dirty_flag_[s]) {
        dirty_flag_[s] = 1;
        dirty_.push_back(s);
      }
  }
}

// Ship the dirty slots' mirror values to the device: one pinned staging fill, one async H2D, one
// scatter launch on the internal stream (no host wait unless the staging buffer is still in
// flight from two flushes ago).
void BlockStore::flush_annotations_locked() {
  if (!device_evict_active()) {
    for (uint32_t s : dirty_) dirty_flag_[s] = 0;
    dirty_.clear();
    return;
  }
  ensure_dev_slots_locked(crf_.size());
  if (dirty_.empty()) return;
  set_device();
  const size_t n = dirty_.size();
  const int k = upd_pos_;
  upd_pos_ ^= 1;
  HIP_OK(hipEventSynchronize(upd_ev_[k]));
  if (h_upd_cap_[k] < n) {
    if (h_upd_[k]) hipHostFree(h_upd_[k]);
    h_upd_[k] = nullptr;
    const size_t cap = std::max<size_t>(n, 4096);
    HIP_OK(hipHostMalloc((void**)&h_upd_[k], cap * sizeof(SlotUpdate), hipHostMallocDefault));
    h_upd_cap_[k] = cap;
  }
  if (d_upd_cap_ < n) {
    // stream-ordered: the previous scatter finished reading the old buffer before this point
    HIP_OK(hipStreamSynchronize(internal_stream_));
    if (d_upd_) hipFree(d_upd_);
    d_upd_ = nullptr;
    const size_t cap = std::max<size_t>(n, 4096);
    HIP_OK(hipMalloc((void**)&d_upd_, cap * sizeof(SlotUpdate)));
    d_upd_cap_ = cap;
  }
  SlotUpdate* u = h_upd_[k];
  for (size_t i = 0; i < n; ++i) {
    const uint32_t s = dirty_[i];
    u[i].slot = s;
    u[i].flags = kSlotSetState | kSlotReset;
    u[i].dir = slot_dir_[s];
    u[i].crf = crf_[s];
    u[i].fbytes = slot_fb_[s];
    u[i].t = last_[s];
    dirty_flag_[s] = 0;
  }
  dirty_.clear();
  HIP_OK(hipMemcpyAsync(d_upd_, u, n * sizeof(SlotUpdate), hipMemcpyHostToDevice, internal_stream_));
  HIP_OK(launch_slot_update(dev_state(clock_.load()), d_upd_, (uint32_t)n, internal_stream_));
  HIP_OK(hipEventRecord(upd_ev_[k], internal_stream_));
  ++stats_.annotation_flushes;
  stats_.annotation_updates += n;
}

// Device selection of victims in `dir` for `need` bytes.  Called with mu_ held; mu_ is released
// for the device round trip (launches + one stream sync) and re-acquired before returning.
std::vector<uint32_t> BlockStore::select_victims_device(std::unique_lock<std::mutex>& lk, int dir, uint64_t need,
                                                       uint64_t dir_mask, bool unit, bool invert) {
  flush_annotations_locked();
  // dynamic exclusions: locked or moving blocks (few; evictable() re-checks at removal anyway)
  std::vector<uint32_t> excl;
  for (auto& kv : locks_) {
    const BlockMeta* b = find(kv.second.block);
    if (b) excl.push_back(b->slot);
  }
  for (int64_t id : evicting_ids_) {
    const BlockMeta* b = find(id);
    if (b) excl.push_back(b->slot);
  }
  EvictState st = dev_state(clock_.load());
  st.dir_mask = dir_mask;
  st.unit = unit ? 1 : 0;
  st.invert = invert ? 1 : 0;
  std::vector<uint32_t> picked;
  {
    std::unique_lock<std::mutex> g(ev_mu_);   // mu_ -> ev_mu_ order, then mu_ is dropped
    lk.unlock();
    set_device();
    for (uint32_t s : excl) h_excl_[s >> 5] |= 1u << (s & 31);
    const size_t words = ((size_t)st.n + 31) / 32;
    hipError_t e = hipMemcpyAsync(d_excl_, h_excl_, words * 4, hipMemcpyHostToDevice, internal_stream_);
    if (e == hipSuccess)
      e = launch_evict_select_grid(st, (uint32_t)dir, d_excl_, need, d_keys_, d_ctl_, h_out_dev_, internal_stream_);
    if (e == hipSuccess) e = hipMemcpyAsync(h_ctl_, d_ctl_, sizeof(EvictCtl), hipMemcpyDeviceToHost, internal_stream_);
    if (e == hipSuccess) e = hipStreamSynchronize(internal_stream_);
    for (uint32_t s : excl) h_excl_[s >> 5] &= ~(1u << (s & 31));
    if (e == hipSuccess) picked.assign(h_out_, h_out_ + h_ctl_->count);
    g.unlock();
    lk.lock();
    if (e != hipSuccess) throw StoreError(kErrHip, std::string("device eviction select: ") + hipGetErrorString(e));
  }
  ++stats_.device_selections;
  return picked;
}

std::vector<uint32_t> BlockStore::select_victims_cpu(const std::vector<uint32_t>& cand, uint64_t need) {
  const size_t n = cand.size();
  std::vector<uint32_t> picked;
  if (n == 0 || need == 0) return picked;
  const uint64_t now = clock_.load();
  // identical keys to the device select, full sort
  std::vector<std::pair<uint32_t, uint32_t>> keyed(n);
  for (size_t i = 0; i < n; ++i) keyed[i] = {host_key(cand[i], now), (uint32_t)i};
  std::sort(keyed.begin(), keyed.end());
  uint64_t got = 0;
  for (auto& kv : keyed) {
    if (got >= need) break;
    const uint32_t s = cand[kv.second];
    picked.push_back(s);
    const BlockMeta* b = find(slot_block_[s]);
    got += b ? footprint(*b) : 0;
  }
  return picked;
}

void BlockStore::free_space_locked(std::unique_lock<std::mutex>& lk, int64_t session, uint64_t bytes,
                                   int tier, int dir, const std::string& medium, uint64_t ahead) {
  const auto wait_until = std::chrono::steady_clock::now() + std::chrono::seconds(2);
  // victims are selected for bytes + ahead (the reference's free-ahead: one eviction round makes
  // room for the next creates too); success needs only `bytes`
  const uint64_t goal = bytes + ahead;
  for (int attempt = 0; attempt < 4; ++attempt) {
    // target dir: the one that can reach `bytes` with the most (available + evictable)
    int target = -1;
    uint64_t best = 0;
    for (auto& d : dirs_) {
      if (dir >= 0 && d->index != dir) continue;
      if (!dir_matches(*d, tier, medium)) continue;
      const uint64_t reach = d->available() + dir_ev_bytes_[d->index];
      if (target < 0 || reach > best) { target = d->index; best = reach; }
    }
    if (target < 0) throw StoreError(kErrOutOfSpace, "no storage dir matches the eviction location");
    if (dirs_[target]->available() >= (attempt == 0 ? goal : bytes)) return;
    // arena dirs free whole pages: convert the shortfall into page-rounded bytes
    uint64_t need = (attempt == 0 ? goal : bytes) - std::min<uint64_t>(dirs_[target]->available(),
                                                                       attempt == 0 ? goal : bytes);
    if (dirs_[target]->spec.kind != DirKind::kFile)
      need = ceil_div(need, dirs_[target]->spec.page_size) * dirs_[target]->spec.page_size;
    ++stats_.selections;
    const uint64_t seq = create_seq_;
    std::vector<uint32_t> victims;
    if (device_evict_active()) {
      victims = select_victims_device(lk, target, need);
    } else {
      std::vector<uint32_t> cand;
      for (auto& kv : blocks_)
        if (kv.second.dir == target && evictable(kv.second)) cand.push_back(kv.second.slot);
      stats_.candidates += cand.size();
      victims = select_victims_cpu(cand, need);
    }
    // the store may have changed while it was unlocked: a victim must still be the same block
    // (created before the selection), in the target dir, and evictable now
    std::vector<int64_t> vids;
    size_t lost = 0;
    for (uint32_t s : victims) {
      BlockMeta* b = find(slot_block_[s]);
      if (b && b->seq <= seq && b->dir == target && evictable(*b)) {
        vids.push_back(b->id);
        ++stats_.victims;
      } else {
        ++stats_.revalidated_away;
        ++lost;
      }
    }
    const int lower = demote_on_evict_ ? lower_tier(dirs_[target]->spec.tier) : -1;
    if (lower >= 0 && !vids.empty()) {
      // demote into the next tier (making room there first) in one batched move
      std::vector<int64_t> moved = move_blocks_locked(lk, session, vids, lower, "", true);
      for (int64_t id : moved) {
        const BlockMeta* b = find(id);
        ++stats_.demoted_blocks;
        if (b) stats_.demoted_bytes += b->length;
      }
    }
    // what was not demoted is dropped
    for (int64_t id : vids) {
      BlockMeta* b = find(id);
      if (b && b->dir == target && evictable(*b)) remove_locked(*b, true);
    }
    if (dirs_[target]->available() >= bytes) return;
    // Blocks of the target dir that other threads are demoting right now are neither victims
    // nor free space yet: under concurrent ingest (many creates evicting at once) wait for those
    // moves to land (bounded) instead of failing the create.
    bool moving = false;
    for (int64_t id : evicting_ids_) {
      const BlockMeta* b = find(id);
      if (b && b->dir == target) {
        moving = true;
        break;
      }
    }
    if (moving && std::chrono::steady_clock::now() < wait_until) {
      ++stats_.evict_waits;
      lock_cv_.wait_for(lk, std::chrono::milliseconds(20));
      --attempt;                                     // a wait is not an attempt
      continue;
    }
    // Concurrent evictors select off-lock and pick the same coldest blocks: victims another
    // thread demoted first are revalidated away.  That is contention, not a full tier -- select
    // again (bounded by the same deadline).
    if (lost > 0 && std::chrono::steady_clock::now() < wait_until) {
      ++stats_.evict_retries;
      --attempt;
      continue;
    }
    if (victims.empty()) break;
  }
  throw StoreError(kErrOutOfSpace, "failed to free " + std::to_string(bytes) + " bytes (tier " +
                                       std::to_string(tier) + ", dir " + std::to_string(dir) + ")");
}

std::vector<int64_t> BlockStore::free_space(int64_t session, uint64_t bytes, int tier, int dir) {
  TraceRange trace_("BlockStore.free_space");
  set_device();
  std::unique_lock<std::mutex> lk(mu_);
  std::unordered_set<int64_t> before;
  for (auto& kv : blocks_) before.insert(kv.first);
  free_space_locked(lk, session, bytes, tier, dir, "");
  std::vector<int64_t> gone;
  for (int64_t id : before)
    if (!blocks_.count(id)) gone.push_back(id);
  return gone;
}

// Full annotator order (coldest first): a ranking, so it is the CPU sort (tier management uses
// ranks; eviction itself uses the device select).
std::vector<int64_t> BlockStore::eviction_order(int tier, uint64_t need_bytes) {
  std::unique_lock<std::mutex> lk(mu_);
  std::vector<uint32_t> cand;
  for (auto& kv : blocks_)
    if ((tier < 0 || dirs_[kv.second.dir]->spec.tier == tier) && evictable(kv.second)) cand.push_back(kv.second.slot);
  if (need_bytes == 0) need_bytes = ~0ull;
  std::vector<uint32_t> v = select_victims_cpu(cand, need_bytes);
  std::vector<int64_t> out;
  out.reserve(v.size());
  for (uint32_t s : v) out.push_back(slot_block_[s]);
  return out;
}

std::vector<int64_t> BlockStore::tier_order(int tier, uint32_t k, bool hottest, bool device) {
  set_device();
  std::unique_lock<std::mutex> lk(mu_);
  std::vector<uint32_t> slots;
  uint64_t mask = 0;
  for (auto& d : dirs_)
    if (d->spec.tier == tier && d->index < 64) mask |= 1ull << d->index;
  if (!mask || k == 0) return {};
  if (device && device_evict_active()) {
    // the k extremes by count on the device, O(n); only those k are ordered on the host
    slots = select_victims_device(lk, 0, k, mask, /*unit=*/true, /*invert=*/hottest);
    std::vector<uint32_t> ok;
    for (uint32_t s : slots) {
      const BlockMeta* b = find(slot_block_[s]);
      if (b && evictable(*b) && ((mask >> b->dir) & 1)) ok.push_back(s);
    }
    slots.swap(ok);
  } else {
    for (auto& kv : blocks_)
      if (((mask >> kv.second.dir) & 1) && evictable(kv.second)) slots.push_back(kv.second.slot);
  }
  const uint64_t now = clock_.load();
  std::vector<std::pair<uint32_t, uint32_t>> keyed;
  keyed.reserve(slots.size());
  for (uint32_t s : slots) keyed.push_back({host_key(s, now), s});
  if (hottest)
    std::sort(keyed.begin(), keyed.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
  else
    std::sort(keyed.begin(), keyed.end());
  std::vector<int64_t> out;
  for (size_t i = 0; i < keyed.size() && out.size() < k; ++i) out.push_back(slot_block_[keyed[i].second]);
  return out;
}

std::vector<uint32_t> BlockStore::annotator_keys(const std::vector<int64_t>& ids) {
  std::unique_lock<std::mutex> lk(mu_);
  const uint64_t now = clock_.load();
  std::vector<uint32_t> out;
  out.reserve(ids.size());
  for (int64_t id : ids) {
    const BlockMeta* b = find(id);
    out.push_back(b ? host_key(b->slot, now) : 0xFFFFFFFFu);
  }
  return out;
}

uint64_t BlockStore::dir_mgmt_available(int d) {
  std::unique_lock<std::mutex> lk(mu_);
  return dirs_.at(d)->mgmt_available();
}

std::vector<int64_t> BlockStore::select_for_bench(int dir, uint64_t need, bool device) {
  set_device();
  std::unique_lock<std::mutex> lk(mu_);
  if (dir < 0 || dir >= (int)dirs_.size()) throw StoreError(kErrInvalidArgument, "bad dir");
  std::vector<uint32_t> v;
  if (device) {
    if (!has_device_) throw StoreError(kErrInvalidArgument, "no device");
    const bool was = use_device_evict_;
    if (!was) dev_synced_ = false;
    use_device_evict_ = true;
    try {
      v = select_victims_device(lk, dir, need);
    } catch (...) {
      use_device_evict_ = was;
      throw;
    }
    use_device_evict_ = was;
  } else {
    std::vector<uint32_t> cand;
    for (auto& kv : blocks_)
      if (kv.second.dir == dir && evictable(kv.second)) cand.push_back(kv.second.slot);
    v = select_victims_cpu(cand, need);
  }
  std::vector<int64_t> out;
  out.reserve(v.size());
  for (uint32_t s : v) out.push_back(slot_block_[s]);
  return out;
}

BlockStore::EvictStats BlockStore::evict_stats() {
  std::unique_lock<std::mutex> lk(mu_);
  return stats_;
}

// -------------------------------------------------------------------------------------------
// K7: device page allocation for bulk creates
std::vector<int64_t> BlockStore::device_alloc_pages(std::unique_lock<std::mutex>& lk, int dir, uint32_t want) {
  StorageDir& d = *dirs_[dir];
  if (!d.mag_bits || want == 0) return {};
  // the magazine is refilled by whole host words (no per-page host scan); then one claim
  // kernel takes the pages with atomics and only the page list comes back
  if (d.mag_pages < (int64_t)want) mag_refill(d, (int64_t)want - d.mag_pages + std::min<int64_t>(1024, want));
  const uint32_t nwords = (uint32_t)d.free_bits.size();
  const std::pair<uint32_t, uint32_t> mwin = mag_window(d);
  std::vector<int64_t> pages;
  {
    std::unique_lock<std::mutex> g(ev_mu_);
    set_device();
    // a large claim is split into pieces of <= 1024 pages: one wave each, all in parallel
    constexpr uint32_t kPiece = 1024;
    const uint32_t npieces = (want + kPiece - 1) / kPiece;
    claim_reserve(claim_one_, npieces, want);
    for (uint32_t k = 0; k < npieces; ++k)
      claim_one_.items_h[k] = ClaimItem{0, 0, std::min(kPiece, want - k * kPiece), k * kPiece, 0, 0};
    lk.unlock();
    hipError_t e = hipMemcpyAsync(claim_one_.items_d, claim_one_.items_h, npieces * sizeof(ClaimItem),
                                  hipMemcpyHostToDevice, internal_stream_);
    if (e == hipSuccess)
      e = launch_mag_claim_scatter(d.mag_bits, nwords, claim_one_.items_d, npieces, claim_one_.pages_d,
                                   (uint32_t)claim_one_.pages_cap, claim_one_.got_d, 0, nullptr, 0, internal_stream_,
                                   mwin.first, mwin.second);
    if (e == hipSuccess)
      e = hipMemcpyAsync(claim_one_.got_h, claim_one_.got_d, npieces * sizeof(uint32_t), hipMemcpyDeviceToHost,
                         internal_stream_);
    if (e == hipSuccess)
      e = hipMemcpyAsync(claim_one_.pages_h, claim_one_.pages_d, (size_t)want * 8, hipMemcpyDeviceToHost, internal_stream_);
    if (e == hipSuccess) e = hipStreamSynchronize(internal_stream_);
    if (e == hipSuccess)
      for (uint32_t k = 0; k < npieces; ++k) {
        const ClaimItem& it = claim_one_.items_h[k];
        const uint32_t g = std::min(claim_one_.got_h[k], it.want);
        pages.insert(pages.end(), claim_one_.pages_h + it.page_base, claim_one_.pages_h + it.page_base + g);
      }
    for (int64_t p : pages)
      if (p < 0 || p >= d.num_pages) e = hipErrorInvalidValue;   // never hand out a bogus page
    g.unlock();
    lk.lock();
    if (e != hipSuccess) throw StoreError(kErrHip, std::string("device page claim: ") + hipGetErrorString(e));
  }
  // magazine pages were never in the host pool: only the counts move
  d.free_pages -= (int64_t)pages.size();
  d.mag_pages -= (int64_t)pages.size();
  ++stats_.device_allocs;
  stats_.device_alloc_pages += pages.size();
  return pages;
}

std::vector<int64_t> BlockStore::peek_free_pages(int dir, uint32_t want, bool device) {
  set_device();
  std::unique_lock<std::mutex> lk(mu_);
  if (dir < 0 || dir >= (int)dirs_.size() || dirs_[dir]->spec.kind == DirKind::kFile)
    throw StoreError(kErrInvalidArgument, "peek_free_pages needs an arena dir");
  StorageDir& d = *dirs_[dir];
  if (!device) {
    std::vector<int64_t> out;
    for (int64_t w = 0; w < (int64_t)d.free_bits.size() && out.size() < want; ++w) {
      uint64_t word = d.free_bits[w];
      while (word && out.size() < want) {
        const int b0 = __builtin_ctzll(word);
        word &= word - 1;
        if (w * 64 + b0 < d.num_pages) out.push_back(w * 64 + b0);
      }
    }
    return out;
  }
  if (!has_device_) throw StoreError(kErrInvalidArgument, "no device");
  std::vector<int64_t> got = device_alloc_pages(lk, dir, want);
  // give them back: a peek
  for (int64_t p : got) {
    bit_give(d.free_bits, p);
    ++d.free_pages;
  }
  --stats_.device_allocs;
  stats_.device_alloc_pages -= got.size();
  return got;
}

std::vector<int> BlockStore::create_blocks(int64_t session, const std::vector<int64_t>& ids, int tier,
                                           const std::string& medium, const std::vector<uint64_t>& sizes,
                                           bool evict) {
  TraceRange trace_("BlockStore.create_blocks");
  if (ids.size() != sizes.size()) throw StoreError(kErrInvalidArgument, "ids/sizes length mismatch");
  set_device();
  std::unique_lock<std::mutex> lk(mu_);
  std::unordered_set<int64_t> seen;
  uint64_t total = 0;
  for (size_t i = 0; i < ids.size(); ++i) {
    if (blocks_.count(ids[i]) || !seen.insert(ids[i]).second)
      throw StoreError(kErrAlreadyExists, "block " + std::to_string(ids[i]) + " already exists");
    total += std::max<uint64_t>(sizes[i], 1);
  }
  int d = allocate_dir(tier, medium, total);
  if (d < 0 && evict) {
    free_space_locked(lk, session, total, tier, -1, medium);
    for (int64_t id : ids)
      if (blocks_.count(id)) throw StoreError(kErrAlreadyExists, "block " + std::to_string(id) + " already exists");
    d = allocate_dir(tier, medium, total);
  }
  std::vector<int> out;
  if (d < 0) {
    // no single dir holds all of them: one at a time (each may pick its own dir)
    lk.unlock();
    for (size_t i = 0; i < ids.size(); ++i) out.push_back(create_block(session, ids[i], tier, medium, sizes[i], evict, false));
    return out;
  }
  StorageDir& sd = *dirs_[d];
  std::vector<int64_t> pool;
  size_t pool_pos = 0;
  // K7 pays off per block (the host path walks each block's page list), not per page: the host
  // word scan claims the pages of one huge block faster than a kernel round trip (0.49 vs 1.2 ms at
  // 75k pages, profiles/r3_evict_bench_arc.jsonl), so few-block creates stay on the host
  if (sd.spec.kind == DirKind::kDevice && use_device_alloc_ && ids.size() >= kDeviceAllocMinBlocks) {
    uint64_t want = 0;
    for (uint64_t sz : sizes) want += ceil_div(std::max<uint64_t>(sz, 1), sd.spec.page_size);
    if (want >= device_alloc_min_pages_ && (int64_t)want <= sd.free_pages - sd.reserved_pages)
      pool = device_alloc_pages(lk, d, (uint32_t)want);
  }
  for (size_t i = 0; i < ids.size(); ++i) {
    if (blocks_.count(ids[i])) {
      for (size_t k = pool_pos; k < pool.size(); ++k) { bit_give(sd.free_bits, pool[k]); ++sd.free_pages; }
      throw StoreError(kErrAlreadyExists, "block " + std::to_string(ids[i]) + " already exists");
    }
    BlockMeta b;
    b.id = ids[i];
    b.dir = d;
    b.temp = true;
    b.session = session;
    const uint64_t sz = std::max<uint64_t>(sizes[i], 1);
    if (sd.spec.kind != DirKind::kFile && pool_pos < pool.size()) {
      const size_t np = (size_t)ceil_div(sz, sd.spec.page_size);
      while (b.pages.size() < np && pool_pos < pool.size()) b.pages.push_back(pool[pool_pos++]);
      b.reserved = b.pages.size() * sd.spec.page_size;
    }
    if (!grow_pages(sd, b, sz)) {
      release_storage(b);
      for (size_t k = pool_pos; k < pool.size(); ++k) { bit_give(sd.free_bits, pool[k]); ++sd.free_pages; }
      throw StoreError(kErrOutOfSpace, "bulk allocation ran out of space at block " + std::to_string(ids[i]));
    }
    b.slot = alloc_slot();
    b.seq = ++create_seq_;
    slot_block_[b.slot] = b.id;
    crf_[b.slot] = 0.f;
    last_[b.slot] = clock_.load();
    note_state(b, true);
    if (sd.spec.kind == DirKind::kFile) {
      const std::string p = sd.spec.path + "/.tmp_blocks/" + std::to_string(session) + "-" + std::to_string(b.id);
      int fd = ::open(p.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
      if (fd < 0) throw StoreError(kErrIo, "cannot create " + p);
      ::close(fd);
    }
    session_temps_[session].insert(b.id);
    blocks_.emplace(b.id, std::move(b));
    out.push_back(d);
  }
  for (size_t k = pool_pos; k < pool.size(); ++k) { bit_give(sd.free_bits, pool[k]); ++sd.free_pages; }
  return out;
}

// -------------------------------------------------------------------------------------------
// introspection
bool BlockStore::has_block(int64_t id) {
  std::unique_lock<std::mutex> lk(mu_);
  BlockMeta* b = find(id);
  return b && !b->temp;
}

bool BlockStore::has_temp_block(int64_t id) {
  std::unique_lock<std::mutex> lk(mu_);
  BlockMeta* b = find(id);
  return b && b->temp;
}

BlockInfoOut BlockStore::block_info(int64_t id) {
  std::unique_lock<std::mutex> lk(mu_);
  BlockMeta* b = find(id);
  if (!b) throw StoreError(kErrNotFound, "block " + std::to_string(id) + " does not exist");
  const auto& s = dirs_[b->dir]->spec;
  return BlockInfoOut{b->id, b->length, s.tier, b->dir, s.tier_alias, s.medium, b->temp, b->session,
                      b->readers, b->writer};
}

std::vector<int64_t> BlockStore::block_ids(int tier) {
  std::unique_lock<std::mutex> lk(mu_);
  std::vector<int64_t> out;
  for (auto& kv : blocks_)
    if (!kv.second.temp && (tier < 0 || dirs_[kv.second.dir]->spec.tier == tier)) out.push_back(kv.first);
  std::sort(out.begin(), out.end());
  return out;
}

std::vector<int64_t> BlockStore::block_pages(int64_t id, int* dir_out, uint64_t* ps_out, uint64_t* base_out) {
  std::unique_lock<std::mutex> lk(mu_);
  BlockMeta* b = find(id);
  if (!b) throw StoreError(kErrNotFound, "block " + std::to_string(id) + " does not exist");
  const auto& s = dirs_[b->dir]->spec;
  *dir_out = b->dir;
  *ps_out = s.page_size;
  *base_out = s.base;
  return b->pages;
}

int64_t BlockStore::mag_refill_pages(int dir, int64_t pages) {
  std::unique_lock<std::mutex> lk(mu_);
  StorageDir& d = *dirs_.at(dir);
  const int64_t before = d.mag_pages;
  mag_refill(d, pages);
  return d.mag_pages - before;
}

int64_t BlockStore::mag_pages(int dir) {
  std::unique_lock<std::mutex> lk(mu_);
  return dirs_.at(dir)->mag_pages;
}

int64_t BlockStore::mag_device_count(int dir) {
  std::unique_lock<std::mutex> lk(mu_);
  StorageDir& d = *dirs_.at(dir);
  if (!d.mag_bits) return 0;
  std::vector<uint64_t> w(d.free_bits.size());
  HIP_OK(hipStreamSynchronize(internal_stream_));
  HIP_OK(hipMemcpy(w.data(), d.mag_bits, w.size() * 8, hipMemcpyDeviceToHost));
  int64_t n = 0;
  for (uint64_t x : w) n += __builtin_popcountll(x);
  return n;
}

std::string BlockStore::check_pages(int dir) {
  std::unique_lock<std::mutex> lk(mu_);
  StorageDir& d = *dirs_.at(dir);
  if (d.free_bits.empty()) return "";                       // file dirs: no page accounting
  std::string err;
  auto fail = [&](const std::string& m) {
    if (err.size() < 2000) err += m + "; ";
  };
  std::vector<uint64_t> mag(d.free_bits.size(), 0);
  if (d.mag_bits) {
    HIP_OK(hipStreamSynchronize(internal_stream_));
    HIP_OK(hipMemcpy(mag.data(), d.mag_bits, mag.size() * 8, hipMemcpyDeviceToHost));
  }
  int64_t host_free = 0, mag_n = 0;
  for (size_t w = 0; w < mag.size(); ++w) {
    host_free += __builtin_popcountll(d.free_bits[w]);
    mag_n += __builtin_popcountll(mag[w]);
    if (d.free_bits[w] & mag[w]) fail("word " + std::to_string(w) + " has pages both in the host pool and the magazine");
  }
  if (mag_n != d.mag_pages)
    fail("magazine bitmap holds " + std::to_string(mag_n) + " pages, mag_pages says " + std::to_string(d.mag_pages));
  if (host_free + d.mag_pages != d.free_pages)
    fail("host pool " + std::to_string(host_free) + " + magazine " + std::to_string(d.mag_pages) + " != free_pages " +
         std::to_string(d.free_pages));
  std::vector<uint8_t> owner(d.num_pages, 0);
  int64_t owned = 0;
  for (const auto& kv : blocks_) {
    const BlockMeta& b = kv.second;
    if (b.dir != dir) continue;
    for (int64_t p : b.pages) {
      if (p < 0 || p >= d.num_pages) {
        fail("block " + std::to_string(b.id) + " owns out-of-range page " + std::to_string(p));
        continue;
      }
      const size_t w = (size_t)p / 64;
      const uint64_t bit = 1ull << (p % 64);
      if (owner[p]++) fail("page " + std::to_string(p) + " owned twice (block " + std::to_string(b.id) + ")");
      if ((d.free_bits[w] | mag[w]) & bit) fail("page " + std::to_string(p) + " of block " + std::to_string(b.id) + " is also free");
      ++owned;
    }
  }
  if (owned + d.free_pages != d.num_pages)
    fail("owned " + std::to_string(owned) + " + free " + std::to_string(d.free_pages) + " != " +
         std::to_string(d.num_pages) + " pages");
  return err;
}

std::vector<std::vector<int64_t>> BlockStore::mag_claim_many(int dir, const std::vector<uint32_t>& wants) {
  std::unique_lock<std::mutex> lk(mu_);
  StorageDir& d = *dirs_.at(dir);
  std::vector<std::vector<int64_t>> out(wants.size());
  if (!d.mag_bits || wants.empty()) return out;
  std::unique_lock<std::mutex> g(ev_mu_);
  size_t total = 0;
  for (uint32_t w : wants) total += w;
  claim_reserve(claim_one_, wants.size(), total);
  uint32_t pb = 0;
  for (size_t i = 0; i < wants.size(); ++i) {
    claim_one_.items_h[i] = ClaimItem{0, 0, wants[i], pb, 0, 0};
    pb += wants[i];
  }
  HIP_OK(hipMemcpyAsync(claim_one_.items_d, claim_one_.items_h, wants.size() * sizeof(ClaimItem), hipMemcpyHostToDevice,
                        internal_stream_));
  const std::pair<uint32_t, uint32_t> mwin = mag_window(d);
  HIP_OK(launch_mag_claim_scatter(d.mag_bits, (uint32_t)d.free_bits.size(), claim_one_.items_d, (uint32_t)wants.size(),
                                  claim_one_.pages_d, (uint32_t)claim_one_.pages_cap, claim_one_.got_d, 0, nullptr, 0,
                                  internal_stream_, mwin.first, mwin.second));
  HIP_OK(hipMemcpyAsync(claim_one_.got_h, claim_one_.got_d, wants.size() * 4, hipMemcpyDeviceToHost, internal_stream_));
  HIP_OK(hipMemcpyAsync(claim_one_.pages_h, claim_one_.pages_d, std::max<size_t>(total, 1) * 8, hipMemcpyDeviceToHost,
                        internal_stream_));
  HIP_OK(hipStreamSynchronize(internal_stream_));
  for (size_t i = 0; i < wants.size(); ++i) {
    const ClaimItem& it = claim_one_.items_h[i];
    const uint32_t g = std::min(claim_one_.got_h[i], it.want);
    out[i].assign(claim_one_.pages_h + it.page_base, claim_one_.pages_h + it.page_base + g);
    d.mag_pages -= g;
  }
  return out;
}

void BlockStore::mag_give(int dir, const std::vector<int64_t>& pages) {
  std::unique_lock<std::mutex> lk(mu_);
  StorageDir& d = *dirs_.at(dir);
  for (int64_t p : pages) bit_give(d.free_bits, p);
}

int64_t BlockStore::mag_drain_dir(int dir) {
  std::unique_lock<std::mutex> lk(mu_);
  return mag_drain(*dirs_.at(dir));
}

std::string BlockStore::committed_file(int64_t id) {
  std::unique_lock<std::mutex> lk(mu_);
  BlockMeta* b = find(id);
  if (!b || b->temp || b->dir < 0) return std::string();
  const StorageDir& d = *dirs_[b->dir];
  if (d.spec.kind != DirKind::kFile) return std::string();
  std::string p;
  file_path(d, id, p);
  return p;
}

std::vector<Event> BlockStore::drain_events() {
  std::unique_lock<std::mutex> lk(mu_);
  std::vector<Event> out;
  out.swap(events_);
  return out;
}

uint64_t BlockStore::dir_capacity(int d) {
  std::unique_lock<std::mutex> lk(mu_);
  return dirs_.at(d)->capacity();
}
uint64_t BlockStore::dir_available(int d) {
  std::unique_lock<std::mutex> lk(mu_);
  return dirs_.at(d)->available();
}
uint64_t BlockStore::dir_committed(int d) {
  std::unique_lock<std::mutex> lk(mu_);
  return dirs_.at(d)->committed_bytes;
}
void BlockStore::set_dir_healthy(int d, bool healthy) {
  std::unique_lock<std::mutex> lk(mu_);
  dirs_.at(d)->healthy = healthy;
}
bool BlockStore::dir_healthy(int d) {
  std::unique_lock<std::mutex> lk(mu_);
  return dirs_.at(d)->healthy;
}

std::string BlockStore::stats() {
  std::unique_lock<std::mutex> lk(mu_);
  std::ostringstream os;
  os << "{\"blocks\":" << blocks_.size() << ",\"locks\":" << locks_.size() << ",\"clock\":" << clock_.load()
     << ",\"dirs\":[";
  for (size_t i = 0; i < dirs_.size(); ++i) {
    const auto& d = *dirs_[i];
    os << (i ? "," : "") << "{\"tier\":" << d.spec.tier << ",\"alias\":\"" << d.spec.tier_alias
       << "\",\"medium\":\"" << d.spec.medium << "\",\"capacity\":" << d.capacity()
       << ",\"available\":" << d.available() << ",\"committed\":" << d.committed_bytes << "}";
  }
  os << "]}";
  return os.str();
}

}  // namespace amdx

namespace amdx {

int64_t BlockStore::try_lock_block(int64_t session, int64_t block_id, bool write) {
  try {
    return lock_block(session, block_id, write, 30000);
  } catch (const StoreError& e) {
    if (e.code == kErrNotFound) return -1;
    throw;
  }
}

// -------------------------------------------------------------------------------------------
// ReadSession
ReadSession::ReadSession(BlockStore* store, int64_t session, const std::vector<int64_t>& block_ids,
                         const std::vector<uint64_t>& block_lens, const std::vector<uint64_t>& dst_ptrs,
                         uint64_t buf_bytes, int dst_kind, const std::vector<uint64_t>& start_offsets)
    : store_(store), session_(session), dst_(dst_ptrs), buf_(buf_bytes), kind_(dst_kind) {
  if (buf_ == 0) throw StoreError(kErrInvalidArgument, "buffer size must be > 0");
  reset_file(block_ids, block_lens);
  const size_t n = dst_.size();
  pos_.assign(n, 0);
  for (size_t i = 0; i < n && i < start_offsets.size(); ++i) pos_[i] = file_len_ ? start_offsets[i] % file_len_ : 0;
  cur_block_idx_.assign(n, -1);
  lock_.assign(n, -1);
  reqs_.reserve(2 * n);
}

ReadSession::~ReadSession() {
  try { close(); } catch (...) {}
}

void ReadSession::reset_file(const std::vector<int64_t>& block_ids, const std::vector<uint64_t>& block_lens) {
  if (block_ids.size() != block_lens.size()) throw StoreError(kErrInvalidArgument, "block id/len size mismatch");
  blocks_ = block_ids;
  lens_ = block_lens;
  starts_.assign(blocks_.size(), 0);
  file_len_ = 0;
  for (size_t b = 0; b < blocks_.size(); ++b) {
    starts_[b] = file_len_;
    file_len_ += lens_[b];
  }
}

void ReadSession::switch_block(int i, int64_t b) {
  if (cur_block_idx_[i] == b) return;
  if (lock_[i] >= 0) {
    store_->unlock(lock_[i]);
    lock_[i] = -1;
  }
  cur_block_idx_[i] = -1;
  if (b >= 0) {
    const int64_t l = store_->try_lock_block(session_, blocks_[b], false);
    if (l < 0) throw StoreError(kErrNotFound, "block " + std::to_string(blocks_[b]) + " is not cached on this worker");
    lock_[i] = l;
    cur_block_idx_[i] = b;
  }
}

uint64_t ReadSession::step(uint64_t stream, std::vector<int>* reopened) {
  if (closed_) throw StoreError(kErrInvalidState, "read session closed");
  reqs_.clear();
  uint64_t bytes = 0;
  std::vector<int64_t> touched;
  for (size_t i = 0; i < dst_.size(); ++i) {
    uint64_t p = pos_[i];
    if (p >= file_len_) {  // read() returned -1: close + re-open at offset 0
      switch_block((int)i, -1);
      pos_[i] = 0;
      ++reopens_;
      if (reopened) reopened->push_back((int)i);
      continue;
    }
    uint64_t want = std::min(buf_, file_len_ - p);
    uint64_t out = 0;
    while (want > 0) {
      // block index of position p (blocks are few; linear from the current block)
      int64_t b = cur_block_idx_[i] >= 0 ? cur_block_idx_[i] : 0;
      if (p < starts_[b]) b = 0;
      while (b + 1 < (int64_t)blocks_.size() && p >= starts_[b + 1]) ++b;
      switch_block((int)i, b);
      const uint64_t off = p - starts_[b];
      const uint64_t n = std::min(want, lens_[b] - off);
      reqs_.push_back(ReadReq{blocks_[b], off, n, dst_[i] + out, kind_});
      touched.push_back(blocks_[b]);
      p += n;
      out += n;
      want -= n;
    }
    pos_[i] = p;
    bytes += out;
  }
  // host destinations are consumed by the CPU as soon as read() returns: complete the DMA;
  // device destinations stay ordered on the caller's stream
  if (!reqs_.empty()) store_->read_batch(reqs_, stream, kind_ == (int)MemKind::kHost);
  // annotate accesses once per distinct block per step (LRU/LRFU clock)
  std::sort(touched.begin(), touched.end());
  touched.erase(std::unique(touched.begin(), touched.end()), touched.end());
  store_->access_blocks(touched);
  total_ += bytes;
  return bytes;
}

uint64_t ReadSession::run(int steps, uint64_t stream) {
  uint64_t b = 0;
  for (int s = 0; s < steps; ++s) b += step(stream, nullptr);
  return b;
}

void ReadSession::close() {
  if (closed_) return;
  closed_ = true;
  for (size_t i = 0; i < lock_.size(); ++i) {
    if (lock_[i] >= 0) {
      try { store_->unlock(lock_[i]); } catch (...) {}
      lock_[i] = -1;
    }
  }
}

std::vector<int> BlockStore::ingest_files(int64_t session, const std::vector<int64_t>& ids,
                                          const std::vector<std::string>& paths,
                                          const std::vector<uint64_t>& offsets,
                                          const std::vector<uint64_t>& lengths, uint64_t staging,
                                          uint64_t staging_bytes, int threads, uint64_t stream) {
  TraceRange trace_("BlockStore.ingest_files");
  std::lock_guard<std::mutex> ingest_guard(ingest_mu_);
  for (auto& c : claim_) {                       // nothing of an aborted earlier call carries over
    c.ids.clear();
    c.index.clear();
    c.at.clear();
  }
  const size_t n = ids.size();
  if (paths.size() != n || offsets.size() != n || lengths.size() != n)
    throw StoreError(kErrInvalidArgument, "ingest_files: argument lengths differ");
  if (!staging || staging_bytes < 2) throw StoreError(kErrInvalidArgument, "ingest_files: no staging buffer");
  set_device();
  hipStream_t st = stream_or_default(stream);
  const uint64_t half = staging_bytes / 2;
  for (uint64_t len : lengths)
    if (len > half) throw StoreError(kErrInvalidArgument, "ingest_files: a file is larger than half the staging buffer");
  threads = std::max(1, std::min(threads, 64));
  std::vector<int> status(n, 0);
  // groups of consecutive items that fit one staging half
  std::vector<std::pair<size_t, size_t>> groups;
  for (size_t i = 0; i < n;) {
    size_t j = i;
    uint64_t used = 0;
    while (j < n && used + lengths[j] <= half) used += lengths[j++];
    groups.emplace_back(i, j);
    i = j;
  }
  std::vector<std::vector<int64_t>> pending(2);   // blocks whose copy from staging half h is in flight
  std::vector<uint8_t*> host_half(2, nullptr);
  uint64_t phase_ns[6] = {0, 0, 0, 0, 0, 0};
  auto tick = [t = std::chrono::steady_clock::now()](uint64_t& acc) mutable {
    const auto now = std::chrono::steady_clock::now();
    acc += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(now - t).count();
    t = now;
  };
  uint64_t scratch_ns = 0;
  tick(scratch_ns);
  if (use_device_alloc_ && has_device_) {
    // K7: one magazine refill for the whole call up front -- a refill synchronizes the internal
    // stream, which would otherwise stall the staging double buffer once per group
    std::unique_lock<std::mutex> g2(mu_);
    const int d0 = allocate_dir(0, "", 1);
    if (d0 >= 0 && dirs_[d0]->spec.kind == DirKind::kDevice && dirs_[d0]->mag_bits) {
      StorageDir& sd = *dirs_[d0];
      int64_t need = 0;
      for (uint64_t len : lengths) need += (int64_t)ceil_div(std::max<uint64_t>(len, 1), sd.spec.page_size);
      need = std::min<int64_t>(need, sd.free_pages - sd.reserved_pages);
      if (sd.mag_pages < need) mag_refill(sd, need - sd.mag_pages);
    }
  }
  tick(phase_ns[5]);
  auto finish = [&](int h) {
    if (pending[h].empty() && claim_[h].ids.empty()) return;
    tick(phase_ns[2]);
    if (has_device_) HIP_OK(hipStreamSynchronize(st));
    tick(phase_ns[3]);
    if (!claim_[h].ids.empty()) {
      const std::unordered_set<int64_t> failed = ingest_device_finish(session, h, lengths, host_half[h], status);
      if (!failed.empty()) {
        std::vector<int64_t> keep;
        for (int64_t id : pending[h])
          if (!failed.count(id)) keep.push_back(id);
        pending[h].swap(keep);
      }
    }
    for (int64_t id : pending[h]) commit_block(session, id, false);
    pending[h].clear();
    tick(phase_ns[4]);
  };
  for (size_t g = 0; g < groups.size(); ++g) {
    const int h = (int)(g & 1);
    finish(h);                                     // staging half h is free again
    const size_t lo = groups[g].first, hi = groups[g].second;
    uint8_t* base = reinterpret_cast<uint8_t*>(staging) + h * half;
    host_half[h] = base;
    std::vector<uint64_t> at(hi - lo);
    uint64_t off = 0;
    for (size_t i = lo; i < hi; ++i) { at[i - lo] = off; off += lengths[i]; }
    // 1) temp blocks (skip ones that exist).  K7: blocks bound for an HBM dir are created without
    // pages -- the scatter kernel claims them from the dir's device magazine below
    std::vector<int64_t> gid;
    std::vector<uint64_t> gsz;
    std::vector<size_t> gix;
    int fused_dir = -1;
    {
      std::unique_lock<std::mutex> g2(mu_);
      for (size_t i = lo; i < hi; ++i) {
        if (blocks_.count(ids[i])) { status[i] = 1; continue; }
        gid.push_back(ids[i]);
        gsz.push_back(lengths[i]);
        gix.push_back(i);
      }
      if (!gid.empty() && use_device_alloc_ && has_device_) {
        uint64_t total = 0, want = 0;
        for (uint64_t sz : gsz) total += std::max<uint64_t>(sz, 1);
        int d = allocate_dir(0, "", total);
        if (d < 0) {
          free_space_locked(g2, session, total, 0, -1, "");
          d = allocate_dir(0, "", total);
        }
        bool fresh = true;
        for (int64_t id : gid) fresh = fresh && !blocks_.count(id);
        if (d >= 0 && fresh && dirs_[d]->spec.kind == DirKind::kDevice && dirs_[d]->mag_bits) {
          StorageDir& sd = *dirs_[d];
          for (uint64_t sz : gsz) want += ceil_div(std::max<uint64_t>(sz, 1), sd.spec.page_size);
          if (sd.mag_pages < (int64_t)want) mag_refill(sd, (int64_t)want - sd.mag_pages);
          // reserved now: a group launched before this one finishes must not count these pages
          sd.mag_pages -= (int64_t)want;
          for (size_t k = 0; k < gid.size(); ++k) {
            BlockMeta b;
            b.id = gid[k];
            b.dir = d;
            b.temp = true;
            b.session = session;
            b.slot = alloc_slot();
            b.seq = ++create_seq_;
            slot_block_[b.slot] = b.id;
            crf_[b.slot] = 0.f;
            last_[b.slot] = clock_.load();
            note_state(b, true);
            session_temps_[session].insert(b.id);
            blocks_.emplace(b.id, std::move(b));
          }
          fused_dir = d;
        }
      }
    }
    if (gid.empty()) continue;
    if (fused_dir < 0) {
      try {
        create_blocks(session, gid, 0, "", gsz, true);
      } catch (const StoreError&) {
        // mixed case (a racing creator, or no single dir fits the group): one at a time
        for (size_t k = 0; k < gid.size(); ++k) {
          if (has_temp_block(gid[k]) || has_block(gid[k])) {
            std::lock_guard<std::mutex> g2(mu_);
            BlockMeta* b = find(gid[k]);
            if (b && b->temp && b->session == session) continue;   // created by the bulk call
            status[gix[k]] = 1;
            continue;
          }
          try {
            create_block(session, gid[k], 0, "", std::max<uint64_t>(gsz[k], 1), true, false);
          } catch (const StoreError& e) {
            status[gix[k]] = e.code == kErrAlreadyExists ? 1 : 3;
          }
        }
      }
    }
    tick(phase_ns[0]);
    // 2) parallel preads into the staging half
    std::atomic<size_t> next{0};
    auto reader = [&]() {
      for (size_t k; (k = next.fetch_add(1)) < gix.size();) {
        const size_t i = gix[k];
        if (status[i] != 0) continue;
        int fd = ::open(paths[i].c_str(), O_RDONLY | O_CLOEXEC);
        if (fd < 0) { status[i] = 2; continue; }
        uint64_t got = 0;
        while (got < lengths[i]) {
          ssize_t r = ::pread(fd, base + at[i - lo] + got, lengths[i] - got, (off_t)(offsets[i] + got));
          if (r <= 0) break;
          got += (uint64_t)r;
        }
        ::close(fd);
        if (got != lengths[i]) status[i] = 2;
      }
    };
    const int nt = (int)std::min<size_t>((size_t)threads, gix.size());
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(reader);
    reader();
    for (auto& t : pool) t.join();
    tick(phase_ns[1]);
    for (size_t k = 0; k < gix.size(); ++k)
      if (status[gix[k]] == 2) {
        try { abort_block(session, ids[gix[k]]); } catch (const StoreError&) {}
      }
    // 3) copies into the blocks (async); commit once the half's copies are done.  Blocks in an
    // HBM dir: the used span of the half goes up in ONE DMA to a device staging buffer and one
    // batched-copy launch scatters it into the blocks' pages (one 128 KiB DMA per block runs
    // at ~13 GB/s; the single large DMA at full link rate).
    std::vector<size_t> dev_items, host_items;
    {
      std::lock_guard<std::mutex> g2(mu_);
      for (size_t k = 0; k < gix.size(); ++k) {
        const size_t i = gix[k];
        if (status[i] != 0) continue;
        BlockMeta* b = find(ids[i]);
        const bool dev = b && has_device_ && dirs_[b->dir]->spec.kind == DirKind::kDevice &&
                         (fused_dir >= 0 || b->reserved >= lengths[i]);
        (dev ? dev_items : host_items).push_back(i);
      }
    }
    if (!dev_items.empty()) {
      if (ingest_dev_cap_ < staging_bytes) {
        HIP_OK(hipStreamSynchronize(st));
        if (ingest_dev_) hipFree(ingest_dev_);
        ingest_dev_ = nullptr;
        HIP_OK(hipMalloc(&ingest_dev_, staging_bytes));
        ingest_dev_cap_ = staging_bytes;
      }
      uint8_t* dbase = reinterpret_cast<uint8_t*>(ingest_dev_) + h * half;
      HIP_OK(hipMemcpyAsync(dbase, base, off, hipMemcpyHostToDevice, st));
      if (fused_dir >= 0) {
        ingest_device_group(session, ids, lengths, dev_items, at, lo, dbase, h, st, pending[h]);
        claim_[h].dir = fused_dir;
      } else {
        std::vector<CopySeg> segs;
        {
          std::lock_guard<std::mutex> g2(mu_);
          for (size_t i : dev_items) {
            BlockMeta* b = find(ids[i]);
            b->length = std::max(b->length, lengths[i]);
            plan_block_range(*b, 0, lengths[i], (uint64_t)(dbase + at[i - lo]), (int)MemKind::kDevice, true, segs, st);
            pending[h].push_back(ids[i]);
          }
        }
        if (!segs.empty()) copy_segments(segs, st);
      }
    }
    for (size_t i : host_items) {
      try {
        write(session, ids[i], 0, (uint64_t)(base + at[i - lo]), lengths[i], (int)MemKind::kHost, stream, false);
        pending[h].push_back(ids[i]);
      } catch (const StoreError&) {
        status[i] = 3;
        try { abort_block(session, ids[i]); } catch (const StoreError&) {}
      }
    }
  }
  finish(0);
  finish(1);
  tick(phase_ns[2]);
  {
    std::lock_guard<std::mutex> g(mu_);
    for (int k = 0; k < 6; ++k) stats_.ingest_ns[k] += phase_ns[k];
  }
  return status;
}

void BlockStore::claim_reserve(ClaimScratch& c, size_t items, size_t pages) {
  if (c.items_cap < items) {
    if (c.items_d) hipFree(c.items_d);
    if (c.items_h) hipHostFree(c.items_h);
    if (c.got_d) hipFree(c.got_d);
    if (c.got_h) hipHostFree(c.got_h);
    c.items_d = nullptr;
    c.items_h = nullptr;
    c.got_d = nullptr;
    c.got_h = nullptr;
    const size_t cap = std::max<size_t>(items, 1024);
    HIP_OK(hipMalloc((void**)&c.items_d, cap * sizeof(ClaimItem)));
    HIP_OK(hipHostMalloc((void**)&c.items_h, cap * sizeof(ClaimItem), hipHostMallocDefault));
    HIP_OK(hipMalloc((void**)&c.got_d, cap * sizeof(uint32_t)));
    HIP_OK(hipHostMalloc((void**)&c.got_h, cap * sizeof(uint32_t), hipHostMallocDefault));
    c.items_cap = cap;
  }
  if (c.pages_cap < pages) {
    if (c.pages_d) hipFree(c.pages_d);
    if (c.pages_h) hipHostFree(c.pages_h);
    c.pages_d = nullptr;
    c.pages_h = nullptr;
    const size_t cap = std::max<size_t>(pages, 4096);
    HIP_OK(hipMalloc((void**)&c.pages_d, cap * sizeof(int64_t)));
    HIP_OK(hipHostMalloc((void**)&c.pages_h, cap * sizeof(int64_t), hipHostMallocDefault));
    c.pages_cap = cap;
  }
}

// K7 fused path of ingest_files for one staging half: one item per block (device source, length,
// pages wanted); the claim kernel takes the pages from the dir's magazine and the scatter kernel
// copies each block into them -- no per-page host descriptors, no host bitmap scan.  The page
// lists come back with the half's other results (ingest_device_finish).
bool BlockStore::ingest_device_group(int64_t session, const std::vector<int64_t>& ids,
                                     const std::vector<uint64_t>& lengths, const std::vector<size_t>& items,
                                     const std::vector<uint64_t>& at, size_t lo, uint8_t* dbase, int h,
                                     hipStream_t st, std::vector<int64_t>& pending) {
  (void)session;
  ClaimScratch& c = claim_[h];
  uint64_t ps = 0;
  int d = -1;
  std::pair<uint32_t, uint32_t> mwin{0u, 0u};
  {
    std::lock_guard<std::mutex> g(mu_);
    BlockMeta* b = find(ids[items[0]]);
    d = b->dir;
    ps = dirs_[d]->spec.page_size;
    mwin = mag_window(*dirs_[d]);
  }
  size_t npages = 0, nchunks = 0;
  for (size_t i : items) {
    npages += (size_t)ceil_div(std::max<uint64_t>(lengths[i], 1), ps);
    nchunks += (size_t)ceil_div(std::max<uint64_t>(lengths[i], 1), 64 * 1024);
  }
  claim_reserve(c, items.size(), npages);
  c.ids.clear();
  c.index.clear();
  c.at.clear();
  uint32_t pb = 0, cb = 0;
  for (size_t k = 0; k < items.size(); ++k) {
    const size_t i = items[k];
    const uint64_t len = std::max<uint64_t>(lengths[i], 1);
    const uint32_t want = (uint32_t)ceil_div(len, ps);
    c.items_h[k] = ClaimItem{(uint64_t)(dbase + at[i - lo]), lengths[i], want, pb, cb, 0};
    pb += want;
    cb += (uint32_t)ceil_div(len, 64 * 1024);
    c.ids.push_back(ids[i]);
    c.index.push_back(i);
    c.at.push_back(at[i - lo]);
  }
  const uint32_t nwords = (uint32_t)dirs_[d]->free_bits.size();
  HIP_OK(hipMemcpyAsync(c.items_d, c.items_h, items.size() * sizeof(ClaimItem), hipMemcpyHostToDevice, st));
  HIP_OK(launch_mag_claim_scatter(dirs_[d]->mag_bits, nwords, c.items_d, (uint32_t)items.size(), c.pages_d,
                                  (uint32_t)c.pages_cap, c.got_d, (uint32_t)nchunks,
                                  reinterpret_cast<uint8_t*>(dirs_[d]->spec.base), ps, st, mwin.first, mwin.second));
  HIP_OK(hipMemcpyAsync(c.pages_h, c.pages_d, npages * sizeof(int64_t), hipMemcpyDeviceToHost, st));
  HIP_OK(hipMemcpyAsync(c.got_h, c.got_d, items.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  for (int64_t id : c.ids) pending.push_back(id);
  return true;
}

// After the half's stream work completed: attach the claimed pages to their blocks.  A block
// that came up short (magazine drained meanwhile) gives its pages to the host pool and is
// written the host way from the still-intact staging half.
std::unordered_set<int64_t> BlockStore::ingest_device_finish(int64_t session, int h, const std::vector<uint64_t>& lengths,
                                                             const uint8_t* host_base, std::vector<int>& status) {
  ClaimScratch& c = claim_[h];
  std::vector<size_t> redo;
  std::unordered_set<int64_t> failed;
  {
    std::lock_guard<std::mutex> g(mu_);
    StorageDir& d = *dirs_[c.dir];
    const uint64_t ps = d.spec.page_size;
    for (size_t k = 0; k < c.ids.size(); ++k) {
      const ClaimItem& it = c.items_h[k];
      const uint32_t got = std::min(c.got_h[k], it.want);
      BlockMeta* b = find(c.ids[k]);
      d.mag_pages += (int64_t)it.want - got;     // the group reserved `want`; only `got` left the magazine
      if (!b || got < it.want) {
        ++stats_.mag_short_items;
        for (uint32_t j = 0; j < got; ++j) bit_give(d.free_bits, c.pages_h[it.page_base + j]);
        if (b) redo.push_back(k);
        else failed.insert(c.ids[k]);
        continue;
      }
      b->pages.assign(c.pages_h + it.page_base, c.pages_h + it.page_base + it.want);
      b->reserved = (uint64_t)it.want * ps;
      b->length = std::max(b->length, lengths[c.index[k]]);
      d.free_pages -= it.want;
      ++stats_.device_allocs;
      stats_.device_alloc_pages += it.want;
    }
  }
  for (size_t k : redo) {
    const size_t i = c.index[k];
    try {
      write(session, c.ids[k], 0, (uint64_t)(host_base + c.at[k]), lengths[i], (int)MemKind::kHost, 0, true);
    } catch (const StoreError&) {
      status[i] = 3;
      failed.insert(c.ids[k]);
      try { abort_block(session, c.ids[k]); } catch (const StoreError&) {}
    }
  }
  c.ids.clear();
  c.index.clear();
  c.at.clear();
  return failed;
}

}  // namespace amdx
