// HBM client page cache with a device hash table (see page_cache.h).
#include "page_cache.h"

#include <algorithm>
#include <cstring>
#include <unordered_map>

#include "block_store.h"   // StoreError, MemKind, error codes

namespace amdx {

#define PC_HIP_OK(expr)                                                                       \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess)                                                                     \
      throw StoreError(kErrHip, std::string("HIP error: ") + hipGetErrorString(_e) + " at " + #expr); \
  } while (0)

static uint64_t next_pow2(uint64_t x) {
  uint64_t p = 64;
  while (p < x) p <<= 1;
  return p;
}

DevicePageCache::DevicePageCache(int device, uint64_t capacity_bytes, uint64_t page_size, bool use_device)
    : device_(device), use_device_(use_device), page_size_(page_size) {
  if (page_size == 0 || page_size % 16 != 0)
    throw StoreError(kErrInvalidArgument, "page size must be a positive multiple of 16");
  const uint64_t n = capacity_bytes / page_size;
  if (n == 0 || n > (1u << 30)) throw StoreError(kErrInvalidArgument, "cache must hold 1..2^30 pages");
  nslots_ = (uint32_t)n;
  // 4x the slots: a device put of a whole cache's worth of fresh keys claims its entries while the
  // pages it replaces still hold theirs, and the load must stay <= 1/2 through that batch
  table_h_.assign(next_pow2(4 * n), PageTableEntry{kPageKeyEmpty, -1, 0});
  dirty_flag_.assign(table_h_.size(), 0);
  slot_key_.assign(nslots_, kPageKeyEmpty);
  stamp_h_.assign(nslots_, 0);
  free_.reserve(nslots_);
  for (uint32_t s = nslots_; s-- > 0;) free_.push_back(s);
  if (use_device_) {
    PC_HIP_OK(hipSetDevice(device_));
    void* p = nullptr;
    PC_HIP_OK(hipMalloc(&p, nslots_ * page_size_));
    arena_ = (uint64_t)p;
    PC_HIP_OK(hipMalloc((void**)&table_d_, table_h_.size() * sizeof(PageTableEntry)));
    PC_HIP_OK(hipMalloc((void**)&stamps_d_, nslots_ * sizeof(uint32_t)));
    PC_HIP_OK(hipMemset(stamps_d_, 0, nslots_ * sizeof(uint32_t)));
    PC_HIP_OK(hipMalloc((void**)&slot_key_d_, nslots_ * sizeof(uint64_t)));
    PC_HIP_OK(hipMalloc((void**)&slot_tidx_d_, nslots_ * sizeof(uint32_t)));
    PC_HIP_OK(hipMalloc((void**)&free_stack_d_, nslots_ * sizeof(uint32_t)));
    PC_HIP_OK(hipMalloc((void**)&hist_d_, kPutAgeBuckets * sizeof(uint32_t)));
    PC_HIP_OK(hipMalloc((void**)&table2_d_, table_h_.size() * sizeof(PageTableEntry)));
    PC_HIP_OK(hipMalloc((void**)&tag_d_, table_h_.size() * sizeof(unsigned long long)));
    PC_HIP_OK(hipMemset(tag_d_, 0, table_h_.size() * sizeof(unsigned long long)));
    PC_HIP_OK(hipMalloc((void**)&ctr_d_, sizeof(PutCounters)));
    PC_HIP_OK(hipMemset(ctr_d_, 0, sizeof(PutCounters)));
    PC_HIP_OK(hipHostMalloc((void**)&ctr_h_, sizeof(PutCounters), hipHostMallocDefault));
    ring_.init();
  } else {
    void* p = std::aligned_alloc(64, ((nslots_ * page_size_ + 63) / 64) * 64);
    if (!p) throw StoreError(kErrOutOfSpace, "host page cache arena allocation failed");
    arena_ = (uint64_t)p;
  }
  full_upload_ = true;
}

DevicePageCache::~DevicePageCache() {
  if (use_device_) {
    hipSetDevice(device_);
    for (hipEvent_t e : pending_ev_) {
      hipEventSynchronize(e);
      hipEventDestroy(e);
    }
    for (hipEvent_t e : ev_pool_) hipEventDestroy(e);
    ring_.release();
    hipFree((void*)arena_);
    hipFree(table_d_);
    hipFree(stamps_d_);
    hipFree(upd_idx_d_);
    hipFree(upd_ent_d_);
    hipFree(keys_d_);
    hipFree(slots_d_);
    hipFree(lens_d_);
    hipFree(slot_key_d_);
    hipFree(slot_tidx_d_);
    hipFree(free_stack_d_);
    hipFree(hist_d_);
    hipFree(table2_d_);
    hipFree(tag_d_);
    hipFree(ctr_d_);
    hipHostFree(ctr_h_);
    hipFree(put_tidx_d_);
    hipFree(put_slot_d_);
    hipFree(put_ev_d_);
  } else {
    std::free((void*)arena_);
  }
}

// ---- host mirror -----------------------------------------------------------------------------
int64_t DevicePageCache::find_index(uint64_t key) const {
  const uint64_t mask = table_h_.size() - 1;
  uint64_t i = page_key_hash(key) & mask;
  for (uint64_t probe = 0; probe <= mask; ++probe, i = (i + 1) & mask) {
    const uint64_t k = table_h_[i].key;
    if (k == key) return (int64_t)i;
    if (k == kPageKeyEmpty) return -1;
  }
  return -1;
}

void DevicePageCache::mark_dirty(uint64_t idx) {
  if (!use_device_ || full_upload_) return;
  if (!dirty_flag_[idx]) {
    dirty_flag_[idx] = 1;
    dirty_.push_back(idx);
    if (dirty_.size() > table_h_.size() / 8) full_upload_ = true;   // cheaper as one copy
  }
}

void DevicePageCache::table_insert(uint64_t key, int32_t slot, uint32_t len) {
  host_changed_ = true;
  const uint64_t mask = table_h_.size() - 1;
  uint64_t i = page_key_hash(key) & mask;
  int64_t tomb = -1;
  for (uint64_t probe = 0; probe <= mask; ++probe, i = (i + 1) & mask) {
    const uint64_t k = table_h_[i].key;
    if (k == key) {                   // overwrite in place
      table_h_[i].slot = slot;
      table_h_[i].len = len;
      mark_dirty(i);
      return;
    }
    if (k == kPageKeyTomb && tomb < 0) tomb = (int64_t)i;
    if (k == kPageKeyEmpty) break;
  }
  const uint64_t at = tomb >= 0 ? (uint64_t)tomb : i;
  if (tomb >= 0) --tombstones_;
  table_h_[at] = PageTableEntry{key, slot, len};
  mark_dirty(at);
}

void DevicePageCache::table_erase_at(uint64_t idx) {
  host_changed_ = true;
  table_h_[idx] = PageTableEntry{kPageKeyTomb, -1, 0};
  ++tombstones_;
  mark_dirty(idx);
  if (tombstones_ > table_h_.size() / 4) rebuild_table();
}

void DevicePageCache::rebuild_table() {
  std::vector<PageTableEntry> old;
  old.swap(table_h_);
  table_h_.assign(old.size(), PageTableEntry{kPageKeyEmpty, -1, 0});
  tombstones_ = 0;
  const bool saved = full_upload_;
  full_upload_ = true;               // everything moves: one full upload
  for (const auto& e : old)
    if (e.key != kPageKeyEmpty && e.key != kPageKeyTomb) table_insert(e.key, e.slot, e.len);
  (void)saved;
  dirty_.clear();
  std::fill(dirty_flag_.begin(), dirty_flag_.end(), 0);
}

void DevicePageCache::flush_table(hipStream_t stream) {
  if (!use_device_) return;
  if (!full_upload_ && dirty_.empty()) return;
  // a gather queued on another stream may still be probing the entries about to change
  order_after_readers(stream);
  if (full_upload_) {
    PC_HIP_OK(hipMemcpyAsync(table_d_, table_h_.data(), table_h_.size() * sizeof(PageTableEntry),
                             hipMemcpyHostToDevice, stream));
    PC_HIP_OK(hipStreamSynchronize(stream));   // the host mirror may change right after
    full_upload_ = false;
    for (uint64_t i : dirty_) dirty_flag_[i] = 0;
    dirty_.clear();
    return;
  }
  if (dirty_.empty()) return;
  const uint32_t n = (uint32_t)dirty_.size();
  if (n > upd_cap_) {
    hipFree(upd_idx_d_);
    hipFree(upd_ent_d_);
    upd_cap_ = std::max<uint32_t>(n, 1024);
    PC_HIP_OK(hipMalloc((void**)&upd_idx_d_, upd_cap_ * sizeof(uint64_t)));
    PC_HIP_OK(hipMalloc((void**)&upd_ent_d_, upd_cap_ * sizeof(PageTableEntry)));
  }
  std::vector<PageTableEntry> ents(n);
  for (uint32_t i = 0; i < n; ++i) {
    ents[i] = table_h_[dirty_[i]];
    dirty_flag_[dirty_[i]] = 0;
  }
  PC_HIP_OK(hipMemcpyAsync(upd_idx_d_, dirty_.data(), n * sizeof(uint64_t), hipMemcpyHostToDevice, stream));
  PC_HIP_OK(hipMemcpyAsync(upd_ent_d_, ents.data(), n * sizeof(PageTableEntry), hipMemcpyHostToDevice, stream));
  PC_HIP_OK(launch_page_table_update(table_d_, upd_idx_d_, upd_ent_d_, n, stream));
  PC_HIP_OK(hipStreamSynchronize(stream));     // pageable sources: keep them alive until copied
  dirty_.clear();
}

// ---- recency / eviction ---------------------------------------------------------------------
void DevicePageCache::sync_device_stamps() {
  if (!use_device_ || !device_stamps_dirty_) return;
  std::vector<uint32_t> dev(nslots_);
  wait_gathers();
  PC_HIP_OK(hipMemcpy(dev.data(), stamps_d_, nslots_ * sizeof(uint32_t), hipMemcpyDeviceToHost));
  for (uint32_t s = 0; s < nslots_; ++s) stamp_h_[s] = std::max(stamp_h_[s], dev[s]);
  device_stamps_dirty_ = false;
}

std::vector<uint64_t> DevicePageCache::evict_lru(uint32_t need) {
  sync_device_stamps();
  std::vector<uint32_t> used;
  used.reserve(nslots_ - free_.size());
  for (uint32_t s = 0; s < nslots_; ++s)
    if (slot_key_[s] != kPageKeyEmpty) used.push_back(s);
  need = std::min<uint32_t>(need, (uint32_t)used.size());
  std::nth_element(used.begin(), used.begin() + need, used.end(),
                   [&](uint32_t a, uint32_t b) { return stamp_h_[a] < stamp_h_[b]; });
  std::vector<uint64_t> out;
  for (uint32_t i = 0; i < need; ++i) {
    const uint32_t s = used[i];
    const uint64_t k = slot_key_[s];
    const int64_t idx = find_index(k);
    if (idx >= 0) table_erase_at((uint64_t)idx);
    slot_key_[s] = kPageKeyEmpty;
    free_.push_back(s);
    out.push_back(k);
  }
  return out;
}

void DevicePageCache::wait_gathers() {
  if (!use_device_) return;
  hipError_t first = hipSuccess;
  for (hipEvent_t ev : pending_ev_) {
    const hipError_t e = hipEventSynchronize(ev);
    if (e != hipSuccess && first == hipSuccess) first = e;
    ev_pool_.push_back(ev);
  }
  pending_ev_.clear();
  PC_HIP_OK(first);
}

void DevicePageCache::track_reader(hipStream_t stream) {
  // completed events are recycled first so the pending list stays short under steady traffic
  size_t w = 0;
  for (size_t i = 0; i < pending_ev_.size(); ++i) {
    if (hipEventQuery(pending_ev_[i]) == hipSuccess) ev_pool_.push_back(pending_ev_[i]);
    else pending_ev_[w++] = pending_ev_[i];
  }
  pending_ev_.resize(w);
  hipEvent_t ev;
  if (!ev_pool_.empty()) {
    ev = ev_pool_.back();
    ev_pool_.pop_back();
  } else {
    PC_HIP_OK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  }
  const hipError_t e = hipEventRecord(ev, stream);
  if (e != hipSuccess) {
    ev_pool_.push_back(ev);
    PC_HIP_OK(e);
  }
  pending_ev_.push_back(ev);
}

void DevicePageCache::order_after_readers(hipStream_t stream) {
  for (hipEvent_t ev : pending_ev_) PC_HIP_OK(hipStreamWaitEvent(stream, ev, 0));
}

// ---- public API -------------------------------------------------------------------------------
std::vector<uint64_t> DevicePageCache::put(uint64_t key, uint64_t src, uint64_t len, int src_kind, uint64_t stream,
                                           bool evict) {
  if (key == kPageKeyEmpty || key == kPageKeyTomb) throw StoreError(kErrInvalidArgument, "reserved page key");
  if (len > page_size_) throw StoreError(kErrInvalidArgument, "page larger than the page size");
  std::lock_guard<std::mutex> g(mu_);
  ensure_host();
  std::vector<uint64_t> evicted;
  int32_t slot;
  const int64_t idx = find_index(key);
  if (idx >= 0) {
    slot = table_h_[idx].slot;
  } else {
    if (free_.empty()) {
      if (!evict) throw StoreError(kErrOutOfSpace, "page cache is full");
      evicted = evict_lru(std::max<uint32_t>(1, nslots_ / 64));   // evict in batches
    }
    slot = (int32_t)free_.back();
    free_.pop_back();
  }
  // a queued gather may still read this slot's previous page (overwritten, evicted or erased
  // and reused): let queued gathers finish before the slot is rewritten
  wait_gathers();
  const uint64_t dst = arena_ + (uint64_t)slot * page_size_;
  if (len) {
    if (use_device_) {
      const hipMemcpyKind kind = src_kind == (int)MemKind::kDevice ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
      PC_HIP_OK(hipMemcpyAsync((void*)dst, (const void*)src, len, kind, (hipStream_t)stream));
      PC_HIP_OK(hipStreamSynchronize((hipStream_t)stream));
    } else {
      std::memcpy((void*)dst, (const void*)src, len);
    }
  }
  slot_key_[slot] = key;
  stamp_h_[slot] = ++epoch_;
  table_insert(key, slot, (uint32_t)len);
  return evicted;
}

// Batched fill: the table work runs on the host for the whole batch and the page bytes move in
// one batched_copy_kernel launch (device sources) instead of one hipMemcpy + sync per page.
// Slot assignments are staged and committed to the table only after their copy succeeded; copies
// are flushed (and committed) before any eviction, so a slot reused later in the batch is written
// by a later launch on the same stream.
std::vector<uint64_t> DevicePageCache::put_many(const std::vector<uint64_t>& keys_in, uint64_t src,
                                                uint64_t src_stride, uint64_t len, int src_kind,
                                                uint64_t stream, bool evict) {
  if (len > page_size_) throw StoreError(kErrInvalidArgument, "page larger than the page size");
  for (uint64_t k : keys_in)
    if (k == kPageKeyEmpty || k == kPageKeyTomb) throw StoreError(kErrInvalidArgument, "reserved page key");
  // de-duplicate: the last occurrence of a key wins (its source index is kept)
  std::vector<std::pair<uint64_t, size_t>> batch;   // (key, source index)
  batch.reserve(keys_in.size());
  {
    std::unordered_map<uint64_t, size_t> last;
    last.reserve(keys_in.size() * 2);
    for (size_t i = 0; i < keys_in.size(); ++i) last[keys_in[i]] = i;
    for (size_t i = 0; i < keys_in.size(); ++i)
      if (last[keys_in[i]] == i) batch.emplace_back(keys_in[i], i);
  }
  std::lock_guard<std::mutex> g(mu_);
  if (use_device_ && src_kind == (int)MemKind::kDevice && !keys_in.empty() && keys_in.size() <= nslots_) {
    // the device put path: upload the keys, resolve + evict + fill on the GPU (device sources
    // only: the fill kernel must never dereference pageable host memory)
    hipStream_t s = (hipStream_t)stream;
    const uint32_t n = (uint32_t)keys_in.size();
    if (n > keys_cap_) {
      wait_gathers();
      hipFree(keys_d_);
      hipFree(slots_d_);
      hipFree(lens_d_);
      keys_d_ = nullptr;
      slots_d_ = nullptr;
      lens_d_ = nullptr;
      keys_cap_ = 0;
      const uint32_t cap = std::max<uint32_t>(n, 4096);
      PC_HIP_OK(hipMalloc((void**)&keys_d_, cap * sizeof(uint64_t)));
      PC_HIP_OK(hipMalloc((void**)&slots_d_, cap * sizeof(int32_t)));
      PC_HIP_OK(hipMalloc((void**)&lens_d_, cap * sizeof(uint32_t)));
      keys_cap_ = cap;
    }
    order_after_readers(s);
    PC_HIP_OK(hipMemcpyAsync(keys_d_, keys_in.data(), n * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    return put_device_locked(keys_d_, n, src, src_stride, len, src_kind, s, evict);
  }
  ensure_host();
  if (!evict) {
    size_t fresh = 0;
    for (const auto& kv : batch) fresh += find_index(kv.first) < 0;
    if (fresh > free_.size()) throw StoreError(kErrOutOfSpace, "page cache is full");
  }
  wait_gathers();
  hipStream_t st = (hipStream_t)stream;
  std::vector<uint64_t> evicted;
  std::vector<CopySeg> segs;
  struct Staged { uint64_t key; int32_t slot; bool fresh; };
  std::vector<Staged> staged;
  auto rollback = [&]() {
    // staged pages hold undefined bytes: new slots go back to the free list, overwritten pages
    // are dropped from the table (a miss, never stale data)
    for (const auto& sp : staged) {
      if (sp.fresh) {
        free_.push_back((uint32_t)sp.slot);
      } else {
        const int64_t idx = find_index(sp.key);
        if (idx >= 0) table_erase_at((uint64_t)idx);
        slot_key_[sp.slot] = kPageKeyEmpty;
        free_.push_back((uint32_t)sp.slot);
      }
    }
    staged.clear();
    segs.clear();
  };
  auto flush = [&]() {
    if (!segs.empty()) {
      try {
        if (!use_device_) {
          for (const auto& sg : segs) std::memcpy((void*)sg.dst, (const void*)sg.src, sg.bytes);
        } else if (src_kind == (int)MemKind::kDevice) {
          PC_HIP_OK(ring_.launch(segs, st));
          PC_HIP_OK(hipStreamSynchronize(st));
        } else {
          for (const auto& sg : segs)
            PC_HIP_OK(hipMemcpyAsync((void*)sg.dst, (const void*)sg.src, sg.bytes, hipMemcpyHostToDevice, st));
          PC_HIP_OK(hipStreamSynchronize(st));
        }
      } catch (...) {
        rollback();
        throw;
      }
    }
    for (const auto& sp : staged) {
      const uint64_t bytes = len;
      slot_key_[sp.slot] = sp.key;
      stamp_h_[sp.slot] = ++epoch_;
      table_insert(sp.key, sp.slot, (uint32_t)bytes);
    }
    staged.clear();
    segs.clear();
  };
  for (const auto& kv : batch) {
    const uint64_t key = kv.first;
    int32_t slot;
    bool fresh = false;
    const int64_t idx = find_index(key);
    if (idx >= 0) {
      slot = table_h_[idx].slot;
    } else {
      if (free_.empty()) {
        flush();
        const auto ev = evict_lru(std::max<uint32_t>(1, nslots_ / 64));
        evicted.insert(evicted.end(), ev.begin(), ev.end());
        if (free_.empty()) throw StoreError(kErrOutOfSpace, "page cache is full");
      }
      slot = (int32_t)free_.back();
      free_.pop_back();
      fresh = true;
    }
    staged.push_back(Staged{key, slot, fresh});
    if (len) segs.push_back(CopySeg{src + kv.second * src_stride, arena_ + (uint64_t)slot * page_size_, len, 0});
  }
  flush();
  return evicted;
}

bool DevicePageCache::erase(uint64_t key) {
  std::lock_guard<std::mutex> g(mu_);
  ensure_host();
  const int64_t idx = find_index(key);
  if (idx < 0) return false;
  const int32_t slot = table_h_[idx].slot;
  table_erase_at((uint64_t)idx);
  slot_key_[slot] = kPageKeyEmpty;
  free_.push_back((uint32_t)slot);
  return true;
}

bool DevicePageCache::contains(uint64_t key) const {
  std::lock_guard<std::mutex> g(mu_);
  const_cast<DevicePageCache*>(this)->ensure_host();
  return find_index(key) >= 0;
}

std::pair<int32_t, uint32_t> DevicePageCache::lookup(uint64_t key) {
  std::lock_guard<std::mutex> g(mu_);
  ensure_host();
  const int64_t idx = find_index(key);
  if (idx < 0) return {-1, 0};
  const auto& e = table_h_[idx];
  stamp_h_[e.slot] = ++epoch_;
  return {e.slot, e.len};
}

bool DevicePageCache::read(uint64_t key, uint64_t offset, uint64_t len, uint64_t dst, int dst_kind,
                           uint64_t stream) {
  std::lock_guard<std::mutex> g(mu_);
  ensure_host();
  const int64_t idx = find_index(key);
  if (idx < 0) return false;
  const auto& e = table_h_[idx];
  if (offset + len > e.len) throw StoreError(kErrInvalidArgument, "read past the end of the page");
  stamp_h_[e.slot] = ++epoch_;
  const uint64_t src = arena_ + (uint64_t)e.slot * page_size_ + offset;
  if (len == 0) return true;
  if (use_device_) {
    const hipMemcpyKind kind = dst_kind == (int)MemKind::kDevice ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    PC_HIP_OK(hipMemcpyAsync((void*)dst, (const void*)src, len, kind, (hipStream_t)stream));
    PC_HIP_OK(hipStreamSynchronize((hipStream_t)stream));
  } else {
    std::memcpy((void*)dst, (const void*)src, len);
  }
  return true;
}

std::vector<int32_t> DevicePageCache::read_segments(const std::vector<uint64_t>& keys,
                                                    const std::vector<uint64_t>& offsets,
                                                    const std::vector<uint64_t>& lens,
                                                    const std::vector<uint64_t>& dsts, int dst_kind,
                                                    uint64_t stream) {
  const size_t n = keys.size();
  if (offsets.size() != n || lens.size() != n || dsts.size() != n)
    throw StoreError(kErrInvalidArgument, "read_segments: keys/offsets/lens/dsts differ in length");
  std::vector<int32_t> missed;
  std::vector<CopySeg> segs;
  segs.reserve(n);
  hipStream_t st = (hipStream_t)stream;
  std::lock_guard<std::mutex> g(mu_);
  ensure_host();
  const uint32_t epoch = ++epoch_;
  for (size_t i = 0; i < n; ++i) {
    const int64_t idx = find_index(keys[i]);
    if (idx < 0 || offsets[i] + lens[i] > table_h_[idx].len) {
      missed.push_back((int32_t)i);
      continue;
    }
    const auto& e = table_h_[idx];
    stamp_h_[e.slot] = epoch;
    if (lens[i]) segs.push_back(CopySeg{arena_ + (uint64_t)e.slot * page_size_ + offsets[i], dsts[i], lens[i], 0});
  }
  if (segs.empty()) return missed;
  if (!use_device_) {
    for (const auto& sg : segs) std::memcpy((void*)sg.dst, (const void*)sg.src, sg.bytes);
    return missed;
  }
  if (dst_kind == (int)MemKind::kDevice) {
    PC_HIP_OK(ring_.launch(segs, st));
    track_reader(st);
  } else {
    for (const auto& sg : segs)
      PC_HIP_OK(hipMemcpyAsync((void*)sg.dst, (const void*)sg.src, sg.bytes, hipMemcpyDeviceToHost, st));
    PC_HIP_OK(hipStreamSynchronize(st));
  }
  return missed;
}

void DevicePageCache::gather(uint64_t keys, uint32_t n, uint64_t dst, uint64_t dst_stride, uint64_t slot_out,
                             uint64_t len_out, uint64_t stream) {
  if (n == 0) return;
  if (dst_stride < page_size_ && n > 1) throw StoreError(kErrInvalidArgument, "dst stride below the page size");
  std::lock_guard<std::mutex> g(mu_);
  gather_locked(keys, n, dst, dst_stride, slot_out, len_out, (hipStream_t)stream);
}

void DevicePageCache::gather_locked(uint64_t keys, uint32_t n, uint64_t dst, uint64_t dst_stride,
                                    uint64_t slot_out, uint64_t len_out, hipStream_t s) {
  const uint32_t epoch = ++epoch_;
  if (!use_device_) {
    const uint64_t* k = (const uint64_t*)keys;
    int32_t* so = (int32_t*)slot_out;
    uint32_t* lo = (uint32_t*)len_out;
    for (uint32_t i = 0; i < n; ++i) {
      const int64_t idx = find_index(k[i]);
      if (idx < 0) {
        so[i] = -1;
        lo[i] = 0;
        continue;
      }
      const auto& e = table_h_[idx];
      so[i] = e.slot;
      lo[i] = e.len;
      stamp_h_[e.slot] = epoch;
      std::memcpy((void*)(dst + (uint64_t)i * dst_stride), (const void*)(arena_ + (uint64_t)e.slot * page_size_), e.len);
    }
    return;
  }
  flush_table(s);
  PageGatherArgs a{table_d_, table_h_.size() - 1, (const uint64_t*)keys, n, (const uint8_t*)arena_, page_size_,
                   (uint8_t*)dst, dst_stride, (int32_t*)slot_out, (uint32_t*)len_out, stamps_d_, epoch};
  PC_HIP_OK(launch_page_lookup_gather(a, s));
  track_reader(s);
  device_stamps_dirty_ = true;
}

std::vector<int32_t> DevicePageCache::gather_host_keys(const std::vector<uint64_t>& keys, uint64_t dst,
                                                       uint64_t dst_stride, uint64_t stream) {
  const uint32_t n = (uint32_t)keys.size();
  std::vector<int32_t> slots(n, -1);
  if (n == 0) return slots;
  if (dst_stride < page_size_ && n > 1) throw StoreError(kErrInvalidArgument, "dst stride below the page size");
  if (!use_device_) {
    std::vector<uint32_t> lens(n);
    gather((uint64_t)keys.data(), n, dst, dst_stride, (uint64_t)slots.data(), (uint64_t)lens.data(), stream);
    return slots;
  }
  hipStream_t s = (hipStream_t)stream;
  // the scratch buffers are shared: upload, gather and read-back all happen under the lock
  std::lock_guard<std::mutex> g(mu_);
  if (n > keys_cap_) {
    wait_gathers();
    hipFree(keys_d_);
    hipFree(slots_d_);
    hipFree(lens_d_);
    keys_d_ = nullptr;
    slots_d_ = nullptr;
    lens_d_ = nullptr;
    keys_cap_ = 0;
    const uint32_t cap = std::max<uint32_t>(n, 4096);
    PC_HIP_OK(hipMalloc((void**)&keys_d_, cap * sizeof(uint64_t)));
    PC_HIP_OK(hipMalloc((void**)&slots_d_, cap * sizeof(int32_t)));
    PC_HIP_OK(hipMalloc((void**)&lens_d_, cap * sizeof(uint32_t)));
    keys_cap_ = cap;
  }
  // an earlier call's gather (another stream) may still read keys_d_
  order_after_readers(s);
  PC_HIP_OK(hipMemcpyAsync(keys_d_, keys.data(), n * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  gather_locked((uint64_t)keys_d_, n, dst, dst_stride, (uint64_t)slots_d_, (uint64_t)lens_d_, s);
  PC_HIP_OK(hipMemcpyAsync(slots.data(), slots_d_, n * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  PC_HIP_OK(hipStreamSynchronize(s));
  return slots;
}

// ---- device put path (page_cache_put.hip) ------------------------------------------------------
void DevicePageCache::reserve_put(uint32_t n) {
  if (n <= put_cap_) return;
  wait_gathers();
  hipFree(put_tidx_d_);
  hipFree(put_slot_d_);
  hipFree(put_ev_d_);
  put_tidx_d_ = nullptr;
  put_slot_d_ = nullptr;
  put_ev_d_ = nullptr;
  put_cap_ = 0;
  const uint32_t cap = std::max<uint32_t>(n, 4096);
  PC_HIP_OK(hipMalloc((void**)&put_tidx_d_, cap * sizeof(uint32_t)));
  PC_HIP_OK(hipMalloc((void**)&put_slot_d_, cap * sizeof(int32_t)));
  PC_HIP_OK(hipMalloc((void**)&put_ev_d_, cap * sizeof(uint64_t)));
  put_cap_ = cap;
}

void DevicePageCache::ensure_device(hipStream_t stream) {
  if (!host_changed_ && !full_upload_ && dirty_.empty()) return;
  sync_device_stamps();                          // gathers' recency first, then push the merge
  flush_table(stream);                           // table entries (dirty or full)
  std::vector<uint32_t> tidx(nslots_, 0);
  for (uint64_t i = 0; i < table_h_.size(); ++i) {
    const auto& e = table_h_[i];
    if (e.key != kPageKeyEmpty && e.key != kPageKeyTomb && e.slot >= 0) tidx[e.slot] = (uint32_t)i;
  }
  PC_HIP_OK(hipMemcpyAsync(slot_key_d_, slot_key_.data(), nslots_ * sizeof(uint64_t), hipMemcpyHostToDevice, stream));
  PC_HIP_OK(hipMemcpyAsync(slot_tidx_d_, tidx.data(), nslots_ * sizeof(uint32_t), hipMemcpyHostToDevice, stream));
  if (!free_.empty())
    PC_HIP_OK(hipMemcpyAsync(free_stack_d_, free_.data(), free_.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                             stream));
  PC_HIP_OK(hipMemcpyAsync(stamps_d_, stamp_h_.data(), nslots_ * sizeof(uint32_t), hipMemcpyHostToDevice, stream));
  ctr_h_->free_top = (int32_t)free_.size();
  PC_HIP_OK(hipMemcpyAsync(&ctr_d_->free_top, &ctr_h_->free_top, sizeof(int32_t), hipMemcpyHostToDevice, stream));
  PC_HIP_OK(hipStreamSynchronize(stream));       // pageable sources
  host_changed_ = false;
}

void DevicePageCache::ensure_host() {
  if (!dev_owner_) return;
  wait_gathers();                                // device puts already completed on their stream
  PC_HIP_OK(hipMemcpy(table_h_.data(), table_d_, table_h_.size() * sizeof(PageTableEntry), hipMemcpyDeviceToHost));
  PC_HIP_OK(hipMemcpy(slot_key_.data(), slot_key_d_, nslots_ * sizeof(uint64_t), hipMemcpyDeviceToHost));
  PC_HIP_OK(hipMemcpy(ctr_h_, ctr_d_, sizeof(PutCounters), hipMemcpyDeviceToHost));
  const int32_t top = std::max<int32_t>(0, ctr_h_->free_top);
  free_.assign(top, 0);
  if (top) PC_HIP_OK(hipMemcpy(free_.data(), free_stack_d_, top * sizeof(uint32_t), hipMemcpyDeviceToHost));
  tombstones_ = 0;
  for (const auto& e : table_h_) tombstones_ += e.key == kPageKeyTomb;
  for (uint64_t i : dirty_) dirty_flag_[i] = 0;
  dirty_.clear();
  full_upload_ = false;                          // the device copy equals what was just pulled
  dev_owner_ = false;
  device_stamps_dirty_ = true;
  sync_device_stamps();
  host_changed_ = false;
}

std::vector<uint64_t> DevicePageCache::put_many_device(uint64_t keys, uint32_t n, uint64_t src, uint64_t src_stride,
                                                       uint64_t len, int src_kind, uint64_t stream, bool evict) {
  if (!use_device_) throw StoreError(kErrInvalidArgument, "put_many_device needs a device cache");
  if (len > page_size_) throw StoreError(kErrInvalidArgument, "page larger than the page size");
  if (n == 0) return {};
  std::lock_guard<std::mutex> g(mu_);
  return put_device_locked((const uint64_t*)keys, n, src, src_stride, len, src_kind, (hipStream_t)stream, evict);
}

std::vector<uint64_t> DevicePageCache::put_device_locked(const uint64_t* keys_d, uint32_t n, uint64_t src,
                                                         uint64_t src_stride, uint64_t len, int src_kind,
                                                         hipStream_t s, bool evict) {
  if (n > nslots_) throw StoreError(kErrInvalidArgument, "device put batch larger than the cache");
  if (src_kind != (int)MemKind::kDevice)
    throw StoreError(kErrInvalidArgument, "device put path needs a device source (host sources: put_many)");
  reserve_put(n);
  ensure_device(s);
  // slots about to be rewritten may still be read by a queued gather on another stream
  order_after_readers(s);
  PutCounters* c = ctr_h_;
  PagePutArgs a{};
  a.table = table_d_;
  a.mask = table_h_.size() - 1;
  a.keys = keys_d;
  a.n = n;
  a.tidx = put_tidx_d_;
  a.tag = tag_d_;
  a.batch = ++batch_;
  a.stamps = stamps_d_;
  a.hist = hist_d_;
  a.epoch = ++epoch_;
  a.nslots = nslots_;
  a.slot_key = slot_key_d_;
  a.slot_tidx = slot_tidx_d_;
  a.free_stack = free_stack_d_;
  a.ctr = ctr_d_;
  a.evicted = put_ev_d_;
  a.slot_of = put_slot_d_;
  a.evict = evict ? 1 : 0;
  a.len = (uint32_t)len;
  a.src = (const uint8_t*)src;
  a.src_stride = src_stride;
  a.arena = (uint8_t*)arena_;
  a.page_size = page_size_;
  // nfresh .. nfail start at 0 (free_top and the CLOCK hand carry over)
  PC_HIP_OK(hipMemsetAsync(&ctr_d_->nfresh, 0, 4 * sizeof(uint32_t), s));
  PC_HIP_OK(launch_page_put_probe(a, s));
  dev_owner_ = true;                             // the device table changed from here on
  if (!evict) {
    PC_HIP_OK(hipMemcpyAsync(c, ctr_d_, sizeof(PutCounters), hipMemcpyDeviceToHost, s));
    PC_HIP_OK(hipStreamSynchronize(s));
    if (c->nfail || (int64_t)c->nfresh > (int64_t)std::max<int32_t>(0, c->free_top)) {
      PC_HIP_OK(launch_page_put_revert(a, s));
      PC_HIP_OK(hipMemcpyAsync(c, ctr_d_, sizeof(PutCounters), hipMemcpyDeviceToHost, s));
      PC_HIP_OK(hipStreamSynchronize(s));
      dev_free_ = std::max<int32_t>(0, c->free_top);
      tombstones_ += c->ntomb;
      throw StoreError(kErrOutOfSpace, "page cache is full");
    }
  }
  if (evict) PC_HIP_OK(launch_page_put_threshold(a, s));
  PC_HIP_OK(launch_page_put_assign(a, s));
  PC_HIP_OK(launch_page_put_fill(a, s));
  // tombstones piling up: rebuild the table on the device, in the same stream order
  const bool rebuild = tombstones_ + n > table_h_.size() / 8;
  if (rebuild) {
    PC_HIP_OK(launch_page_table_rebuild(a, table2_d_, s));
    std::swap(table_d_, table2_d_);
  }
  PC_HIP_OK(hipMemcpyAsync(c, ctr_d_, sizeof(PutCounters), hipMemcpyDeviceToHost, s));
  PC_HIP_OK(hipStreamSynchronize(s));
  std::vector<uint64_t> evicted(std::min<uint32_t>(c->nevicted, n));
  if (!evicted.empty())
    PC_HIP_OK(hipMemcpy(evicted.data(), put_ev_d_, evicted.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
  if (c->free_top < 0) {
    c->free_top = 0;
    PC_HIP_OK(hipMemcpyAsync(&ctr_d_->free_top, &c->free_top, sizeof(int32_t), hipMemcpyHostToDevice, s));
    PC_HIP_OK(hipStreamSynchronize(s));
  }
  dev_free_ = c->free_top;
  tombstones_ = rebuild ? 0 : tombstones_ + c->ntomb;
  device_stamps_dirty_ = true;
  const uint32_t failed = c->nfail;
  if (failed) throw StoreError(kErrOutOfSpace, "page cache could not place " + std::to_string(failed) + " pages");
  return evicted;
}

void DevicePageCache::clear() {
  std::lock_guard<std::mutex> g(mu_);
  wait_gathers();
  dev_owner_ = false;
  host_changed_ = true;
  std::fill(table_h_.begin(), table_h_.end(), PageTableEntry{kPageKeyEmpty, -1, 0});
  tombstones_ = 0;
  std::fill(slot_key_.begin(), slot_key_.end(), kPageKeyEmpty);
  free_.clear();
  for (uint32_t s = nslots_; s-- > 0;) free_.push_back(s);
  dirty_.clear();
  std::fill(dirty_flag_.begin(), dirty_flag_.end(), 0);
  full_upload_ = true;
}

}  // namespace amdx
