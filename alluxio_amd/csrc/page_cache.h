// K9: HBM-resident client page cache with a device hash table (LocalCacheManager's page store on
// MI355X).  Reference: core/client/fs/src/main/java/alluxio/client/file/cache/LocalCacheManager.java
// (put :249-347 two-phase evict + put, get :360), store/LocalPageStore.java, evictor/LRUCacheEvictor.java.
//
// Pages live in fixed slots of one device arena.  The key -> slot index is an open-addressing
// table kept twice: an authoritative host mirror (puts, erases, host lookups) and a device copy
// that the fused lookup+gather kernel probes, so a batch of page keys produced ON the GPU (a
// device-side sampler/shuffle) is served by one launch with no host round trip.  Dirty table
// entries are pushed to the device before every gather on the gather's stream.  Recency: host
// gets bump a host stamp, device gathers write stamps[slot] = epoch; eviction folds both.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "kernels.h"
#include "seg_ring.h"

namespace amdx {

class DevicePageCache {
 public:
  // use_device=false keeps the arena and table in host memory (CPU builds and tests): every
  // operation has the same semantics, the gather runs the same probe on the CPU.
  DevicePageCache(int device, uint64_t capacity_bytes, uint64_t page_size, bool use_device);
  ~DevicePageCache();
  DevicePageCache(const DevicePageCache&) = delete;
  DevicePageCache& operator=(const DevicePageCache&) = delete;

  // Store `len` bytes from `src` (MemKind) as page `key`.  When every slot is taken and `evict`
  // is set, least-recently-used pages are dropped first (returned); otherwise full -> throws.
  std::vector<uint64_t> put(uint64_t key, uint64_t src, uint64_t len, int src_kind, uint64_t stream, bool evict);
  // Store keys[i] <- src + i * src_stride (len bytes each; stride 0 repeats one page) with one
  // batched copy launch; evicted keys are returned as for put().  A key repeated in the batch
  // keeps its last source (as sequential put() calls would).  All-or-nothing: with evict=false a
  // batch that does not fit throws before anything changes, and a failed copy rolls back every
  // page of the batch it had staged (those keys read as misses afterwards).
  std::vector<uint64_t> put_many(const std::vector<uint64_t>& keys, uint64_t src, uint64_t src_stride,
                                 uint64_t len, int src_kind, uint64_t stream, bool evict);
  // Device-resident keys (`keys` = n uint64 in device memory): the whole put runs on the GPU
  // (page_cache_put.hip: probe/claim, free-stack or CLOCK eviction, fill) with the device table
  // authoritative; the host mirror is pulled back lazily by the next host-side operation.
  // n must not exceed the slot count.  Same contract as put_many otherwise (last duplicate wins;
  // evict=false and not enough free slots: nothing changes, throws).
  std::vector<uint64_t> put_many_device(uint64_t keys, uint32_t n, uint64_t src, uint64_t src_stride, uint64_t len,
                                        int src_kind, uint64_t stream, bool evict);
  bool erase(uint64_t key);
  bool contains(uint64_t key) const;
  // (slot, len) or (-1, 0); bumps recency.
  std::pair<int32_t, uint32_t> lookup(uint64_t key);
  uint64_t slot_ptr(int32_t slot) const { return arena_ + (uint64_t)slot * page_size_; }
  // Copy `len` bytes at `offset` of page `key` to dst (MemKind); false on a miss.
  bool read(uint64_t key, uint64_t offset, uint64_t len, uint64_t dst, int dst_kind, uint64_t stream);

  // Copy byte ranges of cached pages: segment i copies lens[i] bytes at offsets[i] of page
  // keys[i] to dsts[i] (MemKind dst_kind).  Slots are resolved and the copies launched (one
  // batched launch for device destinations) under the cache lock and tracked like gathers, so no
  // later put/evict can rewrite a slot before its copy ran.  Returns the indices that missed
  // (page absent, or range beyond the page's valid bytes); those destinations are untouched.
  // Device destinations: asynchronous on `stream`.  Host destinations: complete on return.
  std::vector<int32_t> read_segments(const std::vector<uint64_t>& keys, const std::vector<uint64_t>& offsets,
                                     const std::vector<uint64_t>& lens, const std::vector<uint64_t>& dsts,
                                     int dst_kind, uint64_t stream);

  // Fused lookup + gather: keys/slot_out/len_out are device (or, host mode, host) arrays.
  void gather(uint64_t keys, uint32_t n, uint64_t dst, uint64_t dst_stride, uint64_t slot_out,
              uint64_t len_out, uint64_t stream);
  // Host keys: uploaded, gathered, slots returned (-1 = miss).
  std::vector<int32_t> gather_host_keys(const std::vector<uint64_t>& keys, uint64_t dst, uint64_t dst_stride,
                                        uint64_t stream);

  uint64_t page_size() const { return page_size_; }
  uint32_t slots() const { return nslots_; }
  uint32_t used() const { return (uint32_t)(nslots_ - (dev_owner_ ? (uint64_t)dev_free_ : free_.size())); }
  bool device_owned() const { return dev_owner_; }
  uint64_t table_size() const { return table_h_.size(); }
  uint64_t arena() const { return arena_; }
  bool on_device() const { return use_device_; }
  void clear();

 private:
  int64_t find_index(uint64_t key) const;       // table index or -1
  void table_insert(uint64_t key, int32_t slot, uint32_t len);
  void table_erase_at(uint64_t idx);
  void mark_dirty(uint64_t idx);
  void flush_table(hipStream_t stream);         // push dirty entries to the device copy
  void gather_locked(uint64_t keys, uint32_t n, uint64_t dst, uint64_t dst_stride, uint64_t slot_out,
                     uint64_t len_out, hipStream_t stream);
  void track_reader(hipStream_t stream);         // record an event behind a slot reader
  void order_after_readers(hipStream_t stream);  // stream waits for every tracked reader
  void rebuild_table();                          // drop tombstones
  std::vector<uint64_t> evict_lru(uint32_t need);
  void sync_device_stamps();
  void wait_gathers();
  void ensure_host();                            // device table authoritative -> pull it back
  void ensure_device(hipStream_t stream);        // host changed -> push table, slots, free stack
  std::vector<uint64_t> put_device_locked(const uint64_t* keys_d, uint32_t n, uint64_t src, uint64_t src_stride,
                                          uint64_t len, int src_kind, hipStream_t stream, bool evict);
  void reserve_put(uint32_t n);

  int device_;
  bool use_device_;
  uint64_t page_size_;
  uint32_t nslots_;
  uint64_t arena_ = 0;                           // device or host address
  std::vector<PageTableEntry> table_h_;          // host mirror (authoritative)
  PageTableEntry* table_d_ = nullptr;            // device copy
  uint64_t tombstones_ = 0;
  std::vector<uint64_t> dirty_;
  std::vector<uint8_t> dirty_flag_;
  bool full_upload_ = true;
  std::vector<uint32_t> free_;
  std::vector<uint64_t> slot_key_;               // slot -> key (kPageKeyEmpty if free)
  std::vector<uint32_t> stamp_h_;                // host-side recency stamps per slot
  uint32_t* stamps_d_ = nullptr;                 // device-side recency stamps per slot
  uint32_t epoch_ = 1;
  bool device_stamps_dirty_ = false;
  // scratch for uploads (pinned when on the device)
  uint64_t* upd_idx_d_ = nullptr;
  PageTableEntry* upd_ent_d_ = nullptr;
  uint32_t upd_cap_ = 0;
  uint64_t* keys_d_ = nullptr;
  int32_t* slots_d_ = nullptr;
  uint32_t* lens_d_ = nullptr;
  uint32_t keys_cap_ = 0;
  // outstanding slot readers (gathers, segment reads), one event each, any stream
  std::vector<hipEvent_t> pending_ev_;
  std::vector<hipEvent_t> ev_pool_;
  // device put path state (page_cache_put.hip)
  bool dev_owner_ = false;                       // the device table is ahead of the host mirror
  bool host_changed_ = true;                     // host mirror changed since the last push
  int32_t dev_free_ = 0;                         // free slots while dev_owner_
  unsigned long long batch_ = 0;
  uint64_t* slot_key_d_ = nullptr;
  uint32_t* slot_tidx_d_ = nullptr;
  uint32_t* free_stack_d_ = nullptr;
  uint32_t* hist_d_ = nullptr;                   // [kPutAgeBuckets] eviction-threshold histogram
  PageTableEntry* table2_d_ = nullptr;           // device rebuild target (swapped with table_d_)
  unsigned long long* tag_d_ = nullptr;
  PutCounters* ctr_d_ = nullptr;
  PutCounters* ctr_h_ = nullptr;                 // pinned
  uint32_t* put_tidx_d_ = nullptr;
  int32_t* put_slot_d_ = nullptr;
  uint64_t* put_ev_d_ = nullptr;
  uint32_t put_cap_ = 0;
  SegRing ring_;                                 // descriptors of batched copies
  mutable std::mutex mu_;
};

}  // namespace amdx
