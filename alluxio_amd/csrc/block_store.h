// Native tiered block store for one worker (= one MI355X).
//
// Re-designs the reference TieredBlockStore (core/server/worker/src/main/java/alluxio/worker/
// block/TieredBlockStore.java:85-1009) around page arenas:
//   * tier 0 ("MEM", medium HBM) is a hipMalloc arena on the worker's GPU cut into fixed pages
//     (default 2 MiB); a block is a list of pages, normally one contiguous run;
//   * further tiers are pinned-host arenas (medium DRAM) or file directories (SSD/HDD);
//   * allocation = host bitmap scan for a contiguous run, falling back to scattered pages
//     (reference MaxFree/Greedy/RoundRobin allocators choose the dir, allocator/*.java);
//   * eviction ordering = LRU or LRFU annotations (annotator/LRFUAnnotator.java:81-95) kept
//     resident in HBM per block slot (host mirrors only queue coalesced updates) and selected by a
//     grid-wide byte-weighted radix select (evict_alloc.hip) without holding the store mutex
//     across the device round trip;
//   * batched multi-block creates claim their pages with the device bitmap allocator (K7);
//   * reads/writes are planned into page-contiguous segments and executed by one batched copy
//     kernel launch per batch (kernels.hip, batched_copy_kernel) or by DMA for host endpoints.
// Block locks (BlockLockManager.java), sessions (Sessions.java) and temp->committed lifecycle
// (createBlock/commitBlock/abortBlock) keep the reference semantics.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "kernels.h"

namespace amdx {

struct StoreError : std::runtime_error {
  int code;
  StoreError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
// error codes mirrored in Python (alluxio_amd/ops/native.py)
enum ErrCode {
  kErrNotFound = 1,
  kErrAlreadyExists = 2,
  kErrOutOfSpace = 3,
  kErrInvalidState = 4,
  kErrHip = 5,
  kErrInvalidArgument = 6,
  kErrIo = 7,
  kErrTimeout = 8,
};

enum class DirKind : int { kDevice = 0, kHost = 1, kFile = 2 };
enum class MemKind : int { kHost = 0, kDevice = 1 };
enum class AllocPolicy : int { kMaxFree = 0, kGreedy = 1, kRoundRobin = 2 };
enum class Annotator : int { kLRU = 0, kLRFU = 1 };

struct DirSpec {
  int tier = 0;
  std::string tier_alias = "MEM";
  std::string medium = "HBM";
  DirKind kind = DirKind::kDevice;
  uint64_t base = 0;       // arena base (device or host pointer) for arena kinds
  uint64_t capacity = 0;   // bytes
  uint64_t page_size = 2ull << 20;
  int device = 0;
  std::string path;        // file dirs
  uint64_t reserved = 0;   // reserved bytes (watermark headroom) not used by allocation
  bool owns_base = false;  // device arena allocated for the store: hipFree'd with it
};

struct StorageDir {
  DirSpec spec;
  int index = 0;  // global dir index
  int64_t num_pages = 0;
  std::vector<uint64_t> free_bits;  // arena kinds: 1 = free (host pool)
  int64_t free_pages = 0;           // free pages: host pool + device magazine
  // K7 device magazine of an HBM dir: free pages handed to the GPU (device-resident bitmap,
  // claimed by kernels with atomics), refilled by whole host words, drained only on demand
  uint64_t* mag_bits = nullptr;
  int64_t mag_pages = 0;            // pages in the magazine (refills - claims - drains)
  int64_t mag_cursor = 0;           // next host word a refill looks at
  int64_t mag_lo = -1;              // first word of the arc refills filled since the last drain
  uint64_t* mag_upd = nullptr;      // device staging of refill updates (word, bits) pairs
  size_t mag_upd_cap = 0;
  int64_t reserved_pages = 0;       // kept free for tier management (align/promote swaps)
  uint64_t file_used = 0;  // file dirs: bytes reserved
  uint64_t committed_bytes = 0;
  // host arena registered with the GPU (hipHostRegister mapped): its device-visible address, so
  // tier moves to / from HBM run as one batched copy kernel instead of per-run runtime copies
  uint64_t dev_base = 0;
  bool healthy = true;
  uint64_t available() const;         // for user allocations (excludes the reserved space)
  uint64_t mgmt_available() const;    // for tier-management moves (may use the reserved space)
  uint64_t capacity() const;
};

struct BlockMeta {
  int64_t id = 0;
  int dir = -1;
  uint64_t length = 0;     // bytes written (temp) / final length (committed)
  uint64_t reserved = 0;   // bytes reserved (>= length)
  std::vector<int64_t> pages;
  bool temp = true;
  int64_t session = 0;
  bool pinned_on_create = false;
  int readers = 0;
  bool writer = false;
  bool evicting = false;
  uint32_t slot = 0;
  uint64_t seq = 0;        // creation sequence (victims chosen off-lock are re-validated with it)
  std::vector<uint32_t> crc;
  uint64_t crc_piece = 0;
};

struct ReadReq {
  int64_t block_id;
  uint64_t offset;
  uint64_t length;
  uint64_t dst;
  int dst_kind;  // MemKind
};

struct BlockInfoOut {
  int64_t id;
  uint64_t length;
  int tier;
  int dir;
  std::string tier_alias;
  std::string medium;
  bool temp;
  int64_t session;
  int readers;
  bool writer;
};

struct Event {
  int kind;  // 0 added/committed, 1 removed, 2 moved
  int64_t block_id;
  std::string tier_alias;
  std::string medium;
};

// Bulk creates of at least this many blocks claim their pages with the K7 device magazine.
constexpr size_t kDeviceAllocMinBlocks = 64;

// This thread's non-blocking HIP stream on `device`: one per (thread, device), created on first
// use and destroyed when the thread exits.  Keyed by device, not by store -- a stream belongs to a
// device, so stores that come and go on a pool thread reuse it instead of leaking one each.
hipStream_t thread_stream_on(int device);
// Streams thread_stream_on() has created in this process (tests: flat under store churn).
uint64_t thread_streams_created();

class BlockStore {
 public:
  BlockStore(const std::vector<DirSpec>& dirs, int annotator, int alloc_policy, float lrfu_step,
             float lrfu_attenuation, int device);
  ~BlockStore();

  // ---- lifecycle --------------------------------------------------------------------------
  // Creates a temp block with `initial` reserved bytes.  tier < 0 = any tier (top-down),
  // medium non-empty selects dirs of that medium.  Evicts if allowed and needed.
  int create_block(int64_t session, int64_t block_id, int tier, const std::string& medium,
                   uint64_t initial, bool evict, bool pin);
  // Many temp blocks at once (bulk ingest): one dir choice and, for an HBM dir, one device
  // page-allocation launch (K7) for all of their pages.  Returns the dir of each block.
  std::vector<int> create_blocks(int64_t session, const std::vector<int64_t>& block_ids, int tier,
                                 const std::string& medium, const std::vector<uint64_t>& sizes, bool evict);
  void request_space(int64_t session, int64_t block_id, uint64_t additional);
  // Bulk cache of small files (dataset warm-up / load job): for each (block id, local file path,
  // offset, length) the bytes are pread by `threads` host threads into the caller's pinned
  // staging buffer, copied into fresh temp blocks (async H2D for an HBM dir, the two staging
  // halves double-buffered so reads overlap the copies) and committed.  Returns a status per
  // item: 0 = cached, 1 = already present, 2 = read error, 3 = no space.
  std::vector<int> ingest_files(int64_t session, const std::vector<int64_t>& block_ids,
                                const std::vector<std::string>& paths, const std::vector<uint64_t>& offsets,
                                const std::vector<uint64_t>& lengths, uint64_t staging, uint64_t staging_bytes,
                                int threads, uint64_t stream);
  // Append/overwrite bytes of a temp block (auto-grows).  src_kind: MemKind.
  // Reserve pages for [offset, offset+len) of a temp block and mark those bytes as written by
  // an external producer (RCCL recv / peer DMA straight into the block's pages). Returns the
  // page list so the caller can target the pages directly. Memory dirs only.
  std::vector<int64_t> external_write(int64_t session, int64_t block_id, uint64_t offset, uint64_t len);
  void write(int64_t session, int64_t block_id, uint64_t offset, uint64_t src, uint64_t len,
             int src_kind, uint64_t stream, bool sync);
  void commit_block(int64_t session, int64_t block_id, bool pin);
  void abort_block(int64_t session, int64_t block_id);
  void remove_block(int64_t session, int64_t block_id);
  // move a committed block to another tier/medium; returns new dir index
  int move_block(int64_t session, int64_t block_id, int dst_tier, const std::string& medium,
                 bool evict);
  // Batched move (tier management / demotion): every movable block gets its destination pages,
  // all copies are queued together (one batched-copy launch for HBM<->HBM pieces, async DMA for
  // HBM<->DRAM) and synchronized once; returns the ids that moved.
  std::vector<int64_t> move_blocks(int64_t session, const std::vector<int64_t>& block_ids, int dst_tier,
                                   const std::string& medium, bool evict, bool use_reserved = false);
  // Up to k committed evictable blocks of a tier in annotator order, coldest first (or hottest
  // first): the device grid select picks the k extremes (unit weights, O(n)), the host orders k.
  std::vector<int64_t> tier_order(int tier, uint32_t k, bool hottest, bool device);
  // Annotator keys (larger = hotter; 0xFFFFFFFF = unknown block) for a common order across tiers.
  std::vector<uint32_t> annotator_keys(const std::vector<int64_t>& ids);
  uint64_t dir_mgmt_available(int d);
  // Eviction from a tier that has a lower tier demotes victims into it (batched move, making
  // room there recursively) instead of dropping them.
  void set_demote_on_evict(bool v) { demote_on_evict_ = v; }

  // ---- locks / sessions -------------------------------------------------------------------
  int64_t lock_block(int64_t session, int64_t block_id, bool write, int64_t timeout_ms);
  // Append holds (CACHE_THROUGH tee): a read lock on a committed block that keeps it from being
  // evicted between its commit and the moment the file's UFS stream copies it out (AppendBlock),
  // released by release_hold() once that copy holds its own lock, or after `ttl_ms` (expired holds
  // are swept by the next hold / release).  hold_block is false when the block is not here.
  bool hold_block(int64_t block_id, int64_t ttl_ms);
  bool release_hold(int64_t block_id);
  size_t holds();
  void unlock(int64_t lock_id);
  void cleanup_session(int64_t session);
  void access_block(int64_t session, int64_t block_id);
  void access_blocks(const std::vector<int64_t>& ids);

  // ---- data plane -------------------------------------------------------------------------
  // Batched read of committed (or own temp) blocks into caller buffers.  Device-arena ->
  // device-dst segments are executed by one batched copy launch per ring slot.
  void read_batch(const std::vector<ReadReq>& reqs, uint64_t stream, bool sync);
  // Lock a block if it exists; returns -1 (no throw) when it does not.
  int64_t try_lock_block(int64_t session, int64_t block_id, bool write);
  // CRC32C per piece (piece = page size when 0).
  std::vector<uint32_t> checksum(int64_t block_id, uint64_t piece_bytes);
  // Per-page CRC32C of HBM block `block_id` (temp or committed) enqueued on `stream` behind what
  // it already carries (the block's last H2D): the CRCs land in `dev_buf` (device, `dev_words`
  // words, checksum_async_words) and are copied into `host_out` (pinned, also `dev_words` words:
  // one per page at the front; the rest stages the block's page index array for the single
  // launch over its scattered pages).  Nothing waits: the caller records an event after it.
  // Returns the page count, 0 when the block is not in a device dir or dev_words is too small
  // (checksum() then).
  size_t checksum_async(int64_t block_id, hipStream_t stream, uint32_t* dev_buf, size_t dev_words, uint32_t* host_out,
                        uint64_t* page_size_out);
  // Device words checksum_async needs for a block of `length` bytes in a dir of `page_size` pages.
  static size_t checksum_async_words(uint64_t length, uint64_t page_size);
  // Per-page CRC32C of many blocks: the pages of HBM blocks go to one gather launch (pages up
  // to 256 KiB), others take checksum() (or are skipped with device_only).  Returns (piece bytes,
  // CRCs) per block; missing / skipped blocks get (0, []).
  std::vector<std::pair<uint64_t, std::vector<uint32_t>>> checksum_blocks(const std::vector<int64_t>& block_ids,
                                                                          bool device_only = false);
  void fill_pattern(int64_t session, int64_t block_id, uint64_t length, uint64_t seed);

  // ---- eviction ---------------------------------------------------------------------------
  // Free at least `bytes` in the location (tier < 0 = all tiers, dir >= 0 pins one dir).
  // Returns evicted block ids; throws OutOfSpace when impossible.
  std::vector<int64_t> free_space(int64_t session, uint64_t bytes, int tier, int dir);
  // The annotator's eviction order of up to `limit` evictable blocks in a tier (for tests and
  // tier management), computed by the same kernel/CPU path.
  std::vector<int64_t> eviction_order(int tier, uint64_t need_bytes);
  void set_pinned_files(const std::vector<int64_t>& file_ids);
  void set_use_device_evict(bool v) {
    std::lock_guard<std::mutex> g(mu_);
    if (v && !use_device_evict_) dev_synced_ = false;
    use_device_evict_ = v;
  }
  void set_use_device_alloc(bool v, uint32_t min_pages) {
    use_device_alloc_ = v;
    device_alloc_min_pages_ = min_pages;
  }
  // Victim selection alone (no removal), for benchmarks/tests: device grid select or CPU sort.
  std::vector<int64_t> select_for_bench(int dir, uint64_t need, bool device);
  // K7 alone on a dir's current bitmap, without claiming (benchmarks/tests).
  std::vector<int64_t> peek_free_pages(int dir, uint32_t want, bool device);
  struct EvictStats {
    uint64_t selections = 0, device_selections = 0, candidates = 0, victims = 0, revalidated_away = 0;
    uint64_t device_allocs = 0, device_alloc_pages = 0, annotation_flushes = 0, annotation_updates = 0;
    uint64_t demoted_blocks = 0, demoted_bytes = 0, batched_moves = 0, batched_move_blocks = 0;
    uint64_t mag_refills = 0, mag_refill_pages = 0, mag_drains = 0, mag_drain_pages = 0, mag_short_items = 0;
    uint64_t evict_waits = 0;             // free_space waits for other threads' demotions
    uint64_t evict_retries = 0;           // selections redone after losing victims to other threads
    // ingest_files wall time by phase (ns): 0 block metadata/claims setup, 1 preads, 2 copy/claim
    // launches, 3 waiting on the stream, 4 page attach + commits, 5 up-front magazine refill
    uint64_t ingest_ns[6] = {0, 0, 0, 0, 0, 0};
  };
  EvictStats evict_stats();

  // ---- introspection ----------------------------------------------------------------------
  bool has_block(int64_t block_id);
  bool has_temp_block(int64_t block_id);
  BlockInfoOut block_info(int64_t block_id);
  std::vector<int64_t> block_ids(int tier);
  std::vector<int64_t> block_pages(int64_t block_id, int* dir_out, uint64_t* page_size_out,
                                   uint64_t* base_out);
  // K7 magazine introspection / control (tests, benchmarks): move >= pages into dir's magazine,
  // count the device bitmap, claim for several items at once (their pages stay taken: the caller
  // gives them back with mag_give), hand pages back, drain the magazine into the host pool.
  int64_t mag_refill_pages(int dir, int64_t pages);
  int64_t mag_device_count(int dir);
  // Extra bytes a create / reserve that has to evict frees beyond its own need
  // (alluxio.worker.tieredstore.free.ahead.bytes).
  void set_free_ahead(uint64_t bytes) { free_ahead_ = bytes; }
  // Debug: page accounting of one dir (host pool + K7 magazine + block pages partition the
  // arena; the device magazine bitmap holds exactly mag_pages).  Empty when consistent.
  std::string check_pages(int dir);
  std::vector<std::vector<int64_t>> mag_claim_many(int dir, const std::vector<uint32_t>& wants);
  void mag_give(int dir, const std::vector<int64_t>& pages);
  int64_t mag_drain_dir(int dir);
  int64_t mag_pages(int dir);
  // Path of a committed block held in a file dir (tmpfs / SSD tier), "" otherwise.
  std::string committed_file(int64_t block_id);
  std::vector<Event> drain_events();
  int num_dirs() const { return (int)dirs_.size(); }
  DirSpec dir_spec(int d) const { return dirs_.at(d)->spec; }
  uint64_t dir_capacity(int d);
  uint64_t dir_available(int d);
  uint64_t dir_committed(int d);
  void set_dir_healthy(int d, bool healthy);
  bool dir_healthy(int d);
  uint64_t clock() const { return clock_.load(); }
  int device() const { return device_; }
  bool has_device() const { return has_device_; }
  hipStream_t move_stream();           // this thread's stream on the device (tier moves, tee copies; not internal_stream_)
  void use_device() const { set_device(); }
  std::string stats();

 private:
  BlockMeta& get_committed(int64_t id);
  BlockMeta* find(int64_t id);
  int allocate_dir(int tier, const std::string& medium, uint64_t bytes, bool use_reserved = false);
  bool dir_matches(const StorageDir& d, int tier, const std::string& medium) const;
  bool grow_pages(StorageDir& d, BlockMeta& b, uint64_t new_reserved, bool use_reserved = false);
  void release_storage(BlockMeta& b);
  void free_space_locked(std::unique_lock<std::mutex>& lk, int64_t session, uint64_t bytes,
                         int tier, int dir, const std::string& medium, uint64_t ahead = 0);
  std::vector<uint32_t> select_victims_cpu(const std::vector<uint32_t>& cand_slots, uint64_t need);
  std::vector<uint32_t> select_victims_device(std::unique_lock<std::mutex>& lk, int dir, uint64_t need,
                                              uint64_t dir_mask = 0, bool unit = false, bool invert = false);
  uint32_t host_key(uint32_t slot, uint64_t now) const;
  void remove_locked(BlockMeta& b, bool emit_event);
  std::vector<int64_t> move_blocks_locked(std::unique_lock<std::mutex>& lk, int64_t session,
                                          const std::vector<int64_t>& ids, int dst_tier, const std::string& medium,
                                          bool evict, bool use_reserved = false);
  void copy_block_storage(const BlockMeta& src_snap, const BlockMeta& nb, std::vector<CopySeg>& dev_segs,
                          hipStream_t st);
  int lower_tier(int tier) const;
  // device annotator bookkeeping (all under mu_)
  uint64_t footprint(const BlockMeta& b) const;
  void note_state(const BlockMeta& b, bool live);
  void mark_dirty(uint32_t slot);
  void ensure_dev_slots_locked(size_t n);
  void flush_annotations_locked();
  EvictState dev_state(uint64_t now) const;
  bool device_evict_active() const { return has_device_ && use_device_evict_; }
  std::vector<int64_t> device_alloc_pages(std::unique_lock<std::mutex>& lk, int dir, uint32_t want);
  void mag_refill(StorageDir& d, int64_t want);                    // mu_ held
  int64_t mag_drain(StorageDir& d);                                 // mu_ held
  std::pair<uint32_t, uint32_t> mag_window(const StorageDir& d) const;  // mu_ held
  bool ingest_device_group(int64_t session, const std::vector<int64_t>& ids, const std::vector<uint64_t>& lengths,
                           const std::vector<size_t>& items, const std::vector<uint64_t>& at, size_t lo,
                           uint8_t* dbase, int h, hipStream_t st, std::vector<int64_t>& pending);
  std::unordered_set<int64_t> ingest_device_finish(int64_t session, int h, const std::vector<uint64_t>& lengths,
                                                   const uint8_t* host_base, std::vector<int>& status);
  uint32_t alloc_slot();
  void touch_slot(uint32_t slot);
  bool evictable(const BlockMeta& b) const;
  void emit(int kind, const BlockMeta& b);
  void copy_segments(std::vector<CopySeg>& dev_segs, hipStream_t stream);
  // `ext_mapped`: device-visible address of a host `ext` (0 = none); `mapped_kernel`: copies between
  // HBM and GPU-mapped host memory go into dev_segs (batched copy kernel) instead of hipMemcpyAsync.
  void plan_block_range(const BlockMeta& b, uint64_t offset, uint64_t len, uint64_t ext,
                        int ext_kind, bool to_block, std::vector<CopySeg>& dev_segs,
                        hipStream_t stream, uint64_t ext_mapped = 0, bool mapped_kernel = false);
  void file_path(const StorageDir& d, int64_t id, std::string& out) const;
  void set_device() const;
  hipStream_t stream_or_default(uint64_t s) const;

  std::mutex mu_;
  std::condition_variable lock_cv_;
  std::vector<std::unique_ptr<StorageDir>> dirs_;
  std::unordered_map<int64_t, BlockMeta> blocks_;
  uint64_t free_ahead_ = 0;
  std::unordered_set<int64_t> pinned_files_;
  // lock table
  struct LockRec { int64_t block; int64_t session; bool write; };
  std::unordered_map<int64_t, LockRec> locks_;
  std::unordered_map<int64_t, std::unordered_set<int64_t>> session_locks_;
  std::unordered_map<int64_t, std::unordered_set<int64_t>> session_temps_;
  int64_t next_lock_ = 1;
  // annotator SoA (slot-indexed)
  Annotator annotator_;
  AllocPolicy alloc_policy_;
  float lrfu_step_, lrfu_att_;
  std::vector<float> crf_;
  std::vector<uint64_t> last_;
  std::vector<int64_t> slot_block_;
  std::vector<uint32_t> free_slots_;
  std::atomic<uint64_t> clock_{0};
  uint64_t create_seq_ = 0;
  std::vector<int32_t> slot_dir_;            // mirror of the device dir[] (evictable dir or -1)
  std::vector<uint64_t> slot_fb_;            // mirror of fbytes[]
  std::vector<uint64_t> dir_ev_bytes_;       // per dir: footprint of statically evictable blocks
  std::unordered_set<int64_t> evicting_ids_;
  // slots whose mirror (crf_, last_, slot_dir_, slot_fb_) changed since the last device flush
  std::vector<uint32_t> dirty_;
  std::vector<uint8_t> dirty_flag_;
  bool dev_synced_ = false;                  // device arrays hold every slot's mirror values
  EvictStats stats_;
  std::vector<int> rr_index_;  // round-robin cursor per tier
  std::vector<Event> events_;
  // device resources
  int device_ = -1;
  bool has_device_ = false;
  bool use_device_evict_ = true;
  // K7 measured slower than the host bitmap scan end to end (profiles/r2_evict_bench.jsonl):
  // off unless alluxio.worker.hbm.device.alloc.enabled
  bool use_device_alloc_ = true;              // K7 magazine: bulk creates (>= min pages) and ingest claim on the GPU
  bool demote_on_evict_ = false;
  uint32_t device_alloc_min_pages_ = 1024;     // create_blocks: device claims from this many pages
  hipStream_t internal_stream_ = nullptr;
  static constexpr int kRing = 8;
  static constexpr int kRingSegs = 8192;
  CopySeg* host_ring_ = nullptr;   // pinned
  CopySeg* dev_ring_ = nullptr;
  hipEvent_t ring_ev_[kRing] = {};
  int ring_pos_ = 0;
  std::mutex ring_mu_;
  // device annotator arrays (slot-indexed, grown by doubling under mu_ + ev_mu_)
  size_t dev_slots_ = 0;
  float* d_crf_ = nullptr;
  uint64_t* d_last_ = nullptr;
  uint64_t* d_fbytes_ = nullptr;
  int32_t* d_dir_ = nullptr;
  uint32_t* d_keys_ = nullptr;
  uint32_t* d_excl_ = nullptr;
  uint32_t* h_excl_ = nullptr;       // pinned exclusion bitmap (locked slots of one selection)
  EvictCtl* d_ctl_ = nullptr;
  EvictCtl* h_ctl_ = nullptr;        // pinned readback
  uint32_t* h_out_ = nullptr;        // pinned, device-mapped victim list
  uint32_t* h_out_dev_ = nullptr;
  SlotUpdate* h_upd_[2] = {nullptr, nullptr};
  size_t h_upd_cap_[2] = {0, 0};
  hipEvent_t upd_ev_[2] = {};
  int upd_pos_ = 0;
  SlotUpdate* d_upd_ = nullptr;
  size_t d_upd_cap_ = 0;
  // K7 scratch
  uint64_t* d_bits_ = nullptr;
  size_t d_bits_cap_ = 0;
  uint32_t* d_partial_ = nullptr;
  size_t d_partial_cap_ = 0;
  int64_t* h_pages_ = nullptr;       // pinned, device-mapped page list
  int64_t* h_pages_dev_ = nullptr;
  size_t h_pages_cap_ = 0;
  uint32_t* h_claimed_ = nullptr;
  uint32_t* d_claimed_ = nullptr;
  std::mutex ev_mu_;                 // device selection / allocation scratch (taken after mu_)
  // append holds: block -> [(lock id, expiry ns)]
  std::mutex holds_mu_;
  std::unordered_map<int64_t, std::vector<std::pair<int64_t, int64_t>>> holds_;
  void sweep_holds_locked(int64_t now_ns);
  // checksum scratch
  uint32_t* crc_dev_ = nullptr;
  size_t crc_cap_ = 0;
  // device staging of ingest_files (mirror of the caller's pinned staging)
  void* ingest_dev_ = nullptr;
  uint64_t ingest_dev_cap_ = 0;
  std::mutex ingest_mu_;             // one ingest_files at a time (staging + claim scratch)
  // K7 fused claim + scatter of ingest_files, one scratch set per staging half
  struct ClaimScratch {
    ClaimItem* items_h = nullptr;    // pinned
    ClaimItem* items_d = nullptr;
    int64_t* pages_h = nullptr;      // pinned
    int64_t* pages_d = nullptr;
    uint32_t* got_h = nullptr;       // pinned
    uint32_t* got_d = nullptr;
    size_t items_cap = 0, pages_cap = 0;
    int dir = -1;
    std::vector<int64_t> ids;        // blocks of the in-flight group, item order
    std::vector<size_t> index;       // their positions in the caller's arrays
    std::vector<uint64_t> at;        // their offsets in the host staging half
  } claim_[2], claim_one_;                   // claim_one_: standalone claims (under ev_mu_)
  void claim_reserve(ClaimScratch& c, size_t items, size_t pages);
};

// Many concurrent sequential readers of one file, advanced in lockstep: the native form of
// StressWorkerBench's reader threads (stress/shell/.../StressWorkerBench.java:251-276: each
// thread loops read(buf) and re-opens the file at EOF).  Every ``step`` advances every stream by
// one read of ``buf_bytes`` (or the EOF read that triggers a re-open), keeps a read lock on each
// stream's current block (switching locks at block boundaries like BlockInStream), and executes
// all the stream reads as ONE batched page-gather launch.
class ReadSession {
 public:
  ReadSession(BlockStore* store, int64_t session, const std::vector<int64_t>& block_ids,
              const std::vector<uint64_t>& block_lens, const std::vector<uint64_t>& dst_ptrs,
              uint64_t buf_bytes, int dst_kind, const std::vector<uint64_t>& start_offsets);
  ~ReadSession();
  // Returns bytes read in this step; `reopened` receives the streams that hit EOF.
  uint64_t step(uint64_t stream, std::vector<int>* reopened);
  uint64_t run(int steps, uint64_t stream);  // many steps, no per-step return to Python
  void reset_file(const std::vector<int64_t>& block_ids, const std::vector<uint64_t>& block_lens);
  void close();
  uint64_t total_bytes() const { return total_; }
  uint64_t reopens() const { return reopens_; }
  uint64_t position(int i) const { return pos_.at(i); }

 private:
  void switch_block(int i, int64_t blk);
  BlockStore* store_;
  int64_t session_;
  std::vector<int64_t> blocks_;
  std::vector<uint64_t> lens_, starts_;
  uint64_t file_len_ = 0;
  std::vector<uint64_t> dst_;
  uint64_t buf_;
  int kind_;
  std::vector<uint64_t> pos_;
  std::vector<int64_t> cur_block_idx_, lock_;
  std::vector<ReadReq> reqs_;
  uint64_t total_ = 0, reopens_ = 0;
  bool closed_ = false;
};

}  // namespace amdx
