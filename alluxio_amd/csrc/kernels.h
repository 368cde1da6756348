// Host-side launch interface of the CDNA4 (gfx950) kernels used by the worker data plane.
//
// Reference hot loops these replace:
//   K1/K2  block read/write chunk copy   W/grpc/BlockReadHandler.java:124-130, BlockWriteHandler.java:124-149
//   K4-K6  LRU/LRFU ordering + free-space loop  W/block/annotator/LRFUAnnotator.java:81-95,
//          W/block/TieredBlockStore.java:740-815
//   K10    CRC32C (new; reference only has whole-file MD5 in ChecksumCommand.java:78-88)
//   K11    LZ4 block codec (new)
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

namespace amdx {

// One contiguous copy piece (never crosses a page boundary on the arena side).
struct CopySeg {
  uint64_t src;      // byte address (device or host-pinned mapped)
  uint64_t dst;      // byte address
  uint64_t bytes;
  uint64_t chunk0;   // exclusive prefix of chunk counts (filled by the planner)
};

// Tile (bytes) one workgroup moves per work item of the batched copy.
constexpr uint64_t kCopyChunk = 256 * 1024;

// Batched gather/scatter copy.  `segs` must be device-visible; `total_chunks` = sum of
// ceil(bytes / kCopyChunk).  Grid is capped and grid-strided.
hipError_t launch_batched_copy(const CopySeg* segs, int nseg, uint64_t total_chunks,
                               hipStream_t stream);
// Select the copy kernel variant (cache policy / unroll) and grid cap; used for A/B tuning.
void set_copy_variant(int variant, unsigned grid_cap);

// Device-cursor sequential multi-stream read (StressWorkerBench shape, K1 without per-read
// descriptors).  S streams each issue `depth` consecutive read(buf) calls per launch over one
// cached file whose pages are listed in `ftab` (file page -> arena page).  Stream s's call
// index of launch L is g = c_init[s] + launch_base + k; with cycle = ceil(file_len/buf) + 1
// calls per pass (the last call of a pass hits EOF and reopens), call c = g % cycle reads
// [c*buf, min(file_len, (c+1)*buf)) into dst + s*stream_stride + k*buf (a ring of `depth`
// slots per stream).  Everything the kernel needs is computed from scalars: O(1) host work
// per launch regardless of S and depth.
struct SeqReadArgs {
  const uint8_t* arena;
  const int64_t* ftab;
  const uint64_t* c_init;
  uint8_t* dst;
  uint64_t stream_stride;
  uint64_t file_len;
  uint64_t buf;
  uint64_t launch_base;
  uint32_t cycle;
  uint32_t streams;
  uint32_t depth;
  uint32_t page_shift;
  uint64_t footprint = 0;   // distinct file bytes one launch touches (host estimate; 0 = file_len)
};
constexpr uint32_t kSeqReadMaxStreams = 8192;
hipError_t launch_seq_read(const SeqReadArgs& a, hipStream_t stream);
// A/B switch for the sequential-read kernel (bit0: nontemporal ring stores, bit1: unroll 16).
void set_seq_read_variant(int variant, unsigned grid_cap);

// CRC32C (Castagnoli, reflected, init/xorout 0xFFFFFFFF) of `n` equal-length pieces
// (piece i = base + i*piece_bytes, last may be shorter: total_bytes).  `out` device array.
hipError_t launch_crc32c_pieces(const uint8_t* base, uint64_t total_bytes, uint64_t piece_bytes,
                                uint32_t* out, uint32_t* scratch, uint64_t scratch_words,
                                hipStream_t stream);
// The same per-page CRC32Cs of a block whose pages are scattered in an arena: page i of the block
// is base + page_idx[i] * page_bytes (page_idx: device array).  One launch pair for the whole
// block; hipErrorNotSupported when the active CRC variant has no paged form (use per-run launches).
hipError_t launch_crc32c_pages(const uint8_t* base, const int64_t* page_idx, uint64_t total_bytes,
                               uint64_t page_bytes, uint32_t* out, uint32_t* scratch, uint64_t scratch_words,
                               hipStream_t stream);
// Scratch words launch_crc32c_pages needs.
uint64_t crc32c_pages_scratch_words(uint64_t total_bytes, uint64_t page_bytes);
// Standard CRC32C of n gathered pieces (device pointers/lengths in device memory, each piece
// <= crc32c_gather_max_piece() bytes), one workgroup per piece.
hipError_t launch_crc32c_gather(const uint64_t* ptrs, const uint32_t* lens, uint64_t n, uint32_t* out,
                                hipStream_t stream);
uint64_t crc32c_gather_max_piece();
// 0: per-lane contiguous strips, 1 (default): interleaved coalesced lanes.
void set_crc_variant(int v);
// Scratch words needed by launch_crc32c_pieces (an upper bound for every variant).
uint64_t crc32c_scratch_words(uint64_t total_bytes, uint64_t piece_bytes);

// LZ4 block decompression of `n` independent chunks.
struct Lz4Chunk {
  uint64_t src;       // compressed bytes (device)
  uint64_t dst;       // output (device)
  uint32_t src_bytes;
  uint32_t dst_capacity;
};
hipError_t launch_lz4_decompress(const Lz4Chunk* chunks, int n, int32_t* out_sizes,
                                 hipStream_t stream);
// 0: LDS-window decoder, 1: direct-to-HBM, 2 (default): direct + LDS-staged parse, 3: + LDS ring
// of recent output for near matches.
void set_lz4_decode_variant(int v);
void set_lz4_encode_variant(int v);
// LZ4 block compression (greedy, one wave per chunk, LDS hash table).  out_sizes[i] = -1 if
// the chunk does not fit dst_capacity (caller then stores it raw).
hipError_t launch_lz4_compress(const Lz4Chunk* chunks, int n, int32_t* out_sizes,
                               hipStream_t stream);

// ---- device-resident annotations + grid-wide select (evict_alloc.hip) ----------------------
// Slot-indexed arrays in HBM.  dir[s] = storage dir of a committed, statically evictable block
// (not temp / pinned), -1 otherwise; fbytes = its page-rounded footprint.
struct EvictState {
  float* crf;
  uint64_t* last;
  uint64_t* fbytes;
  int32_t* dir;
  uint32_t n;            // slots in use (grid extent)
  uint64_t now;          // logical access clock
  float step;            // LRFU step factor
  float log2_inv_att;    // log2(1 / attenuation)
  int policy;            // 0 = LRU, 1 = LRFU
  uint64_t dir_mask;     // candidate dirs (bit d = dir d); 0 = the select's target dir only
  int unit;              // 1: every candidate weighs 1 (select by count, not bytes)
  int invert;            // 1: hottest first (select the largest keys)
};
constexpr uint32_t kSlotSetState = 1, kSlotReset = 2, kSlotTouch = 4;
// One coalesced host->device update per slot: state (dir, footprint) and/or annotations
// (reset: crf = crf, last = t; touch: crf = crf_dev * decay(t - last_dev) + crf, last = t).
struct SlotUpdate {
  uint32_t slot;
  uint32_t flags;
  int32_t dir;
  float crf;
  uint64_t fbytes;
  uint64_t t;
};
// Max selection grid (workgroups per pass).
constexpr unsigned kEvSlabRows = 128;
struct EvictCtl {
  unsigned long long hist[256];
  unsigned long long total;     // evictable footprint in the target dir
  unsigned long long acc;       // bytes of keys strictly below the current prefix
  unsigned long long tie_acc;
  unsigned long long freed;
  uint32_t prefix, mask;
  uint32_t all, done;
  uint32_t count, pad;
};
hipError_t launch_slot_update(const EvictState& st, const SlotUpdate* upd, uint32_t n, hipStream_t stream);
// Smallest-key-first victims of `target_dir` whose footprints add up to >= need (all of them if
// the dir holds less); `excl` (bitmap by slot, may be null) removes locked slots.  Victim slots
// go to out_slots (device-visible, e.g. mapped pinned host), their count/bytes to ctl->count/freed.
hipError_t launch_evict_select_grid(const EvictState& st, uint32_t target_dir, const uint32_t* excl,
                                    uint64_t need, uint32_t* keys, EvictCtl* ctl, uint32_t* out_slots,
                                    hipStream_t stream);
// K7: claim the `want` lowest free pages of a free-page bitmap (1 = free) in place; pages_out
// gets the page numbers, *claimed how many (< want if the bitmap ran out).  `partial` needs
// page_alloc_partials(nwords) words.
hipError_t launch_page_alloc(uint64_t* bits, uint32_t nwords, uint32_t want, uint32_t* partial,
                             int64_t* pages_out, uint32_t* claimed, hipStream_t stream);
uint32_t page_alloc_partials(uint32_t nwords);

// K7 device page magazine (evict_alloc.hip): an HBM dir keeps a device-resident bitmap of free
// pages it handed to the device ("magazine"); kernels claim pages from it with atomics, the host
// refills it by whole bitmap words and drains it back only when its own pool runs dry.
struct ClaimItem {
  uint64_t src;          // device source of the item's bytes (scatter) or 0 (claim only)
  uint64_t len;          // bytes
  uint32_t want;         // pages to claim
  uint32_t page_base;    // first index in pages_out
  uint32_t chunk_base;   // first 64 KiB chunk of this item in the scatter grid
  uint32_t pad;
};
// bits[upd[2i]] |= upd[2i+1] (atomic): pages moved into the magazine
hipError_t launch_mag_fill(uint64_t* bits, uint32_t nwords, const uint64_t* upd, uint32_t n, hipStream_t stream);
// out[w] = atomicExch(bits[w], 0): the magazine handed back (no claim can race it)
hipError_t launch_mag_drain(uint64_t* bits, uint32_t nwords, uint64_t* out, hipStream_t stream);
// One wave per item claims item.want pages (atomicAnd on the words, ballot/popcount ranking)
// into pages_out[page_base ...]; got[i] = pages claimed (< want when the magazine ran dry).
// When total_chunks > 0 a second launch copies each item's bytes into its claimed pages (one
// wave per 64 KiB chunk; items that came up short are skipped -- the host finishes them).
// win_lo/win_len: the words the magazine's bits live in (refills fill a contiguous arc of the
// bitmap); items search there first and fall back to the whole bitmap when it runs dry.
hipError_t launch_mag_claim_scatter(uint64_t* bits, uint32_t nwords, const ClaimItem* items, uint32_t nitems,
                                    int64_t* pages_out, uint32_t pages_cap, uint32_t* got, uint32_t total_chunks,
                                    uint8_t* arena, uint64_t page_size, hipStream_t stream, uint32_t win_lo = 0,
                                    uint32_t win_len = 0);

// K9: client page cache lookup.  Open-addressing (linear probing) table of page keys in HBM;
// `key` = (interned file id << 24) | page index, so keys are exact (no hash collisions to
// verify).  Empty slots hold kPageKeyEmpty, erased ones kPageKeyTomb (probing continues).
struct PageTableEntry {
  uint64_t key;
  int32_t slot;    // arena slot of the page
  uint32_t len;    // valid bytes in the page
};
constexpr uint64_t kPageKeyEmpty = ~0ull;
constexpr uint64_t kPageKeyTomb = ~0ull - 1;
__host__ __device__ inline uint64_t page_key_hash(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
// Fused lookup + gather of `n` pages whose keys live in device memory: request i copies the
// valid bytes of page keys[i] from arena slot to dst + i*dst_stride, writes slot_out[i] (-1 on a
// miss) and len_out[i], and stamps[slot] = epoch on a hit (device-side LRU recency).  One wave
// probes 64 table entries per step with a ballot; `chunk_bytes` splits big pages over gridDim.y.
struct PageGatherArgs {
  const PageTableEntry* table;
  uint64_t mask;           // table size - 1 (power of two)
  const uint64_t* keys;
  uint32_t n;
  const uint8_t* arena;
  uint64_t page_size;
  uint8_t* dst;
  uint64_t dst_stride;
  int32_t* slot_out;
  uint32_t* len_out;
  uint32_t* stamps;
  uint32_t epoch;
};
hipError_t launch_page_lookup_gather(const PageGatherArgs& a, hipStream_t stream);
// Largest page size served by the wave-per-request kernel (bigger pages: workgroup per chunk).
void set_page_gather_small_max(uint64_t bytes);
void set_page_gather_wave_variant(int variant);
void set_page_gather_chunk_variant(int v);
// Apply table updates (idx, entry) pairs uploaded by the host mirror.
hipError_t launch_page_table_update(PageTableEntry* table, const uint64_t* idx,
                                    const PageTableEntry* entries, uint32_t n, hipStream_t stream);

// K9 put path on the GPU (page_cache_put.hip): probe/claim -> assign (free stack or CLOCK
// eviction) -> fill, for a batch of device-resident keys; the device table is authoritative.
struct PutCounters {
  int32_t free_top;        // entries left on the device free stack (may go negative)
  uint32_t hand;           // CLOCK hand
  uint32_t nfresh;         // keys this batch claimed new table entries for
  uint32_t nevicted;       // victims (their keys in `evicted`)
  uint32_t ntomb;          // tombstones this batch created
  uint32_t nfail;          // requests that got no slot
  uint32_t min_age;        // victims: slots not touched for >= this many epochs (threshold kernel)
  uint32_t pad;
};
constexpr uint32_t kPutAgeBuckets = 4096;   // recency histogram: age = epoch - stamp, clamped
struct PagePutArgs {
  PageTableEntry* table;
  uint64_t mask;
  const uint64_t* keys;
  uint32_t n;
  uint32_t* tidx;                // [n] table index of each request
  unsigned long long* tag;       // [table size] (batch << 32) | (request + 1) of the winner
  unsigned long long batch;
  uint32_t* stamps;              // [slots] recency (shared with the gather kernel)
  uint32_t* hist;                // [kPutAgeBuckets] slots per age (eviction threshold)
  uint32_t epoch;
  uint32_t nslots;
  uint64_t* slot_key;            // [slots] key held by each slot (kPageKeyEmpty = free)
  uint32_t* slot_tidx;           // [slots] table index of that key
  uint32_t* free_stack;          // [slots]
  PutCounters* ctr;
  uint64_t* evicted;             // [n]
  int32_t* slot_of;              // [n] slot to fill (-1: duplicate or failed)
  int evict;
  uint32_t len;
  const uint8_t* src;
  uint64_t src_stride;
  uint8_t* arena;
  uint64_t page_size;
};
hipError_t launch_page_put_probe(const PagePutArgs& a, hipStream_t stream);
hipError_t launch_page_put_assign(const PagePutArgs& a, hipStream_t stream);
hipError_t launch_page_put_fill(const PagePutArgs& a, hipStream_t stream);
hipError_t launch_page_put_revert(const PagePutArgs& a, hipStream_t stream);
// Age histogram of the evictable slots + the threshold age that frees enough of them.
hipError_t launch_page_put_threshold(const PagePutArgs& a, hipStream_t stream);
// Drop tombstones on the device: live entries of a.table are re-inserted into `fresh` (cleared
// first) and slot_tidx is repointed; the caller swaps the two tables afterwards.
hipError_t launch_page_table_rebuild(const PagePutArgs& a, PageTableEntry* fresh, hipStream_t stream);

// Fill `bytes` at dst with 64-bit words w[i] = splitmix64(seed ^ ((i + word_offset) * K)):
// synthetic bench/test data that is a pure function of the byte offset inside a block.
hipError_t launch_fill_pattern(uint8_t* dst, uint64_t bytes, uint64_t seed, uint64_t word_offset,
                               hipStream_t stream);

}  // namespace amdx
