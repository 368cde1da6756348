// K9 put path on the GPU: resolve, evict and fill a batch of page keys without the host table.
//
// Reference: core/client/fs/src/main/java/alluxio/client/file/cache/LocalCacheManager.java:249-347
// (putInternal: look the page up, evict when the cache is full, store, index).  On MI355X a batch
// of pages (keys already on the GPU, e.g. produced by a device-side sampler) is inserted by three
// launches on one stream, with the open-addressing table in HBM authoritative for the batch:
//
//   1. probe  (thread per request): find the key or claim an EMPTY entry with atomicCAS on the
//      key word; tag the entry with atomicMax((batch << 32) | (i + 1)) so the LAST request of a
//      key in the batch wins (sequential put() semantics); touch the stamp of a found page;
//   2. threshold (evict only): a histogram of the evictable slots' ages (epoch - recency stamp;
//      stamps are written by puts and by the gather kernel) and a one-block scan from the oldest
//      age pick the smallest age A such that the slots untouched for >= A epochs cover the
//      shortfall (fresh keys - free slots): approximate LRU at epoch granularity, no host sort;
//   3. assign (thread per request, winners only): a fresh key pops a slot off the device free
//      stack, or takes a victim under a rotating hand -- both wave-aggregated (one atomic per wave
//      and round, lanes take consecutive positions) -- whose age is >= A; the victim is claimed
//      with atomicCAS on its stamp and its table entry becomes a tombstone;
//   4. fill   (wave per 64 KiB chunk of a request): copy the page bytes into the winner's slot.
//
// Tombstones are never reclaimed by inserts (a concurrent probe of the same batch could otherwise
// miss a key placed behind one); when they pile up the table is rebuilt on the device (live
// entries re-inserted into a cleared second table, slot -> entry index repointed).
#include "kernels.h"

#include <algorithm>

namespace amdx {

typedef unsigned int u32x4p __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t ld_key(const PageTableEntry* e) {
  return __hip_atomic_load(&e->key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void page_put_probe_kernel(PagePutArgs a) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
    const uint64_t key = a.keys[i];
    uint64_t h = page_key_hash(key) & a.mask;
    uint32_t tidx = 0xFFFFFFFFu;
    for (uint64_t probe = 0; probe <= a.mask; ++probe, h = (h + 1) & a.mask) {
      uint64_t k = ld_key(&a.table[h]);
      if (k == kPageKeyEmpty) {
        unsigned long long prev = atomicCAS((unsigned long long*)&a.table[h].key,
                                            (unsigned long long)kPageKeyEmpty, (unsigned long long)key);
        if (prev == kPageKeyEmpty) {           // claimed: a fresh key of this batch
          atomicAdd(&a.ctr->nfresh, 1u);
          tidx = (uint32_t)h;
          break;
        }
        k = prev;                              // lost the race: whoever won holds this entry now
      }
      if (k == key) {
        tidx = (uint32_t)h;
        break;
      }
    }
    a.tidx[i] = tidx;
    if (tidx == 0xFFFFFFFFu) {                 // table full (cannot happen at load <= 1/2)
      atomicAdd(&a.ctr->nfail, 1u);
      continue;
    }
    atomicMax(&a.tag[tidx], (a.batch << 32) | (unsigned long long)(i + 1));
    const int32_t slot = __hip_atomic_load(&a.table[tidx].slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (slot >= 0) atomicMax(&a.stamps[slot], a.epoch);   // a page of this batch is never a victim
  }
}

__device__ __forceinline__ bool page_put_take(const PagePutArgs& a, uint32_t s, uint32_t min_age) {
  const uint32_t st = __hip_atomic_load(&a.stamps[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (st >= a.epoch || a.epoch - st < min_age) return false;   // this batch's page / too recent
  const uint64_t old = __hip_atomic_load(&a.slot_key[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old == kPageKeyEmpty) return false;                      // free slot (owned by the free stack)
  if (atomicCAS(&a.stamps[s], st, a.epoch) != st) return false; // another request took it
  const uint32_t ot = a.slot_tidx[s];
  __hip_atomic_store(&a.table[ot].key, kPageKeyTomb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  a.table[ot].slot = -1;
  a.table[ot].len = 0;
  const uint32_t e = atomicAdd(&a.ctr->nevicted, 1u);
  if (e < a.n) a.evicted[e] = old;
  atomicAdd(&a.ctr->ntomb, 1u);
  return true;
}

__device__ __forceinline__ uint32_t wave_rank(uint64_t m, int lane) {
  return (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

__global__ __launch_bounds__(256) void page_put_assign_kernel(PagePutArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t stride = gridDim.x * blockDim.x;
  const uint32_t min_age = a.evict ? __hip_atomic_load(&a.ctr->min_age, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                   : 0xFFFFFFFFu;
  // wave-uniform trip count: every lane of a wave runs the same iterations (ballots below)
  for (uint32_t base = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < a.n; base += stride) {
    const uint32_t i = base + lane;
    uint32_t tidx = 0xFFFFFFFFu;
    int32_t slot = -1;
    bool winner = false;
    if (i < a.n) {
      tidx = a.tidx[i];
      a.slot_of[i] = -1;
      if (tidx != 0xFFFFFFFFu && a.tag[tidx] == ((a.batch << 32) | (unsigned long long)(i + 1))) {
        winner = true;
        slot = a.table[tidx].slot;
      }
    }
    const bool fresh = winner && slot < 0;
    bool need = fresh;
    uint64_t m = __ballot(need);
    if (m) {                                     // free stack: one atomicSub per wave
      const int leader = __ffsll((long long)m) - 1;
      int32_t top = 0;
      if (lane == leader) top = atomicSub(&a.ctr->free_top, (int32_t)__popcll(m));
      top = __shfl(top, leader);
      const int32_t t = top - 1 - (int32_t)wave_rank(m, lane);
      if (need && t >= 0) {
        slot = (int32_t)a.free_stack[t];
        need = false;
      }
    }
    if (a.evict) {                               // victims: one hand advance per wave and round
      uint64_t scanned = 0;
      const uint64_t budget = 2ull * a.nslots + 64;
      while ((m = __ballot(need)) != 0 && scanned < budget) {
        const int leader = __ffsll((long long)m) - 1;
        const uint32_t cnt = (uint32_t)__popcll(m);
        uint32_t h = 0;
        if (lane == leader) h = atomicAdd(&a.ctr->hand, cnt);
        h = __shfl(h, leader);
        scanned += cnt;
        if (need) {
          const uint32_t s = (uint32_t)(((uint64_t)h + wave_rank(m, lane)) % a.nslots);
          if (page_put_take(a, s, min_age)) {
            slot = (int32_t)s;
            need = false;
          }
        }
      }
    }
    if (!winner) continue;
    if (fresh) {
      if (need) {                                // no space: the claimed entry goes away again
        __hip_atomic_store(&a.table[tidx].key, kPageKeyTomb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        atomicAdd(&a.ctr->ntomb, 1u);
        atomicAdd(&a.ctr->nfail, 1u);
        continue;
      }
      // stamp before the key: a concurrent hand sees either a free slot or this batch's stamp
      atomicMax(&a.stamps[slot], a.epoch);
      __hip_atomic_store(&a.slot_key[slot], a.keys[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      a.slot_tidx[slot] = tidx;
      a.table[tidx].slot = slot;
    }
    a.table[tidx].len = a.len;
    a.slot_of[i] = slot;
  }
}

// Ages of the evictable slots (occupied, not touched by this batch), LDS histogram per block.
__global__ __launch_bounds__(256) void page_put_hist_kernel(PagePutArgs a) {
  __shared__ uint32_t h[kPutAgeBuckets];
  for (uint32_t b = threadIdx.x; b < kPutAgeBuckets; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < a.nslots; s += stride) {
    if (a.slot_key[s] == kPageKeyEmpty) continue;
    const uint32_t st = a.stamps[s];
    if (st >= a.epoch) continue;
    atomicAdd(&h[min(a.epoch - st, kPutAgeBuckets - 1)], 1u);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < kPutAgeBuckets; b += blockDim.x)
    if (h[b]) atomicAdd(&a.hist[b], h[b]);
}

// One block: smallest age A whose tail (ages >= A) covers the shortfall.
__global__ __launch_bounds__(256) void page_put_thresh_kernel(PagePutArgs a) {
  constexpr uint32_t kPer = kPutAgeBuckets / 256;
  __shared__ uint32_t part[256];
  const uint32_t t = threadIdx.x;
  const uint32_t hi = kPutAgeBuckets - 1 - t * kPer;           // this thread: ages hi .. hi-kPer+1
  uint32_t sum = 0;
  for (uint32_t k = 0; k < kPer; ++k) sum += a.hist[hi - k];
  part[t] = sum;
  __syncthreads();
  if (t != 0) return;
  const int64_t need = (int64_t)a.ctr->nfresh - (int64_t)max(a.ctr->free_top, 0);
  uint32_t age = kPutAgeBuckets;                                // nothing to evict
  if (need > 0) {
    age = 1;                                                    // not enough: everything evictable
    int64_t cum = 0;
    for (uint32_t c = 0; c < 256; ++c) {
      if (cum + part[c] < need) {
        cum += part[c];
        continue;
      }
      const uint32_t top = kPutAgeBuckets - 1 - c * kPer;
      for (uint32_t k = 0; k < kPer; ++k) {
        cum += a.hist[top - k];
        if (cum >= need) {
          age = max(top - k, 1u);
          break;
        }
      }
      break;
    }
  }
  a.ctr->min_age = age;
}

__global__ __launch_bounds__(256) void page_table_clear_kernel(PageTableEntry* t, uint64_t size) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < size; i += stride)
    t[i] = PageTableEntry{kPageKeyEmpty, -1, 0};
}

__global__ __launch_bounds__(256) void page_table_reinsert_kernel(PagePutArgs a, PageTableEntry* fresh) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= a.mask; i += stride) {
    const PageTableEntry e = a.table[i];
    if (e.key == kPageKeyEmpty || e.key == kPageKeyTomb || e.slot < 0) continue;
    uint64_t h = page_key_hash(e.key) & a.mask;
    for (uint64_t probe = 0; probe <= a.mask; ++probe, h = (h + 1) & a.mask) {
      const unsigned long long prev = atomicCAS((unsigned long long*)&fresh[h].key,
                                                (unsigned long long)kPageKeyEmpty, (unsigned long long)e.key);
      if (prev == kPageKeyEmpty) {
        fresh[h].slot = e.slot;
        fresh[h].len = e.len;
        a.slot_tidx[e.slot] = (uint32_t)h;
        break;
      }
    }
  }
}

// Wave per (request, 64 KiB chunk): 64 lanes x 16 B x 4 in flight.
constexpr uint64_t kPutChunk = 64 * 1024;

template <bool VEC>
__global__ __launch_bounds__(256) void page_put_fill_kernel(PagePutArgs a, uint32_t nch) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * 4;
  const uint64_t total = (uint64_t)a.n * nch;
  for (uint64_t r = wave; r < total; r += nwaves) {
    const uint32_t i = (uint32_t)(r / nch), c = (uint32_t)(r % nch);
    const int32_t slot = a.slot_of[i];
    if (slot < 0) continue;
    const uint64_t off0 = (uint64_t)c * kPutChunk;
    if (off0 >= a.len) continue;
    const uint64_t bytes = std::min<uint64_t>(kPutChunk, a.len - off0);
    const uint8_t* src = a.src + (uint64_t)i * a.src_stride + off0;
    uint8_t* dst = a.arena + (uint64_t)slot * a.page_size + off0;
    if constexpr (VEC) {
      const u32x4p* s = reinterpret_cast<const u32x4p*>(src);
      u32x4p* d = reinterpret_cast<u32x4p*>(dst);
      const uint64_t nv = bytes >> 4;
      uint64_t v = lane;
      for (; v + 3 * 64 < nv; v += 4 * 64) {
        const u32x4p x0 = s[v], x1 = s[v + 64], x2 = s[v + 128], x3 = s[v + 192];
        d[v] = x0;
        d[v + 64] = x1;
        d[v + 128] = x2;
        d[v + 192] = x3;
      }
      for (; v < nv; v += 64) d[v] = s[v];
      for (uint64_t b = (nv << 4) + lane; b < bytes; b += 64) dst[b] = src[b];
    } else {
      for (uint64_t b = lane; b < bytes; b += 64) dst[b] = src[b];
    }
  }
}

// evict=false overflow: drop every entry this batch claimed (before any slot was assigned).
__global__ __launch_bounds__(256) void page_put_revert_kernel(PagePutArgs a) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
    const uint32_t tidx = a.tidx[i];
    if (tidx == 0xFFFFFFFFu) continue;
    if (a.tag[tidx] != ((a.batch << 32) | (unsigned long long)(i + 1))) continue;
    if (a.table[tidx].slot >= 0) continue;     // an existing page: untouched
    __hip_atomic_store(&a.table[tidx].key, kPageKeyTomb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    atomicAdd(&a.ctr->ntomb, 1u);
  }
}

static unsigned grid_for(uint32_t n) { return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 4096)); }

hipError_t launch_page_put_probe(const PagePutArgs& a, hipStream_t stream) {
  if (a.n == 0) return hipSuccess;
  if ((a.mask & (a.mask + 1)) != 0 || a.nslots == 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(page_put_probe_kernel, dim3(grid_for(a.n)), dim3(256), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_page_put_assign(const PagePutArgs& a, hipStream_t stream) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(page_put_assign_kernel, dim3(grid_for(a.n)), dim3(256), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_page_put_fill(const PagePutArgs& a, hipStream_t stream) {
  if (a.n == 0 || a.len == 0) return hipSuccess;
  if (a.len > a.page_size) return hipErrorInvalidValue;
  const uint32_t nch = (uint32_t)((a.len + kPutChunk - 1) / kPutChunk);
  const uint64_t waves = (uint64_t)a.n * nch;
  const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((waves + 3) / 4, 16384));
  const bool vec = ((uint64_t)a.src % 16 == 0) && (a.src_stride % 16 == 0) && ((uint64_t)a.arena % 16 == 0) &&
                   (a.page_size % 16 == 0);
  if (vec) hipLaunchKernelGGL((page_put_fill_kernel<true>), dim3(grid), dim3(256), 0, stream, a, nch);
  else hipLaunchKernelGGL((page_put_fill_kernel<false>), dim3(grid), dim3(256), 0, stream, a, nch);
  return hipGetLastError();
}

hipError_t launch_page_put_threshold(const PagePutArgs& a, hipStream_t stream) {
  hipError_t e = hipMemsetAsync(a.hist, 0, kPutAgeBuckets * sizeof(uint32_t), stream);
  if (e != hipSuccess) return e;
  const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((a.nslots + 1023) / 1024, 512));
  hipLaunchKernelGGL(page_put_hist_kernel, dim3(grid), dim3(256), 0, stream, a);
  hipLaunchKernelGGL(page_put_thresh_kernel, dim3(1), dim3(256), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_page_table_rebuild(const PagePutArgs& a, PageTableEntry* fresh, hipStream_t stream) {
  const uint64_t size = a.mask + 1;
  const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((size + 255) / 256, 8192));
  hipLaunchKernelGGL(page_table_clear_kernel, dim3(grid), dim3(256), 0, stream, fresh, size);
  hipLaunchKernelGGL(page_table_reinsert_kernel, dim3(grid), dim3(256), 0, stream, a, fresh);
  return hipGetLastError();
}

hipError_t launch_page_put_revert(const PagePutArgs& a, hipStream_t stream) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(page_put_revert_kernel, dim3(grid_for(a.n)), dim3(256), 0, stream, a);
  return hipGetLastError();
}

}  // namespace amdx
