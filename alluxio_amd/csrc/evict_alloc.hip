// K4-K7 on the device: slot-resident LRU/LRFU annotations, multi-workgroup byte-weighted eviction
// select, and the batched bitmap page allocator (gfx950, wave64).
//
// Reference loops these replace:
//   K4/K5 LRU / LRFU ordering   core/server/worker/.../block/annotator/LRFUAnnotator.java:81-95
//                               (CRF = CRF * (1/att)^(step * age) + 1 on every access)
//   K6    free-space loop       core/server/worker/.../block/TieredBlockStore.java:740-815
//                               (walk the annotator order until enough bytes are freed)
//   K7    allocation            core/server/worker/.../block/allocator/MaxFreeAllocator.java:42-110
//
// Design (see block_store.cpp "device annotator"): the annotation arrays live in HBM, indexed by
// block slot, and are only *updated* from the host through SlotUpdate batches (one per dirty slot
// per flush, carrying the host mirror's values; the kernel can also fold an access in place, the
// LRFU decay being multiplicative).  A selection
// never uploads candidate arrays: keys are computed on the fly from the resident arrays, filtered
// by target dir and a small exclusion bitmap (locked blocks), then a 4-pass MSB-first radix select
// over byte-weighted histograms runs across the whole grid: every workgroup builds an LDS
// histogram, adds it to the global one, and the last workgroup to finish a pass (threadfence +
// arrival counter) scans it and fixes the next digit -- no host round trip between passes.  The
// compaction writes victim slots straight to pinned host memory with one atomic per wave.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

#include <algorithm>

namespace amdx {

namespace {

constexpr int kEvBlock = 256;
// The passes are latency- and atomic-bound, not bandwidth-bound (150k keys = 600 KB).  Measured
// on MI355X at 150k keys (profiles/r2_evict_bench.md): 256 workgroups adding their LDS histograms
// to the global one with atomics = 20.6 us/pass; a plain-store slab summed by the last workgroup
// = 27 us (64 rows) / 38 us (256 rows); 128 workgroups with 4-deep unrolled key loads + atomics
// is the default.
constexpr unsigned kEvMaxGrid = kEvSlabRows;

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

__device__ __forceinline__ uint32_t evict_key(const EvictState& st, uint32_t i, uint64_t dir_mask,
                                              const uint32_t* __restrict__ excl) {
  const int32_t d = st.dir[i];
  if (d < 0 || d >= 64 || !((dir_mask >> d) & 1ull)) return 0xFFFFFFFFu;
  if (excl && ((excl[i >> 5] >> (i & 31)) & 1u)) return 0xFFFFFFFFu;
  const uint64_t last = st.last[i];
  const uint64_t age = st.now > last ? st.now - last : 0;
  uint32_t key;
  if (st.policy == 0) {
    key = 0xFFFFFFFEu - (uint32_t)(age < 0xFFFFFFFEull ? age : 0xFFFFFFFEull);
  } else {
    float crf = st.crf[i] * exp2f(st.log2_inv_att * st.step * (float)age);
    if (!(crf >= 0.0f)) crf = 0.0f;
    key = __float_as_uint(crf);   // non-negative floats order like their bits
  }
  if (key >= 0xFFFFFFFEu) key = 0xFFFFFFFDu;
  return st.invert ? 0xFFFFFFFDu - key : key;   // hottest-first selects the largest keys
}

__device__ __forceinline__ unsigned long long weight(const uint64_t* __restrict__ fbytes, uint32_t i, int unit) {
  return unit ? 1ull : (unsigned long long)fbytes[i];
}

// ---- annotation updates ----------------------------------------------------------------------
__global__ __launch_bounds__(kEvBlock) void slot_update_kernel(EvictState st, const SlotUpdate* __restrict__ u,
                                                                uint32_t n) {
  for (uint32_t j = blockIdx.x * kEvBlock + threadIdx.x; j < n; j += gridDim.x * kEvBlock) {
    const SlotUpdate x = u[j];
    const uint32_t s = x.slot;
    if (x.flags & kSlotSetState) {
      st.dir[s] = x.dir;
      st.fbytes[s] = x.fbytes;
    }
    if (x.flags & kSlotReset) {
      st.crf[s] = x.crf;
      st.last[s] = x.t;
    } else if (x.flags & kSlotTouch) {
      const uint64_t last = st.last[s];
      const uint64_t age = x.t > last ? x.t - last : 0;
      st.crf[s] = st.crf[s] * exp2f(st.log2_inv_att * st.step * (float)age) + x.crf;
      st.last[s] = x.t;
    }
  }
}

// ---- selection ---------------------------------------------------------------------------------
__global__ __launch_bounds__(kEvBlock) void ev_keys_kernel(EvictState st, uint64_t dir_mask,
                                                            const uint32_t* __restrict__ excl,
                                                            uint32_t* __restrict__ keys, EvictCtl* ctl) {
  __shared__ unsigned long long s_tot[kEvBlock / 64];
  unsigned long long tot = 0;
  for (uint32_t i = blockIdx.x * kEvBlock + threadIdx.x; i < st.n; i += gridDim.x * kEvBlock) {
    const uint32_t k = evict_key(st, i, dir_mask, excl);
    keys[i] = k;
    if (k != 0xFFFFFFFFu) tot += weight(st.fbytes, i, st.unit);
  }
  tot = wave_sum_u64(tot);
  if (lane_id() == 0) s_tot[threadIdx.x >> 6] = tot;
  __syncthreads();
  if (threadIdx.x == 0) {   // one global atomic per workgroup
    unsigned long long t = 0;
    for (int w = 0; w < kEvBlock / 64; ++w) t += s_tot[w];
    if (t) atomicAdd(&ctl->total, t);
  }
}

__global__ __launch_bounds__(kEvBlock) void ev_hist_kernel(const uint32_t* __restrict__ keys,
                                                            const uint64_t* __restrict__ fbytes, uint32_t n,
                                                            uint64_t need, int pass, EvictCtl* ctl, int unit) {
  __shared__ unsigned long long h[256];
  __shared__ unsigned long long scan[256];
  __shared__ int s_last;
  const int tid = threadIdx.x;
  // pass 0 decides whether everything must go (no select needed)
  if (pass == 0 && ctl->total <= need) {
    if (blockIdx.x == 0 && tid == 0) {
      ctl->all = 1;
      ctl->prefix = 0xFFFFFFFFu;
      ctl->mask = 0xFFFFFFFFu;
    }
    return;
  }
  if (ctl->all) return;
  const int shift = 24 - 8 * pass;
  const uint32_t prefix = ctl->prefix, mask = ctl->mask;
  h[tid] = 0;
  __syncthreads();
  // whole waves iterate together (the uniform-digit fast path needs every lane in the ballot);
  // four keys per lane per round, loads issued before any use
  const uint32_t stride = gridDim.x * kEvBlock;
  const uint32_t rounds = (n + 4 * stride - 1) / (4 * stride);
  for (uint32_t r = 0; r < rounds; ++r) {
    uint32_t kk[4];
    unsigned long long bb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t i = (r * 4 + u) * stride + blockIdx.x * kEvBlock + tid;
      kk[u] = i < n ? keys[i] : 0xFFFFFFFFu;
      bb[u] = i < n ? weight(fbytes, i, unit) : 0ull;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t k = kk[u];
      const bool valid = k != 0xFFFFFFFFu && (k & mask) == prefix;
      const uint32_t dig = (k >> shift) & 255u;
      const unsigned long long vb = valid ? bb[u] : 0ull;
      const unsigned long long vm = __ballot(valid);
      if (!vm) continue;
      // skewed passes (LRU clocks share their high bytes) put a whole wave on one digit: one
      // wave-reduced LDS atomic instead of 64 serialized ones on the same bin
      const uint32_t lead = (uint32_t)__shfl(dig, __builtin_ctzll(vm), 64);
      if (__ballot(valid && dig == lead) == vm) {
        const unsigned long long sum = wave_sum_u64(vb);
        if (lane_id() == 0) atomicAdd(&h[lead], sum);
      } else if (valid) {
        atomicAdd(&h[dig], vb);
      }
    }
  }
  __syncthreads();
  if (h[tid]) atomicAdd(&ctl->hist[tid], h[tid]);
  __threadfence();
  __syncthreads();
  if (tid == 0) s_last = atomicAdd(&ctl->done, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  // last workgroup of the pass: inclusive scan of the global histogram, pick the digit
  __threadfence();
  const unsigned long long v = __hip_atomic_load(&ctl->hist[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  scan[tid] = v;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const unsigned long long add = tid >= o ? scan[tid - o] : 0ull;
    __syncthreads();
    scan[tid] += add;
    __syncthreads();
  }
  const unsigned long long acc = ctl->acc;
  const unsigned long long incl = acc + scan[tid];
  const unsigned long long excl_b = incl - v;
  const bool hit = incl >= need && excl_b < need;
  __shared__ int s_d;
  if (tid == 0) s_d = 255;
  __syncthreads();
  if (hit) s_d = tid;   // exactly one thread (scan is monotone)
  __syncthreads();
  if (tid == 0) {
    const int d = s_d;
    ctl->acc = acc + (d > 0 ? scan[d - 1] : 0ull);
    ctl->prefix = prefix | ((uint32_t)d << shift);
    ctl->mask = mask | (255u << shift);
    ctl->done = 0;
  }
  ctl->hist[tid] = 0;
}

__global__ __launch_bounds__(kEvBlock) void ev_compact_kernel(const uint32_t* __restrict__ keys,
                                                               const uint64_t* __restrict__ fbytes, uint32_t n,
                                                               uint64_t need, EvictCtl* ctl,
                                                               uint32_t* __restrict__ out, int unit) {
  __shared__ uint32_t s_cnt[kEvBlock / 64];
  __shared__ uint32_t s_base;
  __shared__ unsigned long long s_freed[kEvBlock / 64];
  const uint32_t T = ctl->prefix;
  const bool all = ctl->all != 0;
  const unsigned long long below = ctl->acc;
  const uint32_t wave = threadIdx.x >> 6;
  unsigned long long freed = 0;
  // every lane of a wave walks the same number of iterations (ballots need the whole wave)
  const uint32_t stride = gridDim.x * kEvBlock;
  const uint32_t iters = (n + stride - 1) / stride;
  for (uint32_t it = 0; it < iters; ++it) {
    const uint32_t i = it * stride + blockIdx.x * kEvBlock + threadIdx.x;
    bool take = false;
    uint64_t b = 0;
    if (i < n) {
      const uint32_t k = keys[i];
      if (k != 0xFFFFFFFFu) {
        b = weight(fbytes, i, unit);
        take = all || k < T;
        if (!take && k == T) {
          const unsigned long long prev = atomicAdd(&ctl->tie_acc, (unsigned long long)b);
          take = below + prev < need;
        }
      }
    }
    const unsigned long long m = __ballot(take);
    if (lane_id() == 0) s_cnt[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {   // one output reservation per workgroup and iteration
      uint32_t t = 0;
      for (int w = 0; w < kEvBlock / 64; ++w) {
        const uint32_t c = s_cnt[w];
        s_cnt[w] = t;
        t += c;
      }
      s_base = t ? atomicAdd(&ctl->count, t) : 0u;
    }
    __syncthreads();
    if (take) {
      out[s_base + s_cnt[wave] + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull))] = i;
      freed += b;
    }
    __syncthreads();
  }
  freed = wave_sum_u64(freed);
  if (lane_id() == 0) s_freed[wave] = freed;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < kEvBlock / 64; ++w) t += s_freed[w];
    if (t) atomicAdd(&ctl->freed, t);
  }
}

// ---- K7 page allocation -------------------------------------------------------------------------
// Claim the `want` lowest-numbered free pages of a bitmap (1 = free): per-workgroup popcount,
// then each workgroup ranks its words (block scan + sum of the preceding workgroups' counts) and
// claims the free bits whose global rank < want.
constexpr int kPaBlock = 256;

__global__ __launch_bounds__(kPaBlock) void palloc_count_kernel(const uint64_t* __restrict__ bits,
                                                                  uint32_t nwords, uint32_t* __restrict__ partial) {
  const uint32_t w = blockIdx.x * kPaBlock + threadIdx.x;
  unsigned long long c = w < nwords ? (unsigned long long)__popcll(bits[w]) : 0ull;
  c = wave_sum_u64(c);
  __shared__ uint32_t s[kPaBlock / 64];
  if (lane_id() == 0) s[threadIdx.x >> 6] = (uint32_t)c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int i = 0; i < kPaBlock / 64; ++i) t += s[i];
    partial[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kPaBlock) void palloc_emit_kernel(uint64_t* __restrict__ bits, uint32_t nwords,
                                                                 const uint32_t* __restrict__ partial,
                                                                 uint32_t want, int64_t* __restrict__ pages_out,
                                                                 uint32_t* __restrict__ claimed) {
  __shared__ uint32_t s_wave[kPaBlock / 64];
  __shared__ uint32_t s_base;
  const uint32_t tid = threadIdx.x;
  // base = free pages in the preceding workgroups
  uint32_t pre = 0;
  for (uint32_t j = tid; j < blockIdx.x; j += kPaBlock) pre += partial[j];
  pre = (uint32_t)wave_sum_u64(pre);
  if (lane_id() == 0) s_wave[tid >> 6] = pre;
  __syncthreads();
  if (tid == 0) {
    uint32_t t = 0;
    for (int i = 0; i < kPaBlock / 64; ++i) t += s_wave[i];
    s_base = t;
  }
  __syncthreads();
  const uint32_t base = s_base;
  if (base >= want) return;
  const uint32_t w = blockIdx.x * kPaBlock + tid;
  const uint64_t word = w < nwords ? bits[w] : 0ull;
  const uint32_t c = (uint32_t)__popcll(word);
  // exclusive scan of c across the workgroup: wave scan + wave totals
  uint32_t incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(incl, o, 64);
    if ((int)lane_id() >= o) incl += v;
  }
  __syncthreads();
  if (lane_id() == 63) s_wave[tid >> 6] = incl;
  __syncthreads();
  uint32_t wave_off = 0;
  for (uint32_t i = 0; i < (tid >> 6); ++i) wave_off += s_wave[i];
  uint32_t rank = base + wave_off + incl - c;
  if (!c || rank >= want) return;
  uint64_t rest = word, taken = 0;
  while (rest && rank < want) {
    const int b = __builtin_ctzll(rest);
    rest &= rest - 1;
    taken |= 1ull << b;
    pages_out[rank++] = (int64_t)w * 64 + b;
  }
  bits[w] = word & ~taken;
  atomicAdd(claimed, (uint32_t)__popcll(taken));
}

// ---- K7 device page magazine ---------------------------------------------------------------------
__global__ __launch_bounds__(256) void mag_fill_kernel(uint64_t* __restrict__ bits, uint32_t nwords,
                                                       const uint64_t* __restrict__ upd, uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint64_t w = upd[2 * i];
    if (w < nwords) atomicOr((unsigned long long*)&bits[w], (unsigned long long)upd[2 * i + 1]);
  }
}

__global__ __launch_bounds__(256) void mag_drain_kernel(uint64_t* __restrict__ bits, uint32_t nwords,
                                                        uint64_t* __restrict__ out) {
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += gridDim.x * blockDim.x)
    out[w] = atomicExch((unsigned long long*)&bits[w], 0ull);
}

// lowest k set bits of x
__device__ __forceinline__ uint64_t low_bits(uint64_t x, uint32_t k) {
  uint64_t m = 0;
  for (uint32_t j = 0; j < k && x; ++j) {
    const uint64_t b = x & (~x + 1ull);
    m |= b;
    x ^= b;
  }
  return m;
}

// One wave per item: windows of 64 words (one per lane) starting at a per-item offset (spreads
// concurrent items over the bitmap); each lane takes up to its share of the item's remaining
// need from its word with one atomicAnd and keeps the bits it actually won.
__global__ __launch_bounds__(64) void mag_claim_kernel(uint64_t* __restrict__ bits, uint32_t nwords,
                                                       const ClaimItem* __restrict__ items, uint32_t nitems,
                                                       int64_t* __restrict__ pages_out, uint32_t pages_cap,
                                                       uint32_t* __restrict__ got, uint32_t win_lo, uint32_t win_len) {
  // one wave per workgroup and item: the window's free counts, the planned takes and the won
  // counts go through LDS, thread 0 plans and ranks serially (64 entries), barriers order the
  // phases -- no cross-lane shuffles in the plan
  __shared__ uint32_t s_cnt[64];
  __shared__ uint32_t s_take[64];
  __shared__ uint32_t s_have, s_seen;
  const uint32_t lane = threadIdx.x;
  for (uint32_t it = blockIdx.x; it < nitems; it += gridDim.x) {
    const ClaimItem item = items[it];
    const uint32_t hash = (uint32_t)((uint64_t)it * 0x9E3779B1u);
    const uint32_t rot = (uint32_t)((it * 37u) & 63u);      // items start at different bits of a word
    // the magazine's arc first (refills fill words contiguously from a cursor), then, if that
    // runs dry, the whole bitmap (bits a short claim or a racing group left elsewhere)
    bool full = win_len == 0 || win_len >= nwords;
    uint32_t lo = full ? 0u : win_lo % nwords, len = full ? nwords : win_len;
    uint32_t start = hash % len;
    const uint32_t max_rounds = 2 * (64 * ((nwords + 63) / 64) + 64);
    if (lane == 0) s_have = 0;
    __syncthreads();
    uint32_t dry = 0;
    // windows walk the range round and round: a wave that lost a race retries with a fresh
    // snapshot until it has its pages or one whole pass found no free bit (magazine dry)
    for (uint32_t win = 0, rounds = 0; rounds < max_rounds; ++rounds) {
      const uint32_t have = s_have;
      if (have >= item.want) break;
      if (dry >= len) {
        if (full) break;
        full = true;
        lo = 0;
        len = nwords;
        start = hash % len;
        win = 0;
        dry = 0;
      }
      const uint32_t span = len < 64 ? len : 64;            // distinct words per window
      const uint32_t w = (uint32_t)(((uint64_t)lo + ((uint64_t)start + win + lane) % len) % nwords);
      win += span;
      const bool valid = lane < span;
      const uint64_t word = valid ? __hip_atomic_load(&bits[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
      s_cnt[lane] = (uint32_t)__popcll(word);
      __syncthreads();
      if (lane == 0) {
        uint32_t left = item.want - have, seen = 0;
        for (uint32_t l = 0; l < 64; ++l) {
          const uint32_t f = s_cnt[l];
          const uint32_t t = f < left ? f : left;
          s_take[l] = t;
          left -= t;
          seen += f;
        }
        s_seen = seen;
      }
      __syncthreads();
      const uint32_t take = s_take[lane];
      dry = s_seen ? 0u : dry + span;
      uint64_t won = 0;
      if (take) {
        // compare-and-swap on the word: the bits are ours only if the word still holds what we
        // planned against; on a lost race re-plan against the value we got back (bounded)
        uint64_t cur = word;
        for (int tries = 0; tries < 64 && cur; ++tries) {
          const uint32_t n = (uint32_t)__popcll(cur) < take ? (uint32_t)__popcll(cur) : take;
          const uint64_t r = rot ? ((cur >> rot) | (cur << (64 - rot))) : cur;
          const uint64_t mr = low_bits(r, n);
          const uint64_t mask = rot ? ((mr << rot) | (mr >> (64 - rot))) : mr;
          const unsigned long long prev = atomicCAS((unsigned long long*)&bits[w], (unsigned long long)cur,
                                                    (unsigned long long)(cur & ~mask));
          if (prev == (unsigned long long)cur) {
            won = mask;
            break;
          }
          cur = prev;
        }
      }
      __syncthreads();                                   // everyone has read s_take
      s_cnt[lane] = (uint32_t)__popcll(won);
      __syncthreads();
      if (lane == 0) {                                   // exclusive ranks of the won pages
        uint32_t acc = have;
        for (uint32_t l = 0; l < 64; ++l) {
          const uint32_t c = s_cnt[l];
          s_take[l] = acc;
          acc += c;
        }
        s_have = acc;
      }
      __syncthreads();
      uint32_t pos = item.page_base + s_take[lane];
      for (uint64_t r = won; r; r &= r - 1, ++pos)
        if (pos < pages_cap && pos < item.page_base + item.want) pages_out[pos] = (int64_t)w * 64 + __builtin_ctzll(r);
      __syncthreads();                                   // s_take / s_have stable until all used them
    }
    if (lane == 0) got[it] = s_have;
    __syncthreads();
  }
}

constexpr uint64_t kMagChunk = 64 * 1024;

// One wave per 64 KiB chunk: item found by binary search over chunk_base.
__global__ __launch_bounds__(256) void mag_scatter_kernel(const ClaimItem* __restrict__ items, uint32_t nitems,
                                                          uint32_t total_chunks, const int64_t* __restrict__ pages,
                                                          const uint32_t* __restrict__ got, uint8_t* __restrict__ arena,
                                                          uint64_t page_size) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const uint32_t lane = lane_id();
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  for (uint32_t c = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); c < total_chunks; c += nw) {
    uint32_t lo = 0, hi = nitems;                  // last item with chunk_base <= c
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (items[mid].chunk_base <= c) lo = mid; else hi = mid;
    }
    const ClaimItem item = items[lo];
    if (got[lo] < item.want || item.src == 0) continue;
    const uint64_t off = (uint64_t)(c - item.chunk_base) * kMagChunk;
    if (off >= item.len) continue;
    const uint64_t end = min(item.len, off + kMagChunk);
    for (uint64_t pos = off; pos < end;) {         // a chunk may straddle a page boundary
      const uint64_t pi = pos / page_size, po = pos % page_size;
      const uint64_t n = min(end - pos, page_size - po);
      const uint8_t* src = reinterpret_cast<const uint8_t*>(item.src) + pos;
      uint8_t* dst = arena + (uint64_t)pages[item.page_base + pi] * page_size + po;
      if ((((uint64_t)src | (uint64_t)dst | n) & 15) == 0) {
        const u32x4* s4 = reinterpret_cast<const u32x4*>(src);
        u32x4* d4 = reinterpret_cast<u32x4*>(dst);
        for (uint64_t v = lane; v < (n >> 4); v += 64) d4[v] = s4[v];
      } else {
        for (uint64_t b = lane; b < n; b += 64) dst[b] = src[b];
      }
      pos += n;
    }
  }
}

}  // namespace

hipError_t launch_mag_fill(uint64_t* bits, uint32_t nwords, const uint64_t* upd, uint32_t n, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const unsigned grid = (unsigned)std::min<uint32_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(mag_fill_kernel, dim3(grid), dim3(256), 0, stream, bits, nwords, upd, n);
  return hipGetLastError();
}

hipError_t launch_mag_drain(uint64_t* bits, uint32_t nwords, uint64_t* out, hipStream_t stream) {
  if (nwords == 0) return hipSuccess;
  const unsigned grid = (unsigned)std::min<uint32_t>((nwords + 255) / 256, 1024);
  hipLaunchKernelGGL(mag_drain_kernel, dim3(grid), dim3(256), 0, stream, bits, nwords, out);
  return hipGetLastError();
}

hipError_t launch_mag_claim_scatter(uint64_t* bits, uint32_t nwords, const ClaimItem* items, uint32_t nitems,
                                    int64_t* pages_out, uint32_t pages_cap, uint32_t* got, uint32_t total_chunks,
                                    uint8_t* arena, uint64_t page_size, hipStream_t stream, uint32_t win_lo,
                                    uint32_t win_len) {
  if (nitems == 0 || nwords == 0) return hipSuccess;
  const unsigned cgrid = (unsigned)std::min<uint32_t>(nitems, 16384);
  hipLaunchKernelGGL(mag_claim_kernel, dim3(cgrid), dim3(64), 0, stream, bits, nwords, items, nitems, pages_out,
                     pages_cap, got, win_lo, win_len);
  if (total_chunks) {
    const unsigned sgrid = (unsigned)std::min<uint32_t>((total_chunks + 3) / 4, 16384);
    hipLaunchKernelGGL(mag_scatter_kernel, dim3(sgrid), dim3(256), 0, stream, items, nitems, total_chunks, pages_out,
                       got, arena, page_size);
  }
  return hipGetLastError();
}

hipError_t launch_slot_update(const EvictState& st, const SlotUpdate* upd, uint32_t n, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const unsigned grid = (unsigned)((n + kEvBlock - 1) / kEvBlock < 1024 ? (n + kEvBlock - 1) / kEvBlock : 1024);
  hipLaunchKernelGGL(slot_update_kernel, dim3(grid), dim3(kEvBlock), 0, stream, st, upd, n);
  return hipGetLastError();
}

hipError_t launch_evict_select_grid(const EvictState& st, uint32_t target_dir, const uint32_t* excl,
                                    uint64_t need, uint32_t* keys, EvictCtl* ctl, uint32_t* out_slots,
                                    hipStream_t stream) {
  hipError_t e = hipMemsetAsync(ctl, 0, sizeof(EvictCtl), stream);
  if (e != hipSuccess) return e;
  if (st.n == 0) return hipSuccess;
  // >= 1k keys per workgroup (four per thread), at most kEvMaxGrid workgroups
  unsigned grid = (st.n + 1023) / 1024;
  if (grid > kEvMaxGrid) grid = kEvMaxGrid;
  const uint64_t mask = st.dir_mask ? st.dir_mask : (1ull << (target_dir & 63));
  hipLaunchKernelGGL(ev_keys_kernel, dim3(grid), dim3(kEvBlock), 0, stream, st, mask, excl, keys, ctl);
  for (int pass = 0; pass < 4; ++pass)
    hipLaunchKernelGGL(ev_hist_kernel, dim3(grid), dim3(kEvBlock), 0, stream, keys, st.fbytes, st.n, need, pass,
                       ctl, st.unit);
  hipLaunchKernelGGL(ev_compact_kernel, dim3(grid), dim3(kEvBlock), 0, stream, keys, st.fbytes, st.n, need, ctl,
                     out_slots, st.unit);
  return hipGetLastError();
}

hipError_t launch_page_alloc(uint64_t* bits, uint32_t nwords, uint32_t want, uint32_t* partial,
                             int64_t* pages_out, uint32_t* claimed, hipStream_t stream) {
  hipError_t e = hipMemsetAsync(claimed, 0, sizeof(uint32_t), stream);
  if (e != hipSuccess || nwords == 0 || want == 0) return e;
  const unsigned grid = (nwords + kPaBlock - 1) / kPaBlock;
  hipLaunchKernelGGL(palloc_count_kernel, dim3(grid), dim3(kPaBlock), 0, stream, bits, nwords, partial);
  hipLaunchKernelGGL(palloc_emit_kernel, dim3(grid), dim3(kPaBlock), 0, stream, bits, nwords, partial, want,
                     pages_out, claimed);
  return hipGetLastError();
}

uint32_t page_alloc_partials(uint32_t nwords) { return (nwords + kPaBlock - 1) / kPaBlock; }

}  // namespace amdx
