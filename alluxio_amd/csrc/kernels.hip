// CDNA4 (gfx950) kernels for the HBM block store.  Wave64 throughout; all grids grid-stride
// and are capped so a launch always drains.  See kernels.h for the reference hot loops each
// kernel replaces.
#include "kernels.h"

#include <algorithm>
#include <cstring>
#include <mutex>

namespace amdx {

// ---------------------------------------------------------------------------------------------
// K1/K2: batched gather/scatter copy.
//
// The host planner splits every read/write request into page-contiguous segments (a request
// never spans a page boundary inside a segment) and computes an exclusive prefix of
// ceil(bytes / kCopyChunk) per segment.  Each workgroup iteration owns one <=256 KiB chunk: a
// wave-uniform binary search (scalar loads) finds its segment, then 256 lanes stream the chunk
// with 16-B loads, 8 in flight per lane (128 B/lane, 32 KiB per workgroup round).
// ---------------------------------------------------------------------------------------------
constexpr int kCopyThreads = 256;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Load/store cache policies (A/B-able at run time, see set_copy_variant):
//   0 = default, 1 = nontemporal (``nt``: stream past the caches).
template <int P>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
  if constexpr (P == 1) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int P>
__device__ __forceinline__ void st16(u32x4* p, u32x4 v) {
  if constexpr (P == 1) __builtin_nontemporal_store(v, p);
  else *p = v;
}

__device__ __forceinline__ void copy_bytes(const uint8_t* __restrict__ s, uint8_t* __restrict__ d,
                                           uint64_t n, int tid) {
  for (uint64_t i = tid; i < n; i += kCopyThreads) d[i] = s[i];
}

template <int UNROLL, int LP, int SP>
__device__ __forceinline__ void copy_range(uint64_t src, uint64_t dst, uint64_t n, int tid) {
  if (((src | dst) & 15) == 0) {
    const u32x4* __restrict__ s = reinterpret_cast<const u32x4*>(src);
    u32x4* __restrict__ d = reinterpret_cast<u32x4*>(dst);
    const uint64_t n16 = n >> 4;
    uint64_t i = tid;
    constexpr uint64_t kStep = (uint64_t)kCopyThreads * UNROLL;
    for (; i + (UNROLL - 1) * kCopyThreads < n16; i += kStep) {
      u32x4 v[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) v[u] = ld16<LP>(s + i + (uint64_t)u * kCopyThreads);
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) st16<SP>(d + i + (uint64_t)u * kCopyThreads, v[u]);
    }
    for (; i < n16; i += kCopyThreads) st16<SP>(d + i, ld16<LP>(s + i));
    const uint64_t done = n16 << 4;
    if (done < n) copy_bytes(reinterpret_cast<const uint8_t*>(src) + done,
                             reinterpret_cast<uint8_t*>(dst) + done, n - done, tid);
  } else if (((src | dst) & 3) == 0) {
    const uint32_t* __restrict__ s = reinterpret_cast<const uint32_t*>(src);
    uint32_t* __restrict__ d = reinterpret_cast<uint32_t*>(dst);
    const uint64_t n4 = n >> 2;
    for (uint64_t i = tid; i < n4; i += kCopyThreads) d[i] = s[i];
    const uint64_t done = n4 << 2;
    if (done < n) copy_bytes(reinterpret_cast<const uint8_t*>(src) + done,
                             reinterpret_cast<uint8_t*>(dst) + done, n - done, tid);
  } else {
    copy_bytes(reinterpret_cast<const uint8_t*>(src), reinterpret_cast<uint8_t*>(dst), n, tid);
  }
}

template <int UNROLL, int LP, int SP>
__global__ __launch_bounds__(kCopyThreads) void batched_copy_kernel(
    const CopySeg* __restrict__ segs, int nseg, uint64_t total_chunks) {
  const int tid = threadIdx.x;
  for (uint64_t c = blockIdx.x; c < total_chunks; c += gridDim.x) {
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (segs[mid].chunk0 <= c) lo = mid; else hi = mid - 1;
    }
    lo = __builtin_amdgcn_readfirstlane(lo);
    const uint64_t src = segs[lo].src, dst = segs[lo].dst, bytes = segs[lo].bytes;
    const uint64_t off = (c - segs[lo].chunk0) * kCopyChunk;
    const uint64_t n = bytes - off < kCopyChunk ? bytes - off : kCopyChunk;
    copy_range<UNROLL, LP, SP>(src + off, dst + off, n, tid);
  }
}

// variant = unroll_sel * 4 + load_policy * 2 + store_policy; unroll_sel: 0 -> 8, 1 -> 4, 2 -> 16
// Default from tools/copy_tune.py on MI355X (profiles/r1_copy_tune.jsonl): 16-deep unroll,
// cached loads+stores, grid cap 4096 won the bench shape (5.42 TB/s vs 5.24 for 8-deep/2048).
static int g_copy_variant = 8;
static unsigned g_copy_grid_cap = 4096;

void set_copy_variant(int variant, unsigned grid_cap) {
  g_copy_variant = variant;
  if (grid_cap) g_copy_grid_cap = grid_cap;
}

hipError_t launch_batched_copy(const CopySeg* segs, int nseg, uint64_t total_chunks,
                               hipStream_t stream) {
  if (nseg <= 0 || total_chunks == 0) return hipSuccess;
  // 256 CUs x 8 resident 256-thread workgroups; more chunks are grid-strided.
  const dim3 grid((unsigned)std::min<uint64_t>(total_chunks, g_copy_grid_cap));
  const dim3 block(kCopyThreads);
#define AMDX_COPY(U, L, S) hipLaunchKernelGGL((batched_copy_kernel<U, L, S>), grid, block, 0, stream, segs, nseg, total_chunks)
  switch (g_copy_variant) {
    case 1: AMDX_COPY(8, 0, 1); break;
    case 2: AMDX_COPY(8, 1, 0); break;
    case 3: AMDX_COPY(8, 1, 1); break;
    case 4: AMDX_COPY(4, 0, 0); break;
    case 5: AMDX_COPY(4, 0, 1); break;
    case 8: AMDX_COPY(16, 0, 0); break;
    case 9: AMDX_COPY(16, 0, 1); break;
    default: AMDX_COPY(8, 0, 0); break;
  }
#undef AMDX_COPY
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K1': device-cursor multi-stream sequential read (see SeqReadArgs in kernels.h).
//
// The flattened index space is (stream, call k, 16-B vector v).  Each workgroup first computes
// every stream's first call index of this launch (c0[s] = (c_init[s] + launch_base) % cycle) into
// LDS — one 64-bit modulo per stream instead of per vector — then grid-strides over vectors with
// 8 independent 16-B loads in flight per lane before the stores (latency hiding for the
// short, page-table-indirected reads).  Consecutive lanes touch consecutive vectors of the same
// read, so both the arena gather and the ring store coalesce.  A read whose length is not a
// multiple of 16 (the last read of a pass) finishes its tail bytes in the owning lane.
// ---------------------------------------------------------------------------------------------
constexpr int kSeqThreads = 256;

// POW2: vectors-per-read and depth are powers of two -> index math is shifts/masks (the common
// case: 4 KiB reads x 256 calls); otherwise 64-bit division.  SP: store policy of the ring
// writes (1 = nontemporal: the ring is written once and consumed elsewhere, so keep the file's
// pages, not the ring, resident in L2/MALL).
template <bool POW2, int UNROLL, int SP, int LP>
__global__ __launch_bounds__(kSeqThreads) void seq_read_kernel(SeqReadArgs a, uint32_t vpr_shift,
                                                               uint32_t depth_shift) {
  extern __shared__ uint32_t c0[];  // streams entries (dynamic LDS: 1 KiB for 256 streams)
  for (uint32_t s = threadIdx.x; s < a.streams; s += kSeqThreads)
    c0[s] = (uint32_t)((a.c_init[s] + a.launch_base) % a.cycle);
  __syncthreads();
  const uint64_t vpr = a.buf >> 4;  // vectors per read slot (buf % 16 == 0)
  const uint64_t nvec = (uint64_t)a.streams * a.depth * vpr;
  const uint64_t pmask = (1ull << a.page_shift) - 1;
  const uint64_t gstride = (uint64_t)gridDim.x * kSeqThreads;
  for (uint64_t base = (uint64_t)blockIdx.x * kSeqThreads + threadIdx.x; base < nvec;
       base += gstride * UNROLL) {
    u32x4 v[UNROLL];
    uint8_t* d[UNROLL];
    uint32_t nb[UNROLL];  // bytes this lane moves for vector u (16, tail, or 0)
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint64_t i = base + (uint64_t)u * gstride;
      nb[u] = 0;
      d[u] = nullptr;
      if (i >= nvec) continue;
      uint64_t r, vi;
      uint32_t s, k;
      if constexpr (POW2) {
        r = i >> vpr_shift;
        vi = i & (vpr - 1);
        s = (uint32_t)(r >> depth_shift);
        k = (uint32_t)(r & (a.depth - 1));
      } else {
        r = i / vpr;
        vi = i - r * vpr;
        s = (uint32_t)(r / a.depth);
        k = (uint32_t)(r - (uint64_t)s * a.depth);
      }
      uint32_t c = c0[s] + k;
      if (c >= a.cycle) c = (uint32_t)(((uint64_t)c0[s] + k) % a.cycle);
      if (c == a.cycle - 1) continue;                    // EOF call: reopen, no bytes
      const uint64_t off = (uint64_t)c * a.buf + vi * 16;
      const uint64_t rend = ((uint64_t)c + 1) * a.buf;
      const uint64_t end = rend < a.file_len ? rend : a.file_len;
      if (off >= end) continue;
      const uint64_t page = (uint64_t)a.ftab[off >> a.page_shift];
      const uint8_t* src = a.arena + (page << a.page_shift) + (off & pmask);
      d[u] = a.dst + (uint64_t)s * a.stream_stride + (uint64_t)k * a.buf + vi * 16;
      if (end - off >= 16) {
        nb[u] = 16;
        v[u] = ld16<LP>(reinterpret_cast<const u32x4*>(src));
      } else {
        nb[u] = (uint32_t)(end - off);
        // tail of the pass: byte-wise, may cross into the next page
        for (uint32_t b = 0; b < nb[u]; ++b) {
          const uint64_t o = off + b;
          d[u][b] = a.arena[((uint64_t)a.ftab[o >> a.page_shift] << a.page_shift) + (o & pmask)];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
      if (nb[u] == 16) st16<SP>(reinterpret_cast<u32x4*>(d[u]), v[u]);
  }
}

// 0: cached stores, 1: nontemporal stores, +2: unroll 16, +4: nontemporal loads; -1 (default): auto —
// nontemporal LOADS once a launch streams >= 128 MiB of distinct file bytes (half the 256 MB MALL):
// those bytes are read once, so streaming them past L2/MALL leaves the caches to the ring writes
// (16 GiB staggered read: 2.40 -> 2.87 TB/s delivered = 5.7 TB/s of HBM traffic, above the
// runtime's own D2D copy at 2.46 TB/s; staggered 128 MiB: 2.85 -> 2.98 TB/s;
// profiles/r3_ring_tune_large_ntload.json, r3_ring_tune_128m_ntload.jsonl, r3_copy_roof.json);
// cached loads while the streams re-read one window (the lockstep headline shape: 5.9 vs 2.8 TB/s)
static int g_seq_variant = -1;
static unsigned g_seq_grid_cap = 8192;

void set_seq_read_variant(int variant, unsigned grid_cap) {
  g_seq_variant = variant;
  if (grid_cap) g_seq_grid_cap = grid_cap;
}

static inline bool is_pow2(uint64_t x) { return x && !(x & (x - 1)); }
static inline uint32_t log2u(uint64_t x) {
  uint32_t s = 0;
  while ((1ull << s) < x) ++s;
  return s;
}

hipError_t launch_seq_read(const SeqReadArgs& a, hipStream_t stream) {
  if (a.streams == 0 || a.depth == 0 || a.buf == 0 || a.file_len == 0) return hipSuccess;
  if (a.streams > kSeqReadMaxStreams || (a.buf & 15) || (a.stream_stride & 15) ||
      ((uint64_t)a.dst & 15) || ((uint64_t)a.arena & 15))
    return hipErrorInvalidValue;
  const uint64_t vpr = a.buf >> 4;
  const uint64_t nvec = (uint64_t)a.streams * a.depth * vpr;
  const uint64_t fp = a.footprint ? a.footprint : a.file_len;
  const int var = g_seq_variant >= 0 ? g_seq_variant : (fp >= (128ull << 20) ? 4 : 0);
  const int unroll = (var & 2) ? 16 : 8;
  uint64_t blocks = (nvec + (uint64_t)kSeqThreads * unroll - 1) / ((uint64_t)kSeqThreads * unroll);
  if (blocks > g_seq_grid_cap) blocks = g_seq_grid_cap;
  if (blocks < 1) blocks = 1;
  const bool p2 = is_pow2(vpr) && is_pow2(a.depth);
  const uint32_t vs = log2u(vpr), ds = log2u(a.depth);
  const size_t lds = a.streams * sizeof(uint32_t);
  const dim3 g((unsigned)blocks), b(kSeqThreads);
#define AMDX_SEQ(P2, U, SP, LP) \
  hipLaunchKernelGGL((seq_read_kernel<P2, U, SP, LP>), g, b, lds, stream, a, vs, ds)
  const int sp = var & 1, lp = (var >> 2) & 1;
  if (p2) {
    if (unroll == 16) {
      if (lp) { if (sp) AMDX_SEQ(true, 16, 1, 1); else AMDX_SEQ(true, 16, 0, 1); }
      else { if (sp) AMDX_SEQ(true, 16, 1, 0); else AMDX_SEQ(true, 16, 0, 0); }
    } else {
      if (lp) { if (sp) AMDX_SEQ(true, 8, 1, 1); else AMDX_SEQ(true, 8, 0, 1); }
      else { if (sp) AMDX_SEQ(true, 8, 1, 0); else AMDX_SEQ(true, 8, 0, 0); }
    }
  } else {
    if (lp) { if (sp) AMDX_SEQ(false, 8, 1, 1); else AMDX_SEQ(false, 8, 0, 1); }
    else { if (sp) AMDX_SEQ(false, 8, 1, 0); else AMDX_SEQ(false, 8, 0, 0); }
  }
#undef AMDX_SEQ
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K10: CRC32C.  Phase 1: one workgroup per 64 KiB segment; each lane runs slicing-by-8 over its
// own 256 B with the 8 KiB table resident in LDS, then the 256 lane CRCs are folded with a
// log-depth GF(2) "shift" combine (x^(8L) mod P multipliers).  Phase 2: one workgroup per piece
// folds its segment CRCs (variable-length right operands) and applies init/xorout.
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kCrcPoly = 0x82F63B78u;  // reflected Castagnoli
constexpr uint64_t kCrcSeg = 64 * 1024;
constexpr int kCrcThreads = 256;
constexpr uint64_t kCrcLane = kCrcSeg / kCrcThreads;  // 256 B per lane

__constant__ uint32_t c_crc_tab[8][256];
__constant__ uint32_t c_x2n[64];  // x^(2^k) mod P, k = 0..63
__constant__ uint32_t c_crc16[16][256];   // slicing-by-16 (zero-init CRC of a 16-byte word)
__constant__ uint32_t c_shift4k[4][256];  // c -> c * x^(8*4096) mod P, byte-sliced
__constant__ uint32_t c_lane_shift[256];  // x^(128*k) mod P: moves a lane's CRC k 16-B words right
// v4 (11-bit slicing): chunk c of a 16-B word = bits [11c, 11c+11) -> its share of the word's CRC
constexpr int kCrc4Threads = 1024;
__constant__ uint32_t c_crc11[12][2048];
__constant__ uint32_t c_shift16k[4][256];          // c -> c * x^(8*16384), byte-sliced
__constant__ uint32_t c_lane_shift1k[kCrc4Threads];  // x^(128*k), k < 1024
// v5 (conflict-free replicated slicing-by-4): a lane's 64-B chunks are 64 KiB apart
constexpr int kCrc5Threads = 1024;
constexpr uint64_t kCrc5Chunk = 64;
__constant__ uint32_t c_shift5[4][256];                // c -> c * x^(8*(1024-1)*64), byte-sliced
__constant__ uint32_t c_lane_shift5[kCrc5Threads];     // x^(8*64*d), d < 1024

static void host_crc_tables(uint32_t tab[8][256], uint32_t x2n[64]) {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kCrcPoly : c >> 1;
    tab[0][i] = c;
  }
  for (int t = 1; t < 8; ++t)
    for (uint32_t i = 0; i < 256; ++i) tab[t][i] = (tab[t - 1][i] >> 8) ^ tab[0][tab[t - 1][i] & 0xFF];
  // x^1 in reflected representation is 0x40000000; square repeatedly.
  auto mult = [](uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
      if (a & m) { p ^= b; if ((a & (m - 1)) == 0) break; }
      m >>= 1;
      b = (b & 1) ? (b >> 1) ^ kCrcPoly : b >> 1;
    }
    return p;
  };
  uint32_t p = 1u << 30;
  x2n[0] = p;
  for (int k = 1; k < 64; ++k) { p = mult(p, p); x2n[k] = p; }
}

static uint32_t host_gf2_mult(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (uint32_t m = 1u << 31; m; m >>= 1) {
    if (a & m) p ^= b;
    b = (b & 1) ? (b >> 1) ^ kCrcPoly : b >> 1;
  }
  return p;
}

static void host_crc16_tables(const uint32_t tab8[8][256], const uint32_t x2n[64], uint32_t t16[16][256],
                              uint32_t sh[4][256]) {
  for (uint32_t i = 0; i < 256; ++i) t16[0][i] = tab8[0][i];
  for (int t = 1; t < 16; ++t)
    for (uint32_t i = 0; i < 256; ++i) t16[t][i] = (t16[t - 1][i] >> 8) ^ t16[0][t16[t - 1][i] & 0xFF];
  // x^(8*4096) = x^(2^15)
  const uint32_t k = x2n[15];
  for (int b = 0; b < 4; ++b)
    for (uint32_t i = 0; i < 256; ++i) sh[b][i] = host_gf2_mult(k, i << (8 * b));
}

static std::once_flag g_crc_once;
static hipError_t g_crc_init_err = hipSuccess;

static hipError_t ensure_crc_tables() {
  std::call_once(g_crc_once, [] {
    static uint32_t tab[8][256];
    static uint32_t x2n[64];
    host_crc_tables(tab, x2n);
    static uint32_t t16[16][256];
    static uint32_t sh[4][256];
    host_crc16_tables(tab, x2n, t16, sh);
    g_crc_init_err = hipMemcpyToSymbol(HIP_SYMBOL(c_crc_tab), tab, sizeof(tab));
    if (g_crc_init_err == hipSuccess)
      g_crc_init_err = hipMemcpyToSymbol(HIP_SYMBOL(c_x2n), x2n, sizeof(x2n));
    if (g_crc_init_err == hipSuccess)
      g_crc_init_err = hipMemcpyToSymbol(HIP_SYMBOL(c_crc16), t16, sizeof(t16));
    if (g_crc_init_err == hipSuccess)
      g_crc_init_err = hipMemcpyToSymbol(HIP_SYMBOL(c_shift4k), sh, sizeof(sh));
    // v4 tables: E[k] = CRC share of bit k of a 16-B word (byte j uses t16[15 - j])
    static uint32_t t11[12][2048];
    uint32_t e[128];
    for (int k = 0; k < 128; ++k) e[k] = t16[15 - k / 8][1u << (k % 8)];
    for (int c = 0; c < 12; ++c)
      for (uint32_t v = 0; v < 2048; ++v) {
        uint32_t x = 0;
        for (int b = 0; b < 11; ++b)
          if (((v >> b) & 1) && 11 * c + b < 128) x ^= e[11 * c + b];
        t11[c][v] = x;
      }
    static uint32_t sh16k[4][256];
    for (int b = 0; b < 4; ++b)
      for (uint32_t i = 0; i < 256; ++i) sh16k[b][i] = host_gf2_mult(x2n[17], i << (8 * b));
    static uint32_t lane1k[kCrc4Threads];
    lane1k[0] = 1u << 31;
    for (int k = 1; k < kCrc4Threads; ++k) lane1k[k] = host_gf2_mult(lane1k[k - 1], x2n[7]);
    if (g_crc_init_err == hipSuccess)
      g_crc_init_err = hipMemcpyToSymbol(HIP_SYMBOL(c_crc11), t11, sizeof(t11));
    if (g_crc_init_err == hipSuccess)
      g_crc_init_err = hipMemcpyToSymbol(HIP_SYMBOL(c_shift16k), sh16k, sizeof(sh16k));
    if (g_crc_init_err == hipSuccess)
      g_crc_init_err = hipMemcpyToSymbol(HIP_SYMBOL(c_lane_shift1k), lane1k, sizeof(lane1k));
    {
      // v5: skip the other 1023 lanes' chunks = multiply by x^(8 * 1023 * 64)
      const uint64_t nbits = 8ull * (kCrc5Threads - 1) * kCrc5Chunk;
      uint32_t k5 = 1u << 31;
      for (int b = 0; b < 64; ++b)
        if ((nbits >> b) & 1) k5 = host_gf2_mult(x2n[b], k5);
      static uint32_t sh5[4][256];
      for (int b = 0; b < 4; ++b)
        for (uint32_t i = 0; i < 256; ++i) sh5[b][i] = host_gf2_mult(k5, i << (8 * b));
      static uint32_t lane5[kCrc5Threads];
      lane5[0] = 1u << 31;
      for (int d = 1; d < kCrc5Threads; ++d) lane5[d] = host_gf2_mult(lane5[d - 1], x2n[9]);   // * x^512
      if (g_crc_init_err == hipSuccess)
        g_crc_init_err = hipMemcpyToSymbol(HIP_SYMBOL(c_shift5), sh5, sizeof(sh5));
      if (g_crc_init_err == hipSuccess)
        g_crc_init_err = hipMemcpyToSymbol(HIP_SYMBOL(c_lane_shift5), lane5, sizeof(lane5));
    }
    static uint32_t lane_shift[256];
    lane_shift[0] = 1u << 31;  // x^0
    for (int k = 1; k < 256; ++k) lane_shift[k] = host_gf2_mult(lane_shift[k - 1], x2n[7]);  // * x^128
    if (g_crc_init_err == hipSuccess)
      g_crc_init_err = hipMemcpyToSymbol(HIP_SYMBOL(c_lane_shift), lane_shift, sizeof(lane_shift));
  });
  return g_crc_init_err;
}

__device__ __forceinline__ uint32_t gf2_mult(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (int i = 0; i < 32; ++i) {
    if (a & m) p ^= b;
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ kCrcPoly : b >> 1;
  }
  return p;
}

// x^(8*nbytes) mod P by square-and-multiply over the bits of 8*nbytes.
__device__ __forceinline__ uint32_t xpow8n(uint64_t nbytes) {
  uint64_t n = nbytes << 3;
  uint32_t p = 1u << 31;  // x^0
  int k = 0;
  while (n) {
    if (n & 1) p = gf2_mult(c_x2n[k & 63], p);
    n >>= 1;
    ++k;
  }
  return p;
}

__global__ __launch_bounds__(kCrcThreads) void crc32c_segments_kernel(
    const uint8_t* __restrict__ base, uint64_t total_bytes, uint64_t piece_bytes,
    uint64_t segs_per_piece, uint64_t nsegs, uint32_t* __restrict__ seg_crc) {
  __shared__ uint32_t tab[8][256];
  __shared__ uint32_t part[kCrcThreads];
  const int tid = threadIdx.x;
  for (int i = tid; i < 8 * 256; i += kCrcThreads) tab[i >> 8][i & 255] = c_crc_tab[i >> 8][i & 255];
  __syncthreads();
  const uint32_t k_lane = xpow8n(kCrcLane);  // shift by one lane's bytes (uniform)
  for (uint64_t g = blockIdx.x; g < nsegs; g += gridDim.x) {
    const uint64_t piece = g / segs_per_piece;
    const uint64_t seg_in_piece = g % segs_per_piece;
    const uint64_t piece_start = piece * piece_bytes;
    const uint64_t piece_len = std::min(piece_bytes, total_bytes - piece_start);
    const uint64_t seg_start = piece_start + seg_in_piece * kCrcSeg;
    const uint64_t seg_len = std::min(kCrcSeg, piece_start + piece_len - seg_start);
    // lane range inside the segment
    const uint64_t lo = std::min<uint64_t>((uint64_t)tid * kCrcLane, seg_len);
    const uint64_t hi = std::min<uint64_t>(lo + kCrcLane, seg_len);
    const uint8_t* p = base + seg_start + lo;
    uint32_t c = 0;
    uint64_t n = hi - lo;
    if ((((uintptr_t)p) & 15) == 0) {
      while (n >= 16) {
        const uint4 v = *reinterpret_cast<const uint4*>(p);
        uint32_t a = v.x ^ c, b = v.y;
        c = tab[7][a & 255] ^ tab[6][(a >> 8) & 255] ^ tab[5][(a >> 16) & 255] ^ tab[4][a >> 24] ^
            tab[3][b & 255] ^ tab[2][(b >> 8) & 255] ^ tab[1][(b >> 16) & 255] ^ tab[0][b >> 24];
        a = v.z ^ c;
        b = v.w;
        c = tab[7][a & 255] ^ tab[6][(a >> 8) & 255] ^ tab[5][(a >> 16) & 255] ^ tab[4][a >> 24] ^
            tab[3][b & 255] ^ tab[2][(b >> 8) & 255] ^ tab[1][(b >> 16) & 255] ^ tab[0][b >> 24];
        p += 16;
        n -= 16;
      }
    }
    while (n--) c = (c >> 8) ^ tab[0][(c ^ *p++) & 255];
    part[tid] = c;
    __syncthreads();
    // Fold lane CRCs: level s merges (t, t+s); right operand length = bytes of lanes [t+s, t+2s).
    for (int s = 1; s < kCrcThreads; s <<= 1) {
      if ((tid & (2 * s - 1)) == 0 && tid + s < kCrcThreads) {
        const uint64_t r_lo = std::min<uint64_t>((uint64_t)(tid + s) * kCrcLane, seg_len);
        const uint64_t r_hi = std::min<uint64_t>((uint64_t)(tid + 2 * s) * kCrcLane, seg_len);
        const uint64_t rlen = r_hi - r_lo;
        if (rlen) {
          const uint32_t k = (rlen == (uint64_t)s * kCrcLane && s == 1) ? k_lane : xpow8n(rlen);
          part[tid] = gf2_mult(k, part[tid]) ^ part[tid + s];
        }
      }
      __syncthreads();
    }
    if (tid == 0) seg_crc[g] = part[0];
    __syncthreads();
  }
}

// v2: interleaved lanes.  Lane l reads 16-B words l, l+256, l+512, ... of the segment (a wave
// reads 1 KiB contiguous per instruction: fully coalesced), keeping c_l = sum_k crc16(w_k) *
// x^(8*4096*(K-1-k)) via c = shift4k(c) ^ crc16(w) (4 + 16 LDS lookups per 16 B, no dependency
// on other lanes).  At the end each lane's contribution is moved to its final position with one
// multiply by x^(8*bytes-after-its-last-word) and the block XOR-reduces; the <16-B tail is folded
// in by lane 0.  Produces the same raw (zero-init) segment CRC as v1.
constexpr uint64_t kCrcSeg2 = 256 * 1024;

// One segment's raw CRC with the v2 schedule; the result is valid in thread 0.
__device__ __forceinline__ uint32_t seg_crc_v2(const uint8_t* __restrict__ seg, uint64_t seg_len,
                                               const uint32_t (*t16)[256], const uint32_t (*sh)[256],
                                               uint32_t* part, int tid) {
  const uint64_t nwords = seg_len >> 4;
  uint32_t c = 0;
  uint64_t last = ~0ull;
  if ((((uintptr_t)seg) & 15) == 0) {
    for (uint64_t wi = tid; wi < nwords; wi += kCrcThreads) {
      const uint4 v = *reinterpret_cast<const uint4*>(seg + (wi << 4));
      const uint32_t s = sh[0][c & 255] ^ sh[1][(c >> 8) & 255] ^ sh[2][(c >> 16) & 255] ^ sh[3][c >> 24];
      const uint32_t w = t16[15][v.x & 255] ^ t16[14][(v.x >> 8) & 255] ^ t16[13][(v.x >> 16) & 255] ^
                         t16[12][v.x >> 24] ^ t16[11][v.y & 255] ^ t16[10][(v.y >> 8) & 255] ^
                         t16[9][(v.y >> 16) & 255] ^ t16[8][v.y >> 24] ^ t16[7][v.z & 255] ^
                         t16[6][(v.z >> 8) & 255] ^ t16[5][(v.z >> 16) & 255] ^ t16[4][v.z >> 24] ^
                         t16[3][v.w & 255] ^ t16[2][(v.w >> 8) & 255] ^ t16[1][(v.w >> 16) & 255] ^
                         t16[0][v.w >> 24];
      c = (wi < (uint64_t)kCrcThreads ? 0u : s) ^ w;
      last = wi;
    }
  } else {
    // unaligned segment: same schedule with byte loads
    for (uint64_t wi = tid; wi < nwords; wi += kCrcThreads) {
      const uint8_t* q = seg + (wi << 4);
      uint32_t w = 0;
#pragma unroll
      for (int b = 0; b < 16; ++b) w ^= t16[15 - b][q[b]];
      const uint32_t s = sh[0][c & 255] ^ sh[1][(c >> 8) & 255] ^ sh[2][(c >> 16) & 255] ^ sh[3][c >> 24];
      c = (wi < (uint64_t)kCrcThreads ? 0u : s) ^ w;
      last = wi;
    }
  }
  // move the lane's contribution to its position: bytes after its last word inside the words area
  uint32_t contrib = 0;
  if (last != ~0ull) contrib = gf2_mult(xpow8n((nwords - 1 - last) << 4), c);
  part[tid] = contrib;
  __syncthreads();
  for (int s2 = kCrcThreads / 2; s2 > 0; s2 >>= 1) {
    if (tid < s2) part[tid] ^= part[tid + s2];
    __syncthreads();
  }
  uint32_t acc = 0;
  if (tid == 0) {
    acc = part[0];
    const uint64_t tail = seg_len & 15;
    if (tail) {
      acc = gf2_mult(xpow8n(tail), acc);
      uint32_t t = 0;
      const uint8_t* q = seg + (nwords << 4);
      for (uint64_t b = 0; b < tail; ++b) t = (t >> 8) ^ t16[0][(t ^ q[b]) & 255];
      acc ^= t;
    }
  }
  __syncthreads();
  return acc;
}

__global__ __launch_bounds__(kCrcThreads) void crc32c_segments_v2_kernel(
    const uint8_t* __restrict__ base, uint64_t total_bytes, uint64_t piece_bytes, uint64_t seg_bytes,
    uint64_t segs_per_piece, uint64_t nsegs, uint32_t* __restrict__ seg_crc) {
  __shared__ uint32_t t16[16][256];
  __shared__ uint32_t sh[4][256];
  __shared__ uint32_t part[kCrcThreads];
  const int tid = threadIdx.x;
  for (int i = tid; i < 16 * 256; i += kCrcThreads) t16[i >> 8][i & 255] = c_crc16[i >> 8][i & 255];
  for (int i = tid; i < 4 * 256; i += kCrcThreads) sh[i >> 8][i & 255] = c_shift4k[i >> 8][i & 255];
  __syncthreads();
  for (uint64_t g = blockIdx.x; g < nsegs; g += gridDim.x) {
    const uint64_t piece = g / segs_per_piece;
    const uint64_t seg_in_piece = g % segs_per_piece;
    const uint64_t piece_start = piece * piece_bytes;
    const uint64_t piece_len = std::min(piece_bytes, total_bytes - piece_start);
    const uint64_t seg_start = piece_start + seg_in_piece * seg_bytes;
    const uint64_t seg_len = std::min(seg_bytes, piece_start + piece_len - seg_start);
    const uint32_t acc = seg_crc_v2(base + seg_start, seg_len, t16, sh, part, tid);
    if (tid == 0) seg_crc[g] = acc;
  }
}

// v3: the v2 schedule with the per-lane "move to final position" done by one multiply with a
// precomputed x^(128*k) (k < 256 words: a lane's last word is always within the final stride)
// instead of a square-and-multiply xpow8n per lane per segment -- that fold cost ~1/4 of the
// VALU work of a 256 KiB segment.  Same raw (zero-init) segment CRC as v1/v2.
__device__ __forceinline__ uint32_t seg_crc_v3(const uint8_t* __restrict__ seg, uint64_t seg_len,
                                               const uint32_t (*t16)[256], const uint32_t (*sh)[256],
                                               const uint32_t* lane_shift, uint32_t* part, int tid) {
  const uint64_t nwords = seg_len >> 4;
  uint32_t c = 0;
  uint64_t last = ~0ull;
  if ((((uintptr_t)seg) & 15) == 0) {
    uint64_t wi = tid;
    if (wi < nwords) {  // first word: nothing to shift yet
      const uint4 v = *reinterpret_cast<const uint4*>(seg + (wi << 4));
      c = t16[15][v.x & 255] ^ t16[14][(v.x >> 8) & 255] ^ t16[13][(v.x >> 16) & 255] ^ t16[12][v.x >> 24] ^
          t16[11][v.y & 255] ^ t16[10][(v.y >> 8) & 255] ^ t16[9][(v.y >> 16) & 255] ^ t16[8][v.y >> 24] ^
          t16[7][v.z & 255] ^ t16[6][(v.z >> 8) & 255] ^ t16[5][(v.z >> 16) & 255] ^ t16[4][v.z >> 24] ^
          t16[3][v.w & 255] ^ t16[2][(v.w >> 8) & 255] ^ t16[1][(v.w >> 16) & 255] ^ t16[0][v.w >> 24];
      last = wi;
      wi += kCrcThreads;
    }
    for (; wi + 3 * kCrcThreads < nwords; wi += 4 * kCrcThreads) {
      uint4 vv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) vv[u] = *reinterpret_cast<const uint4*>(seg + ((wi + u * kCrcThreads) << 4));
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint4 v = vv[u];
        const uint32_t s = sh[0][c & 255] ^ sh[1][(c >> 8) & 255] ^ sh[2][(c >> 16) & 255] ^ sh[3][c >> 24];
        c = s ^ t16[15][v.x & 255] ^ t16[14][(v.x >> 8) & 255] ^ t16[13][(v.x >> 16) & 255] ^ t16[12][v.x >> 24] ^
            t16[11][v.y & 255] ^ t16[10][(v.y >> 8) & 255] ^ t16[9][(v.y >> 16) & 255] ^ t16[8][v.y >> 24] ^
            t16[7][v.z & 255] ^ t16[6][(v.z >> 8) & 255] ^ t16[5][(v.z >> 16) & 255] ^ t16[4][v.z >> 24] ^
            t16[3][v.w & 255] ^ t16[2][(v.w >> 8) & 255] ^ t16[1][(v.w >> 16) & 255] ^ t16[0][v.w >> 24];
      }
      last = wi + 3 * kCrcThreads;
    }
    for (; wi < nwords; wi += kCrcThreads) {
      const uint4 v = *reinterpret_cast<const uint4*>(seg + (wi << 4));
      const uint32_t s = sh[0][c & 255] ^ sh[1][(c >> 8) & 255] ^ sh[2][(c >> 16) & 255] ^ sh[3][c >> 24];
      c = s ^ t16[15][v.x & 255] ^ t16[14][(v.x >> 8) & 255] ^ t16[13][(v.x >> 16) & 255] ^ t16[12][v.x >> 24] ^
          t16[11][v.y & 255] ^ t16[10][(v.y >> 8) & 255] ^ t16[9][(v.y >> 16) & 255] ^ t16[8][v.y >> 24] ^
          t16[7][v.z & 255] ^ t16[6][(v.z >> 8) & 255] ^ t16[5][(v.z >> 16) & 255] ^ t16[4][v.z >> 24] ^
          t16[3][v.w & 255] ^ t16[2][(v.w >> 8) & 255] ^ t16[1][(v.w >> 16) & 255] ^ t16[0][v.w >> 24];
      last = wi;
    }
  } else {
    for (uint64_t wi = tid; wi < nwords; wi += kCrcThreads) {
      const uint8_t* q = seg + (wi << 4);
      uint32_t w = 0;
#pragma unroll
      for (int b = 0; b < 16; ++b) w ^= t16[15 - b][q[b]];
      const uint32_t s = sh[0][c & 255] ^ sh[1][(c >> 8) & 255] ^ sh[2][(c >> 16) & 255] ^ sh[3][c >> 24];
      c = (wi < (uint64_t)kCrcThreads ? 0u : s) ^ w;
      last = wi;
    }
  }
  uint32_t contrib = 0;
  if (last != ~0ull) contrib = gf2_mult(lane_shift[nwords - 1 - last], c);  // nwords-1-last < kCrcThreads
  part[tid] = contrib;
  __syncthreads();
  for (int s2 = kCrcThreads / 2; s2 > 0; s2 >>= 1) {
    if (tid < s2) part[tid] ^= part[tid + s2];
    __syncthreads();
  }
  uint32_t acc = 0;
  if (tid == 0) {
    acc = part[0];
    const uint64_t tail = seg_len & 15;
    if (tail) {
      acc = gf2_mult(xpow8n(tail), acc);
      uint32_t t = 0;
      const uint8_t* q = seg + (nwords << 4);
      for (uint64_t b = 0; b < tail; ++b) t = (t >> 8) ^ t16[0][(t ^ q[b]) & 255];
      acc ^= t;
    }
  }
  __syncthreads();
  return acc;
}

static_assert(kCrcThreads <= 256, "lane shift table covers 256 words");

__global__ __launch_bounds__(kCrcThreads) void crc32c_segments_v3_kernel(
    const uint8_t* __restrict__ base, uint64_t total_bytes, uint64_t piece_bytes, uint64_t seg_bytes,
    uint64_t segs_per_piece, uint64_t nsegs, uint32_t* __restrict__ seg_crc) {
  __shared__ uint32_t t16[16][256];
  __shared__ uint32_t sh[4][256];
  __shared__ uint32_t lsh[kCrcThreads];
  __shared__ uint32_t part[kCrcThreads];
  const int tid = threadIdx.x;
  for (int i = tid; i < 16 * 256; i += kCrcThreads) t16[i >> 8][i & 255] = c_crc16[i >> 8][i & 255];
  for (int i = tid; i < 4 * 256; i += kCrcThreads) sh[i >> 8][i & 255] = c_shift4k[i >> 8][i & 255];
  lsh[tid] = c_lane_shift[tid];
  __syncthreads();
  for (uint64_t g = blockIdx.x; g < nsegs; g += gridDim.x) {
    const uint64_t piece = g / segs_per_piece;
    const uint64_t seg_in_piece = g % segs_per_piece;
    const uint64_t piece_start = piece * piece_bytes;
    const uint64_t piece_len = std::min(piece_bytes, total_bytes - piece_start);
    const uint64_t seg_start = piece_start + seg_in_piece * seg_bytes;
    const uint64_t seg_len = std::min(seg_bytes, piece_start + piece_len - seg_start);
    const uint32_t acc = seg_crc_v3(base + seg_start, seg_len, t16, sh, lsh, part, tid);
    if (tid == 0) seg_crc[g] = acc;
  }
}

// v4: 11-bit slicing.  A 16-B word is 12 chunks of <= 11 bits; 12 lookups in 2048-entry tables
// (96 KiB of LDS) replace the 16 byte-table lookups, and the running CRC shift is 4 lookups per
// word as before: 16 LDS reads per 16 B instead of 20 (the kernel is bound by bank-conflicted LDS
// reads).  1024-thread workgroups (16 waves share one table copy per CU), a lane's words are 16 KiB
// apart (one wave reads 1 KiB contiguous), 1 MiB segments, grid sized to the CU count.
constexpr uint64_t kCrcSeg4 = 1024 * 1024;
constexpr int kCrc4Batch = 4;

__device__ __forceinline__ uint32_t crc11_word(const uint4 v, const uint32_t (*t)[2048]) {
  const uint64_t lo = (uint64_t)v.x | ((uint64_t)v.y << 32);
  const uint64_t hi = (uint64_t)v.z | ((uint64_t)v.w << 32);
  return t[0][lo & 2047] ^ t[1][(lo >> 11) & 2047] ^ t[2][(lo >> 22) & 2047] ^ t[3][(lo >> 33) & 2047] ^
         t[4][(lo >> 44) & 2047] ^ t[5][((lo >> 55) | (hi << 9)) & 2047] ^ t[6][(hi >> 2) & 2047] ^
         t[7][(hi >> 13) & 2047] ^ t[8][(hi >> 24) & 2047] ^ t[9][(hi >> 35) & 2047] ^
         t[10][(hi >> 46) & 2047] ^ t[11][hi >> 57];
}

__global__ __launch_bounds__(kCrc4Threads) void crc32c_segments_v4_kernel(
    const uint8_t* __restrict__ base, uint64_t total_bytes, uint64_t piece_bytes, uint64_t seg_bytes,
    uint64_t segs_per_piece, uint64_t nsegs, uint32_t* __restrict__ seg_crc) {
  __shared__ uint32_t t11[12][2048];
  __shared__ uint32_t sh[4][256];
  __shared__ uint32_t lsh[kCrc4Threads];
  __shared__ uint32_t part[kCrc4Threads];
  const int tid = threadIdx.x;
  for (int i = tid; i < 12 * 2048; i += kCrc4Threads) t11[i >> 11][i & 2047] = c_crc11[i >> 11][i & 2047];
  for (int i = tid; i < 4 * 256; i += kCrc4Threads) sh[i >> 8][i & 255] = c_shift16k[i >> 8][i & 255];
  lsh[tid] = c_lane_shift1k[tid];
  __syncthreads();
  for (uint64_t g = blockIdx.x; g < nsegs; g += gridDim.x) {
    const uint64_t piece = g / segs_per_piece;
    const uint64_t seg_in_piece = g % segs_per_piece;
    const uint64_t piece_start = piece * piece_bytes;
    const uint64_t piece_len = std::min(piece_bytes, total_bytes - piece_start);
    const uint64_t seg_start = piece_start + seg_in_piece * seg_bytes;
    const uint64_t seg_len = std::min(seg_bytes, piece_start + piece_len - seg_start);
    const uint8_t* seg = base + seg_start;
    const uint64_t nwords = seg_len >> 4;
    uint32_t c = 0;
    uint64_t last = ~0ull;
    if ((((uintptr_t)seg) & 15) == 0) {
      uint64_t wi = tid;
      if (wi < nwords) {
        c = crc11_word(*reinterpret_cast<const uint4*>(seg + (wi << 4)), t11);
        last = wi;
        wi += kCrc4Threads;
      }
      // kCrc4Batch words in flight per lane (16 waves per CU only): issue the loads, then fold
      for (; wi + (kCrc4Batch - 1) * kCrc4Threads < nwords; wi += kCrc4Batch * kCrc4Threads) {
        uint4 v[kCrc4Batch];
#pragma unroll
        for (int u = 0; u < kCrc4Batch; ++u) v[u] = *reinterpret_cast<const uint4*>(seg + ((wi + u * kCrc4Threads) << 4));
#pragma unroll
        for (int u = 0; u < kCrc4Batch; ++u)
          c = sh[0][c & 255] ^ sh[1][(c >> 8) & 255] ^ sh[2][(c >> 16) & 255] ^ sh[3][c >> 24] ^ crc11_word(v[u], t11);
        last = wi + (kCrc4Batch - 1) * kCrc4Threads;
      }
      for (; wi < nwords; wi += kCrc4Threads) {
        const uint4 v = *reinterpret_cast<const uint4*>(seg + (wi << 4));
        c = sh[0][c & 255] ^ sh[1][(c >> 8) & 255] ^ sh[2][(c >> 16) & 255] ^ sh[3][c >> 24] ^ crc11_word(v, t11);
        last = wi;
      }
    } else {
      for (uint64_t wi = tid; wi < nwords; wi += kCrc4Threads) {
        const uint8_t* q = seg + (wi << 4);
        uint4 v;
        uint8_t* vb = reinterpret_cast<uint8_t*>(&v);
#pragma unroll
        for (int b = 0; b < 16; ++b) vb[b] = q[b];
        const uint32_t sft = sh[0][c & 255] ^ sh[1][(c >> 8) & 255] ^ sh[2][(c >> 16) & 255] ^ sh[3][c >> 24];
        c = (wi < (uint64_t)kCrc4Threads ? 0u : sft) ^ crc11_word(v, t11);
        last = wi;
      }
    }
    part[tid] = last != ~0ull ? gf2_mult(lsh[nwords - 1 - last], c) : 0u;
    __syncthreads();
    for (int s2 = kCrc4Threads / 2; s2 > 0; s2 >>= 1) {
      if (tid < s2) part[tid] ^= part[tid + s2];
      __syncthreads();
    }
    if (tid == 0) {
      uint32_t acc = part[0];
      const uint64_t tail = seg_len & 15;
      if (tail) {
        acc = gf2_mult(xpow8n(tail), acc);
        uint32_t t = 0;
        const uint8_t* q = seg + (nwords << 4);
        for (uint64_t b = 0; b < tail; ++b) t = (t >> 8) ^ c_crc16[0][(t ^ q[b]) & 255];
        acc ^= t;
      }
      seg_crc[g] = acc;
    }
    __syncthreads();
  }
}

// v5: slicing-by-4 over per-lane 64-B chunks with the byte tables replicated 32 times in LDS
// (entry x of table t, copy r at dword (t*256 + x)*32 + r; lane l reads copy l mod 32), so every
// ds_read_b32 of a wave hits 32 distinct banks per 32-lane group: the random-index bank conflicts
// that bound v1-v4 (4.7 extra cycles per LDS read, profiles/r2_crc_kernels.md) are gone.  Lane l
// owns chunks l, l+1024, ... of a 1 MiB segment (a wave reads 4 KiB contiguous per step); between
// two of its chunks the running CRC is shifted past the other lanes' bytes with 4 lookups in a
// small (unreplicated) table, so a chunk costs 64 + 4 lookups.  Lane results are moved to their
// final positions with one multiply by a precomputed x^(8*64*d) and XOR-reduced.  Produces the
// same raw (zero-init) segment CRC as v1-v4.
constexpr uint64_t kCrcSeg5 = 1024 * 1024;
constexpr uint64_t kCrcPagedSeg = 256 * 1024;

__device__ __forceinline__ uint32_t crc5_step(uint32_t x, const uint32_t* __restrict__ my) {
  return my[(3 * 256 + (x & 255)) * 32] ^ my[(2 * 256 + ((x >> 8) & 255)) * 32] ^
         my[(1 * 256 + ((x >> 16) & 255)) * 32] ^ my[(x >> 24) * 32];
}

__device__ __forceinline__ uint32_t crc5_chunk(uint32_t c, const uint4 v[4], const uint32_t* __restrict__ my) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    c = crc5_step(c ^ v[u].x, my);
    c = crc5_step(c ^ v[u].y, my);
    c = crc5_step(c ^ v[u].z, my);
    c = crc5_step(c ^ v[u].w, my);
  }
  return c;
}

// page_idx (optional): piece i lives at base + page_idx[i] * piece_bytes instead of base + i *
// piece_bytes -- the scattered pages of one arena block checksummed in one launch.
__global__ __launch_bounds__(kCrc5Threads) void crc32c_segments_v5_kernel(
    const uint8_t* __restrict__ base, uint64_t total_bytes, uint64_t piece_bytes, uint64_t seg_bytes,
    uint64_t segs_per_piece, uint64_t nsegs, uint32_t* __restrict__ seg_crc,
    const int64_t* __restrict__ page_idx) {
  __shared__ uint32_t t4r[4 * 256 * 32];   // 128 KiB
  __shared__ uint32_t sh[4][256];
  __shared__ uint32_t lsh[kCrc5Threads];
  __shared__ uint32_t part[kCrc5Threads];
  const int tid = threadIdx.x;
  for (int i = tid; i < 4 * 256 * 32; i += kCrc5Threads) t4r[i] = c_crc_tab[i >> 13][(i >> 5) & 255];
  for (int i = tid; i < 4 * 256; i += kCrc5Threads) sh[i >> 8][i & 255] = c_shift5[i >> 8][i & 255];
  lsh[tid] = c_lane_shift5[tid];
  __syncthreads();
  const uint32_t* my = t4r + (tid & 31);
  for (uint64_t g = blockIdx.x; g < nsegs; g += gridDim.x) {
    const uint64_t piece = g / segs_per_piece;
    const uint64_t seg_in_piece = g % segs_per_piece;
    const uint64_t piece_start = piece * piece_bytes;
    const uint64_t piece_len = std::min(piece_bytes, total_bytes - piece_start);
    const uint64_t seg_start = piece_start + seg_in_piece * seg_bytes;
    const uint64_t seg_len = std::min(seg_bytes, piece_start + piece_len - seg_start);
    const uint8_t* seg = page_idx ? base + (uint64_t)page_idx[piece] * piece_bytes + seg_in_piece * seg_bytes
                                  : base + seg_start;
    const uint64_t nch = seg_len / kCrc5Chunk;
    uint32_t c = 0;
    uint64_t last = ~0ull;
    if ((((uintptr_t)seg) & 15) == 0) {
      uint64_t k = tid;
      uint4 cur[4], nxt[4];
      if (k < nch) {
        const uint4* q = reinterpret_cast<const uint4*>(seg + k * kCrc5Chunk);
#pragma unroll
        for (int u = 0; u < 4; ++u) cur[u] = q[u];
      }
      for (; k < nch; k += kCrc5Threads) {
        const uint64_t kn = k + kCrc5Threads;
        if (kn < nch) {                              // next chunk's loads in flight meanwhile
          const uint4* q = reinterpret_cast<const uint4*>(seg + kn * kCrc5Chunk);
#pragma unroll
          for (int u = 0; u < 4; ++u) nxt[u] = q[u];
        }
        if (last != ~0ull) c = sh[0][c & 255] ^ sh[1][(c >> 8) & 255] ^ sh[2][(c >> 16) & 255] ^ sh[3][c >> 24];
        c = crc5_chunk(c, cur, my);
        last = k;
#pragma unroll
        for (int u = 0; u < 4; ++u) cur[u] = nxt[u];
      }
    } else {
      for (uint64_t k = tid; k < nch; k += kCrc5Threads) {
        uint4 v[4];
        uint8_t* vb = reinterpret_cast<uint8_t*>(v);
        const uint8_t* q = seg + k * kCrc5Chunk;
        for (int b = 0; b < 64; ++b) vb[b] = q[b];
        if (last != ~0ull) c = sh[0][c & 255] ^ sh[1][(c >> 8) & 255] ^ sh[2][(c >> 16) & 255] ^ sh[3][c >> 24];
        c = crc5_chunk(c, v, my);
        last = k;
      }
    }
    part[tid] = last != ~0ull ? gf2_mult(lsh[nch - 1 - last], c) : 0u;
    __syncthreads();
    for (int s2 = kCrc5Threads / 2; s2 > 0; s2 >>= 1) {
      if (tid < s2) part[tid] ^= part[tid + s2];
      __syncthreads();
    }
    if (tid == 0) {
      uint32_t acc = part[0];
      const uint64_t tail = seg_len - nch * kCrc5Chunk;
      if (tail) {
        acc = gf2_mult(xpow8n(tail), acc);
        uint32_t t = 0;
        const uint8_t* q = seg + nch * kCrc5Chunk;
        for (uint64_t b = 0; b < tail; ++b) t = (t >> 8) ^ my[((t ^ q[b]) & 255) * 32];
        acc ^= t;
      }
      seg_crc[g] = acc;
    }
    __syncthreads();
  }
}

// Gathered pieces (one page of many blocks each, <= kCrcSeg2 bytes): one workgroup per piece,
// standard CRC32C per piece — the per-page CRCs of a whole batch of freshly cached blocks in
// one launch instead of one launch + sync per block.
__global__ __launch_bounds__(kCrcThreads) void crc32c_gather_kernel(
    const uint64_t* __restrict__ ptrs, const uint32_t* __restrict__ lens, uint64_t n,
    uint32_t* __restrict__ out) {
  __shared__ uint32_t t16[16][256];
  __shared__ uint32_t sh[4][256];
  __shared__ uint32_t lsh[kCrcThreads];
  __shared__ uint32_t part[kCrcThreads];
  const int tid = threadIdx.x;
  for (int i = tid; i < 16 * 256; i += kCrcThreads) t16[i >> 8][i & 255] = c_crc16[i >> 8][i & 255];
  for (int i = tid; i < 4 * 256; i += kCrcThreads) sh[i >> 8][i & 255] = c_shift4k[i >> 8][i & 255];
  lsh[tid] = c_lane_shift[tid];
  __syncthreads();
  for (uint64_t g = blockIdx.x; g < n; g += gridDim.x) {
    const uint64_t len = lens[g];
    const uint32_t acc = seg_crc_v3(reinterpret_cast<const uint8_t*>(ptrs[g]), len, t16, sh, lsh, part, tid);
    if (tid == 0) out[g] = acc ^ gf2_mult(xpow8n(len), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
  }
}

hipError_t launch_crc32c_gather(const uint64_t* ptrs, const uint32_t* lens, uint64_t n, uint32_t* out,
                                hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipError_t e = ensure_crc_tables();
  if (e != hipSuccess) return e;
  const unsigned g = (unsigned)std::min<uint64_t>(n, 8192);
  hipLaunchKernelGGL(crc32c_gather_kernel, dim3(g), dim3(kCrcThreads), 0, stream, ptrs, lens, n, out);
  return hipGetLastError();
}

uint64_t crc32c_gather_max_piece() { return kCrcSeg2; }

__global__ __launch_bounds__(kCrcThreads) void crc32c_pieces_kernel(
    const uint32_t* __restrict__ seg_crc, uint64_t total_bytes, uint64_t piece_bytes, uint64_t seg_bytes,
    uint64_t segs_per_piece, uint64_t npieces, uint32_t* __restrict__ out) {
  __shared__ uint32_t part[kCrcThreads];
  __shared__ uint64_t plen[kCrcThreads];
  const int tid = threadIdx.x;
  for (uint64_t pc = blockIdx.x; pc < npieces; pc += gridDim.x) {
    const uint64_t piece_start = pc * piece_bytes;
    const uint64_t piece_len = std::min(piece_bytes, total_bytes - piece_start);
    const uint64_t nseg = (piece_len + seg_bytes - 1) / seg_bytes;
    const uint64_t per = (nseg + kCrcThreads - 1) / kCrcThreads;
    const uint64_t s0 = std::min<uint64_t>((uint64_t)tid * per, nseg);
    const uint64_t s1 = std::min<uint64_t>(s0 + per, nseg);
    uint32_t c = 0;
    uint64_t len = 0;
    for (uint64_t s = s0; s < s1; ++s) {
      const uint64_t sl = std::min(seg_bytes, piece_len - s * seg_bytes);
      c = gf2_mult(xpow8n(sl), c) ^ seg_crc[pc * segs_per_piece + s];
      len += sl;
    }
    part[tid] = c;
    plen[tid] = len;
    __syncthreads();
    for (int s = 1; s < kCrcThreads; s <<= 1) {
      if ((tid & (2 * s - 1)) == 0 && tid + s < kCrcThreads) {
        const uint64_t rlen = plen[tid + s];
        if (rlen) part[tid] = gf2_mult(xpow8n(rlen), part[tid]) ^ part[tid + s];
        plen[tid] += rlen;
      }
      __syncthreads();
    }
    if (tid == 0) {
      // standard CRC = raw ^ shift(0xFFFFFFFF, len) ^ 0xFFFFFFFF
      out[pc] = part[0] ^ gf2_mult(xpow8n(piece_len), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
    }
    __syncthreads();
  }
}

uint64_t crc32c_scratch_words(uint64_t total_bytes, uint64_t piece_bytes) {
  if (total_bytes == 0 || piece_bytes == 0) return 0;
  const uint64_t npieces = (total_bytes + piece_bytes - 1) / piece_bytes;
  const uint64_t spp = (piece_bytes + kCrcSeg - 1) / kCrcSeg;
  return npieces * spp;
}

static int g_crc_variant = 4;  // 0: per-lane contiguous strips (v1), 1: interleaved lanes (v2),
                               // 2: v2 + table lane fold (v3), 3: 11-bit slicing, 1024 threads (v4),
                               // 4: replicated conflict-free slicing-by-4 over 64-B chunks (v5)

void set_crc_variant(int v) { g_crc_variant = v; }

namespace {
// CUs of the current device (queried once per device, not per launch)
int cu_count() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int cus = 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    cache[dev] = cus;
  }
  return cache[dev];
}
}  // namespace

uint64_t crc32c_pages_scratch_words(uint64_t total_bytes, uint64_t page_bytes) {
  if (!total_bytes || !page_bytes) return 0;
  const uint64_t seg = std::min(kCrcPagedSeg, page_bytes);
  return ((total_bytes + page_bytes - 1) / page_bytes) * ((page_bytes + seg - 1) / seg);
}

hipError_t launch_crc32c_pages(const uint8_t* base, const int64_t* page_idx, uint64_t total_bytes,
                               uint64_t page_bytes, uint32_t* out, uint32_t* scratch, uint64_t scratch_words,
                               hipStream_t stream) {
  if (total_bytes == 0) return hipSuccess;
  if (g_crc_variant != 4) return hipErrorNotSupported;   // the paged form exists for v5 only
  hipError_t e = ensure_crc_tables();
  if (e != hipSuccess) return e;
  const uint64_t npieces = (total_bytes + page_bytes - 1) / page_bytes;
  // 256 KiB segments: a 64 MiB block of 2 MiB pages is 256 workgroups, one per CU (1 MiB segments
  // would leave three quarters of the CUs idle)
  const uint64_t seg = std::min(kCrcPagedSeg, page_bytes);
  const uint64_t spp = (page_bytes + seg - 1) / seg;
  const uint64_t nsegs = npieces * spp;
  if (scratch_words < nsegs) return hipErrorInvalidValue;
  const unsigned g4 = (unsigned)std::min<uint64_t>(nsegs, (uint64_t)cu_count());
  hipLaunchKernelGGL(crc32c_segments_v5_kernel, dim3(g4), dim3(kCrc5Threads), 0, stream, base, total_bytes,
                     page_bytes, seg, spp, nsegs, scratch, page_idx);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const unsigned g2 = (unsigned)std::min<uint64_t>(npieces, 4096);
  hipLaunchKernelGGL(crc32c_pieces_kernel, dim3(g2), dim3(kCrcThreads), 0, stream, scratch, total_bytes,
                     page_bytes, seg, spp, npieces, out);
  return hipGetLastError();
}

hipError_t launch_crc32c_pieces(const uint8_t* base, uint64_t total_bytes, uint64_t piece_bytes,
                                uint32_t* out, uint32_t* scratch, uint64_t scratch_words,
                                hipStream_t stream) {
  if (total_bytes == 0) return hipSuccess;
  hipError_t e = ensure_crc_tables();
  if (e != hipSuccess) return e;
  const uint64_t npieces = (total_bytes + piece_bytes - 1) / piece_bytes;
  const uint64_t seg = g_crc_variant == 0   ? kCrcSeg
                       : g_crc_variant == 3 ? std::min(kCrcSeg4, piece_bytes)
                       : g_crc_variant == 4 ? std::min(kCrcSeg5, piece_bytes)
                                            : kCrcSeg2;
  const uint64_t spp = (piece_bytes + seg - 1) / seg;
  const uint64_t nsegs = npieces * spp;
  if (scratch_words < nsegs) return hipErrorInvalidValue;
  const unsigned g1 = (unsigned)std::min<uint64_t>(nsegs, 8192);
  if (g_crc_variant == 0) {
    hipLaunchKernelGGL(crc32c_segments_kernel, dim3(g1), dim3(kCrcThreads), 0, stream, base,
                       total_bytes, piece_bytes, spp, nsegs, scratch);
  } else if (g_crc_variant == 1) {
    hipLaunchKernelGGL(crc32c_segments_v2_kernel, dim3(g1), dim3(kCrcThreads), 0, stream, base,
                       total_bytes, piece_bytes, seg, spp, nsegs, scratch);
  } else if (g_crc_variant == 2) {
    hipLaunchKernelGGL(crc32c_segments_v3_kernel, dim3(g1), dim3(kCrcThreads), 0, stream, base,
                       total_bytes, piece_bytes, seg, spp, nsegs, scratch);
  } else {
    const unsigned g4 = (unsigned)std::min<uint64_t>(nsegs, (uint64_t)cu_count());   // one >100 KiB-LDS WG per CU
    if (g_crc_variant == 4)
      hipLaunchKernelGGL(crc32c_segments_v5_kernel, dim3(g4), dim3(kCrc5Threads), 0, stream, base,
                         total_bytes, piece_bytes, seg, spp, nsegs, scratch, (const int64_t*)nullptr);
    else
      hipLaunchKernelGGL(crc32c_segments_v4_kernel, dim3(g4), dim3(kCrc4Threads), 0, stream, base,
                         total_bytes, piece_bytes, seg, spp, nsegs, scratch);
  }
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const unsigned g2 = (unsigned)std::min<uint64_t>(npieces, 4096);
  hipLaunchKernelGGL(crc32c_pieces_kernel, dim3(g2), dim3(kCrcThreads), 0, stream, scratch,
                     total_bytes, piece_bytes, seg, spp, npieces, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K11: LZ4 block-format codec, one 64-lane workgroup per <=64 KiB chunk, output window in LDS.
// All control flow is wave-uniform (every lane parses the same token stream); literal runs and
// match copies are lane-parallel, overlapping matches proceed in rounds of min(offset, 64).
// ---------------------------------------------------------------------------------------------
constexpr int kLzThreads = 64;
constexpr uint32_t kLzWindow = 64 * 1024;

__global__ __launch_bounds__(kLzThreads) void lz4_decompress_kernel(const Lz4Chunk* __restrict__ ch,
                                                                   int n, int32_t* __restrict__ out_sizes) {
  extern __shared__ __attribute__((aligned(16))) uint8_t win[];
  const int lane = threadIdx.x;
  for (int w = blockIdx.x; w < n; w += gridDim.x) {
    const uint8_t* __restrict__ ip = reinterpret_cast<const uint8_t*>(ch[w].src);
    const uint8_t* const iend = ip + ch[w].src_bytes;
    const uint32_t cap = ch[w].dst_capacity < kLzWindow ? ch[w].dst_capacity : kLzWindow;
    uint32_t op = 0;
    int32_t status = 0;
    while (ip < iend) {
      const uint32_t token = *ip++;
      uint32_t lit = token >> 4;
      if (lit == 15) {
        uint32_t b;
        do {
          if (ip >= iend) { status = -1; break; }
          b = *ip++;
          lit += b;
        } while (b == 255);
        if (status) break;
      }
      if (ip + lit > iend || op + lit > cap) { status = -2; break; }
      for (uint32_t i = lane; i < lit; i += kLzThreads) win[op + i] = ip[i];
      ip += lit;
      op += lit;
      if (ip >= iend) break;  // last sequence carries literals only
      if (ip + 2 > iend) { status = -3; break; }
      const uint32_t off = (uint32_t)ip[0] | ((uint32_t)ip[1] << 8);
      ip += 2;
      uint32_t ml = token & 15;
      if (ml == 15) {
        uint32_t b;
        do {
          if (ip >= iend) { status = -4; break; }
          b = *ip++;
          ml += b;
        } while (b == 255);
        if (status) break;
      }
      ml += 4;
      if (off == 0 || off > op || op + ml > cap) { status = -5; break; }
      __syncthreads();  // literal/match writes of the previous step visible to all lanes
      const uint32_t stride = off < (uint32_t)kLzThreads ? off : (uint32_t)kLzThreads;
      for (uint32_t base = 0; base < ml; base += stride) {
        const uint32_t i = base + lane;
        uint8_t v = 0;
        if (lane < (int)stride && i < ml) v = win[op - off + i];
        __syncthreads();
        if (lane < (int)stride && i < ml) win[op + i] = v;
        __syncthreads();
      }
      op += ml;
    }
    __syncthreads();
    if (status == 0) {
      uint8_t* __restrict__ dst = reinterpret_cast<uint8_t*>(ch[w].dst);
      for (uint32_t i = lane; i < op; i += kLzThreads) dst[i] = win[i];
    }
    if (lane == 0) out_sizes[w] = status ? status : (int32_t)op;
    __syncthreads();
  }
}

// Direct-to-HBM variant: one wave per chunk decodes straight into the destination (no 64 KiB
// LDS window, so occupancy is bounded by registers, not LDS: ~16x more chunks in flight per CU
// than the windowed kernel).  Cross-lane read-after-write through global memory only happens when
// a match's source overlaps output written since the last fence; the wave tracks that frontier
// (`fenced`) and only then issues __threadfence_block() (s_waitcnt on the stores), so matches
// into older output — the common case — cost no extra round trip.
__global__ __launch_bounds__(kLzThreads) void lz4_decompress_direct_kernel(const Lz4Chunk* __restrict__ ch,
                                                                          int n, int32_t* __restrict__ out_sizes) {
  const int lane = threadIdx.x;
  for (int w = blockIdx.x; w < n; w += gridDim.x) {
    const uint8_t* __restrict__ ip = reinterpret_cast<const uint8_t*>(ch[w].src);
    const uint8_t* const iend = ip + ch[w].src_bytes;
    uint8_t* const dst = reinterpret_cast<uint8_t*>(ch[w].dst);
    const uint32_t cap = ch[w].dst_capacity;
    uint32_t op = 0, fenced = 0;
    int32_t status = 0;
    while (ip < iend) {
      const uint32_t token = *ip++;
      uint32_t lit = token >> 4;
      if (lit == 15) {
        uint32_t b;
        do {
          if (ip >= iend) { status = -1; break; }
          b = *ip++;
          lit += b;
        } while (b == 255);
        if (status) break;
      }
      if (ip + lit > iend || op + lit > cap) { status = -2; break; }
      for (uint32_t i = lane; i < lit; i += kLzThreads) dst[op + i] = ip[i];
      ip += lit;
      op += lit;
      if (ip >= iend) break;  // last sequence carries literals only
      if (ip + 2 > iend) { status = -3; break; }
      const uint32_t off = (uint32_t)ip[0] | ((uint32_t)ip[1] << 8);
      ip += 2;
      uint32_t ml = token & 15;
      if (ml == 15) {
        uint32_t b;
        do {
          if (ip >= iend) { status = -4; break; }
          b = *ip++;
          ml += b;
        } while (b == 255);
        if (status) break;
      }
      ml += 4;
      if (off == 0 || off > op || op + ml > cap) { status = -5; break; }
      if (op - off + (ml < off ? ml : off) > fenced) {  // source touches unfenced output
        __threadfence_block();
        fenced = op;
      }
      if (off >= ml) {
        for (uint32_t i = lane; i < ml; i += kLzThreads) dst[op + i] = dst[op - off + i];
      } else {
        // overlapping match: rounds of `off` bytes (<= 64 lanes), each reading the previous round
        const uint32_t stride = off < (uint32_t)kLzThreads ? off : (uint32_t)kLzThreads;
        for (uint32_t base = 0; base < ml; base += stride) {
          const uint32_t i = base + lane;
          if (lane < (int)stride && i < ml) dst[op + i] = dst[op - off + i];
          __threadfence_block();
        }
        fenced = op + ml;
      }
      op += ml;
    }
    if (lane == 0) out_sizes[w] = status ? status : (int32_t)op;
  }
}

// Variant 2: as the direct kernel, but the token/length/offset parse reads the compressed stream
// from a 4 KiB LDS staging buffer refilled lane-parallel (one 64-byte strip per lane), so each
// sequence costs LDS latency instead of 3-4 dependent HBM/L2 round trips; literal runs are
// still copied lane-parallel straight from HBM.
constexpr uint32_t kLzIn = 4096;

__global__ __launch_bounds__(kLzThreads) void lz4_decompress_staged_kernel(const Lz4Chunk* __restrict__ ch,
                                                                          int n, int32_t* __restrict__ out_sizes) {
  __shared__ uint8_t inb[kLzIn];
  const int lane = threadIdx.x;
  for (int w = blockIdx.x; w < n; w += gridDim.x) {
    const uint8_t* __restrict__ src = reinterpret_cast<const uint8_t*>(ch[w].src);
    const uint32_t slen = ch[w].src_bytes;
    uint8_t* const dst = reinterpret_cast<uint8_t*>(ch[w].dst);
    const uint32_t cap = ch[w].dst_capacity;
    uint32_t base = 0, valid = 0;
    auto refill = [&](uint32_t pos) {
      __syncthreads();
      const uint32_t avail = slen - pos < kLzIn ? slen - pos : kLzIn;
      for (uint32_t i = lane; i < avail; i += kLzThreads) inb[i] = src[pos + i];
      base = pos;
      valid = avail;
      __syncthreads();
    };
    auto at = [&](uint32_t pos) -> uint32_t {
      if (pos - base >= valid) refill(pos);
      return inb[pos - base];
    };
    uint32_t ip = 0, op = 0, fenced = 0;
    int32_t status = 0;
    while (ip < slen) {
      const uint32_t token = at(ip++);
      uint32_t lit = token >> 4;
      if (lit == 15) {
        uint32_t b;
        do {
          if (ip >= slen) { status = -1; break; }
          b = at(ip++);
          lit += b;
        } while (b == 255);
        if (status) break;
      }
      if (ip + lit > slen || op + lit > cap) { status = -2; break; }
      if (ip - base + lit <= valid) {
        for (uint32_t i = lane; i < lit; i += kLzThreads) dst[op + i] = inb[ip - base + i];
      } else {
        for (uint32_t i = lane; i < lit; i += kLzThreads) dst[op + i] = src[ip + i];
      }
      ip += lit;
      op += lit;
      if (ip >= slen) break;  // last sequence carries literals only
      if (ip + 2 > slen) { status = -3; break; }
      const uint32_t off = at(ip) | (at(ip + 1) << 8);
      ip += 2;
      uint32_t ml = token & 15;
      if (ml == 15) {
        uint32_t b;
        do {
          if (ip >= slen) { status = -4; break; }
          b = at(ip++);
          ml += b;
        } while (b == 255);
        if (status) break;
      }
      ml += 4;
      if (off == 0 || off > op || op + ml > cap) { status = -5; break; }
      if (op - off + (ml < off ? ml : off) > fenced) {
        __threadfence_block();
        fenced = op;
      }
      if (off >= ml) {
        for (uint32_t i = lane; i < ml; i += kLzThreads) dst[op + i] = dst[op - off + i];
      } else {
        const uint32_t stride = off < (uint32_t)kLzThreads ? off : (uint32_t)kLzThreads;
        for (uint32_t b0 = 0; b0 < ml; b0 += stride) {
          const uint32_t i = b0 + lane;
          if (lane < (int)stride && i < ml) dst[op + i] = dst[op - off + i];
          __threadfence_block();
        }
        fenced = op + ml;
      }
      op += ml;
    }
    if (lane == 0) out_sizes[w] = status ? status : (int32_t)op;
    __syncthreads();
  }
}

// Variant 3: variant 2 plus an 8 KiB LDS ring mirroring the most recent output, so matches with
// offset <= 8 KiB (the bulk of real LZ4 streams) read their source from LDS: the per-sequence
// dependency chain has no HBM load left (output still streams to HBM with plain stores).
constexpr uint32_t kLzRing = 8192;

__global__ __launch_bounds__(kLzThreads) void lz4_decompress_ring_kernel(const Lz4Chunk* __restrict__ ch,
                                                                        int n, int32_t* __restrict__ out_sizes) {
  __shared__ uint8_t inb[kLzIn];
  __shared__ uint8_t ring[kLzRing];
  constexpr uint32_t rmask = kLzRing - 1;
  const int lane = threadIdx.x;
  for (int w = blockIdx.x; w < n; w += gridDim.x) {
    const uint8_t* __restrict__ src = reinterpret_cast<const uint8_t*>(ch[w].src);
    const uint32_t slen = ch[w].src_bytes;
    uint8_t* const dst = reinterpret_cast<uint8_t*>(ch[w].dst);
    const uint32_t cap = ch[w].dst_capacity;
    uint32_t base = 0, valid = 0;
    auto refill = [&](uint32_t pos) {
      __syncthreads();
      const uint32_t avail = slen - pos < kLzIn ? slen - pos : kLzIn;
      for (uint32_t i = lane; i < avail; i += kLzThreads) inb[i] = src[pos + i];
      base = pos;
      valid = avail;
      __syncthreads();
    };
    auto at = [&](uint32_t pos) -> uint32_t {
      if (pos - base >= valid) refill(pos);
      return inb[pos - base];
    };
    uint32_t ip = 0, op = 0, fenced = 0;
    int32_t status = 0;
    while (ip < slen) {
      const uint32_t token = at(ip++);
      uint32_t lit = token >> 4;
      if (lit == 15) {
        uint32_t b;
        do {
          if (ip >= slen) { status = -1; break; }
          b = at(ip++);
          lit += b;
        } while (b == 255);
        if (status) break;
      }
      if (ip + lit > slen || op + lit > cap) { status = -2; break; }
      const bool in_lds = ip - base + lit <= valid;
      for (uint32_t i = lane; i < lit; i += kLzThreads) {
        const uint8_t v = in_lds ? inb[ip - base + i] : src[ip + i];
        dst[op + i] = v;
        ring[(op + i) & rmask] = v;
      }
      ip += lit;
      op += lit;
      if (ip >= slen) break;  // last sequence carries literals only
      if (ip + 2 > slen) { status = -3; break; }
      const uint32_t off = at(ip) | (at(ip + 1) << 8);
      ip += 2;
      uint32_t ml = token & 15;
      if (ml == 15) {
        uint32_t b;
        do {
          if (ip >= slen) { status = -4; break; }
          b = at(ip++);
          ml += b;
        } while (b == 255);
        if (status) break;
      }
      ml += 4;
      if (off == 0 || off > op || op + ml > cap) { status = -5; break; }
      __syncthreads();  // ring writes of the literals visible to every lane
      if (off <= kLzRing - kLzThreads) {
        const uint32_t stride = off < (uint32_t)kLzThreads ? off : (uint32_t)kLzThreads;
        for (uint32_t b0 = 0; b0 < ml; b0 += stride) {
          const uint32_t i = b0 + lane;
          uint8_t v = 0;
          if (lane < (int)stride && i < ml) v = ring[(op - off + i) & rmask];
          __syncthreads();
          if (lane < (int)stride && i < ml) {
            dst[op + i] = v;
            ring[(op + i) & rmask] = v;
          }
          __syncthreads();
        }
      } else {
        // far match (> ring): source is older output in HBM; fence only if it is unfenced
        if (op - off + ml > fenced) {
          __threadfence_block();
          fenced = op;
        }
        for (uint32_t i = lane; i < ml; i += kLzThreads) {
          const uint8_t v = dst[op - off + i];
          dst[op + i] = v;
          ring[(op + i) & rmask] = v;
        }
        __syncthreads();
      }
      op += ml;
    }
    if (lane == 0) out_sizes[w] = status ? status : (int32_t)op;
    __syncthreads();
  }
}

// Variants 4-6: wave-synchronous decode.  The workgroup is ONE wave, so lanes need no
// workgroup barrier to see each other's LDS writes: LDS ops of a wave execute in issue order and
// a wavefront-scope fence + wave barrier only stops the compiler from reordering them
// (rocPRIM's wave_barrier idiom).  The old kernels' __syncthreads() also drained every
// outstanding HBM store (s_waitcnt vmcnt/vscnt 0) once or twice per sequence, which made the
// per-sequence chain ~1800 cycles.  Here:
//   * the parse reads 8 stream bytes per LDS access (token, short literal length, offset and
//     the first match-length byte usually come in one read);
//   * an R-byte LDS ring mirrors the latest output, so matches with offset <= R-64 (the bulk of
//     LZ4 streams) never read HBM; overlapping matches copy 64 bytes per round from the latest
//     period (src = op + b0 - off + (i - b0) % off), so even offset-1 runs take one round per
//     64 bytes instead of one per byte;
//   * output goes to HBM with plain stores that are never read back, except by far matches
//     (offset > R-64), which fence only when their source overlaps unfenced output.
__device__ __forceinline__ void lz_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

typedef __attribute__((address_space(1))) uint8_t gu8;

template <uint32_t R, bool kFast, uint32_t I = kLzIn>
__global__ __launch_bounds__(kLzThreads) void lz4_decompress_wave_kernel(const Lz4Chunk* __restrict__ ch,
                                                                        int n, int32_t* __restrict__ out_sizes) {
  __shared__ __attribute__((aligned(16))) uint8_t inb[I + 16];
  __shared__ uint8_t ring[R];
  constexpr uint32_t rmask = R - 1;
  const uint32_t lane = threadIdx.x;
  for (int w = blockIdx.x; w < n; w += gridDim.x) {
    // global (addrspace 1) pointers: generic/FLAT accesses would also count in lgkmcnt, so
    // every LDS wait of the parse would drain the wave's outstanding HBM stores
    const gu8* __restrict__ src = reinterpret_cast<const gu8*>(ch[w].src);
    const uint32_t slen = ch[w].src_bytes;
    gu8* const dst = reinterpret_cast<gu8*>(ch[w].dst);
    const uint32_t cap = ch[w].dst_capacity;
    uint32_t base = 0, valid = 0;
    auto refill = [&](uint32_t pos) {
      const uint32_t b = pos & ~7u;
      const uint32_t avail = slen - b < I ? slen - b : I;
      lz_wave_sync();
      for (uint32_t i = lane; i < avail; i += kLzThreads) inb[i] = src[b + i];
      base = b;
      valid = avail;
      lz_wave_sync();
    };
    // 8 bytes of the stream from pos (bytes past the stream end are garbage: callers bound-check)
    auto window = [&](uint32_t pos) -> uint64_t {
      if (pos + 8 > base + valid && base + valid < slen) refill(pos);
      const uint32_t r = pos - base;
      const uint32_t a = r & ~7u;
      const uint64_t lo = *reinterpret_cast<const uint64_t*>(inb + a);
      const uint64_t hi = *reinterpret_cast<const uint64_t*>(inb + a + 8);
      const uint32_t sh = (r & 7u) * 8u;
      return sh ? (lo >> sh) | (hi << (64u - sh)) : lo;
    };
    auto byte_at = [&](uint32_t pos) -> uint32_t { return (uint32_t)(window(pos) & 255u); };
    uint32_t ip = 0, op = 0, fenced = 0;
    int32_t status = 0;
    while (ip < slen) {
      const uint64_t wv = window(ip);
      const uint32_t token = (uint32_t)(wv & 255u);
      if constexpr (kFast) {
        // Fast path for the common sequence shape: <= 4 literals and a match of <= 18 bytes
        // whose offset lies in the ring.  The literals and the offset are already in the 8-byte
        // window (no further LDS read), the literal bytes are shifted out of it per lane, the
        // match is one 64-lane round; ~4x fewer scalar instructions and branches than the
        // general path below (which the SQ_INSTS_SALU counts showed to be the limit).
        const uint32_t fl = token >> 4, fm = token & 15u;
        const uint32_t mop = op + fl;
        const uint32_t foff = (uint32_t)((wv >> (8u * (1u + (fl < 4u ? fl : 4u)))) & 0xFFFFu);
        const uint32_t fml = fm + 4u;
        if (fl <= 4u && fm < 15u && ip + 3u + fl < slen && foff != 0u && foff <= mop && mop + fml <= cap &&
            foff + kLzThreads <= R) {
          if (lane < fl) {
            const uint8_t v = (uint8_t)(wv >> (8u * (1u + (lane & 7u))));
            dst[op + lane] = v;
            ring[(op + lane) & rmask] = v;
          }
          lz_wave_sync();
          if (lane < fml) {
            uint32_t s = mop - foff + lane;
            if (foff < fml) {
              const uint32_t q = (uint32_t)((float)lane * __builtin_amdgcn_rcpf((float)foff));
              int32_t r = (int32_t)lane - (int32_t)(q * foff);
              if (r >= (int32_t)foff) r -= foff;
              if (r < 0) r += foff;
              s = mop - foff + (uint32_t)r;
            }
            const uint8_t v = ring[s & rmask];
            dst[mop + lane] = v;
            ring[(mop + lane) & rmask] = v;
          }
          lz_wave_sync();
          ip += 3u + fl;
          op = mop + fml;
          continue;
        }
      }
      uint32_t lit = token >> 4;
      ++ip;
      if (lit == 15) {
        uint32_t b;
        do {
          if (ip >= slen) { status = -1; break; }
          b = byte_at(ip++);
          lit += b;
        } while (b == 255);
        if (status) break;
      }
      if (ip + lit > slen || op + lit > cap) { status = -2; break; }
      if (lit) {
        // CDNA counts stores in vmcnt: waiting for a global load would also drain every HBM
        // store in flight, so literals always come from the LDS staging (refilled at the run when
        // needed) and the global-load loop is kept separate for runs longer than the staging
        if (ip + lit > base + valid && lit + 8 <= I) refill(ip);
        if (ip + lit <= base + valid) {
          for (uint32_t i = lane; i < lit; i += kLzThreads) {
            const uint8_t v = inb[ip - base + i];
            dst[op + i] = v;
            ring[(op + i) & rmask] = v;
          }
        } else {
          for (uint32_t i = lane; i < lit; i += kLzThreads) {
            const uint8_t v = src[ip + i];
            dst[op + i] = v;
            ring[(op + i) & rmask] = v;
          }
        }
      }
      const bool short_lit = (token >> 4) <= 4;   // offset + first ml byte inside wv
      ip += lit;
      op += lit;
      if (ip >= slen) break;  // last sequence carries literals only
      if (ip + 2 > slen) { status = -3; break; }
      uint32_t off, ml = token & 15;
      if (short_lit) {
        const uint32_t sh = 8u * (1u + (token >> 4));
        off = (uint32_t)((wv >> sh) & 0xFFFFu);
      } else {
        const uint64_t ov = window(ip);
        off = (uint32_t)(ov & 0xFFFFu);
      }
      ip += 2;
      if (ml == 15) {
        uint32_t b;
        do {
          if (ip >= slen) { status = -4; break; }
          b = byte_at(ip++);
          ml += b;
        } while (b == 255);
        if (status) break;
      }
      ml += 4;
      if (off == 0 || off > op || op + ml > cap) { status = -5; break; }
      lz_wave_sync();   // literal ring writes before the match reads them
      if (off + kLzThreads <= R) {
        uint32_t lmod = lane;   // lane % off for short offsets (periodic copy), once per match
        if (off < kLzThreads) {
          const uint32_t q = (uint32_t)((float)lane * __builtin_amdgcn_rcpf((float)off));
          int32_t r = (int32_t)lane - (int32_t)(q * off);
          if (r >= (int32_t)off) r -= off;
          if (r < 0) r += off;
          lmod = (uint32_t)r;
        }
        for (uint32_t b0 = 0; b0 < ml; b0 += kLzThreads) {
          const uint32_t i = b0 + lane;
          if (i < ml) {
            const uint32_t s = off >= kLzThreads ? op + i - off : op + b0 - off + lmod;
            const uint8_t v = ring[s & rmask];
            dst[op + i] = v;
            ring[(op + i) & rmask] = v;
          }
          lz_wave_sync();
        }
      } else {
        // far match: source is older output in HBM (off > R-64 >= 64, so a round's source lies
        // before the round); fence only when it overlaps output not yet fenced
        for (uint32_t b0 = 0; b0 < ml; b0 += kLzThreads) {
          if (op + b0 + kLzThreads > fenced + off) {
            __threadfence_block();
            fenced = op + b0;
          }
          const uint32_t i = b0 + lane;
          if (i < ml) {
            const uint8_t v = dst[op + i - off];
            dst[op + i] = v;
            ring[(op + i) & rmask] = v;
          }
          lz_wave_sync();
        }
      }
      op += ml;
    }
    if (lane == 0) out_sizes[w] = status ? status : (int32_t)op;
    lz_wave_sync();
  }
}

// Variants 13-15: lane groups.  The wave-uniform kernels above run the token parse on the
// CU's single scalar pipe, which caps them at ~50-75 GB/s however the copies are done
// (profiles/r2_lz4.md).  Here a wave decodes 64/G chunks at once: each group of G lanes owns one
// chunk and keeps its parse state in VGPRs, so one VALU instruction advances 64/G independent
// token streams and the four SIMDs share the parse work.  Each group has its own input staging
// (I bytes, refilled with aligned dword loads) and output ring (R bytes) in LDS; matches within
// the ring never touch HBM, farther ones read the output back after a fence.
template <uint32_t G, uint32_t R, uint32_t I>
__global__ __launch_bounds__(kLzThreads) void lz4_decompress_groups_kernel(const Lz4Chunk* __restrict__ ch,
                                                                          int n, int32_t* __restrict__ out_sizes) {
  constexpr uint32_t NG = kLzThreads / G;
  constexpr uint32_t rmask = R - 1;
  __shared__ __attribute__((aligned(16))) uint8_t inb_all[NG][I + 16];
  __shared__ uint8_t ring_all[NG][R];
  const uint32_t lane = threadIdx.x, grp = lane / G, gl = lane % G;
  uint8_t* const inb = inb_all[grp];
  uint8_t* const ring = ring_all[grp];
  const int nsets = (n + (int)NG - 1) / (int)NG;
  for (int set = blockIdx.x; set < nsets; set += gridDim.x) {
    const int c = set * (int)NG + (int)grp;
    const bool have = c < n;
    const gu8* src = have ? reinterpret_cast<const gu8*>(ch[c].src) : nullptr;
    const uint32_t slen = have ? ch[c].src_bytes : 0u;
    gu8* const dst = have ? reinterpret_cast<gu8*>(ch[c].dst) : nullptr;
    const uint32_t cap = have ? ch[c].dst_capacity : 0u;
    uint32_t base = 0, valid = 0, ip = 0, op = 0;
    int32_t status = 0;
    bool active = have && slen > 0;
    auto refill = [&](uint32_t pos) {
      const uint32_t b = pos & ~7u;
      const uint32_t avail = slen - b < I ? slen - b : I;
      const uint64_t a0 = reinterpret_cast<uint64_t>(src + b);
      const uint64_t al = a0 & ~3ull;
      const uint32_t lead = (uint32_t)(a0 - al);
      const uint32_t nw = (avail + lead + 3u) / 4u;
      lz_wave_sync();
      for (uint32_t k = gl; k < nw; k += G) {
        const uint32_t wv = *reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(al + 4ull * k);
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
          const int32_t d = (int32_t)(4u * k + j) - (int32_t)lead;
          if (d >= 0 && (uint32_t)d < avail) inb[d] = (uint8_t)(wv >> (8u * j));
        }
      }
      base = b;
      valid = avail;
      lz_wave_sync();
    };
    auto win = [&](uint32_t pos) -> uint64_t {
      if (pos + 8 > base + valid && base + valid < slen) refill(pos);
      const uint32_t r = pos - base;
      const uint32_t a = r & ~7u;
      const uint64_t lo = *reinterpret_cast<const uint64_t*>(inb + a);
      const uint64_t hi = *reinterpret_cast<const uint64_t*>(inb + a + 8);
      const uint32_t sh = (r & 7u) * 8u;
      return sh ? (lo >> sh) | (hi << (64u - sh)) : lo;
    };
    while (__any(active)) {
      if (active) {
        const uint64_t wv = win(ip);
        const uint32_t token = (uint32_t)(wv & 255u);
        uint32_t lit = token >> 4;
        uint32_t p = ip + 1;
        if (lit == 15) {
          uint32_t b = 255;
          while (b == 255 && p < slen) {
            b = (uint32_t)(win(p) & 255u);
            ++p;
            lit += b;
          }
          if (b == 255) status = -1;
        }
        if (!status && (p + lit > slen || op + lit > cap)) status = -2;
        if (!status && lit) {
          if (p + lit > base + valid && lit + 8 <= I) refill(p);
          if (p + lit <= base + valid) {
            for (uint32_t i = gl; i < lit; i += G) {
              const uint8_t v = inb[p - base + i];
              dst[op + i] = v;
              ring[(op + i) & rmask] = v;
            }
          } else {
            for (uint32_t i = gl; i < lit; i += G) {
              const uint8_t v = src[p + i];
              dst[op + i] = v;
              ring[(op + i) & rmask] = v;
            }
          }
          p += lit;
          op += lit;
        }
        if (status || p >= slen) {
          active = false;   // error, or the last sequence (literals only) is done
        } else if (p + 2 > slen) {
          status = -3;
          active = false;
        } else {
          const uint32_t off = (uint32_t)(win(p) & 0xFFFFu);
          p += 2;
          uint32_t ml = token & 15u;
          if (ml == 15) {
            uint32_t b = 255;
            while (b == 255 && p < slen) {
              b = (uint32_t)(win(p) & 255u);
              ++p;
              ml += b;
            }
            if (b == 255) status = -4;
          }
          ml += 4;
          if (!status && (off == 0 || off > op || op + ml > cap)) status = -5;
          if (status) {
            active = false;
          } else {
            lz_wave_sync();   // literal ring writes before the match reads them
            if (off + G <= R) {
              uint32_t lmod = gl;
              if (off < G) lmod = gl % off;
              for (uint32_t b0 = 0; b0 < ml; b0 += G) {
                const uint32_t i = b0 + gl;
                if (i < ml) {
                  const uint32_t s = off >= G ? op + i - off : op + b0 - off + lmod;
                  const uint8_t v = ring[s & rmask];
                  dst[op + i] = v;
                  ring[(op + i) & rmask] = v;
                }
                lz_wave_sync();
              }
            } else {
              // far match: the source is output in HBM; off > R - G >= G keeps each round's
              // source before the round, the fence makes earlier rounds' stores visible
              for (uint32_t b0 = 0; b0 < ml; b0 += G) {
                __threadfence_block();
                const uint32_t i = b0 + gl;
                if (i < ml) {
                  const uint8_t v = dst[op + i - off];
                  dst[op + i] = v;
                  ring[(op + i) & rmask] = v;
                }
                lz_wave_sync();
              }
            }
            op += ml;
            ip = p;
          }
        }
      }
    }
    if (have && gl == 0) out_sizes[c] = status ? status : (int32_t)op;
    lz_wave_sync();
  }
}

// Variants 19-22: window-parallel decode, one wave per chunk.  The kernels above walk the token
// stream one sequence at a time, so a chunk costs (sequences x per-sequence latency): ~10k
// sequences per 64 KiB of text at 1-2k cycles each, and at <= 4k chunks there are not enough
// chunks to hide that (profiles/r2_lz4.md).  Here every step of the wave covers a 64-byte window
// of the compressed stream:
//   1. candidate parse — lane l decodes a sequence header as if a token started at ip + l
//      (lengths, offset, next-token position), all 64 in parallel from an LDS input stage;
//   2. walk — the true token chain from ip is followed through the candidates with readlane
//      (a handful of scalar instructions per sequence instead of the ~140 of the uniform parse),
//      each accepted token gets its window output offset by writelane, until TMAX output bytes;
//   3. codes — each token lane writes one code per output byte: literal (stage index), earlier
//      output (absolute position) or a reference into this window, then references are resolved
//      by pointer jumping in blocks of 64 (earlier blocks are final, so chains only double within
//      one block);
//   4. gather — bytes come from the stage, the R-byte LDS ring (recent output) or HBM (older
//      output, already flushed and fenced), and land in the ring; the ring is flushed to HBM in
//      aligned 16-byte vectors every 1 KiB.
// Sequences whose header or output does not fit a window (long literal runs, long matches) go
// through a per-sequence path that copies with all 64 lanes straight from HBM.
__device__ __forceinline__ uint32_t lz_shfl(uint32_t v, uint32_t src) { return (uint32_t)__shfl((int)v, (int)src, 64); }
__device__ __forceinline__ uint32_t lz_scan_add(uint32_t v, uint32_t lane) {
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}
__device__ __forceinline__ uint32_t lz_scan_max(uint32_t v, uint32_t lane) {
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)v, o, 64);
    if (lane >= o) v = v > t ? v : t;
  }
  return v;
}

// kVec (variants 23-25): the walk and the code build without per-sequence scalar work.  PMC of the
// scalar walk (profiles/r3_lz4_window.md) showed ~36 SALU instructions per sequence, and the CU's
// one scalar unit serves all 16 resident waves: the chain is found by pointer doubling instead
// (each lane's 2^k-step successor and visited-lane mask through ds_bpermute, 6 rounds), output
// offsets by a wave prefix sum, and each output byte finds its sequence by a max-scan of start
// marks -- all VALU/LDS, branch-free.
template <uint32_t R, uint32_t S, uint32_t TMAX, bool kVec = false, bool kPre = false>
__global__ __launch_bounds__(kLzThreads) void lz4_decompress_window_kernel(const Lz4Chunk* __restrict__ ch,
                                                                          int n, int32_t* __restrict__ out_sizes) {
  static_assert((R & (R - 1)) == 0 && R >= 4096 && S % 1024 == 0 && TMAX % 64 == 0 && TMAX <= 4096,
                "window kernel shape");
  constexpr uint32_t rmask = R - 1;
  constexpr uint32_t NB = TMAX / 64;
  constexpr uint32_t kInc = 1u << 24, kFinal = 1u << 25, kErrShift = 26, kNxt = 0xFFFFFFu;
  constexpr uint32_t kRef = 0x80000000u, kOld = 0x40000000u, kVal = 0x3FFFFFFFu;
  constexpr uint32_t kFlush = 1024;
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(1))) v4u gu4;
  __shared__ __attribute__((aligned(16))) uint8_t stage[S + 32];
  __shared__ __attribute__((aligned(16))) uint8_t ring[R];
  __shared__ uint32_t code[TMAX];
  __shared__ uint8_t marks[kVec ? TMAX : 1];
  __shared__ uint8_t winb[kPre ? TMAX : 1];   // the window's output bytes (reference targets)
  const uint32_t lane = threadIdx.x;
  if constexpr (kVec) {
    for (uint32_t i = lane; i < TMAX; i += kLzThreads) marks[i] = 0;
  }
  for (int w = blockIdx.x; w < n; w += gridDim.x) {
    const gu8* __restrict__ src = reinterpret_cast<const gu8*>(ch[w].src);
    const uint32_t slen = ch[w].src_bytes;
    gu8* const dst = reinterpret_cast<gu8*>(ch[w].dst);
    const uint32_t cap = ch[w].dst_capacity;
    const uint64_t daddr = reinterpret_cast<uint64_t>(dst);
    const uint32_t aoff = (uint32_t)daddr & 15u;
    // ring slot of output position pos, aligned to the destination address so that 16-byte
    // address granules are 16-byte ring granules
    auto ridx = [&](uint32_t pos) -> uint32_t { return (pos + aoff) & rmask; };
    uint32_t ip = 0, op = 0, flushed = 0, fenced = 0, vend = 0;
    int32_t sbase = 0;   // stage[0] holds input byte sbase (-15..0 for the first stage)
    bool at_end = false;
    int32_t status = 0;

    auto refill = [&](uint32_t pos) {
      const uint64_t a = (reinterpret_cast<uint64_t>(src) + pos) & ~15ull;
      const uint64_t send = reinterpret_cast<uint64_t>(src) + slen;
      lz_wave_sync();
      // 16-byte granules that hold at least one stream byte: never cross a page the stream
      // does not touch
      for (uint32_t g = lane; g < S / 16; g += kLzThreads) {
        const uint64_t ga = a + 16ull * g;
        if (ga < send) *reinterpret_cast<v4u*>(stage + 16 * g) = *reinterpret_cast<const gu4*>(ga);
      }
      sbase = (int32_t)(int64_t)(a - reinterpret_cast<uint64_t>(src));
      const uint32_t left = (uint32_t)((int32_t)slen - sbase);
      vend = left < S ? left : S;
      at_end = (int32_t)vend + sbase == (int32_t)slen;
      lz_wave_sync();
    };
    // output bytes [lo, hi) from the ring to HBM: whole 16-byte granules as vectors, the
    // partial granules at the ends bytewise
    auto flush = [&](uint32_t lo, uint32_t hi) {
      if (hi <= lo) return;
      const uint64_t b0 = daddr + lo, b1 = daddr + hi;
      const uint64_t a0 = b0 & ~15ull;
      const uint32_t ng = (uint32_t)((b1 - a0 + 15) >> 4);
      for (uint32_t g = lane; g < ng; g += kLzThreads) {
        const uint64_t ga = a0 + 16ull * g;
        if (ga >= b0 && ga + 16 <= b1) {
          *reinterpret_cast<gu4*>(ga) = *reinterpret_cast<const v4u*>(ring + ridx((uint32_t)(ga - daddr)));
        } else {
          for (uint32_t j = 0; j < 16; ++j) {
            const uint64_t ba = ga + j;
            if (ba >= b0 && ba < b1) *reinterpret_cast<gu8*>(ba) = ring[ridx((uint32_t)(ba - daddr))];
          }
        }
      }
    };
    // one sequence at ip with all 64 lanes straight from HBM (headers/literals too long for the
    // stage, outputs longer than TMAX); output goes to HBM and the ring; returns false when done
    auto slow_sequence = [&]() -> bool {
      flush(flushed, op);
      auto gb = [&](uint32_t pos) -> uint32_t { return (uint32_t)src[pos]; };
      // 255-terminated length extension, 64 bytes per step
      auto ext = [&](uint32_t& p, uint32_t& acc) -> bool {
        for (;;) {
          if (p >= slen) return false;
          const uint32_t idx = p + lane;
          const uint32_t b = idx < slen ? gb(idx) : 0u;
          const uint64_t stop = __ballot(idx >= slen || b != 255u);
          if (!stop) {
            acc += 255u * kLzThreads;
            p += kLzThreads;
            continue;
          }
          const uint32_t f = (uint32_t)__builtin_ctzll(stop);
          if (p + f >= slen) return false;
          acc += 255u * f + (uint32_t)__builtin_amdgcn_readlane((int)b, (int)f);
          p += f + 1;
          return true;
        }
      };
      const uint32_t t = gb(ip);
      uint32_t p = ip + 1, lit = t >> 4;
      if (lit == 15 && !ext(p, lit)) { status = -1; return false; }
      if (p + lit > slen || op + lit > cap) { status = -2; return false; }
#pragma unroll 8
      for (uint32_t i = lane; i < lit; i += kLzThreads) {
        const uint8_t v = src[p + i];
        dst[op + i] = v;
        ring[ridx(op + i)] = v;
      }
      p += lit;
      op += lit;
      if (p >= slen) { ip = p; flushed = op; return false; }
      if (p + 2 > slen) { status = -3; return false; }
      const uint32_t off = gb(p) | (gb(p + 1) << 8);
      p += 2;
      uint32_t ml = t & 15u;
      if (ml == 15 && !ext(p, ml)) { status = -4; return false; }
      ml += 4;
      if (off == 0 || off > op || op + ml > cap) { status = -5; return false; }
      lz_wave_sync();
      if (off <= R) {
        const uint32_t lmod = off < kLzThreads ? lane % off : lane;
        for (uint32_t b0 = 0; b0 < ml; b0 += kLzThreads) {
          const uint32_t i = b0 + lane;
          uint8_t v = 0;
          if (i < ml) v = ring[ridx(off >= kLzThreads ? op + i - off : op + b0 - off + lmod)];
          lz_wave_sync();
          if (i < ml) {
            dst[op + i] = v;
            ring[ridx(op + i)] = v;
          }
          lz_wave_sync();
        }
      } else {
        // far: the source is HBM output (all of it stored by now); fence before the first
        // round and whenever a round reads output this match stored
        for (uint32_t b0 = 0; b0 < ml; b0 += kLzThreads) {
          if (op + b0 + kLzThreads > fenced + off) {
            __threadfence_block();
            fenced = op + b0;
          }
          const uint32_t i = b0 + lane;
          if (i < ml) {
            const uint8_t v = dst[op + i - off];
            dst[op + i] = v;
            ring[ridx(op + i)] = v;
          }
          lz_wave_sync();
        }
      }
      op += ml;
      ip = p;
      flushed = op;
      return p < slen;
    };

    bool more = slen > 0;
    while (more) {
      const uint32_t r0 = (uint32_t)((int32_t)ip - sbase);
      if (vend == 0 || (!at_end && r0 + 2 * kLzThreads > vend)) {
        refill(ip);
        continue;
      }
      // 1. candidate headers: a token at stage index r = r0 + lane
      const uint32_t r = r0 + lane;
      uint32_t A = kInc, tot = 0, lit = 0, q = 0, off = 0;
      if (r < vend) {
        const uint32_t a8 = r & ~7u;
        const uint64_t lo = *reinterpret_cast<const uint64_t*>(stage + a8);
        const uint64_t hi = *reinterpret_cast<const uint64_t*>(stage + a8 + 8);
        const uint32_t sh = (r & 7u) * 8u;
        const uint64_t wv = sh ? (lo >> sh) | (hi << (64u - sh)) : lo;
        auto sb = [&](uint32_t idx) -> uint32_t {
          const uint32_t d = idx - r;
          return d < 8 ? (uint32_t)(wv >> (8u * d)) & 255u : (uint32_t)stage[idx];
        };
        const uint32_t t = (uint32_t)wv & 255u;
        uint32_t k = r + 1, err = 0;
        bool inc = false;
        lit = t >> 4;
        if (lit == 15) {
          uint32_t b = 255;
          while (b == 255) {
            if (k >= vend) {
              inc = !at_end;
              err = 1;
              break;
            }
            b = sb(k++);
            lit += b;
          }
        }
        q = k;
        const uint32_t le = k + lit;
        if (!err) {
          if (le > vend) {
            inc = !at_end;
            err = 2;
          } else if (at_end && le == vend) {
            tot = lit;
            A = kFinal;
          } else if (le + 2 > vend) {
            inc = !at_end;
            err = 3;
          } else {
            off = sb(le) | (sb(le + 1) << 8);
            uint32_t e = le + 2, ml = t & 15u;
            if (ml == 15) {
              uint32_t b = 255;
              while (b == 255) {
                if (e >= vend) {
                  inc = !at_end;
                  err = 4;
                  break;
                }
                b = sb(e++);
                ml += b;
              }
            }
            tot = lit + ml + 4;
            A = e - r0;
          }
        }
        if (inc) A = kInc;
        else if (err) A = err << kErrShift;
      }
      // 2. walk the token chain from lane 0
      uint32_t cur = 0, T = 0, cnt = 0, opo = 0;
      uint64_t mask = 0;
      int stop = 0;   // 0: next token at cur, 1: lane cur needs input, 2: error, 3: stream done, 4: too long
      if constexpr (kVec) {
        const uint32_t ecode = A >> kErrShift;
        const bool regular = !(A & (kInc | kFinal)) && !ecode;
        const bool ends = regular && ip + (A & kNxt) >= slen;   // the stream ends after this match
        uint32_t J = regular && !ends && (A & kNxt) < kLzThreads ? (A & kNxt) : kLzThreads;
        uint64_t Rm = 1ull << lane;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          const uint32_t src = J < kLzThreads ? J : lane;
          const uint32_t rlo = lz_shfl((uint32_t)Rm, src), rhi = lz_shfl((uint32_t)(Rm >> 32), src);
          const uint32_t jj = lz_shfl(J, src);
          if (J < kLzThreads) {
            Rm |= ((uint64_t)rhi << 32) | rlo;
            J = jj;
          }
        }
        const uint64_t C = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(Rm >> 32)) << 32) |
                           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)Rm);
        const uint64_t bad = C & __ballot((A & kInc) || ecode);
        const uint32_t fb = bad ? (uint32_t)__builtin_ctzll(bad) : 64u;
        const uint64_t pre = fb < 64 ? C & ((1ull << fb) - 1) : C;
        const uint32_t v = (pre >> lane) & 1ull ? tot : 0u;
        const uint32_t incl = lz_scan_add(v, lane);
        const uint64_t over = pre & __ballot(incl > TMAX);
        const uint32_t fo = over ? (uint32_t)__builtin_ctzll(over) : 64u;
        mask = fo < 64 ? pre & ((1ull << fo) - 1) : pre;
        cnt = (uint32_t)__builtin_popcountll(mask);
        opo = incl - v;
        if (fo < fb) {
          stop = cnt ? 0 : 4;
          cur = fo;
        } else if (fb < 64) {
          const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)A, (int)fb);
          cur = fb;
          if (a & kInc) {
            stop = 1;
          } else {
            stop = 2;
            status = -(int32_t)(a >> kErrShift);
          }
        } else {
          const uint32_t last = 63u - (uint32_t)__builtin_clzll(mask);
          const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)A, (int)last);
          cur = a & kNxt;
          stop = (a & kFinal) || ip + cur >= slen ? 3 : 0;
        }
        if (cnt) T = (uint32_t)__builtin_amdgcn_readlane((int)incl, (int)(63u - (uint32_t)__builtin_clzll(mask)));
      } else {
        while (cur < kLzThreads) {
          const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)A, (int)cur);
          const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)tot, (int)cur);
          if (a & kInc) { stop = 1; break; }
          if (a >> kErrShift) { status = -(int32_t)(a >> kErrShift); stop = 2; break; }
          if (T + b > TMAX) { stop = cnt ? 0 : 4; break; }
          opo = lane == cur ? T : opo;
          mask |= 1ull << cur;
          T += b;
          ++cnt;
          if (a & kFinal) { stop = 3; break; }
          cur = a & kNxt;
          if (ip + cur >= slen) { stop = 3; break; }
        }
      }
      if (stop == 2) break;
      if (cnt == 0) {
        if (stop == 1 && !(r0 < 16 && vend == S)) {
          refill(ip);   // the header runs past the stage: restart the stage at it
          continue;
        }
        more = slow_sequence();   // header longer than a stage, or output longer than TMAX
        if (status) break;
        continue;
      }
      // 3. per-token checks, then one code per output byte
      const bool tok = (mask >> lane) & 1ull;
      const bool fin = tok && (A & kFinal);
      const bool bad_lit = tok && op + opo + lit > cap;
      const bool bad_m = tok && !fin && (off == 0 || off > op + opo + lit || op + opo + tot > cap);
      const uint64_t badm = __ballot(bad_lit || bad_m);
      if (badm) {
        const uint32_t f = (uint32_t)__builtin_ctzll(badm);
        status = __builtin_amdgcn_readlane(bad_lit ? -2 : -5, (int)f);
        break;
      }
      if constexpr (kVec) {
        // start marks, then per block of 64 output bytes: owner = max-scan of the marks
        if (tok && tot) marks[opo] = (uint8_t)(lane + 1);
        lz_wave_sync();
        uint32_t carry = 0;
        for (uint32_t b0 = 0; b0 < T; b0 += kLzThreads) {
          const uint32_t x = b0 + lane;
          const bool in = x < T;
          uint32_t m = 0;
          if (in) {
            m = marks[x];
            marks[x] = 0;
          }
          uint32_t own = lz_scan_max(m, lane);
          own = own ? own : carry;
          carry = (uint32_t)__builtin_amdgcn_readlane((int)own, 63);
          const uint32_t j = own ? own - 1 : 0;
          const uint32_t o_opo = lz_shfl(opo, j), o_lit = lz_shfl(lit, j), o_q = lz_shfl(q, j), o_off = lz_shfl(off, j);
          if (in) {
            const uint32_t k = x - o_opo;
            const int32_t y = (int32_t)x - (int32_t)o_off;
            code[x] = k < o_lit ? o_q + k : (y >= 0 ? (kRef | (uint32_t)y) : (kOld | (uint32_t)((int32_t)op + y)));
          }
        }
      } else if (tok) {
        for (uint32_t k = 0; k < lit; ++k) code[opo + k] = q + k;
        for (uint32_t x = opo + lit; x < opo + tot; ++x) {
          const int32_t y = (int32_t)x - (int32_t)off;
          code[x] = y >= 0 ? (kRef | (uint32_t)y) : (kOld | (uint32_t)((int32_t)op + y));
        }
      }
      lz_wave_sync();
      // 4. resolve references block by block, gather the bytes
      uint32_t outb[NB];
      if constexpr (kVec && kPre) {
        // the bytes of every non-reference position are fetched first (stage / ring / HBM: the
        // far loads are in flight while the references resolve), references resolve to window
        // positions by pointer jumping, then read the window's bytes from LDS
        uint32_t cb[NB];
        bool farb[NB];
        bool anyfar = false;
#pragma unroll
        for (uint32_t bi = 0; bi < NB; ++bi) {
          const uint32_t x = bi * kLzThreads + lane;
          cb[bi] = x < T ? code[x] : kRef;
          const uint32_t cv = cb[bi] & kVal;
          farb[bi] = x < T && (cb[bi] & kOld) && !(cb[bi] & kRef) && op - cv > R;
          anyfar = anyfar || (farb[bi] && cv + 128 > fenced);
        }
        if (__ballot(anyfar)) {
          __threadfence_block();
          fenced = flushed;
        }
#pragma unroll
        for (uint32_t bi = 0; bi < NB; ++bi) {
          const uint32_t c = cb[bi], cv = c & kVal;
          outb[bi] = (c & kRef) ? 0u
                                : (farb[bi] ? (uint32_t)dst[cv] : ((c & kOld) ? (uint32_t)ring[ridx(cv)] : (uint32_t)stage[cv]));
        }
#pragma unroll
        for (uint32_t bi = 0; bi < NB; ++bi) {
          if (bi * kLzThreads < T) {
            const uint32_t x = bi * kLzThreads + lane;
            const bool in = x < T;
            uint32_t c = cb[bi];
            bool done = !in || !(c & kRef);
            while (__ballot(!done)) {
              if (!done) {
                const uint32_t t = code[c & kVal];
                if (t & kRef) c = t;
                else done = true;
              }
              lz_wave_sync();
              if (in && (c & kRef)) code[x] = c;
              lz_wave_sync();
            }
            cb[bi] = c;
          }
        }
#pragma unroll
        for (uint32_t bi = 0; bi < NB; ++bi) {
          const uint32_t x = bi * kLzThreads + lane;
          if (x < T && !(cb[bi] & kRef)) winb[x] = (uint8_t)outb[bi];
        }
        lz_wave_sync();
#pragma unroll
        for (uint32_t bi = 0; bi < NB; ++bi) {
          const uint32_t x = bi * kLzThreads + lane;
          if (x < T && (cb[bi] & kRef)) outb[bi] = winb[cb[bi] & kVal];
        }
      } else
#pragma unroll
      for (uint32_t bi = 0; bi < NB; ++bi) {
        outb[bi] = 0;
        if (bi * kLzThreads < T) {
          const uint32_t x = bi * kLzThreads + lane;
          const bool in = x < T;
          uint32_t c = in ? code[x] : 0u;
          while (__ballot(in && (c & kRef))) {
            if (in && (c & kRef)) c = code[c & kVal];
            lz_wave_sync();
            if (in) code[x] = c;
            lz_wave_sync();
          }
          const uint32_t cv = c & kVal;
          const bool far = in && (c & kOld) && op - cv > R;
          if (__ballot(far && cv + 128 > fenced)) {
            __threadfence_block();
            fenced = flushed;
          }
          if (in) outb[bi] = (c & kOld) ? (far ? (uint32_t)dst[cv] : (uint32_t)ring[ridx(cv)]) : (uint32_t)stage[cv];
        }
      }
      lz_wave_sync();
#pragma unroll
      for (uint32_t bi = 0; bi < NB; ++bi) {
        const uint32_t x = bi * kLzThreads + lane;
        if (x < T) ring[ridx(op + x)] = (uint8_t)outb[bi];
      }
      lz_wave_sync();
      op += T;
      ip += cur;
      if (stop == 3) more = false;
      if (op - flushed >= kFlush) {
        const uint32_t hi = (uint32_t)(((daddr + op) & ~15ull) - daddr);
        flush(flushed, hi);
        flushed = hi;
      }
    }
    if (!status) flush(flushed, op);
    if (lane == 0) out_sizes[w] = status ? status : (int32_t)op;
    lz_wave_sync();
  }
}

// -1 (default): auto — the window-parallel kernel (23) below 24k chunks, lane groups of 4 (17)
// from there up, where enough chunks exist to fill the CUs 16 per wave (profiles/r3_lz4_window.md:
// at 4096 chunks 23 decodes text 121 / csv 139 GB/s vs 39 / 55 for the wave-per-chunk kernel 2;
// at 32768 chunks 17 reaches 215 / 186).
// 0: LDS window, 1: direct, 2: staged parse, 3: + LDS ring, 4-12: wave-synchronous, 13-18: groups.
static int g_lz4_decode_variant = -1;
constexpr int kLzGroupMinChunks = 24576;

void set_lz4_decode_variant(int v) { g_lz4_decode_variant = v; }

hipError_t launch_lz4_decompress(const Lz4Chunk* chunks, int n, int32_t* out_sizes,
                                 hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  int variant = g_lz4_decode_variant;
  if (variant < 0) variant = n >= kLzGroupMinChunks ? 17 : 23;
  if (variant == 0) {
    const unsigned grid = (unsigned)std::min(n, 4096);
    hipLaunchKernelGGL(lz4_decompress_kernel, dim3(grid), dim3(kLzThreads), kLzWindow, stream,
                       chunks, n, out_sizes);
  } else if (variant == 1) {
    const unsigned grid = (unsigned)std::min(n, 65536);
    hipLaunchKernelGGL(lz4_decompress_direct_kernel, dim3(grid), dim3(kLzThreads), 0, stream,
                       chunks, n, out_sizes);
  } else if (variant == 2) {
    const unsigned grid = (unsigned)std::min(n, 65536);
    hipLaunchKernelGGL(lz4_decompress_staged_kernel, dim3(grid), dim3(kLzThreads), 0, stream,
                       chunks, n, out_sizes);
  } else if (variant == 3) {
    const unsigned grid = (unsigned)std::min(n, 65536);
    hipLaunchKernelGGL(lz4_decompress_ring_kernel, dim3(grid), dim3(kLzThreads), 0, stream,
                       chunks, n, out_sizes);
  } else {
    const unsigned grid = (unsigned)std::min(n, 65536);
    switch (variant) {
      case 4: hipLaunchKernelGGL((lz4_decompress_wave_kernel<8192, false>), dim3(grid), dim3(kLzThreads), 0, stream, chunks, n, out_sizes); break;
      case 5: hipLaunchKernelGGL((lz4_decompress_wave_kernel<16384, false>), dim3(grid), dim3(kLzThreads), 0, stream, chunks, n, out_sizes); break;
      case 6: hipLaunchKernelGGL((lz4_decompress_wave_kernel<32768, false>), dim3(grid), dim3(kLzThreads), 0, stream, chunks, n, out_sizes); break;
      case 7: hipLaunchKernelGGL((lz4_decompress_wave_kernel<8192, true>), dim3(grid), dim3(kLzThreads), 0, stream, chunks, n, out_sizes); break;
      case 8: hipLaunchKernelGGL((lz4_decompress_wave_kernel<16384, true>), dim3(grid), dim3(kLzThreads), 0, stream, chunks, n, out_sizes); break;
      case 9: hipLaunchKernelGGL((lz4_decompress_wave_kernel<32768, true>), dim3(grid), dim3(kLzThreads), 0, stream, chunks, n, out_sizes); break;
      case 10: hipLaunchKernelGGL((lz4_decompress_wave_kernel<4096, true, 1024>), dim3(grid), dim3(kLzThreads), 0, stream, chunks, n, out_sizes); break;
      case 11: hipLaunchKernelGGL((lz4_decompress_wave_kernel<2048, true, 1024>), dim3(grid), dim3(kLzThreads), 0, stream, chunks, n, out_sizes); break;
      case 12: hipLaunchKernelGGL((lz4_decompress_wave_kernel<4096, true, 512>), dim3(grid), dim3(kLzThreads), 0, stream, chunks, n, out_sizes); break;
      case 13: {
        const unsigned g = (unsigned)std::min((n + 7) / 8, 65536);
        hipLaunchKernelGGL((lz4_decompress_groups_kernel<8, 2048, 512>), dim3(g), dim3(kLzThreads), 0, stream, chunks, n, out_sizes);
        break;
      }
      case 14: {
        const unsigned g = (unsigned)std::min((n + 15) / 16, 65536);
        hipLaunchKernelGGL((lz4_decompress_groups_kernel<4, 1024, 256>), dim3(g), dim3(kLzThreads), 0, stream, chunks, n, out_sizes);
        break;
      }
      case 15: {
        const unsigned g = (unsigned)std::min((n + 3) / 4, 65536);
        hipLaunchKernelGGL((lz4_decompress_groups_kernel<16, 4096, 1024>), dim3(g), dim3(kLzThreads), 0, stream, chunks, n, out_sizes);
        break;
      }
      case 16: {
        const unsigned g = (unsigned)std::min((n + 31) / 32, 65536);
        hipLaunchKernelGGL((lz4_decompress_groups_kernel<2, 512, 128>), dim3(g), dim3(kLzThreads), 0, stream, chunks, n, out_sizes);
        break;
      }
      case 17: {
        const unsigned g = (unsigned)std::min((n + 15) / 16, 65536);
        hipLaunchKernelGGL((lz4_decompress_groups_kernel<4, 512, 256>), dim3(g), dim3(kLzThreads), 0, stream, chunks, n, out_sizes);
        break;
      }
      case 18: {
        const unsigned g = (unsigned)std::min((n + 15) / 16, 65536);
        hipLaunchKernelGGL((lz4_decompress_groups_kernel<4, 2048, 256>), dim3(g), dim3(kLzThreads), 0, stream, chunks, n, out_sizes);
        break;
      }
      case 19: hipLaunchKernelGGL((lz4_decompress_window_kernel<8192, 1024, 512>), dim3(grid), dim3(kLzThreads), 0, stream, chunks, n, out_sizes); break;
      case 20: hipLaunchKernelGGL((lz4_decompress_window_kernel<4096, 1024, 256>), dim3(grid), dim3(kLzThreads), 0, stream, chunks, n, out_sizes); break;
      case 21: hipLaunchKernelGGL((lz4_decompress_window_kernel<8192, 2048, 512>), dim3(grid), dim3(kLzThreads), 0, stream, chunks, n, out_sizes); break;
      case 22: hipLaunchKernelGGL((lz4_decompress_window_kernel<16384, 1024, 512>), dim3(grid), dim3(kLzThreads), 0, stream, chunks, n, out_sizes); break;
      case 23: hipLaunchKernelGGL((lz4_decompress_window_kernel<4096, 1024, 256, true>), dim3(grid), dim3(kLzThreads), 0, stream, chunks, n, out_sizes); break;
      case 24: hipLaunchKernelGGL((lz4_decompress_window_kernel<8192, 1024, 256, true>), dim3(grid), dim3(kLzThreads), 0, stream, chunks, n, out_sizes); break;
      case 25: hipLaunchKernelGGL((lz4_decompress_window_kernel<4096, 1024, 512, true>), dim3(grid), dim3(kLzThreads), 0, stream, chunks, n, out_sizes); break;
      default: hipLaunchKernelGGL((lz4_decompress_window_kernel<4096, 1024, 256, true, true>), dim3(grid), dim3(kLzThreads), 0, stream, chunks, n, out_sizes); break;
    }
  }
  return hipGetLastError();
}

// Compression: chunk staged into LDS, 4096-entry u16 hash table in LDS.  Lanes evaluate 64
// candidate positions at once (hash, probe, match length) against the table state at batch
// start; a wave ballot then drives the greedy parse.  Output is standard LZ4 block format.
constexpr int kLzHashLog = 12;
constexpr uint32_t kLzMinMatch = 4;
constexpr uint32_t kLzLastLiterals = 5;
constexpr uint32_t kLzMfLimit = 12;

__device__ __forceinline__ uint32_t lz_read32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint32_t lz_hash(uint32_t v) {
  return (v * 2654435761u) >> (32 - kLzHashLog);
}

__global__ __launch_bounds__(kLzThreads) void lz4_compress_kernel(const Lz4Chunk* __restrict__ ch,
                                                                 int n, int32_t* __restrict__ out_sizes) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* src = smem;                                            // 64 KiB
  uint16_t* table = reinterpret_cast<uint16_t*>(smem + kLzWindow);  // 8 KiB
  const int lane = threadIdx.x;
  for (int w = blockIdx.x; w < n; w += gridDim.x) {
    const uint8_t* __restrict__ gsrc = reinterpret_cast<const uint8_t*>(ch[w].src);
    uint8_t* __restrict__ dst = reinterpret_cast<uint8_t*>(ch[w].dst);
    const uint32_t len = ch[w].src_bytes < kLzWindow ? ch[w].src_bytes : kLzWindow;
    const uint32_t cap = ch[w].dst_capacity;
    for (uint32_t i = lane; i < len; i += kLzThreads) src[i] = gsrc[i];
    for (uint32_t i = lane; i < (1u << kLzHashLog); i += kLzThreads) table[i] = 0xFFFF;
    __syncthreads();
    uint32_t op = 0, anchor = 0, ip = 0;
    int32_t status = 0;
    const uint32_t match_limit = len > kLzMfLimit ? len - kLzMfLimit : 0;   // last match start
    const uint32_t end_match = len > kLzLastLiterals ? len - kLzLastLiterals : 0;
    while (ip < match_limit && status == 0) {
      // each lane probes position ip + lane
      const uint32_t pos = ip + lane;
      uint32_t cand = 0xFFFFFFFFu, mlen = 0;
      uint32_t h = 0;
      if (pos < match_limit) {
        const uint32_t v = lz_read32(src + pos);
        h = lz_hash(v);
        const uint32_t c = table[h];
        if (c != 0xFFFF && c < pos && pos - c <= 65535 && lz_read32(src + c) == v) {
          cand = c;
          mlen = kLzMinMatch;
          while (pos + mlen < end_match && src[c + mlen] == src[pos + mlen]) ++mlen;
        }
      }
      __syncthreads();
      if (pos < match_limit) table[h] = (uint16_t)pos;  // last writer wins: any entry is valid
      __syncthreads();
      const unsigned long long hits = __ballot(cand != 0xFFFFFFFFu);
      if (hits == 0) { ip += kLzThreads; continue; }
      const int first = __ffsll((long long)hits) - 1;
      const uint32_t mpos = ip + first;
      const uint32_t moff = mpos - __shfl(cand, first);
      const uint32_t ml = __shfl(mlen, first);
      // emit sequence: literals [anchor, mpos) + match (moff, ml)
      const uint32_t lit = mpos - anchor;
      const uint32_t need = 1 + (lit >= 15 ? (lit - 15) / 255 + 1 : 0) + lit + 2 +
                            ((ml - 4) >= 15 ? (ml - 4 - 15) / 255 + 1 : 0);
      if (op + need > cap) { status = -1; break; }
      uint32_t o = op;
      if (lane == 0) {
        const uint32_t mcode = ml - 4;
        dst[o] = (uint8_t)(((lit >= 15 ? 15 : lit) << 4) | (mcode >= 15 ? 15 : mcode));
        uint32_t q = o + 1;
        if (lit >= 15) { uint32_t r = lit - 15; while (r >= 255) { dst[q++] = 255; r -= 255; } dst[q++] = (uint8_t)r; }
        op = q;  // lane-0 local; broadcast below
      }
      o = __shfl(op, 0);
      for (uint32_t i = lane; i < lit; i += kLzThreads) dst[o + i] = src[anchor + i];
      o += lit;
      if (lane == 0) {
        dst[o] = (uint8_t)(moff & 255);
        dst[o + 1] = (uint8_t)(moff >> 8);
        uint32_t q = o + 2;
        const uint32_t mcode = ml - 4;
        if (mcode >= 15) { uint32_t r = mcode - 15; while (r >= 255) { dst[q++] = 255; r -= 255; } dst[q++] = (uint8_t)r; }
        op = q;
      }
      op = __shfl(op, 0);
      ip = mpos + ml;
      anchor = ip;
    }
    if (status == 0) {
      const uint32_t lit = len - anchor;
      const uint32_t need = 1 + (lit >= 15 ? (lit - 15) / 255 + 1 : 0) + lit;
      if (op + need > cap) {
        status = -1;
      } else {
        uint32_t o = op;
        if (lane == 0) {
          dst[o] = (uint8_t)((lit >= 15 ? 15 : lit) << 4);
          uint32_t q = o + 1;
          if (lit >= 15) { uint32_t r = lit - 15; while (r >= 255) { dst[q++] = 255; r -= 255; } dst[q++] = (uint8_t)r; }
          op = q;
        }
        o = __shfl(op, 0);
        for (uint32_t i = lane; i < lit; i += kLzThreads) dst[o + i] = src[anchor + i];
        op = o + lit;
      }
    }
    if (lane == 0) out_sizes[w] = status ? -1 : (int32_t)op;
    __syncthreads();
  }
}

// Batch-parse encoder.  The first kernel above emits ONE sequence per 64-position probe batch and
// throws the other 63 lanes' matches away, so text (≈8-byte sequences) costs one full probe round
// (two barriers, a ballot, a serial token write) per ~8 input bytes.  Here every probe batch is
// parsed completely: a uniform greedy walk over the ballot of hits selects every non-overlapping
// match in position order (hits inside a taken match are masked off in one step), each selected
// lane sizes its own sequence, a wave prefix sum places all of them, and the owning lanes write
// their tokens / length bytes / offsets in parallel while literal runs are copied by the whole
// wave.  Match extension compares 4 bytes at a time.  STAGE: chunk staged in LDS (72 KiB per
// wave) vs read from global/L2 with only the 8 KiB hash table in LDS (8x the waves per CU).
template <bool STAGE>
__device__ __forceinline__ uint32_t lzb_read32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

__device__ __forceinline__ uint32_t lz_len_bytes(uint32_t v) {  // extra length bytes for a 4-bit field
  return v >= 15 ? (v - 15) / 255 + 1 : 0;
}

__device__ __forceinline__ uint32_t lz_put_len(uint8_t* __restrict__ dst, uint32_t q, uint32_t v) {
  if (v >= 15) {
    uint32_t r = v - 15;
    while (r >= 255) { dst[q++] = 255; r -= 255; }
    dst[q++] = (uint8_t)r;
  }
  return q;
}

template <bool STAGE>
__global__ __launch_bounds__(kLzThreads) void lz4_compress_batch_kernel(const Lz4Chunk* __restrict__ ch,
                                                                       int n, int32_t* __restrict__ out_sizes) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint16_t* table = reinterpret_cast<uint16_t*>(smem);                     // 8 KiB
  uint8_t* stage = smem + (sizeof(uint16_t) << kLzHashLog);                // 64 KiB (STAGE)
  const int lane = threadIdx.x;
  for (int w = blockIdx.x; w < n; w += gridDim.x) {
    const uint8_t* __restrict__ gsrc = reinterpret_cast<const uint8_t*>(ch[w].src);
    uint8_t* __restrict__ dst = reinterpret_cast<uint8_t*>(ch[w].dst);
    const uint32_t len = ch[w].src_bytes < kLzWindow ? ch[w].src_bytes : kLzWindow;
    const uint32_t cap = ch[w].dst_capacity;
    const uint8_t* src = gsrc;
    if constexpr (STAGE) {
      for (uint32_t i = lane; i < len; i += kLzThreads) stage[i] = gsrc[i];
      src = stage;
    }
    for (uint32_t i = lane; i < (1u << kLzHashLog); i += kLzThreads) table[i] = 0xFFFF;
    __syncthreads();
    uint32_t op = 0, anchor = 0, ip = 0;
    int32_t status = 0;
    const uint32_t match_limit = len > kLzMfLimit ? len - kLzMfLimit : 0;
    const uint32_t end_match = len > kLzLastLiterals ? len - kLzLastLiterals : 0;
    while (ip < match_limit) {
      const uint32_t pos = ip + lane;
      uint32_t cand = 0xFFFFFFFFu, mlen = 0, h = 0;
      if (pos < match_limit) {
        const uint32_t v = lzb_read32<STAGE>(src + pos);
        h = lz_hash(v);
        const uint32_t c = table[h];
        if (c != 0xFFFF && c < pos && pos - c <= 65535 && lzb_read32<STAGE>(src + c) == v) {
          cand = c;
          mlen = kLzMinMatch;
          while (pos + mlen + 4 <= end_match && lzb_read32<STAGE>(src + c + mlen) == lzb_read32<STAGE>(src + pos + mlen))
            mlen += 4;
          while (pos + mlen < end_match && src[c + mlen] == src[pos + mlen]) ++mlen;
        }
      }
      __syncthreads();
      if (pos < match_limit) table[h] = (uint16_t)pos;  // last writer wins: any entry is verified
      __syncthreads();
      unsigned long long m = __ballot(cand != 0xFFFFFFFFu);
      if (m == 0) { ip += kLzThreads; continue; }
      // uniform greedy walk: take the first hit at/after the end of the last taken match
      unsigned long long sel = 0;
      uint32_t my_lit = 0, last_end = ip, prev_end = anchor;
      while (m) {
        const int g = __ffsll((long long)m) - 1;
        const uint32_t gml = __shfl(mlen, g);
        if (lane == g) my_lit = prev_end;
        sel |= 1ull << g;
        prev_end = last_end = ip + g + gml;
        const uint32_t skip = last_end - ip;       // hits before last_end overlap the match (skip > g)
        m = skip >= 64 ? 0ull : (m & (~0ull << skip));
      }
      const bool mine = (sel >> lane) & 1ull;
      const uint32_t lit = mine ? pos - my_lit : 0;
      const uint32_t need = mine ? 1 + lz_len_bytes(lit) + lit + 2 + lz_len_bytes(mlen - 4) : 0;
      uint32_t incl = need;                          // wave inclusive prefix sum of sequence sizes
#pragma unroll
      for (int d = 1; d < kLzThreads; d <<= 1) {
        const uint32_t t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
      }
      const uint32_t total = __shfl(incl, kLzThreads - 1);
      if (op + total > cap) { status = -1; break; }
      const uint32_t o = op + incl - need;
      if (mine) {
        const uint32_t mcode = mlen - 4;
        dst[o] = (uint8_t)(((lit >= 15 ? 15 : lit) << 4) | (mcode >= 15 ? 15 : mcode));
        uint32_t q = lz_put_len(dst, o + 1, lit) + lit;
        const uint32_t moff = pos - cand;
        dst[q] = (uint8_t)(moff & 255);
        dst[q + 1] = (uint8_t)(moff >> 8);
        lz_put_len(dst, q + 2, mcode);
      }
      // literal runs, one selected sequence at a time, copied by the whole wave
      unsigned long long rest = sel;
      while (rest) {
        const int g = __ffsll((long long)rest) - 1;
        rest &= rest - 1;
        const uint32_t gl = __shfl(lit, g);
        if (gl == 0) continue;
        const uint32_t gs = __shfl(my_lit, g);
        const uint32_t go = __shfl(o, g) + 1 + lz_len_bytes(gl);
        for (uint32_t i = lane; i < gl; i += kLzThreads) dst[go + i] = src[gs + i];
      }
      op += total;
      anchor = prev_end;
      ip = last_end > ip + kLzThreads ? last_end : ip + kLzThreads;
    }
    if (status == 0) {
      const uint32_t lit = len - anchor;
      const uint32_t need = 1 + lz_len_bytes(lit) + lit;
      if (op + need > cap) {
        status = -1;
      } else {
        const uint32_t q = op + 1 + lz_len_bytes(lit);
        if (lane == 0) {
          dst[op] = (uint8_t)((lit >= 15 ? 15 : lit) << 4);
          lz_put_len(dst, op + 1, lit);
        }
        for (uint32_t i = lane; i < lit; i += kLzThreads) dst[q + i] = src[anchor + i];
        op = q + lit;
      }
    }
    if (lane == 0) out_sizes[w] = status ? -1 : (int32_t)op;
    __syncthreads();
  }
}

// Segmented encoder for batches too small to fill the chip (one wave per 64 KiB chunk leaves
// 1k chunks at one wave per SIMD, latency-bound).  Each chunk is cut into up to S segments of
// >= 4 KiB parsed by S independent waves: a wave first re-hashes the `warm` bytes before its
// segment into its own table (so matches into the preceding data are still found), then runs the
// batch parse over its segment with matches confined to it.  The first sequence's literal run of a
// segment depends on where the previous segments' parses ended, so a wave writes its sequences to
// scratch WITHOUT that first header + literals; the merge kernel places the segments back to back
// and writes each first header with the literal run joined across the boundary.  Output is the
// same standard LZ4 block; ratio differs from the one-wave parse only at segment boundaries.
struct LzSeg {
  uint32_t first_mpos;   // position of the segment's first match (0xFFFFFFFF: no match)
  uint32_t first_mcode;  // its match length - 4
  uint32_t bytes;        // scratch bytes (0xFFFFFFFF: overflow)
  uint32_t tail;         // anchor after the segment's last match
};
constexpr uint32_t kLzSegMin = 4096;

__device__ __forceinline__ uint32_t lz_seg_count(uint32_t len, int S) {
  const uint32_t k = len / kLzSegMin;
  return k == 0 ? 1u : (k < (uint32_t)S ? k : (uint32_t)S);
}

__device__ __forceinline__ void lz_seg_bounds(uint32_t len, uint32_t nseg, uint32_t s, uint32_t* b, uint32_t* e) {
  const uint32_t seg = ((len + nseg - 1) / nseg + 63) & ~63u;
  *b = s * seg < len ? s * seg : len;
  *e = (s + 1) * seg < len && s + 1 < nseg ? (s + 1) * seg : len;
}

__global__ __launch_bounds__(kLzThreads) void lz4_seg_parse_kernel(const Lz4Chunk* __restrict__ ch, int n, int S,
                                                                  uint8_t* __restrict__ scratch, uint32_t seg_cap,
                                                                  LzSeg* __restrict__ segs, uint32_t warm) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint16_t* table = reinterpret_cast<uint16_t*>(smem);                     // 8 KiB
  const int lane = threadIdx.x;
  for (int t = blockIdx.x; t < n * S; t += gridDim.x) {
    const int w = t / S, s = t - (t / S) * S;
    const uint8_t* __restrict__ src = reinterpret_cast<const uint8_t*>(ch[w].src);
    const uint32_t len = ch[w].src_bytes < kLzWindow ? ch[w].src_bytes : kLzWindow;
    const uint32_t nseg = lz_seg_count(len, S);
    if ((uint32_t)s >= nseg) {
      if (lane == 0) segs[t] = LzSeg{0xFFFFFFFFu, 0, 0, 0};
      continue;
    }
    uint32_t sb, se;
    lz_seg_bounds(len, nseg, (uint32_t)s, &sb, &se);
    const bool last = (uint32_t)s + 1 == nseg;
    uint8_t* __restrict__ dst = scratch + (size_t)t * seg_cap;
    for (uint32_t i = lane; i < (1u << kLzHashLog); i += kLzThreads) table[i] = 0xFFFF;
    __syncthreads();
    for (uint32_t p = (sb > warm ? sb - warm : 0) + lane; p < sb; p += kLzThreads)
      table[lz_hash(lzb_read32<false>(src + p))] = (uint16_t)p;
    __syncthreads();
    // a match starts before match_limit and ends by end_match; inner segments keep their
    // matches inside the segment (the block-end rules only bind the last one)
    const uint32_t match_limit = last ? (len > kLzMfLimit ? len - kLzMfLimit : 0) : se - 3;
    const uint32_t end_match = last ? (len > kLzLastLiterals ? len - kLzLastLiterals : 0) : se;
    uint32_t op = 0, anchor = sb, ip = sb;
    bool have_first = false, overflow = false;
    uint32_t first_mpos = 0xFFFFFFFFu, first_mcode = 0;
    while (ip < match_limit) {
      const uint32_t pos = ip + lane;
      uint32_t cand = 0xFFFFFFFFu, mlen = 0, h = 0;
      if (pos < match_limit) {
        const uint32_t v = lzb_read32<false>(src + pos);
        h = lz_hash(v);
        const uint32_t c = table[h];
        if (c != 0xFFFF && c < pos && pos - c <= 65535 && lzb_read32<false>(src + c) == v) {
          cand = c;
          mlen = kLzMinMatch;
          while (pos + mlen + 4 <= end_match && lzb_read32<false>(src + c + mlen) == lzb_read32<false>(src + pos + mlen))
            mlen += 4;
          while (pos + mlen < end_match && src[c + mlen] == src[pos + mlen]) ++mlen;
        }
      }
      __syncthreads();
      if (pos < match_limit) table[h] = (uint16_t)pos;
      __syncthreads();
      unsigned long long m = __ballot(cand != 0xFFFFFFFFu);
      if (m == 0) { ip += kLzThreads; continue; }
      unsigned long long sel = 0;
      uint32_t my_lit = 0, last_end = ip, prev_end = anchor;
      while (m) {
        const int g = __ffsll((long long)m) - 1;
        const uint32_t gml = __shfl(mlen, g);
        if (lane == g) my_lit = prev_end;
        sel |= 1ull << g;
        prev_end = last_end = ip + g + gml;
        const uint32_t skip = last_end - ip;
        m = skip >= 64 ? 0ull : (m & (~0ull << skip));
      }
      const int g0 = __ffsll((long long)sel) - 1;
      const bool is_first = !have_first && lane == g0;   // header + literals written by the merge
      if (!have_first) {
        first_mpos = ip + g0;
        first_mcode = __shfl(mlen, g0) - 4;
        have_first = true;
      }
      const bool mine = (sel >> lane) & 1ull;
      const uint32_t lit = mine && !is_first ? pos - my_lit : 0;
      const uint32_t need = !mine ? 0
                          : is_first ? 2 + lz_len_bytes(mlen - 4)
                                     : 1 + lz_len_bytes(lit) + lit + 2 + lz_len_bytes(mlen - 4);
      uint32_t incl = need;
#pragma unroll
      for (int d = 1; d < kLzThreads; d <<= 1) {
        const uint32_t tt = __shfl_up(incl, d);
        if (lane >= d) incl += tt;
      }
      const uint32_t total = __shfl(incl, kLzThreads - 1);
      if (op + total > seg_cap) { overflow = true; break; }
      const uint32_t o = op + incl - need;
      if (mine) {
        const uint32_t mcode = mlen - 4;
        const uint32_t moff = pos - cand;
        uint32_t q = o;
        if (!is_first) {
          dst[q] = (uint8_t)(((lit >= 15 ? 15 : lit) << 4) | (mcode >= 15 ? 15 : mcode));
          q = lz_put_len(dst, q + 1, lit) + lit;
        }
        dst[q] = (uint8_t)(moff & 255);
        dst[q + 1] = (uint8_t)(moff >> 8);
        lz_put_len(dst, q + 2, mcode);
      }
      unsigned long long rest = sel;
      while (rest) {
        const int g = __ffsll((long long)rest) - 1;
        rest &= rest - 1;
        const uint32_t gl = __shfl(lit, g);
        if (gl == 0) continue;
        const uint32_t gs = __shfl(my_lit, g);
        const uint32_t go = __shfl(o, g) + 1 + lz_len_bytes(gl);
        for (uint32_t i = lane; i < gl; i += kLzThreads) dst[go + i] = src[gs + i];
      }
      op += total;
      anchor = prev_end;
      ip = last_end > ip + kLzThreads ? last_end : ip + kLzThreads;
    }
    if (lane == 0) segs[t] = LzSeg{first_mpos, first_mcode, overflow ? 0xFFFFFFFFu : op, anchor};
    __syncthreads();
  }
}

constexpr int kLzMergeThreads = 256;
constexpr int kLzMaxSeg = 16;

__global__ __launch_bounds__(kLzMergeThreads) void lz4_seg_merge_kernel(const Lz4Chunk* __restrict__ ch, int n, int S,
                                                                       const uint8_t* __restrict__ scratch,
                                                                       uint32_t seg_cap, const LzSeg* __restrict__ segs,
                                                                       int32_t* __restrict__ out_sizes) {
  __shared__ uint32_t s_off[kLzMaxSeg], s_p[kLzMaxSeg], s_fin[3];
  __shared__ int s_bad;
  const int tid = threadIdx.x;
  for (int w = blockIdx.x; w < n; w += gridDim.x) {
    const uint8_t* __restrict__ src = reinterpret_cast<const uint8_t*>(ch[w].src);
    uint8_t* __restrict__ dst = reinterpret_cast<uint8_t*>(ch[w].dst);
    const uint32_t len = ch[w].src_bytes < kLzWindow ? ch[w].src_bytes : kLzWindow;
    const LzSeg* sg = segs + (size_t)w * S;
    if (tid == 0) {
      uint32_t P = 0, out = 0;
      int bad = 0;
      for (int s = 0; s < S; ++s) {
        const LzSeg g = sg[s];
        if (g.bytes == 0xFFFFFFFFu) bad = 1;
        if (g.first_mpos == 0xFFFFFFFFu) { s_off[s] = 0xFFFFFFFFu; continue; }
        const uint32_t lit = g.first_mpos - P;
        s_off[s] = out;
        s_p[s] = P;
        out += 1 + lz_len_bytes(lit) + lit + g.bytes;
        P = g.tail;
      }
      const uint32_t lit = len - P;
      s_fin[0] = P;
      s_fin[1] = out;
      out += 1 + lz_len_bytes(lit) + lit;
      s_fin[2] = out;
      s_bad = bad || out > ch[w].dst_capacity;
    }
    __syncthreads();
    if (s_bad) {
      if (tid == 0) out_sizes[w] = -1;
      __syncthreads();
      continue;
    }
    for (int s = 0; s < S; ++s) {
      if (s_off[s] == 0xFFFFFFFFu) continue;
      const LzSeg g = sg[s];
      const uint32_t P = s_p[s], lit = g.first_mpos - P, o = s_off[s];
      if (tid == 0) {
        dst[o] = (uint8_t)(((lit >= 15 ? 15 : lit) << 4) | (g.first_mcode >= 15 ? 15 : g.first_mcode));
        lz_put_len(dst, o + 1, lit);
      }
      const uint32_t q = o + 1 + lz_len_bytes(lit);
      for (uint32_t i = tid; i < lit; i += kLzMergeThreads) dst[q + i] = src[P + i];
      const uint8_t* sc = scratch + ((size_t)w * S + s) * seg_cap;
      for (uint32_t i = tid; i < g.bytes; i += kLzMergeThreads) dst[q + lit + i] = sc[i];
    }
    {
      const uint32_t P = s_fin[0], o = s_fin[1], lit = len - P;
      if (tid == 0) {
        dst[o] = (uint8_t)((lit >= 15 ? 15 : lit) << 4);
        lz_put_len(dst, o + 1, lit);
      }
      const uint32_t q = o + 1 + lz_len_bytes(lit);
      for (uint32_t i = tid; i < lit; i += kLzMergeThreads) dst[q + i] = src[P + i];
    }
    if (tid == 0) out_sizes[w] = (int32_t)s_fin[2];
    __syncthreads();
  }
}

static hipError_t launch_lz4_compress_segmented(const Lz4Chunk* chunks, int n, int32_t* out_sizes, int S,
                                                hipStream_t stream) {
  S = S < 1 ? 1 : (S > kLzMaxSeg ? kLzMaxSeg : S);
  // seg_cap: LZ4's bound for the largest segment (64 KiB / S rounded up to 64, or 4 KiB minimum)
  const uint32_t seg = std::max<uint32_t>(kLzSegMin * 2, ((kLzWindow + S - 1) / S + 63) & ~63u);
  const uint32_t seg_cap = (seg + seg / 255 + 16 + 15) & ~15u;
  const size_t nseg = (size_t)n * S;
  void* mem = nullptr;
  hipError_t e = hipMallocAsync(&mem, nseg * seg_cap + nseg * sizeof(LzSeg), stream);
  if (e != hipSuccess) return e;
  uint8_t* scratch = static_cast<uint8_t*>(mem);
  LzSeg* segs = reinterpret_cast<LzSeg*>(scratch + nseg * seg_cap);
  const size_t table = sizeof(uint16_t) << kLzHashLog;
  hipLaunchKernelGGL(lz4_seg_parse_kernel, dim3((unsigned)std::min<size_t>(nseg, 65536)), dim3(kLzThreads), table,
                     stream, chunks, n, S, scratch, seg_cap, segs, 4096u);
  e = hipGetLastError();
  if (e == hipSuccess) {
    hipLaunchKernelGGL(lz4_seg_merge_kernel, dim3((unsigned)std::min(n, 65536)), dim3(kLzMergeThreads), 0, stream,
                       chunks, n, S, scratch, seg_cap, segs, out_sizes);
    e = hipGetLastError();
  }
  const hipError_t f = hipFreeAsync(mem, stream);
  return e != hipSuccess ? e : f;
}

// 0: one sequence per probe batch (lz4_compress_kernel); 1: batch parse, chunk in LDS;
// 2: batch parse reading the chunk from global/L2 (8 KiB LDS per wave); 3: segmented parse
// (4 waves per chunk) + merge; 4 (default): segmented below 2048 chunks (S = 4096 waves / n,
// 2..8), batch parse above -- the batch parse fills the chip by itself there
static int g_lz4_encode_variant = 4;
void set_lz4_encode_variant(int v) { g_lz4_encode_variant = v; }

hipError_t launch_lz4_compress(const Lz4Chunk* chunks, int n, int32_t* out_sizes,
                               hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const size_t table = sizeof(uint16_t) << kLzHashLog;
  if (g_lz4_encode_variant == 0) {
    const unsigned grid = (unsigned)std::min(n, 4096);
    hipLaunchKernelGGL(lz4_compress_kernel, dim3(grid), dim3(kLzThreads), kLzWindow + table, stream,
                       chunks, n, out_sizes);
  } else if (g_lz4_encode_variant == 1) {
    const unsigned grid = (unsigned)std::min(n, 4096);
    hipLaunchKernelGGL((lz4_compress_batch_kernel<true>), dim3(grid), dim3(kLzThreads), table + kLzWindow,
                       stream, chunks, n, out_sizes);
  } else if (g_lz4_encode_variant == 3) {
    return launch_lz4_compress_segmented(chunks, n, out_sizes, 4, stream);
  } else if (g_lz4_encode_variant == 4 && n < 2048) {
    return launch_lz4_compress_segmented(chunks, n, out_sizes, std::max(2, std::min(8, 4096 / n)), stream);
  } else {
    const unsigned grid = (unsigned)std::min(n, 65536);
    hipLaunchKernelGGL((lz4_compress_batch_kernel<false>), dim3(grid), dim3(kLzThreads), table, stream,
                       chunks, n, out_sizes);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Synthetic data generator (bench / tests): splitmix64 of (seed, 8-byte word index).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void fill_pattern_kernel(uint8_t* __restrict__ dst, uint64_t bytes,
                                                           uint64_t seed, uint64_t word_offset) {
  const uint64_t nwords = bytes >> 3;
  uint64_t* d = reinterpret_cast<uint64_t*>(dst);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords;
       i += (uint64_t)gridDim.x * blockDim.x)
    d[i] = splitmix64(seed ^ ((i + word_offset) * 0xD1B54A32D192ED03ull));
  const uint64_t tail = bytes & 7;
  if (tail && blockIdx.x == 0 && threadIdx.x < tail) {
    const uint64_t w = splitmix64(seed ^ ((nwords + word_offset) * 0xD1B54A32D192ED03ull));
    dst[(nwords << 3) + threadIdx.x] = (uint8_t)(w >> (8 * threadIdx.x));
  }
}

hipError_t launch_fill_pattern(uint8_t* dst, uint64_t bytes, uint64_t seed, uint64_t word_offset,
                               hipStream_t stream) {
  if (bytes == 0) return hipSuccess;
  if (((uintptr_t)dst & 7) != 0) return hipErrorInvalidValue;
  const uint64_t words = (bytes + 7) >> 3;
  const unsigned grid = (unsigned)std::min<uint64_t>((words + 255) / 256, 4096);
  hipLaunchKernelGGL(fill_pattern_kernel, dim3(grid), dim3(256), 0, stream, dst, bytes, seed,
                     word_offset);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K9: client page cache -- fused device hash lookup + page gather.
//
// Grid (x = request, y = chunk of the page).  Wave 0 of each workgroup resolves the key: every
// lane loads one of 64 consecutive table entries (16 B each, one coalesced 1 KiB read), a ballot
// finds the first matching key and the first empty entry; a match before the first empty entry
// is a hit (linear probing never places a key past an empty slot; tombstones keep probing).  The
// slot is broadcast through LDS and the 256 lanes copy this workgroup's chunk with 16-B vectors.
// ---------------------------------------------------------------------------------------------
constexpr int kPgThreads = 256;
constexpr uint64_t kPgChunk = 128 * 1024;

template <int LP>
__global__ __launch_bounds__(kPgThreads) void page_lookup_gather_kernel(PageGatherArgs a) {
  __shared__ int32_t s_slot;
  __shared__ uint32_t s_len;
  const int tid = threadIdx.x;
  const uint64_t chunk0 = (uint64_t)blockIdx.y * kPgChunk;
  for (uint32_t req = blockIdx.x; req < a.n; req += gridDim.x) {
    if (tid < 64) {
      const uint64_t key = a.keys[req];
      const uint64_t h = page_key_hash(key);
      int32_t slot = -1;
      uint32_t len = 0;
      for (uint64_t probe = 0; probe <= a.mask; probe += 64) {
        const PageTableEntry e = a.table[(h + probe + tid) & a.mask];
        const uint64_t hit = __ballot(e.key == key);
        const uint64_t empty = __ballot(e.key == kPageKeyEmpty);
        if (hit) {
          const int first_hit = __ffsll((unsigned long long)hit) - 1;
          const int first_empty = empty ? __ffsll((unsigned long long)empty) - 1 : 64;
          if (first_hit < first_empty) {
            slot = __shfl(e.slot, first_hit, 64);
            len = __shfl(e.len, first_hit, 64);
          }
          break;
        }
        if (empty) break;
      }
      if (tid == 0) {
        s_slot = slot;
        s_len = len;
      }
    }
    __syncthreads();
    const int32_t slot = s_slot;
    const uint64_t len = s_len;
    if (blockIdx.y == 0 && tid == 0) {
      a.slot_out[req] = slot;
      a.len_out[req] = slot >= 0 ? (uint32_t)len : 0u;
      if (slot >= 0 && a.stamps) a.stamps[slot] = a.epoch;
    }
    if (slot >= 0 && chunk0 < len) {
      const uint64_t rem = len - chunk0;
      const uint64_t n = rem < kPgChunk ? rem : kPgChunk;
      const uint64_t src = (uint64_t)(a.arena + (uint64_t)slot * a.page_size + chunk0);
      const uint64_t dst = (uint64_t)(a.dst + (uint64_t)req * a.dst_stride + chunk0);
      copy_range<4, LP, 0>(src, dst, n, tid);
    }
    __syncthreads();      // s_slot is rewritten by the next request of this workgroup
  }
}

// Small pages (<= g_pg_small_max, 16-B aligned rows): one wave per request and kPgPW requests per wave,
// no LDS and no barriers.  The wave first issues the keys and the first 64-entry probe window of
// all kPgPW requests back to back (independent loads in flight together), resolves them with
// ballots (a chain longer than 64 entries falls back to the loop), then copies the pages with
// kPgPW x kPgUnr 16-B loads in flight per lane before the stores.
// Page sizes up to g_pg_small_max take the wave-per-request kernel (tools/page_cache_bench.py
// --variants both on MI355X: 4 KiB pages 2.56 vs 2.40 TB/s, 64 KiB pages 2.25 vs 2.59 TB/s).
static uint64_t g_pg_small_max = 16 * 1024;
void set_page_gather_small_max(uint64_t bytes) { g_pg_small_max = bytes; }
// Wave-kernel variant (requests per wave, 16-B loads per lane per page, store policy):
// 0 = 4/4/plain, 1 = 8/2/plain, 2 = 4/4/nontemporal, 3 = 8/4/plain, 4 = 4/4/nontemporal loads,
// 5 = 4/4/nontemporal loads and stores.
static int g_pg_wave_variant = 2;  // nt stores: 4 KiB 3.03 vs 2.56 TB/s, 16 KiB 2.64 vs 2.42 TB/s (profiles/r1_page_cache_wave.jsonl)
void set_page_gather_wave_variant(int v) { g_pg_wave_variant = v; }
// chunk kernel (pages above g_pg_small_max): 0 = cached loads, 1 = nontemporal loads, -1 (default)
// = nontemporal loads up to 512 KiB pages (64 KiB pages over an 8 GiB cache: 2.57 -> 2.72 TB/s;
// 2 MiB pages equal within noise; profiles/r3_page_gather_ntload.jsonl)
static int g_pg_chunk_variant = -1;
void set_page_gather_chunk_variant(int v) { g_pg_chunk_variant = v; }

__device__ __forceinline__ void pg_resolve(const PageGatherArgs& a, uint64_t key, uint64_t h,
                                           PageTableEntry e, int lane, int32_t& slot, uint32_t& len) {
  slot = -1;
  len = 0;
  for (uint64_t probe = 0;;) {
    const uint64_t hit = __ballot(e.key == key);
    const uint64_t empty = __ballot(e.key == kPageKeyEmpty);
    if (hit) {
      const int fh = __ffsll((unsigned long long)hit) - 1;
      const int fe = empty ? __ffsll((unsigned long long)empty) - 1 : 64;
      if (fh < fe) {
        slot = __shfl(e.slot, fh, 64);
        len = __shfl(e.len, fh, 64);
      }
      return;
    }
    if (empty) return;
    probe += 64;
    if (probe > a.mask) return;
    e = a.table[(h + probe + lane) & a.mask];
  }
}

template <int kPgPW, int kPgUnr, int SP, int LP = 0>
__global__ __launch_bounds__(256) void page_lookup_gather_small_kernel(PageGatherArgs a) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * 4;
  for (uint32_t r0 = wave * kPgPW; r0 < a.n; r0 += nwaves * kPgPW) {
    uint64_t key[kPgPW], h[kPgPW];
    PageTableEntry e[kPgPW];
#pragma unroll
    for (int u = 0; u < kPgPW; ++u) key[u] = (r0 + u < a.n) ? a.keys[r0 + u] : kPageKeyEmpty;
#pragma unroll
    for (int u = 0; u < kPgPW; ++u) {
      h[u] = page_key_hash(key[u]);
      e[u] = a.table[(h[u] + lane) & a.mask];
    }
    int32_t slot[kPgPW];
    uint32_t len[kPgPW];
    uint32_t maxlen = 0;
#pragma unroll
    for (int u = 0; u < kPgPW; ++u) {
      slot[u] = -1;
      len[u] = 0;
      if (r0 + u < a.n) pg_resolve(a, key[u], h[u], e[u], lane, slot[u], len[u]);
      if (slot[u] < 0) len[u] = 0;
      maxlen = len[u] > maxlen ? len[u] : maxlen;
    }
    if (lane == 0) {
#pragma unroll
      for (int u = 0; u < kPgPW; ++u) {
        if (r0 + u >= a.n) continue;
        a.slot_out[r0 + u] = slot[u];
        a.len_out[r0 + u] = len[u];
        if (slot[u] >= 0 && a.stamps) a.stamps[slot[u]] = a.epoch;
      }
    }
    const uint8_t* src[kPgPW];
    uint8_t* dst[kPgPW];
#pragma unroll
    for (int u = 0; u < kPgPW; ++u) {
      src[u] = a.arena + (uint64_t)(slot[u] < 0 ? 0 : slot[u]) * a.page_size;
      dst[u] = a.dst + (uint64_t)(r0 + u) * a.dst_stride;
    }
    for (uint64_t base = 0; base + 16 <= maxlen; base += 64 * 16 * kPgUnr) {
      u32x4 v[kPgPW][kPgUnr];
#pragma unroll
      for (int u = 0; u < kPgPW; ++u)
#pragma unroll
        for (int k = 0; k < kPgUnr; ++k) {
          const uint64_t off = base + (uint64_t)(k * 64 + lane) * 16;
          if (off + 16 <= len[u]) v[u][k] = ld16<LP>(reinterpret_cast<const u32x4*>(src[u] + off));
        }
#pragma unroll
      for (int u = 0; u < kPgPW; ++u)
#pragma unroll
        for (int k = 0; k < kPgUnr; ++k) {
          const uint64_t off = base + (uint64_t)(k * 64 + lane) * 16;
          if (off + 16 <= len[u]) st16<SP>(reinterpret_cast<u32x4*>(dst[u] + off), v[u][k]);
        }
    }
#pragma unroll
    for (int u = 0; u < kPgPW; ++u) {
      const uint32_t full = len[u] & ~15u;
      if ((uint32_t)lane < len[u] - full) dst[u][full + lane] = src[u][full + lane];
    }
  }
}

hipError_t launch_page_lookup_gather(const PageGatherArgs& a, hipStream_t stream) {
  if (a.n == 0) return hipSuccess;
  if ((a.mask & (a.mask + 1)) != 0) return hipErrorInvalidValue;
  if (a.page_size <= g_pg_small_max && a.page_size % 16 == 0 && a.dst_stride % 16 == 0 &&
      ((uintptr_t)a.dst & 15) == 0 && ((uintptr_t)a.arena & 15) == 0) {
    const int pw = (g_pg_wave_variant == 1 || g_pg_wave_variant == 3) ? 8 : 4;
    const uint64_t waves = (a.n + pw - 1) / pw;
    const unsigned grid = (unsigned)std::min<uint64_t>((waves + 3) / 4, 8192);
#define AMDX_PG(PW, U, S) hipLaunchKernelGGL((page_lookup_gather_small_kernel<PW, U, S>), dim3(grid), dim3(256), 0, stream, a)
    switch (g_pg_wave_variant) {
      case 1: AMDX_PG(8, 2, 0); break;
      case 2: AMDX_PG(4, 4, 1); break;
      case 3: AMDX_PG(8, 4, 0); break;
      case 4: hipLaunchKernelGGL((page_lookup_gather_small_kernel<4, 4, 0, 1>), dim3(grid), dim3(256), 0, stream, a); break;
      case 5: hipLaunchKernelGGL((page_lookup_gather_small_kernel<4, 4, 1, 1>), dim3(grid), dim3(256), 0, stream, a); break;
      default: AMDX_PG(4, 4, 0); break;
    }
#undef AMDX_PG
    return hipGetLastError();
  }
  const unsigned gy = (unsigned)std::max<uint64_t>(1, (a.page_size + kPgChunk - 1) / kPgChunk);
  const unsigned gx = (unsigned)std::min<uint64_t>(a.n, 65535);
  if (g_pg_chunk_variant == 1 || (g_pg_chunk_variant < 0 && a.page_size <= (512u << 10)))
    hipLaunchKernelGGL(page_lookup_gather_kernel<1>, dim3(gx, gy), dim3(kPgThreads), 0, stream, a);
  else
    hipLaunchKernelGGL(page_lookup_gather_kernel<0>, dim3(gx, gy), dim3(kPgThreads), 0, stream, a);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void page_table_update_kernel(PageTableEntry* __restrict__ table,
                                                                const uint64_t* __restrict__ idx,
                                                                const PageTableEntry* __restrict__ e,
                                                                uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    table[idx[i]] = e[i];
}

hipError_t launch_page_table_update(PageTableEntry* table, const uint64_t* idx,
                                    const PageTableEntry* entries, uint32_t n, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const unsigned grid = std::min<unsigned>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(page_table_update_kernel, dim3(grid), dim3(256), 0, stream, table, idx, entries, n);
  return hipGetLastError();
}

}  // namespace amdx
