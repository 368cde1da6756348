#include "cpu_codecs.h"

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

namespace amdx {

static constexpr uint32_t kPoly = 0x82F63B78u;
static uint32_t g_tab[8][256];
static std::once_flag g_once;

static void init_tables() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
    g_tab[0][i] = c;
  }
  for (int t = 1; t < 8; ++t)
    for (uint32_t i = 0; i < 256; ++i) g_tab[t][i] = (g_tab[t - 1][i] >> 8) ^ g_tab[0][g_tab[t - 1][i] & 0xFF];
}

#if defined(__x86_64__)
// The x86 CRC32 instruction computes exactly this polynomial (Castagnoli): 8 bytes per
// instruction instead of eight table lookups (the HDFS packet checksums, the CPU-side CRC of
// pulled blocks and the shell's checksum all run here).
__attribute__((target("sse4.2"))) static uint32_t crc32c_x86(const uint8_t* p, size_t n, uint32_t c) {
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    c = __builtin_ia32_crc32qi(c, *p++);
    --n;
  }
  uint64_t c64 = c;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c64 = __builtin_ia32_crc32di(c64, v);
    p += 8;
    n -= 8;
  }
  c = (uint32_t)c64;
  while (n--) c = __builtin_ia32_crc32qi(c, *p++);
  return c;
}
static bool have_sse42() {
  static const bool ok = [] {
    __builtin_cpu_init();
    return __builtin_cpu_supports("sse4.2") != 0;
  }();
  return ok;
}
#endif

uint32_t crc32c_sw(const void* data, size_t n, uint32_t crc) {
#if defined(__x86_64__)
  if (have_sse42()) return ~crc32c_x86(static_cast<const uint8_t*>(data), n, ~crc);
#endif
  std::call_once(g_once, init_tables);
  const uint8_t* p = static_cast<const uint8_t*>(data);
  uint32_t c = ~crc;
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    c = (c >> 8) ^ g_tab[0][(c ^ *p++) & 0xFF];
    --n;
  }
  while (n >= 8) {
    uint32_t a, b;
    std::memcpy(&a, p, 4);
    std::memcpy(&b, p + 4, 4);
    a ^= c;
    c = g_tab[7][a & 255] ^ g_tab[6][(a >> 8) & 255] ^ g_tab[5][(a >> 16) & 255] ^ g_tab[4][a >> 24] ^
        g_tab[3][b & 255] ^ g_tab[2][(b >> 8) & 255] ^ g_tab[1][(b >> 16) & 255] ^ g_tab[0][b >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ g_tab[0][(c ^ *p++) & 0xFF];
  return ~c;
}

static uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ kPoly : b >> 1;
  }
  return p;
}

static uint32_t x8nmodp(uint64_t n) {
  uint32_t p = 1u << 31;
  uint32_t x2k = 1u << 30;  // x^1
  uint64_t e = n << 3;
  while (e) {
    if (e & 1) p = multmodp(x2k, p);
    x2k = multmodp(x2k, x2k);
    e >>= 1;
  }
  return p;
}

uint32_t crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
  return multmodp(x8nmodp(len_b), crc_a) ^ crc_b;
}

static inline void put_be32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
}

#if defined(__x86_64__)
// Four full chunks of `bpc` bytes (bpc % 8 == 0) at once: independent CRC32 chains overlap the
// instruction's 3-cycle latency.
__attribute__((target("sse4.2"))) static void crc32c_x4(const uint8_t* p, size_t bpc, uint32_t out[4]) {
  uint64_t c0 = 0xFFFFFFFFu, c1 = 0xFFFFFFFFu, c2 = 0xFFFFFFFFu, c3 = 0xFFFFFFFFu;
  const uint8_t *p0 = p, *p1 = p + bpc, *p2 = p + 2 * bpc, *p3 = p + 3 * bpc;
  for (size_t i = 0; i < bpc; i += 8) {
    uint64_t v0, v1, v2, v3;
    std::memcpy(&v0, p0 + i, 8);
    std::memcpy(&v1, p1 + i, 8);
    std::memcpy(&v2, p2 + i, 8);
    std::memcpy(&v3, p3 + i, 8);
    c0 = __builtin_ia32_crc32di(c0, v0);
    c1 = __builtin_ia32_crc32di(c1, v1);
    c2 = __builtin_ia32_crc32di(c2, v2);
    c3 = __builtin_ia32_crc32di(c3, v3);
  }
  out[0] = ~(uint32_t)c0;
  out[1] = ~(uint32_t)c1;
  out[2] = ~(uint32_t)c2;
  out[3] = ~(uint32_t)c3;
}
#endif

void crc32c_chunks_be(const uint8_t* data, size_t n, uint32_t bpc, uint8_t* out) {
  size_t off = 0, i = 0;
#if defined(__x86_64__)
  if (have_sse42() && bpc % 8 == 0) {
    uint32_t c[4];
    for (; off + 4 * (size_t)bpc <= n; off += 4 * (size_t)bpc, i += 4) {
      crc32c_x4(data + off, bpc, c);
      for (int k = 0; k < 4; ++k) put_be32(out + 4 * (i + k), c[k]);
    }
  }
#endif
  for (; off < n; off += bpc, ++i) put_be32(out + 4 * i, crc32c_sw(data + off, std::min<size_t>(bpc, n - off), 0));
}

int64_t crc32c_chunks_verify(const uint8_t* data, size_t n, uint32_t bpc, const uint8_t* expect) {
  uint8_t got[4 * 64];
  const size_t group = 64 * (size_t)bpc;     // chunks per pass
  for (size_t off = 0; off < n; off += group) {
    const size_t m = std::min(group, n - off);
    crc32c_chunks_be(data + off, m, bpc, got);
    const size_t chunks = (m + bpc - 1) / bpc;
    if (std::memcmp(got, expect + 4 * (off / bpc), 4 * chunks) != 0) {
      for (size_t k = 0; k < chunks; ++k)
        if (std::memcmp(got + 4 * k, expect + 4 * (off / bpc + k), 4) != 0) return (int64_t)(off / bpc + k);
    }
  }
  return -1;
}

// ------------------------------------------------------------------------------------------
// LZ4 block format.
// ------------------------------------------------------------------------------------------
static constexpr int kHashLog = 14;
static constexpr size_t kMinMatch = 4, kLastLiterals = 5, kMfLimit = 12;

static inline uint32_t rd32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
static inline uint32_t hash4(uint32_t v) { return (v * 2654435761u) >> (32 - kHashLog); }

size_t lz4_compress_bound(size_t n) { return n + n / 255 + 16; }

static inline bool put_len(uint8_t*& op, uint8_t* oend, size_t len) {
  while (len >= 255) {
    if (op >= oend) return false;
    *op++ = 255;
    len -= 255;
  }
  if (op >= oend) return false;
  *op++ = static_cast<uint8_t>(len);
  return true;
}

int64_t lz4_compress_block(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap) {
  std::vector<int64_t> table(size_t(1) << kHashLog, -1);
  uint8_t* op = dst;
  uint8_t* const oend = dst + dst_cap;
  size_t anchor = 0, ip = 0;
  const size_t match_limit = n > kMfLimit ? n - kMfLimit : 0;
  const size_t end_match = n > kLastLiterals ? n - kLastLiterals : 0;
  while (ip < match_limit) {
    const uint32_t v = rd32(src + ip);
    const uint32_t h = hash4(v);
    const int64_t c = table[h];
    table[h] = static_cast<int64_t>(ip);
    if (c < 0 || ip - static_cast<size_t>(c) > 65535 || rd32(src + c) != v) {
      ++ip;
      continue;
    }
    size_t ml = kMinMatch;
    while (ip + ml < end_match && src[c + ml] == src[ip + ml]) ++ml;
    const size_t lit = ip - anchor;
    if (op >= oend) return -1;
    uint8_t* tok = op++;
    const size_t mcode = ml - kMinMatch;
    *tok = static_cast<uint8_t>(((lit >= 15 ? 15 : lit) << 4) | (mcode >= 15 ? 15 : mcode));
    if (lit >= 15 && !put_len(op, oend, lit - 15)) return -1;
    if (op + lit + 2 > oend) return -1;
    std::memcpy(op, src + anchor, lit);
    op += lit;
    const size_t off = ip - static_cast<size_t>(c);
    *op++ = static_cast<uint8_t>(off & 255);
    *op++ = static_cast<uint8_t>(off >> 8);
    if (mcode >= 15 && !put_len(op, oend, mcode - 15)) return -1;
    ip += ml;
    anchor = ip;
  }
  const size_t lit = n - anchor;
  if (op >= oend) return -1;
  *op++ = static_cast<uint8_t>((lit >= 15 ? 15 : lit) << 4);
  if (lit >= 15 && !put_len(op, oend, lit - 15)) return -1;
  if (op + lit > oend) return -1;
  std::memcpy(op, src + anchor, lit);
  op += lit;
  return op - dst;
}

int64_t lz4_decompress_block(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap) {
  const uint8_t* ip = src;
  const uint8_t* const iend = src + n;
  size_t op = 0;
  while (ip < iend) {
    const uint32_t token = *ip++;
    size_t lit = token >> 4;
    if (lit == 15) {
      uint32_t b;
      do {
        if (ip >= iend) return -1;
        b = *ip++;
        lit += b;
      } while (b == 255);
    }
    if (static_cast<size_t>(iend - ip) < lit || op + lit > dst_cap) return -2;
    std::memcpy(dst + op, ip, lit);
    ip += lit;
    op += lit;
    if (ip >= iend) break;
    if (iend - ip < 2) return -3;
    const size_t off = ip[0] | (static_cast<size_t>(ip[1]) << 8);
    ip += 2;
    size_t ml = token & 15;
    if (ml == 15) {
      uint32_t b;
      do {
        if (ip >= iend) return -4;
        b = *ip++;
        ml += b;
      } while (b == 255);
    }
    ml += kMinMatch;
    if (off == 0 || off > op || op + ml > dst_cap) return -5;
    for (size_t i = 0; i < ml; ++i) dst[op + i] = dst[op - off + i];
    op += ml;
  }
  return static_cast<int64_t>(op);
}

}  // namespace amdx
