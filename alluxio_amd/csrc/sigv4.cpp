// SHA-256 (FIPS 180-4), HMAC (RFC 2104) and AWS SigV4 header signing (see sigv4.h).
#include "sigv4.h"

#include <cstring>
#include <ctime>

namespace amdx {

namespace {

constexpr uint32_t kK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

std::string hex(const uint8_t* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; ++i) {
    s[2 * i] = d[p[i] >> 4];
    s[2 * i + 1] = d[p[i] & 15];
  }
  return s;
}

std::string hmac_raw(const std::string& key, const std::string& msg) {
  uint8_t out[32];
  hmac_sha256(key, msg, out);
  return std::string(reinterpret_cast<const char*>(out), 32);
}

}  // namespace

Sha256::Sha256() {
  static const uint32_t init[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  std::memcpy(h_, init, sizeof(h_));
}

void Sha256::block(const uint8_t* p) {
  uint32_t w[64];
  for (int i = 0; i < 16; ++i)
    w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) | ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
  for (int i = 16; i < 64; ++i) {
    const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
    const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h_[0], b = h_[1], c = h_[2], d = h_[3], e = h_[4], f = h_[5], g = h_[6], h = h_[7];
  for (int i = 0; i < 64; ++i) {
    const uint32_t t1 = h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + kK[i] + w[i];
    const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  h_[0] += a; h_[1] += b; h_[2] += c; h_[3] += d;
  h_[4] += e; h_[5] += f; h_[6] += g; h_[7] += h;
}

void Sha256::update(const void* data, size_t n) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  total_ += n;
  if (used_) {
    const size_t k = std::min(n, 64 - used_);
    std::memcpy(buf_ + used_, p, k);
    used_ += k;
    p += k;
    n -= k;
    if (used_ < 64) return;
    block(buf_);
    used_ = 0;
  }
  for (; n >= 64; p += 64, n -= 64) block(p);
  std::memcpy(buf_, p, n);
  used_ = n;
}

void Sha256::finish(uint8_t out[32]) {
  const uint64_t bits = total_ * 8;
  const uint8_t pad = 0x80;
  update(&pad, 1);
  const uint8_t zero[64] = {0};
  update(zero, (used_ <= 56) ? 56 - used_ : 120 - used_);
  uint8_t len[8];
  for (int i = 0; i < 8; ++i) len[i] = (uint8_t)(bits >> (56 - 8 * i));
  update(len, 8);
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (uint8_t)(h_[i] >> 24);
    out[4 * i + 1] = (uint8_t)(h_[i] >> 16);
    out[4 * i + 2] = (uint8_t)(h_[i] >> 8);
    out[4 * i + 3] = (uint8_t)h_[i];
  }
}

std::string sha256_hex(const void* p, size_t n) {
  Sha256 s;
  s.update(p, n);
  uint8_t out[32];
  s.finish(out);
  return hex(out, 32);
}

void hmac_sha256(const std::string& key, const std::string& msg, uint8_t out[32]) {
  uint8_t k[64] = {0};
  if (key.size() > 64) {
    Sha256 s;
    s.update(key.data(), key.size());
    s.finish(k);
  } else {
    std::memcpy(k, key.data(), key.size());
  }
  uint8_t ipad[64], opad[64];
  for (int i = 0; i < 64; ++i) {
    ipad[i] = k[i] ^ 0x36;
    opad[i] = k[i] ^ 0x5c;
  }
  uint8_t inner[32];
  Sha256 a;
  a.update(ipad, 64);
  a.update(msg.data(), msg.size());
  a.finish(inner);
  Sha256 b;
  b.update(opad, 64);
  b.update(inner, 32);
  b.finish(out);
}

std::string uri_encode_path(const std::string& path) {
  static const char* d = "0123456789ABCDEF";
  std::string o;
  o.reserve(path.size() + 16);
  for (unsigned char ch : path) {
    if ((ch >= 'A' && ch <= 'Z') || (ch >= 'a' && ch <= 'z') || (ch >= '0' && ch <= '9') || ch == '-' ||
        ch == '_' || ch == '.' || ch == '~' || ch == '/') {
      o.push_back((char)ch);
    } else {
      o.push_back('%');
      o.push_back(d[ch >> 4]);
      o.push_back(d[ch & 15]);
    }
  }
  return o;
}

std::string s3_header_lines(const S3Credentials& c, const std::string& method, const std::string& path,
                            const std::string& canonical_query, const std::string& payload_hash,
                            const std::string& amz_date_in) {
  std::string amz_date = amz_date_in;
  if (amz_date.empty()) {
    const std::time_t now = std::time(nullptr);
    std::tm tm{};
    gmtime_r(&now, &tm);
    char b[20];
    std::strftime(b, sizeof(b), "%Y%m%dT%H%M%SZ", &tm);
    amz_date = b;
  }
  std::string lines = "host: " + c.host_header + "\r\nx-amz-date: " + amz_date +
                      "\r\nx-amz-content-sha256: " + payload_hash + "\r\n";
  if (c.access_key.empty()) return lines;
  const std::string date = amz_date.substr(0, 8);
  const std::string signed_headers = "host;x-amz-content-sha256;x-amz-date";
  const std::string creq = method + "\n" + uri_encode_path(path) + "\n" + canonical_query + "\n" + "host:" +
                           c.host_header + "\nx-amz-content-sha256:" + payload_hash + "\nx-amz-date:" + amz_date +
                           "\n\n" + signed_headers + "\n" + payload_hash;
  const std::string scope = date + "/" + c.region + "/s3/aws4_request";
  const std::string sts =
      "AWS4-HMAC-SHA256\n" + amz_date + "\n" + scope + "\n" + sha256_hex(creq.data(), creq.size());
  std::string k = hmac_raw("AWS4" + c.secret_key, date);
  k = hmac_raw(k, c.region);
  k = hmac_raw(k, "s3");
  k = hmac_raw(k, "aws4_request");
  uint8_t sig[32];
  hmac_sha256(k, sts, sig);
  lines += "authorization: AWS4-HMAC-SHA256 Credential=" + c.access_key + "/" + scope +
           ", SignedHeaders=" + signed_headers + ", Signature=" + hex(sig, 32) + "\r\n";
  return lines;
}

}  // namespace amdx
