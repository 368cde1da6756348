// AWS Signature Version 4 for the native S3 data path: SHA-256 / HMAC-SHA-256 and the signed
// header lines of one request, so a worker I/O or ingest thread can issue an authenticated ranged
// GET or part PUT without calling back into Python (underfs/s3.py S3Client._headers is the same
// algorithm for the control calls).
//
// Reference: the AWS SDK signer behind underfs/s3a/src/main/java/alluxio/underfs/s3a/
// S3AUnderFileSystem.java (AmazonS3Client with AWS4 signing).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace amdx {

struct Sha256 {
  Sha256();
  void update(const void* p, size_t n);
  void finish(uint8_t out[32]);

 private:
  void block(const uint8_t* p);
  uint32_t h_[8];
  uint8_t buf_[64];
  size_t used_ = 0;
  uint64_t total_ = 0;
};

std::string sha256_hex(const void* p, size_t n);
void hmac_sha256(const std::string& key, const std::string& msg, uint8_t out[32]);
// Percent-encoding of a path the way the Python signer quotes it (safe = "/-_.~", RFC 3986).
std::string uri_encode_path(const std::string& path);

struct S3Credentials {
  std::string host_header;   // "host[:port]" as sent in Host (signed)
  std::string access_key, secret_key, region = "us-east-1";
};

// Header lines ("name: value\r\n" each) of a request `method` on `path` (not yet encoded) with an
// empty query, whose body hashes to `payload_sha256_hex` ("UNSIGNED-PAYLOAD" for streamed parts).
// `amz_date` is "YYYYMMDDTHHMMSSZ" (empty = now).  Without an access key the request goes
// unsigned (the x-amz-* headers are still sent).
std::string s3_header_lines(const S3Credentials& c, const std::string& method, const std::string& path,
                            const std::string& canonical_query, const std::string& payload_sha256_hex,
                            const std::string& amz_date = std::string());

}  // namespace amdx
