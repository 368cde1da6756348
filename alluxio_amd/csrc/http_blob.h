// Native S3 data path: an HTTP/1.1 ranged reader that receives object bytes straight into caller
// memory (the K3 pipeline's pinned staging buffers), and an S3-style object endpoint over a
// directory tree that serves GETs with sendfile.
//
// Why: the S3 under file system's control calls (HEAD, LIST, PUT, DELETE, multipart) are a few
// per file and stay in Python (underfs/s3.py, SigV4 signing there), but its data reads went
// through `requests` -> bytes -> BufferedReader -> staging: two extra copies and a GIL-held
// parse per 8 MiB, ~0.6 GB/s end to end (profiles/r2_ufs_ingest_config5.md).  The reference
// reads S3 ranges with the AWS SDK's pooled HTTP connections (underfs/s3a/.../S3AInputStream.java,
// alluxio.underfs.object.store.multi.range.chunk.size); here a block read is split into
// multi-range-chunk-sized sub-ranges fetched in parallel over pooled keep-alive connections, each
// recv()ing into its slice of the destination with the GIL released.
//
// BlobServer is the S3 endpoint used to measure that path (config 5) and to run the S3 UFS
// contract natively: <root>/<bucket>/<key> files, folder-marker objects ("dir/") as a hidden
// marker file inside the directory, ListObjectsV2 with prefix/delimiter/continuation, ranged GET
// via sendfile, PUT/copy, DELETE, multi-object delete and multipart upload (initiate, parts,
// complete, abort, ListMultipartUploads).  No authentication.
#pragma once
#include <atomic>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace amdx {

class BlobServer {
 public:
  BlobServer(const std::string& root, const std::string& host, int port);
  ~BlobServer();
  int port() const { return port_; }
  void start();
  void stop();
  uint64_t requests() const { return requests_.load(); }
  uint64_t bytes_sent() const { return bytes_.load(); }

 private:
  void accept_loop();
  void serve(int fd);
  void serve_conn(int fd);

  std::string root_, host_;
  int port_;
  int lfd_ = -1;
  std::atomic<bool> running_{false};
  std::thread acceptor_;
  std::mutex mu_;
  std::vector<std::thread> conns_;
  std::vector<int> fds_;
  std::atomic<uint64_t> requests_{0}, bytes_{0}, upload_seq_{0};
  // multipart uploads: parts of the upload's stride (the size of the first part to arrive) are
  // written straight into <upload>/data at (partNumber - 1) * stride, so completing the usual
  // fixed-part-size upload appends at most its (shorter) last part instead of copying the object
  std::mutex up_mu_;
  std::map<std::string, uint64_t> stride_;
};

class HttpRangeReader {
 public:
  HttpRangeReader(const std::string& host, int port, int max_idle);
  ~HttpRangeReader();
  // GET `target` (path, already percent-encoded) bytes [offset, offset + length) into `dst`.
  // `head_lines` are the request header lines ("name: value\r\n" each) including Host (SigV4
  // signs the Host value, so the caller spells it).
  // The range is split into up to `parallel` sub-ranges of at least `min_part` bytes fetched
  // concurrently.  Returns `length`, or -HTTP status (-1 for a transport error).
  int64_t get_into(const std::string& target, const std::string& head_lines, uint64_t offset, uint64_t length,
                   uint64_t dst, int parallel, uint64_t min_part);
  // PUT `target` (encoded path plus query) with the `length` bytes at `src` as the body over a
  // pooled connection (the streaming multipart writer's part uploads).  Returns the HTTP status
  // (-1 for a transport error); *etag gets the ETag response header.
  int put_from(const std::string& target, const std::string& head_lines, uint64_t src, uint64_t length,
               std::string* etag);
  // Any request with a body from memory; the response body (up to 1 MiB) goes to *resp.
  int request(const std::string& method, const std::string& target, const std::string& head_lines,
              const uint8_t* body, uint64_t length, std::string* resp, std::string* etag);
  uint64_t requests() const { return requests_.load(); }
  uint64_t connects() const { return connects_.load(); }

 private:
  int64_t one(const std::string& target, const std::string& head, uint64_t off, uint64_t len, uint8_t* dst);
  int take(bool& reused);
  void give(int fd);

  std::string host_;
  int port_;
  size_t max_idle_;
  std::mutex mu_;
  std::vector<int> idle_;
  std::atomic<uint64_t> requests_{0}, connects_{0};
};

}  // namespace amdx
