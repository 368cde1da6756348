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
  // Fault injection (tests of the clients' timeouts and retries): the `count` requests whose
  // method matches `method` ("" = any), starting with the `nth` such request from now (1-based),
  // fail as `kind` says: 1 = 503 SlowDown (body drained, connection kept), 2 = connection reset
  // (RST, no response), 3 = stall (no response for `stall_ms`, then a close), 4 = body stall (a
  // GET's headers and half its body, then `stall_ms` of silence and a close).  Faults add up.
  void inject(int kind, const std::string& method, uint64_t nth, uint64_t count, int stall_ms);
  void clear_faults();
  uint64_t injected() const { return injected_.load(); }

 private:
  struct Fault {
    int kind;
    std::string method;
    uint64_t skip, left;
    int stall_ms;
  };
  // The fault for this request, if any (kind 0 = none).
  int take_fault(const std::string& method, int* stall_ms);
  void stall(int ms) const;
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
  std::mutex fault_mu_;
  std::vector<Fault> faults_;
  std::atomic<uint64_t> injected_{0};
};

// Timeouts and retries of the native object-store client (reference S3AUnderFileSystem.java:
// 150-191 wires alluxio.underfs.s3.{socket.timeout, request.timeout, max.error.retry} into the AWS
// client; PropertyKey.java:946-1002 has the defaults).
struct HttpOptions {
  int connect_timeout_ms = 10000;    // TCP connect
  int socket_timeout_ms = 50000;     // longest silence of the socket while a request is under way
  int request_timeout_ms = 60000;    // one call, all its attempts included (0 = no limit)
  int max_retries = 3;               // further attempts after a retryable failure (AWS SDK default)
  int backoff_base_ms = 50;          // capped exponential back-off with jitter between attempts
  int backoff_max_ms = 2000;
};

// Results of the client below besides an HTTP status: a transport failure (connection refused or
// reset, short body), a timeout, a cancel.  Retryable: these three but the cancel, and 500, 502,
// 503 (SlowDown), 504 and 429.
constexpr int64_t kHttpTransportError = -1;
constexpr int64_t kHttpTimeout = -2;
constexpr int64_t kHttpCancelled = -3;

class HttpRangeReader {
 public:
  HttpRangeReader(const std::string& host, int port, int max_idle, HttpOptions opts = HttpOptions());
  ~HttpRangeReader();
  void set_options(const HttpOptions& o) { opts_ = o; }
  const HttpOptions& options() const { return opts_; }
  // GET `target` (path, already percent-encoded) bytes [offset, offset + length) into `dst`.
  // `head_lines` are the request header lines ("name: value\r\n" each) including Host (SigV4
  // signs the Host value, so the caller spells it).
  // The range is split into up to `parallel` sub-ranges of at least `min_part` bytes fetched
  // concurrently, each retried by itself (the same sub-range again).  Returns `length`, or
  // -HTTP status, or kHttpTransportError / kHttpTimeout / kHttpCancelled.  `cancel` (may be null)
  // is polled while a request waits on its socket (every ~100 ms) and between attempts.
  int64_t get_into(const std::string& target, const std::string& head_lines, uint64_t offset, uint64_t length,
                   uint64_t dst, int parallel, uint64_t min_part, const std::atomic<bool>* cancel = nullptr);
  // PUT `target` (encoded path plus query) with the `length` bytes at `src` as the body over a
  // pooled connection (the streaming multipart writer's part uploads).  Returns the HTTP status
  // (or one of the negative codes above); *etag gets the ETag response header.
  int put_from(const std::string& target, const std::string& head_lines, uint64_t src, uint64_t length,
               std::string* etag, const std::atomic<bool>* cancel = nullptr);
  // Any request with a body from memory; the response body (up to 1 MiB) goes to *resp.  A
  // retryable failure sends the same request again (the body is in memory; a SigV4 signature
  // stays valid for minutes).
  int request(const std::string& method, const std::string& target, const std::string& head_lines,
              const uint8_t* body, uint64_t length, std::string* resp, std::string* etag,
              const std::atomic<bool>* cancel = nullptr);
  uint64_t requests() const { return requests_.load(); }
  uint64_t connects() const { return connects_.load(); }
  uint64_t retries() const { return retries_.load(); }
  uint64_t timeouts() const { return timeouts_.load(); }
  static bool retryable(int64_t code);

 private:
  struct Io;                          // deadline + cancel of one attempt (http_blob.cpp)
  int64_t one(const std::string& target, const std::string& head, uint64_t off, uint64_t len, uint8_t* dst,
              Io& io);
  int request_once(const std::string& req, const uint8_t* body, uint64_t len, std::string* resp, std::string* etag,
                   Io& io);
  // Sleeps the back-off before attempt `attempt` (1-based); false when cancelled or past the deadline.
  bool backoff(int attempt, Io& io);
  int take(bool& reused, Io& io);
  void give(int fd);

  std::string host_;
  int port_;
  size_t max_idle_;
  HttpOptions opts_;
  std::mutex mu_;
  std::vector<int> idle_;
  std::atomic<uint64_t> requests_{0}, connects_{0}, retries_{0}, timeouts_{0};
};

}  // namespace amdx
