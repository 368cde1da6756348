// Native framed-RPC transport for unary control-plane calls (master metadata hot path).
//
// Why: the reference serves metadata RPCs from a JVM gRPC server with hundreds of handler
// threads (core/server/common/src/main/java/alluxio/grpc/GrpcServerBuilder.java; published master
// throughput in docs/en/operation/Scalability-Tuning.md:142-148).  A Python gRPC server pays a
// thread hand-off and a GIL acquisition per call, which caps it at a few thousand calls/s.  This
// transport keeps sockets, framing, queueing and waiting in C++ with the GIL released; Python
// handler threads pull *batches* of decoded requests (one GIL acquisition per batch) and push
// responses back.  Payloads are the same protobuf messages as the gRPC services, so one Python
// servicer serves both transports; gRPC stays the wire-compatible path.
//
// The same port also speaks gRPC (HTTP/2 cleartext, prior knowledge): a connection that opens with
// the HTTP/2 client preface is served by libnghttp2 framing on the I/O thread and its unary /
// server-streaming calls go through the same lanes, Python dispatchers and reply cache, so a
// stock gRPC client (a Java Alluxio client) gets the native path too.
//
// Frames (little endian):
//   request  : u32 len | u32 call_id | u16 path_len | path | payload           (len = bytes after len)
//   response : u32 len | u32 call_id | u16 status | u32 msg_len | msg | payload
// The first request of a connection is path "@auth" with payload "TYPE\0user\0password"; the
// server's Python side validates it (same authenticator as SASL PLAIN) and binds the user to the
// connection.  Status codes are gRPC status codes.
#pragma once
#include <sys/types.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace amdx {

struct FrameReply {
  uint64_t token;
  int status;
  std::string msg;
  std::string payload;
};

struct FrameRequest {
  uint64_t token;      // (conn id << 32) | call id
  uint32_t method;     // registered method index (0 = "@auth", unknown = 0xffffffff)
  std::string user;    // authenticated user of the connection ("" before @auth)
  std::string payload;
};

// A piece of response body handed to the socket without a copy (NativeStream::produce_spans).
struct ByteSpan {
  const uint8_t* p;
  size_t n;
};

// A gRPC call whose responses are produced in C++ on the I/O threads (the worker's ReadBlock data
// path, csrc/data_server.cpp), instead of by a Python servicer.
class NativeStream {
 public:
  virtual ~NativeStream() = default;
  // A further request message of the call (e.g. ReadRequest.offset_received acks).
  virtual void on_message(const char* p, size_t n) = 0;
  // Writes up to `max` bytes of gRPC-framed response body into dst and returns the count.  0 with
  // *eof unset = nothing to send until the next request message arrives (flow-control window);
  // *eof = the call is complete.  -1 = the call failed with *status / *msg (sent as trailers).
  virtual ssize_t produce(uint8_t* dst, size_t max, bool* eof, int* status, std::string* msg) = 0;
  // Zero-copy produce(): up to `max` bytes as at most `max_spans` spans of memory the stream owns,
  // which must stay valid and unchanged until its next produce / produce_spans call (the server
  // writes them to the socket -- the DATA frame's header, then the spans -- before that).
  // -2 = not supported for this call (the server uses produce()).
  virtual ssize_t produce_spans(size_t max, ByteSpan* spans, int max_spans, int* nspans, bool* eof, int* status,
                                std::string* msg) {
    return -2;
  }
  // The client half-closed the request stream.  true = finish the call in Python: the server
  // queues {*method, *payload} on that method's lane as an internal unary request (caller string
  // prefixed "\x02") and hands its reply to on_reply(); false = produce() decides.
  virtual bool on_end(uint32_t* method, std::string* payload) { return false; }
  // The Python reply of the request on_end() posted (status 0: `payload` is the serialized reply).
  virtual void on_reply(int status, const std::string& msg, const std::string& payload) {}
  // Installed by the server right after the factory accepted the call.  `wake` may be called from
  // any thread (a background UFS reader, a HIP host callback): produce() is then polled again on
  // the connection's I/O thread.  It never runs produce() inline and stays safe to call after the
  // call or the server is gone.
  virtual void set_waker(std::function<void()> wake) {}
  // Polled after every produce(): true = post {*method, *payload} to Python now as an internal
  // request (as on_end() does at the half-close); the reply comes back through on_reply().
  virtual bool take_post(uint32_t* method, std::string* payload) { return false; }
  // false = the call holds enough unprocessed request bytes: stop returning receive window to the
  // client (it pauses its uploads) until the stream calls its waker with accepting() true again.
  virtual bool accepting() { return true; }
};
// Builds the native stream of a call from its first request message and the caller's identity
// (the channel-id and alluxio-user headers).  nullptr with *status == 0 hands the call to the
// Python servicer (kind 2 bridge); nullptr with *status != 0 fails the call with it.
// `unix_peer`: the call arrived on the Unix domain socket (a same-node client).
using NativeStreamFactory = std::function<std::unique_ptr<NativeStream>(
    const std::string& first, const std::string& channel_id, const std::string& user, bool unix_peer, int* status,
    std::string* msg)>;

class FrameRpcServer {
 public:
  // `methods`: paths ("/svc/Method") in registration order, `lanes`: dispatch lane per method.
  FrameRpcServer(const std::string& host, int port, const std::vector<std::string>& methods,
                 const std::vector<int>& lanes, int io_threads);
  ~FrameRpcServer();
  int port() const { return port_; }
  // Also accept connections on a Unix domain socket at `path` (set before start()).
  void listen_unix(const std::string& path) { unix_path_ = path; }
  void start();
  void stop();
  // Up to `max_n` requests of `lane`, waiting at most timeout_ms for the first (GIL released).
  std::vector<FrameRequest> poll(int lane, int max_n, int timeout_ms);
  void respond(uint64_t token, int status, const std::string& msg, const std::string& payload);
  // Many replies: those of one connection go out under one write lock with one flush / send
  // (a journal group commit releases dozens of deferred replies at once).
  void respond_batch(const std::vector<FrameReply>& replies);
  // Bind a user to the connection of `token` (after a successful @auth).
  void set_user(uint64_t token, const std::string& user);
  uint64_t requests() const { return requests_.load(); }

  // ---- reply cache (read-only metadata methods) --------------------------------------------
  // A request of a cacheable method whose (method, user, request bytes) were answered while the
  // metadata epoch had its current value is answered on the I/O thread, without Python.  Python
  // bumps the epoch inside every critical section that changes state a cached reply depends on
  // (namespace, block locations, mount table) and tags each put with the epoch it read BEFORE
  // running the handler, so a reply computed across a change is never served.
  void set_cacheable(uint32_t method, bool on);
  // gRPC connections (HTTP/2, detected per connection by the client preface; see H2 in
  // frame_rpc.cpp): kind 1 = server-streaming method, whose Python reply is a sequence of
  // u32-length-prefixed messages (sent as one gRPC message each); 0 = unary.
  // 2 = client- or bidi-streaming method bridged to Python: the dispatcher gets the first request
  // message as the payload and pulls the rest with stream_recv; responses go out with stream_send
  // and the call ends with stream_finish.
  void set_method_kind(uint32_t method, int kind);
  // Serve `method` from C++ when the factory accepts the call (gRPC connections only).
  void set_native_stream(uint32_t method, NativeStreamFactory factory);
  // Re-poll the native stream of `token` ((conn id << 32) | stream id) on its I/O thread.
  void wake(uint64_t token);
  // A poster of internal requests (as a native stream's on_end posts) that belong to no call:
  // queued on the method's lane as caller {cid, user}, their replies dropped.  The returned
  // function stays safe to call from any thread after the call or the server is gone.
  std::function<void(uint32_t, std::string)> internal_poster(const std::string& cid, const std::string& user);
  // Like internal_poster, but the reply comes back: `done(status, msg, payload)` runs on the
  // Python thread that answers (it must not block), or with UNAVAILABLE (14) at once when the
  // server has stopped, or from stop() for calls still unanswered then.
  using ReplyFn = std::function<void(int, const std::string&, const std::string&)>;
  std::function<void(uint32_t, std::string, ReplyFn)> internal_caller(const std::string& cid, const std::string& user);
  // ---- kind-2 bridge (Python side; the GIL is released around the blocking calls) ----------
  // 0 = a message in *out, 1 = the client half-closed, 2 = cancelled / connection gone, 3 = timeout.
  int stream_recv(uint64_t token, int timeout_ms, std::string* out);
  // Queue one response message; waits (up to timeout_ms) while more than `backlog` bytes of this
  // call are unsent.  False once the call is cancelled or its connection closed.
  bool stream_send(uint64_t token, const std::string& msg, int timeout_ms, size_t backlog = 8u << 20);
  void stream_finish(uint64_t token, int status, const std::string& msg);
  // Channels authenticated by the SASL service (gRPC calls served in C++ check channel-id here).
  void allow_channel(const std::string& cid, const std::string& user);
  void revoke_channel(const std::string& cid);
  bool channel_user(const std::string& cid, std::string* user);
  void set_require_channel_auth(bool on) { require_auth_ = on; }
  bool require_channel_auth() const { return require_auth_; }
  // Receive-window size advertised to gRPC clients for request streams (uploads).
  void set_stream_window(uint32_t bytes) { stream_window_ = bytes; }
  uint64_t grpc_requests() const { return grpc_requests_.load(); }
  static bool grpc_available();
  uint64_t epoch() const { return epoch_.load(std::memory_order_acquire); }
  void bump_epoch() { epoch_.fetch_add(1, std::memory_order_acq_rel); }
  void cache_put(uint32_t method, const std::string& user, const std::string& request, const std::string& reply,
                 uint64_t epoch, int status = 0, const std::string& msg = std::string());
  void cache_clear();
  uint64_t cache_hits() const { return cache_hits_.load(); }
  size_t cache_size();
  void set_cache_capacity(size_t entries) { cache_cap_ = entries; }

 private:
  struct Conn;
  struct H2;
  void accept_loop();
  void add_conn(int fd, bool unix_peer);
  void io_loop(int idx);
  void on_readable(const std::shared_ptr<Conn>& c, int ep);
  void close_conn(uint32_t id);
  void on_writable(const std::shared_ptr<Conn>& c);
  struct Bridge;
  std::shared_ptr<Bridge> bridge(uint64_t token);
  std::shared_ptr<Conn> find(uint32_t id);

  std::string host_;
  int port_;
  int listen_fd_ = -1;
  int unix_fd_ = -1;
  std::string unix_path_;
  std::unordered_map<std::string, uint32_t> method_ids_;
  std::vector<int> lanes_;
  int nthreads_;
  std::vector<int> epolls_;
  std::vector<uint32_t> ep_conns_;   // live connections per I/O thread (under conns_mu_)
  std::vector<std::thread> threads_;
  std::thread acceptor_;
  std::atomic<bool> running_{false};
  std::mutex conns_mu_;
  std::unordered_map<uint32_t, std::shared_ptr<Conn>> conns_;
  uint32_t next_conn_ = 1;
  struct Lane {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<FrameRequest> q;
  };
  std::vector<std::unique_ptr<Lane>> lane_q_;
  std::atomic<uint64_t> requests_{0};
  std::atomic<uint64_t> grpc_requests_{0};
  std::vector<uint8_t> kinds_;
  std::vector<NativeStreamFactory> natives_;
  std::mutex bridges_mu_;
  std::unordered_map<uint64_t, std::shared_ptr<Bridge>> bridges_;
  std::mutex chan_mu_;
  std::unordered_map<std::string, std::string> channels_;
  bool require_auth_ = false;
  uint32_t stream_window_ = 1u << 20;
  // wake(): one eventfd + token queue per I/O thread; the hub outlives the server for wakers
  // still held by background producers (it is cleared in stop()).
  struct WakeHub {
    std::mutex mu;
    FrameRpcServer* srv = nullptr;
  };
  struct WakeQueue {
    std::mutex mu;
    std::vector<uint64_t> tokens;
  };
  std::shared_ptr<WakeHub> hub_;
  // internal_caller() calls waiting for their reply: token (0 << 32) | id, id > 0
  struct InternalCalls {
    std::mutex mu;
    uint32_t next = 1;
    bool stopped = false;
    std::unordered_map<uint32_t, ReplyFn> pending;
  };
  std::shared_ptr<InternalCalls> calls_ = std::make_shared<InternalCalls>();
  void deliver_internal(uint32_t id, int status, const std::string& msg, const std::string& payload);
  std::vector<int> wake_fds_;
  std::vector<std::unique_ptr<WakeQueue>> wake_qs_;
  void run_wakes(int idx);

  static std::string cache_key(uint32_t method, const std::string& user, const char* req, size_t n);
  // a cached reply: status 0 + body, or an error status + message (NOT_FOUND lookups)
  struct CachedReply {
    int status = 0;
    std::string msg;
    std::string body;
  };
  bool cache_get(const std::string& key, CachedReply* reply);
  struct CacheEntry {
    uint64_t epoch;
    std::string reply;
  };
  struct CacheShard {
    std::mutex mu;
    uint64_t epoch = 0;   // entries are all of this epoch; a newer put/get resets the shard
    std::unordered_map<std::string, CachedReply> map;
  };
  static constexpr int kShards = 16;
  CacheShard shards_[kShards];
  std::vector<uint8_t> cacheable_;
  std::atomic<uint64_t> epoch_{1};
  std::atomic<uint64_t> cache_hits_{0};
  size_t cache_cap_ = 200000;
};

// Client side: a pool of blocking connections; call() is thread-safe, one in-flight call per
// connection, connections created on demand (the GIL is released for the whole call).
class FrameRpcClient {
 public:
  FrameRpcClient(const std::string& host, int port, const std::string& auth_payload, int timeout_ms);
  ~FrameRpcClient();
  // Returns (status, message, payload).
  std::tuple<int, std::string, std::string> call(const std::string& path, const std::string& payload,
                                                 int timeout_ms);
  void close();

 private:
  int connect_one(int timeout_ms);
  std::string host_;
  int port_;
  std::string auth_;
  int timeout_ms_;
  std::mutex mu_;
  std::vector<int> idle_;
  std::atomic<uint32_t> next_id_{1};
  bool closed_ = false;
};

}  // namespace amdx
