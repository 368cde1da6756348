// Native framed-RPC transport (see frame_rpc.h).
#include "frame_rpc.h"
#include "h2_abi.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <pthread.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <unordered_map>

namespace amdx {

namespace {

constexpr uint32_t kMaxFrame = 256u << 20;

inline void put_u32(std::string& s, uint32_t v) { s.append(reinterpret_cast<const char*>(&v), 4); }
inline void put_u16(std::string& s, uint16_t v) { s.append(reinterpret_cast<const char*>(&v), 2); }
inline uint32_t get_u32(const char* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
inline uint16_t get_u16(const char* p) {
  uint16_t v;
  std::memcpy(&v, p, 2);
  return v;
}

std::string make_response(uint32_t call_id, int status, const std::string& msg, const std::string& payload) {
  std::string f;
  const uint32_t len = 4 + 2 + 4 + (uint32_t)msg.size() + (uint32_t)payload.size();
  f.reserve(4 + len);
  put_u32(f, len);
  put_u32(f, call_id);
  put_u16(f, (uint16_t)status);
  put_u32(f, (uint32_t)msg.size());
  f += msg;
  f += payload;
  return f;
}

std::string make_request(uint32_t call_id, const std::string& path, const std::string& payload) {
  std::string f;
  const uint32_t len = 4 + 2 + (uint32_t)path.size() + (uint32_t)payload.size();
  f.reserve(4 + len);
  put_u32(f, len);
  put_u32(f, call_id);
  put_u16(f, (uint16_t)path.size());
  f += path;
  f += payload;
  return f;
}

// Blocking socket helpers (client side and the server's EAGAIN fallback).
bool send_all(int fd, const char* p, size_t n, int timeout_ms) {
  while (n) {
    const ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w > 0) {
      p += w;
      n -= (size_t)w;
      continue;
    }
    if (w < 0 && errno == EINTR) continue;
    if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      pollfd pf{fd, POLLOUT, 0};
      const int r = ::poll(&pf, 1, timeout_ms);
      if (r <= 0) return false;
      continue;
    }
    return false;
  }
  return true;
}

bool recv_all(int fd, char* p, size_t n) {
  while (n) {
    const ssize_t r = ::recv(fd, p, n, 0);
    if (r > 0) {
      p += r;
      n -= (size_t)r;
      continue;
    }
    if (r < 0 && errno == EINTR) continue;
    return false;   // EOF, timeout (EAGAIN under SO_RCVTIMEO) or error
  }
  return true;
}

void set_timeouts(int fd, int timeout_ms) {
  timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
  ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
}

// grpc-message: percent-encode everything outside printable ASCII, and '%'
std::string grpc_message(const std::string& m) {
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  for (unsigned char c : m) {
    if (c < 0x20 || c > 0x7E || c == '%') {
      o.push_back('%');
      o.push_back(hex[c >> 4]);
      o.push_back(hex[c & 15]);
    } else {
      o.push_back((char)c);
    }
  }
  return o;
}

using h2::put_be32;
constexpr size_t kOutHighWater = 4u << 20;   // unsent bytes per connection before nghttp2 is paused
constexpr size_t kBridgeQueued = 4u << 20;   // request bytes queued for Python before the window closes

}  // namespace

// gRPC over HTTP/2 on the framed-RPC port: per-connection nghttp2 server session, driven on the
// I/O thread (receive, EPOLLOUT) and the responding threads (send), always under the connection's
// wmu.  Output is non-blocking: what the socket does not take stays in Conn::out and nghttp2 is not
// asked for more frames until it drains below kOutHighWater (EPOLLOUT resumes it), so one slow
// reader never parks an I/O thread.

// A kind-2 call bridged to a Python servicer: request messages queue here for stream_recv.
struct FrameRpcServer::Bridge {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::pair<std::string, size_t>> inbound;   // (message, bytes it took on the wire)
  size_t queued = 0;       // wire bytes of `inbound`
  size_t deferred = 0;     // received bytes whose stream window is returned once Python catches up
  bool half_closed = false, cancelled = false;
  uint32_t conn = 0;
  int32_t sid = 0;
};

struct FrameRpcServer::H2 {
  struct Stream {
    uint32_t method = UINT32_MAX;
    std::string path, cid, auser, in, out;
    size_t out_off = 0;
    bool dispatched = false, headers_sent = false, finished = false;
    size_t held = 0;           // native stream: received bytes whose window is returned when it accepts again
    int fin_status = 0;
    std::string fin_msg;
    std::shared_ptr<Bridge> bridge;
    std::unique_ptr<NativeStream> native;
    bool spans_ok = true;      // native stream offers produce_spans (until it says -2)
    ByteSpan spans[4];
    int nspans = 0;
  };
  struct Session {
    FrameRpcServer* srv = nullptr;
    Conn* conn = nullptr;
    void* ng = nullptr;
    std::unordered_map<int32_t, Stream> streams;
    size_t consume_conn = 0;                                   // window returns queued during mem_recv
    std::vector<std::pair<int32_t, size_t>> consume_streams;
    ~Session();
  };
  static void* callbacks();
  static int on_begin_headers(void*, const void* frame, void* ud);
  static int on_header(void*, const void* frame, const uint8_t* name, size_t namelen, const uint8_t* value,
                       size_t valuelen, uint8_t, void* ud);
  static int on_data(void*, uint8_t, int32_t sid, const uint8_t* data, size_t len, void* ud);
  static int on_frame(void*, const void* frame, void* ud);
  static int on_close(void*, int32_t sid, uint32_t, void* ud);
  static ssize_t read_body(void* session, int32_t sid, uint8_t* buf, size_t length, uint32_t* flags, h2::DataSource*,
                           void* ud);
  static int send_data(void* session, void* frame, const uint8_t* framehd, size_t length, h2::DataSource*, void* ud);
  static void take_messages(Session& S, int32_t sid, Stream& st, bool end_stream);
  static void post_python(Session& S, int32_t sid, Stream& st, uint32_t method, std::string payload);
  static void dispatch(Session& S, int32_t sid, Stream& st, std::string msg);
  static void start_response(Session& S, int32_t sid, Stream& st);
  static void fail_locked(Session& S, int32_t sid, Stream& st, int status, const std::string& msg);
  static void respond_locked(Session& S, int32_t sid, int status, const std::string& msg, const std::string& payload);
  static void apply_consumed(Session& S);
  static bool flush_locked(Session& S);
  static bool start(FrameRpcServer& srv, Conn& c);
};

struct FrameRpcServer::Conn {
  int fd;
  uint32_t id;
  int ep = -1;                            // epoll set of the connection's I/O thread
  std::string in;
  size_t in_off = 0;
  std::mutex wmu;
  std::mutex umu;
  std::string user;
  std::atomic<bool> closed{false};
  int proto = 0;                          // 0 undecided, 1 framed, 2 gRPC/HTTP2
  bool unix_peer = false;                 // accepted on the Unix domain socket
  std::unique_ptr<H2::Session> h2;
  std::string out;                        // unsent bytes (gRPC connections), under wmu
  size_t out_off = 0;
  bool want_out = false;                  // EPOLLOUT armed
  Conn(int f, uint32_t i) : fd(f), id(i) {}
  ~Conn() {
    h2.reset();
    if (fd >= 0) ::close(fd);
  }
};

FrameRpcServer::H2::Session::~Session() {
  if (ng) h2::lib().session_del(ng);
}

void* FrameRpcServer::H2::callbacks() {
  static void* cbs = [] {
    const h2::Lib& g = h2::lib();
    void* c = nullptr;
    if (!g.ok || g.callbacks_new(&c) != 0) return (void*)nullptr;
    g.set_on_frame_recv(c, &H2::on_frame);
    g.set_on_begin_headers(c, &H2::on_begin_headers);
    g.set_on_data_chunk_recv(c, &H2::on_data);
    g.set_on_stream_close(c, &H2::on_close);
    g.set_on_header(c, &H2::on_header);
    g.set_read_length(c, &h2::read_length);
    g.set_send_data(c, &H2::send_data);
    return c;
  }();
  return cbs;
}

bool FrameRpcServer::grpc_available() { return H2::callbacks() != nullptr; }

bool FrameRpcServer::H2::start(FrameRpcServer& srv, Conn& c) {
  const h2::Lib& g = h2::lib();
  void* cbs = callbacks();
  if (!cbs) return false;
  auto S = std::make_unique<Session>();
  S->srv = &srv;
  S->conn = &c;
  // windows are returned by hand: a bridged upload's bytes only once Python has taken them
  void* opt = nullptr;
  if (g.option_new(&opt) != 0) return false;
  g.option_no_auto_window_update(opt, 1);
  const int rc = g.server_new2(&S->ng, cbs, S.get(), opt);
  g.option_del(opt);
  if (rc != 0) {
    S->ng = nullptr;
    return false;
  }
  const h2::SettingsEntry iv[] = {{h2::kSettingsMaxConcurrentStreams, 1024},
                                  {h2::kSettingsInitialWindowSize, srv.stream_window_},
                                  {h2::kSettingsMaxFrameSize, h2::kMaxFramePayload}};
  g.submit_settings(S->ng, 0, iv, 3);
  g.set_local_window_size(S->ng, 0, 0, 64 << 20);   // connection window: many streams in flight
  c.h2 = std::move(S);
  return true;
}

int FrameRpcServer::H2::on_begin_headers(void*, const void* frame, void* ud) {
  const h2::FrameHd* hd = static_cast<const h2::FrameHd*>(frame);
  if (hd->type == h2::kTypeHeaders) static_cast<Session*>(ud)->streams[hd->stream_id];
  return 0;
}

int FrameRpcServer::H2::on_header(void*, const void* frame, const uint8_t* name, size_t namelen, const uint8_t* value,
                                  size_t valuelen, uint8_t, void* ud) {
  Session& S = *static_cast<Session*>(ud);
  const h2::FrameHd* hd = static_cast<const h2::FrameHd*>(frame);
  auto it = S.streams.find(hd->stream_id);
  if (it == S.streams.end() || it->second.dispatched) return 0;   // trailers of a request are ignored
  Stream& st = it->second;
  const std::string n(reinterpret_cast<const char*>(name), namelen);
  const std::string v(reinterpret_cast<const char*>(value), valuelen);
  if (n == ":path") {
    st.path = v;
    auto m = S.srv->method_ids_.find(v);
    if (m != S.srv->method_ids_.end() && m->second != 0) st.method = m->second;   // 0 is the framed @auth
  } else if (n == "channel-id") {
    st.cid = v;
  } else if (n == "alluxio-user") {
    st.auser = v;
  }
  return 0;
}

int FrameRpcServer::H2::on_data(void*, uint8_t, int32_t sid, const uint8_t* data, size_t len, void* ud) {
  Session& S = *static_cast<Session*>(ud);
  S.consume_conn += len;
  auto it = S.streams.find(sid);
  if (it == S.streams.end() || it->second.finished) {
    S.consume_streams.emplace_back(sid, len);     // unknown / answered call: drop the bytes
    return 0;
  }
  it->second.in.append(reinterpret_cast<const char*>(data), len);
  // a native stream takes every message as soon as it is complete: return its window as the
  // bytes arrive, so a message larger than the stream window cannot stall the call
  if (it->second.native) {
    if (it->second.native->accepting()) S.consume_streams.emplace_back(sid, len);
    else it->second.held += len;            // backpressure: the client waits for this window
  }
  return 0;
}

int FrameRpcServer::H2::on_frame(void*, const void* frame, void* ud) {
  Session& S = *static_cast<Session*>(ud);
  const h2::FrameHd* hd = static_cast<const h2::FrameHd*>(frame);
  if (hd->type != h2::kTypeData && hd->type != h2::kTypeHeaders) return 0;
  auto it = S.streams.find(hd->stream_id);
  if (it == S.streams.end()) return 0;
  take_messages(S, hd->stream_id, it->second, (hd->flags & h2::kFlagEndStream) != 0);
  return 0;
}

// Complete gRPC messages of a request stream: the first dispatches the call, later ones go to the
// native stream (acks) or the Python bridge; END_STREAM half-closes a bridged call.
void FrameRpcServer::H2::take_messages(Session& S, int32_t sid, Stream& st, bool end_stream) {
  size_t off = 0;
  while (!st.finished && st.in.size() - off >= 5) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(st.in.data()) + off;
    const uint32_t len = ((uint32_t)p[1] << 24) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 8) | p[4];
    if (p[0] != 0) {
      fail_locked(S, sid, st, 12 /*UNIMPLEMENTED*/, "compressed gRPC messages are not supported");
      break;
    }
    if (len > kMaxFrame) {
      fail_locked(S, sid, st, 8 /*RESOURCE_EXHAUSTED*/, "message too large");
      break;
    }
    if (st.in.size() - off - 5 < len) break;
    const size_t wire = 5 + (size_t)len;
    const char* body = st.in.data() + off + 5;     // valid until st.in is erased below
    off += wire;
    if (!st.dispatched) {
      st.dispatched = true;
      S.consume_streams.emplace_back(sid, wire);
      dispatch(S, sid, st, std::string(body, len));
      // bytes after the first message arrived before the stream was native: return them now
      // (later ones are returned on arrival, in on_data)
      if (st.native && st.in.size() > off) {
        if (st.native->accepting()) S.consume_streams.emplace_back(sid, st.in.size() - off);
        else st.held += st.in.size() - off;
      }
    } else if (st.native) {
      st.native->on_message(body, len);             // no copy: data chunks go straight to the store
      h2::lib().resume_data(S.ng, sid);     // the message may reopen the window
    } else if (st.bridge) {
      Bridge& b = *st.bridge;
      std::lock_guard<std::mutex> g(b.mu);
      b.inbound.emplace_back(std::string(body, len), wire);
      b.queued += wire;
      if (b.queued > kBridgeQueued) b.deferred += wire;     // window returns when Python catches up
      else S.consume_streams.emplace_back(sid, wire);
      b.cv.notify_all();
    } else {
      S.consume_streams.emplace_back(sid, wire);           // extra message of a unary call
    }
  }
  if (off) st.in.erase(0, off);
  if (st.finished && !st.in.empty()) {
    S.consume_streams.emplace_back(sid, st.in.size());
    st.in.clear();
  }
  if (end_stream && !st.finished) {
    if (!st.dispatched) {
      st.dispatched = true;
      fail_locked(S, sid, st, 13 /*INTERNAL*/, "request stream ended without a message");
    } else if (st.bridge) {
      std::lock_guard<std::mutex> g(st.bridge->mu);
      st.bridge->half_closed = true;
      st.bridge->cv.notify_all();
    } else if (st.native) {
      uint32_t m = 0;
      std::string payload;
      if (st.native->on_end(&m, &payload)) post_python(S, sid, st, m, std::move(payload));
      else h2::lib().resume_data(S.ng, sid);
    }
  }
}

// Queues an internal request of a native stream for Python (see NativeStream::on_end); its reply
// comes back through respond() -> respond_locked() -> NativeStream::on_reply.
void FrameRpcServer::H2::post_python(Session& S, int32_t sid, Stream& st, uint32_t method, std::string payload) {
  FrameRpcServer& srv = *S.srv;
  if (method >= srv.lanes_.size()) {
    fail_locked(S, sid, st, 13 /*INTERNAL*/, "native stream posted an unknown method");
    return;
  }
  FrameRequest rq;
  rq.token = ((uint64_t)S.conn->id << 32) | (uint32_t)sid;
  rq.method = method;
  rq.user = "\x02\x01" + st.cid;
  rq.user.push_back('\0');
  rq.user += st.auser;
  rq.payload = std::move(payload);
  Lane& l = *srv.lane_q_[srv.lanes_[method]];
  {
    std::lock_guard<std::mutex> g(l.mu);
    l.q.push_back(std::move(rq));
  }
  l.cv.notify_one();
}

int FrameRpcServer::H2::on_close(void*, int32_t sid, uint32_t, void* ud) {
  Session& S = *static_cast<Session*>(ud);
  auto it = S.streams.find(sid);
  if (it == S.streams.end()) return 0;
  if (it->second.bridge) {
    Bridge& b = *it->second.bridge;
    std::lock_guard<std::mutex> g(b.mu);
    b.cancelled = true;
    b.cv.notify_all();
  }
  S.streams.erase(it);
  return 0;
}

void FrameRpcServer::H2::dispatch(Session& S, int32_t sid, Stream& st, std::string msg) {
  FrameRpcServer& srv = *S.srv;
  if (st.method == UINT32_MAX) {
    fail_locked(S, sid, st, 12 /*UNIMPLEMENTED*/, "unknown method " + st.path);
    return;
  }
  srv.requests_.fetch_add(1, std::memory_order_relaxed);
  srv.grpc_requests_.fetch_add(1, std::memory_order_relaxed);
  if (st.method < srv.natives_.size() && srv.natives_[st.method]) {
    int status = 0;
    std::string err;
    std::unique_ptr<NativeStream> ns =
        srv.natives_[st.method](msg, st.cid, st.auser, S.conn->unix_peer, &status, &err);
    if (ns) {
      st.native = std::move(ns);
      std::shared_ptr<WakeHub> hub = srv.hub_;
      const uint64_t tok = ((uint64_t)S.conn->id << 32) | (uint32_t)sid;
      st.native->set_waker([hub, tok] {
        std::lock_guard<std::mutex> g(hub->mu);
        if (hub->srv) hub->srv->wake(tok);
      });
      start_response(S, sid, st);
      return;
    }
    if (status != 0) {
      fail_locked(S, sid, st, status, err);
      return;
    }
  }
  // the Python side resolves the caller: channel-id (SASL channels) or alluxio-user (NOSASL)
  std::string user = "\x01" + st.cid;
  user.push_back('\0');
  user += st.auser;
  const uint64_t token = ((uint64_t)S.conn->id << 32) | (uint32_t)sid;
  if (st.method < srv.kinds_.size() && srv.kinds_[st.method] == 2) {
    auto b = std::make_shared<Bridge>();
    b->conn = S.conn->id;
    b->sid = sid;
    st.bridge = b;
    std::lock_guard<std::mutex> g(srv.bridges_mu_);
    srv.bridges_[token] = b;
  } else if (srv.cacheable_[st.method]) {
    CachedReply reply;
    if (srv.cache_get(cache_key(st.method, user, msg.data(), msg.size()), &reply)) {
      srv.cache_hits_.fetch_add(1, std::memory_order_relaxed);
      respond_locked(S, sid, reply.status, reply.msg, reply.body);
      return;
    }
  }
  FrameRequest rq;
  rq.token = token;
  rq.method = st.method;
  rq.user = std::move(user);
  rq.payload = std::move(msg);
  Lane& l = *srv.lane_q_[srv.lanes_[st.method]];
  {
    std::lock_guard<std::mutex> g(l.mu);
    l.q.push_back(std::move(rq));
  }
  l.cv.notify_one();
}

void FrameRpcServer::H2::start_response(Session& S, int32_t sid, Stream& st) {
  if (st.headers_sent) {
    h2::lib().resume_data(S.ng, sid);
    return;
  }
  st.headers_sent = true;
  const h2::Nv nva[] = {h2::nv(":status", "200"), h2::nv("content-type", "application/grpc")};
  h2::DataProvider dp;
  dp.source.ptr = &S;
  dp.read_callback = &H2::read_body;
  h2::lib().submit_response(S.ng, sid, nva, 2, &dp);
}

void FrameRpcServer::H2::fail_locked(Session& S, int32_t sid, Stream& st, int status, const std::string& msg) {
  if (st.finished) return;
  st.finished = true;
  st.fin_status = status;
  st.fin_msg = msg;
  st.out.clear();
  st.out_off = 0;
  if (st.headers_sent) {     // trailers after the data already sent
    h2::lib().resume_data(S.ng, sid);
    return;
  }
  st.headers_sent = true;    // trailers-only response
  const std::string code = std::to_string(status), m = grpc_message(msg);
  const h2::Nv nva[] = {h2::nv(":status", "200"), h2::nv("content-type", "application/grpc"),
                        h2::nv("grpc-status", code), h2::nv("grpc-message", m)};
  h2::lib().submit_response(S.ng, sid, nva, 4, nullptr);
}

void FrameRpcServer::H2::respond_locked(Session& S, int32_t sid, int status, const std::string& msg,
                                        const std::string& payload) {
  auto it = S.streams.find(sid);
  if (it == S.streams.end() || it->second.finished) return;   // cancelled or answered
  Stream& st = it->second;
  if (st.native) {                 // the reply of a native stream's internal request
    st.native->on_reply(status, msg, payload);
    h2::lib().resume_data(S.ng, sid);
    return;
  }
  if (status != 0) {
    fail_locked(S, sid, st, status, msg);
    return;
  }
  const bool streaming = st.method < S.srv->kinds_.size() && S.srv->kinds_[st.method] == 1;
  std::string body;
  if (streaming) {
    body.reserve(payload.size() + payload.size() / 64 + 16);
    for (size_t p = 0; p + 4 <= payload.size();) {
      const uint32_t n = get_u32(payload.data() + p);
      if (p + 4 + n > payload.size()) break;
      body.push_back('\0');
      put_be32(body, n);
      body.append(payload, p + 4, n);
      p += 4 + n;
    }
  } else {
    body.reserve(payload.size() + 5);
    body.push_back('\0');
    put_be32(body, (uint32_t)payload.size());
    body += payload;
  }
  st.out = std::move(body);
  st.out_off = 0;
  st.finished = true;
  start_response(S, sid, st);
}

ssize_t FrameRpcServer::H2::read_body(void* session, int32_t sid, uint8_t* buf, size_t length, uint32_t* flags,
                                      h2::DataSource*, void* ud) {
  Session& S = *static_cast<Session*>(ud);
  auto it = S.streams.find(sid);
  if (it == S.streams.end()) {
    *flags |= h2::kDataEof;
    return 0;
  }
  Stream& st = it->second;
  size_t n = 0;
  if (st.native && !st.finished) {
    bool eof = false;
    int status = 0;
    std::string m;
    ssize_t got = -2;
    if (st.spans_ok) {
      int ns = 0;
      got = st.native->produce_spans(length, st.spans, 4, &ns, &eof, &status, &m);
      if (got == -2) st.spans_ok = false;
      else if (got > 0) {
        st.nspans = ns;
        *flags |= h2::kDataNoCopy;     // send_data() writes the spans straight to the socket
      }
    }
    if (got == -2) got = st.native->produce(buf, length, &eof, &status, &m);
    uint32_t post_method = 0;
    std::string post_payload;
    if (got >= 0 && !eof && st.native->take_post(&post_method, &post_payload))
      post_python(S, sid, st, post_method, std::move(post_payload));
    if (got < 0) {
      st.finished = true;
      st.fin_status = status ? status : 13;
      st.fin_msg = m;
    } else {
      n = (size_t)got;
      if (eof) st.finished = true;
    }
    if (n == 0 && !st.finished) return h2::kErrDeferred;
  } else {
    n = std::min(length, st.out.size() - st.out_off);
    std::memcpy(buf, st.out.data() + st.out_off, n);
    st.out_off += n;
    if (st.out_off == st.out.size()) {
      st.out.clear();
      if (st.out.capacity() > (1u << 20)) st.out.shrink_to_fit();
      st.out_off = 0;
    }
    if (n == 0 && !st.finished) return h2::kErrDeferred;
  }
  if (st.finished && st.out_off == st.out.size()) {
    *flags |= h2::kDataEof | h2::kDataNoEndStream;
    const std::string code = std::to_string(st.fin_status), m = grpc_message(st.fin_msg);
    if (st.fin_status == 0) {
      const h2::Nv t[] = {h2::nv("grpc-status", "0")};
      h2::lib().submit_trailer(session, sid, t, 1);
    } else {
      const h2::Nv t[] = {h2::nv("grpc-status", code), h2::nv("grpc-message", m)};
      h2::lib().submit_trailer(session, sid, t, 2);
    }
    st.native.reset();    // release the block lock as soon as the last byte is out
  }
  return (ssize_t)n;
}

// DATA frame of a produce_spans() stream: the 9-byte frame header and the stream's spans go to the
// socket in one sendmsg, no copy; what the socket does not take now is kept in Conn::out.
int FrameRpcServer::H2::send_data(void*, void* frame, const uint8_t* framehd, size_t length, h2::DataSource*,
                                  void* ud) {
  Session& S = *static_cast<Session*>(ud);
  Conn& c = *S.conn;
  const h2::DataFrame* f = static_cast<const h2::DataFrame*>(frame);
  auto it = S.streams.find(f->hd.stream_id);
  if (it == S.streams.end()) return h2::kErrCallbackFailure;
  Stream& st = it->second;
  static const uint8_t zeros[256] = {0};
  iovec iov[8];
  int n = 0;
  iov[n++] = iovec{const_cast<uint8_t*>(framehd), 9};
  uint8_t padfield = 0;
  const size_t padlen = f->padlen;
  if (padlen > 0) {                  // never requested here, but keep the frame well-formed
    padfield = (uint8_t)(padlen - 1);
    iov[n++] = iovec{&padfield, 1};
  }
  size_t data = 0;
  for (int i = 0; i < st.nspans && n < 7; ++i) {
    iov[n++] = iovec{const_cast<uint8_t*>(st.spans[i].p), st.spans[i].n};
    data += st.spans[i].n;
  }
  if (padlen > 1) iov[n++] = iovec{const_cast<uint8_t*>(zeros), std::min<size_t>(padlen - 1, sizeof(zeros))};
  st.nspans = 0;
  if (data != length) return h2::kErrCallbackFailure;
  size_t total = 0;
  for (int i = 0; i < n; ++i) total += iov[i].iov_len;
  size_t sent = 0;
  if (c.out_off == c.out.size()) {   // nothing queued ahead of this frame: straight to the socket
    msghdr mh{};
    mh.msg_iov = iov;
    mh.msg_iovlen = (size_t)n;
    for (;;) {
      const ssize_t w = ::sendmsg(c.fd, &mh, MSG_NOSIGNAL | MSG_DONTWAIT);
      if (w < 0 && errno == EINTR) continue;
      if (w < 0 && errno != EAGAIN && errno != EWOULDBLOCK) return h2::kErrCallbackFailure;
      sent = w > 0 ? (size_t)w : 0;
      break;
    }
    if (sent == total) return 0;
    if (c.out_off == c.out.size()) {
      c.out.clear();
      c.out_off = 0;
    }
  }
  size_t skip = sent;                // the rest waits in Conn::out (EPOLLOUT)
  for (int i = 0; i < n; ++i) {
    const size_t len = iov[i].iov_len;
    if (skip >= len) {
      skip -= len;
      continue;
    }
    c.out.append(static_cast<const char*>(iov[i].iov_base) + skip, len - skip);
    skip = 0;
  }
  return 0;
}

void FrameRpcServer::H2::apply_consumed(Session& S) {
  const h2::Lib& g = h2::lib();
  if (S.consume_conn) g.consume_connection(S.ng, S.consume_conn);
  S.consume_conn = 0;
  for (auto& kv : S.consume_streams)
    if (S.streams.count(kv.first)) g.consume_stream(S.ng, kv.first, kv.second);
  S.consume_streams.clear();
}

// Sends what nghttp2 has queued without blocking; keeps the rest in Conn::out and arms EPOLLOUT.
bool FrameRpcServer::H2::flush_locked(Session& S) {
  const h2::Lib& g = h2::lib();
  Conn& c = *S.conn;
  auto send_some = [&](const char* p, size_t n) -> ssize_t {
    size_t done = 0;
    while (done < n) {
      const ssize_t w = ::send(c.fd, p + done, n - done, MSG_NOSIGNAL | MSG_DONTWAIT);
      if (w > 0) {
        done += (size_t)w;
        continue;
      }
      if (w < 0 && errno == EINTR) continue;
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
      return -1;
    }
    return (ssize_t)done;
  };
  if (c.out_off < c.out.size()) {
    const ssize_t w = send_some(c.out.data() + c.out_off, c.out.size() - c.out_off);
    if (w < 0) return false;
    c.out_off += (size_t)w;
    if (c.out_off == c.out.size()) {
      c.out.clear();
      if (c.out.capacity() > (8u << 20)) c.out.shrink_to_fit();
      c.out_off = 0;
    }
  }
  while (c.out.size() - c.out_off < kOutHighWater) {
    const uint8_t* d = nullptr;
    const ssize_t n = g.mem_send(S.ng, &d);
    if (n < 0) return false;
    if (n == 0) break;
    if (c.out_off == c.out.size()) {
      const ssize_t w = send_some(reinterpret_cast<const char*>(d), (size_t)n);
      if (w < 0) return false;
      if (w < n) {
        c.out.assign(reinterpret_cast<const char*>(d) + w, (size_t)(n - w));
        c.out_off = 0;
      }
    } else {
      c.out.append(reinterpret_cast<const char*>(d), (size_t)n);
    }
  }
  const bool pending = c.out_off < c.out.size();
  if (pending != c.want_out && c.ep >= 0) {
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP | (pending ? EPOLLOUT : 0u);
    ev.data.u64 = c.id;
    ::epoll_ctl(c.ep, EPOLL_CTL_MOD, c.fd, &ev);
    c.want_out = pending;
  }
  return true;
}

FrameRpcServer::FrameRpcServer(const std::string& host, int port, const std::vector<std::string>& methods,
                               const std::vector<int>& lanes, int io_threads)
    : host_(host), port_(port), lanes_(lanes), nthreads_(std::max(1, io_threads)) {
  if (methods.size() != lanes.size()) throw std::invalid_argument("methods/lanes length mismatch");
  int nl = 1;
  for (size_t i = 0; i < methods.size(); ++i) {
    method_ids_[methods[i]] = (uint32_t)i;
    nl = std::max(nl, lanes[i] + 1);
  }
  for (int i = 0; i < nl; ++i) lane_q_.emplace_back(new Lane());
  cacheable_.assign(methods.size(), 0);
  kinds_.assign(methods.size(), 0);
  natives_.resize(methods.size());
}

void FrameRpcServer::set_native_stream(uint32_t method, NativeStreamFactory factory) {
  if (method < natives_.size()) natives_[method] = std::move(factory);
}

// ---- kind-2 bridge --------------------------------------------------------------------------
std::shared_ptr<FrameRpcServer::Bridge> FrameRpcServer::bridge(uint64_t token) {
  std::lock_guard<std::mutex> g(bridges_mu_);
  auto it = bridges_.find(token);
  return it == bridges_.end() ? nullptr : it->second;
}

int FrameRpcServer::stream_recv(uint64_t token, int timeout_ms, std::string* out) {
  auto b = bridge(token);
  if (!b) return 2;
  size_t give_back = 0;
  int rc;
  {
    std::unique_lock<std::mutex> lk(b->mu);
    b->cv.wait_for(lk, std::chrono::milliseconds(std::max(0, timeout_ms)),
                   [&] { return !b->inbound.empty() || b->half_closed || b->cancelled; });
    if (!b->inbound.empty()) {
      *out = std::move(b->inbound.front().first);
      b->queued -= b->inbound.front().second;
      b->inbound.pop_front();
      if (b->deferred && b->queued <= kBridgeQueued / 2) {
        give_back = b->deferred;
        b->deferred = 0;
      }
      rc = 0;
    } else {
      rc = b->cancelled ? 2 : b->half_closed ? 1 : 3;
    }
  }
  if (give_back) {   // Python caught up: reopen the stream's receive window
    auto c = find(b->conn);
    if (c && !c->closed) {
      bool ok = true;
      {
        std::lock_guard<std::mutex> g(c->wmu);
        if (c->h2 && c->h2->streams.count(b->sid)) {
          h2::lib().consume_stream(c->h2->ng, b->sid, give_back);
          ok = H2::flush_locked(*c->h2);
        }
      }
      if (!ok) close_conn(c->id);
    }
  }
  return rc;
}

bool FrameRpcServer::stream_send(uint64_t token, const std::string& msg, int timeout_ms, size_t backlog) {
  auto b = bridge(token);
  if (!b) return false;
  auto c = find(b->conn);
  if (!c || c->closed) return false;
  auto pending = [&]() -> long {   // unsent bytes of this call, -1 when it is gone
    auto it = c->h2->streams.find(b->sid);
    if (it == c->h2->streams.end()) return -1;
    return (long)(it->second.out.size() - it->second.out_off);
  };
  bool ok = true;
  {
    std::lock_guard<std::mutex> g(c->wmu);
    if (!c->h2) return false;
    auto it = c->h2->streams.find(b->sid);
    if (it == c->h2->streams.end() || it->second.finished) return false;
    H2::Stream& st = it->second;
    st.out.push_back('\0');
    put_be32(st.out, (uint32_t)msg.size());
    st.out += msg;
    H2::start_response(*c->h2, b->sid, st);
    ok = H2::flush_locked(*c->h2);
  }
  if (!ok) {
    close_conn(c->id);
    return false;
  }
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(std::max(1, timeout_ms));
  for (;;) {
    long left;
    {
      std::lock_guard<std::mutex> g(c->wmu);
      left = c->closed ? -1 : pending();
    }
    if (left < 0) return false;
    if ((size_t)left <= backlog) return true;
    {
      std::lock_guard<std::mutex> g(b->mu);
      if (b->cancelled) return false;
    }
    if (std::chrono::steady_clock::now() > deadline) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(500));
  }
}

void FrameRpcServer::stream_finish(uint64_t token, int status, const std::string& msg) {
  std::shared_ptr<Bridge> b;
  {
    std::lock_guard<std::mutex> g(bridges_mu_);
    auto it = bridges_.find(token);
    if (it == bridges_.end()) return;
    b = it->second;
    bridges_.erase(it);
  }
  auto c = find(b->conn);
  if (!c || c->closed) return;
  bool ok = true;
  {
    std::lock_guard<std::mutex> g(c->wmu);
    if (!c->h2) return;
    auto it = c->h2->streams.find(b->sid);
    if (it == c->h2->streams.end() || it->second.finished) return;
    H2::Stream& st = it->second;
    if (status != 0) {
      H2::fail_locked(*c->h2, b->sid, st, status, msg);
    } else {
      st.finished = true;
      H2::start_response(*c->h2, b->sid, st);
    }
    ok = H2::flush_locked(*c->h2);
  }
  if (!ok) close_conn(c->id);
}

void FrameRpcServer::allow_channel(const std::string& cid, const std::string& user) {
  std::lock_guard<std::mutex> g(chan_mu_);
  channels_[cid] = user;
}

void FrameRpcServer::revoke_channel(const std::string& cid) {
  std::lock_guard<std::mutex> g(chan_mu_);
  channels_.erase(cid);
}

bool FrameRpcServer::channel_user(const std::string& cid, std::string* user) {
  std::lock_guard<std::mutex> g(chan_mu_);
  auto it = channels_.find(cid);
  if (it == channels_.end()) return false;
  if (user) *user = it->second;
  return true;
}

// ---- reply cache --------------------------------------------------------------------------
std::string FrameRpcServer::cache_key(uint32_t method, const std::string& user, const char* req, size_t n) {
  std::string k;
  k.reserve(4 + user.size() + 1 + n);
  put_u32(k, method);
  k += user;
  k.push_back('\0');
  k.append(req, n);
  return k;
}

void FrameRpcServer::set_cacheable(uint32_t method, bool on) {
  if (method < cacheable_.size()) cacheable_[method] = on ? 1 : 0;
}

void FrameRpcServer::set_method_kind(uint32_t method, int kind) {
  if (method < kinds_.size()) kinds_[method] = (uint8_t)kind;
}

bool FrameRpcServer::cache_get(const std::string& key, CachedReply* reply) {
  const uint64_t ep = epoch();
  CacheShard& sh = shards_[std::hash<std::string>{}(key) % kShards];
  std::lock_guard<std::mutex> g(sh.mu);
  if (sh.epoch != ep) {   // stale shard: every entry predates a metadata change
    sh.map.clear();
    sh.epoch = ep;
    return false;
  }
  auto it = sh.map.find(key);
  if (it == sh.map.end()) return false;
  *reply = it->second;
  return true;
}

void FrameRpcServer::cache_put(uint32_t method, const std::string& user, const std::string& request,
                               const std::string& reply, uint64_t ep, int status, const std::string& msg) {
  if (method >= cacheable_.size() || !cacheable_[method]) return;
  if (ep != epoch()) return;   // something changed while the reply was computed
  std::string key = cache_key(method, user, request.data(), request.size());
  CacheShard& sh = shards_[std::hash<std::string>{}(key) % kShards];
  std::lock_guard<std::mutex> g(sh.mu);
  if (sh.epoch != ep) {
    if (sh.epoch > ep) return;   // the shard already moved to a newer epoch
    sh.map.clear();
    sh.epoch = ep;
  }
  if (sh.map.size() >= cache_cap_ / kShards + 1) sh.map.clear();
  CachedReply& r = sh.map[std::move(key)];
  r.status = status;
  r.msg = msg;
  r.body = reply;
}

void FrameRpcServer::cache_clear() {
  for (auto& sh : shards_) {
    std::lock_guard<std::mutex> g(sh.mu);
    sh.map.clear();
  }
}

size_t FrameRpcServer::cache_size() {
  size_t n = 0;
  for (auto& sh : shards_) {
    std::lock_guard<std::mutex> g(sh.mu);
    n += sh.map.size();
  }
  return n;
}

FrameRpcServer::~FrameRpcServer() { stop(); }

void FrameRpcServer::start() {
  if (running_) return;
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (listen_fd_ < 0) throw std::runtime_error("frame rpc: socket() failed");
  int one = 1;
  ::setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port_);
  if (host_.empty() || host_ == "0.0.0.0") a.sin_addr.s_addr = INADDR_ANY;
  else if (::inet_pton(AF_INET, host_ == "localhost" ? "127.0.0.1" : host_.c_str(), &a.sin_addr) != 1)
    a.sin_addr.s_addr = INADDR_ANY;
  if (::bind(listen_fd_, (sockaddr*)&a, sizeof(a)) != 0 || ::listen(listen_fd_, 1024) != 0) {
    ::close(listen_fd_);
    listen_fd_ = -1;
    throw std::runtime_error("frame rpc: cannot bind " + host_ + ":" + std::to_string(port_));
  }
  socklen_t sl = sizeof(a);
  ::getsockname(listen_fd_, (sockaddr*)&a, &sl);
  port_ = ntohs(a.sin_port);
  if (!unix_path_.empty()) {
    sockaddr_un ua{};
    ua.sun_family = AF_UNIX;
    if (unix_path_.size() >= sizeof(ua.sun_path)) throw std::runtime_error("frame rpc: unix socket path too long");
    std::memcpy(ua.sun_path, unix_path_.c_str(), unix_path_.size() + 1);
    ::unlink(unix_path_.c_str());
    unix_fd_ = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (unix_fd_ < 0 || ::bind(unix_fd_, (sockaddr*)&ua, sizeof(ua)) != 0 || ::listen(unix_fd_, 1024) != 0) {
      if (unix_fd_ >= 0) ::close(unix_fd_);
      unix_fd_ = -1;
      ::close(listen_fd_);
      listen_fd_ = -1;
      throw std::runtime_error("frame rpc: cannot bind unix:" + unix_path_);
    }
  }
  running_ = true;
  hub_ = std::make_shared<WakeHub>();
  hub_->srv = this;
  for (int i = 0; i < nthreads_; ++i) {
    const int ep = ::epoll_create1(EPOLL_CLOEXEC);
    if (ep < 0) throw std::runtime_error("frame rpc: epoll_create1 failed");
    epolls_.push_back(ep);
    const int wfd = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (wfd < 0) throw std::runtime_error("frame rpc: eventfd failed");
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = 0;                    // connection ids start at 1: 0 is the wake fd
    ::epoll_ctl(ep, EPOLL_CTL_ADD, wfd, &ev);
    wake_fds_.push_back(wfd);
    wake_qs_.emplace_back(new WakeQueue());
  }
  for (int i = 0; i < nthreads_; ++i)
    threads_.emplace_back([this, i] {
      char name[16];
      std::snprintf(name, sizeof(name), "frpc-io-%d", i);   // per-thread CPU in /proc (benches)
      pthread_setname_np(pthread_self(), name);
      io_loop(i);
    });
  acceptor_ = std::thread([this] { accept_loop(); });
}

void FrameRpcServer::stop() {
  if (!running_.exchange(false)) return;
  if (hub_) {
    std::lock_guard<std::mutex> g(hub_->mu);   // no waker touches this server once stop() returns
    hub_->srv = nullptr;
  }
  if (listen_fd_ >= 0) ::shutdown(listen_fd_, SHUT_RDWR);
  if (unix_fd_ >= 0) ::shutdown(unix_fd_, SHUT_RDWR);
  if (acceptor_.joinable()) acceptor_.join();
  if (listen_fd_ >= 0) ::close(listen_fd_);
  listen_fd_ = -1;
  if (unix_fd_ >= 0) {
    ::close(unix_fd_);
    ::unlink(unix_path_.c_str());
  }
  unix_fd_ = -1;
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
  for (int ep : epolls_) ::close(ep);
  epolls_.clear();
  for (int fd : wake_fds_) ::close(fd);
  wake_fds_.clear();
  {
    std::lock_guard<std::mutex> g(conns_mu_);
    for (auto& kv : conns_) {
      kv.second->closed = true;
      ::shutdown(kv.second->fd, SHUT_RDWR);
    }
    conns_.clear();
  }
  for (auto& l : lane_q_) {
    std::lock_guard<std::mutex> g(l->mu);
    l->q.clear();
    l->cv.notify_all();
  }
  {
    std::unordered_map<uint32_t, ReplyFn> left;
    {
      std::lock_guard<std::mutex> g(calls_->mu);
      calls_->stopped = true;
      left.swap(calls_->pending);
    }
    for (auto& kv : left) kv.second(14, "the data server stopped", std::string());
  }
  std::lock_guard<std::mutex> g(bridges_mu_);
  for (auto& kv : bridges_) {
    std::lock_guard<std::mutex> bg(kv.second->mu);
    kv.second->cancelled = true;
    kv.second->cv.notify_all();
  }
}

void FrameRpcServer::accept_loop() {
  while (running_) {
    pollfd pf[2] = {{listen_fd_, POLLIN, 0}, {unix_fd_, POLLIN, 0}};
    const int np = unix_fd_ >= 0 ? 2 : 1;
    if (::poll(pf, np, 200) <= 0) continue;
    for (int k = 0; k < np; ++k) {
      if (!(pf[k].revents & (POLLIN | POLLERR | POLLHUP))) continue;
      const int fd = ::accept4(pf[k].fd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) {
        if (errno == EINTR || errno == ECONNABORTED || errno == EAGAIN) continue;
        if (!running_) break;
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
        continue;
      }
      add_conn(fd, k == 1);
    }
  }
}

void FrameRpcServer::add_conn(int fd, bool unix_peer) {
  {
    int one = 1;
    if (!unix_peer) {
      ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    } else {
      // a Unix stream socket's in-flight bytes count against the SENDER's buffer: the 208 KiB
      // default caps every write at a few 16 KiB frames before the I/O thread has to wait for the
      // reader (capped by net.core.wmem_max)
      int sb = 8 << 20;
      ::setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sb, sizeof(sb));
    }
    std::shared_ptr<Conn> c;
    {
      std::lock_guard<std::mutex> g(conns_mu_);
      // the I/O thread with the fewest live connections takes it (round robin skews under churn:
      // every block a client writes opens a connection, and two busy streams on one thread halve
      // both); the id is picked so that id % threads names that thread (wake() and close_conn
      // find the thread from the id)
      const uint32_t nt = (uint32_t)epolls_.size();
      if (ep_conns_.size() != nt) ep_conns_.assign(nt, 0);
      uint32_t target = next_conn_ % nt;
      for (uint32_t k = 0; k < nt; ++k) {
        const uint32_t j = (next_conn_ + k) % nt;
        if (ep_conns_[j] < ep_conns_[target]) target = j;
      }
      uint32_t id = next_conn_ + (target + nt - next_conn_ % nt) % nt;
      if (id == 0) id = nt + target;                 // 0 marks the wake eventfd
      while (conns_.count(id)) id += nt;             // after a wrap: skip ids still in use
      next_conn_ = id + 1;
      if (next_conn_ == 0) next_conn_ = 1;
      ++ep_conns_[id % nt];
      c = std::make_shared<Conn>(fd, id);
      c->unix_peer = unix_peer;
      c->ep = epolls_[id % epolls_.size()];
      conns_[id] = c;
    }
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP;
    ev.data.u64 = c->id;
    if (::epoll_ctl(c->ep, EPOLL_CTL_ADD, fd, &ev) != 0) close_conn(c->id);
  }
}

std::shared_ptr<FrameRpcServer::Conn> FrameRpcServer::find(uint32_t id) {
  std::lock_guard<std::mutex> g(conns_mu_);
  auto it = conns_.find(id);
  return it == conns_.end() ? nullptr : it->second;
}

void FrameRpcServer::close_conn(uint32_t id) {
  std::shared_ptr<Conn> c;
  {
    std::lock_guard<std::mutex> g(conns_mu_);
    auto it = conns_.find(id);
    if (it == conns_.end()) return;
    c = it->second;
    conns_.erase(it);
    if (!ep_conns_.empty() && ep_conns_[id % ep_conns_.size()] > 0) --ep_conns_[id % ep_conns_.size()];
  }
  c->closed = true;
  ::epoll_ctl(epolls_[id % epolls_.size()], EPOLL_CTL_DEL, c->fd, nullptr);
  ::shutdown(c->fd, SHUT_RDWR);   // the fd itself closes with the last reference
  std::lock_guard<std::mutex> g(c->wmu);
  if (c->h2) {
    for (auto& kv : c->h2->streams) {
      if (!kv.second.bridge) continue;
      std::lock_guard<std::mutex> bg(kv.second.bridge->mu);
      kv.second.bridge->cancelled = true;
      kv.second.bridge->cv.notify_all();
    }
    c->h2->streams.clear();   // native streams release their block locks now
  }
}

void FrameRpcServer::on_writable(const std::shared_ptr<Conn>& c) {
  bool ok = true;
  {
    std::lock_guard<std::mutex> g(c->wmu);
    if (c->h2) ok = H2::flush_locked(*c->h2);
  }
  if (!ok) close_conn(c->id);
}

void FrameRpcServer::wake(uint64_t token) {
  if (!running_ || epolls_.empty()) return;
  const size_t idx = (uint32_t)(token >> 32) % epolls_.size();
  WakeQueue& q = *wake_qs_[idx];
  bool first;
  {
    std::lock_guard<std::mutex> g(q.mu);
    first = q.tokens.empty();
    q.tokens.push_back(token);
  }
  if (first) {
    const uint64_t one = 1;
    ssize_t w = ::write(wake_fds_[idx], &one, sizeof(one));
    (void)w;
  }
}

std::function<void(uint32_t, std::string)> FrameRpcServer::internal_poster(const std::string& cid,
                                                                          const std::string& user) {
  std::shared_ptr<WakeHub> hub = hub_;
  std::string caller = "\x02\x01" + cid;
  caller.push_back('\0');
  caller += user;
  return [hub, caller](uint32_t method, std::string payload) {
    if (!hub) return;
    std::lock_guard<std::mutex> g(hub->mu);
    FrameRpcServer* srv = hub->srv;
    if (!srv || method >= srv->lanes_.size()) return;
    FrameRequest rq;
    rq.token = 0;               // connection 0 never exists: respond() drops the reply
    rq.method = method;
    rq.user = caller;
    rq.payload = std::move(payload);
    Lane& l = *srv->lane_q_[srv->lanes_[method]];
    {
      std::lock_guard<std::mutex> lg(l.mu);
      l.q.push_back(std::move(rq));
    }
    l.cv.notify_one();
  };
}

std::function<void(uint32_t, std::string, FrameRpcServer::ReplyFn)> FrameRpcServer::internal_caller(
    const std::string& cid, const std::string& user) {
  std::shared_ptr<WakeHub> hub = hub_;
  std::shared_ptr<InternalCalls> calls = calls_;
  std::string caller = "\x02\x01" + cid;
  caller.push_back('\0');
  caller += user;
  return [hub, calls, caller](uint32_t method, std::string payload, ReplyFn done) {
    if (!hub) {                 // asked for before start()
      done(14, "the data server is not running", std::string());
      return;
    }
    std::lock_guard<std::mutex> g(hub->mu);
    FrameRpcServer* srv = hub->srv;
    uint32_t id = 0;
    {
      std::lock_guard<std::mutex> cg(calls->mu);
      if (srv && !calls->stopped && method < srv->lanes_.size()) {
        do {
          id = calls->next++ & 0x7fffffffu;
        } while (id == 0 || calls->pending.count(id));
        calls->pending.emplace(id, done);
      }
    }
    if (!id) {
      done(14, "the data server has stopped", std::string());
      return;
    }
    FrameRequest rq;
    rq.token = id;              // connection 0: respond() hands the reply to deliver_internal
    rq.method = method;
    rq.user = caller;
    rq.payload = std::move(payload);
    Lane& l = *srv->lane_q_[srv->lanes_[method]];
    {
      std::lock_guard<std::mutex> lg(l.mu);
      l.q.push_back(std::move(rq));
    }
    l.cv.notify_one();
  };
}

void FrameRpcServer::run_wakes(int idx) {
  uint64_t cnt;
  while (::read(wake_fds_[idx], &cnt, sizeof(cnt)) > 0) {
  }
  std::vector<uint64_t> toks;
  {
    std::lock_guard<std::mutex> g(wake_qs_[idx]->mu);
    toks.swap(wake_qs_[idx]->tokens);
  }
  for (uint64_t t : toks) {
    auto c = find((uint32_t)(t >> 32));
    if (!c || c->closed || c->proto != 2) continue;
    bool ok;
    {
      std::lock_guard<std::mutex> g(c->wmu);
      if (!c->h2) continue;
      const int32_t sid = (int32_t)(t & 0x7fffffffu);
      auto it = c->h2->streams.find(sid);
      if (it != c->h2->streams.end() && it->second.held && it->second.native && it->second.native->accepting()) {
        h2::lib().consume_stream(c->h2->ng, sid, it->second.held);   // the paused upload resumes
        it->second.held = 0;
      }
      h2::lib().resume_data(c->h2->ng, sid);
      ok = H2::flush_locked(*c->h2);
    }
    if (!ok) close_conn(c->id);
  }
}

void FrameRpcServer::io_loop(int idx) {
  const int ep = epolls_[idx];
  epoll_event evs[64];
  while (running_) {
    const int n = ::epoll_wait(ep, evs, 64, 100);
    for (int i = 0; i < n; ++i) {
      const uint32_t id = (uint32_t)evs[i].data.u64;
      if (id == 0) {
        run_wakes(idx);
        continue;
      }
      auto c = find(id);
      if (!c) continue;
      if (evs[i].events & (EPOLLERR | EPOLLHUP)) {
        close_conn(id);
        continue;
      }
      if (evs[i].events & EPOLLOUT) on_writable(c);
      if (evs[i].events & (EPOLLIN | EPOLLRDHUP)) on_readable(c, ep);
    }
  }
}

void FrameRpcServer::on_readable(const std::shared_ptr<Conn>& c, int ep) {
  (void)ep;
  if (c->proto == 2) {
    // HTTP/2: every socket read goes straight into nghttp2 (no staging of the whole socket
    // backlog in c->in -- uploads arrive at GB/s), window returns and writes after the batch
    thread_local std::vector<char> big(256u << 10);
    bool eof = false, ok = true;
    for (int reads = 0; reads < 64 && ok; ++reads) {   // bounded: other connections get a turn
      const ssize_t r = ::recv(c->fd, big.data(), big.size(), 0);
      if (r > 0) {
        std::lock_guard<std::mutex> g(c->wmu);
        if (!c->h2) return;
        ok = h2::lib().mem_recv(c->h2->ng, reinterpret_cast<const uint8_t*>(big.data()), (size_t)r) >= 0;
        if ((size_t)r < big.size()) break;
        continue;
      }
      if (r == 0) {
        eof = true;
        break;
      }
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      eof = true;
      break;
    }
    {
      std::lock_guard<std::mutex> g(c->wmu);
      if (!c->h2) return;
      H2::apply_consumed(*c->h2);
      ok = ok && H2::flush_locked(*c->h2);
    }
    if (!ok || eof) close_conn(c->id);
    return;
  }
  char buf[65536];
  bool eof = false;
  for (;;) {
    const ssize_t r = ::recv(c->fd, buf, sizeof(buf), 0);
    if (r > 0) {
      c->in.append(buf, (size_t)r);
      if ((size_t)r < sizeof(buf)) break;
      continue;
    }
    if (r == 0) {
      eof = true;
      break;
    }
    if (errno == EINTR) continue;
    if (errno == EAGAIN || errno == EWOULDBLOCK) break;
    eof = true;
    break;
  }
  // protocol of a new connection: gRPC (HTTP/2 client preface) or framed RPC
  if (c->proto == 0 && c->in.size() >= 3) {
    if (c->in.compare(0, 3, "PRI") == 0) {
      if (c->in.size() < sizeof(h2::kPreface) - 1) {
        if (eof) close_conn(c->id);
        return;
      }
      bool ok = c->in.compare(0, sizeof(h2::kPreface) - 1, h2::kPreface) == 0;
      if (ok) {
        std::lock_guard<std::mutex> g(c->wmu);
        ok = H2::start(*this, *c);
      }
      if (!ok) {
        close_conn(c->id);
        return;
      }
      c->proto = 2;
    } else {
      c->proto = 1;
    }
  }
  if (c->proto == 2) {
    bool ok;
    {
      std::lock_guard<std::mutex> g(c->wmu);
      if (!c->h2) return;
      const ssize_t r = h2::lib().mem_recv(c->h2->ng, reinterpret_cast<const uint8_t*>(c->in.data()), c->in.size());
      c->in.clear();
      if (c->in.capacity() > (4u << 20)) c->in.shrink_to_fit();
      H2::apply_consumed(*c->h2);
      ok = r >= 0 && H2::flush_locked(*c->h2);
    }
    if (!ok || eof) close_conn(c->id);
    return;
  }
  // parse complete frames
  std::string user;
  {
    std::lock_guard<std::mutex> g(c->umu);
    user = c->user;
  }
  size_t off = c->in_off;
  while (c->in.size() - off >= 4) {
    const uint32_t len = get_u32(c->in.data() + off);
    if (len < 6 || len > kMaxFrame) {
      eof = true;
      break;
    }
    if (c->in.size() - off - 4 < len) break;
    const char* p = c->in.data() + off + 4;
    const uint32_t call_id = get_u32(p);
    const uint16_t plen = get_u16(p + 4);
    if (6u + plen > len) {
      eof = true;
      break;
    }
    std::string path(p + 6, plen);
    auto it = method_ids_.find(path);
    if (it == method_ids_.end()) {
      const std::string resp = make_response(call_id, 12 /*UNIMPLEMENTED*/, "unknown method " + path, "");
      std::lock_guard<std::mutex> g(c->wmu);
      send_all(c->fd, resp.data(), resp.size(), 5000);
    } else if (cacheable_[it->second] && [&] {
                 CachedReply reply;
                 const std::string key = cache_key(it->second, user, p + 6 + plen, len - 6 - plen);
                 if (!cache_get(key, &reply)) return false;
                 const std::string resp = make_response(call_id, reply.status, reply.msg, reply.body);
                 requests_.fetch_add(1, std::memory_order_relaxed);
                 cache_hits_.fetch_add(1, std::memory_order_relaxed);
                 std::lock_guard<std::mutex> g(c->wmu);
                 if (!send_all(c->fd, resp.data(), resp.size(), 30000)) eof = true;
                 return true;
               }()) {
      // answered from the reply cache on this I/O thread
    } else {
      FrameRequest rq;
      rq.token = ((uint64_t)c->id << 32) | call_id;
      rq.method = it->second;
      rq.user = user;
      rq.payload.assign(p + 6 + plen, len - 6 - plen);
      requests_.fetch_add(1, std::memory_order_relaxed);
      Lane& l = *lane_q_[lanes_[it->second]];
      {
        std::lock_guard<std::mutex> g(l.mu);
        l.q.push_back(std::move(rq));
      }
      l.cv.notify_one();
    }
    off += 4 + len;
  }
  if (off == c->in.size()) {
    c->in.clear();
    off = 0;
  } else if (off > (1u << 20)) {
    c->in.erase(0, off);
    off = 0;
  }
  c->in_off = off;
  if (eof) close_conn(c->id);
}

std::vector<FrameRequest> FrameRpcServer::poll(int lane, int max_n, int timeout_ms) {
  std::vector<FrameRequest> out;
  if (lane < 0 || lane >= (int)lane_q_.size()) return out;
  Lane& l = *lane_q_[lane];
  std::unique_lock<std::mutex> g(l.mu);
  if (l.q.empty())
    l.cv.wait_for(g, std::chrono::milliseconds(timeout_ms), [&] { return !l.q.empty() || !running_; });
  while (!l.q.empty() && (int)out.size() < max_n) {
    out.push_back(std::move(l.q.front()));
    l.q.pop_front();
  }
  return out;
}

void FrameRpcServer::deliver_internal(uint32_t id, int status, const std::string& msg, const std::string& payload) {
  ReplyFn fn;
  {
    std::lock_guard<std::mutex> g(calls_->mu);
    auto it = calls_->pending.find(id);
    if (it == calls_->pending.end()) return;   // internal_poster's (id 0) or already failed by stop()
    fn = std::move(it->second);
    calls_->pending.erase(it);
  }
  fn(status, msg, payload);
}

void FrameRpcServer::respond(uint64_t token, int status, const std::string& msg, const std::string& payload) {
  if ((token >> 32) == 0) {            // an internal request (no connection): its caller's callback
    deliver_internal((uint32_t)token, status, msg, payload);
    return;
  }
  auto c = find((uint32_t)(token >> 32));
  if (!c || c->closed) return;
  if (c->proto == 2) {
    bool ok;
    {
      std::lock_guard<std::mutex> g(c->wmu);
      if (!c->h2) return;
      H2::respond_locked(*c->h2, (int32_t)(token & 0x7fffffffu), status, msg, payload);
      ok = H2::flush_locked(*c->h2);
    }
    if (!ok) close_conn(c->id);
    return;
  }
  const std::string f = make_response((uint32_t)token, status, msg, payload);
  bool ok;
  {
    std::lock_guard<std::mutex> g(c->wmu);
    ok = send_all(c->fd, f.data(), f.size(), 30000);
  }
  if (!ok) close_conn(c->id);
}

void FrameRpcServer::respond_batch(const std::vector<FrameReply>& replies) {
  if (replies.size() == 1) {
    const FrameReply& r = replies[0];
    respond(r.token, r.status, r.msg, r.payload);
    return;
  }
  // group by connection, keeping each connection's reply order
  std::vector<std::pair<uint32_t, std::vector<const FrameReply*>>> groups;
  for (const FrameReply& r : replies) {
    const uint32_t cid = (uint32_t)(r.token >> 32);
    if (cid == 0) {
      deliver_internal((uint32_t)r.token, r.status, r.msg, r.payload);
      continue;
    }
    auto it = std::find_if(groups.begin(), groups.end(), [&](const auto& g) { return g.first == cid; });
    if (it == groups.end()) {
      groups.emplace_back(cid, std::vector<const FrameReply*>());
      it = groups.end() - 1;
    }
    it->second.push_back(&r);
  }
  for (auto& g : groups) {
    auto c = find(g.first);
    if (!c || c->closed) continue;
    bool ok = true;
    if (c->proto == 2) {
      std::lock_guard<std::mutex> lk(c->wmu);
      if (!c->h2) continue;
      for (const FrameReply* r : g.second)
        H2::respond_locked(*c->h2, (int32_t)(r->token & 0x7fffffffu), r->status, r->msg, r->payload);
      ok = H2::flush_locked(*c->h2);
    } else {
      std::string buf;
      for (const FrameReply* r : g.second) buf += make_response((uint32_t)r->token, r->status, r->msg, r->payload);
      std::lock_guard<std::mutex> lk(c->wmu);
      ok = send_all(c->fd, buf.data(), buf.size(), 30000);
    }
    if (!ok) close_conn(c->id);
  }
}

void FrameRpcServer::set_user(uint64_t token, const std::string& user) {
  auto c = find((uint32_t)(token >> 32));
  if (!c) return;
  std::lock_guard<std::mutex> g(c->umu);
  c->user = user;
}

// ---- client ---------------------------------------------------------------------------------
FrameRpcClient::FrameRpcClient(const std::string& host, int port, const std::string& auth_payload, int timeout_ms)
    : host_(host), port_(port), auth_(auth_payload), timeout_ms_(timeout_ms) {}

FrameRpcClient::~FrameRpcClient() { close(); }

void FrameRpcClient::close() {
  std::lock_guard<std::mutex> g(mu_);
  closed_ = true;
  for (int fd : idle_) ::close(fd);
  idle_.clear();
}

int FrameRpcClient::connect_one(int timeout_ms) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (::getaddrinfo(host_.c_str(), std::to_string(port_).c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("frame rpc: cannot resolve " + host_);
  const int fd = ::socket(res->ai_family, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) {
    ::freeaddrinfo(res);
    throw std::runtime_error("frame rpc: socket() failed");
  }
  set_timeouts(fd, timeout_ms);
  const int rc = ::connect(fd, res->ai_addr, res->ai_addrlen);
  ::freeaddrinfo(res);
  if (rc != 0) {
    ::close(fd);
    throw std::runtime_error("frame rpc: connect to " + host_ + ":" + std::to_string(port_) + " failed");
  }
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  // handshake
  const std::string f = make_request(0, "@auth", auth_);
  char hdr[4];
  if (!send_all(fd, f.data(), f.size(), timeout_ms) || !recv_all(fd, hdr, 4)) {
    ::close(fd);
    throw std::runtime_error("frame rpc: handshake with " + host_ + " failed");
  }
  const uint32_t len = get_u32(hdr);
  std::string body(len, '\0');
  if (len < 10 || len > kMaxFrame || !recv_all(fd, &body[0], len)) {
    ::close(fd);
    throw std::runtime_error("frame rpc: bad handshake response");
  }
  const uint16_t status = get_u16(body.data() + 4);
  if (status != 0) {
    const uint32_t ml = get_u32(body.data() + 6);
    ::close(fd);
    throw std::runtime_error("frame rpc: authentication rejected: " + body.substr(10, ml));
  }
  return fd;
}

std::tuple<int, std::string, std::string> FrameRpcClient::call(const std::string& path, const std::string& payload,
                                                               int timeout_ms) {
  if (timeout_ms <= 0) timeout_ms = timeout_ms_;
  int fd = -1;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (closed_) throw std::runtime_error("frame rpc: client closed");
    if (!idle_.empty()) {
      fd = idle_.back();
      idle_.pop_back();
    }
  }
  if (fd < 0) fd = connect_one(timeout_ms_);
  if (timeout_ms != timeout_ms_) set_timeouts(fd, timeout_ms);
  const uint32_t id = next_id_.fetch_add(1) | 1u;   // never 0 (the handshake id)
  const std::string f = make_request(id, path, payload);
  char hdr[4];
  std::string body;
  bool ok = send_all(fd, f.data(), f.size(), timeout_ms) && recv_all(fd, hdr, 4);
  if (ok) {
    const uint32_t len = get_u32(hdr);
    ok = len >= 10 && len <= kMaxFrame;
    if (ok) {
      body.resize(len);
      ok = recv_all(fd, &body[0], len) && get_u32(body.data()) == id;
    }
  }
  if (!ok) {
    ::close(fd);
    throw std::runtime_error("frame rpc: call " + path + " to " + host_ + ":" + std::to_string(port_) +
                             " failed (connection lost or deadline exceeded)");
  }
  if (timeout_ms != timeout_ms_) set_timeouts(fd, timeout_ms_);
  {
    std::lock_guard<std::mutex> g(mu_);
    if (closed_) ::close(fd);
    else idle_.push_back(fd);
  }
  const int status = get_u16(body.data() + 4);
  const uint32_t ml = get_u32(body.data() + 6);
  if (10u + ml > body.size()) throw std::runtime_error("frame rpc: malformed response");
  return {status, body.substr(10, ml), body.substr(10 + ml)};
}

}  // namespace amdx
