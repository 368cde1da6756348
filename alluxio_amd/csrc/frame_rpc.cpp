// Native framed-RPC transport (see frame_rpc.h).
#include "frame_rpc.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <dlfcn.h>

#include <chrono>
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

// ---- libnghttp2 (HTTP/2 framing for the gRPC connections) -----------------------------------
// The image ships the runtime library without headers: the entry points used below are declared
// from its stable C ABI and resolved with dlopen (no library -> gRPC connections are refused).
struct NgNv {
  uint8_t* name;
  uint8_t* value;
  size_t namelen;
  size_t valuelen;
  uint8_t flags;
};
struct NgFrameHd {   // the first member of every nghttp2_frame variant
  size_t length;
  int32_t stream_id;
  uint8_t type;
  uint8_t flags;
  uint8_t reserved;
};
union NgDataSource {
  int fd;
  void* ptr;
};
typedef ssize_t (*NgReadCb)(void* session, int32_t stream_id, uint8_t* buf, size_t length, uint32_t* data_flags,
                            NgDataSource* source, void* user_data);
struct NgDataProvider {
  NgDataSource source;
  NgReadCb read_callback;
};
struct NgSettingsEntry {
  int32_t settings_id;
  uint32_t value;
};
typedef int (*NgFrameCb)(void* session, const void* frame, void* user_data);
typedef int (*NgDataChunkCb)(void* session, uint8_t flags, int32_t stream_id, const uint8_t* data, size_t len,
                             void* user_data);
typedef int (*NgCloseCb)(void* session, int32_t stream_id, uint32_t error_code, void* user_data);
typedef int (*NgHeaderCb)(void* session, const void* frame, const uint8_t* name, size_t namelen,
                          const uint8_t* value, size_t valuelen, uint8_t flags, void* user_data);
constexpr uint8_t kNgFlagEndStream = 0x01;
constexpr uint32_t kNgDataEof = 0x01, kNgDataNoEndStream = 0x02;
constexpr uint8_t kNgTypeData = 0, kNgTypeHeaders = 1;
const char kH2Preface[] = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";

struct Ng {
  bool ok = false;
  int (*callbacks_new)(void**) = nullptr;
  void (*set_on_frame_recv)(void*, NgFrameCb) = nullptr;
  void (*set_on_begin_headers)(void*, NgFrameCb) = nullptr;
  void (*set_on_data_chunk_recv)(void*, NgDataChunkCb) = nullptr;
  void (*set_on_stream_close)(void*, NgCloseCb) = nullptr;
  void (*set_on_header)(void*, NgHeaderCb) = nullptr;
  int (*server_new)(void**, const void*, void*) = nullptr;
  void (*session_del)(void*) = nullptr;
  ssize_t (*mem_recv)(void*, const uint8_t*, size_t) = nullptr;
  ssize_t (*mem_send)(void*, const uint8_t**) = nullptr;
  int (*submit_settings)(void*, uint8_t, const NgSettingsEntry*, size_t) = nullptr;
  int (*submit_response)(void*, int32_t, const NgNv*, size_t, const NgDataProvider*) = nullptr;
  int (*submit_trailer)(void*, int32_t, const NgNv*, size_t) = nullptr;
  void* cbs = nullptr;   // one callbacks object shared by every session
};

// name/value must outlive the submit call (nghttp2 copies them there): literals or named strings
NgNv nv(const char* n, const char* v) {
  return NgNv{reinterpret_cast<uint8_t*>(const_cast<char*>(n)), reinterpret_cast<uint8_t*>(const_cast<char*>(v)),
              std::strlen(n), std::strlen(v), 0};
}
NgNv nv(const char* n, const std::string& v) {
  return NgNv{reinterpret_cast<uint8_t*>(const_cast<char*>(n)),
              reinterpret_cast<uint8_t*>(const_cast<char*>(v.data())), std::strlen(n), v.size(), 0};
}
NgNv nv(const char* n, std::string&&) = delete;

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

inline void put_be32(std::string& s, uint32_t v) {
  const char b[4] = {(char)(v >> 24), (char)(v >> 16), (char)(v >> 8), (char)v};
  s.append(b, 4);
}

}  // namespace

// gRPC over HTTP/2 on the framed-RPC port: per-connection nghttp2 server session, driven on the
// I/O thread (receive) and the responding threads (send), always under the connection's wmu.
struct FrameRpcServer::H2 {
  struct Stream {
    uint32_t method = UINT32_MAX;
    std::string path, cid, auser, in, out;
    size_t out_off = 0;
    bool dispatched = false, responded = false;
  };
  struct Session {
    FrameRpcServer* srv = nullptr;
    Conn* conn = nullptr;
    void* ng = nullptr;
    std::unordered_map<int32_t, Stream> streams;
    ~Session();
  };
  static const Ng& lib();
  static int on_begin_headers(void*, const void* frame, void* ud);
  static int on_header(void*, const void* frame, const uint8_t* name, size_t namelen, const uint8_t* value,
                       size_t valuelen, uint8_t, void* ud);
  static int on_data(void*, uint8_t, int32_t sid, const uint8_t* data, size_t len, void* ud);
  static int on_frame(void*, const void* frame, void* ud);
  static int on_close(void*, int32_t sid, uint32_t, void* ud);
  static ssize_t read_body(void* session, int32_t sid, uint8_t* buf, size_t length, uint32_t* flags, NgDataSource*,
                           void* ud);
  static void dispatch(Session& S, int32_t sid, Stream& st, std::string msg);
  static void respond_locked(Session& S, int32_t sid, int status, const std::string& msg, const std::string& payload);
  static bool flush_locked(Session& S);
  static bool start(FrameRpcServer& srv, Conn& c);
};

struct FrameRpcServer::Conn {
  int fd;
  uint32_t id;
  std::string in;
  size_t in_off = 0;
  std::mutex wmu;
  std::mutex umu;
  std::string user;
  std::atomic<bool> closed{false};
  int proto = 0;                          // 0 undecided, 1 framed, 2 gRPC/HTTP2
  std::unique_ptr<H2::Session> h2;
  Conn(int f, uint32_t i) : fd(f), id(i) {}
  ~Conn() {
    h2.reset();
    if (fd >= 0) ::close(fd);
  }
};

FrameRpcServer::H2::Session::~Session() {
  if (ng) lib().session_del(ng);
}

const Ng& FrameRpcServer::H2::lib() {
  static const Ng n = [] {
    Ng g;
    void* h = ::dlopen("libnghttp2.so.14", RTLD_NOW | RTLD_LOCAL);
    if (!h) return g;
    auto sym = [&](const char* name) { return ::dlsym(h, name); };
    g.callbacks_new = reinterpret_cast<int (*)(void**)>(sym("nghttp2_session_callbacks_new"));
    g.set_on_frame_recv = reinterpret_cast<void (*)(void*, NgFrameCb)>(sym("nghttp2_session_callbacks_set_on_frame_recv_callback"));
    g.set_on_begin_headers = reinterpret_cast<void (*)(void*, NgFrameCb)>(sym("nghttp2_session_callbacks_set_on_begin_headers_callback"));
    g.set_on_data_chunk_recv = reinterpret_cast<void (*)(void*, NgDataChunkCb)>(sym("nghttp2_session_callbacks_set_on_data_chunk_recv_callback"));
    g.set_on_stream_close = reinterpret_cast<void (*)(void*, NgCloseCb)>(sym("nghttp2_session_callbacks_set_on_stream_close_callback"));
    g.set_on_header = reinterpret_cast<void (*)(void*, NgHeaderCb)>(sym("nghttp2_session_callbacks_set_on_header_callback"));
    g.server_new = reinterpret_cast<int (*)(void**, const void*, void*)>(sym("nghttp2_session_server_new"));
    g.session_del = reinterpret_cast<void (*)(void*)>(sym("nghttp2_session_del"));
    g.mem_recv = reinterpret_cast<ssize_t (*)(void*, const uint8_t*, size_t)>(sym("nghttp2_session_mem_recv"));
    g.mem_send = reinterpret_cast<ssize_t (*)(void*, const uint8_t**)>(sym("nghttp2_session_mem_send"));
    g.submit_settings = reinterpret_cast<int (*)(void*, uint8_t, const NgSettingsEntry*, size_t)>(sym("nghttp2_submit_settings"));
    g.submit_response = reinterpret_cast<int (*)(void*, int32_t, const NgNv*, size_t, const NgDataProvider*)>(sym("nghttp2_submit_response"));
    g.submit_trailer = reinterpret_cast<int (*)(void*, int32_t, const NgNv*, size_t)>(sym("nghttp2_submit_trailer"));
    if (!g.callbacks_new || !g.set_on_frame_recv || !g.set_on_begin_headers || !g.set_on_data_chunk_recv ||
        !g.set_on_stream_close || !g.set_on_header || !g.server_new || !g.session_del || !g.mem_recv || !g.mem_send ||
        !g.submit_settings || !g.submit_response || !g.submit_trailer)
      return g;
    if (g.callbacks_new(&g.cbs) != 0) return g;
    g.set_on_frame_recv(g.cbs, &H2::on_frame);
    g.set_on_begin_headers(g.cbs, &H2::on_begin_headers);
    g.set_on_data_chunk_recv(g.cbs, &H2::on_data);
    g.set_on_stream_close(g.cbs, &H2::on_close);
    g.set_on_header(g.cbs, &H2::on_header);
    g.ok = true;
    return g;
  }();
  return n;
}

bool FrameRpcServer::grpc_available() { return H2::lib().ok; }

bool FrameRpcServer::H2::start(FrameRpcServer& srv, Conn& c) {
  const Ng& g = lib();
  if (!g.ok) return false;
  auto S = std::make_unique<Session>();
  S->srv = &srv;
  S->conn = &c;
  if (g.server_new(&S->ng, g.cbs, S.get()) != 0) {
    S->ng = nullptr;
    return false;
  }
  const NgSettingsEntry iv[] = {{3 /*MAX_CONCURRENT_STREAMS*/, 1024}, {4 /*INITIAL_WINDOW_SIZE*/, 1u << 20}};
  g.submit_settings(S->ng, 0, iv, 2);
  c.h2 = std::move(S);
  return true;
}

int FrameRpcServer::H2::on_begin_headers(void*, const void* frame, void* ud) {
  const NgFrameHd* hd = static_cast<const NgFrameHd*>(frame);
  if (hd->type == kNgTypeHeaders) static_cast<Session*>(ud)->streams[hd->stream_id];
  return 0;
}

int FrameRpcServer::H2::on_header(void*, const void* frame, const uint8_t* name, size_t namelen, const uint8_t* value,
                                  size_t valuelen, uint8_t, void* ud) {
  Session& S = *static_cast<Session*>(ud);
  const NgFrameHd* hd = static_cast<const NgFrameHd*>(frame);
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
  auto it = S.streams.find(sid);
  if (it != S.streams.end() && !it->second.dispatched) it->second.in.append(reinterpret_cast<const char*>(data), len);
  return 0;
}

int FrameRpcServer::H2::on_frame(void*, const void* frame, void* ud) {
  Session& S = *static_cast<Session*>(ud);
  const NgFrameHd* hd = static_cast<const NgFrameHd*>(frame);
  if (hd->type != kNgTypeData && hd->type != kNgTypeHeaders) return 0;
  auto it = S.streams.find(hd->stream_id);
  if (it == S.streams.end()) return 0;
  Stream& st = it->second;
  if (!st.dispatched && st.in.size() >= 5) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(st.in.data());
    const uint32_t len = ((uint32_t)p[1] << 24) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 8) | p[4];
    if (p[0] != 0) {
      st.dispatched = true;
      respond_locked(S, hd->stream_id, 12 /*UNIMPLEMENTED*/, "compressed gRPC messages are not supported", "");
    } else if (len > kMaxFrame) {
      st.dispatched = true;
      respond_locked(S, hd->stream_id, 8 /*RESOURCE_EXHAUSTED*/, "message too large", "");
    } else if (st.in.size() >= 5 + (size_t)len) {
      // one request message per call: unary and server-streaming methods, and the first
      // message of the SASL handshake stream
      st.dispatched = true;
      std::string msg = st.in.substr(5, len);
      st.in.clear();
      st.in.shrink_to_fit();
      dispatch(S, hd->stream_id, st, std::move(msg));
    }
  }
  if ((hd->flags & kNgFlagEndStream) && !st.dispatched) {
    st.dispatched = true;
    respond_locked(S, hd->stream_id, 13 /*INTERNAL*/, "request stream ended without a message", "");
  }
  return 0;
}

int FrameRpcServer::H2::on_close(void*, int32_t sid, uint32_t, void* ud) {
  static_cast<Session*>(ud)->streams.erase(sid);
  return 0;
}

void FrameRpcServer::H2::dispatch(Session& S, int32_t sid, Stream& st, std::string msg) {
  FrameRpcServer& srv = *S.srv;
  if (st.method == UINT32_MAX) {
    respond_locked(S, sid, 12 /*UNIMPLEMENTED*/, "unknown method " + st.path, "");
    return;
  }
  // the Python side resolves the caller: channel-id (SASL channels) or alluxio-user (NOSASL)
  std::string user = "\x01" + st.cid;
  user.push_back('\0');
  user += st.auser;
  srv.requests_.fetch_add(1, std::memory_order_relaxed);
  srv.grpc_requests_.fetch_add(1, std::memory_order_relaxed);
  if (srv.cacheable_[st.method]) {
    CachedReply reply;
    if (srv.cache_get(cache_key(st.method, user, msg.data(), msg.size()), &reply)) {
      srv.cache_hits_.fetch_add(1, std::memory_order_relaxed);
      respond_locked(S, sid, reply.status, reply.msg, reply.body);
      return;
    }
  }
  FrameRequest rq;
  rq.token = ((uint64_t)S.conn->id << 32) | (uint32_t)sid;
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

void FrameRpcServer::H2::respond_locked(Session& S, int32_t sid, int status, const std::string& msg,
                                        const std::string& payload) {
  auto it = S.streams.find(sid);
  if (it == S.streams.end() || it->second.responded) return;   // cancelled or answered
  Stream& st = it->second;
  st.responded = true;
  const Ng& g = lib();
  if (status != 0) {   // trailers-only response
    const std::string code = std::to_string(status), m = grpc_message(msg);
    const NgNv nva[] = {nv(":status", "200"), nv("content-type", "application/grpc"), nv("grpc-status", code),
                        nv("grpc-message", m)};
    g.submit_response(S.ng, sid, nva, 4, nullptr);
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
  const NgNv nva[] = {nv(":status", "200"), nv("content-type", "application/grpc")};
  NgDataProvider dp;
  dp.source.ptr = &S;
  dp.read_callback = &H2::read_body;
  g.submit_response(S.ng, sid, nva, 2, &dp);
}

ssize_t FrameRpcServer::H2::read_body(void* session, int32_t sid, uint8_t* buf, size_t length, uint32_t* flags,
                                      NgDataSource*, void* ud) {
  Session& S = *static_cast<Session*>(ud);
  auto it = S.streams.find(sid);
  if (it == S.streams.end()) {
    *flags |= kNgDataEof;
    return 0;
  }
  Stream& st = it->second;
  const size_t n = std::min(length, st.out.size() - st.out_off);
  std::memcpy(buf, st.out.data() + st.out_off, n);
  st.out_off += n;
  if (st.out_off == st.out.size()) {
    *flags |= kNgDataEof | kNgDataNoEndStream;
    const NgNv t[] = {nv("grpc-status", "0")};
    lib().submit_trailer(session, sid, t, 1);
    st.out.clear();
    st.out.shrink_to_fit();
    st.out_off = 0;
  }
  return (ssize_t)n;
}

bool FrameRpcServer::H2::flush_locked(Session& S) {
  const Ng& g = lib();
  std::string out;
  for (;;) {
    const uint8_t* d = nullptr;
    const ssize_t n = g.mem_send(S.ng, &d);
    if (n < 0) return false;
    if (n == 0) break;
    out.append(reinterpret_cast<const char*>(d), (size_t)n);
  }
  return out.empty() || send_all(S.conn->fd, out.data(), out.size(), 30000);
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
  running_ = true;
  for (int i = 0; i < nthreads_; ++i) {
    const int ep = ::epoll_create1(EPOLL_CLOEXEC);
    if (ep < 0) throw std::runtime_error("frame rpc: epoll_create1 failed");
    epolls_.push_back(ep);
  }
  for (int i = 0; i < nthreads_; ++i) threads_.emplace_back([this, i] { io_loop(i); });
  acceptor_ = std::thread([this] { accept_loop(); });
}

void FrameRpcServer::stop() {
  if (!running_.exchange(false)) return;
  if (listen_fd_ >= 0) ::shutdown(listen_fd_, SHUT_RDWR);
  if (acceptor_.joinable()) acceptor_.join();
  if (listen_fd_ >= 0) ::close(listen_fd_);
  listen_fd_ = -1;
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
  for (int ep : epolls_) ::close(ep);
  epolls_.clear();
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
}

void FrameRpcServer::accept_loop() {
  while (running_) {
    const int fd = ::accept4(listen_fd_, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (fd < 0) {
      if (errno == EINTR || errno == ECONNABORTED) continue;
      if (!running_) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
      continue;
    }
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    std::shared_ptr<Conn> c;
    {
      std::lock_guard<std::mutex> g(conns_mu_);
      uint32_t id = next_conn_++;
      if (next_conn_ == 0) next_conn_ = 1;
      c = std::make_shared<Conn>(fd, id);
      conns_[id] = c;
    }
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP;
    ev.data.u64 = c->id;
    if (::epoll_ctl(epolls_[c->id % epolls_.size()], EPOLL_CTL_ADD, fd, &ev) != 0) close_conn(c->id);
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
  }
  c->closed = true;
  ::epoll_ctl(epolls_[id % epolls_.size()], EPOLL_CTL_DEL, c->fd, nullptr);
  ::shutdown(c->fd, SHUT_RDWR);   // the fd itself closes with the last reference
}

void FrameRpcServer::io_loop(int idx) {
  const int ep = epolls_[idx];
  epoll_event evs[64];
  while (running_) {
    const int n = ::epoll_wait(ep, evs, 64, 100);
    for (int i = 0; i < n; ++i) {
      const uint32_t id = (uint32_t)evs[i].data.u64;
      auto c = find(id);
      if (!c) continue;
      if (evs[i].events & (EPOLLERR | EPOLLHUP)) {
        close_conn(id);
        continue;
      }
      on_readable(c, ep);
    }
  }
}

void FrameRpcServer::on_readable(const std::shared_ptr<Conn>& c, int ep) {
  (void)ep;
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
      if (c->in.size() < sizeof(kH2Preface) - 1) {
        if (eof) close_conn(c->id);
        return;
      }
      bool ok = c->in.compare(0, sizeof(kH2Preface) - 1, kH2Preface) == 0;
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
      const ssize_t r = H2::lib().mem_recv(c->h2->ng, reinterpret_cast<const uint8_t*>(c->in.data()), c->in.size());
      c->in.clear();
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

void FrameRpcServer::respond(uint64_t token, int status, const std::string& msg, const std::string& payload) {
  auto c = find((uint32_t)(token >> 32));
  if (!c || c->closed) return;
  if (c->proto == 2) {
    bool ok;
    {
      std::lock_guard<std::mutex> g(c->wmu);
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
