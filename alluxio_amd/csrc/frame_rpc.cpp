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

#include <chrono>
#include <cstring>
#include <stdexcept>

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

}  // namespace

struct FrameRpcServer::Conn {
  int fd;
  uint32_t id;
  std::string in;
  size_t in_off = 0;
  std::mutex wmu;
  std::mutex umu;
  std::string user;
  std::atomic<bool> closed{false};
  Conn(int f, uint32_t i) : fd(f), id(i) {}
  ~Conn() {
    if (fd >= 0) ::close(fd);
  }
};

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
