#include "http_blob.h"

#include <atomic>

#include <arpa/inet.h>
#include <dirent.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/sendfile.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <map>
#include <stdexcept>

namespace amdx {
namespace {

constexpr const char* kMarker = ".__s3_folder_marker";
constexpr size_t kMaxHead = 1 << 20;

bool send_all(int fd, const char* p, size_t n) {
  while (n) {
    const ssize_t r = ::send(fd, p, n, MSG_NOSIGNAL);
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += r;
    n -= (size_t)r;
  }
  return true;
}

bool recv_all(int fd, uint8_t* p, size_t n) {
  while (n) {
    const ssize_t r = ::recv(fd, p, n, 0);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    p += r;
    n -= (size_t)r;
  }
  return true;
}

std::string lower(std::string s) {
  for (auto& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}

std::string pct_decode(const std::string& s, bool plus_space) {
  std::string o;
  o.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size() && std::isxdigit((unsigned char)s[i + 1]) &&
        std::isxdigit((unsigned char)s[i + 2])) {
      o.push_back((char)std::stoi(s.substr(i + 1, 2), nullptr, 16));
      i += 2;
    } else if (plus_space && s[i] == '+') {
      o.push_back(' ');
    } else {
      o.push_back(s[i]);
    }
  }
  return o;
}

std::string xml_escape(const std::string& s) {
  std::string o;
  o.reserve(s.size());
  for (char c : s) {
    switch (c) {
      case '&': o += "&amp;"; break;
      case '<': o += "&lt;"; break;
      case '>': o += "&gt;"; break;
      case '"': o += "&quot;"; break;
      case '\'': o += "&apos;"; break;
      default: o.push_back(c);
    }
  }
  return o;
}

std::string xml_unescape(const std::string& s) {
  std::string o;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] != '&') {
      o.push_back(s[i]);
      continue;
    }
    const size_t e = s.find(';', i);
    if (e == std::string::npos) {
      o.push_back(s[i]);
      continue;
    }
    const std::string ent = s.substr(i + 1, e - i - 1);
    if (ent == "amp") o.push_back('&');
    else if (ent == "lt") o.push_back('<');
    else if (ent == "gt") o.push_back('>');
    else if (ent == "quot") o.push_back('"');
    else if (ent == "apos") o.push_back('\'');
    else o += s.substr(i, e - i + 1);
    i = e;
  }
  return o;
}

bool starts_with(const std::string& s, const std::string& p) { return s.compare(0, p.size(), p) == 0; }

bool is_dir(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

bool is_file(const std::string& p, struct stat* out = nullptr) {
  struct stat st;
  if (::stat(p.c_str(), &st) != 0 || !S_ISREG(st.st_mode)) return false;
  if (out) *out = st;
  return true;
}

void mkdirs(const std::string& p) {
  for (size_t i = 1; i <= p.size(); ++i)
    if (i == p.size() || p[i] == '/') ::mkdir(p.substr(0, i).c_str(), 0755);
}

std::string etag_of(const struct stat& st) {
  char b[64];
  std::snprintf(b, sizeof b, "\"%llx-%llx\"", (unsigned long long)st.st_size,
                (unsigned long long)st.st_mtim.tv_sec * 1000000000ull + (unsigned long long)st.st_mtim.tv_nsec);
  return b;
}

std::string http_date(time_t t) {
  char b[64];
  struct tm tmv;
  gmtime_r(&t, &tmv);
  std::strftime(b, sizeof b, "%a, %d %b %Y %H:%M:%S GMT", &tmv);
  return b;
}

std::string iso_date(time_t t) {
  char b[64];
  struct tm tmv;
  gmtime_r(&t, &tmv);
  std::strftime(b, sizeof b, "%Y-%m-%dT%H:%M:%S.000Z", &tmv);
  return b;
}

const char* reason(int code) {
  switch (code) {
    case 200: return "OK";
    case 204: return "No Content";
    case 206: return "Partial Content";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 409: return "Conflict";
    case 416: return "Range Not Satisfiable";
    default: return "Internal Server Error";
  }
}

struct Entry {
  std::string key;
  bool prefix;
  uint64_t size;
  time_t mtime;
  std::string etag;
};

// remove empty, marker-less directories from `dir` up to (not including) `stop`
void prune(std::string dir, const std::string& stop) {
  while (dir.size() > stop.size() && starts_with(dir, stop)) {
    if (::rmdir(dir.c_str()) != 0) return;
    const size_t s = dir.rfind('/');
    if (s == std::string::npos) return;
    dir.resize(s);
  }
}

void walk(const std::string& fsdir, const std::string& keydir, const std::string& prefix, std::vector<Entry>& out) {
  struct stat st;
  if (!keydir.empty() && starts_with(keydir, prefix) && ::stat((fsdir + "/" + kMarker).c_str(), &st) == 0)
    out.push_back({keydir, false, 0, st.st_mtim.tv_sec, "\"d41d8cd98f00b204e9800998ecf8427e\""});
  DIR* d = ::opendir(fsdir.c_str());
  if (!d) return;
  while (dirent* e = ::readdir(d)) {
    const std::string name = e->d_name;
    if (name == "." || name == ".." || name == kMarker) continue;
    const std::string p = fsdir + "/" + name;
    if (::stat(p.c_str(), &st) != 0) continue;
    if (S_ISDIR(st.st_mode)) {
      const std::string k = keydir + name + "/";
      if (starts_with(prefix, k) || starts_with(k, prefix)) walk(p, k, prefix, out);
    } else if (S_ISREG(st.st_mode)) {
      const std::string k = keydir + name;
      if (starts_with(k, prefix)) out.push_back({k, false, (uint64_t)st.st_size, st.st_mtim.tv_sec, etag_of(st)});
    }
  }
  ::closedir(d);
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// BlobServer
// ------------------------------------------------------------------------------------------------
BlobServer::BlobServer(const std::string& root, const std::string& host, int port)
    : root_(root), host_(host), port_(port) {
  while (root_.size() > 1 && root_.back() == '/') root_.pop_back();
}

BlobServer::~BlobServer() { stop(); }

void BlobServer::start() {
  if (running_) return;
  mkdirs(root_);
  lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (lfd_ < 0) throw std::runtime_error("BlobServer: socket failed");
  int one = 1;
  ::setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port_);
  if (::inet_pton(AF_INET, host_.c_str(), &a.sin_addr) != 1) a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (::bind(lfd_, (sockaddr*)&a, sizeof a) != 0 || ::listen(lfd_, 256) != 0) {
    ::close(lfd_);
    lfd_ = -1;
    throw std::runtime_error("BlobServer: bind/listen failed");
  }
  socklen_t len = sizeof a;
  ::getsockname(lfd_, (sockaddr*)&a, &len);
  port_ = ntohs(a.sin_port);
  running_ = true;
  acceptor_ = std::thread([this] { accept_loop(); });
}

void BlobServer::stop() {
  if (!running_.exchange(false)) return;
  if (acceptor_.joinable()) acceptor_.join();
  if (lfd_ >= 0) ::close(lfd_);
  lfd_ = -1;
  std::vector<std::thread> ts;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (int fd : fds_) ::shutdown(fd, SHUT_RDWR);
    ts.swap(conns_);
  }
  for (auto& t : ts)
    if (t.joinable()) t.join();
  std::lock_guard<std::mutex> g(mu_);
  fds_.clear();
}

void BlobServer::inject(int kind, const std::string& method, uint64_t nth, uint64_t count, int stall_ms) {
  std::lock_guard<std::mutex> g(fault_mu_);
  faults_.push_back(Fault{kind, method, nth ? nth - 1 : 0, count, stall_ms});
}

void BlobServer::clear_faults() {
  std::lock_guard<std::mutex> g(fault_mu_);
  faults_.clear();
}

int BlobServer::take_fault(const std::string& method, int* stall_ms) {
  std::lock_guard<std::mutex> g(fault_mu_);
  int kind = 0;
  for (Fault& f : faults_) {
    if (!f.left || (!f.method.empty() && f.method != method)) continue;
    if (f.skip) {
      --f.skip;
      continue;
    }
    if (!kind) {           // the first armed fault wins; the others still count this request
      kind = f.kind;
      *stall_ms = f.stall_ms;
      --f.left;
    }
  }
  if (kind) ++injected_;
  return kind;
}

void BlobServer::stall(int ms) const {
  for (int t = 0; t < ms && running_; t += 20) std::this_thread::sleep_for(std::chrono::milliseconds(20));
}

void BlobServer::accept_loop() {
  while (running_) {
    pollfd p{lfd_, POLLIN, 0};
    if (::poll(&p, 1, 200) <= 0) continue;
    const int fd = ::accept4(lfd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) continue;
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    std::lock_guard<std::mutex> g(mu_);
    if (!running_) {
      ::close(fd);
      break;
    }
    fds_.push_back(fd);
    conns_.emplace_back([this, fd] { serve(fd); });
  }
}

void BlobServer::serve(int fd) {
  try {
    serve_conn(fd);
  } catch (...) {
    // a malformed request ends the connection
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    fds_.erase(std::remove(fds_.begin(), fds_.end(), fd), fds_.end());
  }
  ::close(fd);
}

void BlobServer::serve_conn(int fd) {
  std::string buf;
  std::vector<char> tmp(1 << 16);
  auto recv_more = [&]() -> bool {
    const ssize_t r = ::recv(fd, tmp.data(), tmp.size(), 0);
    if (r <= 0) return false;
    buf.append(tmp.data(), (size_t)r);
    return true;
  };
  while (running_) {
    size_t hend;
    while ((hend = buf.find("\r\n\r\n")) == std::string::npos) {
      if (buf.size() > kMaxHead || !recv_more()) goto done;
    }
    {
      const std::string head = buf.substr(0, hend);
      buf.erase(0, hend + 4);
      ++requests_;
      // request line + headers
      const size_t le = head.find("\r\n");
      const std::string line = head.substr(0, le);
      const size_t s1 = line.find(' '), s2 = line.rfind(' ');
      if (s1 == std::string::npos || s2 <= s1) goto done;
      const std::string method = line.substr(0, s1);
      const std::string target = line.substr(s1 + 1, s2 - s1 - 1);
      std::map<std::string, std::string> h;
      for (size_t p = le == std::string::npos ? head.size() : le + 2; p < head.size();) {
        size_t e = head.find("\r\n", p);
        if (e == std::string::npos) e = head.size();
        const std::string l = head.substr(p, e - p);
        const size_t c = l.find(':');
        if (c != std::string::npos) {
          size_t v = c + 1;
          while (v < l.size() && l[v] == ' ') ++v;
          h[lower(l.substr(0, c))] = l.substr(v);
        }
        p = e + 2;
      }
      const uint64_t clen = h.count("content-length") ? std::stoull(h["content-length"]) : 0;
      const bool keep = lower(h.count("connection") ? h["connection"] : "") != "close";
      uint64_t body_left = clen;
      // body helpers: the first bytes may already sit in buf
      auto body_string = [&]() -> std::string {
        std::string out;
        while (body_left) {
          if (buf.empty() && !recv_more()) break;
          const size_t k = (size_t)std::min<uint64_t>(body_left, buf.size());
          out.append(buf, 0, k);
          buf.erase(0, k);
          body_left -= k;
        }
        return out;
      };
      // the request body into `out` at file offset `at` (pwrite / splice with an explicit offset)
      auto body_to_fd = [&](int out, uint64_t at = 0) -> bool {
        bool ok = true;
        loff_t pos = (loff_t)at;
        // what already arrived with the headers
        if (!buf.empty() && body_left) {
          const size_t k = (size_t)std::min<uint64_t>(body_left, buf.size());
          size_t w = 0;
          while (ok && w < k) {
            const ssize_t r = ::pwrite(out, buf.data() + w, k - w, pos);
            if (r <= 0) ok = false;
            else {
              w += (size_t)r;
              pos += r;
            }
          }
          buf.erase(0, k);
          body_left -= k;
        }
        // the rest socket -> pipe -> file with splice (no user-space copy), else through a buffer
        int pp[2] = {-1, -1};
        if (ok && body_left >= (1u << 20) && ::pipe2(pp, O_CLOEXEC) == 0) {
          (void)::fcntl(pp[1], F_SETPIPE_SZ, 1 << 20);
          while (ok && body_left) {
            const ssize_t n = ::splice(fd, nullptr, pp[1], nullptr, (size_t)std::min<uint64_t>(body_left, 1u << 20),
                                       SPLICE_F_MOVE | SPLICE_F_MORE);
            if (n < 0 && errno == EINTR) continue;
            if (n <= 0) {
              ok = false;
              break;
            }
            ssize_t moved = 0;
            while (moved < n) {
              const ssize_t m = ::splice(pp[0], nullptr, out, &pos, (size_t)(n - moved), SPLICE_F_MOVE);
              if (m < 0 && errno == EINTR) continue;
              if (m <= 0) {
                ok = false;
                break;
              }
              moved += m;
            }
            body_left -= (uint64_t)n;
          }
          ::close(pp[0]);
          ::close(pp[1]);
          return ok;
        }
        std::vector<char> big((size_t)std::min<uint64_t>(std::max<uint64_t>(body_left, 1), 1u << 20));
        while (ok && body_left) {
          const ssize_t r = ::recv(fd, big.data(), (size_t)std::min<uint64_t>(body_left, big.size()), 0);
          if (r < 0 && errno == EINTR) continue;
          if (r <= 0) return false;
          size_t w = 0;
          while (ok && w < (size_t)r) {
            const ssize_t k = ::pwrite(out, big.data() + w, (size_t)r - w, pos);
            if (k <= 0) ok = false;
            else {
              w += (size_t)k;
              pos += k;
            }
          }
          body_left -= (uint64_t)r;
        }
        return ok;
      };
      auto reply = [&](int code, const std::string& extra, const std::string& body, bool head_only = false,
                       int64_t len = -1) -> bool {
        std::string r = "HTTP/1.1 " + std::to_string(code) + " " + reason(code) + "\r\nContent-Length: " +
                        std::to_string(len >= 0 ? (uint64_t)len : body.size()) +
                        "\r\nServer: alluxio-amd-blob\r\n" + extra + "\r\n";
        if (!head_only) r += body;
        return send_all(fd, r.data(), r.size());
      };
      auto error = [&](int code, const std::string& what, const std::string& msg) -> bool {
        return reply(code, "Content-Type: application/xml\r\n",
                     "<?xml version=\"1.0\" encoding=\"UTF-8\"?><Error><Code>" + what + "</Code><Message>" +
                         xml_escape(msg) + "</Message></Error>",
                     method == "HEAD");
      };
      int fault_ms = 0;
      const int fault = take_fault(method, &fault_ms);
      if (fault == 1) {                 // 503 SlowDown, connection kept
        body_string();
        if (!error(503, "SlowDown", "Please reduce your request rate.") || !keep) goto done;
        continue;
      }
      if (fault == 2) {                 // connection reset: RST instead of a FIN, nothing sent
        linger lg{1, 0};
        ::setsockopt(fd, SOL_SOCKET, SO_LINGER, &lg, sizeof lg);
        goto done;
      }
      if (fault == 3) {                 // the server goes silent
        stall(fault_ms);
        goto done;
      }
      // target -> bucket / key / query
      const size_t qm = target.find('?');
      const std::string path = pct_decode(target.substr(0, qm), false);
      std::map<std::string, std::string> q;
      if (qm != std::string::npos) {
        const std::string qs = target.substr(qm + 1);
        for (size_t p = 0; p <= qs.size();) {
          size_t e = qs.find('&', p);
          if (e == std::string::npos) e = qs.size();
          const std::string kv = qs.substr(p, e - p);
          if (!kv.empty()) {
            const size_t eq = kv.find('=');
            q[pct_decode(kv.substr(0, eq), true)] = eq == std::string::npos ? "" : pct_decode(kv.substr(eq + 1), true);
          }
          p = e + 1;
        }
      }
      std::string rest = path.size() > 1 ? path.substr(1) : "";
      const size_t sl = rest.find('/');
      const std::string bucket = rest.substr(0, sl);
      const std::string key = sl == std::string::npos ? "" : rest.substr(sl + 1);
      bool bad = bucket.empty() || bucket[0] == '.' || key.find('\0') != std::string::npos;
      for (size_t p = 0; !bad && p <= key.size();) {
        size_t e = key.find('/', p);
        if (e == std::string::npos) e = key.size();
        const std::string comp = key.substr(p, e - p);
        if (comp == ".." || comp == "." || comp == kMarker) bad = true;
        p = e + 1;
      }
      bool ok = true;
      const std::string bdir = root_ + "/" + bucket;
      const bool marker_key = !key.empty() && key.back() == '/';
      const std::string fpath = bdir + "/" + (marker_key ? key.substr(0, key.size() - 1) : key);
      if (bad) {
        body_string();
        ok = error(400, "InvalidArgument", "bad bucket or key");
      } else if (key.empty()) {
        // ---- bucket operations ----
        if (method == "PUT") {
          body_string();
          mkdirs(bdir);
          ok = reply(200, "", "");
        } else if (method == "HEAD") {
          ok = is_dir(bdir) ? reply(200, "", "", true) : error(404, "NoSuchBucket", bucket);
        } else if (method == "POST" && q.count("delete")) {
          const std::string body = body_string();
          for (size_t p = 0; (p = body.find("<Key>", p)) != std::string::npos;) {
            const size_t e = body.find("</Key>", p);
            if (e == std::string::npos) break;
            const std::string k = xml_unescape(body.substr(p + 5, e - p - 5));
            p = e;
            if (k.empty() || k.find("..") != std::string::npos) continue;
            if (k.back() == '/') {
              const std::string d = bdir + "/" + k.substr(0, k.size() - 1);
              ::unlink((d + "/" + kMarker).c_str());
              prune(d, bdir);
            } else {
              const std::string f = bdir + "/" + k;
              if (::unlink(f.c_str()) == 0) prune(f.substr(0, f.rfind('/')), bdir);
            }
          }
          ok = reply(200, "Content-Type: application/xml\r\n",
                     "<?xml version=\"1.0\" encoding=\"UTF-8\"?><DeleteResult></DeleteResult>");
        } else if (method == "GET" && q.count("uploads")) {
          // ListMultipartUploads: the uploads of this bucket (under `prefix`) still open
          const std::string prefix = q.count("prefix") ? q["prefix"] : "";
          std::string items;
          const std::string ud = root_ + "/.uploads";
          if (DIR* d = ::opendir(ud.c_str())) {
            while (dirent* e = ::readdir(d)) {
              const std::string id = e->d_name;
              if (id == "." || id == "..") continue;
              std::string meta;
              const int mf = ::open((ud + "/" + id + "/.meta").c_str(), O_RDONLY | O_CLOEXEC);
              if (mf < 0) continue;
              char mb[4096];
              const ssize_t r = ::read(mf, mb, sizeof mb);
              ::close(mf);
              if (r <= 0) continue;
              meta.assign(mb, (size_t)r);
              const size_t nl = meta.find('\n');
              if (nl == std::string::npos || meta.substr(0, nl) != bucket) continue;
              std::string k = meta.substr(nl + 1);
              if (!k.empty() && k.back() == '\n') k.pop_back();
              if (!starts_with(k, prefix)) continue;
              const size_t dash = id.find('-');
              const long long t0 = dash == std::string::npos ? 0 : std::atoll(id.c_str() + dash + 1);
              items += "<Upload><Key>" + xml_escape(k) + "</Key><UploadId>" + xml_escape(id) + "</UploadId><Initiated>" +
                       iso_date((time_t)t0) + "</Initiated></Upload>";
            }
            ::closedir(d);
          }
          ok = reply(200, "Content-Type: application/xml\r\n",
                     "<?xml version=\"1.0\" encoding=\"UTF-8\"?><ListMultipartUploadsResult><Bucket>" + xml_escape(bucket) +
                         "</Bucket><Prefix>" + xml_escape(prefix) + "</Prefix><IsTruncated>false</IsTruncated>" + items +
                         "</ListMultipartUploadsResult>");
        } else if (method == "GET") {
          if (!is_dir(bdir)) {
            ok = error(404, "NoSuchBucket", bucket);
          } else {
            const std::string prefix = q.count("prefix") ? q["prefix"] : "";
            const std::string delim = q.count("delimiter") ? q["delimiter"] : "";
            std::string after = q.count("continuation-token") ? q["continuation-token"]
                                                              : (q.count("start-after") ? q["start-after"] : "");
            const size_t max_keys = q.count("max-keys") ? (size_t)std::max(1L, std::stol(q["max-keys"])) : 1000;
            std::vector<Entry> ents;
            if (prefix.find("..") != std::string::npos) {
              // nothing matches
            } else if (delim == "/") {
              const size_t cut = prefix.rfind('/');
              const std::string dirpart = cut == std::string::npos ? "" : prefix.substr(0, cut + 1);
              const std::string base = prefix.substr(dirpart.size());
              const std::string fsdir = bdir + (dirpart.empty() ? "" : "/" + dirpart.substr(0, dirpart.size() - 1));
              struct stat st;
              if (base.empty() && !dirpart.empty() && ::stat((fsdir + "/" + kMarker).c_str(), &st) == 0)
                ents.push_back({dirpart, false, 0, st.st_mtim.tv_sec, "\"d41d8cd98f00b204e9800998ecf8427e\""});
              if (DIR* d = ::opendir(fsdir.c_str())) {
                while (dirent* e = ::readdir(d)) {
                  const std::string name = e->d_name;
                  if (name == "." || name == ".." || name == kMarker || !starts_with(name, base)) continue;
                  const std::string p = fsdir + "/" + name;
                  if (::stat(p.c_str(), &st) != 0) continue;
                  if (S_ISDIR(st.st_mode)) ents.push_back({dirpart + name + "/", true, 0, 0, ""});
                  else if (S_ISREG(st.st_mode))
                    ents.push_back({dirpart + name, false, (uint64_t)st.st_size, st.st_mtim.tv_sec, etag_of(st)});
                }
                ::closedir(d);
              }
            } else {
              walk(bdir, "", prefix, ents);
            }
            std::sort(ents.begin(), ents.end(), [](const Entry& a, const Entry& b) { return a.key < b.key; });
            std::string x = "<?xml version=\"1.0\" encoding=\"UTF-8\"?><ListBucketResult "
                            "xmlns=\"http://s3.amazonaws.com/doc/2006-03-01/\"><Name>" +
                            xml_escape(bucket) + "</Name><Prefix>" + xml_escape(prefix) + "</Prefix>";
            if (!delim.empty()) x += "<Delimiter>" + xml_escape(delim) + "</Delimiter>";
            std::string items, last;
            size_t n = 0;
            bool truncated = false;
            for (const Entry& e : ents) {
              if (!after.empty() && e.key <= after) continue;
              if (n == max_keys) {
                truncated = true;
                break;
              }
              ++n;
              last = e.key;
              if (e.prefix) {
                items += "<CommonPrefixes><Prefix>" + xml_escape(e.key) + "</Prefix></CommonPrefixes>";
              } else {
                items += "<Contents><Key>" + xml_escape(e.key) + "</Key><LastModified>" + iso_date(e.mtime) +
                         "</LastModified><ETag>" + xml_escape(e.etag) + "</ETag><Size>" + std::to_string(e.size) +
                         "</Size><StorageClass>STANDARD</StorageClass></Contents>";
              }
            }
            x += "<KeyCount>" + std::to_string(n) + "</KeyCount><MaxKeys>" + std::to_string(max_keys) +
                 "</MaxKeys><IsTruncated>" + (truncated ? "true" : "false") + "</IsTruncated>";
            if (truncated) x += "<NextContinuationToken>" + xml_escape(last) + "</NextContinuationToken>";
            x += items + "</ListBucketResult>";
            ok = reply(200, "Content-Type: application/xml\r\n", x);
          }
        } else {
          body_string();
          ok = error(400, "InvalidRequest", method);
        }
      } else if (q.count("uploads") && method == "POST") {
        // ---- multipart upload ----
        body_string();
        const std::string id = std::to_string(++upload_seq_) + "-" + std::to_string((long long)::time(nullptr));
        mkdirs(root_ + "/.uploads/" + id);
        {   // bucket and key of the upload, for ListMultipartUploads (hidden from the part list)
          const int mf = ::open((root_ + "/.uploads/" + id + "/.meta").c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC,
                                0644);
          if (mf >= 0) {
            const std::string meta = bucket + "\n" + key + "\n";
            ssize_t w = ::write(mf, meta.data(), meta.size());
            (void)w;
            ::close(mf);
          }
        }
        ok = reply(200, "Content-Type: application/xml\r\n",
                   "<?xml version=\"1.0\" encoding=\"UTF-8\"?><InitiateMultipartUploadResult><Bucket>" +
                       xml_escape(bucket) + "</Bucket><Key>" + xml_escape(key) + "</Key><UploadId>" + id +
                       "</UploadId></InitiateMultipartUploadResult>");
      } else if (q.count("uploadId")) {
        const std::string id = q["uploadId"];
        const std::string udir = root_ + "/.uploads/" + id;
        if (id.find('/') != std::string::npos || id.find("..") != std::string::npos || !is_dir(udir)) {
          body_string();
          ok = error(404, "NoSuchUpload", id);
        } else if (method == "PUT" && q.count("partNumber")) {
          const int pn = std::atoi(q["partNumber"].c_str());
          char name[32];
          uint64_t stride;
          {
            std::lock_guard<std::mutex> g(up_mu_);
            auto it = stride_.find(id);
            if (it == stride_.end()) it = stride_.emplace(id, body_left).first;
            stride = it->second;
          }
          bool wrote;
          if (pn >= 1 && stride && body_left == stride) {      // in place: <udir>/data at (pn-1)*stride
            std::snprintf(name, sizeof name, "/%08d.d", pn);
            const int out = ::open((udir + "/data").c_str(), O_WRONLY | O_CREAT | O_CLOEXEC, 0644);
            wrote = out >= 0 && body_to_fd(out, (uint64_t)(pn - 1) * stride);
            if (out >= 0) ::close(out);
            const int mk = ::open((udir + name).c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
            if (mk >= 0) ::close(mk);
            else wrote = false;
          } else {
            std::snprintf(name, sizeof name, "/%08d", pn);
            const int out = ::open((udir + name).c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
            wrote = out >= 0 && body_to_fd(out);
            if (out >= 0) ::close(out);
          }
          if (!wrote) {
            body_string();
            ok = error(500, "InternalError", "part write failed");
          } else {
            ok = reply(200, "ETag: \"part" + std::to_string(pn) + "\"\r\n", "");
          }
        } else if (method == "POST") {
          body_string();
          std::vector<std::string> parts;
          std::map<int, bool> in_data;      // part number -> stored in <udir>/data
          if (DIR* d = ::opendir(udir.c_str())) {
            while (dirent* e = ::readdir(d)) {
              const std::string n = e->d_name;
              if (n[0] == '.' || n == "data") continue;
              const bool dd = n.size() > 2 && n.compare(n.size() - 2, 2, ".d") == 0;
              in_data[std::atoi(n.c_str())] = dd;
              if (!dd) parts.push_back(n);
            }
            ::closedir(d);
          }
          uint64_t stride = 0;
          {
            std::lock_guard<std::mutex> g(up_mu_);
            auto it = stride_.find(id);
            if (it != stride_.end()) stride = it->second;
            stride_.erase(id);
          }
          std::sort(parts.begin(), parts.end());
          mkdirs(fpath.substr(0, fpath.rfind('/')));
          // fast path: parts 1..k in place in <udir>/data, at most the last one (k+1) separate
          int k = 0;
          while (in_data.count(k + 1) && in_data[k + 1]) ++k;
          const int nparts = in_data.empty() ? 0 : in_data.rbegin()->first;
          const bool fast = stride && k >= 1 && (int)in_data.size() == nparts &&
                            (k == nparts || (k == nparts - 1 && parts.size() == 1));
          if (fast) {
            const std::string dataf = udir + "/data";
            uint64_t total = (uint64_t)k * stride;
            bool ok2 = true;
            if (k < nparts) {            // append the short last part
              const int in = ::open((udir + "/" + parts[0]).c_str(), O_RDONLY | O_CLOEXEC);
              const int out = ::open(dataf.c_str(), O_WRONLY | O_CLOEXEC);
              struct stat st;
              if (in < 0 || out < 0 || ::fstat(in, &st) != 0) {
                ok2 = false;
              } else {
                loff_t oi = 0, oo = (loff_t)total;
                uint64_t left = (uint64_t)st.st_size;
                while (ok2 && left) {
                  const ssize_t r = ::copy_file_range(in, &oi, out, &oo, (size_t)left, 0);
                  if (r <= 0) ok2 = false;
                  else left -= (uint64_t)r;
                }
                total += (uint64_t)st.st_size;
              }
              if (in >= 0) ::close(in);
              if (out >= 0) ::close(out);
            }
            struct stat st;
            if (ok2 && ::truncate(dataf.c_str(), (off_t)total) == 0 && ::rename(dataf.c_str(), fpath.c_str()) == 0 &&
                is_file(fpath, &st)) {
              if (DIR* d = ::opendir(udir.c_str())) {
                while (dirent* e = ::readdir(d))
                  if (std::strcmp(e->d_name, ".") != 0 && std::strcmp(e->d_name, "..") != 0)
                    ::unlink((udir + "/" + e->d_name).c_str());
                ::closedir(d);
              }
              ::rmdir(udir.c_str());
              ok = reply(200, "Content-Type: application/xml\r\n",
                         "<?xml version=\"1.0\" encoding=\"UTF-8\"?><CompleteMultipartUploadResult><Bucket>" +
                             xml_escape(bucket) + "</Bucket><Key>" + xml_escape(key) + "</Key><ETag>" +
                             xml_escape(etag_of(st)) + "</ETag></CompleteMultipartUploadResult>");
              if (!ok || !keep) goto done;
              continue;
            }
          }
          // general case: every part (in place or separate) copied into a fresh file
          std::vector<std::pair<std::string, uint64_t>> srcs;   // (file, offset in it) per part, in order
          std::vector<uint64_t> src_len;
          for (const auto& kv : in_data) {
            char nm[32];
            if (kv.second) {
              srcs.emplace_back(udir + "/data", (uint64_t)(kv.first - 1) * stride);
              src_len.push_back(stride);
            } else {
              std::snprintf(nm, sizeof nm, "/%08d", kv.first);
              struct stat pst;
              srcs.emplace_back(udir + nm, 0);
              src_len.push_back(::stat((udir + nm).c_str(), &pst) == 0 ? (uint64_t)pst.st_size : 0);
            }
          }
          parts.clear();
          for (size_t i = 0; i < srcs.size(); ++i) parts.push_back(srcs[i].first);
          const std::string tmpf = fpath + ".__upload";
          const int out = ::open(tmpf.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
          bool good = out >= 0;
          // the object is the parts in order: sized once, then every part copied into its slice
          // by a few threads at once (in-kernel copy_file_range), so completing a multi-GB upload
          // costs a parallel copy rather than one serial pass
          std::vector<uint64_t> sizes(parts.size()), offs(parts.size());
          uint64_t total = 0;
          for (size_t i = 0; i < parts.size(); ++i) {
            sizes[i] = src_len[i];
            offs[i] = total;
            total += sizes[i];
          }
          if (good && ::ftruncate(out, (off_t)total) != 0) good = false;
          std::atomic<size_t> next{0};
          std::atomic<bool> all_ok{good};
          auto copier = [&] {
            for (size_t i; all_ok && (i = next.fetch_add(1)) < parts.size();) {
              const int in = ::open(srcs[i].first.c_str(), O_RDONLY | O_CLOEXEC);
              if (in < 0) {
                all_ok = false;
                break;
              }
              loff_t oi = (loff_t)srcs[i].second, oo = (loff_t)offs[i];
              uint64_t left = sizes[i];
              while (left) {
                ssize_t r = ::copy_file_range(in, &oi, out, &oo, (size_t)std::min<uint64_t>(left, 1ull << 30), 0);
                if (r < 0 && errno == EINTR) continue;
                if (r <= 0) {     // no in-kernel copy here: pread/pwrite
                  char buf[1 << 16];
                  const ssize_t k = ::pread(in, buf, sizeof buf, oi);
                  if (k <= 0 || ::pwrite(out, buf, (size_t)k, oo) != k) {
                    all_ok = false;
                    break;
                  }
                  r = k;
                  oi += k;
                  oo += k;
                }
                left -= (uint64_t)r;
              }
              ::close(in);
            }
          };
          if (good) {
            std::vector<std::thread> ts;
            const size_t nt = std::min<size_t>(8, parts.size());
            for (size_t t = 1; t < nt; ++t) ts.emplace_back(copier);
            copier();
            for (auto& t : ts) t.join();
            good = all_ok;
          }
          if (out >= 0) ::close(out);
          if (DIR* d = ::opendir(udir.c_str())) {
            while (dirent* e = ::readdir(d))
              if (std::strcmp(e->d_name, ".") != 0 && std::strcmp(e->d_name, "..") != 0)
                ::unlink((udir + "/" + e->d_name).c_str());
            ::closedir(d);
          }
          ::rmdir(udir.c_str());
          struct stat st;
          if (good && ::rename(tmpf.c_str(), fpath.c_str()) == 0 && is_file(fpath, &st)) {
            ok = reply(200, "Content-Type: application/xml\r\n",
                       "<?xml version=\"1.0\" encoding=\"UTF-8\"?><CompleteMultipartUploadResult><Bucket>" +
                           xml_escape(bucket) + "</Bucket><Key>" + xml_escape(key) + "</Key><ETag>" +
                           xml_escape(etag_of(st)) + "</ETag></CompleteMultipartUploadResult>");
          } else {
            ::unlink(tmpf.c_str());
            ok = error(500, "InternalError", "complete failed");
          }
        } else if (method == "DELETE") {
          {
            std::lock_guard<std::mutex> g(up_mu_);
            stride_.erase(id);
          }
          if (DIR* d = ::opendir(udir.c_str())) {
            while (dirent* e = ::readdir(d))
              if (std::strcmp(e->d_name, ".") != 0 && std::strcmp(e->d_name, "..") != 0)
                ::unlink((udir + "/" + e->d_name).c_str());
            ::closedir(d);
          }
          ::rmdir(udir.c_str());
          ok = reply(204, "", "");
        } else {
          body_string();
          ok = error(400, "InvalidRequest", method);
        }
      } else if (method == "GET" || method == "HEAD") {
        // ---- object reads ----
        struct stat st;
        if (marker_key) {
          if (::stat((fpath + "/" + kMarker).c_str(), &st) == 0)
            ok = reply(200, "ETag: \"d41d8cd98f00b204e9800998ecf8427e\"\r\nLast-Modified: " + http_date(st.st_mtim.tv_sec) +
                                "\r\n",
                       "", method == "HEAD");
          else
            ok = error(404, "NoSuchKey", key);
        } else if (!is_file(fpath, &st)) {
          ok = error(404, "NoSuchKey", key);
        } else {
          const uint64_t size = (uint64_t)st.st_size;
          uint64_t a = 0, b = size ? size - 1 : 0;
          bool ranged = false, unsat = false;
          if (h.count("range") && starts_with(h["range"], "bytes=")) {
            const std::string r = h["range"].substr(6);
            const size_t dash = r.find('-');
            if (dash != std::string::npos) {
              ranged = true;
              if (dash == 0) {  // suffix range
                const uint64_t n = std::stoull(r.substr(1));
                a = n >= size ? 0 : size - n;
              } else {
                a = std::stoull(r.substr(0, dash));
                if (dash + 1 < r.size()) b = std::min<uint64_t>(std::stoull(r.substr(dash + 1)), size ? size - 1 : 0);
              }
              unsat = a >= size || b < a;
            }
          }
          const std::string common = "ETag: " + etag_of(st) + "\r\nLast-Modified: " + http_date(st.st_mtim.tv_sec) +
                                     "\r\nAccept-Ranges: bytes\r\nContent-Type: application/octet-stream\r\n";
          if (ranged && unsat) {
            ok = reply(416, "Content-Range: bytes */" + std::to_string(size) + "\r\n", "", method == "HEAD");
          } else {
            const uint64_t n = size ? b - a + 1 : 0;
            const int code = ranged ? 206 : 200;
            std::string extra = common;
            if (ranged)
              extra += "Content-Range: bytes " + std::to_string(a) + "-" + std::to_string(b) + "/" + std::to_string(size) +
                       "\r\n";
            ok = reply(code, extra, "", true, (int64_t)n);
            if (ok && method == "GET" && n) {
              const int in = ::open(fpath.c_str(), O_RDONLY | O_CLOEXEC);
              if (in < 0) {
                ok = false;
              } else {
                off_t o = (off_t)a;
                uint64_t left = n;
                const uint64_t stop_at = fault == 4 ? n / 2 : 0;   // body stall: half, then silence
                while (left > stop_at) {
                  const ssize_t r = ::sendfile(fd, in, &o, (size_t)std::min<uint64_t>(left - stop_at, 1ull << 30));
                  if (r < 0 && (errno == EINTR || errno == EAGAIN)) continue;
                  if (r <= 0) break;
                  left -= (uint64_t)r;
                  bytes_ += (uint64_t)r;
                }
                ::close(in);
                if (fault == 4) {
                  stall(fault_ms);
                  goto done;
                }
                ok = left == 0;
              }
            }
          }
        }
      } else if (method == "PUT") {
        // ---- object writes ----
        if (h.count("x-amz-copy-source")) {
          body_string();
          std::string srcp = pct_decode(h["x-amz-copy-source"], false);
          if (!srcp.empty() && srcp[0] == '/') srcp = srcp.substr(1);
          struct stat st;
          const std::string sfile = root_ + "/" + srcp;
          if (srcp.find("..") != std::string::npos) {
            ok = error(400, "InvalidArgument", srcp);
          } else if (!srcp.empty() && srcp.back() == '/') {
            mkdirs(fpath);
            const int m = ::open((fpath + "/" + kMarker).c_str(), O_WRONLY | O_CREAT | O_CLOEXEC, 0644);
            if (m >= 0) ::close(m);
            ok = reply(200, "Content-Type: application/xml\r\n", "<CopyObjectResult></CopyObjectResult>");
          } else if (!is_file(sfile, &st)) {
            ok = error(404, "NoSuchKey", srcp);
          } else {
            mkdirs(fpath.substr(0, fpath.rfind('/')));
            const std::string tmpf = fpath + ".__copy";
            const int in = ::open(sfile.c_str(), O_RDONLY | O_CLOEXEC);
            const int out = ::open(tmpf.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
            bool good = in >= 0 && out >= 0;
            off_t o = 0;
            while (good && o < st.st_size) {
              const ssize_t r = ::sendfile(out, in, &o, (size_t)(st.st_size - o));
              if (r <= 0) good = false;
            }
            if (in >= 0) ::close(in);
            if (out >= 0) ::close(out);
            if (good && ::rename(tmpf.c_str(), fpath.c_str()) == 0 && is_file(fpath, &st)) {
              ok = reply(200, "Content-Type: application/xml\r\n",
                         "<CopyObjectResult><ETag>" + xml_escape(etag_of(st)) + "</ETag><LastModified>" +
                             iso_date(st.st_mtim.tv_sec) + "</LastModified></CopyObjectResult>");
            } else {
              ::unlink(tmpf.c_str());
              ok = error(500, "InternalError", "copy failed");
            }
          }
        } else if (marker_key) {
          body_string();
          mkdirs(fpath);
          const int m = ::open((fpath + "/" + kMarker).c_str(), O_WRONLY | O_CREAT | O_CLOEXEC, 0644);
          if (m >= 0) ::close(m);
          ok = reply(200, "ETag: \"d41d8cd98f00b204e9800998ecf8427e\"\r\n", "");
        } else if (is_dir(fpath)) {
          body_string();
          ok = error(409, "InvalidRequest", "a prefix of that name exists");
        } else {
          mkdirs(fpath.substr(0, fpath.rfind('/')));
          const std::string tmpf = fpath + ".__put" + std::to_string(++upload_seq_);
          const int out = ::open(tmpf.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
          const bool wrote = out >= 0 && body_to_fd(out);
          if (out >= 0) ::close(out);
          struct stat st;
          if (wrote && ::rename(tmpf.c_str(), fpath.c_str()) == 0 && is_file(fpath, &st)) {
            ok = reply(200, "ETag: " + etag_of(st) + "\r\n", "");
          } else {
            ::unlink(tmpf.c_str());
            body_string();
            ok = error(500, "InternalError", "write failed");
          }
        }
      } else if (method == "DELETE") {
        body_string();
        if (marker_key) {
          ::unlink((fpath + "/" + kMarker).c_str());
          prune(fpath, bdir);
        } else if (::unlink(fpath.c_str()) == 0) {
          prune(fpath.substr(0, fpath.rfind('/')), bdir);
        }
        ok = reply(204, "", "");
      } else {
        body_string();
        ok = error(400, "InvalidRequest", method);
      }
      if (!ok || !keep) goto done;
    }
  }
done:
  return;
}

// ------------------------------------------------------------------------------------------------
// HttpRangeReader
// ------------------------------------------------------------------------------------------------

// One attempt's limits: the call's deadline (all attempts), the socket's silence limit, a cancel
// flag.  Sockets carry a short SO_RCVTIMEO/SO_SNDTIMEO slice, so a blocked recv/send comes back
// every kSliceMs to look at these without a poll() per call on the fast path.
struct HttpRangeReader::Io {
  int64_t deadline_ns = 0;            // 0 = none
  int socket_ms = 0;                  // 0 = no silence limit
  const std::atomic<bool>* cancel = nullptr;
  int64_t err = 0;                    // first failure of the attempt: kHttp* code
  bool expired() const { return deadline_ns && mono_ns() >= deadline_ns; }
  bool cancelled() const { return cancel && cancel->load(std::memory_order_relaxed); }
  static int64_t mono_ns() {
    timespec t;
    ::clock_gettime(CLOCK_MONOTONIC, &t);
    return (int64_t)t.tv_sec * 1000000000LL + t.tv_nsec;
  }
};

namespace {
constexpr int kSliceMs = 100;

// Waits out one EAGAIN of a socket with a SO_*TIMEO slice: false (with io.err set) once the call is
// cancelled, past its deadline, or the socket has been silent for socket_ms since `since_ns`.
template <class IoT>
bool still_waiting(IoT& io, int64_t since_ns) {
  if (io.cancelled()) {
    io.err = kHttpCancelled;
    return false;
  }
  const int64_t now = IoT::mono_ns();
  if ((io.deadline_ns && now >= io.deadline_ns) ||
      (io.socket_ms > 0 && now - since_ns >= (int64_t)io.socket_ms * 1000000LL)) {
    io.err = kHttpTimeout;
    return false;
  }
  return true;
}

template <class IoT>
bool io_send_all(int fd, const char* p, size_t n, IoT& io) {
  int64_t since = IoT::mono_ns();
  while (n) {
    const ssize_t r = ::send(fd, p, n, MSG_NOSIGNAL);
    if (r > 0) {
      p += r;
      n -= (size_t)r;
      since = IoT::mono_ns();
      continue;
    }
    if (r < 0 && errno == EINTR) continue;
    if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      if (!still_waiting(io, since)) return false;
      continue;
    }
    io.err = kHttpTransportError;
    return false;
  }
  return true;
}

// Up to n bytes (at least 1); 0 with io.err set on EOF / error / timeout / cancel.
template <class IoT>
size_t io_recv_some(int fd, uint8_t* p, size_t n, IoT& io) {
  const int64_t since = IoT::mono_ns();
  for (;;) {
    const ssize_t r = ::recv(fd, p, n, 0);
    if (r > 0) return (size_t)r;
    if (r < 0 && errno == EINTR) continue;
    if (r < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      if (!still_waiting(io, since)) return 0;
      continue;
    }
    io.err = kHttpTransportError;       // EOF (a reset or a closed keep-alive) or an error
    return 0;
  }
}

template <class IoT>
bool io_recv_all(int fd, uint8_t* p, size_t n, IoT& io) {
  while (n) {
    const size_t r = io_recv_some(fd, p, n, io);
    if (!r) return false;
    p += r;
    n -= r;
  }
  return true;
}

void set_slices(int fd) {
  timeval tv{0, kSliceMs * 1000};
  ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
}
}  // namespace

HttpRangeReader::HttpRangeReader(const std::string& host, int port, int max_idle, HttpOptions opts)
    : host_(host), port_(port), max_idle_((size_t)std::max(1, max_idle)), opts_(opts) {}

HttpRangeReader::~HttpRangeReader() {
  for (int fd : idle_) ::close(fd);
}

bool HttpRangeReader::retryable(int64_t code) {
  return code == kHttpTransportError || code == kHttpTimeout || code == -500 || code == -502 || code == -503 ||
         code == -504 || code == -429 || code == 500 || code == 502 || code == 503 || code == 504 || code == 429;
}

int HttpRangeReader::take(bool& reused, Io& io) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!idle_.empty()) {
      const int fd = idle_.back();
      idle_.pop_back();
      reused = true;
      return fd;
    }
  }
  reused = false;
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (::getaddrinfo(host_.c_str(), std::to_string(port_).c_str(), &hints, &res) != 0 || !res) {
    io.err = kHttpTransportError;
    return -1;
  }
  // non-blocking connect bounded by the connect timeout (and the call's deadline / cancel)
  const int fd = ::socket(res->ai_family, res->ai_socktype | SOCK_CLOEXEC | SOCK_NONBLOCK, res->ai_protocol);
  int rc = fd < 0 ? -1 : ::connect(fd, res->ai_addr, res->ai_addrlen);
  ::freeaddrinfo(res);
  if (fd < 0) {
    io.err = kHttpTransportError;
    return -1;
  }
  if (rc != 0 && errno == EINPROGRESS) {
    const int64_t t0 = Io::mono_ns();
    const int64_t limit = (int64_t)std::max(1, opts_.connect_timeout_ms) * 1000000LL;
    rc = -1;
    for (;;) {
      pollfd pf{fd, POLLOUT, 0};
      const int pr = ::poll(&pf, 1, kSliceMs);
      if (pr == 1) {
        int e = 0;
        socklen_t el = sizeof e;
        rc = (::getsockopt(fd, SOL_SOCKET, SO_ERROR, &e, &el) == 0 && e == 0) ? 0 : -1;
        if (rc != 0) io.err = kHttpTransportError;
        break;
      }
      if (pr < 0 && errno != EINTR) {
        io.err = kHttpTransportError;
        break;
      }
      if (io.cancelled()) {
        io.err = kHttpCancelled;
        break;
      }
      if (io.expired() || Io::mono_ns() - t0 >= limit) {
        io.err = kHttpTimeout;
        break;
      }
    }
  } else if (rc != 0) {
    io.err = kHttpTransportError;
  }
  if (rc != 0) {
    ::close(fd);
    return -1;
  }
  const int fl = ::fcntl(fd, F_GETFL);
  ::fcntl(fd, F_SETFL, fl & ~O_NONBLOCK);
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  int rcv = 8 << 20;
  ::setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &rcv, sizeof rcv);
  set_slices(fd);
  ++connects_;
  return fd;
}

void HttpRangeReader::give(int fd) {
  std::lock_guard<std::mutex> g(mu_);
  if (idle_.size() < max_idle_) idle_.push_back(fd);
  else ::close(fd);
}

bool HttpRangeReader::backoff(int attempt, Io& io) {
  thread_local uint64_t seed = (uint64_t)Io::mono_ns() ^ (uint64_t)(uintptr_t)&seed;
  seed = seed * 6364136223846793005ULL + 1442695040888963407ULL;
  const int64_t cap = (int64_t)opts_.backoff_max_ms;
  const int64_t exp = std::min<int64_t>(cap, (int64_t)opts_.backoff_base_ms << std::min(attempt - 1, 20));
  const int64_t ms = exp / 2 + (int64_t)((seed >> 33) % (uint64_t)(exp / 2 + 1));   // "equal jitter"
  const int64_t until = Io::mono_ns() + ms * 1000000LL;
  while (Io::mono_ns() < until) {
    if (io.cancelled()) {
      io.err = kHttpCancelled;
      return false;
    }
    if (io.expired()) {
      io.err = kHttpTimeout;
      return false;
    }
    ::usleep((useconds_t)std::min<int64_t>(kSliceMs * 1000, std::max<int64_t>(1, (until - Io::mono_ns()) / 1000)));
  }
  return true;
}

int64_t HttpRangeReader::one(const std::string& target, const std::string& head, uint64_t off, uint64_t len,
                             uint8_t* dst, Io& io) {
  const std::string req = "GET " + target + " HTTP/1.1\r\n" + head +
                          "Range: bytes=" + std::to_string(off) + "-" + std::to_string(off + len - 1) + "\r\n\r\n";
  int stale = 0;                         // pooled connections the server had closed: free retries
  for (int attempt = 0;;) {
    io.err = 0;
    bool reused = false;
    const int fd = take(reused, io);
    int64_t result = 0;
    if (fd < 0) {
      result = io.err ? io.err : kHttpTransportError;
    } else {
      ++requests_;
      std::string hb;
      char tmp[16384];
      size_t hend = std::string::npos;
      bool fail = !io_send_all(fd, req.data(), req.size(), io);
      while (!fail && (hend = hb.find("\r\n\r\n")) == std::string::npos) {
        const size_t r = io_recv_some(fd, reinterpret_cast<uint8_t*>(tmp), sizeof tmp, io);
        if (!r || hb.size() > kMaxHead) {
          if (!io.err) io.err = kHttpTransportError;
          fail = true;
          break;
        }
        hb.append(tmp, r);
      }
      if (fail) {
        ::close(fd);
        if (reused && hb.empty() && io.err == kHttpTransportError && stale++ < 4) continue;
        result = io.err;
      } else {
        int code = 0;
        if (hb.size() > 12) code = std::atoi(hb.c_str() + 9);
        uint64_t clen = 0;
        bool close_after = false;
        for (size_t p = hb.find("\r\n"); p != std::string::npos && p < hend;) {
          const size_t e = hb.find("\r\n", p + 2);
          const std::string l = lower(hb.substr(p + 2, e - p - 2));
          if (starts_with(l, "content-length:")) clen = std::stoull(l.substr(15));
          if (starts_with(l, "connection:") && l.find("close") != std::string::npos) close_after = true;
          p = e;
        }
        const size_t have = hb.size() - (hend + 4);
        const uint8_t* pre = reinterpret_cast<const uint8_t*>(hb.data() + hend + 4);
        // the body: the requested range lands in dst, anything else is drained
        uint64_t skip = 0, take_n = 0;
        if ((code == 206 && clen == len) || (code == 200 && clen == len && off == 0)) {
          take_n = len;
          result = (int64_t)len;
        } else if (code == 200 && clen >= off + len) {
          skip = off;              // the server ignored the range: the object from byte 0
          take_n = len;
          result = (int64_t)len;
        } else {
          result = code ? -(int64_t)code : kHttpTransportError;
        }
        uint64_t pos = 0;          // body bytes consumed
        auto consume = [&](const uint8_t* p, size_t n) {
          for (size_t i = 0; i < n;) {
            if (pos < skip) {
              const size_t k = (size_t)std::min<uint64_t>(skip - pos, n - i);
              pos += k;
              i += k;
            } else if (pos < skip + take_n) {
              const size_t k = (size_t)std::min<uint64_t>(skip + take_n - pos, n - i);
              std::memcpy(dst + (pos - skip), p + i, k);
              pos += k;
              i += k;
            } else {
              pos += n - i;
              i = n;
            }
          }
        };
        consume(pre, (size_t)std::min<uint64_t>(have, clen));
        bool ok = true;
        while (ok && pos < clen) {
          if (pos >= skip && pos < skip + take_n) {
            const size_t k = (size_t)(skip + take_n - pos);     // straight into the destination
            if (!io_recv_all(fd, dst + (pos - skip), k, io)) ok = false;
            else pos += k;
          } else {
            const size_t k = (size_t)std::min<uint64_t>(clen - pos, sizeof tmp);
            const size_t r = io_recv_some(fd, reinterpret_cast<uint8_t*>(tmp), k, io);
            if (!r) ok = false;
            else consume(reinterpret_cast<const uint8_t*>(tmp), r);
          }
        }
        if (!ok) {
          ::close(fd);
          result = io.err ? io.err : kHttpTransportError;   // a short body: the whole range again
        } else if (close_after) {
          ::close(fd);
        } else {
          give(fd);
        }
      }
    }
    if (result >= 0 || !retryable(result) || attempt >= opts_.max_retries) {
      if (result == kHttpTimeout) ++timeouts_;
      return result;
    }
    ++attempt;
    ++retries_;
    if (!backoff(attempt, io)) {
      if (io.err == kHttpTimeout) ++timeouts_;
      return io.err;
    }
  }
}

int HttpRangeReader::put_from(const std::string& target, const std::string& head, uint64_t src, uint64_t len,
                              std::string* etag, const std::atomic<bool>* cancel) {
  return request("PUT", target, head, reinterpret_cast<const uint8_t*>(src), len, nullptr, etag, cancel);
}

int HttpRangeReader::request_once(const std::string& req, const uint8_t* body, uint64_t len, std::string* resp,
                                  std::string* etag, Io& io) {
  for (int stale = 0;;) {
    io.err = 0;
    bool reused = false;
    const int fd = take(reused, io);
    if (fd < 0) return (int)(io.err ? io.err : kHttpTransportError);
    ++requests_;
    if (!io_send_all(fd, req.data(), req.size(), io) ||
        (len && !io_send_all(fd, reinterpret_cast<const char*>(body), (size_t)len, io))) {
      ::close(fd);
      if (reused && io.err == kHttpTransportError && stale++ < 4) continue;   // closed keep-alive: fresh
      return (int)io.err;
    }
    std::string hb;
    char tmp[16384];
    size_t hend;
    bool fail = false;
    while ((hend = hb.find("\r\n\r\n")) == std::string::npos) {
      const size_t r = io_recv_some(fd, reinterpret_cast<uint8_t*>(tmp), sizeof tmp, io);
      if (!r || hb.size() > kMaxHead) {
        if (!io.err) io.err = kHttpTransportError;
        fail = true;
        break;
      }
      hb.append(tmp, r);
    }
    if (fail) {
      ::close(fd);
      if (reused && hb.empty() && io.err == kHttpTransportError && stale++ < 4) continue;
      return (int)io.err;
    }
    const int code = hb.size() > 12 ? std::atoi(hb.c_str() + 9) : 0;
    uint64_t clen = 0;
    bool close_after = false;
    for (size_t p = hb.find("\r\n"); p != std::string::npos && p < hend;) {
      const size_t e = hb.find("\r\n", p + 2);
      const std::string line = hb.substr(p + 2, e - p - 2);
      const std::string l = lower(line);
      if (starts_with(l, "content-length:")) clen = std::stoull(l.substr(15));
      if (starts_with(l, "connection:") && l.find("close") != std::string::npos) close_after = true;
      if (starts_with(l, "etag:") && etag) {
        std::string v = line.substr(5);
        while (!v.empty() && (v.front() == ' ' || v.front() == '\t')) v.erase(0, 1);
        *etag = v;
      }
      p = e;
    }
    uint64_t have = hb.size() - (hend + 4);
    if (resp) resp->assign(hb, hend + 4, std::string::npos);
    bool ok = true;
    while (ok && have < clen) {   // the body (kept up to 1 MiB), drained so the connection is reusable
      const size_t r = io_recv_some(fd, reinterpret_cast<uint8_t*>(tmp), (size_t)std::min<uint64_t>(clen - have, sizeof tmp), io);
      if (!r) {
        ok = false;
      } else {
        if (resp && resp->size() < (1u << 20)) resp->append(tmp, r);
        have += r;
      }
    }
    if (!ok || close_after) ::close(fd);
    else give(fd);
    if (!ok) return (int)(io.err ? io.err : kHttpTransportError);
    return code ? code : (int)kHttpTransportError;
  }
}

int HttpRangeReader::request(const std::string& method, const std::string& target, const std::string& head,
                             const uint8_t* body, uint64_t len, std::string* resp, std::string* etag,
                             const std::atomic<bool>* cancel) {
  const std::string req = method + " " + target + " HTTP/1.1\r\n" + head + "Content-Length: " +
                          std::to_string(len) + "\r\n\r\n";
  Io io;
  io.cancel = cancel;
  io.socket_ms = opts_.socket_timeout_ms;
  if (opts_.request_timeout_ms > 0) io.deadline_ns = Io::mono_ns() + (int64_t)opts_.request_timeout_ms * 1000000LL;
  for (int attempt = 0;;) {
    if (resp) resp->clear();
    const int code = request_once(req, body, len, resp, etag, io);
    if (!retryable(code) || attempt >= opts_.max_retries) {
      if (code == kHttpTimeout) ++timeouts_;
      return code;
    }
    ++attempt;
    ++retries_;
    if (!backoff(attempt, io)) {
      if (io.err == kHttpTimeout) ++timeouts_;
      return (int)io.err;
    }
  }
}

int64_t HttpRangeReader::get_into(const std::string& target, const std::string& head_lines, uint64_t offset,
                                  uint64_t length, uint64_t dst, int parallel, uint64_t min_part,
                                  const std::atomic<bool>* cancel) {
  if (!length) return 0;
  uint8_t* const out = reinterpret_cast<uint8_t*>(dst);
  min_part = std::max<uint64_t>(min_part, 64 << 10);
  const uint64_t nparts = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(1, parallel),
                                                                   (length + min_part - 1) / min_part));
  uint64_t part = (length + nparts - 1) / nparts;
  part = (part + (64 << 10) - 1) & ~uint64_t((64 << 10) - 1);
  std::vector<int64_t> res((size_t)nparts, 0);
  const int64_t deadline =
      opts_.request_timeout_ms > 0 ? Io::mono_ns() + (int64_t)opts_.request_timeout_ms * 1000000LL : 0;
  auto run = [&](size_t i, uint64_t a, uint64_t n) {
    Io io;
    io.cancel = cancel;
    io.socket_ms = opts_.socket_timeout_ms;
    io.deadline_ns = deadline;
    res[i] = one(target, head_lines, offset + a, n, out + a, io);
  };
  std::vector<std::thread> ts;
  for (uint64_t i = 1; i < nparts; ++i) {
    const uint64_t a = i * part;
    if (a >= length) break;
    const uint64_t n = std::min(part, length - a);
    ts.emplace_back([&, i, a, n] { run((size_t)i, a, n); });
  }
  run(0, 0, std::min(part, length));
  for (auto& t : ts) t.join();
  for (int64_t r : res)
    if (r < 0) return r;
  return (int64_t)length;
}

}  // namespace amdx
