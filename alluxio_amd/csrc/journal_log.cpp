// Native UFS journal log writer with group commit (see journal_log.h).
#include "journal_log.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <stdexcept>

namespace amdx {
namespace {

constexpr uint64_t kUnknownSeq = (1ull << 63) - 1;
constexpr int kUnavailable = 14;   // gRPC UNAVAILABLE (the status the Python path returns too)

void put_varint(std::string& out, uint64_t v) {
  while (v >= 0x80) {
    out.push_back((char)((v & 0x7f) | 0x80));
    v >>= 7;
  }
  out.push_back((char)v);
}

size_t varint_len(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++n;
  }
  return n;
}

std::string seg_name(uint64_t start, uint64_t end) {
  char b[64];
  std::snprintf(b, sizeof(b), "0x%llx-0x%llx", (unsigned long long)start, (unsigned long long)end);
  return b;
}

bool write_all(int fd, const char* p, size_t n, std::string* err) {
  while (n > 0) {
    const ssize_t w = ::write(fd, p, n);
    if (w < 0) {
      if (errno == EINTR) continue;
      *err = std::string("journal write: ") + std::strerror(errno);
      return false;
    }
    p += w;
    n -= (size_t)w;
  }
  return true;
}

void send_grouped(std::vector<std::pair<FrameRpcServer*, FrameReply>>& out) {
  // one respond_batch per server
  while (!out.empty()) {
    FrameRpcServer* srv = out.front().first;
    std::vector<FrameReply> batch;
    std::vector<std::pair<FrameRpcServer*, FrameReply>> rest;
    for (auto& x : out) {
      if (x.first == srv) batch.push_back(std::move(x.second));
      else rest.push_back(std::move(x));
    }
    srv->respond_batch(batch);
    out.swap(rest);
  }
}

}  // namespace

JournalLog::JournalLog(const std::string& log_dir, uint64_t next_seq, uint64_t max_log_bytes, bool fsync,
                       double batch_ms)
    : dir_(log_dir), max_bytes_(max_log_bytes ? max_log_bytes : (10ull << 20)), fsync_(fsync),
      batch_s_(batch_ms / 1000.0), next_seq_(next_seq), file_seq_(next_seq) {
  thread_ = std::thread([this] { run(); });
}

JournalLog::~JournalLog() { close(); }

uint64_t JournalLog::append(const std::string& entry) {
  std::lock_guard<std::mutex> g(mu_);
  if (closed_) throw std::runtime_error("closed: journal is closed");
  if (!error_.empty()) throw std::runtime_error("failed: journal write failed: " + error_);
  const uint64_t seq = next_seq_++;
  // JournalEntry{sequence_number=1 (varint), ...entry}: field 1 first, as a serializer orders it
  const size_t body = 1 + varint_len(seq) + entry.size();
  std::string f;
  f.reserve(varint_len(body) + body);
  put_varint(f, body);
  f.push_back((char)0x08);
  put_varint(f, seq);
  f.append(entry);
  queue_.push_back(std::move(f));
  queued_at_.push_back(std::chrono::steady_clock::now());
  return ++appended_;
}

void JournalLog::request(uint64_t counter) {
  std::lock_guard<std::mutex> g(mu_);
  if (counter > requested_) {
    requested_ = counter;
    cv_.notify_one();
  }
}

int JournalLog::wait_flushed(uint64_t counter, int timeout_ms) {
  std::unique_lock<std::mutex> lk(mu_);
  if (counter > requested_) {
    requested_ = counter;
    cv_.notify_one();
  }
  auto ready = [&] { return flushed_ >= counter || !error_.empty() || finished_; };
  if (timeout_ms < 0) done_cv_.wait(lk, ready);
  else if (!done_cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready)) return 1;
  if (flushed_ >= counter) return 0;
  if (!error_.empty()) throw std::runtime_error("failed: journal flush failed: " + error_);
  throw std::runtime_error("closed: journal closed before flush");
}

void JournalLog::reply_when_flushed(uint64_t counter, FrameRpcServer* srv, FrameReply reply) {
  std::unique_lock<std::mutex> lk(mu_);
  if (flushed_ < counter && error_.empty() && !finished_) {
    replies_.emplace(counter, std::make_pair(srv, std::move(reply)));
    if (counter > requested_) {
      requested_ = counter;
      cv_.notify_one();
    }
    return;
  }
  if (flushed_ < counter) {
    reply.status = kUnavailable;
    reply.msg = error_.empty() ? std::string("journal closed before flush") : "journal flush failed: " + error_;
    reply.payload.clear();
  }
  lk.unlock();
  srv->respond_batch({reply});
}

void JournalLog::close() {
  std::lock_guard<std::mutex> cg(close_mu_);
  {
    std::lock_guard<std::mutex> g(mu_);
    closed_ = true;
    stop_ = true;
    requested_ = appended_;
    cv_.notify_all();
  }
  if (thread_.joinable() && std::this_thread::get_id() != thread_.get_id()) thread_.join();
  std::vector<std::pair<FrameRpcServer*, FrameReply>> out;
  {
    std::lock_guard<std::mutex> g(mu_);
    fail_waiters_locked(error_.empty() ? std::string("journal closed before flush") : error_, &out);
    done_cv_.notify_all();
  }
  send_grouped(out);
}

uint64_t JournalLog::next_seq() {
  std::lock_guard<std::mutex> g(mu_);
  return next_seq_;
}

uint64_t JournalLog::appended() {
  std::lock_guard<std::mutex> g(mu_);
  return appended_;
}

uint64_t JournalLog::flushed() {
  std::lock_guard<std::mutex> g(mu_);
  return flushed_;
}

std::vector<uint64_t> JournalLog::stats() {
  std::lock_guard<std::mutex> g(mu_);
  return {st_entries_, flushes_, st_write_us_, st_fsync_us_, st_reply_us_, st_wait_us_, st_wait_max_};
}

std::string JournalLog::error() {
  std::lock_guard<std::mutex> g(mu_);
  return error_;
}

void JournalLog::fail_waiters_locked(const std::string& err,
                                     std::vector<std::pair<FrameRpcServer*, FrameReply>>* out) {
  for (auto& kv : replies_) {
    FrameReply r = std::move(kv.second.second);
    r.status = kUnavailable;
    r.msg = err;
    r.payload.clear();
    out->emplace_back(kv.second.first, std::move(r));
  }
  replies_.clear();
}

bool JournalLog::complete_current(std::string* err) {
  if (fd_ < 0) return true;
  bool ok = true;
  if (fsync_ && ::fdatasync(fd_) != 0) {
    *err = std::string("journal fsync: ") + std::strerror(errno);
    ok = false;
  }
  ::close(fd_);
  fd_ = -1;
  if (!ok) return false;
  const std::string fin = dir_ + "/" + seg_name(cur_start_, file_seq_);
  if (file_seq_ <= cur_start_) {
    ::unlink(cur_path_.c_str());
  } else if (::rename(cur_path_.c_str(), fin.c_str()) != 0) {
    *err = std::string("journal complete: ") + std::strerror(errno);
    return false;
  }
  return true;
}

bool JournalLog::rotate(uint64_t start_seq, std::string* err) {
  if (!complete_current(err)) return false;
  cur_start_ = start_seq;
  cur_bytes_ = 0;
  cur_path_ = dir_ + "/" + seg_name(start_seq, kUnknownSeq);
  fd_ = ::open(cur_path_.c_str(), O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
  if (fd_ < 0) {
    *err = "journal open " + cur_path_ + ": " + std::strerror(errno);
    return false;
  }
  ++segments_;
  return true;
}

bool JournalLog::write_batch(std::vector<std::string>& batch, uint64_t first_seq, std::string* err) {
  std::string buf;
  size_t total = 0;
  for (auto& f : batch) total += f.size();
  buf.reserve(std::min<size_t>(total, 8u << 20));
  uint64_t seq = first_seq;
  for (auto& f : batch) {
    if (fd_ < 0 || cur_bytes_ >= max_bytes_) {
      if (!buf.empty()) {
        if (!write_all(fd_, buf.data(), buf.size(), err)) return false;
        buf.clear();
      }
      file_seq_ = seq;               // entries before `seq` are in the current segment
      if (!rotate(seq, err)) return false;
    }
    buf.append(f);
    cur_bytes_ += f.size();
    ++seq;
  }
  if (!buf.empty() && !write_all(fd_, buf.data(), buf.size(), err)) return false;
  file_seq_ = seq;
  last_write_done_ = std::chrono::steady_clock::now();
  if (fsync_ && fd_ >= 0 && ::fdatasync(fd_) != 0) {
    *err = std::string("journal fsync: ") + std::strerror(errno);
    return false;
  }
  return true;
}

void JournalLog::run() {
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    bool have_since = false;
    auto since = std::chrono::steady_clock::now();
    for (;;) {
      if (stop_ && queue_.empty()) goto out;
      if (!queue_.empty() && (requested_ > written_ || closed_)) break;
      if (!queue_.empty()) {
        const auto now = std::chrono::steady_clock::now();
        if (!have_since) {
          since = now;
          have_since = true;
        }
        const double el = std::chrono::duration<double>(now - since).count();
        if (el >= batch_s_) break;
        cv_.wait_for(lk, std::chrono::duration<double>(batch_s_ - el));
      } else {
        have_since = false;
        cv_.wait_for(lk, std::chrono::milliseconds(100));
      }
    }
    {
      std::vector<std::string> batch;
      batch.swap(queue_);
      std::vector<std::chrono::steady_clock::time_point> at;
      at.swap(queued_at_);
      const uint64_t n = batch.size();
      const auto t0 = std::chrono::steady_clock::now();
      const uint64_t first = next_seq_ - (appended_ - written_);   // seq of the oldest unwritten entry
      lk.unlock();
      std::string err;
      const bool ok = write_batch(batch, first, &err);
      batch.clear();
      std::vector<std::pair<FrameRpcServer*, FrameReply>> out;
      lk.lock();
      if (!ok) {
        error_ = err;
        fail_waiters_locked("journal flush failed: " + err, &out);
        done_cv_.notify_all();
        lk.unlock();
        send_grouped(out);
        lk.lock();
        stop_ = true;
        queue_.clear();
        break;
      }
      const auto t1 = std::chrono::steady_clock::now();
      auto us = [](std::chrono::steady_clock::duration d) {
        return (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(d).count();
      };
      st_write_us_ += us(last_write_done_ - t0);
      st_fsync_us_ += us(t1 - last_write_done_);
      st_entries_ += n;
      for (auto& a : at) {
        const uint64_t w = us(t1 - a);
        st_wait_us_ += w;
        st_wait_max_ = std::max(st_wait_max_, w);
      }
      written_ += n;
      flushed_ = written_;
      ++flushes_;
      while (!replies_.empty() && replies_.begin()->first <= flushed_) {
        out.push_back(std::move(replies_.begin()->second));
        replies_.erase(replies_.begin());
      }
      done_cv_.notify_all();
      if (!out.empty()) {
        lk.unlock();
        send_grouped(out);
        const uint64_t r = us(std::chrono::steady_clock::now() - t1);
        lk.lock();
        st_reply_us_ += r;
      }
    }
  }
out:
  {
    std::string err;
    lk.unlock();
    const bool ok = complete_current(&err);
    lk.lock();
    if (!ok && error_.empty()) error_ = err;
  }
  finished_ = true;
  done_cv_.notify_all();
}

}  // namespace amdx
