// Native UFS journal log writer with group commit (the master's metadata write path).
//
// Reference: core/server/common/src/main/java/alluxio/master/journal/AsyncJournalWriter.java
// (:243-295 doFlush, :334 flush) over ufs/UfsJournalLogWriter.java (:115-209 write / rotate /
// complete).  The Python AsyncJournalWriter ran its flush loop on a Python thread: under load it
// waited for the GIL twice per group commit (to write the batch and to release the waiting RPCs),
// so one commit took several GIL switch intervals on top of the fsync.  Here the flush thread never
// touches Python: handlers append serialized entries, the thread frames them (length-delimited,
// the sequence number prepended as JournalEntry field 1), writes and fdatasyncs the current log
// segment, rotates segments by size, and sends the replies of the RPCs the commit released
// straight through the native RPC server (FrameRpcServer::respond_batch).
//
// Segment files follow the UFS journal layout: "0x<start>-0x7fffffffffffffff" while being written,
// renamed to "0x<start>-0x<end>" (end exclusive) when rotated or closed.
#pragma once
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "frame_rpc.h"

namespace amdx {

class JournalLog {
 public:
  JournalLog(const std::string& log_dir, uint64_t next_seq, uint64_t max_log_bytes, bool fsync, double batch_ms);
  ~JournalLog();
  // Queue one serialized JournalEntry (its sequence_number unset); returns its counter (1-based
  // count of entries appended).  Throws std::runtime_error once closed or failed.
  uint64_t append(const std::string& entry);
  // Ask for a flush up to `counter` without waiting.
  void request(uint64_t counter);
  // Wait (up to timeout_ms; < 0 = forever) until entries up to `counter` are durable: 0 = done,
  // 1 = timed out; throws on a failed / closed journal.
  int wait_flushed(uint64_t counter, int timeout_ms);
  // Send `reply` through `srv` once entries up to `counter` are durable (an UNAVAILABLE reply if
  // the journal fails first).  `srv` must outlive the journal (the master stops the journal first).
  void reply_when_flushed(uint64_t counter, FrameRpcServer* srv, FrameReply reply);
  // Flush what is queued, fsync and complete the current segment; later appends throw.
  void close();
  uint64_t next_seq();
  uint64_t appended();
  uint64_t flushed();
  std::string error();
  uint64_t flushes() const { return flushes_; }
  // Commit timing: {entries, flushes, write_us, fsync_us, reply_us, wait_us (sum over entries of
  // append -> durable), wait_max_us}.
  std::vector<uint64_t> stats();
  uint64_t segments() const { return segments_; }

 private:
  void run();
  bool write_batch(std::vector<std::string>& batch, uint64_t first_seq, std::string* err);
  bool rotate(uint64_t start_seq, std::string* err);
  bool complete_current(std::string* err);
  void fail_waiters_locked(const std::string& err, std::vector<std::pair<FrameRpcServer*, FrameReply>>* out);

  const std::string dir_;
  const uint64_t max_bytes_;
  const bool fsync_;
  const double batch_s_;
  std::mutex mu_;
  std::condition_variable cv_;       // flush thread wakeups
  std::condition_variable done_cv_;  // flush progress (wait_flushed)
  std::vector<std::string> queue_;
  std::vector<std::chrono::steady_clock::time_point> queued_at_;
  uint64_t st_entries_ = 0, st_write_us_ = 0, st_fsync_us_ = 0, st_reply_us_ = 0, st_wait_us_ = 0, st_wait_max_ = 0;
  uint64_t next_seq_;                // sequence number of the next appended entry
  uint64_t appended_ = 0, written_ = 0, flushed_ = 0, requested_ = 0;
  bool closed_ = false, stop_ = false, finished_ = false;
  std::mutex close_mu_;
  std::string error_;
  std::multimap<uint64_t, std::pair<FrameRpcServer*, FrameReply>> replies_;
  // current segment (flush thread only)
  int fd_ = -1;
  std::string cur_path_;
  uint64_t cur_start_ = 0, cur_bytes_ = 0, file_seq_ = 0;
  uint64_t flushes_ = 0, segments_ = 0;
  std::chrono::steady_clock::time_point last_write_done_;
  std::thread thread_;
};

}  // namespace amdx
