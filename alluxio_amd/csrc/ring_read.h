// Device-cursor multi-stream sequential reader (see SeqReadArgs in kernels.h).
//
// The StressWorkerBench loop (stress/shell/.../StressWorkerBench.java:251-276: T threads each
// call read(buf) over one file and reopen at EOF) with `depth` calls per stream issued per
// launch into a per-stream ring of `depth` buffers.  The session read-locks every block of the
// file for its lifetime, uploads the file's page table once, and then each step is ONE kernel
// launch whose arguments are scalars — host work is O(1) per step, independent of the number of
// streams or calls, which is what makes small (4 KiB) reads run at HBM speed.
#pragma once
#include <cstdint>
#include <vector>

#include "block_store.h"

namespace amdx {

class RingReadSession {
 public:
  RingReadSession(BlockStore* store, int64_t session, const std::vector<int64_t>& block_ids,
                  const std::vector<uint64_t>& block_lens, uint64_t dst_base, uint64_t stream_stride,
                  uint64_t buf_bytes, uint32_t depth, uint32_t streams, int dst_kind,
                  const std::vector<uint64_t>& start_offsets);
  // Remote (peer) form: the file's pages live in an arena that is already addressable from this
  // process (a peer worker's HBM mapped through HIP IPC, read over xGMI by the kernel running on
  // `device`), described by `file_pages` (arena page index per file page).  Block locks are held
  // by the caller (OpenDeviceBlock) for the session's lifetime.  device < 0: host arena (tests).
  RingReadSession(uint64_t arena_base, const std::vector<int64_t>& file_pages, uint64_t page_size,
                  uint64_t file_len, int device, uint64_t dst_base, uint64_t stream_stride, uint64_t buf_bytes,
                  uint32_t depth, uint32_t streams, int dst_kind, const std::vector<uint64_t>& start_offsets);
  ~RingReadSession();
  // One launch: every stream issues `depth` read calls.  Returns bytes read; *eofs = EOF calls
  // (reopens) in this step.
  uint64_t step(uint64_t stream, uint64_t* eofs);
  void close();
  uint64_t total_bytes() const { return total_; }
  uint64_t reopens() const { return reopens_; }
  uint64_t calls() const { return calls_per_stream_; }
  // File offset of stream s's next read.
  uint64_t position(uint32_t s) const;
  // (file offset, length) of stream s's k-th call in the most recent step (length 0 = EOF).
  std::pair<uint64_t, uint64_t> last_call(uint32_t s, uint32_t k) const;
  uint64_t file_len() const { return file_len_; }

 private:
  uint64_t bytes_before(uint64_t g) const;  // bytes read by calls [0, g) of one stream
  void check_shape();
  void finish_init(const std::vector<uint64_t>& start_offsets);
  void set_device() const;
  BlockStore* store_;                       // null for the remote form
  int64_t session_;
  std::vector<int64_t> blocks_, locks_;
  uint64_t file_len_ = 0, buf_, stride_, dst_;
  uint32_t depth_, streams_, cycle_;
  int kind_;
  bool on_device_ = false;
  int device_ = -1;
  int dir_ = -1;
  uint64_t page_size_ = 0, arena_ = 0;
  uint32_t page_shift_ = 0;
  std::vector<int64_t> ftab_;
  std::vector<uint64_t> c_init_;
  uint64_t footprint_ = 0;   // distinct file bytes one step touches (see finish_init)
  int64_t* d_ftab_ = nullptr;
  uint64_t* d_cinit_ = nullptr;
  uint64_t calls_per_stream_ = 0, total_ = 0, reopens_ = 0;
  bool closed_ = false;
};

}  // namespace amdx
