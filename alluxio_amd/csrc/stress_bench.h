// Native client of StressWorkerBench: T C++ threads in one process, each looping read(buf) over
// one file and re-opening it at EOF, with no interpreter in the loop.
//
// Reference: stress/shell/src/main/java/alluxio/stress/cli/worker/StressWorkerBench.java:153,251-276
// (256 JVM threads, one FileInStream each, read(buf) until EOF, then a fresh stream) and
// stress/common/src/main/java/alluxio/stress/worker/WorkerBenchSummary.java:59-71 (MB/s = bytes
// read after warmup / duration).  Python threads share one interpreter lock, so the Python form of
// the bench (alluxio_amd/stress/worker_bench.py --mode threads) measures the interpreter at 4 KiB;
// this one measures the worker.
//
// Each thread owns a HostInStream (csrc/block_source.h: two chunk buffers, prefetch of the next
// chunk): a 4 KiB read(buf) inside the current chunk is a memcpy.  A re-open starts a new stream
// whose block sources are opened on first touch -- over gRPC a new ReadBlock call per block per
// pass (the reference's GrpcDataReader), over the short circuit a new view of the block's pages in
// the mapped arena (the worker lock of the block is taken once for the run).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "block_source.h"

namespace amdx {

// How one block of the file is opened.
struct BenchBlock {
  uint64_t length = 0;
  int kind = 0;                        // 0 gRPC ReadBlock, 1 HBM arena (HIP IPC), 2 host arena
  GrpcBlockSource::Options grpc;       // kind 0
  uint64_t base = 0;                   // kind 1/2: mapped arena base
  std::vector<int64_t> pages;
  uint64_t page_size = 0;
  int device = 0;
};

struct BenchResult {
  uint64_t bytes = 0;                  // read while recording
  uint64_t reads = 0;                  // read(buf) calls while recording
  uint64_t opens = 0;                  // file (re)opens over the whole run
  uint64_t block_opens = 0;            // block sources opened over the whole run
  double seconds = 0;                  // recording window
  std::vector<uint64_t> per_thread;    // bytes per thread while recording
  std::vector<std::string> errors;     // first error of each failed thread
};

// Runs `threads` readers over the file (`blocks` in order, `block_size` each but the last) for
// `warmup_s` + `duration_s` seconds, counting only the bytes read in the second window.
BenchResult run_stress_reads(const std::vector<BenchBlock>& blocks, uint64_t block_size, int threads,
                             uint64_t buffer, uint64_t chunk, double warmup_s, double duration_s, bool prefetch);

}  // namespace amdx
