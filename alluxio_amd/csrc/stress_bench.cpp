// Native StressWorkerBench client (see stress_bench.h).
#include "stress_bench.h"

#include <pthread.h>

#include <atomic>
#include <chrono>
#include <memory>
#include <mutex>
#include <thread>

namespace amdx {

namespace {

std::shared_ptr<BlockSource> open_source(const BenchBlock& b) {
  switch (b.kind) {
    case 1: return std::make_shared<DeviceArenaSource>(b.base, b.pages, b.page_size, b.length, b.device);
    case 2: return std::make_shared<HostArenaSource>(b.base, b.pages, b.page_size, b.length);
    default: return std::make_shared<GrpcBlockSource>(b.grpc, b.length);
  }
}

}  // namespace

BenchResult run_stress_reads(const std::vector<BenchBlock>& blocks, uint64_t block_size, int threads,
                             uint64_t buffer, uint64_t chunk, double warmup_s, double duration_s, bool prefetch) {
  BenchResult res;
  if (blocks.empty() || threads <= 0 || buffer == 0 || block_size == 0) return res;
  uint64_t length = 0;
  for (const auto& b : blocks) length += b.length;
  // 0 warming up, 1 recording, 2 stop: one relaxed load per read(buf)
  std::atomic<int> phase{0};
  std::vector<uint64_t> bytes((size_t)threads, 0), reads((size_t)threads, 0), opens((size_t)threads, 0),
      block_opens((size_t)threads, 0);
  std::mutex err_mu;
  std::vector<std::thread> ts;
  ts.reserve((size_t)threads);
  for (int t = 0; t < threads; ++t) {
    ts.emplace_back([&, t] {
      pthread_setname_np(pthread_self(), "stress-reader");
      std::vector<uint8_t> buf(buffer);
      uint64_t my_bytes = 0, my_reads = 0, my_opens = 0, my_blocks = 0;
      try {
        while (phase.load(std::memory_order_relaxed) < 2) {
          HostInStream s(length, block_size, chunk, prefetch);     // FileSystem.openFile
          ++my_opens;
          while (s.pos() < length) {
            const int ph = phase.load(std::memory_order_relaxed);
            if (ph >= 2) break;
            const uint64_t n = std::min<uint64_t>(buffer, length - s.pos());
            if (!s.fast(buf.data(), n)) {
              uint64_t done = 0;
              while (done < n) {
                const int64_t idx = (int64_t)(s.pos() / block_size);
                if (s.block_index() != idx || !s.source()) {
                  s.set_source(idx, open_source(blocks[(size_t)idx]));
                  ++my_blocks;
                }
                const uint64_t have = s.copy_buffered(buf.data() + done, n - done);
                if (have) {
                  done += have;
                  continue;
                }
                done += s.read_block_part(buf.data() + done, n - done);
              }
            }
            if (ph == 1) {
              my_bytes += n;
              ++my_reads;
            }
          }
          s.drop_source();                                        // FileInStream.close
        }
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> g(err_mu);
        res.errors.push_back(e.what());
      }
      bytes[(size_t)t] = my_bytes;
      reads[(size_t)t] = my_reads;
      opens[(size_t)t] = my_opens;
      block_opens[(size_t)t] = my_blocks;
    });
  }
  using clock = std::chrono::steady_clock;
  std::this_thread::sleep_for(std::chrono::duration<double>(warmup_s));
  const auto t0 = clock::now();
  phase.store(1, std::memory_order_relaxed);
  std::this_thread::sleep_for(std::chrono::duration<double>(duration_s));
  phase.store(2, std::memory_order_relaxed);
  const auto t1 = clock::now();
  for (auto& th : ts) th.join();
  res.seconds = std::chrono::duration<double>(t1 - t0).count();
  res.per_thread = bytes;
  for (int t = 0; t < threads; ++t) {
    res.bytes += bytes[(size_t)t];
    res.reads += reads[(size_t)t];
    res.opens += opens[(size_t)t];
    res.block_opens += block_opens[(size_t)t];
  }
  return res;
}

}  // namespace amdx
