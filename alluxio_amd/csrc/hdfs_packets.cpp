// HDFS DataTransferProtocol packets (see hdfs_packets.h).
#include "hdfs_packets.h"

#include <errno.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <exception>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "cpu_codecs.h"

namespace amdx {

namespace {

void wait_fd(int fd, short ev, int timeout_ms, const char* what) {
  pollfd pf{fd, ev, 0};
  const int r = ::poll(&pf, 1, timeout_ms);
  if (r == 0) throw StoreError(kErrTimeout, std::string("hdfs data transfer: ") + what + " timed out");
  if (r < 0 && errno != EINTR) throw StoreError(kErrIo, std::string("hdfs data transfer: poll failed on ") + what);
}

void send_iov(int fd, iovec* iov, int n, int timeout_ms) {
  while (n > 0) {
    const ssize_t w = ::writev(fd, iov, n);
    if (w < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        wait_fd(fd, POLLOUT, timeout_ms, "send");
        continue;
      }
      throw StoreError(kErrIo, "hdfs data transfer: connection lost while sending packets");
    }
    size_t left = (size_t)w;
    while (n > 0 && left >= iov->iov_len) {
      left -= iov->iov_len;
      ++iov;
      --n;
    }
    if (n > 0) {
      iov->iov_base = static_cast<char*>(iov->iov_base) + left;
      iov->iov_len -= left;
    }
  }
}

void recv_full(int fd, uint8_t* p, size_t n, int timeout_ms) {
  while (n) {
    const ssize_t r = ::recv(fd, p, n, 0);
    if (r > 0) {
      p += r;
      n -= (size_t)r;
      continue;
    }
    if (r == 0) throw StoreError(kErrIo, "hdfs data transfer: connection closed mid-packet");
    if (errno == EINTR) continue;
    if (errno == EAGAIN || errno == EWOULDBLOCK) {
      wait_fd(fd, POLLIN, timeout_ms, "receive");
      continue;
    }
    throw StoreError(kErrIo, "hdfs data transfer: connection lost while receiving packets");
  }
}

inline void put_le(uint8_t* p, uint64_t v, int n) {
  for (int i = 0; i < n; ++i) p[i] = (uint8_t)(v >> (8 * i));
}

// PacketHeaderProto as protobuf serializes it (every required field present).
size_t packet_header(uint8_t* h, uint64_t offset, uint64_t seqno, bool last, uint32_t data_len) {
  h[0] = 0x09;                      // offsetInBlock: field 1, fixed64
  put_le(h + 1, offset, 8);
  h[9] = 0x11;                      // seqno: field 2, fixed64
  put_le(h + 10, seqno, 8);
  h[18] = 0x18;                     // lastPacketInBlock: field 3, varint
  h[19] = last ? 1 : 0;
  h[20] = 0x25;                     // dataLen: field 4, fixed32
  put_le(h + 21, data_len, 4);
  return 25;
}

// PacketHeaderProto fields (any encoding order): offsetInBlock=1 seqno=2 lastPacketInBlock=3 dataLen=4
bool parse_packet_header(const uint8_t* hdr, size_t hlen, int64_t* offset, int64_t* seqno, bool* last,
                         int64_t* data_len) {
  *offset = 0;
  *seqno = 0;
  *last = false;
  *data_len = -1;
  size_t i = 0;
  while (i < hlen) {
    const uint8_t key = hdr[i++];
    const int field = key >> 3, wt = key & 7;
    uint64_t v = 0;
    if (wt == 1) {
      if (i + 8 > hlen) return false;
      for (int k = 7; k >= 0; --k) v = (v << 8) | hdr[i + k];
      i += 8;
    } else if (wt == 5) {
      if (i + 4 > hlen) return false;
      for (int k = 3; k >= 0; --k) v = (v << 8) | hdr[i + k];
      i += 4;
    } else if (wt == 0) {
      int shift = 0;
      while (i < hlen) {
        const uint8_t b = hdr[i++];
        v |= (uint64_t)(b & 0x7F) << shift;
        if (b < 0x80) break;
        shift += 7;
      }
    } else {
      return false;
    }
    if (field == 1) *offset = (int64_t)v;
    else if (field == 2) *seqno = (int64_t)v;
    else if (field == 3) *last = v != 0;
    else if (field == 4) *data_len = (int64_t)(int32_t)(uint32_t)v;
  }
  return true;
}

void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back((char)((v & 0x7F) | 0x80));
    v >>= 7;
  }
  s.push_back((char)v);
}

bool get_varint(const uint8_t* p, size_t n, size_t* i, uint64_t* v) {
  *v = 0;
  for (int shift = 0; *i < n && shift < 64; shift += 7) {
    const uint8_t b = p[(*i)++];
    *v |= (uint64_t)(b & 0x7F) << shift;
    if (b < 0x80) return true;
  }
  return false;
}

void put_be32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
}

}  // namespace

namespace {

// One packet's worth of staged data: filled (source read + CRC32C) by the producer thread, sent by
// the caller's thread.
struct Slot {
  uint8_t* buf = nullptr;
  bool pinned = false;
  std::vector<uint8_t> sums;
  uint64_t pos = 0, n = 0;
  bool full = false;
};

}  // namespace

uint64_t dn_send_block(int fd, BlockSource& src, uint64_t offset, uint64_t length, const DnSendOptions& o) {
  const uint32_t bpc = o.bytes_per_checksum ? o.bytes_per_checksum : 512;
  // whole chunks per packet
  const uint64_t per_packet = std::max<uint64_t>(bpc, (o.packet_bytes / bpc) * bpc);
  const uint64_t end = offset + length;
  const uint64_t npackets = (length + per_packet - 1) / per_packet;
  // Blocks of several packets run as a 2-stage pipeline over kSlots buffers: a producer thread
  // reads the source (HBM: D2H DMA) and checksums packet i+1.. while this thread's writev pushes
  // packet i -- the DataNode's BlockSender does the three serially.
  constexpr int kSlots = 3;
  const int nslots = npackets > 1 ? kSlots : 1;
  Slot slots[kSlots];
  struct Release {
    Slot* s;
    int n;
    uint64_t bytes;
    ~Release() {
      for (int i = 0; i < n; ++i)
        if (s[i].buf) host_buffer_release(s[i].buf, bytes, s[i].pinned);
    }
  } release{slots, nslots, per_packet};
  for (int i = 0; i < nslots; ++i) {
    slots[i].buf = host_buffer_alloc(per_packet, &slots[i].pinned);
    slots[i].sums.resize((size_t)((per_packet + bpc - 1) / bpc) * 4);
  }
  auto fill = [&](Slot& sl, uint64_t pos) {
    sl.pos = pos;
    sl.n = std::min(per_packet, end - pos);
    src.read(pos, sl.n, sl.buf);
    crc32c_chunks_be(sl.buf, (size_t)sl.n, bpc, sl.sums.data());
    if (o.fault_flip_bits) sl.buf[0] ^= 1;     // corrupt AFTER checksumming (test hook)
  };
  std::mutex mu;
  std::condition_variable cv;
  bool stop = false;
  std::exception_ptr perr;
  uint64_t produced = 0;                         // packets filled so far
  std::thread producer;
  const uint64_t to_send = o.fault_truncate ? std::min<uint64_t>(npackets, 1) : npackets;
  if (nslots > 1) {
    producer = std::thread([&] {
      try {
        for (uint64_t i = 0; i < to_send; ++i) {
          Slot& sl = slots[i % nslots];
          {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return stop || !sl.full; });
            if (stop) return;
          }
          fill(sl, offset + i * per_packet);
          std::lock_guard<std::mutex> lk(mu);
          sl.full = true;
          produced = i + 1;
          cv.notify_all();
        }
      } catch (...) {
        std::lock_guard<std::mutex> lk(mu);
        perr = std::current_exception();
        cv.notify_all();
      }
    });
  }
  struct Join {
    std::thread& t;
    std::mutex& mu;
    std::condition_variable& cv;
    bool& stop;
    ~Join() {
      if (!t.joinable()) return;
      {
        std::lock_guard<std::mutex> lk(mu);
        stop = true;
      }
      cv.notify_all();
      t.join();
    }
  } join{producer, mu, cv, stop};
  uint8_t pre[6 + 32];
  uint64_t sent = 0, seq = 0, pos = offset;
  for (uint64_t i = 0; i < to_send; ++i) {
    Slot& sl = slots[i % nslots];
    if (nslots > 1) {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return perr || produced > i; });
      if (produced <= i) std::rethrow_exception(perr);
    } else {
      fill(sl, offset + i * per_packet);
    }
    const size_t ns = (size_t)((sl.n + bpc - 1) / bpc) * 4;
    const size_t hl = packet_header(pre + 6, sl.pos, seq, false, (uint32_t)sl.n);
    put_be32(pre, (uint32_t)(4 + ns + sl.n));
    pre[4] = (uint8_t)(hl >> 8);
    pre[5] = (uint8_t)hl;
    iovec iov[3] = {{pre, 6 + hl}, {sl.sums.data(), ns}, {sl.buf, (size_t)sl.n}};
    send_iov(fd, iov, 3, o.timeout_ms);
    pos = sl.pos + sl.n;
    sent += sl.n;
    ++seq;
    if (nslots > 1) {
      std::lock_guard<std::mutex> lk(mu);
      sl.full = false;
      cv.notify_all();
    }
  }
  const size_t hl = packet_header(pre + 6, pos, seq, true, 0);
  put_be32(pre, 4);
  pre[4] = (uint8_t)(hl >> 8);
  pre[5] = (uint8_t)hl;
  iovec last[1] = {{pre, 6 + hl}};
  send_iov(fd, last, 1, o.timeout_ms);
  return sent;
}

// ---- receive -----------------------------------------------------------------------------------
DnPacketReader::DnPacketReader(int fd, uint32_t bpc, bool verify, uint64_t skip, int timeout_ms)
    : fd_(fd), bpc_(bpc ? bpc : 512), verify_(verify), skip_(skip), timeout_ms_(timeout_ms) {}

bool DnPacketReader::next_packet() {
  uint8_t pre[6];
  recv_full(fd_, pre, 6, timeout_ms_);
  const uint32_t plen = ((uint32_t)pre[0] << 24) | ((uint32_t)pre[1] << 16) | ((uint32_t)pre[2] << 8) | pre[3];
  const uint16_t hlen = (uint16_t)((pre[4] << 8) | pre[5]);
  if (plen < 4 || plen > (64u << 20) || hlen > 1024)
    throw StoreError(kErrIo, "hdfs data transfer: malformed packet lengths");
  uint8_t hdr[1024];
  recv_full(fd_, hdr, hlen, timeout_ms_);
  // PacketHeaderProto: offsetInBlock=1 seqno=2 lastPacketInBlock=3 dataLen=4 (any encoding order)
  int64_t offset_in_block = 0;
  bool last = false;
  int64_t data_len = -1;
  size_t i = 0;
  while (i < hlen) {
    const uint8_t key = hdr[i++];
    const int field = key >> 3, wt = key & 7;
    uint64_t v = 0;
    if (wt == 1) {
      if (i + 8 > hlen) break;
      for (int k = 7; k >= 0; --k) v = (v << 8) | hdr[i + k];
      i += 8;
    } else if (wt == 5) {
      if (i + 4 > hlen) break;
      for (int k = 3; k >= 0; --k) v = (v << 8) | hdr[i + k];
      i += 4;
    } else if (wt == 0) {
      int shift = 0;
      while (i < hlen) {
        const uint8_t b = hdr[i++];
        v |= (uint64_t)(b & 0x7F) << shift;
        if (b < 0x80) break;
        shift += 7;
      }
    } else {
      throw StoreError(kErrIo, "hdfs data transfer: unexpected packet header encoding");
    }
    if (field == 1) offset_in_block = (int64_t)v;
    else if (field == 3) last = v != 0;
    else if (field == 4) data_len = (int64_t)(int32_t)(uint32_t)v;
  }
  if (data_len < 0 || (uint64_t)data_len > plen - 4)
    throw StoreError(kErrIo, "hdfs data transfer: packet without a valid dataLen");
  const size_t nsums = plen - 4 - (size_t)data_len;
  sums_.resize(nsums);
  recv_full(fd_, sums_.data(), nsums, timeout_ms_);
  // the whole packet fits the caller's request: receive and verify it in place (no bounce)
  uint8_t* into = nullptr;
  if (direct_dst_ && !skip_ && (uint64_t)data_len <= direct_room_) {
    into = direct_dst_;
    pend_.clear();
  } else {
    pend_.resize((size_t)data_len);
    into = pend_.data();
  }
  pend_off_ = 0;
  recv_full(fd_, into, (size_t)data_len, timeout_ms_);
  ++packets_;
  if (verify_ && data_len && nsums) {
    const size_t chunks = ((size_t)data_len + bpc_ - 1) / bpc_;
    if (nsums < chunks * 4) throw StoreError(kErrIo, "hdfs data transfer: packet checksums missing");
    const int64_t bad = crc32c_chunks_verify(into, (size_t)data_len, bpc_, sums_.data());
    if (bad >= 0)
      throw StoreError(kErrIo, "checksum error in hdfs packet at block offset " +
                                   std::to_string(offset_in_block + bad * (int64_t)bpc_));
  }
  direct_got_ = into == direct_dst_ ? (uint64_t)data_len : 0;
  if (skip_) {
    const size_t k = (size_t)std::min<uint64_t>(skip_, pend_.size());
    pend_off_ = k;
    skip_ -= k;
  }
  if (last || data_len == 0) done_ = true;
  return !done_;
}

uint64_t DnPacketReader::readinto(uint8_t* dst, uint64_t n) {
  uint64_t got = 0;
  while (got < n) {
    if (pend_off_ == pend_.size()) {
      if (done_) break;
      direct_dst_ = dst + got;
      direct_room_ = n - got;
      next_packet();
      direct_dst_ = nullptr;
      got += direct_got_;
      direct_got_ = 0;
      continue;
    }
    const size_t k = (size_t)std::min<uint64_t>(n - got, pend_.size() - pend_off_);
    std::memcpy(dst + got, pend_.data() + pend_off_, k);
    pend_off_ += k;
    got += k;
  }
  return got;
}

void DnPacketReader::drain() {
  direct_dst_ = nullptr;
  pend_off_ = pend_.size();
  while (!done_) {
    const bool v = verify_;
    verify_ = false;
    next_packet();
    verify_ = v;
    pend_off_ = pend_.size();
  }
}

}  // namespace amdx

namespace amdx {

// ---- WRITE_BLOCK: client packets ---------------------------------------------------------------
DnPacketWriter::DnPacketWriter(int fd, uint32_t bpc, uint32_t packet_bytes, uint32_t max_in_flight, int timeout_ms)
    : fd_(fd), bpc_(bpc ? bpc : 512), max_in_flight_(max_in_flight ? max_in_flight : 80), timeout_ms_(timeout_ms) {
  packet_ = std::max<uint32_t>(bpc_, (packet_bytes ? packet_bytes : (64u << 10)) / bpc_ * bpc_);
  sums_.resize((size_t)(packet_ / bpc_ + 1) * 4);
}

void DnPacketWriter::send_packet(const uint8_t* data, uint32_t n, bool last) {
  const size_t ns = n ? (size_t)((n + bpc_ - 1) / bpc_) * 4 : 0;
  if (n) crc32c_chunks_be(data, n, bpc_, sums_.data());
  uint8_t pre[6 + 32];
  const size_t hl = packet_header(pre + 6, off_, seq_, last, n);
  put_be32(pre, (uint32_t)(4 + ns + n));
  pre[4] = (uint8_t)(hl >> 8);
  pre[5] = (uint8_t)hl;
  iovec iov[3] = {{pre, 6 + hl}, {sums_.data(), ns}, {const_cast<uint8_t*>(data), n}};
  send_iov(fd_, iov, n ? 3 : 1, timeout_ms_);
  off_ += n;
  ++seq_;
  ++inflight_;
}

// PipelineAckProto: seqno=1 (sint64), reply=2 (repeated Status, packed or not), others skipped.
void DnPacketWriter::read_acks() {
  for (;;) {
    // parse whole delimited messages already buffered
    size_t i = 0;
    for (;;) {
      size_t j = i;
      uint64_t len;
      if (!get_varint(reinterpret_cast<const uint8_t*>(rbuf_.data()), rbuf_.size(), &j, &len)) break;
      if (rbuf_.size() - j < len) break;
      const uint8_t* m = reinterpret_cast<const uint8_t*>(rbuf_.data()) + j;
      size_t k = 0;
      int bad = -1;
      while (k < len) {
        uint64_t key;
        if (!get_varint(m, len, &k, &key)) throw StoreError(kErrIo, "hdfs pipeline: malformed ack");
        const uint32_t field = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
        if (wt == 0) {
          uint64_t v;
          if (!get_varint(m, len, &k, &v)) throw StoreError(kErrIo, "hdfs pipeline: malformed ack");
          if (field == 2 && v != 0 && bad < 0) bad = (int)v;
        } else if (wt == 2) {
          uint64_t l;
          if (!get_varint(m, len, &k, &l) || l > len - k) throw StoreError(kErrIo, "hdfs pipeline: malformed ack");
          if (field == 2) {                         // packed replies
            size_t q = k;
            while (q < k + l) {
              uint64_t v;
              if (!get_varint(m, k + l, &q, &v)) break;
              if (v != 0 && bad < 0) bad = (int)v;
            }
          }
          k += (size_t)l;
        } else if (wt == 1) {
          k += 8;
        } else if (wt == 5) {
          k += 4;
        } else {
          throw StoreError(kErrIo, "hdfs pipeline: malformed ack");
        }
      }
      if (bad >= 0)
        throw StoreError(bad == 2 ? kErrInvalidState : kErrIo,
                         "hdfs pipeline ack error status " + std::to_string(bad) + " at block offset " +
                             std::to_string(off_));
      if (inflight_) --inflight_;
      i = j + (size_t)len;
    }
    if (i) rbuf_.erase(0, i);
    if (!inflight_) return;        // nothing outstanding (the DataNode may close after its last ack)
    // then drain what is already in the socket, without waiting
    char tmp[4096];
    const ssize_t r = ::recv(fd_, tmp, sizeof(tmp), MSG_DONTWAIT);
    if (r > 0) {
      rbuf_.append(tmp, (size_t)r);
      continue;
    }
    if (r == 0) throw StoreError(kErrIo, "hdfs pipeline: datanode closed the connection");
    return;
  }
}

void DnPacketWriter::write(const uint8_t* p, uint64_t n) {
  uint64_t i = 0;
  // complete a held tail first
  if (!tail_.empty()) {
    const uint64_t take = std::min<uint64_t>(n, packet_ - tail_.size());
    tail_.insert(tail_.end(), p, p + take);
    i += take;
    if (tail_.size() == packet_) {
      send_packet(tail_.data(), packet_, false);
      tail_.clear();
    }
  }
  while (n - i >= packet_) {
    send_packet(p + i, packet_, false);
    i += packet_;
    read_acks();
    while (inflight_ >= max_in_flight_) {
      wait_fd(fd_, POLLIN, timeout_ms_, "pipeline ack");
      char tmp[4096];
      const ssize_t r = ::recv(fd_, tmp, sizeof(tmp), 0);
      if (r == 0) throw StoreError(kErrIo, "hdfs pipeline: datanode closed the connection");
      if (r > 0) rbuf_.append(tmp, (size_t)r);
      read_acks();
    }
  }
  if (i < n) tail_.insert(tail_.end(), p + i, p + n);
}

uint64_t DnPacketWriter::finish() {
  if (!tail_.empty()) {
    send_packet(tail_.data(), (uint32_t)tail_.size(), false);
    tail_.clear();
  }
  send_packet(nullptr, 0, true);
  while (inflight_) {
    read_acks();
    if (!inflight_) break;
    wait_fd(fd_, POLLIN, timeout_ms_, "pipeline ack");
    char tmp[4096];
    const ssize_t r = ::recv(fd_, tmp, sizeof(tmp), 0);
    if (r == 0) throw StoreError(kErrIo, "hdfs pipeline: datanode closed the connection before the last ack");
    if (r > 0) rbuf_.append(tmp, (size_t)r);
  }
  return off_;
}

// ---- WRITE_BLOCK: DataNode side --------------------------------------------------------------------
DnPacketReceiver::DnPacketReceiver(int fd, uint32_t bpc, int timeout_ms)
    : fd_(fd), bpc_(bpc ? bpc : 512), timeout_ms_(timeout_ms) {}

uint64_t DnPacketReceiver::receive(uint8_t* dst, uint64_t cap, uint64_t batch, bool* last, int* status) {
  constexpr uint64_t kMaxPacket = 16u << 20;
  pending_.clear();
  *last = false;
  *status = 0;
  uint64_t got = 0;
  while (!*last && *status == 0 && got < batch && cap - got >= kMaxPacket) {
    // batch only what is already arriving: a sender that waits for each ack (a relaying
    // DataNode, a stop-and-wait client) gets it as soon as its packet is stored
    if (!pending_.empty()) {
      pollfd pf{fd_, POLLIN, 0};
      if (::poll(&pf, 1, 0) <= 0) break;
    }
    uint8_t pre[6];
    recv_full(fd_, pre, 6, timeout_ms_);
    const uint32_t plen = ((uint32_t)pre[0] << 24) | ((uint32_t)pre[1] << 16) | ((uint32_t)pre[2] << 8) | pre[3];
    const uint16_t hlen = (uint16_t)((pre[4] << 8) | pre[5]);
    if (plen < 4 || plen > kMaxPacket + (kMaxPacket / 512 + 1) * 4 + 4 || hlen > 1024) {
      *status = 1;
      break;
    }
    uint8_t hdr[1024];
    recv_full(fd_, hdr, hlen, timeout_ms_);
    int64_t offset, seqno, data_len;
    bool lastp;
    if (!parse_packet_header(hdr, hlen, &offset, &seqno, &lastp, &data_len) || data_len < 0 ||
        (uint64_t)data_len > plen - 4 || (uint64_t)data_len > kMaxPacket) {
      *status = 1;
      break;
    }
    const size_t nsums = plen - 4 - (size_t)data_len;
    sums_.resize(nsums);
    recv_full(fd_, sums_.data(), nsums, timeout_ms_);
    recv_full(fd_, dst + got, (size_t)data_len, timeout_ms_);
    pending_.push_back(seqno);
    if (data_len) {
      if ((uint64_t)offset != received_) {
        *status = 1;
      } else {
        const size_t chunks = ((size_t)data_len + bpc_ - 1) / bpc_;
        if (nsums < chunks * 4 || crc32c_chunks_verify(dst + got, (size_t)data_len, bpc_, sums_.data()) >= 0) {
          *status = 2;
        } else {
          got += (uint64_t)data_len;
          received_ += (uint64_t)data_len;
        }
      }
    }
    if (lastp) *last = true;
  }
  return got;
}

void DnPacketReceiver::ack(int status) {
  if (pending_.empty()) return;
  std::string out;
  for (int64_t seq : pending_) {
    std::string m;
    m.push_back((char)(1 << 3));                  // seqno: sint64 (zigzag)
    put_varint(m, ((uint64_t)seq << 1) ^ (uint64_t)(seq >> 63));
    m.push_back((char)(2 << 3));                  // reply: Status
    put_varint(m, (uint64_t)status);
    put_varint(out, m.size());
    out += m;
  }
  pending_.clear();
  iovec iov[1] = {{&out[0], out.size()}};
  send_iov(fd_, iov, 1, timeout_ms_);
}

}  // namespace amdx
