// HDFS DataTransferProtocol packet I/O in native code: the DataNode side of READ_BLOCK for the
// HDFS-protocol gateway (proxy/hdfs_gateway.py) and the receive side of this repository's Hadoop
// client (underfs/hadoop_rpc.py BlockReader).
//
// Wire format (DataTransferProtocol v28, PacketReceiver / BlockSender): per packet
//   u32 PLEN (= 4 + checksum bytes + data bytes) | u16 HLEN | PacketHeaderProto | CRC32C per
//   bytes-per-checksum chunk (big endian) | data
// with PacketHeaderProto{offsetInBlock sfixed64=1, seqno sfixed64=2, lastPacketInBlock bool=3,
// dataLen sfixed32=4}; the block ends with an empty packet whose lastPacketInBlock is set.
//
// Reference: the Java DataNode's BlockSender.sendPacket and the client's PacketReceiver; here the
// gateway's bytes come from a native BlockSource (HBM chunks D2H into a pinned buffer, DRAM arenas
// copied in place), checksums are computed with the hardware CRC32C instruction, and each packet
// leaves with one writev -- no Python frame per packet on either end.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "block_source.h"

namespace amdx {

struct DnSendOptions {
  uint32_t bytes_per_checksum = 512;
  uint32_t packet_bytes = 1u << 20;   // data bytes per packet (the client accepts up to 16 MiB)
  int timeout_ms = 60000;
  bool fault_flip_bits = false;       // test hooks (the gateway's fault injection)
  bool fault_truncate = false;
};

// Sends block bytes [offset, offset + length) of `src` (offset chunk-aligned by the caller) on the
// connected socket `fd` as packets starting at seqno 0, then the final empty packet.  Returns the
// data bytes sent; throws on I/O errors.
uint64_t dn_send_block(int fd, BlockSource& src, uint64_t offset, uint64_t length, const DnSendOptions& o);

// Receives the packets of one READ_BLOCK response: copies data into caller buffers, verifying
// CRC32C per chunk.  `skip` leading bytes are dropped (the DataNode starts at a chunk boundary).
class DnPacketReader {
 public:
  DnPacketReader(int fd, uint32_t bytes_per_checksum, bool verify, uint64_t skip, int timeout_ms);
  // Copies up to n bytes; 0 once the block's last packet was consumed.
  uint64_t readinto(uint8_t* dst, uint64_t n);
  bool done() const { return done_ && pend_off_ == pend_.size(); }
  // Reads (and discards) packets up to the final one (before sending CHECKSUM_OK).
  void drain();
  uint64_t packets() const { return packets_; }

 private:
  bool next_packet();                 // false when the last packet arrived
  int fd_;
  uint32_t bpc_;
  bool verify_;
  uint64_t skip_;
  int timeout_ms_;
  bool done_ = false;
  std::vector<uint8_t> pend_;         // data of the current packet not yet handed out
  size_t pend_off_ = 0;
  std::vector<uint8_t> sums_;
  uint64_t packets_ = 0;
  uint8_t* direct_dst_ = nullptr;     // where next_packet() may land a packet that fits whole
  uint64_t direct_room_ = 0;
  uint64_t direct_got_ = 0;
};

// The client side of WRITE_BLOCK (DFSClient's DataStreamer + ResponseProcessor): the caller's
// bytes leave as chunk-aligned packets of `packet_bytes` (CRC32C per bytes-per-checksum chunk,
// one writev each; a short tail is held back until more data or finish()), at most `max_in_flight`
// packets un-acked; PipelineAckProto replies are parsed as they arrive and any non-SUCCESS reply
// fails the write.
class DnPacketWriter {
 public:
  DnPacketWriter(int fd, uint32_t bytes_per_checksum, uint32_t packet_bytes, uint32_t max_in_flight, int timeout_ms);
  void write(const uint8_t* p, uint64_t n);
  // Sends the held tail and the final empty packet, waits for every ack; returns the block length.
  uint64_t finish();
  uint64_t offset() const { return off_ + tail_.size(); }

 private:
  void send_packet(const uint8_t* data, uint32_t n, bool last);
  void read_acks();   // parses buffered acks, then drains the socket without waiting
  int fd_;
  uint32_t bpc_, packet_;
  uint32_t max_in_flight_;
  int timeout_ms_;
  uint64_t off_ = 0, seq_ = 0, inflight_ = 0;
  std::vector<uint8_t> sums_, tail_;
  std::string rbuf_;
};

// The DataNode side of WRITE_BLOCK for the gateway: packets received straight into the caller's
// buffer (CRC32C-verified, offsets checked) in batches; the caller stores the batch, then ack()
// answers every packet of it with one PipelineAckProto each (one writev).
class DnPacketReceiver {
 public:
  DnPacketReceiver(int fd, uint32_t bytes_per_checksum, int timeout_ms);
  // Packets into dst until >= batch data bytes, the last packet, an error, cap - got < 16 MiB, or
  // no further packet is already waiting on the socket.
  // status: 0 SUCCESS, 1 ERROR (bad offset / framing), 2 ERROR_CHECKSUM.
  uint64_t receive(uint8_t* dst, uint64_t cap, uint64_t batch, bool* last, int* status);
  void ack(int status);
  uint64_t received() const { return received_; }

 private:
  int fd_;
  uint32_t bpc_;
  int timeout_ms_;
  uint64_t received_ = 0;
  std::vector<int64_t> pending_;     // seqnos of the last receive()
  std::vector<uint8_t> sums_;
};

}  // namespace amdx
