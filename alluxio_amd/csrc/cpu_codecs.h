// Host reference implementations of the block codecs: CRC32C (slicing-by-8) and LZ4 block
// format (greedy hash-chain-free encoder + safe decoder).  They are (a) the codec used for host
// tiers and (b) the numerics oracle the HIP kernels are tested against.
#pragma once
#include <cstddef>
#include <cstdint>

namespace amdx {

uint32_t crc32c_sw(const void* data, size_t n, uint32_t crc = 0);  // standard (init/xorout ~0)
uint32_t crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);
// One CRC32C per `bpc`-byte chunk of data[0, n) (the last chunk may be short), stored big endian
// at out[4*i] -- the HDFS packet checksum layout.  Four chunks run interleaved on x86 (four
// independent CRC32 dependency chains), ~4x the throughput of chaining one.
void crc32c_chunks_be(const uint8_t* data, size_t n, uint32_t bpc, uint8_t* out);
// Same, comparing against `expect` (big endian); returns the first mismatching chunk or -1.
int64_t crc32c_chunks_verify(const uint8_t* data, size_t n, uint32_t bpc, const uint8_t* expect);

// Returns compressed size, or -1 if dst_cap is too small.
int64_t lz4_compress_block(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap);
// Returns decompressed size, or a negative error code on malformed input / overflow.
int64_t lz4_decompress_block(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap);
size_t lz4_compress_bound(size_t n);

}  // namespace amdx
