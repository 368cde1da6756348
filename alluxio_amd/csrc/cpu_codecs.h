// Host reference implementations of the block codecs: CRC32C (slicing-by-8) and LZ4 block
// format (greedy hash-chain-free encoder + safe decoder).  They are (a) the codec used for host
// tiers and (b) the numerics oracle the HIP kernels are tested against.
#pragma once
#include <cstddef>
#include <cstdint>

namespace amdx {

uint32_t crc32c_sw(const void* data, size_t n, uint32_t crc = 0);  // standard (init/xorout ~0)
uint32_t crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

// Returns compressed size, or -1 if dst_cap is too small.
int64_t lz4_compress_block(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap);
// Returns decompressed size, or a negative error code on malformed input / overflow.
int64_t lz4_decompress_block(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap);
size_t lz4_compress_bound(size_t n);

}  // namespace amdx
