// Batch protobuf encoders for bulk metadata (see meta_codec.cpp).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace amdx {

// Body of a batched JournalEntry (repeated `journal_entries` = 39) holding one inode_file entry
// per file: `tmpl` = serialized InodeFileEntry constant fields; blocks are derived from the file
// id's container and the length.
std::string encode_inode_file_batch(const std::string& tmpl, const std::vector<int64_t>& ids,
                                    const std::vector<int64_t>& parent_ids, const std::vector<std::string>& names,
                                    const std::vector<int64_t>& lengths, int64_t block_size,
                                    const std::vector<std::string>& fingerprints, const std::vector<int64_t>& mtimes,
                                    int64_t ctime);
// Body of a batched JournalEntry holding one block_info entry per block.
std::string encode_block_info_batch(const std::vector<int64_t>& block_ids, const std::vector<int64_t>& lengths);
// FileInfo messages of the files of one directory: `tmpl` = serialized constant fields,
// `block_infos` = serialized BlockInfo of every block of every file, in order ("" = not cached:
// encoded here from the id and length, with the file's ufsPath as ufsStringLocations when
// `ufs_locations`, i.e. the files are persisted).  out_field != 0
// wraps each FileInfo as that field (1 = ListStatusPResponse.fileInfos); 0 = varint-delimited.
std::string encode_file_infos(const std::string& tmpl, const std::vector<int64_t>& ids,
                              const std::vector<std::string>& names, const std::string& parent_path,
                              const std::string& parent_ufs, const std::vector<int64_t>& lengths, int64_t block_size,
                              const std::vector<int64_t>& ctimes, const std::vector<int64_t>& mtimes,
                              const std::vector<int64_t>& atimes, const std::vector<std::string>& fingerprints,
                              const std::vector<std::string>& block_infos, const std::vector<int32_t>& in_alluxio,
                              const std::vector<int32_t>& in_memory, uint32_t out_field, bool ufs_locations);

// Columns of the FileInfos in serialized ListStatusPResponse chunks (fileInfos = field 1): the
// fields a dataset index needs plus each FileInfo's (chunk, offset, size) span for lazy parsing.
struct FileInfoColumns {
  std::vector<int64_t> ids, lengths, block_sizes, first_blocks, nblocks, offset, size, mtimes, atimes;
  std::vector<int32_t> modes;
  std::vector<uint8_t> folder, completed;
  std::vector<int32_t> chunk;
  std::vector<std::string> paths;
};
void decode_file_infos(const std::vector<std::string>& chunks, FileInfoColumns& out);

}  // namespace amdx
