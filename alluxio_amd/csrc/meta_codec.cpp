// Batch protobuf encoders for the master's bulk metadata paths (config 4: 1 M files).
//
// The per-file Python cost of building a JournalEntry (InodeFileEntry + BlockInfoEntry) and a
// FileInfo reply dominates a large metadata load / listing.  These encoders take a TEMPLATE
// (the serialized constant fields, produced once by the Python protobuf runtime) plus columns of
// the per-file fields and emit the wire bytes directly.  Protobuf parsing is order-independent
// and last-one-wins for singular fields, so template + appended varying fields is the same
// message the Python runtime would build.  Reference messages: proto/journal/file.proto
// (InodeFileEntry), proto/journal/block.proto (BlockInfoEntry), proto/journal/journal.proto
// (JournalEntry, batched in `journal_entries` = 39), grpc/file_system_master.proto (FileInfo).
#include "meta_codec.h"

#include <cstring>
#include <stdexcept>

namespace amdx {
namespace {

inline void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back((char)(v | 0x80));
    v >>= 7;
  }
  o.push_back((char)v);
}
inline void put_tag(std::string& o, uint32_t field, uint32_t wire) { put_varint(o, ((uint64_t)field << 3) | wire); }
inline void put_i64(std::string& o, uint32_t field, int64_t v) {
  put_tag(o, field, 0);
  put_varint(o, (uint64_t)v);
}
inline void put_bytes(std::string& o, uint32_t field, const char* p, size_t n) {
  put_tag(o, field, 2);
  put_varint(o, n);
  o.append(p, n);
}
inline void put_str(std::string& o, uint32_t field, const std::string& s) { put_bytes(o, field, s.data(), s.size()); }
inline size_t varint_len(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++n;
  }
  return n;
}
// wrap `body` as field `field` (length-delimited) of the enclosing message
inline void put_msg(std::string& o, uint32_t field, const std::string& body) { put_bytes(o, field, body.data(), body.size()); }

constexpr int64_t kMaxSeq = (1ll << 24) - 1;   // BlockId.java: 24-bit sequence numbers

}  // namespace

std::string encode_inode_file_batch(const std::string& tmpl, const std::vector<int64_t>& ids,
                                    const std::vector<int64_t>& parent_ids, const std::vector<std::string>& names,
                                    const std::vector<int64_t>& lengths, int64_t block_size,
                                    const std::vector<std::string>& fingerprints, const std::vector<int64_t>& mtimes,
                                    int64_t ctime) {
  const size_t n = ids.size();
  if (parent_ids.size() != n || names.size() != n || lengths.size() != n || fingerprints.size() != n ||
      mtimes.size() != n)
    throw std::invalid_argument("encode_inode_file_batch: column lengths differ");
  if (block_size <= 0) throw std::invalid_argument("encode_inode_file_batch: block size must be positive");
  std::string out, entry, inode;
  out.reserve(n * (tmpl.size() + 96));
  for (size_t i = 0; i < n; ++i) {
    inode.assign(tmpl);
    put_i64(inode, 1, ids[i]);                   // id
    put_i64(inode, 2, parent_ids[i]);            // parent_id
    put_str(inode, 3, names[i]);                 // name
    put_i64(inode, 6, ctime);                    // creation_time_ms
    put_i64(inode, 7, mtimes[i]);                // last_modification_time_ms
    put_i64(inode, 9, lengths[i]);               // length
    // blocks: container id of the file || sequence 0..k-1 (unpacked proto2 repeated int64)
    const int64_t container = ids[i] >> 24;
    const int64_t nb = (lengths[i] + block_size - 1) / block_size;
    if (nb > kMaxSeq) throw std::invalid_argument("encode_inode_file_batch: too many blocks in a file");
    for (int64_t s = 0; s < nb; ++s) put_i64(inode, 12, (container << 24) | s);
    put_str(inode, 18, fingerprints[i]);         // ufs_fingerprint
    put_i64(inode, 29, mtimes[i]);               // last_access_time_ms
    entry.clear();
    put_msg(entry, 11, inode);                   // JournalEntry.inode_file
    put_msg(out, 39, entry);                     // batch: JournalEntry.journal_entries
  }
  return out;
}

std::string encode_block_info_batch(const std::vector<int64_t>& block_ids, const std::vector<int64_t>& lengths) {
  const size_t n = block_ids.size();
  if (lengths.size() != n) throw std::invalid_argument("encode_block_info_batch: column lengths differ");
  std::string out, bi, entry;
  out.reserve(n * 24);
  for (size_t i = 0; i < n; ++i) {
    bi.clear();
    put_i64(bi, 1, block_ids[i]);
    put_i64(bi, 2, lengths[i]);
    entry.clear();
    put_msg(entry, 4, bi);                       // JournalEntry.block_info
    put_msg(out, 39, entry);
  }
  return out;
}

std::string encode_file_infos(const std::string& tmpl, const std::vector<int64_t>& ids,
                              const std::vector<std::string>& names, const std::string& parent_path,
                              const std::string& parent_ufs, const std::vector<int64_t>& lengths, int64_t block_size,
                              const std::vector<int64_t>& ctimes, const std::vector<int64_t>& mtimes,
                              const std::vector<int64_t>& atimes, const std::vector<std::string>& fingerprints,
                              const std::vector<std::string>& block_infos, const std::vector<int32_t>& in_alluxio,
                              const std::vector<int32_t>& in_memory, uint32_t out_field, bool ufs_locations) {
  const size_t n = ids.size();
  if (names.size() != n || lengths.size() != n || ctimes.size() != n || mtimes.size() != n || atimes.size() != n ||
      fingerprints.size() != n || in_alluxio.size() != n || in_memory.size() != n)
    throw std::invalid_argument("encode_file_infos: column lengths differ");
  std::string out, fi, fbi, tmp;
  out.reserve(n * (tmpl.size() + 160));
  size_t bpos = 0;                               // block_infos: one serialized BlockInfo per block, in order
  const std::string pp = parent_path.size() > 1 ? parent_path : std::string();
  const std::string pu = parent_ufs;
  for (size_t i = 0; i < n; ++i) {
    fi.assign(tmpl);
    put_i64(fi, 1, ids[i]);                      // fileId
    put_str(fi, 2, names[i]);                    // name
    tmp.assign(pp);
    tmp.push_back('/');
    tmp.append(names[i]);
    put_str(fi, 3, tmp);                         // path
    if (!pu.empty()) {
      tmp.assign(pu);
      if (tmp.back() != '/') tmp.push_back('/');
      tmp.append(names[i]);
      put_str(fi, 4, tmp);                       // ufsPath
    }
    put_i64(fi, 5, lengths[i]);                  // length
    put_i64(fi, 7, ctimes[i]);                   // creationTimeMs
    const int64_t container = ids[i] >> 24;
    const int64_t nb = block_size > 0 ? (lengths[i] + block_size - 1) / block_size : 0;
    for (int64_t s = 0; s < nb; ++s) put_i64(fi, 13, (container << 24) | s);   // blockIds
    put_i64(fi, 14, mtimes[i]);                  // lastModificationTimeMs
    for (int64_t s = 0; s < nb; ++s) {           // fileBlockInfos
      if (bpos >= block_infos.size()) throw std::invalid_argument("encode_file_infos: too few block infos");
      const std::string& b = block_infos[bpos++];
      fbi.clear();
      if (b.empty()) {                           // not cached: BlockInfo{blockId, length}
        tmp.clear();
        put_i64(tmp, 1, (container << 24) | s);
        const int64_t rem = lengths[i] - s * block_size;
        put_i64(tmp, 2, rem < block_size ? rem : block_size);
        put_msg(fbi, 1, tmp);
      } else {
        put_bytes(fbi, 1, b.data(), b.size());   // blockInfo (with locations)
      }
      put_i64(fbi, 2, s * block_size);           // offset
      if (b.empty() && ufs_locations && !pu.empty()) {   // ufsStringLocations of a persisted file
        tmp.assign(pu);
        if (tmp.back() != '/') tmp.push_back('/');
        tmp.append(names[i]);
        put_str(fbi, 4, tmp);
      }
      put_msg(fi, 21, fbi);
    }
    put_i64(fi, 24, in_alluxio[i]);              // inAlluxioPercentage
    put_i64(fi, 25, in_memory[i]);               // inMemoryPercentage
    put_str(fi, 26, fingerprints[i]);            // ufsFingerprint
    put_i64(fi, 31, atimes[i]);                  // lastAccessTimeMs
    if (out_field) put_msg(out, out_field, fi);
    else {
      put_varint(out, fi.size());
      out.append(fi);
    }
  }
  if (bpos != block_infos.size()) throw std::invalid_argument("encode_file_infos: block info count mismatch");
  (void)varint_len;
  return out;
}

namespace {

bool get_varint(const uint8_t*& p, const uint8_t* end, uint64_t& v) {
  v = 0;
  for (int sh = 0; sh < 64 && p < end; sh += 7) {
    const uint8_t b = *p++;
    v |= (uint64_t)(b & 0x7F) << sh;
    if (!(b & 0x80)) return true;
  }
  return false;
}

bool skip_field(const uint8_t*& p, const uint8_t* end, uint32_t wire) {
  uint64_t v;
  switch (wire) {
    case 0: return get_varint(p, end, v);
    case 1: if (end - p < 8) return false; p += 8; return true;
    case 2: if (!get_varint(p, end, v) || (uint64_t)(end - p) < v) return false; p += v; return true;
    case 5: if (end - p < 4) return false; p += 4; return true;
    default: return false;
  }
}

}  // namespace

void decode_file_infos(const std::vector<std::string>& chunks, FileInfoColumns& out) {
  for (size_t c = 0; c < chunks.size(); ++c) {
    const uint8_t* p = (const uint8_t*)chunks[c].data();
    const uint8_t* end = p + chunks[c].size();
    while (p < end) {
      uint64_t key, len;
      if (!get_varint(p, end, key)) throw std::invalid_argument("decode_file_infos: bad tag");
      if ((key >> 3) != 1 || (key & 7) != 2) {
        if (!skip_field(p, end, (uint32_t)(key & 7))) throw std::invalid_argument("decode_file_infos: bad field");
        continue;
      }
      if (!get_varint(p, end, len) || (uint64_t)(end - p) < len) throw std::invalid_argument("decode_file_infos: bad length");
      const uint8_t* q = p;
      const uint8_t* fe = p + len;
      int64_t id = 0, length = 0, bsz = 0, first = -1, nblk = 0, mtime = 0, atime = 0;
      int32_t mode = 0;
      bool folder = false, completed = false;
      std::string path;
      while (q < fe) {
        uint64_t k, v;
        if (!get_varint(q, fe, k)) throw std::invalid_argument("decode_file_infos: bad FileInfo");
        const uint32_t f = (uint32_t)(k >> 3), w = (uint32_t)(k & 7);
        if (w == 0 && (f == 1 || f == 5 || f == 6 || f == 8 || f == 9 || f == 13 || f == 14 || f == 18 || f == 31)) {
          if (!get_varint(q, fe, v)) throw std::invalid_argument("decode_file_infos: bad varint");
          if (f == 1) id = (int64_t)v;
          else if (f == 5) length = (int64_t)v;
          else if (f == 6) bsz = (int64_t)v;
          else if (f == 8) completed = v != 0;
          else if (f == 9) folder = v != 0;
          else if (f == 14) mtime = (int64_t)v;
          else if (f == 18) mode = (int32_t)v;
          else if (f == 31) atime = (int64_t)v;
          else {
            if (nblk == 0) first = (int64_t)v;
            ++nblk;
          }
        } else if (w == 2 && f == 13) {            // packed blockIds
          if (!get_varint(q, fe, v) || (uint64_t)(fe - q) < v) throw std::invalid_argument("decode_file_infos: bad packed");
          const uint8_t* pe = q + v;
          while (q < pe) {
            uint64_t b;
            if (!get_varint(q, pe, b)) throw std::invalid_argument("decode_file_infos: bad packed varint");
            if (nblk == 0) first = (int64_t)b;
            ++nblk;
          }
        } else if (w == 2 && f == 3) {
          if (!get_varint(q, fe, v) || (uint64_t)(fe - q) < v) throw std::invalid_argument("decode_file_infos: bad path");
          path.assign((const char*)q, v);
          q += v;
        } else if (!skip_field(q, fe, w)) {
          throw std::invalid_argument("decode_file_infos: bad FileInfo field");
        }
      }
      out.ids.push_back(id);
      out.lengths.push_back(length);
      out.block_sizes.push_back(bsz);
      out.first_blocks.push_back(first);
      out.nblocks.push_back(nblk);
      out.folder.push_back(folder ? 1 : 0);
      out.completed.push_back(completed ? 1 : 0);
      out.mtimes.push_back(mtime);
      out.atimes.push_back(atime);
      out.modes.push_back(mode);
      out.paths.push_back(std::move(path));
      out.chunk.push_back((int32_t)c);
      out.offset.push_back((int64_t)(p - (const uint8_t*)chunks[c].data()));
      out.size.push_back((int64_t)len);
      p = fe;
    }
  }
}

}  // namespace amdx
