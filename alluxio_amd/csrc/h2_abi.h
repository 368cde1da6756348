// The slice of libnghttp2's stable C ABI used by the gRPC (HTTP/2) server front end
// (frame_rpc.cpp) and the native gRPC block-read client (block_source.cpp).
//
// The image ships the runtime library (libnghttp2.so.14) without its headers, so the structs and
// entry points below are declared from the public ABI and resolved once with dlopen; without the
// library the gRPC paths report themselves unavailable.
#pragma once
#include <dlfcn.h>
#include <sys/types.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <string>
#include <type_traits>

namespace amdx {
namespace h2 {

struct Nv {
  uint8_t* name;
  uint8_t* value;
  size_t namelen;
  size_t valuelen;
  uint8_t flags;
};
struct FrameHd {   // the first member of every nghttp2_frame variant
  size_t length;
  int32_t stream_id;
  uint8_t type;
  uint8_t flags;
  uint8_t reserved;
};
struct DataFrame {   // nghttp2_data
  FrameHd hd;
  size_t padlen;     // includes the 1-byte Pad Length field when > 0
};
union DataSource {
  int fd;
  void* ptr;
};
typedef ssize_t (*ReadCb)(void* session, int32_t stream_id, uint8_t* buf, size_t length, uint32_t* data_flags,
                          DataSource* source, void* user_data);
struct DataProvider {
  DataSource source;
  ReadCb read_callback;
};
struct SettingsEntry {
  int32_t settings_id;
  uint32_t value;
};
typedef int (*FrameCb)(void* session, const void* frame, void* user_data);
typedef int (*DataChunkCb)(void* session, uint8_t flags, int32_t stream_id, const uint8_t* data, size_t len,
                           void* user_data);
typedef int (*CloseCb)(void* session, int32_t stream_id, uint32_t error_code, void* user_data);
typedef int (*HeaderCb)(void* session, const void* frame, const uint8_t* name, size_t namelen, const uint8_t* value,
                        size_t valuelen, uint8_t flags, void* user_data);
typedef int (*SendDataCb)(void* session, void* frame, const uint8_t* framehd, size_t length, DataSource* source,
                          void* user_data);
typedef ssize_t (*ReadLengthCb)(void* session, uint8_t frame_type, int32_t stream_id, int32_t session_remote_window,
                                int32_t stream_remote_window, uint32_t remote_max_frame_size, void* user_data);

constexpr uint8_t kFlagEndStream = 0x01;
constexpr uint32_t kDataEof = 0x01, kDataNoEndStream = 0x02, kDataNoCopy = 0x04;
constexpr uint8_t kTypeData = 0, kTypeHeaders = 1, kTypeRstStream = 3, kTypeGoaway = 7;
constexpr int kErrDeferred = -508;
constexpr int kErrCallbackFailure = -902;
constexpr int32_t kSettingsEnablePush = 2, kSettingsMaxConcurrentStreams = 3, kSettingsInitialWindowSize = 4,
                  kSettingsMaxFrameSize = 5;
constexpr uint32_t kCancel = 0x8;   // RST_STREAM error code
// Largest DATA frame either side offers or sends (the HTTP/2 default is 16 KiB).  gRPC data streams
// move 1 MiB chunks, so bigger frames cut per-frame work on both ends; the extra 64 bytes let a
// 1 MiB chunk's message (data + ~13-byte gRPC/protobuf header) travel as one frame instead of a
// 1 MiB frame plus a 13-byte tail.  Not larger: several frames stay in flight within the
// offset_received window (alluxio.worker.network.reader.buffer.size, 4 MiB).
constexpr uint32_t kMaxFramePayload = (1u << 20) + 64;
const char kPreface[] = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";

struct Lib {
  bool ok = false;
  int (*callbacks_new)(void**) = nullptr;
  void (*set_on_frame_recv)(void*, FrameCb) = nullptr;
  void (*set_on_begin_headers)(void*, FrameCb) = nullptr;
  void (*set_on_data_chunk_recv)(void*, DataChunkCb) = nullptr;
  void (*set_on_stream_close)(void*, CloseCb) = nullptr;
  void (*set_on_header)(void*, HeaderCb) = nullptr;
  void (*set_read_length)(void*, ReadLengthCb) = nullptr;
  void (*set_send_data)(void*, SendDataCb) = nullptr;
  int (*option_new)(void**) = nullptr;
  void (*option_del)(void*) = nullptr;
  void (*option_no_auto_window_update)(void*, int) = nullptr;
  int (*server_new2)(void**, const void*, void*, const void*) = nullptr;
  int (*client_new2)(void**, const void*, void*, const void*) = nullptr;
  void (*session_del)(void*) = nullptr;
  ssize_t (*mem_recv)(void*, const uint8_t*, size_t) = nullptr;
  ssize_t (*mem_send)(void*, const uint8_t**) = nullptr;
  int (*submit_settings)(void*, uint8_t, const SettingsEntry*, size_t) = nullptr;
  int (*submit_response)(void*, int32_t, const Nv*, size_t, const DataProvider*) = nullptr;
  int32_t (*submit_request)(void*, const void*, const Nv*, size_t, const DataProvider*, void*) = nullptr;
  int (*submit_trailer)(void*, int32_t, const Nv*, size_t) = nullptr;
  int (*submit_rst_stream)(void*, uint8_t, int32_t, uint32_t) = nullptr;
  int (*resume_data)(void*, int32_t) = nullptr;
  int (*consume_connection)(void*, size_t) = nullptr;
  int (*consume_stream)(void*, int32_t, size_t) = nullptr;
  int (*set_local_window_size)(void*, uint8_t, int32_t, int32_t) = nullptr;
  int (*want_read)(void*) = nullptr;
  int (*want_write)(void*) = nullptr;
};

// The loaded library (ok == false when absent or incomplete).
inline const Lib& lib() {
  static const Lib l = [] {
    Lib g;
    void* h = ::dlopen("libnghttp2.so.14", RTLD_NOW | RTLD_LOCAL);
    if (!h) return g;
    bool all = true;
    auto sym = [&](auto& fn, const char* name) {
      void* p = ::dlsym(h, name);
      if (!p) all = false;
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(p);
    };
    sym(g.callbacks_new, "nghttp2_session_callbacks_new");
    sym(g.set_on_frame_recv, "nghttp2_session_callbacks_set_on_frame_recv_callback");
    sym(g.set_on_begin_headers, "nghttp2_session_callbacks_set_on_begin_headers_callback");
    sym(g.set_on_data_chunk_recv, "nghttp2_session_callbacks_set_on_data_chunk_recv_callback");
    sym(g.set_on_stream_close, "nghttp2_session_callbacks_set_on_stream_close_callback");
    sym(g.set_on_header, "nghttp2_session_callbacks_set_on_header_callback");
    sym(g.set_read_length, "nghttp2_session_callbacks_set_data_source_read_length_callback");
    sym(g.set_send_data, "nghttp2_session_callbacks_set_send_data_callback");
    sym(g.option_new, "nghttp2_option_new");
    sym(g.option_del, "nghttp2_option_del");
    sym(g.option_no_auto_window_update, "nghttp2_option_set_no_auto_window_update");
    sym(g.server_new2, "nghttp2_session_server_new2");
    sym(g.client_new2, "nghttp2_session_client_new2");
    sym(g.session_del, "nghttp2_session_del");
    sym(g.mem_recv, "nghttp2_session_mem_recv");
    sym(g.mem_send, "nghttp2_session_mem_send");
    sym(g.submit_settings, "nghttp2_submit_settings");
    sym(g.submit_response, "nghttp2_submit_response");
    sym(g.submit_request, "nghttp2_submit_request");
    sym(g.submit_trailer, "nghttp2_submit_trailer");
    sym(g.submit_rst_stream, "nghttp2_submit_rst_stream");
    sym(g.resume_data, "nghttp2_session_resume_data");
    sym(g.consume_connection, "nghttp2_session_consume_connection");
    sym(g.consume_stream, "nghttp2_session_consume_stream");
    sym(g.set_local_window_size, "nghttp2_session_set_local_window_size");
    sym(g.want_read, "nghttp2_session_want_read");
    sym(g.want_write, "nghttp2_session_want_write");
    g.ok = all;
    return g;
  }();
  return l;
}

// name/value must outlive the submit call (nghttp2 copies them there): literals or named strings
inline Nv nv(const char* n, const char* v) {
  return Nv{reinterpret_cast<uint8_t*>(const_cast<char*>(n)), reinterpret_cast<uint8_t*>(const_cast<char*>(v)),
            std::strlen(n), std::strlen(v), 0};
}
inline Nv nv(const char* n, const std::string& v) {
  return Nv{reinterpret_cast<uint8_t*>(const_cast<char*>(n)), reinterpret_cast<uint8_t*>(const_cast<char*>(v.data())),
            std::strlen(n), v.size(), 0};
}
Nv nv(const char* n, std::string&&) = delete;

// DATA frame payload size: the whole window up to the peer's frame limit and kMaxFramePayload.
inline ssize_t read_length(void*, uint8_t, int32_t, int32_t session_window, int32_t stream_window,
                           uint32_t remote_max_frame, void*) {
  int64_t n = std::min<int64_t>(session_window, stream_window);
  n = std::min<int64_t>(n, remote_max_frame);
  n = std::min<int64_t>(n, kMaxFramePayload);
  return (ssize_t)std::max<int64_t>(n, 1);
}

// ---- protobuf / gRPC framing helpers ------------------------------------------------------
inline void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back((char)((v & 0x7F) | 0x80));
    v >>= 7;
  }
  s.push_back((char)v);
}
inline size_t varint_len(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++n;
  }
  return n;
}
// Reads a varint at p[*i..n); returns false when truncated/overlong.
inline bool get_varint(const uint8_t* p, size_t n, size_t* i, uint64_t* out) {
  uint64_t v = 0;
  for (int shift = 0; shift < 64 && *i < n; shift += 7) {
    const uint8_t b = p[(*i)++];
    v |= (uint64_t)(b & 0x7F) << shift;
    if (b < 0x80) {
      *out = v;
      return true;
    }
  }
  return false;
}
inline void put_be32(std::string& s, uint32_t v) {
  const char b[4] = {(char)(v >> 24), (char)(v >> 16), (char)(v >> 8), (char)v};
  s.append(b, 4);
}
// gRPC length prefix + ReadResponse{chunk{data = <n bytes>}} protobuf prefix of a data message
// (the bytes protobuf produces for that message; ReadResponseMarshaller's header).
inline std::string read_response_prefix(uint64_t n) {
  const uint64_t inner = 1 + varint_len(n) + n;
  const uint64_t outer = 1 + varint_len(inner) + inner;
  std::string h;
  h.reserve(16);
  h.push_back('\0');
  put_be32(h, (uint32_t)outer);
  h.push_back((char)0x0A);
  put_varint(h, inner);
  h.push_back((char)0x0A);
  put_varint(h, n);
  return h;
}

}  // namespace h2
}  // namespace amdx
