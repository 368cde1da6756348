// pybind11 bindings of the native worker data plane (module alluxio_amd._C).
// All entry points release the GIL: the Python worker serves many concurrent gRPC streams.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <pybind11/numpy.h>

#include <cmath>
#include <cstring>
#include <vector>

#include "block_store.h"
#include "trace.h"
#include "cpu_codecs.h"
#include "ipc.h"
#include "numa_host.h"
#include "ring_read.h"
#include "kernels.h"
#include "seg_ring.h"
#include "frame_rpc.h"
#include "journal_log.h"
#include "meta_codec.h"
#include "fuse_server.h"
#include "http_blob.h"

namespace py = pybind11;
using namespace amdx;

void bind_data_path(py::module_& m);   // data_path_bind.cpp

namespace {

#define HIP_CHECK(expr)                                                                   \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess) throw StoreError(kErrHip, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  explicit DevBuf(size_t n) { HIP_CHECK(hipMalloc(&p, n ? n : 1)); }
  ~DevBuf() { if (p) (void)hipFree(p); }
};

int hip_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

std::vector<uint32_t> crc32c_device(uint64_t ptr, uint64_t len, uint64_t piece, uint64_t stream) {
  if (piece == 0) piece = len ? len : 1;
  const uint64_t np = len ? (len + piece - 1) / piece : 0;
  std::vector<uint32_t> out(np);
  if (!np) return out;
  const uint64_t sw = crc32c_scratch_words(len, piece);
  DevBuf d((np + sw) * 4);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  HIP_CHECK(launch_crc32c_pieces(reinterpret_cast<const uint8_t*>(ptr), len, piece, (uint32_t*)d.p,
                                 (uint32_t*)d.p + np, sw, st));
  HIP_CHECK(hipMemcpyAsync(out.data(), d.p, np * 4, hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
  return out;
}

// Per-page CRC32C of pages scattered in an arena at `base` (page i of the block is
// base + pages[i] * page_bytes), one launch pair -- the form BlockStore::checksum_async uses.
std::vector<uint32_t> crc32c_device_pages(uint64_t base, const std::vector<int64_t>& pages, uint64_t len,
                                          uint64_t page_bytes) {
  if (!page_bytes) throw std::invalid_argument("page_bytes must be > 0");
  const uint64_t np = len ? (len + page_bytes - 1) / page_bytes : 0;
  if (pages.size() < np) throw std::invalid_argument("fewer pages than the length covers");
  std::vector<uint32_t> out(np);
  if (!np) return out;
  const uint64_t sw = crc32c_pages_scratch_words(len, page_bytes);
  DevBuf d((np + sw) * 4);
  DevBuf idx(np * sizeof(int64_t));
  HIP_CHECK(hipMemcpy(idx.p, pages.data(), np * sizeof(int64_t), hipMemcpyHostToDevice));
  HIP_CHECK(launch_crc32c_pages(reinterpret_cast<const uint8_t*>(base), (const int64_t*)idx.p, len, page_bytes,
                                (uint32_t*)d.p, (uint32_t*)d.p + np, sw, 0));
  HIP_CHECK(hipMemcpy(out.data(), d.p, np * 4, hipMemcpyDeviceToHost));
  return out;
}

// chunks: list of (src_ptr, dst_ptr, src_bytes, dst_capacity) on the device
std::vector<int32_t> lz4_device(const std::vector<std::tuple<uint64_t, uint64_t, uint32_t, uint32_t>>& chunks,
                                bool compress, uint64_t stream) {
  const int n = (int)chunks.size();
  std::vector<int32_t> sizes(n, 0);
  if (!n) return sizes;
  std::vector<Lz4Chunk> h(n);
  for (int i = 0; i < n; ++i) {
    h[i].src = std::get<0>(chunks[i]);
    h[i].dst = std::get<1>(chunks[i]);
    h[i].src_bytes = std::get<2>(chunks[i]);
    h[i].dst_capacity = std::get<3>(chunks[i]);
  }
  DevBuf dch(sizeof(Lz4Chunk) * n), dsz(sizeof(int32_t) * n);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  HIP_CHECK(hipMemcpyAsync(dch.p, h.data(), sizeof(Lz4Chunk) * n, hipMemcpyHostToDevice, st));
  if (compress) HIP_CHECK(launch_lz4_compress((Lz4Chunk*)dch.p, n, (int32_t*)dsz.p, st));
  else HIP_CHECK(launch_lz4_decompress((Lz4Chunk*)dch.p, n, (int32_t*)dsz.p, st));
  HIP_CHECK(hipMemcpyAsync(sizes.data(), dsz.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
  return sizes;
}

// Kernel-only timing of an LZ4 batch: the chunk table is uploaded once, `reps` launches are
// bracketed by HIP events (no per-call allocation / table upload / size download in the number).
double lz4_device_kernel_ms(const std::vector<std::tuple<uint64_t, uint64_t, uint32_t, uint32_t>>& chunks,
                            bool compress, int reps) {
  const int n = (int)chunks.size();
  if (!n || reps <= 0) return 0.0;
  std::vector<Lz4Chunk> h(n);
  for (int i = 0; i < n; ++i)
    h[i] = Lz4Chunk{std::get<0>(chunks[i]), std::get<1>(chunks[i]), std::get<2>(chunks[i]), std::get<3>(chunks[i])};
  DevBuf dch(sizeof(Lz4Chunk) * n), dsz(sizeof(int32_t) * n);
  HIP_CHECK(hipMemcpy(dch.p, h.data(), sizeof(Lz4Chunk) * n, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  HIP_CHECK(hipEventCreate(&a));
  HIP_CHECK(hipEventCreate(&b));
  auto launch = [&] {
    if (compress) HIP_CHECK(launch_lz4_compress((Lz4Chunk*)dch.p, n, (int32_t*)dsz.p, 0));
    else HIP_CHECK(launch_lz4_decompress((Lz4Chunk*)dch.p, n, (int32_t*)dsz.p, 0));
  };
  launch();
  HIP_CHECK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) launch();
  HIP_CHECK(hipEventRecord(b, 0));
  HIP_CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  HIP_CHECK(hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms / reps;
}

// Process-wide descriptor ring for ad-hoc batched copies (IPC reads, peer pulls): no per-call
// hipMalloc/hipFree (hipFree may synchronize the device).  Without a HIP device the segments are
// plain host memory and are copied with memcpy (CPU builds, shared-memory DRAM arenas).
SegRing& global_ring() {
  static SegRing* r = [] {
    auto* x = new SegRing();
    x->init();
    return x;
  }();
  return *r;
}

void batched_copy(const std::vector<std::tuple<uint64_t, uint64_t, uint64_t>>& segs, uint64_t stream, bool sync) {
  const size_t n = segs.size();
  if (!n) return;
  if (hip_device_count() == 0) {
    for (const auto& t : segs)
      std::memmove(reinterpret_cast<void*>(std::get<1>(t)), reinterpret_cast<const void*>(std::get<0>(t)),
                   std::get<2>(t));
    return;
  }
  std::vector<CopySeg> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = CopySeg{std::get<0>(segs[i]), std::get<1>(segs[i]), std::get<2>(segs[i]), 0};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  HIP_CHECK(global_ring().launch(h, st));
  if (sync) HIP_CHECK(hipStreamSynchronize(st));
}

// Stand-alone run of the grid-wide select (evict_alloc.hip) on caller arrays: slot i is a
// candidate of dir 0 when evictable[i]; `bytes` are the footprints.  Returns (slots, freed).
py::tuple evict_select_device(const std::vector<float>& crf, const std::vector<uint64_t>& last,
                              const std::vector<uint64_t>& bytes, const std::vector<uint8_t>& evictable,
                              uint64_t now, float step, float att, int policy, uint64_t need) {
  const size_t n = crf.size();
  if (last.size() != n || bytes.size() != n || evictable.size() != n)
    throw StoreError(kErrInvalidArgument, "evict_select_device: array length mismatch");
  std::vector<uint32_t> out;
  uint64_t freed = 0;
  {
    py::gil_scoped_release rel;
    std::vector<int32_t> dir(n);
    for (size_t i = 0; i < n; ++i) dir[i] = evictable[i] ? 0 : -1;
    DevBuf dc(n * 4 + 4), dl(n * 8 + 8), db(n * 8 + 8), dd(n * 4 + 4), dk(n * 4 + 4), dout(n * 4 + 4),
        dctl(sizeof(EvictCtl));
    HIP_CHECK(hipMemcpy(dc.p, crf.data(), n * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dl.p, last.data(), n * 8, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(db.p, bytes.data(), n * 8, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dd.p, dir.data(), n * 4, hipMemcpyHostToDevice));
    EvictState st;
    st.crf = (float*)dc.p;
    st.last = (uint64_t*)dl.p;
    st.fbytes = (uint64_t*)db.p;
    st.dir = (int32_t*)dd.p;
    st.n = (uint32_t)n;
    st.now = now;
    st.step = step;
    st.log2_inv_att = (float)std::log2(1.0 / (double)att);
    st.policy = policy;
    st.dir_mask = 0;
    st.unit = 0;
    st.invert = 0;
    HIP_CHECK(launch_evict_select_grid(st, 0, nullptr, need, (uint32_t*)dk.p, (EvictCtl*)dctl.p, (uint32_t*)dout.p,
                                       nullptr));
    EvictCtl ctl;
    HIP_CHECK(hipMemcpy(&ctl, dctl.p, sizeof(ctl), hipMemcpyDeviceToHost));
    freed = ctl.freed;
    out.resize(ctl.count);
    if (ctl.count) HIP_CHECK(hipMemcpy(out.data(), dout.p, ctl.count * 4, hipMemcpyDeviceToHost));
  }
  return py::make_tuple(out, freed);
}

// K7 stand-alone: claim `want` free pages from a caller bitmap (returns (pages, new_bitmap)).
py::tuple page_alloc_device(const std::vector<uint64_t>& bits, uint32_t want) {
  const uint32_t nw = (uint32_t)bits.size();
  std::vector<int64_t> pages;
  std::vector<uint64_t> after(nw);
  {
    py::gil_scoped_release rel;
    DevBuf db((size_t)nw * 8 + 8), dp((size_t)page_alloc_partials(nw) * 4 + 4), dout((size_t)want * 8 + 8), dc(8);
    if (nw) HIP_CHECK(hipMemcpy(db.p, bits.data(), (size_t)nw * 8, hipMemcpyHostToDevice));
    HIP_CHECK(launch_page_alloc((uint64_t*)db.p, nw, want, (uint32_t*)dp.p, (int64_t*)dout.p, (uint32_t*)dc.p,
                                nullptr));
    uint32_t got = 0;
    HIP_CHECK(hipMemcpy(&got, dc.p, 4, hipMemcpyDeviceToHost));
    pages.resize(got);
    if (got) HIP_CHECK(hipMemcpy(pages.data(), dout.p, (size_t)got * 8, hipMemcpyDeviceToHost));
    if (nw) HIP_CHECK(hipMemcpy(after.data(), db.p, (size_t)nw * 8, hipMemcpyDeviceToHost));
  }
  return py::make_tuple(pages, after);
}

}  // namespace

#include "page_cache_bind.h"

PYBIND11_MODULE(_C, m) {
  m.doc() = "MI355X-native worker data plane: HBM page store + CDNA4 kernels";
  bind_page_cache(m);
  m.def("encode_inode_file_batch",
        [](const std::string& tmpl, const std::vector<int64_t>& ids, const std::vector<int64_t>& parents,
           const std::vector<std::string>& names, const std::vector<int64_t>& lengths, int64_t block_size,
           const std::vector<std::string>& fps, const std::vector<int64_t>& mtimes, int64_t ctime) {
          std::string out;
          {
            py::gil_scoped_release rel;
            out = encode_inode_file_batch(tmpl, ids, parents, names, lengths, block_size, fps, mtimes, ctime);
          }
          return py::bytes(out);
        });
  m.def("decode_file_infos", [](const std::vector<std::string>& chunks) {
    FileInfoColumns c;
    {
      py::gil_scoped_release rel;
      decode_file_infos(chunks, c);
    }
    auto arr = [](const auto& v) {
      using T = typename std::decay_t<decltype(v)>::value_type;
      py::array_t<T> a(v.size());
      if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
      return a;
    };
    py::dict d;
    d["ids"] = arr(c.ids);
    d["lengths"] = arr(c.lengths);
    d["block_sizes"] = arr(c.block_sizes);
    d["first_blocks"] = arr(c.first_blocks);
    d["nblocks"] = arr(c.nblocks);
    d["folder"] = arr(c.folder);
    d["completed"] = arr(c.completed);
    d["mtimes"] = arr(c.mtimes);
    d["atimes"] = arr(c.atimes);
    d["modes"] = arr(c.modes);
    d["chunk"] = arr(c.chunk);
    d["offset"] = arr(c.offset);
    d["size"] = arr(c.size);
    d["paths"] = py::cast(c.paths);
    return d;
  });
  m.def("encode_block_info_batch", [](const std::vector<int64_t>& ids, const std::vector<int64_t>& lengths) {
    std::string out;
    {
      py::gil_scoped_release rel;
      out = encode_block_info_batch(ids, lengths);
    }
    return py::bytes(out);
  });
  m.def("encode_file_infos",
        [](const std::string& tmpl, const std::vector<int64_t>& ids, const std::vector<std::string>& names,
           const std::string& parent_path, const std::string& parent_ufs, const std::vector<int64_t>& lengths,
           int64_t block_size, const std::vector<int64_t>& ctimes, const std::vector<int64_t>& mtimes,
           const std::vector<int64_t>& atimes, const std::vector<std::string>& fps,
           const std::vector<std::string>& block_infos, const std::vector<int32_t>& in_alluxio,
           const std::vector<int32_t>& in_memory, uint32_t out_field, bool ufs_locations) {
          std::string out;
          {
            py::gil_scoped_release rel;
            out = encode_file_infos(tmpl, ids, names, parent_path, parent_ufs, lengths, block_size, ctimes, mtimes,
                                    atimes, fps, block_infos, in_alluxio, in_memory, out_field, ufs_locations);
          }
          return py::bytes(out);
        });

  static py::exception<StoreError> store_error(m, "StoreError");
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const StoreError& e) {
      // args = (code, message); alluxio_amd/ops/native.py maps code -> status exception
      py::object inst = py::reinterpret_steal<py::object>(
          PyObject_CallFunction(store_error.ptr(), "is", e.code, e.what()));
      PyErr_SetObject(store_error.ptr(), inst.ptr());
    }
  });

  py::enum_<DirKind>(m, "DirKind").value("DEVICE", DirKind::kDevice).value("HOST", DirKind::kHost)
      .value("FILE", DirKind::kFile);

  py::class_<DirSpec>(m, "DirSpec")
      .def(py::init<>())
      .def_readwrite("tier", &DirSpec::tier)
      .def_readwrite("tier_alias", &DirSpec::tier_alias)
      .def_readwrite("medium", &DirSpec::medium)
      .def_readwrite("kind", &DirSpec::kind)
      .def_readwrite("base", &DirSpec::base)
      .def_readwrite("capacity", &DirSpec::capacity)
      .def_readwrite("page_size", &DirSpec::page_size)
      .def_readwrite("device", &DirSpec::device)
      .def_readwrite("path", &DirSpec::path)
      .def_readwrite("owns_base", &DirSpec::owns_base)
      .def_readwrite("reserved", &DirSpec::reserved);

  py::class_<BlockInfoOut>(m, "BlockInfo")
      .def_readonly("id", &BlockInfoOut::id)
      .def_readonly("length", &BlockInfoOut::length)
      .def_readonly("tier", &BlockInfoOut::tier)
      .def_readonly("dir", &BlockInfoOut::dir)
      .def_readonly("tier_alias", &BlockInfoOut::tier_alias)
      .def_readonly("medium", &BlockInfoOut::medium)
      .def_readonly("temp", &BlockInfoOut::temp)
      .def_readonly("session", &BlockInfoOut::session)
      .def_readonly("readers", &BlockInfoOut::readers)
      .def_readonly("writer", &BlockInfoOut::writer);

  py::class_<Event>(m, "Event")
      .def_readonly("kind", &Event::kind)
      .def_readonly("block_id", &Event::block_id)
      .def_readonly("tier_alias", &Event::tier_alias)
      .def_readonly("medium", &Event::medium);

  using G = py::call_guard<py::gil_scoped_release>;
  py::class_<BlockStore, std::shared_ptr<BlockStore>>(m, "BlockStore", py::dynamic_attr())
      .def(py::init<const std::vector<DirSpec>&, int, int, float, float, int>(), py::arg("dirs"),
           py::arg("annotator") = 0, py::arg("alloc_policy") = 0, py::arg("lrfu_step") = 0.25f,
           py::arg("lrfu_attenuation") = 2.0f, py::arg("device") = 0)
      .def("create_block", &BlockStore::create_block, G(), py::arg("session"), py::arg("block_id"),
           py::arg("tier") = -1, py::arg("medium") = "", py::arg("initial") = 1 << 20,
           py::arg("evict") = true, py::arg("pin") = false)
      .def("request_space", &BlockStore::request_space, G())
      .def("write", &BlockStore::write, G(), py::arg("session"), py::arg("block_id"), py::arg("offset"),
           py::arg("src"), py::arg("length"), py::arg("src_kind"), py::arg("stream") = 0,
           py::arg("sync") = true)
      .def("external_write", &BlockStore::external_write, G(), py::arg("session"), py::arg("block_id"),
           py::arg("offset"), py::arg("length"))
      .def("commit_block", &BlockStore::commit_block, G(), py::arg("session"), py::arg("block_id"),
           py::arg("pin") = false)
      .def("abort_block", &BlockStore::abort_block, G())
      .def("remove_block", &BlockStore::remove_block, G())
      .def("move_block", &BlockStore::move_block, G(), py::arg("session"), py::arg("block_id"),
           py::arg("tier"), py::arg("medium") = "", py::arg("evict") = true)
      .def("lock_block", &BlockStore::lock_block, G(), py::arg("session"), py::arg("block_id"),
           py::arg("write") = false, py::arg("timeout_ms") = -1)
      .def("unlock", &BlockStore::unlock, G())
      .def("hold_block", &BlockStore::hold_block, G(), py::arg("block_id"), py::arg("ttl_ms") = 120000)
      .def("release_hold", &BlockStore::release_hold, G())
      .def_property_readonly("holds", &BlockStore::holds)
      .def("cleanup_session", &BlockStore::cleanup_session, G())
      .def("access_block", &BlockStore::access_block, G())
      .def("access_blocks", &BlockStore::access_blocks, G())
      .def("read_batch",
           [](BlockStore& s, const std::vector<std::tuple<int64_t, uint64_t, uint64_t, uint64_t, int>>& reqs,
              uint64_t stream, bool sync) {
             std::vector<ReadReq> rs;
             rs.reserve(reqs.size());
             for (auto& t : reqs)
               rs.push_back(ReadReq{std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t), std::get<4>(t)});
             py::gil_scoped_release rel;
             s.read_batch(rs, stream, sync);
           },
           py::arg("reqs"), py::arg("stream") = 0, py::arg("sync") = true)
      // The same batched read from parallel arrays (no per-request Python tuples): the record
      // gather of a training input batch (models/dataset.py).
      .def("read_batch_arrays",
           [](BlockStore& s, py::array_t<int64_t, py::array::c_style | py::array::forcecast> ids,
              py::array_t<uint64_t, py::array::c_style | py::array::forcecast> offs,
              py::array_t<uint64_t, py::array::c_style | py::array::forcecast> lens,
              py::array_t<uint64_t, py::array::c_style | py::array::forcecast> dsts, int kind, uint64_t stream,
              bool sync) {
             const ssize_t n = ids.size();
             if (offs.size() != n || lens.size() != n || dsts.size() != n)
               throw StoreError(kErrInvalidArgument, "read_batch_arrays: length mismatch");
             std::vector<ReadReq> rs((size_t)n);
             const int64_t* pi = ids.data();
             const uint64_t *po = offs.data(), *pl = lens.data(), *pd = dsts.data();
             for (ssize_t i = 0; i < n; ++i) rs[(size_t)i] = ReadReq{pi[i], po[i], pl[i], pd[i], kind};
             py::gil_scoped_release rel;
             s.read_batch(rs, stream, sync);
           },
           py::arg("block_ids"), py::arg("offsets"), py::arg("lengths"), py::arg("dsts"), py::arg("dst_kind"),
           py::arg("stream") = 0, py::arg("sync") = true)
      .def("read", [](BlockStore& s, int64_t id, uint64_t off, uint64_t len, uint64_t dst, int kind,
                      uint64_t stream, bool sync) {
             std::vector<ReadReq> rs{ReadReq{id, off, len, dst, kind}};
             py::gil_scoped_release rel;
             s.read_batch(rs, stream, sync);
           },
           py::arg("block_id"), py::arg("offset"), py::arg("length"), py::arg("dst"), py::arg("dst_kind"),
           py::arg("stream") = 0, py::arg("sync") = true)
      // One gRPC data frame: ``header`` (hand-encoded protobuf prefix) followed by ``length`` block
      // bytes, built in a single bytes object the transport sends as-is -- the block bytes are
      // copied once (HBM/DRAM -> frame), not through a protobuf message (ReadResponseMarshaller).
      .def("read_frame", [](BlockStore& s, int64_t id, uint64_t off, uint64_t len, py::bytes header) {
             char* hp = nullptr;
             Py_ssize_t hn = 0;
             PyBytes_AsStringAndSize(header.ptr(), &hp, &hn);
             PyObject* out = PyBytes_FromStringAndSize(nullptr, hn + static_cast<Py_ssize_t>(len));
             if (out == nullptr) throw py::error_already_set();
             py::bytes frame = py::reinterpret_steal<py::bytes>(out);
             char* dst = PyBytes_AS_STRING(out);
             std::memcpy(dst, hp, static_cast<size_t>(hn));
             std::vector<ReadReq> rs{ReadReq{id, off, len, reinterpret_cast<uint64_t>(dst + hn), 0}};
             {
               py::gil_scoped_release rel;
               s.read_batch(rs, 0, true);
             }
             return frame;
           },
           py::arg("block_id"), py::arg("offset"), py::arg("length"), py::arg("header"))
      .def("checksum", &BlockStore::checksum, G(), py::arg("block_id"), py::arg("piece_bytes") = 0)
      .def("fill_pattern", &BlockStore::fill_pattern, G())
      .def("free_space", &BlockStore::free_space, G(), py::arg("session"), py::arg("bytes"),
           py::arg("tier") = -1, py::arg("dir") = -1)
      .def("eviction_order", &BlockStore::eviction_order, G(), py::arg("tier") = -1, py::arg("need_bytes") = 0)
      .def("set_pinned_files", &BlockStore::set_pinned_files, G())
      .def("set_use_device_evict", &BlockStore::set_use_device_evict, G())
      .def("set_use_device_alloc", &BlockStore::set_use_device_alloc, py::arg("enabled"), py::arg("min_pages") = 64)
      .def("set_demote_on_evict", &BlockStore::set_demote_on_evict)
      .def("move_blocks", &BlockStore::move_blocks, G(), py::arg("session"), py::arg("block_ids"), py::arg("tier"),
           py::arg("medium") = "", py::arg("evict") = true, py::arg("use_reserved") = false)
      .def("tier_order", &BlockStore::tier_order, G(), py::arg("tier"), py::arg("k"), py::arg("hottest") = false,
           py::arg("device") = true)
      .def("annotator_keys", &BlockStore::annotator_keys, G())
      .def("dir_mgmt_available", &BlockStore::dir_mgmt_available, G())
      .def("checksum_blocks", &BlockStore::checksum_blocks, G(), py::arg("block_ids"),
           py::arg("device_only") = false)
      .def("ingest_files", &BlockStore::ingest_files, G(), py::arg("session"), py::arg("block_ids"),
           py::arg("paths"), py::arg("offsets"), py::arg("lengths"), py::arg("staging"), py::arg("staging_bytes"),
           py::arg("threads") = 8, py::arg("stream") = 0)
      .def("create_blocks", &BlockStore::create_blocks, G(), py::arg("session"), py::arg("block_ids"),
           py::arg("tier") = -1, py::arg("medium") = "", py::arg("sizes") = std::vector<uint64_t>{},
           py::arg("evict") = true)
      .def("select_for_bench", &BlockStore::select_for_bench, G(), py::arg("dir"), py::arg("need"),
           py::arg("device"))
      .def("peek_free_pages", &BlockStore::peek_free_pages, G(), py::arg("dir"), py::arg("want"), py::arg("device"))
      .def("evict_stats", [](BlockStore& s) {
             auto st = s.evict_stats();
             py::dict d;
             d["selections"] = st.selections;
             d["device_selections"] = st.device_selections;
             d["candidates"] = st.candidates;
             d["victims"] = st.victims;
             d["revalidated_away"] = st.revalidated_away;
             d["device_allocs"] = st.device_allocs;
             d["device_alloc_pages"] = st.device_alloc_pages;
             d["annotation_flushes"] = st.annotation_flushes;
             d["annotation_updates"] = st.annotation_updates;
             d["demoted_blocks"] = st.demoted_blocks;
             d["demoted_bytes"] = st.demoted_bytes;
             d["batched_moves"] = st.batched_moves;
             d["batched_move_blocks"] = st.batched_move_blocks;
             d["mag_refills"] = st.mag_refills;
             d["mag_refill_pages"] = st.mag_refill_pages;
             d["mag_drains"] = st.mag_drains;
             d["mag_drain_pages"] = st.mag_drain_pages;
             d["mag_short_items"] = st.mag_short_items;
             d["evict_waits"] = st.evict_waits;
             d["evict_retries"] = st.evict_retries;
             d["ingest_ns"] = std::vector<uint64_t>(st.ingest_ns, st.ingest_ns + 6);
             return d;
           })
      .def("mag_refill", &BlockStore::mag_refill_pages, G())
      .def("mag_pages", &BlockStore::mag_pages, G())
      .def("mag_device_count", &BlockStore::mag_device_count, G())
      .def("check_pages", &BlockStore::check_pages, G())
      .def("set_free_ahead", &BlockStore::set_free_ahead, py::arg("bytes"))
      .def("mag_claim_many", &BlockStore::mag_claim_many, G())
      .def("mag_give", &BlockStore::mag_give, G())
      .def("mag_drain", &BlockStore::mag_drain_dir, G())
      .def("has_block", &BlockStore::has_block, G())
      .def("has_temp_block", &BlockStore::has_temp_block, G())
      .def("block_info", &BlockStore::block_info, G())
      .def("block_ids", &BlockStore::block_ids, G(), py::arg("tier") = -1)
      .def("block_pages", [](BlockStore& s, int64_t id) {
             int dir = 0;
             uint64_t ps = 0, base = 0;
             std::vector<int64_t> pages;
             {
               py::gil_scoped_release rel;
               pages = s.block_pages(id, &dir, &ps, &base);
             }
             return py::make_tuple(pages, dir, ps, base);
           })
      .def("drain_events", &BlockStore::drain_events, G())
      .def("num_dirs", &BlockStore::num_dirs)
      .def("dir_spec", &BlockStore::dir_spec)
      .def("dir_capacity", &BlockStore::dir_capacity, G())
      .def("dir_available", &BlockStore::dir_available, G())
      .def("dir_committed", &BlockStore::dir_committed, G())
      .def("set_dir_healthy", &BlockStore::set_dir_healthy, G())
      .def("dir_healthy", &BlockStore::dir_healthy, G())
      .def("clock", &BlockStore::clock)
      .def("device", &BlockStore::device)
      .def("stats", &BlockStore::stats, G());

  py::class_<ReadSession>(m, "ReadSession")
      .def(py::init<BlockStore*, int64_t, const std::vector<int64_t>&, const std::vector<uint64_t>&,
                    const std::vector<uint64_t>&, uint64_t, int, const std::vector<uint64_t>&>(),
           py::arg("store"), py::arg("session"), py::arg("block_ids"), py::arg("block_lens"), py::arg("dst_ptrs"),
           py::arg("buf_bytes"), py::arg("dst_kind"), py::arg("start_offsets") = std::vector<uint64_t>{},
           py::keep_alive<1, 2>())
      .def("step", [](ReadSession& r, uint64_t stream) {
             std::vector<int> reopened;
             uint64_t b;
             {
               py::gil_scoped_release rel;
               b = r.step(stream, &reopened);
             }
             return py::make_tuple(b, reopened);
           }, py::arg("stream") = 0)
      .def("run", &ReadSession::run, G(), py::arg("steps"), py::arg("stream") = 0)
      .def("reset_file", &ReadSession::reset_file, G())
      .def("close", &ReadSession::close, G())
      .def("position", &ReadSession::position)
      .def_property_readonly("total_bytes", &ReadSession::total_bytes)
      .def_property_readonly("reopens", &ReadSession::reopens);

  py::class_<RingReadSession>(m, "RingReadSession")
      .def(py::init([](BlockStore& store, int64_t session, const std::vector<int64_t>& blocks,
                       const std::vector<uint64_t>& lens, uint64_t dst_base, uint64_t stride, uint64_t buf,
                       uint32_t depth, uint32_t streams, int kind, const std::vector<uint64_t>& starts) {
             py::gil_scoped_release rel;
             return new RingReadSession(&store, session, blocks, lens, dst_base, stride, buf, depth, streams, kind,
                                        starts);
           }),
           py::arg("store"), py::arg("session"), py::arg("block_ids"), py::arg("block_lens"), py::arg("dst_base"),
           py::arg("stream_stride"), py::arg("buf_bytes"), py::arg("depth"), py::arg("streams"),
           py::arg("dst_kind"), py::arg("start_offsets") = std::vector<uint64_t>{}, py::keep_alive<1, 2>())
      .def_static("remote", [](uint64_t arena, const std::vector<int64_t>& pages, uint64_t page_size, uint64_t file_len,
                               int device, uint64_t dst_base, uint64_t stride, uint64_t buf, uint32_t depth,
                               uint32_t streams, int kind, const std::vector<uint64_t>& starts) {
             py::gil_scoped_release rel;
             return std::unique_ptr<RingReadSession>(new RingReadSession(arena, pages, page_size, file_len, device,
                                                                         dst_base, stride, buf, depth, streams,
                                                                         kind, starts));
           },
           py::arg("arena_base"), py::arg("file_pages"), py::arg("page_size"), py::arg("file_len"), py::arg("device"),
           py::arg("dst_base"), py::arg("stream_stride"), py::arg("buf_bytes"), py::arg("depth"), py::arg("streams"),
           py::arg("dst_kind"), py::arg("start_offsets") = std::vector<uint64_t>{})
      .def("step", [](RingReadSession& r, uint64_t stream) {
             uint64_t eofs = 0, n;
             {
               py::gil_scoped_release rel;
               n = r.step(stream, &eofs);
             }
             return py::make_tuple(n, eofs);
           }, py::arg("stream") = 0)
      .def("close", &RingReadSession::close, G())
      .def("position", &RingReadSession::position)
      .def("last_call", &RingReadSession::last_call)
      .def_property_readonly("total_bytes", &RingReadSession::total_bytes)
      .def_property_readonly("reopens", &RingReadSession::reopens)
      .def_property_readonly("calls", &RingReadSession::calls)
      .def_property_readonly("file_len", &RingReadSession::file_len);

  // ---- native S3 data path (http_blob.cpp) --------------------------------------------------
  py::class_<BlobServer>(m, "BlobServer")
      .def(py::init<const std::string&, const std::string&, int>(), py::arg("root"), py::arg("host") = "127.0.0.1",
           py::arg("port") = 0)
      .def("start", &BlobServer::start, G())
      .def("stop", &BlobServer::stop, G())
      .def_property_readonly("port", &BlobServer::port)
      .def_property_readonly("requests", &BlobServer::requests)
      .def_property_readonly("bytes_sent", &BlobServer::bytes_sent)
      .def("inject", &BlobServer::inject, py::arg("kind"), py::arg("method") = "", py::arg("nth") = 1,
           py::arg("count") = 1, py::arg("stall_ms") = 0)
      .def("clear_faults", &BlobServer::clear_faults)
      .def_property_readonly("injected", &BlobServer::injected);
  py::class_<HttpRangeReader>(m, "HttpRangeReader")
      .def(py::init([](const std::string& host, int port, int max_idle, int connect_timeout_ms, int socket_timeout_ms,
                       int request_timeout_ms, int max_retries, int backoff_base_ms, int backoff_max_ms) {
             HttpOptions o;
             o.connect_timeout_ms = connect_timeout_ms;
             o.socket_timeout_ms = socket_timeout_ms;
             o.request_timeout_ms = request_timeout_ms;
             o.max_retries = std::max(0, max_retries);
             o.backoff_base_ms = std::max(1, backoff_base_ms);
             o.backoff_max_ms = std::max(o.backoff_base_ms, backoff_max_ms);
             return new HttpRangeReader(host, port, max_idle, o);
           }),
           py::arg("host"), py::arg("port"), py::arg("max_idle") = 16, py::arg("connect_timeout_ms") = 10000,
           py::arg("socket_timeout_ms") = 50000, py::arg("request_timeout_ms") = 60000, py::arg("max_retries") = 3,
           py::arg("backoff_base_ms") = 50, py::arg("backoff_max_ms") = 2000)
      .def_property_readonly("retries", &HttpRangeReader::retries)
      .def_property_readonly("timeouts", &HttpRangeReader::timeouts)
      .def("get_into", [](HttpRangeReader& r, const std::string& target, const std::string& head, uint64_t offset,
                          uint64_t length, uint64_t dst, int parallel, uint64_t min_part) {
             py::gil_scoped_release rel;
             return r.get_into(target, head, offset, length, dst, parallel, min_part);
           }, py::arg("target"), py::arg("head_lines"), py::arg("offset"),
           py::arg("length"), py::arg("dst"), py::arg("parallel") = 1, py::arg("min_part") = 4 << 20)
      .def("put_from", [](HttpRangeReader& r, const std::string& target, const std::string& head, uint64_t src,
                          uint64_t length) {
             std::string etag;
             int code;
             {
               py::gil_scoped_release rel;
               code = r.put_from(target, head, src, length, &etag);
             }
             return py::make_tuple(code, etag);
           }, py::arg("target"), py::arg("head_lines"), py::arg("src"), py::arg("length"))
      .def_property_readonly("requests", &HttpRangeReader::requests)
      .def_property_readonly("connects", &HttpRangeReader::connects);

  // ---- native framed RPC (control-plane fast path) ----------------------------------------
  py::class_<FrameRpcServer>(m, "FrameRpcServer")
      .def(py::init<const std::string&, int, const std::vector<std::string>&, const std::vector<int>&, int>(),
           py::arg("host"), py::arg("port"), py::arg("methods"), py::arg("lanes"), py::arg("io_threads") = 2)
      .def("start", &FrameRpcServer::start, G())
      .def("stop", &FrameRpcServer::stop, G())
      .def_property_readonly("port", &FrameRpcServer::port)
      .def_property_readonly("requests", &FrameRpcServer::requests)
      .def("poll", [](FrameRpcServer& s, int lane, int max_n, int timeout_ms) {
             std::vector<FrameRequest> v;
             {
               py::gil_scoped_release rel;
               v = s.poll(lane, max_n, timeout_ms);
             }
             py::list out;
             for (auto& r : v)
               out.append(py::make_tuple(r.token, r.method, py::str(r.user), py::bytes(r.payload)));
             return out;
           }, py::arg("lane"), py::arg("max_n"), py::arg("timeout_ms"))
      .def("respond", [](FrameRpcServer& s, uint64_t token, int status, const std::string& msg, py::bytes payload) {
             std::string p = payload;
             py::gil_scoped_release rel;
             s.respond(token, status, msg, p);
           }, py::arg("token"), py::arg("status"), py::arg("message"), py::arg("payload"))
      .def("respond_many", [](FrameRpcServer& s, const py::list& items) {
             std::vector<FrameReply> v;
             v.reserve(items.size());
             for (auto it : items) {
               auto t = it.cast<py::tuple>();
               v.push_back(FrameReply{t[0].cast<uint64_t>(), t[1].cast<int>(), t[2].cast<std::string>(),
                                      std::string(t[3].cast<py::bytes>())});
             }
             py::gil_scoped_release rel;
             s.respond_batch(v);
           })
      .def("set_user", &FrameRpcServer::set_user)
      .def("set_cacheable", &FrameRpcServer::set_cacheable)
      .def("set_method_kind", &FrameRpcServer::set_method_kind)
      .def_property_readonly("grpc_requests", &FrameRpcServer::grpc_requests)
      .def_static("grpc_available", &FrameRpcServer::grpc_available)
      .def("epoch", &FrameRpcServer::epoch)
      .def("bump_epoch", &FrameRpcServer::bump_epoch)
      .def("cache_put", [](FrameRpcServer& s, uint32_t method, const std::string& user, py::bytes request,
                           py::bytes reply, uint64_t ep, int status, const std::string& msg) {
             std::string rq = request, rp = reply;
             s.cache_put(method, user, rq, rp, ep, status, msg);
           }, py::arg("method"), py::arg("user"), py::arg("request"), py::arg("reply"), py::arg("epoch"),
           py::arg("status") = 0, py::arg("msg") = std::string())
      .def("cache_clear", &FrameRpcServer::cache_clear)
      .def("set_cache_capacity", &FrameRpcServer::set_cache_capacity)
      .def_property_readonly("cache_size", &FrameRpcServer::cache_size)
      .def_property_readonly("cache_hits", &FrameRpcServer::cache_hits);
  py::class_<FuseServer>(m, "FuseServer")
      .def(py::init([](int fd, int threads, py::object store, int64_t session, int keep_cache) {
             BlockStore* bs = store.is_none() ? nullptr : store.cast<BlockStore*>();
             return new FuseServer(fd, threads, bs, session, keep_cache);
           }),
           py::arg("fd"), py::arg("threads") = 4, py::arg("store") = py::none(), py::arg("session") = 0,
           py::arg("keep_cache") = 2, py::keep_alive<1, 4>())
      .def("start", &FuseServer::start, G())
      .def("stop", &FuseServer::stop, G())
      .def_property_readonly("alive", &FuseServer::alive)
      .def("poll", [](FuseServer& s, int max_n, int timeout_ms) {
             std::vector<FuseRequest> v;
             {
               py::gil_scoped_release rel;
               v = s.poll(max_n, timeout_ms);
             }
             py::list out;
             for (auto& r : v)
               out.append(py::make_tuple(r.unique, r.opcode, r.nodeid, r.uid, r.gid, r.pid, py::bytes(r.body)));
             return out;
           })
      .def("reply", [](FuseServer& s, uint64_t unique, int err, py::bytes payload) {
             std::string p = payload;
             py::gil_scoped_release rel;
             s.reply(unique, err, p);
           }, py::arg("unique"), py::arg("err"), py::arg("payload") = py::bytes())
      .def("node_of", &FuseServer::node_of, G())
      .def("path_of", [](FuseServer& s, uint64_t nodeid) -> py::object {
             bool ok = false;
             std::string p = s.path_of(nodeid, &ok);
             if (!ok) return py::none();
             return py::str(p);
           })
      .def("forget_path", &FuseServer::forget_path, G())
      .def("register_write_handle", &FuseServer::register_write_handle, py::arg("fh"), py::arg("offset") = 0, G())
      .def("unregister_write_handle", &FuseServer::unregister_write_handle, G())
      .def("batch_done", &FuseServer::batch_done, G())
      .def("wait_batches", &FuseServer::wait_batches, py::arg("fh"), py::arg("timeout_ms") = 120000, G())
      .def_property_readonly("write_batches", &FuseServer::write_batches)
      .def("moved", &FuseServer::moved, G())
      .def("put_attr", [](FuseServer& s, const std::string& path, py::bytes attr, int64_t ttl_ms, uint32_t valid_s,
                          int64_t file_id, bool complete, const std::vector<int64_t>& blocks,
                          const std::vector<int64_t>& lens) {
             std::string a = attr;
             s.put_attr(path, a, ttl_ms, valid_s, file_id, complete, blocks, lens);
           }, py::arg("path"), py::arg("attr"), py::arg("ttl_ms"), py::arg("valid_s"), py::arg("file_id") = 0,
           py::arg("complete") = false, py::arg("blocks") = std::vector<int64_t>{},
           py::arg("lens") = std::vector<int64_t>{})
      .def("invalidate", &FuseServer::invalidate, G(), py::arg("path"), py::arg("subtree") = true)
      .def("clear_attrs", &FuseServer::clear_attrs, G())
      .def("keep_open", &FuseServer::keep_open, G())
      .def("set_no_open", &FuseServer::set_no_open)
      .def("cache_listing", [](FuseServer& s, const std::vector<std::string>& chunks, const std::string& strip,
                               uint32_t uid, uint32_t gid, uint32_t file_ttl_s, uint32_t dir_ttl_s) {
             py::gil_scoped_release rel;
             return s.cache_listing(chunks, strip, uid, gid, file_ttl_s, dir_ttl_s);
           }, py::arg("chunks"), py::arg("strip"), py::arg("uid"), py::arg("gid"), py::arg("file_ttl_s") = 60,
           py::arg("dir_ttl_s") = 1)
      .def("entry", [](FuseServer& s, const std::string& path) -> py::object {
             std::string out;
             bool ok;
             {
               py::gil_scoped_release rel;
               ok = s.entry_reply(path, out);
             }
             if (!ok) return py::none();
             return py::bytes(out);
           })
      .def("add_arena", &FuseServer::add_arena)
      .def("set_passthrough", &FuseServer::set_passthrough)
      .def_property_readonly("passthrough_opens", &FuseServer::passthrough_opens)
      .def("stats", &FuseServer::stats)
      .def_property_readonly("native_opens", &FuseServer::native_opens)
      .def_property_readonly("native_reads", &FuseServer::native_reads)
      .def_property_readonly("fallback_opens", &FuseServer::fallback_opens);
  py::class_<JournalLog>(m, "JournalLog")
      .def(py::init<const std::string&, uint64_t, uint64_t, bool, double>(), py::arg("log_dir"),
           py::arg("next_seq"), py::arg("max_log_bytes"), py::arg("fsync") = true, py::arg("batch_ms") = 5.0)
      .def("append", [](JournalLog& j, py::bytes entry) {
             std::string e = entry;   // short critical section: no GIL release
             return j.append(e);
           })
      .def("request", &JournalLog::request)
      .def("wait_flushed", &JournalLog::wait_flushed, py::arg("counter"), py::arg("timeout_ms") = -1,
           py::call_guard<py::gil_scoped_release>())
      .def("reply_when_flushed", [](JournalLog& j, uint64_t counter, FrameRpcServer& srv, const py::tuple& t) {
             FrameReply r{t[0].cast<uint64_t>(), t[1].cast<int>(), t[2].cast<std::string>(),
                          std::string(t[3].cast<py::bytes>())};
             py::gil_scoped_release rel;
             j.reply_when_flushed(counter, &srv, std::move(r));
           })
      .def("close", &JournalLog::close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("next_seq", &JournalLog::next_seq)
      .def_property_readonly("appended", &JournalLog::appended)
      .def_property_readonly("flushed", &JournalLog::flushed)
      .def_property_readonly("error", &JournalLog::error)
      .def_property_readonly("flushes", &JournalLog::flushes)
      .def_property_readonly("segments", &JournalLog::segments)
      .def("stats", &JournalLog::stats);

  py::class_<FrameRpcClient>(m, "FrameRpcClient")
      .def(py::init<const std::string&, int, const std::string&, int>(), py::arg("host"), py::arg("port"),
           py::arg("auth"), py::arg("timeout_ms") = 60000)
      .def("call", [](FrameRpcClient& c, const std::string& path, py::bytes payload, int timeout_ms) {
             std::string p = payload;
             std::tuple<int, std::string, std::string> r;
             {
               py::gil_scoped_release rel;
               r = c.call(path, p, timeout_ms);
             }
             return py::make_tuple(std::get<0>(r), py::str(std::get<1>(r)), py::bytes(std::get<2>(r)));
           }, py::arg("path"), py::arg("payload"), py::arg("timeout_ms") = 0)
      .def("close", &FrameRpcClient::close, G());
  bind_data_path(m);

  // ---- codecs / kernels ------------------------------------------------------------------
  m.def("device_count", &hip_device_count);

  // ---- HIP IPC (short-circuit device reads) -------------------------------------------------
  m.def("ipc_export", [](uint64_t ptr) {
          IpcExport e = ipc_export(ptr);
          return py::make_tuple(py::bytes(e.handle), e.offset, e.alloc_bytes);
        }, py::arg("ptr"));
  m.def("ipc_open", [](py::bytes handle, int device) {
          std::string h = handle;
          py::gil_scoped_release rel;
          return ipc_open(h, device);
        }, py::arg("handle"), py::arg("device"));
  m.def("ipc_open_bounded", [](py::bytes handle, int device, int timeout_ms) {
          std::string h = handle;
          py::gil_scoped_release rel;
          return ipc_open_bounded(h, device, timeout_ms);
        }, py::arg("handle"), py::arg("device"), py::arg("timeout_ms"));
  py::register_exception<IpcTimeout>(m, "IpcTimeout", PyExc_TimeoutError);
  m.def("ipc_close", [](uint64_t base) { py::gil_scoped_release rel; ipc_close(base); });
  m.def("gpu_numa_node", &gpu_numa_node, py::arg("device"));
  m.def("process_placement", &process_placement);
  m.def("device_arena_alloc", [](uint64_t bytes, int device) {
          py::gil_scoped_release rel;
          return device_arena_alloc(bytes, device);
        }, py::arg("bytes"), py::arg("device"));
  m.def("device_arena_free", [](uint64_t ptr, int device) {
          py::gil_scoped_release rel;
          device_arena_free(ptr, device);
        }, py::arg("ptr"), py::arg("device"));
  m.def("enable_peer_access", &enable_peer_access, py::arg("device"), py::arg("peer"));
  // page-lock an existing host mapping (shared-memory DRAM arenas) so kernels can read it
  m.def("host_register", [](uint64_t ptr, uint64_t n) {
          if (hip_device_count() == 0) return false;
          HIP_CHECK(hipHostRegister(reinterpret_cast<void*>(ptr), n, hipHostRegisterMapped));
          return true;
        }, py::arg("ptr"), py::arg("nbytes"));
  m.def("host_unregister", [](uint64_t ptr) {
          if (hip_device_count() > 0) (void)hipHostUnregister(reinterpret_cast<void*>(ptr));
        }, py::arg("ptr"));
  m.def("can_access_peer", &can_access_peer, py::arg("device"), py::arg("peer"));
  m.def("crc32c", [](py::buffer data, uint32_t crc) {      // zero-copy over any buffer
          py::buffer_info bi = data.request();
          const size_t n = static_cast<size_t>(bi.size) * bi.itemsize;
          py::gil_scoped_release rel;
          return crc32c_sw(bi.ptr, n, crc);
        }, py::arg("data"), py::arg("crc") = 0);
  m.def("crc32c_ptr", [](uint64_t ptr, uint64_t n, uint32_t crc) {
          py::gil_scoped_release rel;
          return crc32c_sw(reinterpret_cast<const void*>(ptr), n, crc);
        }, py::arg("ptr"), py::arg("n"), py::arg("crc") = 0);
  // HDFS data-transfer checksums: one big-endian CRC32C per bytes_per_checksum chunk (the last
  // chunk may be short), the layout a DataTransferProtocol packet carries before its data
  m.def("crc32c_chunks", [](py::buffer data, uint32_t bpc) {
          py::buffer_info bi = data.request();
          const auto* p = static_cast<const uint8_t*>(bi.ptr);
          const size_t n = static_cast<size_t>(bi.size) * bi.itemsize;
          if (bpc == 0) throw StoreError(kErrInvalidArgument, "bytes_per_checksum must be > 0");
          const size_t nc = (n + bpc - 1) / bpc;
          std::string out(nc * 4, '\0');
          {
            py::gil_scoped_release rel;
            for (size_t i = 0; i < nc; ++i) {
              const size_t off = i * bpc;
              const uint32_t c = crc32c_sw(p + off, std::min<size_t>(bpc, n - off), 0);
              out[4 * i] = char(c >> 24); out[4 * i + 1] = char(c >> 16);
              out[4 * i + 2] = char(c >> 8); out[4 * i + 3] = char(c);
            }
          }
          return py::bytes(out);
        }, py::arg("data"), py::arg("bytes_per_checksum") = 512);
  m.def("crc32c_combine", &crc32c_combine);
  m.def("crc32c_device_pages", &crc32c_device_pages, G(), py::arg("base"), py::arg("pages"), py::arg("length"),
        py::arg("page_bytes"));
  m.def("crc32c_device", &crc32c_device, G(), py::arg("ptr"), py::arg("length"), py::arg("piece") = 0,
        py::arg("stream") = 0);
  m.def("lz4_compress", [](py::bytes data) {
          std::string s = data;
          std::string out(lz4_compress_bound(s.size()), '\0');
          int64_t n;
          {
            py::gil_scoped_release rel;
            n = lz4_compress_block((const uint8_t*)s.data(), s.size(), (uint8_t*)&out[0], out.size());
          }
          if (n < 0) throw StoreError(kErrInvalidArgument, "lz4 compression failed");
          out.resize((size_t)n);
          return py::bytes(out);
        });
  m.def("lz4_decompress", [](py::bytes data, size_t capacity) {
          std::string s = data;
          std::string out(capacity, '\0');
          int64_t n;
          {
            py::gil_scoped_release rel;
            n = lz4_decompress_block((const uint8_t*)s.data(), s.size(), (uint8_t*)&out[0], out.size());
          }
          if (n < 0) throw StoreError(kErrInvalidArgument, "malformed lz4 block (" + std::to_string(n) + ")");
          out.resize((size_t)n);
          return py::bytes(out);
        });
  m.def("lz4_compress_bound", &lz4_compress_bound);
  m.def("trace_push", [](const std::string& name) { roctxRangePushA(name.c_str()); }, py::arg("name"));
  m.def("trace_pop", [] { roctxRangePop(); });
  m.def("trace_mark", [](const std::string& name) { roctxMarkA(name.c_str()); }, py::arg("name"));
  m.def("lz4_device", &lz4_device, G(), py::arg("chunks"), py::arg("compress"), py::arg("stream") = 0);
  m.def("lz4_device_kernel_ms", &lz4_device_kernel_ms, G(), py::arg("chunks"), py::arg("compress"),
        py::arg("reps") = 5);
  m.def("batched_copy", &batched_copy, G(), py::arg("segments"), py::arg("stream") = 0, py::arg("sync") = true);
  m.def("fill_pattern", [](uint64_t ptr, uint64_t bytes, uint64_t seed, uint64_t word_offset, uint64_t stream) {
          py::gil_scoped_release rel;
          HIP_CHECK(launch_fill_pattern(reinterpret_cast<uint8_t*>(ptr), bytes, seed, word_offset,
                                        reinterpret_cast<hipStream_t>(stream)));
        }, py::arg("ptr"), py::arg("bytes"), py::arg("seed"), py::arg("word_offset") = 0, py::arg("stream") = 0);
  m.def("evict_select_device", &evict_select_device);
  m.def("page_alloc_device", &page_alloc_device);
  m.def("set_copy_variant", &set_copy_variant, py::arg("variant"), py::arg("grid_cap") = 0);
  m.def("set_crc_variant", &set_crc_variant, py::arg("variant"));
  m.def("set_lz4_decode_variant", &set_lz4_decode_variant, py::arg("variant"));
  m.def("set_lz4_encode_variant", &set_lz4_encode_variant, py::arg("variant"));
  m.def("set_seq_read_variant", &set_seq_read_variant, py::arg("variant"), py::arg("grid_cap") = 0);
  m.def("set_page_gather_chunk_variant", &set_page_gather_chunk_variant, py::arg("variant"));
  m.attr("COPY_CHUNK") = kCopyChunk;
}
