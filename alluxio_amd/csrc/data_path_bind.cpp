// pybind11 bindings of the host-reader data path: block sources, the chunk-buffered HostInStream
// (with a raw vectorcall readinto for the per-call hot path) and the native block data server.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <pthread.h>

#include <condition_variable>
#include <cstddef>
#include <deque>
#include <functional>
#include <future>
#include <mutex>
#include <thread>

#include "block_source.h"
#include "data_server.h"
#include "stress_bench.h"
#include "hdfs_packets.h"
#include "frame_rpc.h"

namespace py = pybind11;
using namespace amdx;

namespace {

// Helper threads of sink_write_pair (immortal: a call blocked on a slow peer never blocks exit).
class PairPool {
 public:
  static PairPool& get() {
    static PairPool* p = new PairPool(16);
    return *p;
  }
  std::future<void> run(std::function<void()> f) {
    auto task = std::make_shared<std::packaged_task<void()>>(std::move(f));
    std::future<void> fut = task->get_future();
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back([task] { (*task)(); });
    }
    cv_.notify_one();
    return fut;
  }

 private:
  explicit PairPool(int n) {
    for (int i = 0; i < n; ++i)
      std::thread([this] {
        pthread_setname_np(pthread_self(), "sink-pair");
        for (;;) {
          std::function<void()> f;
          {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return !q_.empty(); });
            f = std::move(q_.front());
            q_.pop_front();
          }
          f();
        }
      }).detach();
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
};

PyObject* g_store_error = nullptr;   // alluxio_amd._C.StoreError

void set_store_error(int code, const char* msg) {
  if (!g_store_error) {
    PyErr_SetString(PyExc_RuntimeError, msg);
    return;
  }
  PyObject* inst = PyObject_CallFunction(g_store_error, "is", code, msg);
  if (inst) {
    PyErr_SetObject(g_store_error, inst);
    Py_DECREF(inst);
  }
}

// A Python BlockReader (UFS streams, fallbacks): read_into(offset, length, ptr, HOST) with the GIL.
class PySource : public BlockSource {
 public:
  PySource(py::object reader, uint64_t length) : BlockSource(length), reader_(std::move(reader)) {}
  ~PySource() override {
    py::gil_scoped_acquire g;
    reader_ = py::object();
  }
  void read(uint64_t off, uint64_t n, uint8_t* dst) override {
    py::gil_scoped_acquire g;
    reader_.attr("read_into")(off, n, reinterpret_cast<uint64_t>(dst), 0);
  }
  bool needs_gil() const override { return true; }

 private:
  py::object reader_;
};

// FileInStream's native core: `opener(block_index, failed)` returns the BlockSource of a block
// (failed=True: the previous source of that block broke; pick another location).
struct PyInStream {
  HostInStream s;
  py::object opener;
  bool closed = false;
  PyInStream(uint64_t length, uint64_t block_size, uint64_t chunk, py::object op, bool prefetch)
      : s(length, block_size, chunk, prefetch), opener(std::move(op)) {}

  // The next block's source, opened and started while a read that runs into it still reads the
  // current block (network sources: its ReadBlock request is out, so its first bytes -- and for a
  // cold block the worker's first UFS reads -- are under way when the reader gets there).
  int64_t next_idx = -1;
  std::shared_ptr<BlockSource> next_src;
  bool start_next_enabled = false;   // alluxio.user.native.reader.next.block.start.enabled

  void open_block(int64_t idx, bool failed) {
    if (!failed && idx == next_idx && next_src) {
      s.set_source(idx, std::move(next_src));
      next_idx = -1;
      return;
    }
    next_src.reset();
    next_idx = -1;
    py::object src = opener(idx, failed);
    s.set_source(idx, src.cast<std::shared_ptr<BlockSource>>());
  }

  // A read continuing past block idx: open and start idx + 1 now (best effort: a failure here is
  // left to the read of that block, which opens it again).
  void start_next(int64_t idx, uint64_t read_end) {
    const int64_t nx = idx + 1;
    if (!start_next_enabled || nx == next_idx || read_end <= (uint64_t)nx * s.block_size() || (uint64_t)nx * s.block_size() >= s.length())
      return;
    if (!s.source() || !s.source()->waits_on_network()) return;
    try {
      py::object src = opener(nx, false);
      auto bs = src.cast<std::shared_ptr<BlockSource>>();
      if (!bs->waits_on_network()) return;
      {
        py::gil_scoped_release rel;
        bs->start();
      }
      next_src = std::move(bs);
      next_idx = nx;
    } catch (const std::exception&) {
      next_src.reset();
      next_idx = -1;
    }
  }

  // Reads exactly n bytes at pos() (n <= bytes left); the GIL is held on entry.
  void read(uint8_t* dst, uint64_t n) {
    if (closed) throw py::value_error("I/O operation on closed file");
    uint64_t done = 0;
    int failures = 0;
    const uint64_t read_end = s.pos() + n;
    while (done < n) {
      const int64_t idx = (int64_t)(s.pos() / s.block_size());
      if (s.block_index() != idx || !s.source()) open_block(idx, false);
      start_next(idx, read_end);
      // what the current chunk (or the completed prefetch of the next) holds: no GIL release
      const uint64_t have = s.copy_buffered(dst + done, n - done);
      if (have) {
        done += have;
        continue;
      }
      try {
        uint64_t got;
        // refills release the GIL (holding it was measured slower at 16-256 threads:
        // profiles/r4_worker_bench_host_gil_hold.jsonl)
        if (s.source()->needs_gil()) {
          got = s.read_block_part(dst + done, n - done);
        } else {
          py::gil_scoped_release rel;
          got = s.read_block_part(dst + done, n - done);
        }
        done += got;
        failures = 0;
      } catch (const StoreError& e) {
        if (e.code == kErrInvalidArgument || e.code == kErrInvalidState || ++failures > 2) throw;
        s.drop_source();
        open_block(idx, true);   // another location of the block, or the UFS
      } catch (const std::runtime_error& e) {
        if (++failures > 2) throw StoreError(kErrIo, e.what());
        s.drop_source();
        open_block(idx, true);
      }
    }
  }

  uint64_t clamp(uint64_t n) const {
    const uint64_t left = s.length() - std::min(s.pos(), s.length());
    return n < left ? n : left;
  }

  void close() {
    closed = true;
    s.drop_source();
    next_src.reset();
    next_idx = -1;
  }
};

// ---- raw vectorcall readinto: the per-call path of StressWorkerBench's read(buf) loop ---------
struct FastRead {
  PyObject_HEAD
  vectorcallfunc vc;
  PyInStream* s;
  PyObject* owner;   // the HostInStream Python object (keeps `s` alive)
};

PyObject* fast_readinto(PyObject* self, PyObject* const* args, size_t nargsf, PyObject* kwnames) {
  FastRead* f = reinterpret_cast<FastRead*>(self);
  if (PyVectorcall_NARGS(nargsf) != 1 || (kwnames && PyTuple_GET_SIZE(kwnames))) {
    PyErr_SetString(PyExc_TypeError, "readinto(buffer) takes exactly one buffer");
    return nullptr;
  }
  PyInStream& s = *f->s;
  if (s.closed) {
    PyErr_SetString(PyExc_ValueError, "I/O operation on closed file");
    return nullptr;
  }
  Py_buffer v;
  if (PyObject_GetBuffer(args[0], &v, PyBUF_WRITABLE) < 0) return nullptr;
  const uint64_t n = s.clamp((uint64_t)v.len);
  if (n == 0 || s.s.fast(static_cast<uint8_t*>(v.buf), n)) {
    PyBuffer_Release(&v);
    return PyLong_FromUnsignedLongLong(n);
  }
  PyObject* r = nullptr;
  try {
    s.read(static_cast<uint8_t*>(v.buf), n);
    r = PyLong_FromUnsignedLongLong(n);
  } catch (py::error_already_set& e) {
    e.restore();
  } catch (const py::builtin_exception& e) {
    e.set_error();
  } catch (const StoreError& e) {
    set_store_error(e.code, e.what());
  } catch (const std::exception& e) {
    set_store_error(kErrIo, e.what());
  }
  PyBuffer_Release(&v);
  return r;
}

void fast_dealloc(PyObject* self) {
  Py_XDECREF(reinterpret_cast<FastRead*>(self)->owner);
  PyObject_Del(self);
}

PyTypeObject g_fast_type = {PyVarObject_HEAD_INIT(nullptr, 0)};

}  // namespace

void bind_data_path(py::module_& m) {
  g_store_error = m.attr("StoreError").ptr();
  Py_INCREF(g_store_error);

  g_fast_type.tp_name = "alluxio_amd._C.FastReadInto";
  g_fast_type.tp_basicsize = sizeof(FastRead);
  g_fast_type.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_VECTORCALL;
  g_fast_type.tp_vectorcall_offset = offsetof(FastRead, vc);
  g_fast_type.tp_call = PyVectorcall_Call;
  g_fast_type.tp_dealloc = fast_dealloc;
  g_fast_type.tp_doc = "readinto(buffer) -> bytes read (HostInStream fast path)";
  if (PyType_Ready(&g_fast_type) < 0) throw py::error_already_set();

  using G = py::call_guard<py::gil_scoped_release>;
  py::class_<BlockSource, std::shared_ptr<BlockSource>>(m, "BlockSource")
      .def_property_readonly("length", &BlockSource::length)
      .def_property_readonly("direct", &BlockSource::direct)
      .def("read_into", [](BlockSource& s, uint64_t off, uint64_t n, uint64_t ptr) {
             if (s.needs_gil()) {
               s.read(off, n, reinterpret_cast<uint8_t*>(ptr));
               return;
             }
             py::gil_scoped_release rel;
             s.read(off, n, reinterpret_cast<uint8_t*>(ptr));
           }, py::arg("offset"), py::arg("length"), py::arg("ptr"))
      .def("close", &BlockSource::close);
  py::class_<DeviceArenaSource, BlockSource, std::shared_ptr<DeviceArenaSource>>(m, "DeviceArenaSource")
      .def(py::init<uint64_t, std::vector<int64_t>, uint64_t, uint64_t, int>(), py::arg("base"), py::arg("pages"),
           py::arg("page_size"), py::arg("length"), py::arg("device"));
  py::class_<HostArenaSource, BlockSource, std::shared_ptr<HostArenaSource>>(m, "HostArenaSource")
      .def(py::init<uint64_t, std::vector<int64_t>, uint64_t, uint64_t>(), py::arg("base"), py::arg("pages"),
           py::arg("page_size"), py::arg("length"));
  py::class_<StoreSource, BlockSource, std::shared_ptr<StoreSource>>(m, "StoreSource")
      .def(py::init<BlockStore*, int64_t, uint64_t, bool>(), py::arg("store"), py::arg("block_id"), py::arg("length"),
           py::arg("device_tier"), py::keep_alive<1, 2>())
      .def_property_readonly("bytes", &StoreSource::bytes);
  py::class_<GrpcBlockSource, BlockSource, std::shared_ptr<GrpcBlockSource>>(m, "GrpcBlockSource")
      .def(py::init([](const std::string& host, int port, int64_t block_id, uint64_t length, uint64_t chunk,
                       py::bytes ufs_options, bool promote, const std::string& channel_id, const std::string& user,
                       int timeout_ms, const std::string& unix_path) {
             GrpcBlockSource::Options o;
             o.host = host;
             o.port = port;
             o.unix_path = unix_path;
             o.block_id = block_id;
             o.chunk = chunk ? chunk : (1u << 20);
             o.ufs_options = ufs_options;
             o.promote = promote;
             o.channel_id = channel_id;
             o.user = user;
             o.timeout_ms = timeout_ms;
             py::gil_scoped_release rel;
             try {
               return std::make_shared<GrpcBlockSource>(std::move(o), length);
             } catch (const StoreError&) {
               throw;
             } catch (const std::exception& e) {
               throw StoreError(kErrIo, e.what());
             }
           }),
           py::arg("host"), py::arg("port"), py::arg("block_id"), py::arg("length"), py::arg("chunk") = 1u << 20,
           py::arg("ufs_options") = py::bytes(), py::arg("promote") = false, py::arg("channel_id") = "",
           py::arg("user") = "", py::arg("timeout_ms") = 60000, py::arg("unix_path") = "");
  m.def("source_read", [](std::shared_ptr<BlockSource> src, uint64_t off, uint64_t n, uint64_t ptr, int kind,
                          int device) {
          if (src->needs_gil()) throw std::runtime_error("source_read needs a native source");
          py::gil_scoped_release rel;
          try {
            if (kind == (int)MemKind::kDevice)
              source_read_to_device(*src, off, n, reinterpret_cast<uint8_t*>(ptr), device);
            else
              src->read(off, n, reinterpret_cast<uint8_t*>(ptr));
          } catch (const StoreError&) {
            throw;
          } catch (const std::exception& e) {
            throw StoreError(kErrIo, e.what());
          }
        }, py::arg("source"), py::arg("offset"), py::arg("length"), py::arg("ptr"), py::arg("kind"),
        py::arg("device") = 0);
  py::class_<ArenaSink, std::shared_ptr<ArenaSink>>(m, "ArenaSink")
      .def(py::init<uint64_t, std::vector<int64_t>, uint64_t, uint64_t, int, bool>(), py::arg("base"),
           py::arg("pages"), py::arg("page_size"), py::arg("capacity"), py::arg("device"), py::arg("host_arena"))
      .def("write_ptr", [](ArenaSink& s, uint64_t off, uint64_t ptr, uint64_t n) {
             py::gil_scoped_release rel;
             s.write(off, reinterpret_cast<const uint8_t*>(ptr), n);
           }, py::arg("offset"), py::arg("ptr"), py::arg("n"))
      .def_property_readonly("length", &ArenaSink::length);
  py::class_<GrpcBlockSink, std::shared_ptr<GrpcBlockSink>>(m, "GrpcBlockSink")
      .def(py::init([](const std::string& host, int port, int64_t block_id, int tier, const std::string& medium,
                       uint64_t reserve, bool pin, uint64_t chunk, const std::string& channel_id,
                       const std::string& user, int timeout_ms, const std::string& unix_path,
                       const py::bytes& command) {
             GrpcBlockSink::Options o;
             o.host = host;
             o.port = port;
             o.unix_path = unix_path;
             o.block_id = block_id;
             o.tier = tier;
             o.medium = medium;
             o.reserve = reserve ? reserve : (1u << 20);
             o.pin = pin;
             o.chunk = chunk ? chunk : (1u << 20);
             o.channel_id = channel_id;
             o.user = user;
             o.timeout_ms = timeout_ms;
             o.command = command;
             py::gil_scoped_release rel;
             try {
               return std::make_shared<GrpcBlockSink>(std::move(o));
             } catch (const StoreError&) {
               throw;
             } catch (const std::exception& e) {
               throw StoreError(kErrIo, e.what());
             }
           }),
           py::arg("host"), py::arg("port"), py::arg("block_id"), py::arg("tier") = 0, py::arg("medium") = "",
           py::arg("reserve") = 1u << 20, py::arg("pin") = false, py::arg("chunk") = 1u << 20,
           py::arg("channel_id") = "", py::arg("user") = "", py::arg("timeout_ms") = 60000,
           py::arg("unix_path") = "", py::arg("command") = py::bytes(""))
      .def("write_ptr", [](GrpcBlockSink& s, uint64_t ptr, uint64_t n) {
             py::gil_scoped_release rel;
             try {
               s.write(reinterpret_cast<const uint8_t*>(ptr), n);
             } catch (const StoreError&) {
               throw;
             } catch (const std::exception& e) {
               throw StoreError(kErrIo, e.what());
             }
           }, py::arg("ptr"), py::arg("n"))
      .def("append_block", [](GrpcBlockSink& s, int64_t block_id, uint64_t length) {
             py::gil_scoped_release rel;
             try {
               s.append_block(block_id, length);
             } catch (const StoreError&) {
               throw;
             } catch (const std::exception& e) {
               throw StoreError(kErrIo, e.what());
             }
           }, py::arg("block_id"), py::arg("length"))
      .def("commit", [](GrpcBlockSink& s, bool hold_for_append) {
             py::gil_scoped_release rel;
             try {
               return s.commit(hold_for_append);
             } catch (const StoreError&) {
               throw;
             } catch (const std::exception& e) {
               throw StoreError(kErrIo, e.what());
             }
           }, py::arg("hold_for_append") = false)
      .def("cancel", [](GrpcBlockSink& s) {
             py::gil_scoped_release rel;
             s.cancel();
           })
      .def_property_readonly("written", &GrpcBlockSink::written);
  // CACHE_THROUGH: the same bytes to the cache-tier block stream and the UFS stream at once, one
  // GIL release for both (the second sink's write runs on a pooled helper thread)
  m.def("sink_write_pair", [](GrpcBlockSink& a, GrpcBlockSink& b, uint64_t ptr, uint64_t n) {
        py::gil_scoped_release rel;
        const uint8_t* p = reinterpret_cast<const uint8_t*>(ptr);
        auto fut = PairPool::get().run([&b, p, n] { b.write(p, n); });
        std::exception_ptr ea;
        try {
          a.write(p, n);
        } catch (...) {
          ea = std::current_exception();
        }
        std::exception_ptr eb;
        try {
          fut.get();
        } catch (...) {
          eb = std::current_exception();
        }
        for (auto e : {ea, eb}) {
          if (!e) continue;
          try {
            std::rethrow_exception(e);
          } catch (const StoreError&) {
            throw;
          } catch (const std::exception& x) {
            throw StoreError(kErrIo, x.what());
          }
        }
      }, py::arg("a"), py::arg("b"), py::arg("ptr"), py::arg("n"));
  py::class_<PySource, BlockSource, std::shared_ptr<PySource>>(m, "PySource")
      .def(py::init<py::object, uint64_t>(), py::arg("reader"), py::arg("length"));

  py::class_<PyInStream>(m, "HostInStream")
      .def(py::init([](uint64_t length, uint64_t block_size, uint64_t chunk, py::object opener, bool prefetch,
                       bool start_next) {
             auto p = std::make_unique<PyInStream>(length, block_size, chunk, std::move(opener), prefetch);
             p->start_next_enabled = start_next;
             return p;
           }),
           py::arg("length"), py::arg("block_size"), py::arg("chunk"), py::arg("opener"), py::arg("prefetch") = true,
           py::arg("start_next") = false)
      .def_property("pos", [](const PyInStream& s) { return s.s.pos(); },
                    [](PyInStream& s, uint64_t p) { s.s.seek(p); })
      .def_property_readonly("length", [](const PyInStream& s) { return s.s.length(); })
      .def_property_readonly("bytes_read", [](const PyInStream& s) { return s.s.bytes(); })
      .def_property_readonly("refills", [](const PyInStream& s) { return s.s.refills(); })
      .def_property_readonly("prefetch_hits", [](const PyInStream& s) { return s.s.prefetch_hits(); })
      .def_property_readonly("closed", [](const PyInStream& s) { return s.closed; })
      .def("readinto", [](PyInStream& s, py::buffer b) {
             py::buffer_info bi = b.request(true);
             const uint64_t n = s.clamp((uint64_t)(bi.size * bi.itemsize));
             if (n && !s.s.fast(static_cast<uint8_t*>(bi.ptr), n)) s.read(static_cast<uint8_t*>(bi.ptr), n);
             return n;
           })
      .def("read_ptr", [](PyInStream& s, uint64_t ptr, uint64_t n) {
             n = s.clamp(n);
             if (n && !s.s.fast(reinterpret_cast<uint8_t*>(ptr), n)) s.read(reinterpret_cast<uint8_t*>(ptr), n);
             return n;
           }, py::arg("ptr"), py::arg("n"))
      .def("read", [](PyInStream& s, int64_t size) {
             const uint64_t n = s.clamp(size < 0 ? UINT64_MAX : (uint64_t)size);
             PyObject* out = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)n);
             if (!out) throw py::error_already_set();
             py::bytes b = py::reinterpret_steal<py::bytes>(out);
             uint8_t* dst = reinterpret_cast<uint8_t*>(PyBytes_AS_STRING(out));
             if (n && !s.s.fast(dst, n)) s.read(dst, n);
             return b;
           }, py::arg("size") = -1)
      .def("close", &PyInStream::close)
      // A callable readinto(buffer) that skips pybind11's dispatcher: FileInStream binds it as
      // its instance's readinto.
      .def_property_readonly("fast_readinto", [](py::object self) {
             FastRead* f = PyObject_New(FastRead, &g_fast_type);
             if (!f) throw py::error_already_set();
             f->vc = fast_readinto;
             f->s = self.cast<PyInStream*>();
             f->owner = self.ptr();
             Py_INCREF(f->owner);
             return py::reinterpret_steal<py::object>(reinterpret_cast<PyObject*>(f));
           });

  // ---- native data server + streaming bridge of the HTTP/2 front end ------------------------
  py::class_<DataServerStats, std::shared_ptr<DataServerStats>>(m, "DataServerStats")
      .def(py::init<>())
      .def_property_readonly("streams", [](const DataServerStats& s) { return s.streams.load(); })
      .def_property_readonly("declined", [](const DataServerStats& s) { return s.declined.load(); })
      .def_property_readonly("bytes", [](const DataServerStats& s) { return s.bytes.load(); })
      .def_property_readonly("domain_bytes", [](const DataServerStats& s) { return s.domain_bytes.load(); })
      .def_property_readonly("chunks", [](const DataServerStats& s) { return s.chunks.load(); })
      .def_property_readonly("staged_bytes", [](const DataServerStats& s) { return s.staged_bytes.load(); })
      .def_property_readonly("write_streams", [](const DataServerStats& s) { return s.write_streams.load(); })
      .def_property_readonly("write_declined", [](const DataServerStats& s) { return s.write_declined.load(); })
      .def_property_readonly("write_bytes", [](const DataServerStats& s) { return s.write_bytes.load(); })
      .def_property_readonly("write_evict_waits", [](const DataServerStats& s) { return s.write_evict_waits.load(); })
      .def_property_readonly("ufs_write_streams", [](const DataServerStats& s) { return s.ufs_write_streams.load(); })
      .def_property_readonly("ufs_write_bytes", [](const DataServerStats& s) { return s.ufs_write_bytes.load(); })
      .def_property_readonly("cold_streams", [](const DataServerStats& s) { return s.cold_streams.load(); })
      .def_property_readonly("cold_cached", [](const DataServerStats& s) { return s.cold_cached.load(); })
      .def_property_readonly("cold_aborted", [](const DataServerStats& s) { return s.cold_aborted.load(); })
      .def_property_readonly("cold_bytes", [](const DataServerStats& s) { return s.cold_bytes.load(); })
      .def_property_readonly("cold_active", [](const DataServerStats& s) { return s.cold_active.load(); })
      .def_property_readonly("store_tasks", [](const DataServerStats& s) { return s.store_tasks.load(); })
      .def_property_readonly("prefetched", [](const DataServerStats& s) { return s.prefetched.load(); })
      .def_property_readonly("promoted", [](const DataServerStats& s) { return s.promoted.load(); })
      .def_property_readonly("zero_copy_frames", [](const DataServerStats& s) { return s.zero_copy_frames.load(); })
      .def_property_readonly("ufs_tee_bytes", [](const DataServerStats& s) { return s.ufs_tee_bytes.load(); })
      .def_property_readonly("commits", [](const DataServerStats& s) { return s.commits.load(); })
      .def_property_readonly("commit_batches", [](const DataServerStats& s) { return s.commit_batches.load(); })
      .def_property_readonly("commit_failures", [](const DataServerStats& s) { return s.commit_failures.load(); })
      .def_property_readonly("crc_streamed", [](const DataServerStats& s) { return s.crc_streamed.load(); })
      .def_property_readonly("send_timing", [](const DataServerStats& s) {
        py::dict out;
        const char* names[2] = {"cached", "cold"};
        for (int k = 0; k < 2; ++k) {
          const auto& t = s.send[k];
          py::dict d;
          d["streams"] = t.streams.load();
          d["life_ns"] = t.life_ns.load();
          d["first_ns"] = t.first_ns.load();
          d["window_stalls"] = t.window_stalls.load();
          d["window_ns"] = t.window_ns.load();
          d["data_stalls"] = t.data_stalls.load();
          d["data_ns"] = t.data_ns.load();
          out[names[k]] = d;
        }
        return out;
      })
      .def_property_readonly("cold_timing_ns", [](const DataServerStats& s) {
        py::dict d;
        d["queue"] = s.cold_queue_ns.load();
        d["setup"] = s.cold_setup_ns.load();
        d["first_slot"] = s.cold_first_ns.load();
        d["ufs_read"] = s.cold_read_ns.load();
        d["slot_wait"] = s.cold_slot_wait_ns.load();
        d["dma_wait"] = s.cold_dma_wait_ns.load();
        d["device"] = s.cold_device_ns.load();
        d["slot_alloc"] = s.cold_slot_alloc_ns.load();
        d["first_read"] = s.cold_first_read_ns.load();
        return d;
      })
      .def_property_readonly("cold_readahead_bytes", [](const DataServerStats& s) { return s.cold_readahead_bytes.load(); })
      .def_property_readonly("cold_readahead_hits", [](const DataServerStats& s) { return s.cold_readahead_hits.load(); })
      .def("stop_background_reads", [](DataServerStats& s) { s.stopping.store(true); });
  py::class_<BlockCommitter, std::shared_ptr<BlockCommitter>>(m, "BlockCommitter")
      .def(py::init<std::shared_ptr<BlockStore>, uint32_t, bool, bool, std::shared_ptr<DataServerStats>>(),
           py::arg("store"), py::arg("method"), py::arg("crc_device"), py::arg("crc_host"), py::arg("stats"));
  m.def("thread_streams_created", &thread_streams_created);
  m.def("unlink_deferred", [](const std::string& path, uint64_t defer_bytes, size_t max_pending) {
        py::gil_scoped_release nogil;
        return unlink_deferred(path, defer_bytes, max_pending);
      }, py::arg("path"), py::arg("defer_bytes") = 8u << 20, py::arg("max_pending") = 256);
  m.def("reclaimed_files", &reclaimed_files);
  m.def("reclaim_pending", &reclaim_pending);
  // Native StressWorkerBench client (csrc/stress_bench.h): `blocks` = one dict per block of the
  // file: {"length", "kind": "grpc"|"ipc"|"host", grpc: "host", "port", "unix_path", "block_id",
  // "chunk", "channel_id", "user", "timeout_ms"; arenas: "base", "pages", "page_size", "device"}.
  m.def("run_stress_reads", [](py::list blocks, uint64_t block_size, int threads, uint64_t buffer, uint64_t chunk,
                               double warmup_s, double duration_s, bool prefetch) {
          std::vector<BenchBlock> bs;
          for (py::handle h : blocks) {
            py::dict d = py::reinterpret_borrow<py::dict>(h);
            BenchBlock b;
            b.length = d["length"].cast<uint64_t>();
            const std::string kind = d["kind"].cast<std::string>();
            b.kind = kind == "ipc" ? 1 : kind == "host" ? 2 : 0;
            if (b.kind == 0) {
              b.grpc.host = d["host"].cast<std::string>();
              b.grpc.port = d["port"].cast<int>();
              b.grpc.unix_path = d.contains("unix_path") ? d["unix_path"].cast<std::string>() : "";
              b.grpc.block_id = d["block_id"].cast<int64_t>();
              b.grpc.chunk = d.contains("chunk") ? d["chunk"].cast<uint64_t>() : (1u << 20);
              b.grpc.channel_id = d.contains("channel_id") ? d["channel_id"].cast<std::string>() : "";
              b.grpc.user = d.contains("user") ? d["user"].cast<std::string>() : "";
              b.grpc.timeout_ms = d.contains("timeout_ms") ? d["timeout_ms"].cast<int>() : 60000;
            } else {
              b.base = d["base"].cast<uint64_t>();
              b.pages = d["pages"].cast<std::vector<int64_t>>();
              b.page_size = d["page_size"].cast<uint64_t>();
              b.device = d.contains("device") ? d["device"].cast<int>() : 0;
            }
            bs.push_back(std::move(b));
          }
          BenchResult r;
          {
            py::gil_scoped_release rel;
            r = run_stress_reads(bs, block_size, threads, buffer, chunk, warmup_s, duration_s, prefetch);
          }
          py::dict out;
          out["bytes"] = r.bytes;
          out["reads"] = r.reads;
          out["opens"] = r.opens;
          out["block_opens"] = r.block_opens;
          out["seconds"] = r.seconds;
          out["per_thread"] = r.per_thread;
          out["errors"] = r.errors;
          return out;
        }, py::arg("blocks"), py::arg("block_size"), py::arg("threads"), py::arg("buffer"), py::arg("chunk"),
        py::arg("warmup_s"), py::arg("duration_s"), py::arg("prefetch") = true);
  auto mounts = py::class_<UfsMounts, std::shared_ptr<UfsMounts>>(m, "UfsMounts")
      .def(py::init<>())
      .def("set", &UfsMounts::set, py::arg("mount_id"), py::arg("root"))
      .def("set_s3",
           [](UfsMounts& u, int64_t mount_id, const std::string& host, int port, const std::string& bucket,
              const std::string& ak, const std::string& sk, const std::string& region, int parallel, uint64_t part,
              uint64_t upload_part, int upload_inflight, int connect_timeout_ms, int socket_timeout_ms,
              int request_timeout_ms, int max_retries) {
             HttpOptions o;
             o.connect_timeout_ms = connect_timeout_ms;
             o.socket_timeout_ms = socket_timeout_ms;
             o.request_timeout_ms = request_timeout_ms;
             o.max_retries = std::max(0, max_retries);
             u.set_s3(mount_id, host, port, bucket, ak, sk, region, parallel, part, upload_part, upload_inflight, o);
           },
           py::arg("mount_id"), py::arg("host"), py::arg("port"), py::arg("bucket"),
           py::arg("access_key"), py::arg("secret_key"), py::arg("region"), py::arg("parallel"), py::arg("part"),
           py::arg("upload_part") = 64u << 20, py::arg("upload_inflight") = 4, py::arg("connect_timeout_ms") = 10000,
           py::arg("socket_timeout_ms") = 50000, py::arg("request_timeout_ms") = 60000, py::arg("max_retries") = 3)
      .def("remove", &UfsMounts::remove, py::arg("mount_id"))
      .def("__len__", &UfsMounts::size)
      .def("resolve", [](const UfsMounts& r, int64_t mount_id, const std::string& path) -> py::object {
             std::string local;
             if (!r.resolve(mount_id, path, &local)) return py::none();
             return py::str(local);
           })
      .def("resolve_s3", [](const UfsMounts& r, int64_t mount_id, const std::string& path) -> py::object {
             std::shared_ptr<const S3Mount> mt;
             std::string key;
             if (!r.resolve_s3(mount_id, path, &mt, &key)) return py::none();
             return py::make_tuple(mt->bucket, key);
           });
  m.attr("LocalUfsRoots") = mounts;
  m.def("sigv4_headers", [](const std::string& host_header, const std::string& access, const std::string& secret,
                            const std::string& region, const std::string& method, const std::string& path,
                            const std::string& query, const std::string& payload_hash, const std::string& amz_date) {
          S3Credentials c;
          c.host_header = host_header;
          c.access_key = access;
          c.secret_key = secret;
          c.region = region;
          return s3_header_lines(c, method, path, query, payload_hash, amz_date);
        });
  m.def("sha256_hex", [](py::bytes b) {
          std::string v = b;
          return sha256_hex(v.data(), v.size());
        });
  m.def("serve_block_reads", [](FrameRpcServer& srv, uint32_t method, std::shared_ptr<BlockStore> store, uint64_t max_chunk,
                                uint64_t window, std::shared_ptr<UfsMounts> mounts, uint32_t commit_method,
                                uint64_t ufs_slot_bytes, int ufs_depth, int ufs_max_active,
                                std::shared_ptr<DataServerStats> stats, std::shared_ptr<BlockCommitter> committer,
                                uint32_t resolve_method, uint32_t read_range_method, bool ufs_readahead,
                                int ufs_create_after_reads) {
          if (!stats) stats = std::make_shared<DataServerStats>();
          ColdReadConfig cold;
          cold.commit_method = commit_method;
          cold.resolve_method = resolve_method;
          cold.read_range_method = read_range_method;
          cold.slot_bytes = ufs_slot_bytes;
          cold.depth = ufs_depth;
          cold.max_active = ufs_max_active;
          cold.readahead = ufs_readahead;
          cold.create_after_reads = ufs_create_after_reads;
          serve_block_reads(srv, method, store, max_chunk, window, stats, mounts, cold, committer);
          return stats;
        }, py::arg("server"), py::arg("method"), py::arg("store"), py::arg("max_chunk"), py::arg("window"),
        py::arg("mounts") = nullptr, py::arg("commit_method") = UINT32_MAX, py::arg("ufs_slot_bytes") = 8u << 20,
        py::arg("ufs_depth") = 3, py::arg("ufs_max_active") = 256, py::arg("stats") = nullptr,
        py::arg("committer") = nullptr, py::arg("resolve_method") = UINT32_MAX,
        py::arg("read_range_method") = UINT32_MAX, py::arg("ufs_readahead") = true,
        py::arg("ufs_create_after_reads") = 2, py::keep_alive<1, 3>());
  m.def("serve_block_writes", [](FrameRpcServer& srv, uint32_t method, uint32_t commit_method, std::shared_ptr<BlockStore> store,
                                 uint64_t stage_bytes, std::shared_ptr<DataServerStats> stats,
                                 std::shared_ptr<UfsMounts> ufs_roots, std::shared_ptr<BlockCommitter> committer) {
          serve_block_writes(srv, method, commit_method, store, stage_bytes, stats, ufs_roots, committer);
        }, py::arg("server"), py::arg("method"), py::arg("commit_method"), py::arg("store"), py::arg("stage_bytes"),
        py::arg("stats"), py::arg("ufs_roots") = nullptr, py::arg("committer") = nullptr, py::keep_alive<1, 4>());
  m.def("stream_recv", [](FrameRpcServer& srv, uint64_t token, int timeout_ms) -> py::tuple {
          std::string msg;
          int rc;
          {
            py::gil_scoped_release rel;
            rc = srv.stream_recv(token, timeout_ms, &msg);
          }
          if (rc == 0) return py::make_tuple(rc, py::bytes(msg));
          return py::make_tuple(rc, py::object(py::none()));
        }, py::arg("server"), py::arg("token"), py::arg("timeout_ms"));
  m.def("stream_send", [](FrameRpcServer& srv, uint64_t token, py::buffer msg, int timeout_ms) {
          py::buffer_info bi = msg.request();
          std::string m(static_cast<const char*>(bi.ptr), (size_t)(bi.size * bi.itemsize));
          py::gil_scoped_release rel;
          return srv.stream_send(token, m, timeout_ms);
        }, py::arg("server"), py::arg("token"), py::arg("message"), py::arg("timeout_ms") = 60000);
  m.def("stream_finish", [](FrameRpcServer& srv, uint64_t token, int status, const std::string& msg) {
          py::gil_scoped_release rel;
          srv.stream_finish(token, status, msg);
        }, py::arg("server"), py::arg("token"), py::arg("status"), py::arg("message") = "");
  m.def("allow_channel", [](FrameRpcServer& srv, const std::string& cid, const std::string& user) {
          srv.allow_channel(cid, user);
        });
  m.def("revoke_channel", [](FrameRpcServer& srv, const std::string& cid) { srv.revoke_channel(cid); });
  m.def("set_require_channel_auth", [](FrameRpcServer& srv, bool on) { srv.set_require_channel_auth(on); });
  m.def("set_stream_window", [](FrameRpcServer& srv, uint32_t bytes) { srv.set_stream_window(bytes); });
  m.def("set_prefetch_threads", &set_prefetch_threads, py::arg("threads"));

  // ---- HDFS DataTransferProtocol packets (gateway DataNode reads, Hadoop client reads) -------
  m.def("dn_send_block", [](int fd, std::shared_ptr<BlockSource> src, uint64_t offset, uint64_t length,
                            uint32_t bpc, uint32_t packet_bytes, int timeout_ms, bool flip, bool truncate) {
          DnSendOptions o;
          o.bytes_per_checksum = bpc;
          o.packet_bytes = packet_bytes;
          o.timeout_ms = timeout_ms;
          o.fault_flip_bits = flip;
          o.fault_truncate = truncate;
          if (src->needs_gil()) return dn_send_block(fd, *src, offset, length, o);
          py::gil_scoped_release rel;
          return dn_send_block(fd, *src, offset, length, o);
        }, py::arg("fd"), py::arg("source"), py::arg("offset"), py::arg("length"), py::arg("bytes_per_checksum") = 512,
        py::arg("packet_bytes") = 1u << 20, py::arg("timeout_ms") = 60000, py::arg("flip_bits") = false,
        py::arg("truncate") = false);
  py::class_<DnPacketReader>(m, "DnPacketReader")
      .def(py::init<int, uint32_t, bool, uint64_t, int>(), py::arg("fd"), py::arg("bytes_per_checksum"),
           py::arg("verify"), py::arg("skip"), py::arg("timeout_ms") = 60000)
      .def("readinto", [](DnPacketReader& r, py::buffer b, uint64_t n) {
             py::buffer_info bi = b.request(true);
             n = std::min<uint64_t>(n, (uint64_t)(bi.size * bi.itemsize));
             py::gil_scoped_release rel;
             return r.readinto(static_cast<uint8_t*>(bi.ptr), n);
           }, py::arg("buffer"), py::arg("n"))
      .def("drain", &DnPacketReader::drain, G())
      .def_property_readonly("done", &DnPacketReader::done)
      .def_property_readonly("packets", &DnPacketReader::packets);
  py::class_<DnPacketWriter>(m, "DnPacketWriter")
      .def(py::init<int, uint32_t, uint32_t, uint32_t, int>(), py::arg("fd"), py::arg("bytes_per_checksum") = 512,
           py::arg("packet_bytes") = 64u << 10, py::arg("max_in_flight") = 80, py::arg("timeout_ms") = 60000)
      .def("write", [](DnPacketWriter& w, py::buffer b) {
             py::buffer_info bi = b.request();
             const uint64_t n = (uint64_t)(bi.size * bi.itemsize);
             py::gil_scoped_release rel;
             w.write(static_cast<const uint8_t*>(bi.ptr), n);
           }, py::arg("data"))
      .def("finish", &DnPacketWriter::finish, G())
      .def_property_readonly("offset", &DnPacketWriter::offset);
  py::class_<DnPacketReceiver>(m, "DnPacketReceiver")
      .def(py::init<int, uint32_t, int>(), py::arg("fd"), py::arg("bytes_per_checksum") = 512,
           py::arg("timeout_ms") = 60000)
      .def("receive", [](DnPacketReceiver& r, py::buffer b, uint64_t batch) {
             py::buffer_info bi = b.request(true);
             bool last = false;
             int status = 0;
             uint64_t n;
             {
               py::gil_scoped_release rel;
               n = r.receive(static_cast<uint8_t*>(bi.ptr), (uint64_t)(bi.size * bi.itemsize), batch, &last, &status);
             }
             return py::make_tuple(n, last, status);
           }, py::arg("buffer"), py::arg("batch"))
      .def("ack", &DnPacketReceiver::ack, G(), py::arg("status"))
      .def_property_readonly("received", &DnPacketReceiver::received);
  m.def("listen_unix", [](FrameRpcServer& srv, const std::string& path) { srv.listen_unix(path); });
}
