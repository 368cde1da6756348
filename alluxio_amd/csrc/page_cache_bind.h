// pybind11 bindings of the K9 HBM client page cache (included by bindings.cpp).
#pragma once
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include <cstring>

#include <string>

#include "block_store.h"
#include "page_cache.h"

namespace amdx {

inline void bind_page_cache(pybind11::module_& m) {
  namespace py = pybind11;
  using G = py::call_guard<py::gil_scoped_release>;
  py::class_<DevicePageCache>(m, "PageCache")
      .def(py::init<int, uint64_t, uint64_t, bool>(), py::arg("device"), py::arg("capacity"),
           py::arg("page_size"), py::arg("use_device"))
      .def("put", &DevicePageCache::put, G(), py::arg("key"), py::arg("src"), py::arg("length"),
           py::arg("src_kind"), py::arg("stream") = 0, py::arg("evict") = true)
      .def("put_bytes", [](DevicePageCache& c, uint64_t key, py::buffer data, bool evict) {
             py::buffer_info bi = data.request();
             const uint64_t n = (uint64_t)bi.size * (uint64_t)bi.itemsize;
             py::gil_scoped_release rel;
             return c.put(key, (uint64_t)bi.ptr, n, (int)MemKind::kHost, 0, evict);
           }, py::arg("key"), py::arg("data"), py::arg("evict") = true)
      .def("put_many", &DevicePageCache::put_many, G(), py::arg("keys"), py::arg("src"),
           py::arg("src_stride"), py::arg("length"), py::arg("src_kind"), py::arg("stream"),
           py::arg("evict"))
      .def("put_many_device", [](DevicePageCache& c, uint64_t keys, uint32_t n, uint64_t src, uint64_t stride,
                                 uint64_t len, int kind, uint64_t stream, bool evict, bool as_array) -> py::object {
             std::vector<uint64_t> ev;
             {
               py::gil_scoped_release rel;
               ev = c.put_many_device(keys, n, src, stride, len, kind, stream, evict);
             }
             if (!as_array) return py::cast(ev);
             // a whole cache's worth of evicted keys: one memcpy instead of a Python int per key
             py::array_t<uint64_t> out(ev.size());
             if (!ev.empty()) std::memcpy(out.mutable_data(), ev.data(), ev.size() * sizeof(uint64_t));
             return std::move(out);
           }, py::arg("keys"), py::arg("n"), py::arg("src"), py::arg("src_stride"), py::arg("length"),
           py::arg("src_kind"), py::arg("stream"), py::arg("evict"), py::arg("as_array") = false)
      .def_property_readonly("device_owned", &DevicePageCache::device_owned)
      .def("erase", &DevicePageCache::erase, G())
      .def("contains", &DevicePageCache::contains, G())
      .def("lookup", &DevicePageCache::lookup, G())
      .def("slot_ptr", &DevicePageCache::slot_ptr)
      .def("read", &DevicePageCache::read, G(), py::arg("key"), py::arg("offset"), py::arg("length"),
           py::arg("dst"), py::arg("dst_kind"), py::arg("stream") = 0)
      .def("get_bytes", [](DevicePageCache& c, uint64_t key, uint64_t offset, uint64_t length) -> py::object {
             std::string out(length, '\0');
             bool hit;
             {
               py::gil_scoped_release rel;
               hit = c.read(key, offset, length, (uint64_t)out.data(), (int)MemKind::kHost, 0);
             }
             if (!hit) return py::none();
             return py::bytes(out);
           }, py::arg("key"), py::arg("offset"), py::arg("length"))
      .def("read_segments", &DevicePageCache::read_segments, G(), py::arg("keys"), py::arg("offsets"),
           py::arg("lengths"), py::arg("dsts"), py::arg("dst_kind"), py::arg("stream") = 0)
      .def("gather", &DevicePageCache::gather, G(), py::arg("keys"), py::arg("n"), py::arg("dst"),
           py::arg("dst_stride"), py::arg("slot_out"), py::arg("len_out"), py::arg("stream") = 0)
      .def("gather_host_keys", &DevicePageCache::gather_host_keys, G(), py::arg("keys"), py::arg("dst"),
           py::arg("dst_stride"), py::arg("stream") = 0)
      .def("clear", &DevicePageCache::clear, G())
      .def_property_readonly("page_size", &DevicePageCache::page_size)
      .def_property_readonly("slots", &DevicePageCache::slots)
      .def_property_readonly("used", &DevicePageCache::used)
      .def_property_readonly("table_size", &DevicePageCache::table_size)
      .def_property_readonly("arena", &DevicePageCache::arena)
      .def_property_readonly("on_device", &DevicePageCache::on_device);
  m.attr("PAGE_KEY_EMPTY") = kPageKeyEmpty;
  m.def("set_page_gather_small_max", &set_page_gather_small_max, py::arg("bytes"));
  m.def("set_page_gather_wave_variant", &set_page_gather_wave_variant, py::arg("variant"));
}

}  // namespace amdx
