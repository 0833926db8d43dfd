// pybind11 module `_native`: host runtime (TensorBundle checkpoint I/O, CRC32C,
// synthetic data source / prefetching loader).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "native_common.h"

namespace py = pybind11;
using namespace tdgn;

namespace {
py::dict entry_dict(const BundleEntry& e) {
  py::dict d;
  d["dtype"] = e.dtype;
  d["shape"] = e.shape;
  d["shard_id"] = e.shard_id;
  d["offset"] = e.offset;
  d["size"] = e.size;
  d["crc32c"] = e.crc32c;
  return d;
}
BundleEntry entry_from(const py::dict& d) {
  BundleEntry e;
  e.dtype = d.contains("dtype") ? d["dtype"].cast<int>() : 0;
  e.shape = d.contains("shape") ? d["shape"].cast<std::vector<int64_t>>() : std::vector<int64_t>{};
  e.shard_id = d.contains("shard_id") ? d["shard_id"].cast<int>() : 0;
  e.offset = d.contains("offset") ? d["offset"].cast<int64_t>() : 0;
  e.size = d.contains("size") ? d["size"].cast<int64_t>() : 0;
  e.crc32c = d.contains("crc32c") ? d["crc32c"].cast<uint32_t>() : 0;
  return e;
}
std::pair<const uint8_t*, size_t> buf_of(const py::buffer& b) {
  py::buffer_info info = b.request();
  if (info.ndim > 1) {
    // require C-contiguity
    ssize_t expect = info.itemsize;
    for (ssize_t i = info.ndim - 1; i >= 0; --i) {
      if (info.strides[i] != expect) throw std::runtime_error("buffer must be C-contiguous");
      expect *= info.shape[i];
    }
  }
  return {(const uint8_t*)info.ptr, (size_t)(info.size * info.itemsize)};
}
}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "host runtime: TensorBundle I/O, CRC32C, synthetic data loader";

  m.def("crc32c", [](py::bytes b, uint32_t init) {
    std::string s = b;
    return crc32c_extend(init, (const uint8_t*)s.data(), s.size());
  }, py::arg("data"), py::arg("init") = 0);
  m.def("crc32c_buffer", [](py::buffer b) {
    auto p = buf_of(b);
    uint32_t c;
    {
      py::gil_scoped_release r;
      c = crc32c_extend(0, p.first, p.second);
    }
    return c;
  });
  m.def("crc_mask", &crc_mask);
  m.def("crc_unmask", &crc_unmask);
  m.def("encode_entry", [](py::dict d) { return py::bytes(encode_entry(entry_from(d))); });
  m.def("decode_entry", [](py::bytes b) { return entry_dict(decode_entry(std::string(b))); });
  m.def("encode_header", [](int shards, int producer) {
    return py::bytes(encode_header(shards, producer));
  });
  m.def("build_sstable", [](const std::vector<std::pair<py::bytes, py::bytes>>& kv) {
    std::vector<std::pair<std::string, std::string>> v;
    for (const auto& p : kv) v.emplace_back(std::string(p.first), std::string(p.second));
    return py::bytes(build_sstable(v));
  });
  m.def("parse_sstable", [](py::bytes file, bool verify) {
    py::list out;
    for (auto& kv : parse_sstable(std::string(file), verify))
      out.append(py::make_tuple(py::bytes(kv.first), py::bytes(kv.second)));
    return out;
  }, py::arg("file"), py::arg("verify") = true);

  py::class_<BundleWriter>(m, "BundleWriter")
      .def(py::init<const std::string&>())
      .def("add", [](BundleWriter& w, const std::string& key, int dtype,
                     const std::vector<int64_t>& shape, py::buffer data) {
        auto p = buf_of(data);
        py::gil_scoped_release r;
        w.add(key, dtype, shape, p.first, p.second);
      })
      .def("add_string", [](BundleWriter& w, const std::string& key, py::bytes v) {
        w.add_string(key, std::string(v));
      })
      .def("finish", &BundleWriter::finish);

  py::class_<BundleReader>(m, "BundleReader")
      .def(py::init<const std::string&, bool>(), py::arg("prefix"), py::arg("verify") = true)
      .def("keys", &BundleReader::keys)
      .def("entry", [](const BundleReader& r, const std::string& k) { return entry_dict(r.entry(k)); })
      .def("read", [](const BundleReader& r, const std::string& k, bool verify) {
        std::string s;
        {
          py::gil_scoped_release rel;
          s = r.read(k, verify);
        }
        return py::bytes(s);
      }, py::arg("key"), py::arg("verify") = true)
      .def("num_shards", &BundleReader::num_shards);

  py::class_<SynthConfig>(m, "SynthConfig")
      .def(py::init<>())
      .def_readwrite("seed", &SynthConfig::seed)
      .def_readwrite("rank", &SynthConfig::rank)
      .def_readwrite("world", &SynthConfig::world)
      .def_readwrite("batch", &SynthConfig::batch)
      .def_readwrite("src_len", &SynthConfig::src_len)
      .def_readwrite("tgt_len", &SynthConfig::tgt_len)
      .def_readwrite("src_vocab", &SynthConfig::src_vocab)
      .def_readwrite("tgt_vocab", &SynthConfig::tgt_vocab)
      .def_readwrite("min_len", &SynthConfig::min_len)
      .def_readwrite("start_id", &SynthConfig::start_id)
      .def_readwrite("end_id", &SynthConfig::end_id)
      .def_readwrite("copy_task", &SynthConfig::copy_task);

  // fill int64 host buffers (e.g. pinned torch tensors) given raw addresses
  m.def("synth_fill", [](const SynthConfig& c, int64_t step, uintptr_t src, uintptr_t tgt) {
    py::gil_scoped_release r;
    synth_fill(c, step, (int64_t*)src, (int64_t*)tgt);
  });

  py::class_<Prefetcher>(m, "Prefetcher")
      .def(py::init<const SynthConfig&, int, int>(), py::arg("cfg"), py::arg("depth") = 4,
           py::arg("threads") = 2)
      .def("get", [](Prefetcher& p, int64_t step, uintptr_t src, uintptr_t tgt) {
        py::gil_scoped_release r;
        p.get(step, (int64_t*)src, (int64_t*)tgt);
      });
}
