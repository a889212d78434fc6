// Host-side C++ runtime of consensusml_amd (module `_runtime`, pybind11, no torch / no HIP, so it
// also loads in the CPU-only container):
//
//   RecordLoader  multi-threaded, seeded-shuffle batch assembler over a memory-mapped file of
//                 fixed-size records, filling a ring of caller-owned (pinned) host buffers ahead
//                 of the training loop; each rank reads a disjoint 1/world share per epoch.
//   Watchdog      failure detection: a monitor thread that fires when the training loop stops
//                 calling beat() for `timeout` seconds (writes a report; optional hard abort so a
//                 hung collective cannot hold the GPU forever).
//   plan_buckets  flat-buffer bucket layout (same rule as consensusml_amd/parallel/flat.py).
//   crc32_file / write_file_atomic   checkpoint integrity + atomic publish.
//   write_csv     CSV writer for the consensus (standard output) table.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "runtime_core.h"

namespace py = pybind11;

namespace cmlrt {

// columns: list of (name, list[float]|list[str]); all the same length. NaN / None -> "NA" (R style,
// as in the reference's standouttable.csv). Strings are double-quoted like R's write.csv.
void write_csv(const std::string& path, const std::vector<std::string>& row_names,
               const std::vector<std::pair<std::string, py::object>>& cols) {
  const size_t n = row_names.size();
  std::vector<std::string> names;
  std::vector<std::vector<std::string>> cells(cols.size());
  for (size_t c = 0; c < cols.size(); ++c) {
    names.push_back(cols[c].first);
    py::list lst = py::list(cols[c].second);
    if (static_cast<size_t>(py::len(lst)) != n) throw std::invalid_argument("write_csv: ragged column " + cols[c].first);
    cells[c].resize(n);
    for (size_t i = 0; i < n; ++i) {
      py::handle h = lst[i];
      if (py::isinstance<py::str>(h)) cells[c][i] = "\"" + h.cast<std::string>() + "\"";
      else if (h.is_none()) cells[c][i] = "NA";
      else cells[c][i] = format_number(h.cast<double>());
    }
  }
  write_file_atomic(path, format_csv(row_names, names, cells));
}

py::tuple loader_next(RecordLoader& L) {
  RecordLoader::Batch b;
  {
    py::gil_scoped_release nogil;
    b = L.next_batch();
  }
  return py::make_tuple(b.slot, b.rows, b.epoch, b.ticket);
}

}  // namespace cmlrt

PYBIND11_MODULE(_runtime, m) {
  using namespace cmlrt;
  m.doc() = "consensusml_amd host runtime (loader, watchdog, bucket planner, checkpoint IO)";
  py::class_<RecordLoader>(m, "RecordLoader")
      .def(py::init<const std::string&, int64_t, int64_t, int64_t, int64_t, uint64_t, int, bool>(),
           py::arg("path"), py::arg("record_bytes"), py::arg("batch"), py::arg("rank") = 0,
           py::arg("world") = 1, py::arg("seed") = 0, py::arg("threads") = 4,
           py::arg("drop_last") = true)
      .def("num_records", &RecordLoader::num_records)
      .def("batches_per_epoch", &RecordLoader::batches_per_epoch)
      .def("batch_indices", &RecordLoader::batch_indices)
      .def("start", &RecordLoader::start, py::arg("slots"), py::arg("slot_bytes"), py::arg("epoch0") = 0)
      .def("next", &loader_next)
      .def("release", &RecordLoader::release)
      .def("stop", &RecordLoader::stop, py::call_guard<py::gil_scoped_release>());
  py::class_<Watchdog>(m, "Watchdog")
      .def(py::init<double, const std::string&, bool>(), py::arg("timeout_s"),
           py::arg("report_path") = "", py::arg("hard_abort") = false)
      .def("beat", &Watchdog::beat)
      .def("set_phase", &Watchdog::set_phase)
      .def("fired", &Watchdog::fired)
      .def("stop", &Watchdog::stop, py::call_guard<py::gil_scoped_release>());
  py::class_<BucketPlan>(m, "BucketPlan")
      .def_readonly("offsets", &BucketPlan::offsets)
      .def_readonly("lengths", &BucketPlan::lengths)
      .def_readonly("shards", &BucketPlan::shards)
      .def_readonly("param_offsets", &BucketPlan::param_offsets)
      .def_readonly("param_bucket", &BucketPlan::param_bucket)
      .def_readonly("total", &BucketPlan::total)
      .def_readonly("shard_total", &BucketPlan::shard_total);
  m.def("plan_buckets", &plan_buckets, py::arg("numels"), py::arg("world"), py::arg("align"),
        py::arg("bucket_elems"));
  m.def("crc32_file", &crc32_file);
  m.def("write_file_atomic", [](const std::string& p, const py::bytes& d) { write_file_atomic(p, std::string(d)); });
  m.def("write_csv", &write_csv, py::arg("path"), py::arg("row_names"), py::arg("cols"));
}
