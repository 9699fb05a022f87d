// pybind11 bindings for the native fault-tolerance runtime (`_runtime.so`).
#include <hip/hip_runtime_api.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <torch/extension.h>

#include "runtime.h"

namespace py = pybind11;
using namespace ftrt;

// Runs without the GIL (the background prealloc thread pins 16-48 GB while the training
// thread keeps running). `device` >= 0 is made current in the calling thread first: HIP's
// current device is per thread, and the pinned pages should belong to this rank's GPU.
static torch::Tensor pinned_empty(uint64_t nbytes, int device) {
  if (device >= 0 && hipSetDevice(device) != hipSuccess) throw std::runtime_error("hipSetDevice failed");
  uintptr_t p = pinned_alloc(nbytes);
  return torch::from_blob(
      reinterpret_cast<void*>(p), {(int64_t)nbytes},
      [](void* q) { hipHostFree(q); },
      torch::TensorOptions().dtype(torch::kUInt8).device(torch::kCPU));
}

// A stream whose kernels may only be dispatched to the CUs set in `mask` (bit i = CU i,
// 32 CUs per word). Returned as a raw handle for torch.cuda.ExternalStream; lives for the
// process. Used to give memory-bound optimizer kernels a fixed CU share beside GEMMs.
static uint64_t cu_mask_stream(int device, const std::vector<uint32_t>& mask) {
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("hipSetDevice failed");
  hipStream_t s = nullptr;
  hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data());
  if (e != hipSuccess) throw std::runtime_error(std::string("hipExtStreamCreateWithCUMask: ") + hipGetErrorString(e));
  return reinterpret_cast<uint64_t>(s);
}

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "Native fault-tolerance runtime: signal flags, snapshot engine, zip checkpoint writer";

  m.def("signals_install", &signals_install);
  m.def("signals_restore_default", &signals_restore_default);
  m.def("signals_pending", &signals_pending);
  m.def("signals_mask", &signals_mask);
  m.def("signals_count", &signals_count);
  m.def("signals_clear", &signals_clear);
  m.def("signals_block", &signals_block, py::arg("signums"), py::arg("block"));

  py::class_<ZipStats>(m, "ZipStats")
      .def_readonly("seconds", &ZipStats::seconds)
      .def_readonly("write_seconds", &ZipStats::write_seconds)
      .def_readonly("fsync_seconds", &ZipStats::fsync_seconds)
      .def_readonly("wait_seconds", &ZipStats::wait_seconds)
      .def_readonly("bytes", &ZipStats::bytes)
      .def_readonly("direct_bytes", &ZipStats::direct_bytes)
      .def_readonly("error", &ZipStats::error);

  py::class_<ZipWriter>(m, "ZipWriter")
      .def(py::init<std::string, std::string, std::string, int, uint64_t, bool>(), py::arg("tmp_path"),
           py::arg("final_path"), py::arg("archive"), py::arg("nthreads") = 8,
           py::arg("chunk_bytes") = (64ull << 20), py::arg("direct") = true)
      .def("add_bytes",
           [](ZipWriter& w, const std::string& name, py::bytes b) { w.add_bytes(name, std::string(b)); })
      .def("add_buffer", &ZipWriter::add_buffer)
      .def("add_external", &ZipWriter::add_external)
      .def("set_external_crc", &ZipWriter::set_external_crc)
      .def("layout_records", &ZipWriter::layout_records)
      .def("create_file", &ZipWriter::create_file)
      .def("total_size", &ZipWriter::total_size)
      .def("start", &ZipWriter::start, py::arg("wait_event") = 0, py::arg("fsync") = true)
      .def("run_sync", &ZipWriter::run_sync, py::arg("wait_event") = 0, py::arg("fsync") = true,
           py::call_guard<py::gil_scoped_release>())
      .def("done", &ZipWriter::done)
      .def("wait", &ZipWriter::wait, py::call_guard<py::gil_scoped_release>());

  py::class_<SnapshotEngine>(m, "SnapshotEngine")
      .def(py::init<int>())
      .def("begin", &SnapshotEngine::begin)
      .def("copy", &SnapshotEngine::copy)
      .def("mark", &SnapshotEngine::mark)
      .def("stream_wait", &SnapshotEngine::stream_wait)
      .def("query", &SnapshotEngine::query)
      .def("sync", &SnapshotEngine::sync, py::call_guard<py::gil_scoped_release>())
      .def("event_handle", &SnapshotEngine::event_handle)
      .def("stream_handle", &SnapshotEngine::stream_handle)
      .def("num_events", &SnapshotEngine::num_events);

  m.def("write_pieces", &write_pieces, py::arg("path"), py::arg("file_offs"), py::arg("ptrs"), py::arg("lens"),
        py::arg("nthreads") = 8, py::arg("wait_event") = 0, py::arg("fsync") = true, py::arg("direct") = true,
        py::call_guard<py::gil_scoped_release>(),
        "Sharded save: CRC + pwrite this rank's pieces into an existing file; returns per-piece CRC32s");
  m.def("crc32_combine", &crc32_combine_u32);
  py::class_<FileReader>(m, "FileReader")
      .def(py::init<const std::string&, int, bool>(), py::arg("path"), py::arg("threads") = 8,
           py::arg("direct") = true)
      .def("read", &FileReader::read, py::arg("offset"), py::arg("ptr"), py::arg("nbytes"),
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("bytes", &FileReader::bytes)
      .def_property_readonly("direct_bytes", &FileReader::direct_bytes);
  m.def("cu_mask_stream", &cu_mask_stream, py::arg("device"), py::arg("mask"));
  m.def("pinned_empty", &pinned_empty, py::arg("nbytes"), py::arg("device") = -1,
        py::call_guard<py::gil_scoped_release>(),
        "Exact-size pinned host buffer (hipHostMalloc) as a uint8 tensor");
}
