// Host-side native runtime of the inference engine (pybind11 module `_lsa_runtime`).
//
//  * BlockAllocator  — paged-KV block pool (64-token blocks).  Block 0 is reserved as the scratch
//                      block that idle decode slots point at, so a replayed decode graph never
//                      touches a block owned by a live request.
//  * Scheduler       — continuous batching: FCFS admission of waiting requests into fixed decode
//                      slots (stable rows of the device-side decode state, so no compaction between
//                      steps), prefill token budget per step, KV reservation of prompt + max_new
//                      tokens at admission (no preemption needed: 288 GB of HBM makes the
//                      reservation cheap), release on finish / abort.
//  * levenshtein     — character edit distance over Unicode code points (the eval harness metric of
//                      Model_Evaluation_&_Comparision.py:51,125, which used the python-Levenshtein C
//                      extension).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "runtime_core.h"

namespace py = pybind11;

PYBIND11_MODULE(_lsa_runtime, m) {
  m.doc() = "native host runtime: KV block allocator, continuous-batching scheduler, edit distance";
  m.def("levenshtein", &levenshtein, py::arg("a"), py::arg("b"));
  m.def(
      "levenshtein_batch",
      [](const std::vector<std::string>& a, const std::vector<std::string>& b) {
        if (a.size() != b.size()) throw std::invalid_argument("length mismatch");
        std::vector<int> out(a.size());
        py::gil_scoped_release nogil;
        for (size_t i = 0; i < a.size(); ++i) out[i] = levenshtein(a[i], b[i]);
        return out;
      },
      py::arg("a"), py::arg("b"));
  py::class_<BlockAllocator>(m, "BlockAllocator")
      .def(py::init<int, int>(), py::arg("num_blocks"), py::arg("block_size") = 64)
      .def("blocks_for", &BlockAllocator::blocks_for)
      .def("can_alloc", &BlockAllocator::can_alloc)
      .def("alloc", &BlockAllocator::alloc)
      .def("release", &BlockAllocator::release)
      .def_property_readonly("num_free", &BlockAllocator::num_free)
      .def_property_readonly("num_blocks", &BlockAllocator::num_blocks)
      .def_property_readonly("block_size", &BlockAllocator::block_size);
  py::class_<Scheduler>(m, "Scheduler")
      .def(py::init<int, int, int, int, int, int>(), py::arg("num_blocks"), py::arg("block_size"), py::arg("max_slots"),
           py::arg("max_prefill_tokens"), py::arg("max_blocks_per_seq"), py::arg("reserve_tokens") = 64)
      .def("add", &Scheduler::add)
      .def("grow", &Scheduler::grow, py::arg("id"), py::arg("tokens"))
      .def("preempt", &Scheduler::preempt, py::arg("id"), py::arg("prompt_len"), py::arg("max_new"))
      .def("youngest_first", &Scheduler::youngest_first)
      .def("admit", &Scheduler::admit)
      .def("finish", &Scheduler::finish)
      .def("block_table", &Scheduler::block_table)
      .def("slot", &Scheduler::slot)
      .def("slot_owners", &Scheduler::slot_owners)
      .def("running", &Scheduler::running)
      .def_property_readonly("num_waiting", &Scheduler::num_waiting)
      .def_property_readonly("num_running", &Scheduler::num_running)
      .def_property_readonly("highest_slot", &Scheduler::highest_slot)
      .def_property_readonly("kv_usage", &Scheduler::kv_usage)
      .def_property_readonly("free_blocks", &Scheduler::free_blocks)
      .def_property_readonly("reserve_tokens", &Scheduler::reserve_tokens);
}
