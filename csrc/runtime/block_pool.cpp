// hipserve native runtime module: Python bindings of the paged KV-cache block
// pool (block_pool.h) and the per-step batch builder (block tables, slot
// mapping, positions) — the CPU-side hot path of every engine step.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "block_pool.h"

#include <cstdint>
#include <cstring>
#include <list>
#include <stdexcept>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

using hipserve_rt::BlockPool;

py::tuple match_prefix_py(BlockPool& pool, const std::vector<int>& tokens) {
  auto r = pool.match_prefix(tokens);
  return py::make_tuple(r.first, r.second);
}

// Build the flat per-step tensors for a batch in one pass.
//   tables: per sequence list of block ids; starts/ends: token range [start,end)
//   of each sequence processed this step. Returns (block_table[n, W] int32,
//   slot_mapping[T] int64, positions[T] int64).
py::tuple build_batch(const std::vector<std::vector<int>>& tables, const std::vector<int>& starts,
                      const std::vector<int>& ends, int block_size, int width) {
  const size_t n = tables.size();
  size_t T = 0;
  int maxw = 1;
  for (size_t i = 0; i < n; ++i) {
    T += (size_t)(ends[i] - starts[i]);
    maxw = std::max(maxw, (int)tables[i].size());
  }
  if (width <= 0) width = maxw;
  if (maxw > width) throw std::runtime_error("block table wider than the captured width");
  py::array_t<int32_t> bt({(py::ssize_t)n, (py::ssize_t)width});
  py::array_t<int64_t> slots((py::ssize_t)T);
  py::array_t<int64_t> pos((py::ssize_t)T);
  auto B = bt.mutable_unchecked<2>();
  auto S = slots.mutable_unchecked<1>();
  auto P = pos.mutable_unchecked<1>();
  size_t t = 0;
  for (size_t i = 0; i < n; ++i) {
    const auto& tb = tables[i];
    int j = 0;
    for (; j < (int)tb.size(); ++j) B(i, j) = tb[j];
    for (; j < width; ++j) B(i, j) = tb.empty() ? 0 : tb.back();
    for (int p = starts[i]; p < ends[i]; ++p, ++t) {
      const int blk = p / block_size;
      if (blk >= (int)tb.size()) throw std::runtime_error("slot beyond allocated blocks");
      S(t) = (int64_t)tb[blk] * block_size + (p % block_size);
      P(t) = p;
    }
  }
  return py::make_tuple(bt, slots, pos);
}

}  // namespace

void register_shm_broadcast(py::module_& m);  // shm_broadcast.cpp

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "hipserve native runtime (KV block pool, batch builder, shared-memory step broadcast)";
  register_shm_broadcast(m);
  py::class_<BlockPool>(m, "BlockPool")
      .def(py::init<int, int, bool>(), py::arg("num_blocks"), py::arg("block_size"),
           py::arg("prefix_caching") = true)
      .def_property_readonly("num_blocks", &BlockPool::num_blocks)
      .def_property_readonly("block_size", &BlockPool::block_size)
      .def("num_free", &BlockPool::num_free)
      .def("num_cached", &BlockPool::num_cached)
      .def("usage", &BlockPool::usage)
      .def("allocate", &BlockPool::allocate)
      .def("free", &BlockPool::free)
      .def("block_hash", &BlockPool::block_hash)
      .def("match_prefix", &match_prefix_py)
      .def("register_full_blocks", &BlockPool::register_full_blocks)
      .def("register_blocks", &BlockPool::register_blocks)
      .def("reset_prefix_cache", &BlockPool::reset_prefix_cache)
      .def("refcount", &BlockPool::refcount);
  m.def("build_batch", &build_batch, py::arg("tables"), py::arg("starts"), py::arg("ends"),
        py::arg("block_size"), py::arg("width") = 0);
}
