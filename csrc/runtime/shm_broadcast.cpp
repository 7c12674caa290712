// Python binding of the shared-memory step ring (core: shm_ring.h). The GIL is
// released while a publisher waits for a free slot or a reader waits for the
// next message, so the engine's HTTP thread keeps running.
#include <pybind11/pybind11.h>

#include "shm_ring.h"

namespace py = pybind11;
using hipserve_rt::ShmRing;

namespace {

class PyShmBroadcast {
 public:
  PyShmBroadcast(const std::string& name, int readers, int64_t slot_cap, int nslots, int rank, bool create)
      : ring_(name, readers, slot_cap, nslots, rank, create) {}

  void publish(py::bytes data) {
    char* buf;
    Py_ssize_t len;
    PyBytes_AsStringAndSize(data.ptr(), &buf, &len);  // `data` keeps the buffer alive
    py::gil_scoped_release nogil;
    ring_.publish(buf, (size_t)len);
  }

  // timeout_s < 0 waits forever; None on timeout
  py::object recv(double timeout_s) {
    const char* p = nullptr;
    size_t n = 0;
    bool ok;
    {
      py::gil_scoped_release nogil;
      ok = ring_.wait_next(timeout_s, &p, &n);
    }
    if (!ok) return py::none();
    py::bytes out(p, n);
    ring_.ack();
    return out;
  }

  void close() { ring_.close_ring(); }
  uint64_t published() const { return ring_.published(); }
  uint64_t received() const { return ring_.received(); }
  uint64_t slot_capacity() const { return ring_.slot_capacity(); }

 private:
  ShmRing ring_;
};

}  // namespace

void register_shm_broadcast(py::module_& m) {
  py::class_<PyShmBroadcast>(m, "ShmBroadcast")
      .def(py::init<const std::string&, int, int64_t, int, int, bool>(), py::arg("name"), py::arg("readers"),
           py::arg("slot_cap"), py::arg("nslots"), py::arg("rank"), py::arg("create"))
      .def("publish", &PyShmBroadcast::publish)
      .def("recv", &PyShmBroadcast::recv, py::arg("timeout_s") = -1.0)
      .def("close", &PyShmBroadcast::close)
      .def_property_readonly("published", &PyShmBroadcast::published)
      .def_property_readonly("received", &PyShmBroadcast::received)
      .def_property_readonly("slot_capacity", &PyShmBroadcast::slot_capacity);
}
