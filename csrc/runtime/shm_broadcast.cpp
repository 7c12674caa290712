// Shared-memory step broadcast: the rank-0 scheduler publishes
// each step's metadata (a few KB of serialized StepInputs) to the TP workers of
// the same pod through a POSIX shared-memory ring instead of a gloo TCP
// broadcast. One writer, (world-1) readers, NSLOTS slots:
//
//   header | reader acks [R] | slot 0 | slot 1 | ...
//   slot = { uint64 seq (atomic), uint64 len, bytes[cap] }
//
// publish(): wait until every reader acked seq-NSLOTS (slot free), copy the
//            payload, then store seq with release order.
// recv():    spin (then yield, then sleep) until slot.seq == expected (acquire),
//            copy out, store ack (release).
// Messages larger than a slot fail loudly (the caller falls back to gloo).
// Reference: the engine's step broadcast is vLLM-internal there
// (vllm-models/helm-chart/templates/model-deployments.yaml:37-38 sets TP only).
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

#include <pybind11/pybind11.h>

namespace py = pybind11;

namespace {

constexpr uint64_t kMagic = 0x6869707365727665ull;  // "hipserve"
constexpr int kMaxReaders = 63;

struct Header {
  uint64_t magic;
  uint64_t nslots;
  uint64_t slot_cap;
  uint64_t readers;
  std::atomic<uint64_t> closed;
  uint64_t pad[3];
  std::atomic<uint64_t> ack[kMaxReaders + 1];  // per reader: last consumed seq
};

struct SlotHdr {
  std::atomic<uint64_t> seq;
  uint64_t len;
  uint64_t pad[6];  // 64-byte header
};

inline void backoff(uint64_t& spins) {
  ++spins;
  if (spins < 2000) {
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  } else if (spins < 20000) {
    sched_yield();
  } else {
    timespec ts{0, 50000};  // 50 us: idle engine, no need to burn a core
    nanosleep(&ts, nullptr);
  }
}

}  // namespace

class ShmBroadcast {
 public:
  ShmBroadcast(const std::string& name, int readers, int64_t slot_cap, int nslots, int rank, bool create)
      : name_(name), rank_(rank) {
    if (readers < 1 || readers > kMaxReaders) throw std::invalid_argument("readers must be in [1, 63]");
    if (rank < 0 || rank > readers) throw std::invalid_argument("rank out of range");
    cap_ = (uint64_t)((slot_cap + 63) / 64 * 64);
    nslots_ = (uint64_t)nslots;
    stride_ = sizeof(SlotHdr) + cap_;
    size_ = sizeof(Header) + nslots_ * stride_;
    int fd = -1;
    if (create) {
      shm_unlink(name.c_str());
      fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm_open(create) failed: " + std::string(strerror(errno)));
      if (ftruncate(fd, (off_t)size_) != 0) {
        close(fd);
        throw std::runtime_error("ftruncate failed");
      }
    } else {
      const auto t0 = std::chrono::steady_clock::now();
      while ((fd = shm_open(name.c_str(), O_RDWR, 0600)) < 0) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120))
          throw std::runtime_error("shm_open(attach) timed out for " + name);
        usleep(1000);
      }
      struct stat st;
      while (fstat(fd, &st) == 0 && (uint64_t)st.st_size < size_) usleep(1000);
    }
    void* p = mmap(nullptr, size_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("mmap failed");
    base_ = static_cast<char*>(p);
    hdr_ = reinterpret_cast<Header*>(base_);
    if (create) {
      std::memset(base_, 0, size_);
      hdr_->nslots = nslots_;
      hdr_->slot_cap = cap_;
      hdr_->readers = (uint64_t)readers;
      for (uint64_t i = 0; i < nslots_; ++i) slot(i)->seq.store(0, std::memory_order_relaxed);
      std::atomic_thread_fence(std::memory_order_release);
      reinterpret_cast<std::atomic<uint64_t>*>(&hdr_->magic)->store(kMagic, std::memory_order_release);
    } else {
      uint64_t spins = 0;
      while (reinterpret_cast<std::atomic<uint64_t>*>(&hdr_->magic)->load(std::memory_order_acquire) != kMagic)
        backoff(spins);
      if (hdr_->nslots != nslots_ || hdr_->slot_cap != cap_ || hdr_->readers != (uint64_t)readers)
        throw std::runtime_error("shm ring geometry mismatch");
    }
    readers_ = readers;
  }

  ~ShmBroadcast() {
    if (base_) munmap(base_, size_);
    if (rank_ == 0) shm_unlink(name_.c_str());
  }

  // writer (rank 0)
  void publish(py::bytes data) {
    if (rank_ != 0) throw std::runtime_error("publish() is rank-0 only");
    char* buf;
    Py_ssize_t len;
    PyBytes_AsStringAndSize(data.ptr(), &buf, &len);
    if ((uint64_t)len > cap_) throw std::length_error("message larger than slot capacity");
    const uint64_t seq = ++wseq_;
    SlotHdr* s = slot((seq - 1) % nslots_);
    if (seq > nslots_) {  // slot reuse: all readers must have consumed seq - nslots
      const uint64_t need = seq - nslots_;
      py::gil_scoped_release nogil;
      for (int r = 1; r <= readers_; ++r) {
        uint64_t spins = 0;
        while (hdr_->ack[r].load(std::memory_order_acquire) < need) {
          if (hdr_->closed.load(std::memory_order_relaxed)) throw std::runtime_error("ring closed");
          backoff(spins);
        }
      }
    }
    std::memcpy(reinterpret_cast<char*>(s) + sizeof(SlotHdr), buf, (size_t)len);
    s->len = (uint64_t)len;
    s->seq.store(seq, std::memory_order_release);
  }

  // reader (rank >= 1); timeout_s < 0 waits forever. Returns None on timeout.
  py::object recv(double timeout_s) {
    if (rank_ == 0) throw std::runtime_error("recv() is for ranks >= 1");
    const uint64_t seq = rseq_ + 1;
    SlotHdr* s = slot((seq - 1) % nslots_);
    {
      py::gil_scoped_release nogil;
      uint64_t spins = 0;
      const auto t0 = std::chrono::steady_clock::now();
      while (s->seq.load(std::memory_order_acquire) != seq) {
        if (hdr_->closed.load(std::memory_order_relaxed)) throw std::runtime_error("ring closed");
        if (timeout_s >= 0 && (spins & 1023) == 0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
          return py::none();
        backoff(spins);
      }
    }
    py::bytes out(reinterpret_cast<char*>(s) + sizeof(SlotHdr), (size_t)s->len);
    rseq_ = seq;
    hdr_->ack[rank_].store(seq, std::memory_order_release);
    return out;
  }

  void close_ring() { hdr_->closed.store(1, std::memory_order_relaxed); }
  uint64_t published() const { return wseq_; }
  uint64_t received() const { return rseq_; }
  uint64_t slot_capacity() const { return cap_; }

 private:
  SlotHdr* slot(uint64_t i) { return reinterpret_cast<SlotHdr*>(base_ + sizeof(Header) + i * stride_); }

  std::string name_;
  int rank_;
  int readers_ = 0;
  uint64_t cap_ = 0, nslots_ = 0, stride_ = 0, size_ = 0;
  char* base_ = nullptr;
  Header* hdr_ = nullptr;
  uint64_t wseq_ = 0, rseq_ = 0;
};

void register_shm_broadcast(py::module_& m) {
  py::class_<ShmBroadcast>(m, "ShmBroadcast")
      .def(py::init<const std::string&, int, int64_t, int, int, bool>(), py::arg("name"), py::arg("readers"),
           py::arg("slot_cap"), py::arg("nslots"), py::arg("rank"), py::arg("create"))
      .def("publish", &ShmBroadcast::publish)
      .def("recv", &ShmBroadcast::recv, py::arg("timeout_s") = -1.0)
      .def("close", &ShmBroadcast::close_ring)
      .def_property_readonly("published", &ShmBroadcast::published)
      .def_property_readonly("received", &ShmBroadcast::received)
      .def_property_readonly("slot_capacity", &ShmBroadcast::slot_capacity);
}
