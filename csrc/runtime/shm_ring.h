// Shared-memory step ring — pybind-free core, shared by the
// Python binding (shm_broadcast.cpp) and the sanitizer stress test
// (csrc/tests/runtime_stress.cpp, built with -fsanitize=thread / address).
//
// The rank-0 scheduler publishes each step's metadata (a few KB of serialized
// StepInputs) to the TP workers of the same pod. One writer, R readers, NSLOTS
// slots in one POSIX shared-memory object:
//
//   Header | slot 0 | slot 1 | ...      slot = { atomic seq, len, bytes[cap] }
//
// publish(): wait until every reader acked seq-NSLOTS (slot free), copy the
//            payload, then store seq with release order.
// wait_next()/ack(): spin (then yield, then sleep) until slot.seq == expected
//            (acquire), hand out a pointer into the slot; ack() stores the
//            reader's consumed seq (release) so the writer may reuse the slot.
// Reference: the engine's step broadcast is vLLM-internal there
// (vllm-models/helm-chart/templates/model-deployments.yaml:37-38 sets TP only).
#pragma once

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

namespace hipserve_rt {

constexpr uint64_t kRingMagic = 0x6869707365727665ull;  // "hipserve"
constexpr int kRingMaxReaders = 63;

struct RingHeader {
  std::atomic<uint64_t> magic;
  uint64_t nslots;
  uint64_t slot_cap;
  uint64_t readers;
  std::atomic<uint64_t> closed;
  uint64_t pad[3];
  std::atomic<uint64_t> ack[kRingMaxReaders + 1];  // per reader: last consumed seq
};

struct RingSlot {
  std::atomic<uint64_t> seq;
  uint64_t len;
  uint64_t pad[6];  // 64-byte slot header
};

inline void ring_backoff(uint64_t& spins) {
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

class ShmRing {
 public:
  // Create (rank 0) or attach (rank >= 1) the named ring.
  ShmRing(const std::string& name, int readers, int64_t slot_cap, int nslots, int rank, bool create)
      : name_(name), rank_(rank), owner_(true) {
    if (readers < 1 || readers > kRingMaxReaders) throw std::invalid_argument("readers must be in [1, 63]");
    if (rank < 0 || rank > readers) throw std::invalid_argument("rank out of range");
    if (nslots < 2) throw std::invalid_argument("need at least 2 slots");
    cap_ = (uint64_t)((slot_cap + 63) / 64 * 64);
    nslots_ = (uint64_t)nslots;
    stride_ = sizeof(RingSlot) + cap_;
    size_ = sizeof(RingHeader) + nslots_ * stride_;
    readers_ = readers;
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
    hdr_ = reinterpret_cast<RingHeader*>(base_);
    if (create) {
      std::memset(base_, 0, size_);
      hdr_->nslots = nslots_;
      hdr_->slot_cap = cap_;
      hdr_->readers = (uint64_t)readers;
      for (uint64_t i = 0; i < nslots_; ++i) slot(i)->seq.store(0, std::memory_order_relaxed);
      hdr_->magic.store(kRingMagic, std::memory_order_release);
    } else {
      uint64_t spins = 0;
      while (hdr_->magic.load(std::memory_order_acquire) != kRingMagic) ring_backoff(spins);
      if (hdr_->nslots != nslots_ || hdr_->slot_cap != cap_ || hdr_->readers != (uint64_t)readers)
        throw std::runtime_error("shm ring geometry mismatch");
    }
  }

  // In-process view of `owner`'s mapping for reader `rank` (threads of one
  // process share the exact addresses, which is what ThreadSanitizer checks).
  ShmRing(const ShmRing& owner, int rank)
      : name_(owner.name_), rank_(rank), owner_(false), readers_(owner.readers_), cap_(owner.cap_),
        nslots_(owner.nslots_), stride_(owner.stride_), size_(owner.size_), base_(owner.base_),
        hdr_(owner.hdr_) {
    if (rank < 1 || rank > readers_) throw std::invalid_argument("view rank out of range");
  }

  ShmRing(const ShmRing&) = delete;
  ShmRing& operator=(const ShmRing&) = delete;

  ~ShmRing() {
    if (!owner_) return;
    if (base_) munmap(base_, size_);
    if (rank_ == 0) shm_unlink(name_.c_str());
  }

  // writer (rank 0): blocks while the slot is still being read
  void publish(const char* buf, size_t len) {
    if (rank_ != 0) throw std::runtime_error("publish() is rank-0 only");
    if ((uint64_t)len > cap_) throw std::length_error("message larger than slot capacity");
    const uint64_t seq = wseq_ + 1;
    RingSlot* s = slot((seq - 1) % nslots_);
    if (seq > nslots_) {  // slot reuse: all readers must have consumed seq - nslots
      const uint64_t need = seq - nslots_;
      for (int r = 1; r <= readers_; ++r) {
        uint64_t spins = 0;
        while (hdr_->ack[r].load(std::memory_order_acquire) < need) {
          if (hdr_->closed.load(std::memory_order_relaxed)) throw std::runtime_error("ring closed");
          ring_backoff(spins);
        }
      }
    }
    std::memcpy(reinterpret_cast<char*>(s) + sizeof(RingSlot), buf, len);
    s->len = (uint64_t)len;
    s->seq.store(seq, std::memory_order_release);
    wseq_ = seq;
  }

  // reader (rank >= 1): wait for the next message; false on timeout
  // (timeout_s < 0 waits forever). The payload stays valid until ack().
  bool wait_next(double timeout_s, const char** data, size_t* len) {
    if (rank_ == 0) throw std::runtime_error("wait_next() is for ranks >= 1");
    const uint64_t seq = rseq_ + 1;
    RingSlot* s = slot((seq - 1) % nslots_);
    uint64_t spins = 0;
    const auto t0 = std::chrono::steady_clock::now();
    while (s->seq.load(std::memory_order_acquire) != seq) {
      if (hdr_->closed.load(std::memory_order_relaxed)) throw std::runtime_error("ring closed");
      if (timeout_s >= 0 && (spins & 1023) == 0 &&
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
        return false;
      ring_backoff(spins);
    }
    *data = reinterpret_cast<const char*>(s) + sizeof(RingSlot);
    *len = (size_t)s->len;
    return true;
  }

  void ack() {
    rseq_ += 1;
    hdr_->ack[rank_].store(rseq_, std::memory_order_release);
  }

  void close_ring() { hdr_->closed.store(1, std::memory_order_relaxed); }
  uint64_t published() const { return wseq_; }
  uint64_t received() const { return rseq_; }
  uint64_t slot_capacity() const { return cap_; }

 private:
  RingSlot* slot(uint64_t i) const { return reinterpret_cast<RingSlot*>(base_ + sizeof(RingHeader) + i * stride_); }

  std::string name_;
  int rank_;
  bool owner_;
  int readers_ = 0;
  uint64_t cap_ = 0, nslots_ = 0, stride_ = 0, size_ = 0;
  char* base_ = nullptr;
  RingHeader* hdr_ = nullptr;
  uint64_t wseq_ = 0, rseq_ = 0;
};

}  // namespace hipserve_rt
