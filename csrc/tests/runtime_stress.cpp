// Sanitizer stress test of the native CPU runtime (SURVEY §5 "Race detection /
// sanitizers"): built by hipserve/_build.py --sanitize {thread,address} as a
// standalone host binary (no Python, no GPU) and run by
// tests/test_native_sanitizers.py.
//
//  * shm ring: one writer thread and R reader threads on ONE mapping of the
//    shared-memory step ring (csrc/runtime/shm_ring.h), thousands of messages of
//    varying size through a small slot ring, every payload checksummed. Under
//    ThreadSanitizer any missing acquire/release pairing between the slot
//    sequence number, the payload copy and the reader acks is reported as a race;
//    under AddressSanitizer any out-of-slot copy is reported.
//  * block pool: randomized allocate / free / prefix-match / register sequences
//    against a reference refcount model (csrc/runtime/block_pool.h).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include "../runtime/block_pool.h"
#include "../runtime/shm_ring.h"

using hipserve_rt::BlockPool;
using hipserve_rt::ShmRing;

#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(2);                                                      \
    }                                                                    \
  } while (0)

static uint32_t fnv(const char* p, size_t n) {
  uint32_t h = 2166136261u;
  for (size_t i = 0; i < n; ++i) h = (h ^ (uint8_t)p[i]) * 16777619u;
  return h;
}

static int ring_stress(int readers, int messages, int slot_cap, int nslots) {
  const std::string name = "/hipserve_stress_" + std::to_string(getpid());
  ShmRing writer(name, readers, slot_cap, nslots, 0, true);
  std::vector<std::unique_ptr<ShmRing>> views;
  for (int r = 1; r <= readers; ++r) views.emplace_back(new ShmRing(writer, r));
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int r = 0; r < readers; ++r) {
    th.emplace_back([&, r] {
      ShmRing& ring = *views[r];
      for (int i = 0; i < messages; ++i) {
        const char* p = nullptr;
        size_t n = 0;
        if (!ring.wait_next(30.0, &p, &n)) { bad++; return; }
        // payload: [u32 index][u32 checksum of the rest][bytes]
        uint32_t idx, sum;
        std::memcpy(&idx, p, 4);
        std::memcpy(&sum, p + 4, 4);
        if (idx != (uint32_t)i || sum != fnv(p + 8, n - 8)) bad++;
        ring.ack();
      }
    });
  }
  std::mt19937 rng(1234);
  std::vector<char> buf(slot_cap);
  for (int i = 0; i < messages; ++i) {
    const size_t n = 8 + rng() % (slot_cap - 8);
    for (size_t j = 8; j < n; ++j) buf[j] = (char)(rng() & 0xFF);
    const uint32_t idx = i, sum = fnv(buf.data() + 8, n - 8);
    std::memcpy(buf.data(), &idx, 4);
    std::memcpy(buf.data() + 4, &sum, 4);
    writer.publish(buf.data(), n);
  }
  for (auto& t : th) t.join();
  CHECK(bad.load() == 0);
  CHECK(writer.published() == (uint64_t)messages);
  return 0;
}

static int pool_stress(int iters) {
  const int nb = 257, bs = 16;
  BlockPool pool(nb, bs, true);
  std::mt19937 rng(99);
  struct Seq {
    std::vector<int> blocks, tokens;
  };
  std::vector<Seq> live;
  for (int it = 0; it < iters; ++it) {
    const int op = rng() % 4;
    if (op == 0 || live.empty()) {  // new sequence, maybe sharing a cached prefix
      Seq s;
      const int ntok = 1 + rng() % (6 * bs);
      const int family = rng() % 3;  // shared prefixes across sequences
      for (int t = 0; t < ntok; ++t) s.tokens.push_back(t < 2 * bs ? family * 1000 + t : (int)(rng() % 50000));
      auto hit = pool.match_prefix(s.tokens);
      s.blocks = hit.first;
      CHECK(hit.second == (int)hit.first.size() * bs);
      const int need = (ntok + bs - 1) / bs - (int)s.blocks.size();
      if (need > pool.num_free()) {
        pool.free(s.blocks);
        continue;
      }
      auto got = pool.allocate(need);
      s.blocks.insert(s.blocks.end(), got.begin(), got.end());
      pool.register_full_blocks(s.blocks, s.tokens, 0, (int)s.blocks.size());
      live.push_back(std::move(s));
    } else if (op == 1) {  // finish a sequence
      const size_t i = rng() % live.size();
      pool.free(live[i].blocks);
      live.erase(live.begin() + i);
    } else if (op == 2) {  // grow a sequence by one block
      auto& s = live[rng() % live.size()];
      if (pool.num_free() > 0) {
        auto got = pool.allocate(1);
        s.blocks.push_back(got[0]);
        for (int t = 0; t < bs; ++t) s.tokens.push_back((int)(rng() % 50000));
      }
    } else {
      pool.reset_prefix_cache();
    }
    // invariants: refcounts match the live sequences exactly
    if (it % 64 == 0) {
      std::vector<int> ref(nb, 0);
      for (auto& s : live)
        for (int b : s.blocks) ref[b]++;
      for (int b = 0; b < nb; ++b) CHECK(pool.refcount(b) == ref[b]);
      int used = 0;
      for (int b = 0; b < nb; ++b) used += ref[b] > 0;
      CHECK(pool.num_free() == nb - used);
    }
  }
  for (auto& s : live) pool.free(s.blocks);
  CHECK(pool.num_free() == nb);
  return 0;
}

int main(int argc, char** argv) {
  const int messages = argc > 1 ? std::atoi(argv[1]) : 20000;
  ring_stress(3, messages, 512, 4);
  ring_stress(1, messages, 4096, 2);
  pool_stress(20000);
  std::printf("runtime_stress ok\n");
  return 0;
}
