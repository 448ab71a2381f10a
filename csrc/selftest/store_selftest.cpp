// Standalone self-test of the rendezvous store and socket layer, built with
// AddressSanitizer + UndefinedBehaviorSanitizer (no torch / HIP dependency):
//   g++ -std=c++17 -O1 -g -fsanitize=address,undefined -Icsrc \
//       csrc/selftest/store_selftest.cpp csrc/store/tcp_store.cpp -lpthread
// Threads play the ranks: concurrent set/get/add/wait/barrier/compare_set
// traffic against one server (sanitizer builds of host code).
#include <atomic>
#include <cstdio>
#include <thread>
#include <vector>

#include "common.h"
#include "store/tcp_store.h"

using dcp::TCPStore;

int main() {
  const int world = 8;
  std::unique_ptr<TCPStore> master;
  std::atomic<int> failures{0};
  master = std::make_unique<TCPStore>("127.0.0.1", 0, world, true, 20000, false);
  const int port = master->port();
  std::vector<std::thread> ts;
  for (int r = 0; r < world; ++r) {
    ts.emplace_back([&, r] {
      try {
        TCPStore s("127.0.0.1", port, world, false, 20000, false);
        for (int i = 0; i < 200; ++i) {
          s.set("k/" + std::to_string(r) + "/" + std::to_string(i), std::string(static_cast<size_t>(i % 97), 'x'));
          s.add("counter", 1);
        }
        s.barrier("phase1");
        for (int j = 0; j < world; ++j) {
          auto v = s.get("k/" + std::to_string(j) + "/150");
          if (v.size() != 150 % 97) failures++;
        }
        if (s.add("counter", 0) != world * 200) failures++;
        s.compare_set("cas", "", "first");
        s.barrier("phase2");
        try {
          s.set_timeout_ms(50);
          s.get("missing-key");
          failures++;
        } catch (const dcp::TimeoutError&) {
        }
      } catch (const std::exception& e) {
        std::fprintf(stderr, "rank %d: %s\n", r, e.what());
        failures++;
      }
    });
  }
  for (auto& t : ts) t.join();
  if (master->compare_set("cas", "", "x") != "first") failures++;
  master.reset();
  std::printf("store_selftest: %s (%d failures)\n", failures == 0 ? "OK" : "FAILED", failures.load());
  return failures == 0 ? 0 : 1;
}
