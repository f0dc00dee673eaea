// Host sanitizer driver for the TCP bootstrap (mscclpp_amd/csrc/host/bootstrap.cpp), built with
// -fsanitize=thread or -fsanitize=address,undefined by tests/test_host_sanitizers.py: n ranks as
// threads of one process around one root thread, each running rounds of all-gather, barrier,
// broadcast from a rotating root and point-to-point send / recv around a ring (tags per round),
// every result checked.  Prints "bootstrap stress OK" and returns 0 on success.
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <thread>
#include <vector>

#include "bootstrap.hpp"

using mscclpp_amd::BootstrapId;
using mscclpp_amd::StarBootstrap;

static void rankMain(int rank, int n, BootstrapId id, int rounds, int* bad) {
  try {
    StarBootstrap b(rank, n, id, 60);
    std::vector<int> mine(16), all(16 * n);
    for (int it = 0; it < rounds; ++it) {
      for (int k = 0; k < 16; ++k) mine[k] = rank * 1000 + it * 16 + k;
      b.allGather(mine.data(), all.data(), mine.size() * sizeof(int));
      for (int r = 0; r < n; ++r)
        for (int k = 0; k < 16; ++k)
          if (all[r * 16 + k] != r * 1000 + it * 16 + k) ++*bad;
      b.barrier();
      int root = it % n, val = rank == root ? 7000 + it : -1;
      b.broadcast(&val, sizeof(val), root);
      if (val != 7000 + it) ++*bad;
      const int next = (rank + 1) % n, prev = (rank + n - 1) % n;
      int out = rank * 100 + it, in = -1;
      b.send(&out, sizeof(out), next, it);
      b.recv(&in, sizeof(in), prev, it);
      if (in != prev * 100 + it) ++*bad;
      if (it % 5 == 0) {
        // every rank sends 1 MiB to every peer before receiving any: the relay must keep reading
        // from a rank it cannot yet write to (a blocking relay stalls once the socket buffers fill)
        std::vector<std::vector<int>> big(n, std::vector<int>(1 << 18));
        for (int q = 0; q < n; ++q) {
          if (q == rank) continue;
          for (size_t k = 0; k < big[q].size(); ++k) big[q][k] = rank * 7 + q * 13 + (int)k + it;
          b.send(big[q].data(), big[q].size() * sizeof(int), q, 100000 + it);
        }
        std::vector<int> got(1 << 18);
        for (int q = 0; q < n; ++q) {
          if (q == rank) continue;
          b.recv(got.data(), got.size() * sizeof(int), q, 100000 + it);
          for (size_t k = 0; k < got.size(); k += 4099)
            if (got[k] != q * 7 + rank * 13 + (int)k + it) ++*bad;
        }
        // a second thread waits in recv for a message its peer sends only after an all-gather that
        // needs this rank's main thread: the waiting recv must not hold up this rank's all-gather
        int late = -1;
        std::thread waiter([&] { b.recv(&late, sizeof(late), prev, 200000 + it); });
        std::vector<int> one(1), every(n);
        one[0] = rank;
        b.allGather(one.data(), every.data(), sizeof(int));
        for (int r = 0; r < n; ++r)
          if (every[r] != r) ++*bad;
        const int v = 9000 + rank;
        b.send(&v, sizeof(v), next, 200000 + it);
        waiter.join();
        if (late != 9000 + prev) ++*bad;
      }
    }
    b.barrier();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "rank %d: %s\n", rank, e.what());
    ++*bad;
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 8;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 50;
  const BootstrapId id = mscclpp_amd::bootstrapCreateRoot();
  std::vector<int> bad(n, 0);
  std::vector<std::thread> ts;
  for (int r = 0; r < n; ++r) ts.emplace_back(rankMain, r, n, id, rounds, &bad[r]);
  for (auto& t : ts) t.join();
  int total = 0;
  for (int v : bad) total += v;
  if (total) {
    std::fprintf(stderr, "bootstrap stress: %d mismatches\n", total);
    return 1;
  }
  std::printf("bootstrap stress OK\n");
  return 0;
}
