// TCP bootstrap for the setup plane (runs once per communicator; never on the data path).
//
// Replaces the reference's TcpBootstrap (src/core/bootstrap/bootstrap.cc:169-611): same job --
// a 128-byte unique id names a rendezvous point, ranks exchange small blobs through it -- but a
// simpler shape for the single-node scope: the process that creates the id runs a root thread
// that every rank connects to (a star), and all collective exchanges (all-gather, barrier,
// broadcast) are rounds relayed by that thread.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace mscclpp_amd {

struct BootstrapId {
  char magic[8];      // "MSCAMD1\0"
  uint32_t addr;      // IPv4, network byte order
  uint16_t port;      // network byte order
  uint16_t pad;
  uint64_t nonce;
  char reserved[128 - 24];
};
static_assert(sizeof(BootstrapId) == 128, "unique id must be 128 bytes (nccl.h:21-24)");

// Creates a listening root (a detached thread in this process) and returns its id.
BootstrapId bootstrapCreateRoot();
bool bootstrapIdValid(const BootstrapId& id);

class Bootstrap {
 public:
  Bootstrap(int rank, int nranks, const BootstrapId& id, int timeoutSec);
  ~Bootstrap();
  Bootstrap(const Bootstrap&) = delete;
  Bootstrap& operator=(const Bootstrap&) = delete;

  int rank() const { return rank_; }
  int nranks() const { return nranks_; }
  // recv receives nranks * bytes, rank r's contribution at r * bytes.
  void allGather(const void* send, void* recv, size_t bytes);
  void barrier();
  void broadcast(void* buf, size_t bytes, int root);

 private:
  int rank_;
  int nranks_;
  int fd_;
};

}  // namespace mscclpp_amd
