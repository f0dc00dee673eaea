// TCP bootstrap for the setup plane (runs once per communicator; never on the data path).
//
// Replaces the reference's TcpBootstrap (src/core/bootstrap/bootstrap.cc:169-611): same job --
// a 128-byte unique id names a rendezvous point, ranks exchange small blobs through it -- but a
// simpler shape for the single-node scope: the process that creates the id runs a root thread
// that every rank connects to (a star).  Collective exchanges (all-gather, barrier, broadcast) are
// rounds relayed by that thread; point-to-point messages (send / recv matched by source and tag,
// bootstrap.cc:537-560) are forwarded by it to their destination, where they wait in a mailbox until
// received.
#pragma once

#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <deque>
#include <map>
#include <mutex>
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
// The id of "ip:port" / "interface:ip:port"; createRoot: also listen there (the caller is rank 0).
BootstrapId bootstrapIdFromIpPort(const std::string& ifIpPortTrio, bool createRoot);
bool bootstrapIdValid(const BootstrapId& id);

class StarBootstrap {
 public:
  StarBootstrap(int rank, int nranks, const BootstrapId& id, int timeoutSec);
  ~StarBootstrap();
  StarBootstrap(const StarBootstrap&) = delete;
  StarBootstrap& operator=(const StarBootstrap&) = delete;

  int rank() const { return rank_; }
  int nranks() const { return nranks_; }
  // recv receives nranks * bytes, rank r's contribution at r * bytes.
  void allGather(const void* send, void* recv, size_t bytes);
  void barrier();
  void broadcast(void* buf, size_t bytes, int root);
  // Point-to-point: send never waits for the receiver; recv returns the oldest message from `peer`
  // with `tag` (throws if its size differs from `bytes`).
  void send(const void* data, size_t bytes, int peer, int tag);
  void recv(void* data, size_t bytes, int peer, int tag);

 private:
  // Read one message from the root (the caller holds the reader role, not mu_): point-to-point
  // deliveries go to the mailbox, all-gather results to agResults_.
  void readOne();
  // Wait until `ready()` (called under mu_) holds, taking the reader role while nobody else has it,
  // so a thread blocked in a socket read never holds mu_ and other threads' sends proceed.
  template <typename Ready>
  void waitFor(Ready ready);
  int rank_;
  int nranks_;
  int fd_;
  std::mutex sendMu_;  // one writer of the socket at a time
  std::mutex agMu_;    // one all-gather round at a time (results arrive in round order)
  std::mutex mu_;      // mailbox_, agResults_, reading_
  std::condition_variable cv_;
  bool reading_ = false;
  std::map<std::pair<int, int>, std::deque<std::vector<char>>> mailbox_;
  std::deque<std::vector<char>> agResults_;
};

}  // namespace mscclpp_amd
