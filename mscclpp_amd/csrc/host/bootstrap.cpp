#include "bootstrap.hpp"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <random>
#include <stdexcept>
#include <thread>

namespace mscclpp_amd {

namespace {

struct Hello {
  uint64_t nonce;
  int32_t rank;
  int32_t nranks;
};

void sendAll(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      throw std::runtime_error("bootstrap: send failed");
    }
    c += k;
    n -= (size_t)k;
  }
}

void recvAll(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    ssize_t k = ::recv(fd, c, n, 0);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      throw std::runtime_error("bootstrap: peer closed or recv timed out");
    }
    c += k;
    n -= (size_t)k;
  }
}

void setTimeouts(int fd, int sec) {
  timeval tv{};
  tv.tv_sec = sec;
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

// Root: accept nranks ranks, then relay all-gather rounds until a rank disconnects.
void rootLoop(int lfd, uint64_t nonce) {
  std::vector<int> fds;
  int nranks = -1;
  try {
    int have = 0;
    while (nranks < 0 || have < nranks) {
      pollfd pf{lfd, POLLIN, 0};
      int r = ::poll(&pf, 1, 600 * 1000);
      if (r <= 0) throw std::runtime_error("bootstrap root: accept timeout");
      int fd = ::accept(lfd, nullptr, nullptr);
      if (fd < 0) continue;
      setTimeouts(fd, 3600);
      Hello h{};
      try {
        recvAll(fd, &h, sizeof(h));
      } catch (...) {
        ::close(fd);
        continue;
      }
      if (h.nonce != nonce || h.nranks <= 0 || h.rank < 0 || h.rank >= h.nranks ||
          (nranks >= 0 && h.nranks != nranks)) {
        ::close(fd);
        continue;
      }
      if (nranks < 0) {
        nranks = h.nranks;
        fds.assign(nranks, -1);
      }
      if (fds[h.rank] >= 0)
        ::close(fds[h.rank]);
      else
        ++have;
      fds[h.rank] = fd;
    }
    ::close(lfd);
    lfd = -1;
    for (int fd : fds) setTimeouts(fd, 0);  // relay phase: ranks may stay idle indefinitely
    // rounds: every rank sends {u64 len, data}; root replies with the concatenation
    std::vector<char> buf;
    for (;;) {
      uint64_t len = 0;
      recvAll(fds[0], &len, sizeof(len));
      buf.resize(len * fds.size());
      recvAll(fds[0], buf.data(), len);
      for (size_t r = 1; r < fds.size(); ++r) {
        uint64_t l2 = 0;
        recvAll(fds[r], &l2, sizeof(l2));
        if (l2 != len) throw std::runtime_error("bootstrap root: mismatched round sizes");
        recvAll(fds[r], buf.data() + r * len, len);
      }
      for (size_t r = 0; r < fds.size(); ++r) sendAll(fds[r], buf.data(), buf.size());
    }
  } catch (...) {
  }
  if (lfd >= 0) ::close(lfd);
  for (int fd : fds)
    if (fd >= 0) ::close(fd);
}

}  // namespace

BootstrapId bootstrapCreateRoot() {
  BootstrapId id{};
  std::memcpy(id.magic, "MSCAMD1", 8);
  const char* addrEnv = std::getenv("MSCCLPP_AMD_BOOTSTRAP_ADDR");
  in_addr a{};
  if (!addrEnv || inet_pton(AF_INET, addrEnv, &a) != 1) inet_pton(AF_INET, "127.0.0.1", &a);
  int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (lfd < 0) throw std::runtime_error("bootstrap: socket() failed");
  int one = 1;
  setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_addr = a;
  sa.sin_port = 0;
  if (::bind(lfd, (sockaddr*)&sa, sizeof(sa)) != 0 || ::listen(lfd, 256) != 0) {
    ::close(lfd);
    throw std::runtime_error("bootstrap: bind/listen failed");
  }
  socklen_t sl = sizeof(sa);
  getsockname(lfd, (sockaddr*)&sa, &sl);
  std::random_device rd;
  id.nonce = ((uint64_t)rd() << 32) ^ rd() ^ (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
  id.addr = sa.sin_addr.s_addr;
  id.port = sa.sin_port;
  std::thread(rootLoop, lfd, id.nonce).detach();
  return id;
}

bool bootstrapIdValid(const BootstrapId& id) { return std::memcmp(id.magic, "MSCAMD1", 8) == 0; }

Bootstrap::Bootstrap(int rank, int nranks, const BootstrapId& id, int timeoutSec)
    : rank_(rank), nranks_(nranks), fd_(-1) {
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_addr.s_addr = id.addr;
  sa.sin_port = id.port;
  auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(timeoutSec);
  for (;;) {
    fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd_ >= 0 && ::connect(fd_, (sockaddr*)&sa, sizeof(sa)) == 0) break;
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
    if (std::chrono::steady_clock::now() > deadline) throw std::runtime_error("bootstrap: cannot reach root");
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  setTimeouts(fd_, timeoutSec);
  Hello h{id.nonce, rank, nranks};
  sendAll(fd_, &h, sizeof(h));
}

Bootstrap::~Bootstrap() {
  if (fd_ >= 0) ::close(fd_);
}

void Bootstrap::allGather(const void* send, void* recv, size_t bytes) {
  uint64_t len = bytes;
  sendAll(fd_, &len, sizeof(len));
  if (bytes) sendAll(fd_, send, bytes);
  if (bytes * nranks_) recvAll(fd_, recv, bytes * nranks_);
}

void Bootstrap::barrier() {
  char dummy = 0;
  std::vector<char> all(nranks_);
  allGather(&dummy, all.data(), 1);
}

void Bootstrap::broadcast(void* buf, size_t bytes, int root) {
  std::vector<char> all(bytes * nranks_);
  allGather(buf, all.data(), bytes);
  std::memcpy(buf, all.data() + (size_t)root * bytes, bytes);
}

}  // namespace mscclpp_amd
