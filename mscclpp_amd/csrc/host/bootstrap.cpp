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

// Wire header of every message after the hello, in both directions.
//   rank -> root: kind 1 = all-gather contribution (peer unused); kind 2 = send to `peer` with `tag`
//   root -> rank: kind 1 = all-gather result (n contributions); kind 2 = delivery from `peer`
struct MsgHeader {
  uint32_t kind;
  int32_t peer;
  int64_t tag;
  uint64_t len;
};
constexpr uint32_t kMsgAllGather = 1, kMsgP2P = 2;

// Root: accept nranks ranks, then serve messages until a rank disconnects: all-gather rounds
// complete when every rank has contributed (in order), point-to-point messages are forwarded at once.
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
    std::vector<std::deque<std::vector<char>>> pending(nranks);  // all-gather contributions per rank
    std::vector<pollfd> pfs(nranks);
    for (;;) {
      for (int r = 0; r < nranks; ++r) pfs[r] = pollfd{fds[r], POLLIN, 0};
      if (::poll(pfs.data(), pfs.size(), -1) < 0) {
        if (errno == EINTR) continue;
        throw std::runtime_error("bootstrap root: poll failed");
      }
      for (int r = 0; r < nranks; ++r) {
        if (!(pfs[r].revents & (POLLIN | POLLHUP | POLLERR))) continue;
        MsgHeader h{};
        recvAll(fds[r], &h, sizeof(h));  // throws when the rank has gone: the root ends
        std::vector<char> body(h.len);
        if (h.len) recvAll(fds[r], body.data(), h.len);
        if (h.kind == kMsgP2P) {
          if (h.peer < 0 || h.peer >= nranks) throw std::runtime_error("bootstrap root: bad destination");
          MsgHeader out{kMsgP2P, r, h.tag, h.len};
          sendAll(fds[h.peer], &out, sizeof(out));
          if (h.len) sendAll(fds[h.peer], body.data(), h.len);
        } else {
          pending[r].push_back(std::move(body));
        }
      }
      bool ready = true;
      for (int r = 0; r < nranks; ++r) ready = ready && !pending[r].empty();
      if (!ready) continue;
      const uint64_t len = pending[0].front().size();
      std::vector<char> all(len * nranks);
      for (int r = 0; r < nranks; ++r) {
        if (pending[r].front().size() != len) throw std::runtime_error("bootstrap root: mismatched round sizes");
        if (len) std::memcpy(all.data() + r * len, pending[r].front().data(), len);
        pending[r].pop_front();
      }
      MsgHeader out{kMsgAllGather, -1, 0, (uint64_t)all.size()};
      for (int r = 0; r < nranks; ++r) {
        sendAll(fds[r], &out, sizeof(out));
        if (!all.empty()) sendAll(fds[r], all.data(), all.size());
      }
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

TcpBootstrap::TcpBootstrap(int rank, int nranks, const BootstrapId& id, int timeoutSec)
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

TcpBootstrap::~TcpBootstrap() {
  if (fd_ >= 0) ::close(fd_);
}

bool TcpBootstrap::readOne(void* agOut, size_t agBytes) {
  MsgHeader h{};
  recvAll(fd_, &h, sizeof(h));
  if (h.kind == kMsgAllGather) {
    if (h.len != agBytes) throw std::runtime_error("bootstrap: unexpected all-gather result");
    if (agBytes) recvAll(fd_, agOut, agBytes);
    return true;
  }
  std::vector<char> body(h.len);
  if (h.len) recvAll(fd_, body.data(), h.len);
  mailbox_[{h.peer, (int)h.tag}].push_back(std::move(body));
  return false;
}

void TcpBootstrap::allGather(const void* send, void* recv, size_t bytes) {
  std::lock_guard<std::mutex> lk(mu_);
  MsgHeader h{kMsgAllGather, -1, 0, (uint64_t)bytes};
  sendAll(fd_, &h, sizeof(h));
  if (bytes) sendAll(fd_, send, bytes);
  while (!readOne(recv, bytes * nranks_)) {
  }
}

void TcpBootstrap::send(const void* data, size_t bytes, int peer, int tag) {
  if (peer < 0 || peer >= nranks_) throw std::invalid_argument("bootstrap send: bad peer");
  std::lock_guard<std::mutex> lk(mu_);
  MsgHeader h{kMsgP2P, peer, tag, (uint64_t)bytes};
  sendAll(fd_, &h, sizeof(h));
  if (bytes) sendAll(fd_, data, bytes);
}

void TcpBootstrap::recv(void* data, size_t bytes, int peer, int tag) {
  if (peer < 0 || peer >= nranks_) throw std::invalid_argument("bootstrap recv: bad peer");
  std::lock_guard<std::mutex> lk(mu_);
  const auto key = std::make_pair(peer, tag);
  for (;;) {
    auto it = mailbox_.find(key);
    if (it != mailbox_.end() && !it->second.empty()) {
      std::vector<char> m = std::move(it->second.front());
      it->second.pop_front();
      if (m.size() != bytes)
        throw std::runtime_error("bootstrap recv: message from rank " + std::to_string(peer) + " tag " +
                                 std::to_string(tag) + " has " + std::to_string(m.size()) + " bytes, expected " +
                                 std::to_string(bytes));
      if (bytes) std::memcpy(data, m.data(), bytes);
      return;
    }
    if (readOne(nullptr, 0)) throw std::runtime_error("bootstrap recv: all-gather result while receiving");
  }
}

void TcpBootstrap::barrier() {
  char dummy = 0;
  std::vector<char> all(nranks_);
  allGather(&dummy, all.data(), 1);
}

void TcpBootstrap::broadcast(void* buf, size_t bytes, int root) {
  std::vector<char> all(bytes * nranks_);
  allGather(buf, all.data(), bytes);
  std::memcpy(buf, all.data() + (size_t)root * bytes, bytes);
}

}  // namespace mscclpp_amd
