#include "bootstrap.hpp"

#include <arpa/inet.h>
#include <fcntl.h>
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
// The relay never blocks on one rank: sockets are non-blocking, every rank has an inbound buffer
// (messages are parsed once complete) and an outbound queue written as poll reports POLLOUT, so a
// rank that is itself busy sending a large message to the root cannot stall the others.
struct RelayConn {
  int fd = -1;
  std::vector<char> in;  // bytes received, not yet parsed
  std::deque<std::vector<char>> out;
  size_t outOff = 0;  // bytes of out.front() already sent
};

void enqueue(RelayConn& c, const MsgHeader& h, const char* body) {
  std::vector<char> m(sizeof(h) + h.len);
  std::memcpy(m.data(), &h, sizeof(h));
  if (h.len) std::memcpy(m.data() + sizeof(h), body, h.len);
  c.out.push_back(std::move(m));
}

void rootLoop(int lfd, uint64_t nonce) {
  std::vector<RelayConn> cs;
  std::vector<int> fds;  // accepted ranks' sockets until the relay (cs) owns them
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
    cs.resize(nranks);
    for (int r = 0; r < nranks; ++r) {
      cs[r].fd = fds[r];
      fds[r] = -1;
      setTimeouts(cs[r].fd, 0);  // relay phase: ranks may stay idle indefinitely
      ::fcntl(cs[r].fd, F_SETFL, ::fcntl(cs[r].fd, F_GETFL, 0) | O_NONBLOCK);
    }
    std::vector<std::deque<std::vector<char>>> pending(nranks);  // all-gather contributions per rank
    std::vector<pollfd> pfs(nranks);
    std::vector<char> chunk(1 << 16);
    for (;;) {
      for (int r = 0; r < nranks; ++r)
        pfs[r] = pollfd{cs[r].fd, (short)(POLLIN | (cs[r].out.empty() ? 0 : POLLOUT)), 0};
      if (::poll(pfs.data(), pfs.size(), -1) < 0) {
        if (errno == EINTR) continue;
        throw std::runtime_error("bootstrap root: poll failed");
      }
      for (int r = 0; r < nranks; ++r) {
        RelayConn& c = cs[r];
        if (pfs[r].revents & POLLOUT) {
          while (!c.out.empty()) {
            const std::vector<char>& m = c.out.front();
            ssize_t k = ::send(c.fd, m.data() + c.outOff, m.size() - c.outOff, MSG_NOSIGNAL);
            if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR)) break;
            if (k <= 0) throw std::runtime_error("bootstrap root: send failed");
            c.outOff += (size_t)k;
            if (c.outOff == m.size()) {
              c.out.pop_front();
              c.outOff = 0;
            }
          }
        }
        if (!(pfs[r].revents & (POLLIN | POLLHUP | POLLERR))) continue;
        for (;;) {
          ssize_t k = ::recv(c.fd, chunk.data(), chunk.size(), 0);
          if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
          if (k < 0 && errno == EINTR) continue;
          if (k <= 0) throw std::runtime_error("bootstrap root: a rank has gone");  // the root ends
          c.in.insert(c.in.end(), chunk.data(), chunk.data() + k);
        }
        size_t off = 0;
        while (c.in.size() - off >= sizeof(MsgHeader)) {
          MsgHeader h{};
          std::memcpy(&h, c.in.data() + off, sizeof(h));
          if (c.in.size() - off - sizeof(h) < h.len) break;  // body not complete yet
          const char* body = c.in.data() + off + sizeof(h);
          if (h.kind == kMsgP2P) {
            if (h.peer < 0 || h.peer >= nranks) throw std::runtime_error("bootstrap root: bad destination");
            enqueue(cs[h.peer], MsgHeader{kMsgP2P, r, h.tag, h.len}, body);
          } else {
            pending[r].emplace_back(body, body + h.len);
          }
          off += sizeof(h) + h.len;
        }
        c.in.erase(c.in.begin(), c.in.begin() + (std::ptrdiff_t)off);
      }
      for (;;) {  // every complete all-gather round, in order
        bool ready = true;
        for (int r = 0; r < nranks; ++r) ready = ready && !pending[r].empty();
        if (!ready) break;
        const uint64_t len = pending[0].front().size();
        std::vector<char> all(len * nranks);
        for (int r = 0; r < nranks; ++r) {
          if (pending[r].front().size() != len) throw std::runtime_error("bootstrap root: mismatched round sizes");
          if (len) std::memcpy(all.data() + r * len, pending[r].front().data(), len);
          pending[r].pop_front();
        }
        const MsgHeader out{kMsgAllGather, -1, 0, (uint64_t)all.size()};
        for (int r = 0; r < nranks; ++r) enqueue(cs[r], out, all.data());
      }
    }
  } catch (...) {
  }
  // every socket still open gets closed, so waiting ranks see EOF instead of an open, silent socket
  // (also when the accept phase failed before the relay took the sockets over)
  if (lfd >= 0) ::close(lfd);
  for (int fd : fds)
    if (fd >= 0) ::close(fd);
  for (auto& c : cs)
    if (c.fd >= 0) ::close(c.fd);
}

}  // namespace

// Listen on (addr, port) -- port 0: any -- and run the root thread there; the id names it.
static BootstrapId createRootOn(in_addr a, uint16_t portNet, uint64_t nonce) {
  BootstrapId id{};
  std::memcpy(id.magic, "MSCAMD1", 8);
  int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (lfd < 0) throw std::runtime_error("bootstrap: socket() failed");
  int one = 1;
  setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_addr = a;
  sa.sin_port = portNet;
  if (::bind(lfd, (sockaddr*)&sa, sizeof(sa)) != 0 || ::listen(lfd, 256) != 0) {
    ::close(lfd);
    throw std::runtime_error("bootstrap: bind/listen failed");
  }
  socklen_t sl = sizeof(sa);
  getsockname(lfd, (sockaddr*)&sa, &sl);
  id.nonce = nonce;
  id.addr = sa.sin_addr.s_addr;
  id.port = sa.sin_port;
  std::thread(rootLoop, lfd, id.nonce).detach();
  return id;
}

BootstrapId bootstrapCreateRoot() {
  const char* addrEnv = std::getenv("MSCCLPP_AMD_BOOTSTRAP_ADDR");
  in_addr a{};
  if (!addrEnv || inet_pton(AF_INET, addrEnv, &a) != 1) inet_pton(AF_INET, "127.0.0.1", &a);
  std::random_device rd;
  const uint64_t nonce =
      ((uint64_t)rd() << 32) ^ rd() ^ (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
  return createRootOn(a, 0, nonce);
}

// "ip:port" or "interface:ip:port" (TcpBootstrap::initialize(ifIpPortTrio), bootstrap.cc:232-262):
// every rank derives the same id from the string; rank 0 also runs the root there.  The nonce is
// a hash of the string, so two jobs on different ports never join each other's root.
BootstrapId bootstrapIdFromIpPort(const std::string& trio, bool createRoot) {
  const size_t last = trio.rfind(':');
  if (last == std::string::npos || last + 1 >= trio.size())
    throw std::invalid_argument("bootstrap: expected \"ip:port\" or \"interface:ip:port\", got \"" + trio + "\"");
  std::string ip = trio.substr(0, last);
  const size_t first = ip.rfind(':');
  if (first != std::string::npos) ip = ip.substr(first + 1);  // drop the interface name
  const long port = std::strtol(trio.c_str() + last + 1, nullptr, 10);
  in_addr a{};
  if (port <= 0 || port > 65535 || inet_pton(AF_INET, ip.c_str(), &a) != 1)
    throw std::invalid_argument("bootstrap: bad IPv4 address or port in \"" + trio + "\"");
  uint64_t nonce = 1469598103934665603ull;
  for (char ch : ip + ":" + std::to_string(port)) nonce = (nonce ^ (unsigned char)ch) * 1099511628211ull;
  if (createRoot) return createRootOn(a, htons((uint16_t)port), nonce);
  BootstrapId id{};
  std::memcpy(id.magic, "MSCAMD1", 8);
  id.addr = a.s_addr;
  id.port = htons((uint16_t)port);
  id.nonce = nonce;
  return id;
}

bool bootstrapIdValid(const BootstrapId& id) { return std::memcmp(id.magic, "MSCAMD1", 8) == 0; }

StarBootstrap::StarBootstrap(int rank, int nranks, const BootstrapId& id, int timeoutSec)
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

StarBootstrap::~StarBootstrap() {
  if (fd_ >= 0) ::close(fd_);
}

void StarBootstrap::readOne() {
  MsgHeader h{};
  recvAll(fd_, &h, sizeof(h));
  std::vector<char> body(h.len);
  if (h.len) recvAll(fd_, body.data(), h.len);
  std::lock_guard<std::mutex> lk(mu_);
  if (h.kind == kMsgAllGather)
    agResults_.push_back(std::move(body));
  else
    mailbox_[{h.peer, (int)h.tag}].push_back(std::move(body));
}

template <typename Ready>
void StarBootstrap::waitFor(Ready ready) {
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    if (ready()) return;
    if (!reading_) {
      reading_ = true;
      lk.unlock();
      try {
        readOne();
      } catch (...) {
        lk.lock();
        reading_ = false;
        cv_.notify_all();
        throw;
      }
      lk.lock();
      reading_ = false;
      cv_.notify_all();
    } else {
      cv_.wait(lk);
    }
  }
}

void StarBootstrap::allGather(const void* send, void* recv, size_t bytes) {
  std::lock_guard<std::mutex> round(agMu_);
  {
    std::lock_guard<std::mutex> lk(sendMu_);
    MsgHeader h{kMsgAllGather, -1, 0, (uint64_t)bytes};
    sendAll(fd_, &h, sizeof(h));
    if (bytes) sendAll(fd_, send, bytes);
  }
  std::vector<char> all;
  waitFor([&] {
    if (agResults_.empty()) return false;
    all = std::move(agResults_.front());
    agResults_.pop_front();
    return true;
  });
  if (all.size() != bytes * (size_t)nranks_) throw std::runtime_error("bootstrap: unexpected all-gather result");
  if (!all.empty()) std::memcpy(recv, all.data(), all.size());
}

void StarBootstrap::send(const void* data, size_t bytes, int peer, int tag) {
  if (peer < 0 || peer >= nranks_) throw std::invalid_argument("bootstrap send: bad peer");
  std::lock_guard<std::mutex> lk(sendMu_);
  MsgHeader h{kMsgP2P, peer, tag, (uint64_t)bytes};
  sendAll(fd_, &h, sizeof(h));
  if (bytes) sendAll(fd_, data, bytes);
}

void StarBootstrap::recv(void* data, size_t bytes, int peer, int tag) {
  if (peer < 0 || peer >= nranks_) throw std::invalid_argument("bootstrap recv: bad peer");
  const auto key = std::make_pair(peer, tag);
  std::vector<char> m;
  waitFor([&] {  // under mu_: take the message in the same critical section that found it
    auto it = mailbox_.find(key);
    if (it == mailbox_.end() || it->second.empty()) return false;
    m = std::move(it->second.front());
    it->second.pop_front();
    return true;
  });
  if (m.size() != bytes)
    throw std::runtime_error("bootstrap recv: message from rank " + std::to_string(peer) + " tag " +
                             std::to_string(tag) + " has " + std::to_string(m.size()) + " bytes, expected " +
                             std::to_string(bytes));
  if (bytes) std::memcpy(data, m.data(), bytes);
}

void StarBootstrap::barrier() {
  char dummy = 0;
  std::vector<char> all(nranks_);
  allGather(&dummy, all.data(), 1);
}

void StarBootstrap::broadcast(void* buf, size_t bytes, int root) {
  std::vector<char> all(bytes * nranks_);
  allGather(buf, all.data(), bytes);
  std::memcpy(buf, all.data() + (size_t)root * bytes, bytes);
}

}  // namespace mscclpp_amd
