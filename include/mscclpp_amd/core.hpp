// mscclpp_amd host core API: bootstrap, communicator, registered memory, connections and
// semaphores -- the host half of the include/mscclpp primitive surface for one MI355X node.
//
// Mirrors include/mscclpp/core.hpp:29-975 (same class and member names, argument order and
// meaning), so host code written against the reference ports by changing the namespace:
//   Bootstrap::{getRank,getNranks,getNranksPerNode,send,recv,allGather,barrier}    core.hpp:29-110
//   Transport / TransportFlags / EndpointConfig                                    core.hpp:211-460
//   RegisteredMemory::{data,originalDataPtr,size,transports,serialize,deserialize} core.hpp:585-627
//   Connection::{write,updateAndSync,flush,transport,remoteTransport}              core.hpp:630-689
//   Semaphore (a pair of token memories over a connection)                         core.hpp:691-745
//   Communicator::{bootstrap,registerMemory,sendMemory,recvMemory,connect,
//                  buildSemaphore,remoteRankOf,tagOf}                              core.hpp:812-957
//   DeviceHandle<T>, deviceHandle(t)                                               core.hpp:960-975
//
// MI355X specifics.  One process per GPU, all 8 GPUs of the node in one IPC domain, so the only
// transport is CudaIpc (peer HBM mapped with hipIpcGetMemHandle / hipIpcOpenMemHandle and reached
// over xGMI by shader-core loads/stores, or by the copy engines for Connection::write).  A
// Communicator is a handle over an ncclComm_t of this library (its TCP bootstrap, error word and
// IPC-mapping cache); construct it from one, or let Communicator::create build one.  Futures are
// std::shared_future: the sending half of an exchange happens when the call is made, the receiving
// half when get() is first called (every peer has sent by then if every rank issues its calls in
// the same order, as the reference requires).  Setup calls throw mscclpp_amd::Error.
#ifndef MSCCLPP_AMD_CORE_HPP_
#define MSCCLPP_AMD_CORE_HPP_

#include <hip/hip_runtime_api.h>

#include <array>
#include <cstdint>
#include <future>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "mscclpp_amd/errors.hpp"
#include "mscclpp_amd/nccl.h"

namespace mscclpp_amd {


// ---- bootstrap (core.hpp:29-110) ----------------------------------------------------------------
class Bootstrap {
 public:
  virtual ~Bootstrap() = default;
  virtual int getRank() const = 0;
  virtual int getNranks() const = 0;
  virtual int getNranksPerNode() const = 0;
  // Ranks sharing this rank's GPU IPC domain (bootstrap.cc:459): the whole node here.
  virtual int getNranksPerIpcDomain() const { return getNranksPerNode(); }
  // Point-to-point, matched by (peer, tag); a send never waits for its receive.
  virtual void send(void* data, int size, int peer, int tag) = 0;
  virtual void recv(void* data, int size, int peer, int tag) = 0;
  // In place: allData holds getNranks() * size bytes, this rank's contribution at getRank() * size.
  virtual void allGather(void* allData, int size) = 0;
  virtual void barrier() = 0;
  void send(const std::vector<char>& data, int peer, int tag);  // size-prefixed
  void recv(std::vector<char>& data, int peer, int tag);
};

// The 128-byte rendezvous id (core.hpp:20-24): the ncclUniqueId of this library.
constexpr unsigned int UniqueIdBytes = 128;
using UniqueId = std::array<uint8_t, UniqueIdBytes>;

// TcpBootstrap (core.hpp:113-197).  Ranks meet at a root that the creator of the id runs (a thread
// of createUniqueId()'s process) or, with initialize("ip:port"), that rank 0 runs at that address.
// initialize() also builds this library's communicator for the rank on the current device (the
// IPC-mapped scratch, flags and error word every channel of a Communicator uses), so
// Communicator(bootstrap) shares it; the timeout is MSCCLPP_AMD_BOOTSTRAP_TIMEOUT_S's (default 600 s)
// when timeoutSec is not positive, else timeoutSec.
class TcpBootstrap : public Bootstrap {
 public:
  static UniqueId createUniqueId();
  TcpBootstrap(int rank, int nRanks);
  ~TcpBootstrap() override;
  UniqueId getUniqueId() const;
  void initialize(UniqueId uniqueId, int64_t timeoutSec = 30);
  void initialize(const std::string& ifIpPortTrio, int64_t timeoutSec = 30);
  int getRank() const override;
  int getNranks() const override;
  int getNranksPerNode() const override;
  void send(void* data, int size, int peer, int tag) override;
  void recv(void* data, int size, int peer, int tag) override;
  void allGather(void* allData, int size) override;
  void barrier() override;
  using Bootstrap::recv;
  using Bootstrap::send;
  // The communicator initialize() built (null before).
  ncclComm_t ncclComm() const;

 private:
  struct Impl;
  std::unique_ptr<Impl> pimpl_;
};

// ---- transports and devices (core.hpp:211-466) ---------------------------------------------------
enum class Transport { Unknown, CudaIpc, NumTransports };

class TransportFlags {
 public:
  TransportFlags() = default;
  TransportFlags(Transport t) : bits_(t == Transport::Unknown ? 0u : 1u << (int)t) {}
  bool has(Transport t) const { return (bits_ & TransportFlags(t).bits_) != 0; }
  bool none() const { return bits_ == 0; }
  bool any() const { return bits_ != 0; }
  TransportFlags operator|(TransportFlags o) const { return TransportFlags(bits_ | o.bits_); }
  TransportFlags operator&(TransportFlags o) const { return TransportFlags(bits_ & o.bits_); }
  bool operator==(TransportFlags o) const { return bits_ == o.bits_; }
  bool operator!=(TransportFlags o) const { return bits_ != o.bits_; }

 private:
  explicit TransportFlags(unsigned b) : bits_(b) {}
  unsigned bits_ = 0;
};

enum class DeviceType { Unknown, CPU, GPU };

struct Device {
  Device() = default;
  Device(DeviceType type, int id = -1) : type(type), id(id) {}
  DeviceType type = DeviceType::GPU;
  int id = -1;  // -1: the communicator's GPU
};

// Deviation: the default transport is CudaIpc (the reference's is Unknown), the only one here.
struct EndpointConfig {
  Transport transport = Transport::CudaIpc;
  Device device{DeviceType::GPU};
  int maxWriteQueueSize = -1;
  EndpointConfig() = default;
  EndpointConfig(Transport transport, Device device = DeviceType::GPU, int maxWriteQueueSize = -1)
      : transport(transport), device(device), maxWriteQueueSize(maxWriteQueueSize) {}
};

class Context;
class Connection;
class RegisteredMemory;

// ---- endpoints and contexts (core.hpp:473-545) ----------------------------------------------------
// An endpoint names one side of a connection: a transport and a device of one process on one host.
class Endpoint {
 public:
  Endpoint() = default;
  const EndpointConfig& config() const;
  Transport transport() const;
  const Device& device() const;  // the id resolved to a GPU index
  uint64_t hostHash() const;
  uint64_t pidHash() const;      // the owning process (a random per-process value, not the PID)
  int maxWriteQueueSize() const;
  std::vector<char> serialize() const;
  static Endpoint deserialize(const std::vector<char>& data);
  struct Impl;
  explicit Endpoint(std::shared_ptr<Impl> impl) : pimpl_(std::move(impl)) {}
  bool valid() const { return (bool)pimpl_; }

 private:
  std::shared_ptr<Impl> pimpl_;
};

// ---- registered memory (core.hpp:585-627) -------------------------------------------------------
class RegisteredMemory {
 public:
  RegisteredMemory() = default;
  // Local: the registered pointer.  Received from a peer: the peer's buffer as mapped here (device
  // code may load from and store to it over xGMI).
  void* data() const;
  void* originalDataPtr() const;  // the pointer in the owner's address space
  size_t size() const;
  TransportFlags transports() const;
  int rank() const;  // owner
  // The owner's buffer is coherent with copies made by another agent while a kernel runs: a block
  // of the uncached pool (GpuBuffer, mscclppAmdMallocUncached) or host memory.  A PortChannel
  // destination must be coherent for a running kernel to read what the proxy delivered after
  // wait(); cached device memory (hipMalloc) is guaranteed only to the host and to kernels launched
  // after the receiving one.
  bool coherent() const;
  // Received from another process (data() is this process's mapping of the owner's buffer).
  bool remote() const;
  std::vector<char> serialize() const;
  static RegisteredMemory deserialize(const std::vector<char>& data);
  struct Impl;
  explicit RegisteredMemory(std::shared_ptr<Impl> impl) : pimpl_(std::move(impl)) {}
  bool valid() const { return (bool)pimpl_; }

 private:
  std::shared_ptr<Impl> pimpl_;
};

// ---- connection (core.hpp:630-689) --------------------------------------------------------------
// A host-driven CudaIpc connection to one peer: copies (hipMemcpyAsync, the copy engines) on a
// non-blocking HIP stream of this GPU write into the peer's mapped memory.  All connections of a
// communicator share that stream (as the reference's CUDA build does), so flush() also waits for the
// other connections' copies: HIP multiplexes a process's streams onto four hardware queues, and a
// per-connection stream could land behind a kernel spinning for its own data.
class Connection {
 public:
  Connection() = default;
  // Stream-ordered copy of `size` bytes src[srcOffset..] -> dst[dstOffset..] (dst: a peer's memory).
  void write(RegisteredMemory dst, uint64_t dstOffset, RegisteredMemory src, uint64_t srcOffset, uint64_t size);
  // *src = newValue, then a stream-ordered copy of the value into dst[dstOffset] (8 bytes), after
  // every write issued before it on this connection.
  void updateAndSync(RegisteredMemory dst, uint64_t dstOffset, uint64_t* src, uint64_t newValue);
  // Wait until every write / updateAndSync issued so far has completed (timeoutUsec < 0: no limit).
  void flush(int64_t timeoutUsec = -1);
  Transport transport() const;
  Transport remoteTransport() const;
  std::shared_ptr<Context> context() const;  // the context the connection was made in
  const Device& localDevice() const;
  int getMaxWriteQueueSize() const;
  int remoteRank() const;
  int tag() const;
  hipStream_t stream() const;  // the communicator's shared copy stream
  struct Impl;
  explicit Connection(std::shared_ptr<Impl> impl) : pimpl_(std::move(impl)) {}
  bool valid() const { return (bool)pimpl_; }
  const std::shared_ptr<Impl>& impl() const { return pimpl_; }

 private:
  std::shared_ptr<Impl> pimpl_;
};

// The process-local half of the channel layer (core.hpp:497-545): registrations and connections made
// without a communicator, e.g. between two GPUs driven by one process.  connect() needs both
// endpoints on this host; the remote one may come from another process (Endpoint::deserialize).
// Endpoints of two different GPUs of this process get peer access enabled between them.
class Context : public std::enable_shared_from_this<Context> {
 public:
  static std::shared_ptr<Context> create();
  ~Context();
  RegisteredMemory registerMemory(void* ptr, size_t size, TransportFlags transports);
  Endpoint createEndpoint(EndpointConfig config);
  Connection connect(const Endpoint& localEndpoint, const Endpoint& remoteEndpoint);
  struct Impl;

 private:
  Context();
  std::unique_ptr<Impl> pimpl_;
};

// ---- semaphore (core.hpp:691-745) ---------------------------------------------------------------
// One side's token of a semaphore over a connection (core.hpp:667-690): 8 bytes of uncached device
// memory on the connection's GPU, registered so that it can travel (serialize) to the peer.
class SemaphoreStub {
 public:
  explicit SemaphoreStub(const Connection& connection);
  const RegisteredMemory& memory() const;
  std::vector<char> serialize() const;
  static SemaphoreStub deserialize(const std::vector<char>& data);
  struct Impl;
  explicit SemaphoreStub(std::shared_ptr<Impl> impl) : pimpl_(std::move(impl)) {}
  const std::shared_ptr<Impl>& pimpl() const { return pimpl_; }

 private:
  std::shared_ptr<Impl> pimpl_;
};

// One 64-bit token per side in uncached device memory (semaphore.cc:32-43): localMemory() is the
// token this rank waits on, remoteMemory() the peer's token as mapped here.
class Semaphore {
 public:
  Semaphore() = default;
  // The local stub's token is the one this side waits on, the remote stub's the one it signals.
  Semaphore(const SemaphoreStub& localStub, const SemaphoreStub& remoteStub);
  Connection& connection();
  const Connection& connection() const;
  const RegisteredMemory& localMemory() const;
  const RegisteredMemory& remoteMemory() const;
  struct Impl;
  explicit Semaphore(std::shared_ptr<Impl> impl) : pimpl_(std::move(impl)) {}
  bool valid() const { return (bool)pimpl_; }
  const std::shared_ptr<Impl>& pimpl() const { return pimpl_; }

 private:
  std::shared_ptr<Impl> pimpl_;
};

// ---- communicator (core.hpp:812-957) ------------------------------------------------------------
class Communicator {
 public:
  // A handle over an existing communicator of this library (not owned).
  explicit Communicator(ncclComm_t comm);
  // The reference's constructor (core.hpp:818).  A TcpBootstrap brings the communicator its
  // initialize() built; any other Bootstrap is used to hand rank 0's fresh id to every rank, and the
  // communicator is built here (collective) and owned.  `context` is accepted and ignored.
  explicit Communicator(std::shared_ptr<Bootstrap> bootstrap, std::shared_ptr<Context> context = nullptr);
  ~Communicator();
  Communicator(const Communicator&) = delete;
  Communicator& operator=(const Communicator&) = delete;
  // ncclCommInitRank(nranks, id, rank) on the current device; the communicator owns it.
  static std::shared_ptr<Communicator> create(int rank, int nranks, const ncclUniqueId& id);

  ncclComm_t ncclComm() const { return comm_; }
  int rank() const;
  int nRanks() const;
  int nRanksPerNode() const;  // one MI355X node: == nRanks()
  int device() const;
  std::shared_ptr<Bootstrap> bootstrap();

  RegisteredMemory registerMemory(void* ptr, size_t size, TransportFlags transports);
  void sendMemory(RegisteredMemory memory, int remoteRank, int tag = 0);
  std::shared_future<RegisteredMemory> recvMemory(int remoteRank, int tag = 0);
  std::shared_future<Connection> connect(const EndpointConfig& localConfig, int remoteRank, int tag = 0);
  std::shared_future<Connection> connect(const Endpoint& localEndpoint, int remoteRank, int tag = 0);
  std::shared_ptr<Context> context();  // the context this communicator's connections live in
  std::shared_future<Semaphore> buildSemaphore(const Connection& connection, int remoteRank, int tag = 0);
  int remoteRankOf(const Connection& connection);
  int tagOf(const Connection& connection);

  // Device error word of the communicator: channel handles built from it record wait timeouts here.
  uint32_t* deviceErrorWord() const;
  // Wall-clock bound of every device-side wait (MSCCLPP_AMD_SPIN_TIMEOUT_MS, 10 ns ticks).
  uint64_t spinBudget() const;

  // Collective convenience of this library (the role of registerMemory + sendMemory / recvMemory
  // with every peer): every rank passes its matching buffer (any pointer inside a device
  // allocation) and gets every rank's buffer as mapped in this process (entry [rank()] is `ptr`).
  // Mappings are cached per allocation.
  std::vector<void*> registerMemory(void* ptr);
  // Host-side bootstrap collectives over rank-ordered byte blocks.
  void allGather(const void* sendbuf, void* recvbuf, size_t bytesPerRank);
  void barrier();

 private:
  ncclComm_t comm_;
  bool owned_ = false;
  std::shared_ptr<Bootstrap> bootstrap_;
  std::shared_ptr<Context> context_;
};

// ---- device handles (core.hpp:960-975) ----------------------------------------------------------
template <typename T>
using DeviceHandle = typename T::DeviceHandle;

template <typename T>
DeviceHandle<std::remove_reference_t<T>> deviceHandle(T&& t) {
  return t.deviceHandle();
}

template <typename T>
using PacketPayload = typename T::Payload;

}  // namespace mscclpp_amd

#endif  // MSCCLPP_AMD_CORE_HPP_
