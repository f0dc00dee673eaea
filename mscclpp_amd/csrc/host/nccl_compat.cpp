// The rest of the NCCL ABI surface a framework binds (the symbols libtorch_hip.so imports), so that
// libmscclpp_amd.so can stand in for librccl.so under LD_PRELOAD / LD_AUDIT:
//
//  * native here: ncclBroadcast / ncclBcast (zero-copy pull from the root), ncclCommSplit
//    (nccl.cc:405-435), ncclCommInitRankScalable with one id, ncclCommRegister / Deregister and
//    ncclCommWindowRegister / Deregister (the path registers buffers lazily on first use, so these
//    only hand the pointer back);
//  * forwarded to the vendor library when MSCCLPP_AMD_NCCL_LIB_PATH (or the reference's
//    MSCCLPP_NCCL_LIB_PATH) names it -- the reference's dlopen fallback, nccl.cc:72-160, :323-346:
//    ncclReduce, ncclSend/Recv, ncclAllToAll(v), ncclRedOpCreatePreMulSum/Destroy,
//    ncclGroupSimulateEnd, group calls, and AllReduce / AllGather / ReduceScatter / Broadcast for
//    data types and operations this path does not carry or that
//    MSCCLPP_AMD_FORCE_NCCL_FALLBACK_OPERATION (reference: MSCCLPP_FORCE_NCCL_FALLBACK_OPERATION,
//    "all" or a comma list) forces there.  Without a vendor library they return ncclInternalError,
//    as the reference does for the same cases.
#include <dlfcn.h>
#include <sys/stat.h>

#include <algorithm>

#include "comm_internal.hpp"

namespace mscclpp_amd {
namespace host {

namespace {

template <typename F>
void bind(void* h, F& f, const char* name) {
  f = reinterpret_cast<F>(dlsym(h, name));
}

VendorNccl* loadVendor() {
  const char* path = std::getenv("MSCCLPP_AMD_NCCL_LIB_PATH");
  if (!path || !*path) path = std::getenv("MSCCLPP_NCCL_LIB_PATH");
  if (!path || !*path) return nullptr;
  struct stat st{};
  if (stat(path, &st) == 0 && S_ISDIR(st.st_mode)) {
    warn(std::string("MSCCLPP_AMD_NCCL_LIB_PATH points to a directory: ") + path);
    return nullptr;
  }
  // RTLD_DEEPBIND: the vendor library's own calls bind to itself, not to the symbols this library
  // interposes (nccl.cc:91)
  void* h = dlopen(path, RTLD_LAZY | RTLD_LOCAL | RTLD_NODELETE | RTLD_DEEPBIND);
  if (!h) {
    warn(std::string("cannot open the vendor NCCL library: ") + dlerror());
    return nullptr;
  }
  auto* v = new VendorNccl();
  bind(h, v->GetUniqueId, "ncclGetUniqueId");
  bind(h, v->CommInitRank, "ncclCommInitRank");
  bind(h, v->CommDestroy, "ncclCommDestroy");
  bind(h, v->CommFinalize, "ncclCommFinalize");
  bind(h, v->CommAbort, "ncclCommAbort");
  bind(h, v->AllReduce, "ncclAllReduce");
  bind(h, v->AllGather, "ncclAllGather");
  bind(h, v->ReduceScatter, "ncclReduceScatter");
  bind(h, v->Broadcast, "ncclBroadcast");
  bind(h, v->Reduce, "ncclReduce");
  bind(h, v->Send, "ncclSend");
  bind(h, v->Recv, "ncclRecv");
  bind(h, v->AllToAll, "ncclAllToAll");
  bind(h, v->AllToAllv, "ncclAllToAllv");
  bind(h, v->GroupStart, "ncclGroupStart");
  bind(h, v->GroupEnd, "ncclGroupEnd");
  bind(h, v->GroupSimulateEnd, "ncclGroupSimulateEnd");
  bind(h, v->RedOpCreatePreMulSum, "ncclRedOpCreatePreMulSum");
  bind(h, v->RedOpDestroy, "ncclRedOpDestroy");
  if (!v->GetUniqueId || !v->CommInitRank || !v->CommDestroy || !v->GroupStart || !v->GroupEnd) {
    warn(std::string("the vendor NCCL library lacks core entry points: ") + path);
    delete v;
    return nullptr;
  }
  return v;
}

}  // namespace

const VendorNccl* vendorNccl() {
  static VendorNccl* v = loadVendor();
  return v;
}

bool forcedFallback(const char* op) {
  const char* e = std::getenv("MSCCLPP_AMD_FORCE_NCCL_FALLBACK_OPERATION");
  if (!e || !*e) e = std::getenv("MSCCLPP_FORCE_NCCL_FALLBACK_OPERATION");
  if (!e || !*e) return false;
  const std::string list(e);
  if (list == "all") return true;
  size_t pos = 0;
  while (pos <= list.size()) {
    const size_t next = std::min(list.find(',', pos), list.size());
    if (list.compare(pos, next - pos, op) == 0 && next - pos == std::strlen(op)) return true;
    pos = next + 1;
  }
  return false;
}

void initFallbackComm(ncclComm* c) {
  const VendorNccl* v = vendorNccl();
  if (!v) return;
  ncclUniqueId id{};
  if (c->rank == 0 && v->GetUniqueId(&id) != ncclSuccess) std::memset(&id, 0, sizeof(id));
  std::vector<ncclUniqueId> ids((size_t)c->nranks);
  c->boot->allGather(&id, ids.data(), sizeof(ncclUniqueId));  // rank 0's id to everyone (nccl.cc:332-337)
  ncclComm_t fb = nullptr;
  const ncclResult_t r = v->CommInitRank(&fb, c->nranks, ids[0], c->rank);
  if (r != ncclSuccess) {
    // e.g. several ranks on one device, which the vendor library refuses: run without fallback
    warn("vendor NCCL communicator unavailable (code " + std::to_string((int)r) +
         "); operations outside this path will return ncclInternalError");
    return;
  }
  c->fallback = fb;
}

void destroyFallbackComm(ncclComm* c, bool abort) {
  const VendorNccl* v = vendorNccl();
  if (!v || !c->fallback) return;
  ncclComm_t fb = (ncclComm_t)c->fallback;
  if (abort && v->CommAbort)
    (void)v->CommAbort(fb);
  else
    (void)v->CommDestroy(fb);
  c->fallback = nullptr;
}

}  // namespace host
}  // namespace mscclpp_amd

using mscclpp_amd::host::forcedFallback;
using mscclpp_amd::host::vendorNccl;

// The vendor communicator of `comm`, or null (no vendor library, or it refused this communicator).
static inline ncclComm_t vendorComm(ncclComm_t comm) { return comm ? (ncclComm_t)comm->fallback : nullptr; }

// The reference's answer for an operation it does not carry and cannot forward: ncclInternalError
// with a warning (nccl.cc:521-542, :774-821, :840-844).
static ncclResult_t unavailable(const char* what) {
  warn(std::string(what) + " is not carried by this path and no vendor NCCL library is configured "
                           "(set MSCCLPP_AMD_NCCL_LIB_PATH)");
  return ncclInternalError;
}

extern "C" {

ncclResult_t ncclBroadcast(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype, int root,
                           ncclComm_t comm, void* stream) {
  return (ncclResult_t)guarded([&] {
    if (!comm) return (int)ncclInvalidArgument;
    const size_t bytes = count * ncclTypeBytes(datatype);
    if (comm->nranks == 1) {  // nccl.cc:552-557
      if (sendbuff != recvbuff && bytes)
        HIPCHECK(hipMemcpyAsync(recvbuff, sendbuff, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
      return (int)ncclSuccess;
    }
    if (root < 0 || root >= comm->nranks) return (int)ncclInvalidArgument;
    if ((sendbuff == nullptr && root == comm->rank) || recvbuff == nullptr || bytes == 0)  // nccl.cc:559-564
      return (int)ncclInvalidArgument;
    if (vendorComm(comm) && forcedFallback("broadcast"))
      return (int)vendorNccl()->Broadcast(sendbuff, recvbuff, count, datatype, root, vendorComm(comm), stream);
    return comm->broadcast(sendbuff, recvbuff, bytes, root, 0, 0, (hipStream_t)stream);
  });
}

ncclResult_t ncclBcast(void* buff, size_t count, ncclDataType_t datatype, int root, ncclComm_t comm, void* stream) {
  return ncclBroadcast(buff, buff, count, datatype, root, comm, stream);  // nccl.cc:544-547
}

ncclResult_t ncclCommSplit(ncclComm_t comm, int color, int key, ncclComm_t* newcomm, ncclConfig_t* config) {
  return (ncclResult_t)guarded([&] {
    if (!comm || !newcomm) return (int)ncclInvalidArgument;
    *newcomm = NCCL_COMM_NULL;
    struct Info {
      int color, key, rank;
    };
    std::vector<Info> infos((size_t)comm->nranks);
    Info mine{color, key, comm->rank};
    comm->boot->allGather(&mine, infos.data(), sizeof(Info));
    std::vector<Info> group;
    for (const Info& i : infos)
      if (i.color == color) group.push_back(i);
    std::stable_sort(group.begin(), group.end(), [](const Info& a, const Info& b) {
      return a.key != b.key ? a.key < b.key : a.rank < b.rank;
    });
    int newRank = 0;
    for (size_t i = 0; i < group.size(); ++i)
      if (group[i].rank == comm->rank) newRank = (int)i;
    // the new group's rank 0 creates the id; every rank learns every group's id (nccl.cc:422-430)
    ncclUniqueId id{};
    if (color != NCCL_SPLIT_NOCOLOR && newRank == 0) {
      const ncclResult_t r = ncclGetUniqueId(&id);
      if (r != ncclSuccess) return (int)r;
    }
    std::vector<ncclUniqueId> ids((size_t)comm->nranks);
    comm->boot->allGather(&id, ids.data(), sizeof(ncclUniqueId));
    if (color == NCCL_SPLIT_NOCOLOR) return (int)ncclSuccess;
    return (int)ncclCommInitRankConfig(newcomm, (int)group.size(), ids[(size_t)group.front().rank], newRank, config);
  });
}

ncclResult_t ncclCommInitRankScalable(ncclComm_t* newcomm, int nranks, int myrank, int nId, ncclUniqueId* commIds,
                                      ncclConfig_t* config) {
  if (!newcomm || !commIds || nId < 1) return ncclInvalidArgument;
  if (nId != 1) {
    warn("ncclCommInitRankScalable: one MI355X node needs a single unique id");
    return ncclInvalidUsage;
  }
  return ncclCommInitRankConfig(newcomm, nranks, commIds[0], myrank, config);
}

ncclResult_t ncclReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype, ncclRedOp_t op,
                        int root, ncclComm_t comm, void* stream) {
  return (ncclResult_t)guarded([&] {
    if (!comm) return (int)ncclInvalidArgument;
    if (comm->nranks == 1) {
      const size_t bytes = count * ncclTypeBytes(datatype);
      if (sendbuff != recvbuff && bytes)
        HIPCHECK(hipMemcpyAsync(recvbuff, sendbuff, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
      return (int)ncclSuccess;
    }
    if (vendorComm(comm) && vendorNccl()->Reduce)
      return (int)vendorNccl()->Reduce(sendbuff, recvbuff, count, datatype, op, root, vendorComm(comm), stream);
    return (int)unavailable("ncclReduce");
  });
}

ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      void* stream) {
  if (!comm) return ncclInvalidArgument;
  if (vendorComm(comm) && vendorNccl()->Send)
    return vendorNccl()->Send(sendbuff, count, datatype, peer, vendorComm(comm), stream);
  return unavailable("ncclSend");
}

ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm, void* stream) {
  if (!comm) return ncclInvalidArgument;
  if (vendorComm(comm) && vendorNccl()->Recv)
    return vendorNccl()->Recv(recvbuff, count, datatype, peer, vendorComm(comm), stream);
  return unavailable("ncclRecv");
}

ncclResult_t ncclAllToAll(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype, ncclComm_t comm,
                          void* stream) {
  return (ncclResult_t)guarded([&] {
    if (!comm) return (int)ncclInvalidArgument;
    if (comm->nranks == 1) {  // nccl.cc:796-802
      const size_t bytes = count * ncclTypeBytes(datatype);
      if (sendbuff != recvbuff && bytes)
        HIPCHECK(hipMemcpyAsync(recvbuff, sendbuff, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
      return (int)ncclSuccess;
    }
    if (vendorComm(comm) && vendorNccl()->AllToAll)
      return (int)vendorNccl()->AllToAll(sendbuff, recvbuff, count, datatype, vendorComm(comm), stream);
    return (int)unavailable("ncclAllToAll");
  });
}

ncclResult_t ncclAllToAllv(const void* sendbuff, const size_t sendcounts[], const size_t sdispls[], void* recvbuff,
                           const size_t recvcounts[], const size_t rdispls[], ncclDataType_t datatype, ncclComm_t comm,
                           void* stream) {
  if (!comm) return ncclInvalidArgument;
  if (comm->nranks == 1) {  // nccl.cc:812-818: block 0 to block 0
    return (ncclResult_t)guarded([&] {
      if (!recvcounts || !sdispls || !rdispls) return (int)ncclInvalidArgument;
      const size_t tb = ncclTypeBytes(datatype), bytes = recvcounts[0] * tb;
      if (bytes)
        HIPCHECK(hipMemcpyAsync((char*)recvbuff + rdispls[0] * tb, (const char*)sendbuff + sdispls[0] * tb, bytes,
                                hipMemcpyDeviceToDevice, (hipStream_t)stream));
      return (int)ncclSuccess;
    });
  }
  if (vendorComm(comm) && vendorNccl()->AllToAllv)
    return vendorNccl()->AllToAllv(sendbuff, sendcounts, sdispls, recvbuff, recvcounts, rdispls, datatype,
                                   vendorComm(comm), stream);
  return unavailable("ncclAllToAllv");
}

ncclResult_t ncclRedOpCreatePreMulSum(ncclRedOp_t* op, void* scalar, ncclDataType_t datatype,
                                      ncclScalarResidence_t residence, ncclComm_t comm) {
  if (vendorComm(comm) && vendorNccl()->RedOpCreatePreMulSum)
    return vendorNccl()->RedOpCreatePreMulSum(op, scalar, datatype, residence, vendorComm(comm));
  return unavailable("ncclRedOpCreatePreMulSum");
}

ncclResult_t ncclRedOpDestroy(ncclRedOp_t op, ncclComm_t comm) {
  if (vendorComm(comm) && vendorNccl()->RedOpDestroy) return vendorNccl()->RedOpDestroy(op, vendorComm(comm));
  return unavailable("ncclRedOpDestroy");
}

ncclResult_t ncclGroupSimulateEnd(ncclSimInfo_t* simInfo) {
  if (vendorNccl() && vendorNccl()->GroupSimulateEnd) return vendorNccl()->GroupSimulateEnd(simInfo);
  return unavailable("ncclGroupSimulateEnd");
}

ncclResult_t ncclCommRegister(const ncclComm_t comm, void* buff, size_t size, void** handle) {
  if (!comm || !buff || !size || !handle) return ncclInvalidArgument;
  *handle = buff;  // buffers are registered (IPC-mapped) lazily by the algorithm that first uses them
  return ncclSuccess;
}

ncclResult_t ncclCommDeregister(const ncclComm_t comm, void* handle) {
  if (!comm || !handle) return ncclInvalidArgument;
  return ncclSuccess;
}

ncclResult_t ncclCommWindowRegister(ncclComm_t comm, void* buff, size_t size, ncclWindow_t* win, int) {
  if (!comm || !buff || !size || !win) return ncclInvalidArgument;
  *win = reinterpret_cast<ncclWindow_t>(buff);  // mapped lazily by the algorithm that first uses it
  return ncclSuccess;
}

ncclResult_t ncclCommWindowDeregister(ncclComm_t comm, ncclWindow_t win) {
  if (!comm || !win) return ncclInvalidArgument;
  return ncclSuccess;
}

int mscclppAmdCommVendorComm(ncclComm_t comm, void** vendorComm) {
  if (!comm || !vendorComm) return ncclInvalidArgument;
  *vendorComm = comm->fallback;
  return ncclSuccess;
}

int mscclppAmdCommRegisterBuffer(ncclComm_t comm, void* ptr, void** peers) {
  return guarded([&] {
    if (!comm || !ptr || !peers) return (int)ncclInvalidArgument;
    auto v = comm->cxx->registerMemory(ptr);
    for (int r = 0; r < MSCCLPP_AMD_MAX_RANKS; ++r) peers[r] = r < (int)v.size() ? v[(size_t)r] : nullptr;
    return (int)ncclSuccess;
  });
}

int mscclppAmdCommDeregisterAll(ncclComm_t comm) {
  return guarded([&] {
    if (!comm) return (int)ncclInvalidArgument;
    std::lock_guard<std::mutex> lk(comm->mu);
    comm->dropUserRegistrations();
    return (int)ncclSuccess;
  });
}

// Broadcast for in-process ranks (parity tests): views as for mscclppAmdAllReduceLaunch; input =
// the rank's send buffer (read on the root only), output = its receive buffer, peerInput[root] =
// the root's send buffer.
int mscclppAmdBroadcastLaunch(const mscclppAmdRankView* views, int nviews, int nranks, size_t bytes, int root,
                              int nblocks, int nthreads, uint64_t budgetTicks, void* stream) {
  return guarded([&] {
    if (!views || nviews < 1 || nranks < 2 || nranks > MSCCLPP_AMD_MAX_RANKS || bytes == 0) return (int)ncclInvalidArgument;
    if (nviews != 1 && nviews != nranks) return (int)ncclInvalidArgument;
    if (root < 0 || root >= nranks) return (int)ncclInvalidArgument;
    for (int i = 0; i < nviews; ++i) {
      const mscclppAmdRankView& v = views[i];
      if (!v.output || !v.tokens || !v.expected || !v.err || !v.peerInput[root]) return (int)ncclInvalidArgument;
      if (v.rank == root && !v.input) return (int)ncclInvalidArgument;
      for (int q = 0; q < nranks; ++q)
        if (!v.peerTokens[q]) return (int)ncclInvalidArgument;
    }
    return mscclpp_amd::launchBroadcast(views, nviews, nranks, bytes, root, nblocks, nthreads,
                                        budgetTicks ? budgetTicks : spinBudgetTicks(), (hipStream_t)stream);
  });
}

}  // extern "C"
