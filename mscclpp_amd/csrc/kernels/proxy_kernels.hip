// Device side of the host-proxy path (PortChannel / FIFO / Host2Device semaphores).
//
//  hostOffloadKernel  -- the kernel of test/allgather_test_host_offloading.cu:36-50: thread 0
//                        pushes a trigger whose fst names the semaphore set; every thread t != rank
//                        waits on the Host2Device semaphore of peer t.  The proxy thread of this
//                        rank turns the trigger into hipMemcpyAsync writes + remote token updates.
//  portChannelPutKernel -- the generic PortChannel surface: lane 0 of each block issues
//                        put / putWithSignal / putWithSignalAndFlush for its chunk, then waits.
#include "common.hpp"
#include "mscclpp_amd/port_channel_device.hpp"

namespace mscclpp_amd {

__global__ void hostOffloadKernel(int rank, FifoDeviceHandle fifo, Host2DeviceSemaphoreDeviceHandle* handles,
                                  int handleIndex, uint64_t budget, uint32_t* err) {
  const int tid = threadIdx.x;
  fifo.budget = budget;
  fifo.err = err;
  __syncthreads();
  if (tid == 0) {
    ProxyTrigger t;
    t.fst = (uint64_t)handleIndex;
    t.snd = 0;
    fifo.push(t);
  }
  if (tid != rank) {
    Host2DeviceSemaphoreDeviceHandle h = handles[tid];
    h.budget = budget;
    h.err = err;
    h.wait();
  }
}

// mode 0: put + signal per chunk; 1: putWithSignal; 2: putWithSignalAndFlush; then wait for the
// peer's signal (PortChannel ping of test/mp_unit/port_channel_tests.cu:338-446, bulk form).
__global__ void portChannelPutKernel(PortChannelDeviceHandle* chans, int nchans, const uint64_t* dstOffs,
                                     const uint64_t* srcOffs, uint64_t chunk, int mode) {
  const int c = blockIdx.x;
  if (c >= nchans || threadIdx.x != 0) return;
  PortChannelDeviceHandle& ch = chans[c];
  const uint64_t d = dstOffs[c], s = srcOffs[c];
  if (mode == 0) {
    ch.put(d, s, chunk);
    ch.signal();
  } else if (mode == 1) {
    ch.putWithSignal(d, s, chunk);
  } else {
    ch.putWithSignalAndFlush(d, s, chunk);
  }
  ch.wait();
}

// ---- mscclpp-test allreduce1: ring RS + AG driven through the host proxy ------------------------
// test/mscclpp-test/allreduce_test.cu:730-839.  Thread 0 of block 0 drives two PortChannels to the
// next rank on the ring (first round: my buffer -> its scratch; second round: my buffer -> its
// buffer) and waits on the two from the previous rank; every block sums with vectorSum; blocks meet
// at a grid barrier between steps (DeviceSyncer, concurrency_device.hpp:28-69).  Chunk c is
// reduced starting at rank c+1 and ending at its owner c.  The buffers
// are uncached (mscclpp::GpuBuffer on AMD, gpu_utils.hpp:375-376), so the proxy's copy engine and
// every XCD see each other's writes; the barrier adds system-scope release / acquire anyway.
struct GridBarrier {
  uint32_t count;
  uint32_t gen;
};

__device__ __forceinline__ void grid_sync(GridBarrier* gb, uint64_t budget, uint32_t* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t g = __hip_atomic_load(&gb->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    release_sys();  // this workgroup's stores are written back before it arrives
    if (__hip_atomic_fetch_add(&gb->count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
      __hip_atomic_store(&gb->count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&gb->gen, g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      SpinGuard sg(budget);
      while (__hip_atomic_load(&gb->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
        __builtin_amdgcn_s_sleep(1);
        if (sg.expired()) {
          report_error(err, kErrSemaphoreTimeout);
          break;
        }
      }
    }
    acquire_sys();
  }
  __syncthreads();
}

// dst += src over nElem ints, all blocks (vectorSum, allreduce_test.cu:45-68)
__device__ __forceinline__ void ringVectorSum(int* dst, const int* src, size_t nElem) {
  const size_t n4 = nElem / 4, stride = (size_t)blockDim.x * gridDim.x;
  int4* d4 = (int4*)dst;
  const int4* s4 = (const int4*)src;
  for (size_t i = threadIdx.x + (size_t)blockIdx.x * blockDim.x; i < n4; i += stride) {
    int4 a = d4[i];
    const int4 b = s4[i];
    a.x += b.x;
    a.y += b.y;
    a.z += b.z;
    a.w += b.w;
    d4[i] = a;
  }
  for (size_t i = n4 * 4 + threadIdx.x + (size_t)blockIdx.x * blockDim.x; i < nElem; i += stride) dst[i] += src[i];
}

struct RingChannels {
  PortChannelDeviceHandle fstSend, fstRecv, sndSend, sndRecv;
};

__global__ void __launch_bounds__(1024) ringProxyAllReduceKernel(int* buff, const int* scratch, int rank, int worldSize,
                                                                 size_t nelems, RingChannels ch, GridBarrier* gb,
                                                                 uint64_t budget, uint32_t* err) {
  const bool isComm = threadIdx.x == 0 && blockIdx.x == 0;
  const int n = worldSize;
  const size_t chunkNelem = nelems / n;
  const size_t half = chunkNelem / 2, rest = chunkNelem - half;
  // step 1 (:745-751)
  size_t chunkIndex = (rank + n - 1) % n;
  size_t offset = chunkIndex * chunkNelem * sizeof(int);
  if (isComm && chunkNelem > 1) ch.fstSend.putWithSignal(offset, offset, half * sizeof(int));
  // steps 2 .. n-1 (:753-781).  Deviation: the reference has block 0's thread 0 trigger the put of
  // a half-chunk right after ITS OWN share of the vectorSum that produced it, while the other blocks
  // may still be summing that half (:765-772, :790-797, :803-811); the proxy's copy then reads a
  // partly reduced half.  With large halves (256 MiB at 1 GiB, 2 ranks) the copy engine starts
  // before the sum is done and the result is wrong (seen intermittently here).  A grid barrier
  // between every vectorSum and the put of its output closes the race; nothing else changes.
  for (int step = 2; step < n; ++step) {
    if (isComm) {
      if (chunkNelem > 1) {
        ch.fstRecv.wait();
        ch.fstSend.flush();
      }
      ch.fstSend.putWithSignal(offset + half * sizeof(int), offset + half * sizeof(int), rest * sizeof(int));
    }
    grid_sync(gb, budget, err);
    chunkIndex = (rank + n - step) % n;
    offset = chunkIndex * chunkNelem * sizeof(int);
    int* dst = (int*)((char*)buff + offset);
    const int* src = (const int*)((const char*)scratch + offset);
    ringVectorSum(dst, src, half);
    grid_sync(gb, budget, err);  // the first half is reduced everywhere before it is sent
    if (isComm) {
      ch.fstRecv.wait();
      ch.fstSend.flush();
      if (chunkNelem > 1) ch.fstSend.putWithSignal(offset, offset, half * sizeof(int));
    }
    grid_sync(gb, budget, err);
    ringVectorSum(dst + half, src + half, rest);
    grid_sync(gb, budget, err);  // ... and the second half before the next step sends it
  }
  // step n (:783-815)
  if (isComm) {
    if (chunkNelem > 1) {
      ch.fstRecv.wait();
      ch.fstSend.flush();
    }
    ch.fstSend.putWithSignal(offset + half * sizeof(int), offset + half * sizeof(int), rest * sizeof(int));
  }
  grid_sync(gb, budget, err);
  offset = (size_t)rank * chunkNelem * sizeof(int);
  int* dst = (int*)((char*)buff + offset);
  const int* src = (const int*)((const char*)scratch + offset);
  ringVectorSum(dst, src, half);
  grid_sync(gb, budget, err);
  if (isComm) {
    ch.fstRecv.wait();
    ch.fstSend.flush();
    if (chunkNelem > 1) ch.sndSend.putWithSignal(offset, offset, half * sizeof(int));
  }
  grid_sync(gb, budget, err);
  ringVectorSum(dst + half, src + half, rest);
  grid_sync(gb, budget, err);
  if (isComm) {
    if (chunkNelem > 1) {
      ch.sndRecv.wait();
      ch.sndSend.flush();
    }
    ch.sndSend.putWithSignalAndFlush(offset + half * sizeof(int), offset + half * sizeof(int), rest * sizeof(int));
  }
  // steps n+1 .. 2n-2: forward the reduced chunks around the ring (:817-832)
  for (int i = 1; i < n - 1; ++i) {
    if (isComm) ch.sndRecv.wait();
    grid_sync(gb, budget, err);
    chunkIndex = (rank + n - i) % n;
    if (isComm)
      ch.sndSend.putWithSignalAndFlush(chunkIndex * chunkNelem * sizeof(int), chunkIndex * chunkNelem * sizeof(int),
                                       chunkNelem * sizeof(int));
  }
  if (isComm) ch.sndRecv.wait();  // final receive (:834-838)
}

}  // namespace mscclpp_amd

using namespace mscclpp_amd;

extern "C" int mscclppAmdLaunchRingProxyAllReduce(int* buff, const int* scratch, int rank, int nranks, size_t nelems,
                                                  const void* channels4, void* gridBarrier, int nblocks, int nthreads,
                                                  uint64_t budget, uint32_t* err, void* stream) {
  if (!buff || !scratch || !channels4 || !gridBarrier || nranks < 2 || nblocks <= 0 || nthreads <= 0 ||
      nthreads > 1024 || nthreads % 64)
    return 4;
  if (!grid_coresident(ringProxyAllReduceKernel, nthreads, nblocks)) return 5;
  RingChannels ch = *reinterpret_cast<const RingChannels*>(channels4);
  hipLaunchKernelGGL(ringProxyAllReduceKernel, dim3(nblocks), dim3(nthreads), 0, (hipStream_t)stream, buff, scratch,
                     rank, nranks, nelems, ch, (GridBarrier*)gridBarrier, budget, err);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int mscclppAmdLaunchHostOffloadKernel(int rank, int nranks, const void* fifoHandle, void* semHandles,
                                                 int handleIndex, uint64_t budget, uint32_t* err, void* stream) {
  if (!fifoHandle || !semHandles || nranks <= 0 || nranks > 64) return 4;
  FifoDeviceHandle f = *reinterpret_cast<const FifoDeviceHandle*>(fifoHandle);
  hipLaunchKernelGGL(hostOffloadKernel, dim3(1), dim3(nranks), 0, (hipStream_t)stream, rank, f,
                     (Host2DeviceSemaphoreDeviceHandle*)semHandles, handleIndex, budget, err);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// The host proxy's data mover (CudaIpcConnection::write, connection.cc:138-157, moves bytes with
// cudaMemcpyAsync): a CU copy kernel the proxy thread enqueues on the connection stream.  16-byte
// non-temporal loads, system-scope write-through stores (the destination is usually a peer's
// IPC-mapped memory), a byte loop when the ends are not 16-byte aligned.  Stream order keeps the
// token update enqueued after it behind the data.
__global__ void __launch_bounds__(512) proxyCopyKernel(uint8_t* dst, const uint8_t* src, uint64_t bytes) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const bool aligned = (((uintptr_t)dst | (uintptr_t)src) & 15) == 0;
  const uint64_t body = aligned ? bytes / 16 * 16 : 0;
  if (aligned) {
    const uint64_t nUnits = body / 16;
    for (uint64_t u = tid; u < nUnits; u += stride) {
      // 4 GiB buffer windows: rebase the resource every 2^28 units
      const uint64_t base = (u >> 28) << 32;
      const uint32_t off = (uint32_t)((u & ((1ull << 28) - 1)) * 16);
      store16<kSystem>(make_rsrc(dst + base), off, load16<kNonTemporal>(make_rsrc(src + base), off));
    }
  }
  for (uint64_t i = body + tid; i < bytes; i += stride) dst[i] = src[i];
}

extern "C" int mscclppAmdProxyCopy(void* dst, const void* src, size_t bytes, void* stream) {
  if (!dst || !src) return 4;
  if (bytes == 0) return 0;
  const uint64_t units = (bytes + 15) / 16;
  uint64_t nb = (units + 511) / 512;
  if (nb > 1024) nb = 1024;
  hipLaunchKernelGGL(proxyCopyKernel, dim3((uint32_t)nb), dim3(512), 0, (hipStream_t)stream, (uint8_t*)dst,
                     (const uint8_t*)src, (uint64_t)bytes);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int mscclppAmdLaunchPortChannelPut(void* chans, int nchans, const uint64_t* dstOffs, const uint64_t* srcOffs,
                                              uint64_t chunk, int mode, void* stream) {
  if (!chans || !dstOffs || !srcOffs || nchans <= 0 || nchans > 1024) return 4;
  hipLaunchKernelGGL(portChannelPutKernel, dim3(nchans), dim3(64), 0, (hipStream_t)stream,
                     (PortChannelDeviceHandle*)chans, nchans, dstOffs, srcOffs, chunk, mode);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
