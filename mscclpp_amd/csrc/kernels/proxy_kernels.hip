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
  __syncthreads();
  if (tid == 0) {
    ProxyTrigger t;
    t.fst = (uint64_t)handleIndex;
    t.snd = 0;
    fifo.push(t, budget, err);
  }
  if (tid != rank) handles[tid].wait(budget, err);
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

}  // namespace mscclpp_amd

using namespace mscclpp_amd;

extern "C" int mscclppAmdLaunchHostOffloadKernel(int rank, int nranks, const void* fifoHandle, void* semHandles,
                                                 int handleIndex, uint64_t budget, uint32_t* err, void* stream) {
  if (!fifoHandle || !semHandles || nranks <= 0 || nranks > 64) return 4;
  FifoDeviceHandle f = *reinterpret_cast<const FifoDeviceHandle*>(fifoHandle);
  hipLaunchKernelGGL(hostOffloadKernel, dim3(1), dim3(nranks), 0, (hipStream_t)stream, rank, f,
                     (Host2DeviceSemaphoreDeviceHandle*)semHandles, handleIndex, budget, err);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int mscclppAmdLaunchPortChannelPut(void* chans, int nchans, const uint64_t* dstOffs, const uint64_t* srcOffs,
                                              uint64_t chunk, int mode, void* stream) {
  if (!chans || !dstOffs || !srcOffs || nchans <= 0 || nchans > 1024) return 4;
  hipLaunchKernelGGL(portChannelPutKernel, dim3(nchans), dim3(64), 0, (hipStream_t)stream,
                     (PortChannelDeviceHandle*)chans, nchans, dstOffs, srcOffs, chunk, mode);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
