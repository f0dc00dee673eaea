// Known-answer tests of the GPU -> host trigger FIFO on the device, restating
// test/unit/fifo_tests.cu:12-162 against FifoDeviceHandle::push / sync and the host Fifo::poll / pop:
//   fifo       10000 pushes (> the FIFO size) with fst = snd = i, the producer syncing every lap;
//              the host pops them concurrently and checks each (fifo_tests.cu:15-66)
//   zero       32 all-zero triggers must round-trip (fifo_tests.cu:84-108)
//   wrap       whole laps of triggers fst = i, snd = ~i with the commit bit cleared by the
//              producer: the consumer must neither stall at a lap boundary nor accept a trigger
//              twice (fifo_tests.cu:110-153)
//   reject     a non-power-of-two size throws Error(InvalidUsage) (fifo_tests.cu:155-162); no GPU
//
//   test_fifo cpu      the rejection test only (touches no GPU)
//   test_fifo gpu      everything
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "mscclpp_amd/fifo.hpp"
#include "mscclpp_amd/proxy.hpp"

namespace mscclpp = mscclpp_amd;  // the kernels below are spelled as against include/mscclpp

#define CHECK(cond)                                                               \
  do {                                                                            \
    if (!(cond)) {                                                                \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)
#define HIP_OK(cmd) CHECK((cmd) == hipSuccess)

#define ITER 10000

__constant__ mscclpp::FifoDeviceHandle gFifoTestFifoDeviceHandle;
__global__ void kernelFifoTest() {
  if (threadIdx.x + blockIdx.x * blockDim.x != 0) return;
  mscclpp::FifoDeviceHandle& fifo = gFifoTestFifoDeviceHandle;
  mscclpp::ProxyTrigger trigger;
  for (uint64_t i = 0; i < ITER; ++i) {
    trigger.fst = i;
    trigger.snd = i;
    uint64_t curFifoHead = fifo.push(trigger);
    if (i % fifo.size == 0) fifo.sync(curFifoHead);
  }
}

__constant__ mscclpp::FifoDeviceHandle gFifoZeroTestHandle;
__global__ void kernelFifoZeroTrigger(int count) {
  if (threadIdx.x + blockIdx.x * blockDim.x != 0) return;
  mscclpp::FifoDeviceHandle& fifo = gFifoZeroTestHandle;
  for (int i = 0; i < count; ++i) {
    mscclpp::ProxyTrigger trigger;
    trigger.fst = 0;
    trigger.snd = 0;
    fifo.push(trigger);
  }
}

__constant__ mscclpp::FifoDeviceHandle gFifoWrapTestHandle;
__global__ void kernelFifoWrap(int laps, int fifoSize) {
  if (threadIdx.x + blockIdx.x * blockDim.x != 0) return;
  mscclpp::FifoDeviceHandle& fifo = gFifoWrapTestHandle;
  for (int i = 0; i < laps * fifoSize; ++i) {
    mscclpp::ProxyTrigger trigger;
    trigger.fst = uint64_t(i);
    trigger.snd = ~uint64_t(i);
    trigger.fields.reserved = 0;  // the FIFO owns this bit
    uint64_t head = fifo.push(trigger);
    if ((i + 1) % fifoSize == 0) fifo.sync(head);
  }
}

static double nowUs() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void testReject() {
  bool threw = false;
  try {
    mscclpp::Fifo fifo(500);
  } catch (const mscclpp::Error& e) {
    threw = e.getErrorCode() == mscclpp::ErrorCode::InvalidUsage;
  }
  CHECK(threw);
  std::printf("reject OK\n");
}

static void testFifo() {
  mscclpp::numaBind(mscclpp::getDeviceNumaNode(0));
  mscclpp::Fifo hostFifo;
  CHECK(hostFifo.size() < ITER);
  mscclpp::FifoDeviceHandle devFifo = hostFifo.deviceHandle();
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(gFifoTestFifoDeviceHandle), &devFifo, sizeof(devFifo)));
  hipLaunchKernelGGL(kernelFifoTest, dim3(1), dim3(1), 0, 0);
  HIP_OK(hipGetLastError());
  mscclpp::ProxyTrigger trigger;
  const double t0 = nowUs();
  for (uint64_t i = 0; i < ITER; ++i) {
    const double p0 = nowUs();
    while (!hostFifo.poll(trigger)) {
      if (nowUs() - p0 > 5e6) {
        std::fprintf(stderr, "polling timed out at trigger %llu\n", (unsigned long long)i);
        std::exit(1);
      }
    }
    CHECK(trigger.fst == i);
    CHECK(trigger.snd == i);
    hostFifo.pop();
  }
  std::printf("fifo OK: %.3f us/iter\n", (nowUs() - t0) / ITER);
  HIP_OK(hipDeviceSynchronize());
}

static void testZero() {
  const int count = 32;
  mscclpp::Fifo hostFifo;
  mscclpp::FifoDeviceHandle devFifo = hostFifo.deviceHandle();
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(gFifoZeroTestHandle), &devFifo, sizeof(devFifo)));
  hipLaunchKernelGGL(kernelFifoZeroTrigger, dim3(1), dim3(1), 0, 0, count);
  HIP_OK(hipGetLastError());
  HIP_OK(hipDeviceSynchronize());  // count is below the capacity: the producer never waits here
  mscclpp::ProxyTrigger trigger;
  for (int i = 0; i < count; ++i) {
    uint64_t spin = 0;
    while (!hostFifo.poll(trigger)) CHECK(spin++ < 1000000);
    CHECK(trigger.fst == 0);
    CHECK(trigger.snd == 0);
    hostFifo.pop();
  }
  // nothing more: the next slot still carries the previous lap's (zero) parity
  CHECK(!hostFifo.poll(trigger));
  std::printf("zero OK\n");
}

static void testWrap() {
  const int laps = 4;
  mscclpp::Fifo hostFifo;
  const int fifoSize = hostFifo.size();
  mscclpp::FifoDeviceHandle devFifo = hostFifo.deviceHandle();
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(gFifoWrapTestHandle), &devFifo, sizeof(devFifo)));
  hipLaunchKernelGGL(kernelFifoWrap, dim3(1), dim3(1), 0, 0, laps, fifoSize);
  HIP_OK(hipGetLastError());
  mscclpp::ProxyTrigger trigger;
  for (int i = 0; i < laps * fifoSize; ++i) {
    uint64_t spin = 0;
    while (!hostFifo.poll(trigger)) {
      if (spin++ > 100000000) {
        std::fprintf(stderr, "polling stuck at position %d (lap %d)\n", i, i / fifoSize);
        std::exit(1);
      }
    }
    CHECK(trigger.fst == uint64_t(i));
    mscclpp::ProxyTrigger expected;
    expected.snd = ~uint64_t(i);
    expected.fields.reserved = 0;
    CHECK(trigger.snd == expected.snd);
    hostFifo.pop();
  }
  HIP_OK(hipDeviceSynchronize());
  CHECK(!hostFifo.poll(trigger));  // no trigger accepted twice after the last lap
  std::printf("wrap OK\n");
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "";
  if (mode == "cpu") {
    testReject();
    return 0;
  }
  if (mode == "gpu") {
    testReject();
    HIP_OK(hipSetDevice(0));
    testFifo();
    testZero();
    testWrap();
    std::printf("gpu OK\n");
    return 0;
  }
  std::fprintf(stderr, "usage: %s cpu | gpu\n", argv[0]);
  return 2;
}
