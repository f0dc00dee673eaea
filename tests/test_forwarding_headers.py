"""Every forwarding header under include/mscclpp/ (the reference's include paths)
compiles on its own and together with all the others for gfx950 (host and device passes), and
names resolve through namespace mscclpp as the reference's callers spell them.  CPU only: hipcc
-fsyntax-only, no GPU needed."""
import concurrent.futures as cf
import glob
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# what a reference caller writes after including everything (one name per header family)
SPELLINGS = """
static_assert(sizeof(mscclpp::LL16Packet) == 16, "");
static_assert(sizeof(mscclpp::LL8Packet) == 8, "");
using A = mscclpp::MemoryChannelDeviceHandle;
using B = mscclpp::PortChannelDeviceHandle;
using C = mscclpp::BaseMemoryChannelDeviceHandle;
using D = mscclpp::MemoryDevice2DeviceSemaphoreDeviceHandle;
using E = mscclpp::Host2DeviceSemaphoreDeviceHandle;
using F = mscclpp::FifoDeviceHandle;
using G = mscclpp::DeviceSyncer;
using H = mscclpp::DeviceSemaphore;
using I = mscclpp::TcpBootstrap;
using J = mscclpp::Communicator;
using K = mscclpp::Context;
using L = mscclpp::Endpoint;
using M = mscclpp::SemaphoreStub;
using N = mscclpp::ProxyService;
using O = mscclpp::MemoryChannel;
using P = mscclpp::Executor;
using Q = mscclpp::ExecutionPlan;
using R = mscclpp::collective::AlgorithmCollectionBuilder;
using S = mscclpp::GpuBuffer<int>;
using T = mscclpp::Host2HostSemaphore;
static_assert(MSCCLPP_BULK_AVAILABLE == 0, "no Hopper bulk copies on gfx950");
using U = mscclpp::BulkBarrier;
static const mscclpp::PacketType kPt = mscclpp::PacketType::LL8;
static const mscclpp::DataType kDt = mscclpp::DataType::FLOAT8_E4M3B15;
__global__ void k(mscclpp::MemoryChannelDeviceHandle* h) { h->putPackets<mscclpp::LL16Packet>(0, 0, 64, threadIdx.x, blockDim.x, 1); }
// atomic_device.hpp / poll_device.hpp / assert_device.hpp spellings, as port_channel_device.hpp:28 and
// concurrency_device.hpp:54 use them
__global__ void k2(uint64_t* flushDonePos, uint64_t fifoPos, unsigned int* count) {
  POLL_MAYBE_JAILBREAK((mscclpp::atomicLoad<uint64_t, mscclpp::scopeSystem>(flushDonePos, mscclpp::memoryOrderAcquire) <= fifoPos), 1000000);
  OR_POLL_MAYBE_JAILBREAK(*count == 0, *count == 1, -1);
  mscclpp::atomicStore(count, 1u, mscclpp::memoryOrderRelaxed);
  (void)mscclpp::atomicFetchAdd<unsigned int, mscclpp::scopeDevice>(count, 1u, mscclpp::memoryOrderAcqRel);
  MSCCLPP_ASSERT_DEVICE(*count > 0, "count");
}
int main() {
  try {
    throw mscclpp::Error("x", mscclpp::ErrorCode::InvalidUsage);
  } catch (const mscclpp::BaseError& e) {
    if (e.getErrorCode() != (int)mscclpp::ErrorCode::InvalidUsage) return 1;
  }
  try {
    throw mscclpp::CudaError("y", 1);
  } catch (const mscclpp::BaseError&) {
  }
  std::size_t seed = 0;
  mscclpp::detail::hashCombine(seed, 42);
  (void)mscclpp::getDeviceNumaNode(0);
  if (mscclpp::getIBDeviceCount() != 0 || mscclpp::isFabricMemHandleAvailable()) return 1;
  if (mscclpp::getHostName(1024, '.').empty()) return 1;
  if (mscclpp::env()->logLevel.empty() || mscclpp::env()->ibGidIndex < 0) return 1;
  return mscclpp::errorToString(mscclpp::ErrorCode::Timeout) == "Timeout" ? 0 : 1;
}
"""


def _headers():
    return sorted(os.path.relpath(p, INC) for p in glob.glob(os.path.join(INC, "mscclpp", "**", "*.h*"), recursive=True))


def _check(src):
    with tempfile.NamedTemporaryFile("w", suffix=".hip", delete=False) as f:
        f.write(src)
        path = f.name
    try:
        r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-x", "hip", "-std=c++17", "-fsyntax-only", "-I" + INC,
                            path], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
        return r.returncode, r.stdout
    finally:
        os.unlink(path)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="no hipcc")
def test_each_forwarding_header_compiles_alone():
    hdrs = [h for h in _headers() if not h.endswith("namespace.hpp")]
    assert len(hdrs) >= 19, hdrs
    with cf.ThreadPoolExecutor(max_workers=6) as ex:
        res = list(ex.map(lambda h: (h, _check(f"#include <{h}>\nint main() {{ return 0; }}\n")), hdrs))
    bad = [(h, out[-800:]) for h, (rc, out) in res if rc != 0]
    assert not bad, bad


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="no hipcc")
def test_all_forwarding_headers_together_with_reference_spellings():
    src = "".join(f"#include <{h}>\n" for h in _headers()) + SPELLINGS
    rc, out = _check(src)
    assert rc == 0, out[-3000:]
