// oracle/_ref harness -- TEST INFRASTRUCTURE ONLY.
//
// Runs the reference's OWN device code on the GPU, compiled where it lies under /root/reference
// (nothing is copied): LL16Packet::write/read and LL8Packet (include/mscclpp/packet_device.hpp),
// copyToPackets / copyFromPackets (include/mscclpp/copy_device.hpp:156-232) and the f16x2 /
// bf16x2 / f32x2 operator+ and min with clip (include/mscclpp/gpu_data_types.hpp:315-420, 588-620).
// reduce_kernel.hpp itself cannot be compiled here (it pulls in algorithm.hpp -> core.hpp ->
// the build-generated mscclpp/version.hpp), so the harness calls the operators that its
// calVectorHelper<T, Op> forwards to (reduce_kernel.hpp:28-134) directly.
//
// Built by oracle/build_ref.sh into oracle/_ref/libref.so; used only by tests/.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <vector>

#include <mscclpp/copy_device.hpp>
#include <mscclpp/gpu_data_types.hpp>
#include <mscclpp/memory_channel_device.hpp>
#include <mscclpp/packet_device.hpp>

using namespace mscclpp;

// calVector<T, Op> on one 32-bit word (reduce_kernel.hpp:91-94, 112-134)
template <int DT, int OP>
__device__ uint32_t refWord(uint32_t a, uint32_t b) {
  if constexpr (DT == 0) {  // __half -> f16x2
    f16x2 x = bit_cast<f16x2, uint32_t>(a), y = bit_cast<f16x2, uint32_t>(b);
    return bit_cast<uint32_t, f16x2>(OP == 0 ? x + y : mscclpp::min(x, y));
  } else if constexpr (DT == 1) {  // __bfloat16 -> bf16x2
    bf16x2 x = bit_cast<bf16x2, uint32_t>(a), y = bit_cast<bf16x2, uint32_t>(b);
    return bit_cast<uint32_t, bf16x2>(OP == 0 ? x + y : mscclpp::min(x, y));
  } else if constexpr (DT == 2) {  // float -> f32x2 scalar specialisation (reduce_kernel.hpp:97-109)
    float x = bit_cast<float, uint32_t>(a), y = bit_cast<float, uint32_t>(b);
    return bit_cast<uint32_t, float>(OP == 0 ? x + y : fminf(x, y));
  } else {  // int
    int x = (int)a, y = (int)b;
    return (uint32_t)(OP == 0 ? x + y : (x < y ? x : y));
  }
}

template <int DT, int OP>
__global__ void refReduceKernel(uint32_t* acc, const uint32_t* val, size_t n) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc[i] = refWord<DT, OP>(acc[i], val[i]);
}

__global__ void refPackLL16(void* pkts, const void* src, uint64_t bytes, uint32_t flag) {
  copyToPackets<LL16Packet>(pkts, src, bytes, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x, flag);
}
__global__ void refPackLL8(void* pkts, const void* src, uint64_t bytes, uint32_t flag) {
  copyToPackets<LL8Packet>(pkts, src, bytes, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x, flag);
}

// O = X (op) read(P, flag): the step-2 loop body of allreducePacket for one peer stream
// (allreduce_packet.cu:93-108) with LL16Packet::read.
template <int DT, int OP>
__global__ void refUnpackReduceLL16(const void* pkts, const uint32_t* x, uint32_t* out, uint64_t npkts, uint32_t flag) {
  const LL16Packet* p = reinterpret_cast<const LL16Packet*>(pkts);
  for (uint64_t i = blockIdx.x * blockDim.x + threadIdx.x; i < npkts; i += (uint64_t)gridDim.x * blockDim.x) {
    uint2 v = p[i].read(flag, 100000000);
    out[2 * i] = refWord<DT, OP>(x[2 * i], v.x);
    out[2 * i + 1] = refWord<DT, OP>(x[2 * i + 1], v.y);
  }
}

// ---- OCP FP8 (built without MSCCLPP_ROCM_FP8_FNUZ: gfx950's native formats) -----------------
// calVectorAccum<T, AccumT, Op> (reduce_kernel.hpp:171-189) restated over the reference's own
// operators: T == AccumT -> calVector (f8x4 operator+ / mscclpp::min, :112-134); otherwise
// mscclpp::to<> upcast, calElements<AccumT> per element (a + b / mscclpp::min), to<> downcast.
template <int DT> struct RefFp8;
template <> struct RefFp8<5> { using T = __fp8_e4m3; using A = __fp8_e4m3; };
template <> struct RefFp8<6> { using T = __fp8_e5m2; using A = __fp8_e5m2; };
template <> struct RefFp8<7> { using T = __fp8_e4m3; using A = __half; };
template <> struct RefFp8<8> { using T = __fp8_e5m2; using A = __half; };
template <> struct RefFp8<9> { using T = __fp8_e4m3; using A = float; };
template <> struct RefFp8<10> { using T = __fp8_e5m2; using A = float; };
// uint8 (u8x4 operator+ / min, gpu_data_types.hpp:577-640) and the software e4m3b15
// (f8_e4m3b15x4 operator+ / min and its to<> conversions, :1008-1300), as dispatchByDtype pairs them
template <> struct RefFp8<11> { using T = uint8_t; using A = uint8_t; };
template <> struct RefFp8<12> { using T = __fp8_e4m3b15; using A = __fp8_e4m3b15; };
template <> struct RefFp8<13> { using T = __fp8_e4m3b15; using A = __half; };
template <> struct RefFp8<14> { using T = __fp8_e4m3b15; using A = float; };

template <int DT, int OP>
__global__ void refFp8AccumKernel(const uint32_t* src, int nsrc, size_t n, uint32_t* out) {
  using T = typename RefFp8<DT>::T;
  using A = typename RefFp8<DT>::A;
  using FromVec = VectorType<T, 4>;
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    if constexpr (std::is_same_v<T, A>) {
      FromVec acc = bit_cast<FromVec, uint32_t>(src[i]);
      for (int k = 1; k < nsrc; ++k) {
        FromVec v = bit_cast<FromVec, uint32_t>(src[(size_t)k * n + i]);
        acc = (OP == 0) ? acc + v : mscclpp::min(acc, v);
      }
      out[i] = bit_cast<uint32_t, FromVec>(acc);
    } else {
      using ToVec = VectorType<A, 4>;
      ToVec acc = mscclpp::to<ToVec>(bit_cast<FromVec, uint32_t>(src[i]));
      for (int k = 1; k < nsrc; ++k) {
        ToVec v = mscclpp::to<ToVec>(bit_cast<FromVec, uint32_t>(src[(size_t)k * n + i]));
#pragma unroll
        for (int e = 0; e < 4; ++e) acc.data[e] = (OP == 0) ? acc.data[e] + v.data[e] : mscclpp::min(acc.data[e], v.data[e]);
      }
      out[i] = bit_cast<uint32_t, FromVec>(mscclpp::to<FromVec>(acc));
    }
  }
}

// The conversions themselves: __fp8_e4m3(float) / __fp8_e5m2(float) and float(fp8) of every byte.
__global__ void refFp8ConvertKernel(const float* in, size_t n, uint8_t* e4, uint8_t* e5, float* d4, float* d5) {
  const size_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    e4[i] = __fp8_e4m3(in[i]).__x;
    e5[i] = __fp8_e5m2(in[i]).__x;
  }
  if (i < 256) {
    __fp8_e4m3 a;
    a.__x = (__hip_fp8_storage_t)i;
    __fp8_e5m2 b;
    b.__x = (__hip_fp8_storage_t)i;
    d4[i] = float(a);
    d5[i] = float(b);
  }
}

// e4m3b15 conversions of the reference, every path of its unit test (gpu_data_types_tests.cu:37-92):
// encode by __fp8_e4m3b15(float) and by to<f8_e4m3b15x4>(f32x4); decode by float() and to<f32x4>.
__global__ void refB15ConvertKernel(const float* in, size_t n, uint8_t* enc, uint8_t* encX4, float* dec,
                                    float* decX4) {
  const size_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) enc[i] = __fp8_e4m3b15(in[i]).__x;
  if (i * 4 + 3 < n) {
    mscclpp::f32x4 v;
    for (int k = 0; k < 4; ++k) v.data[k] = in[i * 4 + k];
    const mscclpp::f8_e4m3b15x4 e = mscclpp::to<mscclpp::f8_e4m3b15x4>(v);
    for (int k = 0; k < 4; ++k) encX4[i * 4 + k] = e.data[k].__x;
  }
  if (i < 256) dec[i] = float(__fp8_e4m3b15::fromRaw((uint8_t)i));
  if (i < 64) {
    mscclpp::f8_e4m3b15x4 r;
    for (int k = 0; k < 4; ++k) r.data[k] = __fp8_e4m3b15::fromRaw((uint8_t)(i * 4 + k));
    const mscclpp::f32x4 f = mscclpp::to<mscclpp::f32x4>(r);
    for (int k = 0; k < 4; ++k) decX4[i * 4 + k] = f.data[k];
  }
}

#define REF_DISPATCH(dtype, op, KERNEL, ...)                                         \
  do {                                                                               \
    int key = (dtype) * 2 + (op);                                                    \
    if (key == 0) hipLaunchKernelGGL((KERNEL<0, 0>), __VA_ARGS__);                   \
    else if (key == 1) hipLaunchKernelGGL((KERNEL<0, 1>), __VA_ARGS__);              \
    else if (key == 2) hipLaunchKernelGGL((KERNEL<1, 0>), __VA_ARGS__);              \
    else if (key == 3) hipLaunchKernelGGL((KERNEL<1, 1>), __VA_ARGS__);              \
    else if (key == 4) hipLaunchKernelGGL((KERNEL<2, 0>), __VA_ARGS__);              \
    else if (key == 5) hipLaunchKernelGGL((KERNEL<2, 1>), __VA_ARGS__);              \
    else if (key == 6) hipLaunchKernelGGL((KERNEL<3, 0>), __VA_ARGS__);              \
    else if (key == 7) hipLaunchKernelGGL((KERNEL<3, 1>), __VA_ARGS__);              \
    else return 4;                                                                   \
  } while (0)

extern "C" {

int refReduceWords(int dtype, int op, uint32_t* acc, const uint32_t* val, size_t nwords, void* stream) {
  REF_DISPATCH(dtype, op, refReduceKernel, dim3(256), dim3(256), 0, (hipStream_t)stream, acc, val, nwords);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int refPack(int ll8, void* pkts, const void* src, uint64_t bytes, uint32_t flag, void* stream) {
  if (ll8)
    hipLaunchKernelGGL(refPackLL8, dim3(256), dim3(256), 0, (hipStream_t)stream, pkts, src, bytes, flag);
  else
    hipLaunchKernelGGL(refPackLL16, dim3(256), dim3(256), 0, (hipStream_t)stream, pkts, src, bytes, flag);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// the 1-GPU self-reduce, reference code path: pack (kernel 1), then unpack + reduce (kernel 2)
int refSelfReduceLL16(int dtype, int op, const void* x, const void* y, void* pkts, void* out, uint64_t bytes,
                      uint32_t flag, void* stream) {
  hipLaunchKernelGGL(refPackLL16, dim3(256), dim3(256), 0, (hipStream_t)stream, pkts, y, bytes, flag);
  REF_DISPATCH(dtype, op, refUnpackReduceLL16, dim3(256), dim3(256), 0, (hipStream_t)stream, (const void*)pkts,
               (const uint32_t*)x, (uint32_t*)out, bytes / 8, flag);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// dst = src[0] (op) ... (op) src[nsrc-1] (src: nsrc arrays of nwords words, back to back), fp8
// reduce type dtype 5..10 (element e4m3/e5m2 x AccumT element/half/float), 11 (uint8) or 12..14
// (e4m3b15 x AccumT element/half/float).
int refFp8Accum(int dtype, int op, const uint32_t* src, int nsrc, size_t nwords, uint32_t* out, void* stream) {
  const int key = dtype * 2 + op;
  hipStream_t s = (hipStream_t)stream;
#define REF_FP8(D)                                                                                          \
  if (key == D * 2) hipLaunchKernelGGL((refFp8AccumKernel<D, 0>), dim3(256), dim3(256), 0, s, src, nsrc, nwords, out); \
  else if (key == D * 2 + 1) hipLaunchKernelGGL((refFp8AccumKernel<D, 1>), dim3(256), dim3(256), 0, s, src, nsrc, nwords, out);
  REF_FP8(5) else REF_FP8(6) else REF_FP8(7) else REF_FP8(8) else REF_FP8(9) else REF_FP8(10)
  else REF_FP8(11) else REF_FP8(12) else REF_FP8(13) else REF_FP8(14) else return 4;
#undef REF_FP8
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int refFp8Convert(const float* in, size_t n, uint8_t* e4, uint8_t* e5, float* d4, float* d5, void* stream) {
  const size_t threads = n > 256 ? n : 256;
  hipLaunchKernelGGL(refFp8ConvertKernel, dim3((threads + 255) / 256), dim3(256), 0, (hipStream_t)stream, in, n, e4, e5,
                     d4, d5);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// n floats -> enc[n] (scalar) and encX4[n] (x4 path, n % 4 == 0); dec[256] / decX4[256] of every byte
int refB15Convert(const float* in, size_t n, uint8_t* enc, uint8_t* encX4, float* dec, float* decX4, void* stream) {
  const size_t threads = n > 256 ? n : 256;
  hipLaunchKernelGGL(refB15ConvertKernel, dim3((threads + 255) / 256), dim3(256), 0, (hipStream_t)stream, in, n, enc,
                     encX4, dec, decX4);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// ---- the reference's own LL16 two-hop AllReduce kernel, run as n ranks on one GPU ------------------
// python/mscclpp_benchmark/allreduce.cu:223-289 (allreduce2; the same algorithm and scratch layout as
// test/mscclpp-test/allreduce_test.cu:972-1034 allreduce6), compiled where it lies by build_ref.sh into
// oracle/_ref/bench_allreduce_int.hsaco with TYPE=int.  Each rank loads its own copy of the code object,
// so each has its own `globalFlag` (initially 1, bumped once per call, as in one process per GPU).  The
// kernel spins on packets from the other ranks, so all n launches must be resident together: one stream
// per rank, and the caller runs with GPU_MAX_HW_QUEUES > 8 so no two streams share a hardware queue.
struct RefBench2 {
  int n = 0;
  int elemBytes = 4;  // sizeof(TYPE) the code object was built with (int / float 4, __half 2)
  std::vector<hipModule_t> mod;
  std::vector<hipFunction_t> fn;
  std::vector<hipFunction_t> fn1;                 // allreduce1 of the same code object
  std::vector<MemoryChannelDeviceHandle*> chans;  // device, n - 1 per rank
};

// One stream per rank for the process's life (so cases do not churn hardware queues), each made to
// own its queue before the first real launch (a queue is created at a stream's first submission);
// plus a stream for diagnostics that never waits behind a spinning rank, and the pinned words it
// copies into (allocated here, never freed: hipHostFree synchronizes the device, which waits forever
// behind a rank that spins).
static hipStream_t gRankStream[8];
static hipStream_t gDiagStream;
static uint64_t* gDiagPinned;
static uint32_t* gMeet;  // uncached device words: [0, 8) arrivals, [8, 16) met
static uint32_t gMeetGen;
static int gStreamRecreations;

static bool createRankStreams() {
  for (auto& s : gRankStream) {
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return false;
    hipLaunchKernelGGL((refReduceKernel<3, 0>), dim3(1), dim3(64), 0, s, nullptr, nullptr, (size_t)0);
    if (hipGetLastError() != hipSuccess) return false;
  }
  for (auto& s : gRankStream)
    if (hipStreamSynchronize(s) != hipSuccess) return false;
  return true;
}

static bool rankStreams() {
  if (gDiagStream) return true;
  if (!createRankStreams()) return false;
  if (hipHostMalloc(reinterpret_cast<void**>(&gDiagPinned), sizeof(uint64_t) * 8, hipHostMallocDefault) !=
          hipSuccess ||
      hipExtMallocWithFlags(reinterpret_cast<void**>(&gMeet), 16 * sizeof(uint32_t), hipDeviceMallocUncached) !=
          hipSuccess ||
      hipMemset(gMeet, 0, 16 * sizeof(uint32_t)) != hipSuccess)
    return false;
  if (hipStreamCreateWithFlags(&gDiagStream, hipStreamNonBlocking) != hipSuccess) return false;
  return hipDeviceSynchronize() == hipSuccess;
}

// The precondition of every launch below: the n ranks spin on each other, so their kernels must run
// at the same time, which two streams behind one hardware queue cannot (the second waits for the
// first to finish).  Each rank stream runs a one-wave kernel that announces itself and waits, at most
// `budget` ticks of the 100 MHz clock, until all n have; met[r] = 1 if it saw them all.
__global__ void refStreamsMeetKernel(uint32_t* meet, int r, int n, uint32_t gen, uint64_t budget) {
  if (threadIdx.x != 0) return;
  __hip_atomic_store(meet + r, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  bool all = false;
  while (!all && __builtin_amdgcn_s_memrealtime() - t0 < budget) {
    all = true;
    for (int q = 0; q < n; ++q)
      all = all && __hip_atomic_load(meet + q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == gen;
    if (!all) __builtin_amdgcn_s_sleep(2);
  }
  __hip_atomic_store(meet + 8 + r, all ? 1u : 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// 0 if rank streams 0 .. n-1 ran the meet kernel concurrently, 5 if not, 1 on a HIP error.  Every
// meet kernel ends by itself (100 ms budget), so this never leaves anything spinning.
static int streamsMeet(int n) {
  const uint32_t gen = ++gMeetGen;
  for (int r = 0; r < n; ++r) {
    hipLaunchKernelGGL(refStreamsMeetKernel, dim3(1), dim3(64), 0, gRankStream[r], gMeet, r, n, gen,
                       (uint64_t)10000000);
    if (hipGetLastError() != hipSuccess) return 1;
  }
  for (int r = 0; r < n; ++r)
    if (hipStreamSynchronize(gRankStream[r]) != hipSuccess) return 1;
  uint32_t met[8] = {};
  if (hipMemcpy(met, gMeet + 8, sizeof(uint32_t) * n, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int r = 0; r < n; ++r)
    if (met[r] != 1) return 5;
  return 0;
}

// streamsMeet, and on a failure fresh rank streams (new queues) and again, twice at most.
static int ensureConcurrent(int n) {
  int rc = streamsMeet(n);
  for (int k = 0; k < 2 && rc == 5; ++k) {
    for (auto& s : gRankStream) (void)hipStreamDestroy(s);
    if (!createRankStreams()) return 1;
    ++gStreamRecreations;
    rc = streamsMeet(n);
  }
  return rc;
}

void refBench2Close(void* handle);

// elemBytes: sizeof(TYPE) of the code object (4 for TYPE=int or float, 2 for __half); the kernel takes
// its buffer length in TYPE elements and divides by sizeof(int) / sizeof(TYPE) itself (:229).
void* refBench2OpenTyped(const char* hsaco, int n, int elemBytes) {
  if (n < 2 || n > 8 || (elemBytes != 2 && elemBytes != 4) || !rankStreams()) return nullptr;
  auto* h = new RefBench2;
  h->n = n;
  h->elemBytes = elemBytes;
  h->mod.resize(n);
  h->fn.resize(n);
  h->fn1.resize(n);
  h->chans.resize(n);
  for (int r = 0; r < n; ++r) {
    if (hipModuleLoad(&h->mod[r], hsaco) != hipSuccess ||
        hipModuleGetFunction(&h->fn[r], h->mod[r], "allreduce2") != hipSuccess ||
        hipModuleGetFunction(&h->fn1[r], h->mod[r], "allreduce1") != hipSuccess ||
        hipMalloc(&h->chans[r], sizeof(MemoryChannelDeviceHandle) * (n - 1)) != hipSuccess) {
      refBench2Close(h);
      return nullptr;
    }
  }
  // distinct modules must hold distinct globalFlag words (one per rank, as one per process)
  std::vector<void*> flags(n);
  for (int r = 0; r < n; ++r) {
    size_t bytes = 0;
    if (hipModuleGetGlobal(reinterpret_cast<hipDeviceptr_t*>(&flags[r]), &bytes, h->mod[r], "globalFlag") !=
            hipSuccess ||
        bytes != sizeof(uint64_t)) {
      refBench2Close(h);
      return nullptr;
    }
    for (int q = 0; q < r; ++q)
      if (flags[q] == flags[r]) {
        refBench2Close(h);
        return nullptr;
      }
  }
  // every rank starts at the kernel's initial flag (allreduce.cu:223), written here rather than
  // trusted to the load: ranks at different flags would wait for each other's packets forever
  for (int r = 0; r < n; ++r) {
    const uint64_t one = 1;
    if (hipMemcpy(flags[r], &one, sizeof(one), hipMemcpyHostToDevice) != hipSuccess) {
      refBench2Close(h);
      return nullptr;
    }
  }
  return h;
}

void* refBench2Open(const char* hsaco, int n) { return refBench2OpenTyped(hsaco, n, 4); }

// After a timeout: which ranks' launches finished (done[r]) and each rank's globalFlag (flags[r]),
// read on the diagnostic stream while the others may still spin.  0 on success.
int refBench2Diag(void* handle, int* done, uint64_t* flags) {
  auto* h = static_cast<RefBench2*>(handle);
  if (!h || !gDiagPinned) return 1;
  uint64_t* pinned = gDiagPinned;
  int rc = 0;
  for (int r = 0; r < h->n && rc == 0; ++r) {
    done[r] = hipStreamQuery(gRankStream[r]) == hipSuccess;
    void* g = nullptr;
    size_t bytes = 0;
    if (hipModuleGetGlobal(reinterpret_cast<hipDeviceptr_t*>(&g), &bytes, h->mod[r], "globalFlag") != hipSuccess ||
        hipMemcpyAsync(pinned + r, g, sizeof(uint64_t), hipMemcpyDeviceToHost, gDiagStream) != hipSuccess)
      rc = 1;
  }
  if (rc == 0) {
    const auto t0 = std::chrono::steady_clock::now();
    while (hipStreamQuery(gDiagStream) == hipErrorNotReady)
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
        rc = 2;
        break;
      }
  }
  if (rc == 0)
    for (int r = 0; r < h->n; ++r) flags[r] = pinned[r];
  return rc;
}

// After a timeout: lets spinning ranks finish before the process leaves, by filling the words they
// wait on from the diagnostic stream -- every 32-bit word of ptrs[0 .. nptr) := value (for allreduce2
// the packet scratch and the call's flag, so every flag word matches; for allreduce1 the inbound
// tokens and 0x7fffffff, above any expected count).  0 if rank streams 0 .. n-1 then drain within
// timeoutMs, 2 if not.  The data the ranks then produce is garbage; the caller reports the timeout.
int refReleaseSpin(void* const* ptrs, int nptr, uint64_t words, uint32_t value, int n, int timeoutMs) {
  if (!gDiagStream || n < 1 || n > 8) return 1;
  for (int k = 0; k < nptr; ++k)
    if (hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(ptrs[k]), (int)value, words, gDiagStream) != hipSuccess)
      return 1;
  const auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < n;) {
    if (hipStreamQuery(gRankStream[r]) != hipErrorNotReady) {
      ++r;
      continue;
    }
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeoutMs)) return 2;
  }
  return 0;
}

// After refReleaseSpin ended a stalled allreduce2 call: the state a retry of that call needs -- every
// rank's packet scratch zeroed (the release filled it with the call's flag) and every rank's
// globalFlag set to `flag` (a workgroup that read an already incremented flag may have moved one
// rank on).  0 on success.
int refBench2Reset(void* handle, void* const* scratch, uint64_t bytes, uint64_t flag) {
  auto* h = static_cast<RefBench2*>(handle);
  if (!h) return 1;
  for (int r = 0; r < h->n; ++r) {
    void* g = nullptr;
    size_t gb = 0;
    if (hipMemset(scratch[r], 0, bytes) != hipSuccess ||
        hipModuleGetGlobal(reinterpret_cast<hipDeviceptr_t*>(&g), &gb, h->mod[r], "globalFlag") != hipSuccess ||
        hipMemcpy(g, &flag, sizeof(flag), hipMemcpyHostToDevice) != hipSuccess)
      return 1;
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

// How many times ensureConcurrent replaced the rank streams in this process.
int refStreamRecreations() { return gStreamRecreations; }

// Packet scratch the way the reference allocates it on AMD (GpuBuffer -> hipExtMallocWithFlags with
// hipDeviceMallocUncached, src/core/gpu_utils.cc): the ranks' kernels run on different XCDs, whose
// L2s do not see each other's writes to ordinary (coarse-grained) device memory.  Zero-filled.
void* refMallocUncached(uint64_t bytes) {
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) != hipSuccess) return nullptr;
  if (hipMemset(p, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  return p;
}

void refFree(void* p) { (void)hipFree(p); }

void refBench2Close(void* handle) {
  auto* h = static_cast<RefBench2*>(handle);
  if (!h) return;
  for (int r = 0; r < h->n; ++r) {
    if (h->chans[r]) (void)hipFree(h->chans[r]);
    if (h->mod[r]) (void)hipModuleUnload(h->mod[r]);
  }
  delete h;
}

// Channel handles of allreduce2 (each rank's n - 1 channels: dst the peer's scratch, src its buffer,
// packetBuffer its own scratch), after the shape checks.  0, 4 (shape) or 1 (HIP error).
static int setupBench2(RefBench2* h, void* const* bufs, void* const* scratch, uint64_t nelems, int blocksPerPeer,
                       int threads) {
  const int n = h->n, nPeers = n - 1;
  if (nelems == 0 || nelems % (2 * (uint64_t)n) != 0 || nelems > (1ull << 30) || blocksPerPeer < 1 ||
      blocksPerPeer * nPeers > 64 || threads < 64 || threads > 1024 || threads % 64 != 0)
    return 4;
  for (int r = 0; r < n; ++r) {
    std::vector<MemoryChannelDeviceHandle> hc(nPeers);
    for (int p = 0; p < nPeers; ++p) {
      const int remote = p < r ? p : p + 1;
      std::memset(static_cast<void*>(&hc[p]), 0, sizeof(hc[p]));
      hc[p].dst_ = scratch[remote];
      hc[p].src_ = bufs[r];
      hc[p].packetBuffer_ = scratch[r];
    }
    if (hipMemcpy(h->chans[r], hc.data(), sizeof(hc[0]) * nPeers, hipMemcpyHostToDevice) != hipSuccess) return 1;
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

static int launchBench2(RefBench2* h, int r, void* const* bufs, void* const* scratch, void* const* results,
                        uint64_t nelems, int blocksPerPeer, int threads) {
  MemoryChannelDeviceHandle* c = h->chans[r];
  void* buff = bufs[r];
  void* scr = scratch[r];
  void* res = results[r];
  int rank = r, world = h->n;
  size_t ne = nelems * 4 / (uint64_t)h->elemBytes;  // TYPE elements
  void* args[] = {&c, &buff, &scr, &res, &rank, &world, &ne};
  return hipModuleLaunchKernel(h->fn[r], blocksPerPeer * (h->n - 1), 1, 1, threads, 1, 1, 0, gRankStream[r], args,
                               nullptr) == hipSuccess
             ? 0
             : 1;
}

// Channel handles of allreduce1 (semaphore tokens; channel p of rank r reaches rank p < r ? p : p + 1,
// as :200), after the shape checks.  0, 4 or 1.
static int setupBench1(RefBench2* h, void* const* bufs, void* const* tokens, void* const* expected, uint64_t nelems,
                       int nblocks, int threads) {
  const int n = h->n, nPeers = n - 1;
  if (nelems == 0 || nelems > (1ull << 30) || nblocks < 1 || nblocks > 16 || threads < 64 || threads > 1024 ||
      threads % 64 != 0 || (uint64_t)nblocks * threads < 2 * (uint64_t)nPeers)
    return 4;
  for (int r = 0; r < n; ++r) {
    std::vector<MemoryChannelDeviceHandle> hc(nPeers);
    for (int p = 0; p < nPeers; ++p) {
      const int remote = p < r ? p : p + 1;
      std::memset(static_cast<void*>(&hc[p]), 0, sizeof(hc[p]));
      hc[p].semaphore_.inboundToken = static_cast<uint64_t*>(tokens[r]) + p;
      hc[p].semaphore_.remoteInboundToken = static_cast<uint64_t*>(tokens[remote]) + (r < remote ? r : r - 1);
      hc[p].semaphore_.expectedInboundToken = static_cast<uint64_t*>(expected[r]) + p;
      hc[p].dst_ = bufs[remote];
      hc[p].src_ = bufs[r];
      hc[p].packetBuffer_ = nullptr;
    }
    if (hipMemcpy(h->chans[r], hc.data(), sizeof(hc[0]) * nPeers, hipMemcpyHostToDevice) != hipSuccess) return 1;
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

static int launchBench1(RefBench2* h, int r, void* const* bufs, uint64_t nelems, int nblocks, int threads,
                        int readOnly) {
  MemoryChannelDeviceHandle* c = h->chans[r];
  void* buff = bufs[r];
  int rank = r, world = h->n, ro = readOnly;
  size_t ne = nelems * 4 / (uint64_t)h->elemBytes;  // TYPE elements
  void* args[] = {&c, &buff, &rank, &world, &ne, &ro};
  return hipModuleLaunchKernel(h->fn1[r], nblocks, 1, 1, threads, 1, 1, 0, gRankStream[r], args, nullptr) ==
                 hipSuccess
             ? 0
             : 1;
}

// One AllReduce call on every rank.  bufs/scratch/results: n device pointers each (scratch zeroed by
// the caller before the first call, 4 * nelems / 2 LL16 packets); nelems ints per rank.  Returns 0,
// 4 on a shape the kernel cannot take (it would index past its channel array or split a packet), 1 on
// a HIP error, 2 if the ranks have not finished after timeoutMs, 5 (nothing launched) if the rank
// streams could not run kernels concurrently even on fresh streams (ensureConcurrent).
int refBench2Run(void* handle, void* const* bufs, void* const* scratch, void* const* results, uint64_t nelems,
                 int blocksPerPeer, int threads, int timeoutMs) {
  auto* h = static_cast<RefBench2*>(handle);
  if (!h) return 1;
  const int n = h->n;
  if (const int rc = setupBench2(h, bufs, scratch, nelems, blocksPerPeer, threads)) return rc;
  if (const int mc = ensureConcurrent(n)) return mc;
  for (int r = 0; r < n; ++r)
    if (launchBench2(h, r, bufs, scratch, results, nelems, blocksPerPeer, threads)) return 1;
  const auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < n;) {
    const hipError_t e = hipStreamQuery(gRankStream[r]);
    if (e == hipSuccess) {
      ++r;
      continue;
    }
    if (e != hipErrorNotReady) return 1;
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeoutMs)) return 2;
  }
  return 0;
}

// One in-place allreduce1 call (python/mscclpp_benchmark/allreduce.cu:123-221: signal / wait every
// peer, grid barrier, read-reduce the own chunk from every peer's buffer -- own first, then channel
// (index + rank) mod (n - 1) -- and, read_only == 0, write it back into every peer's buffer; grid
// barrier, signal / wait again; read_only == 1 then gets the peers' chunks instead).  bufs: n device
// buffers of nelems 32-bit words each, uncached (the ranks read and write each other's); tokens /
// expected: n device arrays of n - 1 uint64 each, zeroed before the first call and kept across calls
// (the semaphores are monotonic).  Channel p of rank r reaches rank p < r ? p : p + 1 (as :200).
// Returns as refBench2Run.
int refBench1Run(void* handle, void* const* bufs, void* const* tokens, void* const* expected, uint64_t nelems,
                 int nblocks, int threads, int readOnly, int timeoutMs) {
  auto* h = static_cast<RefBench2*>(handle);
  if (!h) return 1;
  const int n = h->n;
  if (const int rc = setupBench1(h, bufs, tokens, expected, nelems, nblocks, threads)) return rc;
  if (const int mc = ensureConcurrent(n)) return mc;
  for (int r = 0; r < n; ++r)
    if (launchBench1(h, r, bufs, nelems, nblocks, threads, readOnly)) return 1;
  const auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < n;) {
    const hipError_t e = hipStreamQuery(gRankStream[r]);
    if (e == hipSuccess) {
      ++r;
      continue;
    }
    if (e != hipErrorNotReady) return 1;
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeoutMs)) return 2;
  }
  return 0;
}

// `calls` allreduce2 calls queued back to back on every rank stream (rank by rank, call by call), with
// no host synchronisation between them -- how the reference's benchmark times it (bench_time: one
// graph of niter launches).  flagsOut[r] = each rank's globalFlag afterwards (on a timeout: as read
// on the diagnostic stream while the ranks still spun).  Returns as refBench2Run; on 2 the ranks were
// then released by filling every scratch word with each remaining call's flag in turn (scratchWords
// 32-bit words per rank), 3 if even that did not drain them.
// between: what runs on every rank stream between two calls -- 0 nothing, 1 a 1024-workgroup kernel
// that does nothing, 2 the same kernel with a system-scope acquire fence in every wave (each XCD's L2
// invalidated: workgroups are spread over all eight).
__global__ void refBetweenKernel(int inv) {
  if (inv) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

int refBench2RunBackToBack(void* handle, void* const* bufs, void* const* scratch, void* const* results, uint64_t nelems,
                           int blocksPerPeer, int threads, int calls, int timeoutMs, uint64_t scratchWords,
                           int between, uint64_t* flagsOut) {
  auto* h = static_cast<RefBench2*>(handle);
  if (!h || calls < 1 || calls > 64 || !flagsOut || !gDiagPinned) return 1;
  const int n = h->n;
  if (const int rc = setupBench2(h, bufs, scratch, nelems, blocksPerPeer, threads)) return rc;
  if (const int mc = ensureConcurrent(n)) return mc;
  std::vector<void*> g(n, nullptr);
  for (int r = 0; r < n; ++r) {
    size_t bytes = 0;
    if (hipModuleGetGlobal(reinterpret_cast<hipDeviceptr_t*>(&g[r]), &bytes, h->mod[r], "globalFlag") != hipSuccess)
      return 1;
  }
  uint64_t flag0 = 0;
  if (hipMemcpy(&flag0, g[0], sizeof(flag0), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  int rc = 0;
  for (int c = 0; c < calls && rc == 0; ++c)
    for (int r = 0; r < n && rc == 0; ++r) {
      if (c > 0 && between > 0) {
        hipLaunchKernelGGL(refBetweenKernel, dim3(1024), dim3(64), 0, gRankStream[r], between == 2 ? 1 : 0);
        if (hipGetLastError() != hipSuccess) rc = 1;
      }
      if (rc == 0) rc = launchBench2(h, r, bufs, scratch, results, nelems, blocksPerPeer, threads);
    }
  auto drained = [&](int ms) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < n;) {
      if (hipStreamQuery(gRankStream[r]) != hipErrorNotReady) {
        ++r;
        continue;
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(ms)) return false;
    }
    return true;
  };
  if (!drained(timeoutMs)) {
    for (int r = 0; r < n; ++r)
      (void)hipMemcpyAsync(gDiagPinned + r, g[r], sizeof(uint64_t), hipMemcpyDeviceToHost, gDiagStream);
    const auto t0 = std::chrono::steady_clock::now();
    while (hipStreamQuery(gDiagStream) == hipErrorNotReady &&
           std::chrono::steady_clock::now() - t0 < std::chrono::seconds(5)) {
    }
    for (int r = 0; r < n; ++r) flagsOut[r] = gDiagPinned[r];
    // ranks may wait for different calls' flags at once, one past the last included (a workgroup that
    // read a flag already incremented): two passes over flag0 .. flag0 + calls
    bool ok = false;
    for (int pass = 0; pass < 2 && !ok; ++pass)
      for (int c = 0; c <= calls && !ok; ++c) {
        for (int r = 0; r < n; ++r)
          (void)hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(scratch[r]), (int)(uint32_t)(flag0 + c),
                                  scratchWords, gDiagStream);
        ok = drained(200);
      }
    return ok ? 2 : 3;
  }
  for (int r = 0; r < n; ++r)
    if (hipMemcpy(&flagsOut[r], g[r], sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  return rc;
}

}  // extern "C"
