"""mscclpp_amd: MI355X-native LL-packet AllReduce (drop-in for mscclpp's in-kernel AllReduce path).

The product is the C-ABI shared library ``mscclpp_amd/lib/libmscclpp_amd.so`` (HIP kernels for
gfx950 + C++ host runtime; headers in ``include/mscclpp_amd``).  This module is the thin Python
host mirror used by the tests and the benchmark: it loads the library with ctypes and exposes
the reference's operator surface for this path (``ncclAllReduce`` / ``Algorithm::execute`` with
the same argument meaning and error behaviour).  PyTorch is used only for device memory and
streams.  There is no fallback: if the library is missing, importing a GPU entry point raises.
"""
import collections
import ctypes
import os

import torch  # noqa: F401  -- must be loaded first so the library binds to torch's HIP runtime

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libmscclpp_amd.so")

# dtype / op / algorithm codes (include/mscclpp_amd/mscclpp_amd.h)
F16, BF16, F32, I32, U32 = 0, 1, 2, 3, 4
# OCP fp8 reduce types: element type x accumulation type (Algorithm::execute accumDtype)
E4M3, E5M2, E4M3_ACC_F16, E5M2_ACC_F16, E4M3_ACC_F32, E5M2_ACC_F32 = 5, 6, 7, 8, 9, 10
# uint8, and the software fp8 e4m3b15 accumulated in itself / half / float (no torch dtype: pass
# uint8 tensors with accum=E4M3B15..., an explicit reduce-type code)
U8, E4M3B15, E4M3B15_ACC_F16, E4M3B15_ACC_F32 = 11, 12, 13, 14
SUM, MIN = 0, 1
ALGO_AUTO, ALGO_PACKET, ALGO_ALLPAIR, ALGO_FULLMESH, ALGO_RSAG, ALGO_RSAG_ZC, ALGO_RSAG_PIPELINE = 0, 1, 2, 3, 4, 5, 6
ALGO_TEST_K2, ALGO_TEST_K5, ALGO_TEST_K6, ALGO_TEST_K7 = 102, 105, 106, 107  # mscclpp-test allreduce2/5/6/7 (int32)
ALGO_NAMES = {"auto": 0, "packet": 1, "allpair": 2, "fullmesh": 3, "rsag": 4, "rsag_zc": 5, "rsag_pipeline": 6,
              "k2": ALGO_TEST_K2, "k5": ALGO_TEST_K5, "k6": ALGO_TEST_K6, "k7": ALGO_TEST_K7}
MAX_RANKS = 8
FLAG_SLOTS = 4096
MAX_CHANNELS = 256

# ncclDataType_t / ncclRedOp_t (include/mscclpp_amd/nccl.h, values of the reference nccl.h:217-253)
NCCL_DTYPES = {torch.float16: 6, torch.bfloat16: 9, torch.float32: 7, torch.int32: 2, torch.uint8: 1,
               torch.float8_e4m3fn: 10, torch.float8_e5m2: 11}
NCCL_OPS = {"sum": 0, "min": 3}
DTYPE_CODES = {torch.float16: F16, torch.bfloat16: BF16, torch.float32: F32, torch.int32: I32, torch.uint8: U8,
               torch.float8_e4m3fn: E4M3, torch.float8_e5m2: E5M2}
# accumulation dtype (ncclDataType_t) -> reduce-type code, for fp8 buffers
ACCUM_CODES = {(torch.float8_e4m3fn, torch.float16): E4M3_ACC_F16, (torch.float8_e5m2, torch.float16): E5M2_ACC_F16,
               (torch.float8_e4m3fn, torch.float32): E4M3_ACC_F32, (torch.float8_e5m2, torch.float32): E5M2_ACC_F32}


def reduce_code(dtype, accum=None):
    """Reduce-type code of a buffer dtype accumulated in `accum` (None: the element type; an int:
    that reduce-type code itself, e.g. E4M3B15_ACC_F32 over a uint8 buffer)."""
    if isinstance(accum, int):
        return accum
    if accum is None or accum == dtype:
        return DTYPE_CODES[dtype]
    return ACCUM_CODES[(dtype, accum)]

ERRORS = {0: "ncclSuccess", 1: "ncclUnhandledCudaError", 2: "ncclSystemError", 3: "ncclInternalError",
          4: "ncclInvalidArgument", 5: "ncclInvalidUsage", 6: "ncclRemoteError", 7: "ncclInProgress"}


class MscclppError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        super().__init__(f"{what}: {ERRORS.get(code, code)}")


class RankView(ctypes.Structure):
    _fields_ = [
        ("input", ctypes.c_void_p),
        ("output", ctypes.c_void_p),
        ("scratch", ctypes.c_void_p),
        ("peerScratch", ctypes.c_void_p * MAX_RANKS),
        ("peerOutput", ctypes.c_void_p * MAX_RANKS),
        ("tokens", ctypes.c_void_p),
        ("peerTokens", ctypes.c_void_p * MAX_RANKS),
        ("expected", ctypes.c_void_p),
        ("flags", ctypes.c_void_p),
        ("err", ctypes.c_void_p),
        ("scratchBytes", ctypes.c_uint64),
        ("rank", ctypes.c_int32),
        ("pad", ctypes.c_int32),
        ("peerInput", ctypes.c_void_p * MAX_RANKS),
        ("pipeSems", ctypes.c_void_p),
    ]


class UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


_lib = None


def lib():
    """Load libmscclpp_amd.so (raises if it has not been built: no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, i32, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
    sig = {
        "mscclppAmdMallocUncached": [ctypes.POINTER(vp), sz],
        "mscclppAmdMalloc": [ctypes.POINTER(vp), sz],
        "mscclppAmdFree": [vp],
        "mscclppAmdUncachedPoolStats": [ctypes.POINTER(sz), ctypes.POINTER(sz), ctypes.POINTER(sz)],
        "mscclppAmdIpcStats": [ctypes.POINTER(sz), ctypes.POINTER(sz)],
        "mscclppAmdIpcKeptRanges": [ctypes.POINTER(u64), ctypes.POINTER(u64), sz, ctypes.POINTER(sz)],
        "mscclppAmdIpcReleaseKept": [ctypes.POINTER(sz)],
        "mscclppAmdTraceSet": [vp, sz],
        "mscclppAmdFlagsInit": [vp, vp],
        "mscclppAmdSelfReduceLL16": [vp, vp, vp, vp, sz, i32, i32, vp, i32, u64, vp, vp],
        "mscclppAmdAllReduceLaunch": [i32, ctypes.POINTER(RankView), i32, i32, sz, i32, i32, i32, i32, u64, vp],
        "mscclppAmdSelectAlgo": [i32, sz, i32],
        "mscclppAmdTunedConfigLoad": [ctypes.c_char_p],
        "mscclppAmdTunedConfigSource": [ctypes.c_char_p, i32, sz, ctypes.c_char_p, sz],
        "mscclppAmdTunedConfig": [ctypes.c_char_p, i32, sz, ctypes.c_char_p, sz, ctypes.POINTER(i32),
                                  ctypes.POINTER(i32)],
        "mscclppAmdCollectiveLaunch": [i32, i32, ctypes.POINTER(RankView), i32, i32, sz, i32, i32, i32, i32, u64, vp],
        "ncclReduceScatter": [vp, vp, sz, i32, i32, vp, vp],
        "ncclAllGather": [vp, vp, sz, i32, vp, vp],
        "ncclBroadcast": [vp, vp, sz, i32, i32, vp, vp],
        "mscclppAmdCommRegisterBuffer": [vp, vp, ctypes.POINTER(vp)],
        "mscclppAmdCommDeregisterAll": [vp],
        "mscclppAmdCopy": [vp, vp, sz, i32, vp],
        "mscclppAmdSelfReduceStream": [vp, vp, vp, vp, sz, vp],
        "mscclppAmdMixStream": [vp, vp, vp, vp, vp, sz, i32, vp],
        "mscclppAmdCopyJobs": [ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(sz), i32, i32, vp],
        "mscclppAmdCopyJobsPolicy": [ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(sz), i32, i32, i32, i32, vp],
        "mscclppAmdSelfReduceLL16DefaultShape": [sz, vp, vp, vp, vp],
        "ncclCommSplit": [vp, i32, i32, ctypes.POINTER(vp), vp],
        "mscclppAmdBroadcastLaunch": [ctypes.POINTER(RankView), i32, i32, sz, i32, i32, i32, u64, vp],
        "ncclGetUniqueId": [ctypes.POINTER(UniqueId)],
        "ncclCommInitRank": [ctypes.POINTER(vp), i32, UniqueId, i32],
        "ncclCommDestroy": [vp],
        "ncclAllReduce": [vp, vp, sz, i32, i32, vp, vp],
        "ncclCommCount": [vp, ctypes.POINTER(i32)],
        "ncclCommUserRank": [vp, ctypes.POINTER(i32)],
        "ncclCommCuDevice": [vp, ctypes.POINTER(i32)],
        "ncclCommGetAsyncError": [vp, ctypes.POINTER(i32)],
        "ncclGetVersion": [ctypes.POINTER(i32)],
        "mscclppAmdCommAllReduce": [vp, vp, vp, sz, i32, i32, i32, i32, i32, vp],
        "mscclppAmdCommAllReduceAccum": [vp, vp, vp, sz, i32, i32, i32, i32, i32, i32, vp],
        "mscclppAmdReduceType": [i32, i32],
        "mscclppAmdCommBarrier": [vp],
        "mscclppAmdCommGetDeviceError": [vp, ctypes.POINTER(ctypes.c_uint32), i32],
        "mscclppAmdCommGetDeviceErrorDetail": [vp, ctypes.POINTER(ctypes.c_uint32), i32],
        "mscclppAmdCommScratch": [vp, ctypes.POINTER(vp), ctypes.POINTER(sz)],
        "mscclppAmdCommRegistrationStats": [vp, ctypes.POINTER(sz), ctypes.POINTER(sz), ctypes.POINTER(sz)],
        "mscclppAmdCommRegistrationExchanges": [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                                ctypes.POINTER(ctypes.c_int)],
        "mscclppAmdCommFlags": [vp, ctypes.POINTER(vp)],
        "mscclppAmdCommAllGatherHost": [vp, vp, vp, sz],
        "mscclppAmdProxyRingAllReduce": [vp, sz, i32, i32, i32, ctypes.POINTER(ctypes.c_double)],
        "mscclppAmdExecutionPlanCreate": [ctypes.c_char_p, i32, ctypes.POINTER(vp)],
        "mscclppAmdExecutionPlanDestroy": [vp],
        "mscclppAmdExecutionPlanIsInPlace": [vp],
        "mscclppAmdExecutionPlanDescribe": [vp, sz, sz, ctypes.c_char_p, sz, ctypes.POINTER(sz)],
        "mscclppAmdExecutorCreate": [vp, ctypes.POINTER(vp)],
        "mscclppAmdExecutorExecute": [vp, i32, vp, vp, sz, sz, i32, vp, vp, i32],
        "mscclppAmdExecutorReset": [vp],
        "mscclppAmdExecutorDestroy": [vp],
        "mscclppAmdExecutorGetDeviceError": [vp, ctypes.POINTER(ctypes.c_uint32), i32],
    }
    for name, args in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = ctypes.c_int
    L.mscclppAmdScratchRequired.argtypes = [i32, i32, sz, i32]
    L.mscclppAmdScratchRequired.restype = sz
    for name in ("mscclppAmdExecutionPlanName", "mscclppAmdExecutionPlanCollective"):
        getattr(L, name).argtypes = [vp]
        getattr(L, name).restype = ctypes.c_char_p
    for name in ("mscclppAmdExecutionPlanMinMessageSize", "mscclppAmdExecutionPlanMaxMessageSize"):
        getattr(L, name).argtypes = [vp]
        getattr(L, name).restype = sz
    L.ncclGetErrorString.argtypes = [i32]
    L.ncclGetErrorString.restype = ctypes.c_char_p
    _lib = L
    return L


def check(code, what="mscclpp_amd"):
    if code != 0:
        raise MscclppError(code, what)


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


# (op, ptr, nbytes, uncached) of the last DeviceBuffer allocations and frees of this process: what a
# test diagnostic compares a misbehaving buffer's address range with
ALLOC_HISTORY = collections.deque(maxlen=4096)


class DeviceBuffer:
    """Raw device allocation owned by the library (uncached = hipDeviceMallocUncached)."""

    def __init__(self, nbytes, uncached=True):
        self.nbytes = nbytes
        self.uncached = uncached
        p = ctypes.c_void_p()
        fn = lib().mscclppAmdMallocUncached if uncached else lib().mscclppAmdMalloc
        check(fn(ctypes.byref(p), nbytes), "device alloc")
        self.ptr = p.value
        ALLOC_HISTORY.append(("alloc", self.ptr, nbytes, uncached))

    def free(self):
        if self.ptr:
            lib().mscclppAmdFree(ctypes.c_void_p(self.ptr))
            ALLOC_HISTORY.append(("free", self.ptr, self.nbytes, self.uncached))
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def pool_stats():
    """(held, in use, free) bytes of the process-lifetime uncached pool (mscclppAmdUncachedPoolStats)."""
    a, b, c = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
    check(lib().mscclppAmdUncachedPoolStats(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), "pool stats")
    return a.value, b.value, c.value


def ipc_stats():
    """(IPC mappings open in this process, of which kept imports of peers' pooled blocks)."""
    a, b = ctypes.c_size_t(), ctypes.c_size_t()
    check(lib().mscclppAmdIpcStats(ctypes.byref(a), ctypes.byref(b)), "ipc stats")
    return a.value, b.value


def ipc_kept_ranges():
    """[(mapped address, bytes)] of the kept imports of peers' pooled uncached blocks."""
    n = ctypes.c_size_t()
    check(lib().mscclppAmdIpcKeptRanges(None, None, 0, ctypes.byref(n)), "ipc kept ranges")
    cap = n.value
    addrs, sizes = (ctypes.c_uint64 * max(cap, 1))(), (ctypes.c_uint64 * max(cap, 1))()
    check(lib().mscclppAmdIpcKeptRanges(addrs, sizes, cap, ctypes.byref(n)), "ipc kept ranges")
    return [(addrs[i], sizes[i]) for i in range(min(cap, n.value))]


def ipc_release_kept():
    """Forget the kept imports of peers' pooled blocks (mscclppAmdIpcReleaseKept); returns how many."""
    n = ctypes.c_size_t()
    check(lib().mscclppAmdIpcReleaseKept(ctypes.byref(n)), "ipc release kept")
    return n.value


def flags_init(flags_tensor, stream=None):
    check(lib().mscclppAmdFlagsInit(ctypes.c_void_p(flags_tensor.data_ptr()), stream_ptr(stream)), "flags init")


def self_reduce_ll16(x, y, pkts_ptr, out, flags, err, op=SUM, nblocks=0, budget_ticks=0, stream=None, accum=None):
    """out = x (op) unpack(pack(y)) -- the 1-GPU LL16 hot path (BASELINE config 2)."""
    assert x.dtype == y.dtype == out.dtype and x.numel() == y.numel() == out.numel()
    nbytes = x.numel() * x.element_size()
    code = lib().mscclppAmdSelfReduceLL16(
        ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), ctypes.c_void_p(pkts_ptr),
        ctypes.c_void_p(out.data_ptr()), nbytes, reduce_code(x.dtype, accum), op, ctypes.c_void_p(flags.data_ptr()),
        nblocks, budget_ticks or 200_000_000, ctypes.c_void_p(err.data_ptr()), stream_ptr(stream))
    check(code, "self_reduce_ll16")


def tuned_config(collective, nranks, nbytes):
    """(algorithm name, nblocks, nthreads) the tuned-config store picks, or None."""
    name = ctypes.create_string_buffer(128)
    nb, nt = ctypes.c_int(), ctypes.c_int()
    rc = lib().mscclppAmdTunedConfig(collective.encode(), nranks, nbytes, name, 128, ctypes.byref(nb), ctypes.byref(nt))
    if rc == 5:
        return None
    check(rc, "tuned config")
    return name.value.decode(), nb.value, nt.value


def tuned_config_source(collective, nranks, nbytes):
    """Where the tuned-config entry that applies came from ("reference", "fabric-free", "tuned", ...)."""
    buf = ctypes.create_string_buffer(128)
    rc = lib().mscclppAmdTunedConfigSource(collective.encode(), nranks, nbytes, buf, 128)
    if rc == 5:
        return None
    check(rc, "tuned config source")
    return buf.value.decode()


def load_tuned_config(path):
    check(lib().mscclppAmdTunedConfigLoad(os.fsencode(path)), f"tuned config {path}")


TRACE_BLOCKS, TRACE_EVENTS = 256, 8
TRACE_BYTES = MAX_RANKS * TRACE_BLOCKS * TRACE_EVENTS * 8
# phase names per kernel family, in event order (mscclpp_amd.h, mscclppAmdTraceSet)
TRACE_PHASES = {
    "fullmesh": ("rs_put", "rs_handshake", "reduce_ag", "exit_handshake"),
    "rsag": ("rs_put", "rs_handshake", "reduce_ag", "exit_handshake"),
    "rsag_zc": ("entry_handshake", "reduce_ag", "exit_handshake"),
    "packet": ("step1_put", "step2_reduce_bcast", "step3_unpack"),
    "allpair": ("put", "reduce"),
}


class PhaseTrace:
    """Phase stamps of the collective kernels (the reference's NPKit events): while active, every
    launch of this process stamps s_memrealtime at its phase boundaries, lane 0 of each workgroup.

        with PhaseTrace() as tr:
            comm.all_reduce(x, y, algo="fullmesh"); torch.cuda.synchronize()
        tr.phases("fullmesh")   # {"rs_put": {"mean_us": ..., "max_us": ...}, ...}
    """

    def __init__(self, device=None):
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.buf = torch.zeros(TRACE_BYTES // 8, dtype=torch.int64, device=dev)

    def __enter__(self):
        torch.cuda.synchronize()
        self.buf.zero_()
        check(lib().mscclppAmdTraceSet(ctypes.c_void_p(self.buf.data_ptr()), TRACE_BYTES), "mscclppAmdTraceSet")
        return self

    def __exit__(self, *exc):
        torch.cuda.synchronize()
        lib().mscclppAmdTraceSet(None, 0)
        return False

    def stamps(self, view=0):
        """[workgroup][event] ticks (10 ns) of one rank view; rows of workgroups that never stamped are 0."""
        import numpy  # noqa: F401  (.numpy() below)

        return self.buf.view(MAX_RANKS, TRACE_BLOCKS, TRACE_EVENTS)[view].cpu().numpy()

    def phases(self, algo, view=0):
        import numpy as np

        names = TRACE_PHASES[algo]
        st = self.stamps(view)
        rows = st[st[:, 0] != 0][:, : len(names) + 1].astype(np.float64)
        if rows.size == 0:
            return {}
        d = np.diff(rows, axis=1) / 100.0  # ticks -> us
        out = {nm: {"mean_us": round(float(d[:, i].mean()), 2), "max_us": round(float(d[:, i].max()), 2)}
               for i, nm in enumerate(names)}
        out["kernel_span_us"] = round(float((rows[:, -1].max() - rows[:, 0].min()) / 100.0), 2)
        out["workgroups"] = int(rows.shape[0])
        return out


def scratch_required(algo, nranks, nbytes, dtype_code):
    return lib().mscclppAmdScratchRequired(algo, nranks, nbytes, dtype_code)


class InProcessRanks:
    """n ranks of one AllReduce inside this process on one GPU (parity tests).

    Every rank gets its own scratch, flags, tokens and error word; peer arrays hold the other
    ranks' plain device pointers, so the kernels run exactly the multi-rank protocol (one launch,
    blockIdx.y = rank) without IPC.
    """

    def __init__(self, nranks, scratch_bytes, bulk_scratch_bytes=0):
        self.n = nranks
        self.scratch = [DeviceBuffer(scratch_bytes) for _ in range(nranks)]
        self.scratch_bytes = scratch_bytes
        self.bulk = [DeviceBuffer(bulk_scratch_bytes) for _ in range(nranks)] if bulk_scratch_bytes else None
        self.bulk_bytes = bulk_scratch_bytes
        tok_elems = MAX_RANKS * MAX_CHANNELS
        self.tokens = [DeviceBuffer(tok_elems * 8) for _ in range(nranks)]
        dev = torch.device("cuda", torch.cuda.current_device())
        self.expected = [torch.zeros(tok_elems, dtype=torch.int64, device=dev) for _ in range(nranks)]
        self.flags = [torch.ones(FLAG_SLOTS, dtype=torch.int32, device=dev) for _ in range(nranks)]
        self.err = [torch.zeros(64, dtype=torch.int32, device=dev) for _ in range(nranks)]
        self.pipe_sems = [torch.zeros(3 * 256 + 64, dtype=torch.int64, device=dev) for _ in range(nranks)]

    def views(self, inputs, outputs, bulk=False):
        arr = (RankView * self.n)()
        if bulk and self.bulk is None:  # zero-copy kernels (rsag_zc, k5) need no bulk scratch
            bulk = False
        scr = self.bulk if bulk else self.scratch
        sbytes = self.bulk_bytes if bulk else self.scratch_bytes
        for r in range(self.n):
            v = arr[r]
            v.input = inputs[r].data_ptr()
            v.output = outputs[r].data_ptr()
            v.scratch = scr[r].ptr
            for q in range(self.n):
                v.peerScratch[q] = scr[q].ptr
                v.peerOutput[q] = outputs[q].data_ptr()
                v.peerInput[q] = inputs[q].data_ptr()
                v.peerTokens[q] = self.tokens[q].ptr
            v.tokens = self.tokens[r].ptr
            v.expected = self.expected[r].data_ptr()
            v.flags = self.flags[r].data_ptr()
            v.err = self.err[r].data_ptr()
            v.pipeSems = self.pipe_sems[r].data_ptr()
            v.scratchBytes = sbytes
            v.rank = r
        return arr

    def all_reduce(self, inputs, outputs, algo, op=SUM, nblocks=0, nthreads=0, budget_ticks=500_000_000, stream=None,
                   accum=None):
        dt = reduce_code(inputs[0].dtype, accum)
        nbytes = inputs[0].numel() * inputs[0].element_size()
        bulk = algo in (ALGO_FULLMESH, ALGO_RSAG, ALGO_RSAG_ZC, ALGO_RSAG_PIPELINE, ALGO_TEST_K5)
        arr = self.views(inputs, outputs, bulk=bulk)
        code = lib().mscclppAmdAllReduceLaunch(algo, arr, self.n, self.n, nbytes, dt, op, nblocks, nthreads,
                                               budget_ticks, stream_ptr(stream))
        check(code, "in-process all_reduce")

    def collective(self, coll, inputs, outputs, algo=ALGO_FULLMESH, op=SUM, nblocks=8, nthreads=256,
                   budget_ticks=500_000_000, stream=None, accum=None):
        """coll 1 = ReduceScatter (inputs n*block, outputs block), 2 = AllGather (inputs block, outputs n*block)."""
        dt = reduce_code(inputs[0].dtype, accum)
        big = inputs[0] if coll == 1 else outputs[0]
        nbytes = big.numel() * big.element_size()
        arr = self.views(inputs, outputs, bulk=True)
        code = lib().mscclppAmdCollectiveLaunch(coll, algo, arr, self.n, self.n, nbytes, dt, op, nblocks, nthreads,
                                                budget_ticks, stream_ptr(stream))
        check(code, "in-process collective")

    def broadcast(self, sends, recvs, root, nblocks=0, nthreads=0, budget_ticks=500_000_000, stream=None):
        """ncclBroadcast for in-process ranks: recvs[r] <- sends[root] (sends[r] read on the root only)."""
        nbytes = recvs[0].numel() * recvs[0].element_size()
        arr = self.views(sends, recvs)
        for r in range(self.n):
            arr[r].peerInput[root] = sends[root].data_ptr()
        code = lib().mscclppAmdBroadcastLaunch(arr, self.n, self.n, nbytes, root, nblocks, nthreads, budget_ticks,
                                               stream_ptr(stream))
        check(code, "in-process broadcast")

    def errors(self):
        return [int(e[0].item()) for e in self.err]

    def error_details(self):
        return [[int(v) for v in e[:4].tolist()] for e in self.err]

    def scratch_tensor(self, r, nbytes=None, bulk=False):
        """Zero-copy uint8 view of rank r's scratch (for packet-image checks)."""
        buf = (self.bulk if bulk else self.scratch)[r]
        return device_view(buf.ptr, nbytes or buf.nbytes)


class _CudaArray:
    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 2}


def device_view(ptr, nbytes):
    """uint8 torch tensor aliasing raw device memory owned by the library."""
    return torch.as_tensor(_CudaArray(ptr, nbytes), device="cuda")


class Communicator:
    """ncclComm_t wrapper (one rank per process).  Mirrors ncclCommInitRank / ncclAllReduce."""

    def __init__(self, rank, nranks, unique_id_bytes):
        uid = UniqueId()
        ctypes.memmove(ctypes.addressof(uid), unique_id_bytes, 128)
        c = ctypes.c_void_p()
        check(lib().ncclCommInitRank(ctypes.byref(c), nranks, uid, rank), "ncclCommInitRank")
        self.comm = c
        self.rank, self.nranks = rank, nranks

    @staticmethod
    def unique_id():
        uid = UniqueId()
        check(lib().ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        return ctypes.string_at(ctypes.addressof(uid), 128)  # (c_char arrays stop at the first NUL)

    @classmethod
    def from_torch_dist(cls, group=None):
        import torch.distributed as dist

        rank, n = dist.get_rank(group), dist.get_world_size(group)
        obj = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        return cls(rank, n, obj[0])

    def all_reduce(self, send, recv=None, op="sum", algo=None, nblocks=0, nthreads=0, stream=None, accum=None):
        """ncclAllReduce(send, recv, count, dtype, op, comm, stream); algo forces an algorithm, accum
        the accumulation dtype of Algorithm::execute (fp8 buffers: torch.float16 / torch.float32)."""
        recv = send if recv is None else recv
        dt = NCCL_DTYPES[send.dtype]
        if accum is not None:
            code = lib().mscclppAmdCommAllReduceAccum(self.comm, ctypes.c_void_p(send.data_ptr()),
                                                      ctypes.c_void_p(recv.data_ptr()), send.numel(), dt,
                                                      NCCL_OPS[op], NCCL_DTYPES[accum],
                                                      ALGO_NAMES.get(algo or "auto", algo) if isinstance(algo, str) or algo is None else algo,
                                                      nblocks, nthreads, stream_ptr(stream))
        elif algo is None:
            code = lib().ncclAllReduce(ctypes.c_void_p(send.data_ptr()), ctypes.c_void_p(recv.data_ptr()),
                                       send.numel(), dt, NCCL_OPS[op], self.comm, stream_ptr(stream))
        else:
            code = lib().mscclppAmdCommAllReduce(self.comm, ctypes.c_void_p(send.data_ptr()),
                                                 ctypes.c_void_p(recv.data_ptr()), send.numel(), dt, NCCL_OPS[op],
                                                 ALGO_NAMES.get(algo, algo) if isinstance(algo, str) else algo,
                                                 nblocks, nthreads, stream_ptr(stream))
        check(code, "ncclAllReduce")
        return recv

    def reduce_scatter(self, send, recv, op="sum", stream=None):
        """ncclReduceScatter(send, recv, recvcount, dtype, op, comm, stream)."""
        check(lib().ncclReduceScatter(ctypes.c_void_p(send.data_ptr()), ctypes.c_void_p(recv.data_ptr()), recv.numel(),
                                      NCCL_DTYPES[send.dtype], NCCL_OPS[op], self.comm, stream_ptr(stream)),
              "ncclReduceScatter")
        return recv

    def all_gather(self, send, recv, stream=None):
        """ncclAllGather(send, recv, sendcount, dtype, comm, stream)."""
        check(lib().ncclAllGather(ctypes.c_void_p(send.data_ptr()), ctypes.c_void_p(recv.data_ptr()), send.numel(),
                                  NCCL_DTYPES[send.dtype], self.comm, stream_ptr(stream)), "ncclAllGather")
        return recv

    def broadcast(self, send, recv=None, root=0, stream=None):
        """ncclBroadcast(send, recv, count, dtype, root, comm, stream); send is read on the root only."""
        recv = send if recv is None else recv
        check(lib().ncclBroadcast(ctypes.c_void_p(send.data_ptr()), ctypes.c_void_p(recv.data_ptr()), recv.numel(),
                                  NCCL_DTYPES[recv.dtype], root, self.comm, stream_ptr(stream)), "ncclBroadcast")
        return recv

    def register_buffer(self, t):
        """Collective: every rank's matching buffer as mapped here (list of nranks device pointers)."""
        arr = (ctypes.c_void_p * MAX_RANKS)()
        check(lib().mscclppAmdCommRegisterBuffer(self.comm, ctypes.c_void_p(t.data_ptr()), arr), "register_buffer")
        return [arr[r] for r in range(self.nranks)]

    def deregister_all(self):
        """Collective: forget every cached peer-buffer mapping (call after freeing buffers used here)."""
        check(lib().mscclppAmdCommDeregisterAll(self.comm), "deregister_all")

    def split(self, color, key):
        """ncclCommSplit(comm, color, key, &newcomm, NULL) -> Communicator, or None for NCCL_SPLIT_NOCOLOR."""
        c = ctypes.c_void_p()
        check(lib().ncclCommSplit(self.comm, color, key, ctypes.byref(c), None), "ncclCommSplit")
        if not c.value:
            return None
        sub = Communicator.__new__(Communicator)
        sub.comm = c
        r, n = ctypes.c_int(), ctypes.c_int()
        check(lib().ncclCommUserRank(c, ctypes.byref(r)), "ncclCommUserRank")
        check(lib().ncclCommCount(c, ctypes.byref(n)), "ncclCommCount")
        sub.rank, sub.nranks = r.value, n.value
        return sub

    def proxy_ring_all_reduce(self, nelems, iters=20, graph_launches=15, nblocks=0):
        """mscclpp-test allreduce1: int32 ring RS+AG through the host proxy (input = rank).
        Returns (us per AllReduce, correct, proxy NUMA node)."""
        out = (ctypes.c_double * 3)()
        check(lib().mscclppAmdProxyRingAllReduce(self.comm, nelems, iters, graph_launches, nblocks, out),
              "proxy ring allreduce")
        return out[0], out[1] == 1.0, int(out[2])

    def barrier(self):
        check(lib().mscclppAmdCommBarrier(self.comm), "barrier")

    def device_error(self, clear=True):
        c = ctypes.c_uint32()
        check(lib().mscclppAmdCommGetDeviceError(self.comm, ctypes.byref(c), 1 if clear else 0), "device error")
        return c.value

    def device_error_detail(self, clear=True):
        """[code, detail1, detail2, detail3]: for a packet timeout, the flag waited for, the packet's
        byte offset in the polled region and the flag word last read there."""
        w = (ctypes.c_uint32 * 4)()
        check(lib().mscclppAmdCommGetDeviceErrorDetail(self.comm, w, 1 if clear else 0), "device error detail")
        return list(w)

    def async_error(self):
        """ncclCommGetAsyncError: 0 (ncclSuccess), or 6 (ncclRemoteError) once a wait timed out."""
        c = ctypes.c_int32()
        check(lib().ncclCommGetAsyncError(self.comm, ctypes.byref(c)), "ncclCommGetAsyncError")
        return c.value

    def registration_stats(self):
        """(user buffers registered, IPC mappings open in this process, mappings awaiting close)."""
        a, b, c = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        check(lib().mscclppAmdCommRegistrationStats(self.comm, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
              "registration stats")
        return a.value, b.value, c.value

    def registration_exchanges(self):
        """(allocation exchanges, offset exchanges, symmetric memory on) of user-buffer registration."""
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
        check(lib().mscclppAmdCommRegistrationExchanges(self.comm, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
              "registration exchanges")
        return a.value, b.value, bool(c.value)

    def destroy(self):
        if self.comm:
            check(lib().ncclCommDestroy(self.comm), "ncclCommDestroy")
            self.comm = None


# ---- execution plans / executor (include/mscclpp_amd/executor.h; reference executor.hpp) ----------

class DataType:
    """mscclpp.DataType values (gpu_data_types.hpp:169-183)."""
    int32, uint32, float16, float32, bfloat16 = 0, 1, 2, 3, 4
    float8_e4m3fn, float8_e4m3fnuz, float8_e5m2, float8_e5m2fnuz = 5, 6, 7, 8
    uint8, float8_e4m3b15 = 9, 10  # e4m3b15 has no torch dtype: pass it explicitly over a uint8 buffer


EXEC_DTYPES = {torch.int32: DataType.int32, torch.float16: DataType.float16, torch.float32: DataType.float32,
               torch.bfloat16: DataType.bfloat16, torch.float8_e4m3fn: DataType.float8_e4m3fn,
               torch.float8_e5m2: DataType.float8_e5m2, torch.float8_e4m3fnuz: DataType.float8_e4m3fnuz,
               torch.float8_e5m2fnuz: DataType.float8_e5m2fnuz, torch.uint8: DataType.uint8}


class PacketType:
    """mscclpp.PacketType (executor.hpp:15-18)."""
    LL8, LL16 = 0, 1


class ExecutionPlan:
    """mscclpp.ExecutionPlan(plan_path, rank): a JSON plan resolved for one rank."""

    def __init__(self, plan_path, rank):
        p = ctypes.c_void_p()
        check(lib().mscclppAmdExecutionPlanCreate(os.fsencode(plan_path), rank, ctypes.byref(p)),
              f"ExecutionPlan({plan_path})")
        self.handle, self.rank, self.path = p, rank, plan_path

    def name(self):
        return lib().mscclppAmdExecutionPlanName(self.handle).decode()

    def collective(self):
        return lib().mscclppAmdExecutionPlanCollective(self.handle).decode()

    def min_message_size(self):
        return lib().mscclppAmdExecutionPlanMinMessageSize(self.handle)

    def max_message_size(self):
        return lib().mscclppAmdExecutionPlanMaxMessageSize(self.handle)

    def is_in_place(self):
        return bool(lib().mscclppAmdExecutionPlanIsInPlace(self.handle))

    def describe(self, input_bytes, output_bytes):
        """The plan lowered for this rank at these message sizes (host only), as a dict."""
        import json

        need = ctypes.c_size_t()
        check(lib().mscclppAmdExecutionPlanDescribe(self.handle, input_bytes, output_bytes, None, 0, ctypes.byref(need)),
              "ExecutionPlan.describe")
        buf = ctypes.create_string_buffer(need.value)
        check(lib().mscclppAmdExecutionPlanDescribe(self.handle, input_bytes, output_bytes, buf, need.value,
                                                    ctypes.byref(need)), "ExecutionPlan.describe")
        return json.loads(buf.value.decode())

    def __del__(self):
        try:
            if self.handle:
                lib().mscclppAmdExecutionPlanDestroy(self.handle)
                self.handle = None
        except Exception:
            pass


class Executor:
    """mscclpp.Executor(comm): runs execution plans on a Communicator (collective setup)."""

    def __init__(self, comm):
        e = ctypes.c_void_p()
        check(lib().mscclppAmdExecutorCreate(comm.comm, ctypes.byref(e)), "Executor")
        self.handle, self.comm = e, comm

    def execute(self, rank, send_ptr, recv_ptr, send_size, recv_size, dtype, plan, stream=None,
                packet_type=PacketType.LL16):
        """Executor::execute (executor.hpp:85-86); pointers are device addresses, dtype a DataType."""
        sp = stream if isinstance(stream, (int, ctypes.c_void_p)) else stream_ptr(stream)
        check(lib().mscclppAmdExecutorExecute(self.handle, rank, ctypes.c_void_p(send_ptr), ctypes.c_void_p(recv_ptr),
                                              send_size, recv_size, dtype, plan.handle,
                                              sp if isinstance(sp, ctypes.c_void_p) else ctypes.c_void_p(sp),
                                              packet_type), "Executor.execute")

    def reset(self):
        check(lib().mscclppAmdExecutorReset(self.handle), "Executor.reset")

    def device_error(self, clear=True):
        w = (ctypes.c_uint32 * 4)()
        check(lib().mscclppAmdExecutorGetDeviceError(self.handle, w, 1 if clear else 0), "Executor.device_error")
        return list(w)

    def destroy(self):
        if self.handle:
            check(lib().mscclppAmdExecutorDestroy(self.handle), "Executor.destroy")
            self.handle = None
