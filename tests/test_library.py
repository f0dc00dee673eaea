"""CPU checks of the C-ABI library: it loads, exports every symbol include/mscclpp_amd/*.h declares,
and its host-side logic (algorithm selection, scratch sizing) behaves without a GPU."""
import ctypes
import glob
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "mscclpp_amd", "*.h")):
        txt = open(h).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b((?:nccl|mscclppAmd)\w+)\s*\(", txt, re.M):
            names.add(m.group(1))
    return names


def test_exports_every_declared_symbol(built):
    from mscclpp_amd import LIB_PATH

    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    declared = declared_functions()
    assert len(declared) >= 30
    missing = sorted(declared - exported)
    assert not missing, missing


def test_loads_and_host_logic(built):
    import mscclpp_amd as m

    L = m.lib()
    v = ctypes.c_int()
    assert L.ncclGetVersion(ctypes.byref(v)) == 0 and v.value >= 22600
    assert L.ncclGetErrorString(4) == b"invalid argument"
    # selector: algorithm_selector.cc:107-131 for AMD
    assert L.mscclppAmdSelectAlgo(8, 1024, m.F16) == m.ALGO_ALLPAIR
    assert L.mscclppAmdSelectAlgo(8, 16 << 10, m.F16) == m.ALGO_ALLPAIR
    assert L.mscclppAmdSelectAlgo(8, (16 << 10) + 2, m.F16) == m.ALGO_PACKET
    assert L.mscclppAmdSelectAlgo(8, 1 << 20, m.F16) == m.ALGO_PACKET
    assert L.mscclppAmdSelectAlgo(8, 48 << 20, m.F16) == m.ALGO_FULLMESH
    # scratch sizing: LL16 at 1 MiB fp16, 8 ranks: half = 4S + 2S (6*S per half)
    s = m.scratch_required(m.ALGO_PACKET, 8, 1 << 20, m.F16)
    assert s == 2 * 6 * (1 << 20)
    assert m.scratch_required(m.ALGO_ALLPAIR, 8, 16 << 10, m.F16) == 2 * 8 * (16 << 10) * 2


def test_buffer_resource_offset_limits(built):
    """Buckets whose LL offsets would pass 4 GiB from one descriptor are refused (0 = ncclInvalidUsage
    at the call); the bulk pass is capped so the reduce step's n regions stay within 4 GiB."""
    import mscclpp_amd as m

    MiB, GiB = 1 << 20, 1 << 30
    # LL16: the n input regions of a scratch half span 2 * bytes
    assert m.scratch_required(m.ALGO_PACKET, 8, 2 * GiB - MiB, m.F16) > 0
    assert m.scratch_required(m.ALGO_PACKET, 8, 2 * GiB + MiB, m.F16) == 0
    assert m.scratch_required(m.ALGO_TEST_K6, 2, GiB, m.I32) > 0
    assert m.scratch_required(m.ALGO_TEST_K6, 2, 2 * GiB + 16 * MiB, m.I32) == 0
    # LL8: every rank's whole buffer in one half: 2 * n * bytes
    assert m.scratch_required(m.ALGO_ALLPAIR, 8, 255 * MiB, m.F16) > 0
    assert m.scratch_required(m.ALGO_ALLPAIR, 8, 257 * MiB, m.F16) == 0
    assert m.scratch_required(m.ALGO_TEST_K2, 8, 257 * MiB, m.I32) == 0
    # bulk: n regions of one pass within 4 GiB of the reduce step's descriptor
    for n in (2, 8):
        s = m.scratch_required(m.ALGO_FULLMESH, n, 48 * GiB, m.F16)
        assert 0 < s <= 4 * GiB - 64
    assert m.scratch_required(m.ALGO_FULLMESH, 8, 48 * MiB, m.F16) == 48 * MiB  # one pass, as before


def test_invalid_arguments_rejected_without_gpu(built):
    import mscclpp_amd as m

    L = m.lib()
    assert L.ncclAllReduce(None, None, 0, 6, 0, None, None) == 4  # null comm
    assert L.ncclCommInitRank(None, 2, m.UniqueId(), 0) == 4
    arr = (m.RankView * 1)()
    assert L.mscclppAmdAllReduceLaunch(1, arr, 1, 1, 1024, 0, 0, 0, 0, 0, None) == 4  # nranks < 2
    assert L.mscclppAmdAllReduceLaunch(1, arr, 1, 8, 1024, 9, 0, 0, 0, 0, None) == 4  # bad dtype


def test_exports_every_nccl_symbol_torch_imports(built):
    """Under LD_PRELOAD / LD_AUDIT the library stands in for librccl: every ncclXxx symbol that
    libtorch_hip.so binds must resolve to it, or torch would call the vendor library with this
    library's communicator."""
    import glob
    import subprocess

    import torch

    import mscclpp_amd as m

    libs = glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "libtorch_hip.so"))
    if not libs:
        pytest.skip("no libtorch_hip.so in this torch build")
    undef = subprocess.run(["nm", "-D", "--undefined-only", libs[0]], stdout=subprocess.PIPE, text=True).stdout
    wanted = {ln.split()[-1].split("@")[0] for ln in undef.splitlines() if " nccl" in ln}
    ours = subprocess.run(["nm", "-D", "--defined-only", m.LIB_PATH], stdout=subprocess.PIPE, text=True).stdout
    have = {ln.split()[-1] for ln in ours.splitlines() if " T " in ln}
    assert wanted, "expected torch to import NCCL symbols"
    assert not (wanted - have), sorted(wanted - have)


def test_vendor_fallback_absent_means_invalid_usage(built):
    """Without MSCCLPP_AMD_NCCL_LIB_PATH, operations outside the path answer ncclInvalidUsage /
    ncclInvalidArgument instead of crashing (no communicator or GPU needed for these checks)."""
    import mscclpp_amd as m

    L = m.lib()
    vp = ctypes.c_void_p
    L.ncclSend.argtypes = [vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, vp, vp]
    L.ncclCommRegister.argtypes = [vp, vp, ctypes.c_size_t, ctypes.POINTER(vp)]
    assert L.ncclSend(None, 1, 7, 0, None, None) == 4  # null communicator
    h = vp()
    assert L.ncclCommRegister(None, None, 0, ctypes.byref(h)) == 4
    assert L.ncclGroupStart() == 0 and L.ncclGroupEnd() == 0


# Every entry point src/ext/nccl/nccl.cc defines (NCCL_API functions of the reference's shim).
REFERENCE_NCCL_SYMBOLS = """ncclAllGather ncclAllReduce ncclAllToAll ncclAllToAllv ncclBcast ncclBroadcast ncclCommAbort
ncclCommCount ncclCommCuDevice ncclCommDeregister ncclCommDestroy ncclCommFinalize ncclCommGetAsyncError
ncclCommInitAll ncclCommInitRank ncclCommInitRankConfig ncclCommInitRankScalable ncclCommRegister ncclCommSplit
ncclCommUserRank ncclCommWindowDeregister ncclCommWindowRegister ncclGetErrorString ncclGetLastError
ncclGetUniqueId ncclGetVersion ncclGroupEnd ncclGroupSimulateEnd ncclGroupStart ncclMemAlloc ncclMemFree
ncclRecv ncclRedOpCreatePreMulSum ncclRedOpDestroy ncclReduce ncclReduceScatter ncclSend""".split()


def test_exports_every_reference_nccl_entry_point(built):
    """The drop-in exports every function of the reference's NCCL shim (a binary built against its
    nccl.h resolves all of them), and the window registration hands the buffer back like
    ncclCommRegister (nccl.cc:511-519)."""
    import mscclpp_amd as m

    ours = subprocess.run(["nm", "-D", "--defined-only", m.LIB_PATH], stdout=subprocess.PIPE, text=True).stdout
    have = {ln.split()[-1] for ln in ours.splitlines() if " T " in ln}
    assert not (set(REFERENCE_NCCL_SYMBOLS) - have), sorted(set(REFERENCE_NCCL_SYMBOLS) - have)
    L = m.lib()
    vp = ctypes.c_void_p
    L.ncclCommWindowRegister.argtypes = [vp, vp, ctypes.c_size_t, ctypes.POINTER(vp), ctypes.c_int]
    L.ncclCommWindowDeregister.argtypes = [vp, vp]
    w = vp()
    assert L.ncclCommWindowRegister(None, None, 0, ctypes.byref(w), 0) == 4
    assert L.ncclCommWindowDeregister(None, None) == 4


def test_flag_alignment_and_mix_sizes_rejected_without_gpu(built):
    """Round 4: flag buffers are refreshed 16 bytes at a time, so a misaligned flag pointer is an
    invalid argument (checked before any launch), and the generic mix ceiling takes whole 4 KiB passes."""
    import mscclpp_amd as m

    L = m.lib()
    vp = ctypes.c_void_p
    fake = vp(1 << 20)
    assert L.mscclppAmdSelfReduceLL16(fake, fake, fake, fake, 4096, m.F16, m.SUM, vp((1 << 20) + 4), 0, 1000, fake,
                                      None) == 4
    arr = (m.RankView * 2)()
    for r in range(2):
        v = arr[r]
        v.input = v.output = v.scratch = v.tokens = v.expected = v.err = 1 << 20
        v.flags = (1 << 20) + 8  # not 16-byte aligned
        v.scratchBytes = 1 << 20
        v.rank = r
        for q in range(2):
            v.peerScratch[q] = v.peerOutput[q] = v.peerInput[q] = v.peerTokens[q] = 1 << 20
    assert L.mscclppAmdAllReduceLaunch(m.ALGO_ALLPAIR, arr, 2, 2, 1024, m.F16, m.SUM, 0, 0, 1000, None) == 4
    assert L.mscclppAmdMixStream(fake, fake, fake, fake, fake, 4096 + 16, 0, None) == 4


def test_build_all_reports_what_it_built(built):
    """build() prints one line naming what it compiled and linked (the driver's build check can tell a
    real build from an up-to-date tree); right after the session build nothing is out of date."""
    from mscclpp_amd import _build

    line = _build.build_all()
    assert line.startswith("build: 0 objects compiled, 0 artefacts linked (all up to date)"), line
    assert "oracle/_ref:" in line
