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


def test_invalid_arguments_rejected_without_gpu(built):
    import mscclpp_amd as m

    L = m.lib()
    assert L.ncclAllReduce(None, None, 0, 6, 0, None, None) == 4  # null comm
    assert L.ncclCommInitRank(None, 2, m.UniqueId(), 0) == 4
    arr = (m.RankView * 1)()
    assert L.mscclppAmdAllReduceLaunch(1, arr, 1, 1, 1024, 0, 0, 0, 0, 0, None) == 4  # nranks < 2
    assert L.mscclppAmdAllReduceLaunch(1, arr, 1, 8, 1024, 9, 0, 0, 0, 0, None) == 4  # bad dtype
