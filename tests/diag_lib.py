"""Test diagnostics: read a device buffer through every XCD's L2 (tests/diag/xcd_probe.hip, built into
tests/bin/libxcdprobe.so by mscclpp_amd/_build.py) and say which XCDs see which words wrong.

A word only some XCDs read wrong is a stale line in those XCDs' L2s (memory holds the right value);
a word every XCD reads wrong is missing from memory itself."""
import ctypes
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = ctypes.CDLL(os.path.join(ROOT, "tests", "bin", "libxcdprobe.so"))
        _LIB.xcdCompare.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                    ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.c_void_p]
        _LIB.xcdCompare.restype = ctypes.c_int
    return _LIB


def xcd_compare(t, expect_words, workgroups=64):
    """Per-XCD view of device tensor `t` (any dtype) against `expect_words` (numpy uint32, the words
    `t` should hold).  Returns {xcd: {"bad", "first", "last", "workgroups"}} for XCDs that ran."""
    nw = t.numel() * t.element_size() // 4
    exp = torch.from_numpy(np.ascontiguousarray(expect_words[:nw]).view(np.int32)).pin_memory()
    out = (ctypes.c_uint64 * 32)()
    rc = lib().xcdCompare(ctypes.c_void_p(t.data_ptr()), nw, ctypes.c_void_p(exp.data_ptr()), out, workgroups,
                          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, f"xcdCompare rc {rc}"
    res = {}
    for x in range(8):
        wg = int(out[x * 4 + 3])
        if wg:
            bad = int(out[x * 4 + 0]) // wg  # every workgroup reads the whole buffer
            res[x] = {"bad": bad, "first": int(out[x * 4 + 1]) if bad else None,
                      "last": int(out[x * 4 + 2]) if bad else None, "workgroups": wg}
    return res
