"""GPU tests of the device primitive surface (include/mscclpp_amd/memory_channel_device.hpp):
LL16 / LL8 packet ping-pong through putPackets / unpackPackets with flag = iteration + 1
(test/mp_unit/memory_channel_tests.cu:246-338) and put + signal / wait round trips."""
import ctypes

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode,name", [(0, "ll16_pingpong"), (1, "ll8_pingpong"), (2, "put_signal_wait")])
@pytest.mark.parametrize("nelem", [2, 1024, 1 << 18])
def test_memory_channel_selftest(built, mode, name, nelem):
    import mscclpp_amd as m

    L = m.lib()
    L.mscclppAmdMemChannelSelfTest.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                               ctypes.POINTER(ctypes.c_uint32)]
    fails, err = ctypes.c_int(-1), ctypes.c_uint32(99)
    assert L.mscclppAmdMemChannelSelfTest(mode, nelem, 20, ctypes.byref(fails), ctypes.byref(err)) == 0
    assert err.value == 0, f"{name}: device error {err.value}"
    assert fails.value == 0, f"{name}: {fails.value} mismatches"


@pytest.mark.parametrize("mode,unit", [(3, 16), (4, 8)])
def test_unpack_packets_timeout_record(built, mode, unit):
    """a packet that never arrives ends unpackPackets at the handle's budget (20 ms
    here) with the whole error record: kErrPacketTimeout, the flag waited for (7), the byte offset of
    a packet inside the polled region, and the flag word found there (0: never written)."""
    import mscclpp_amd as m

    L = m.lib()
    L.mscclppAmdMemChannelSelfTest.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                               ctypes.POINTER(ctypes.c_uint32)]
    fails, rec = ctypes.c_int(-1), (ctypes.c_uint32 * 4)()
    nelem = 4096
    assert L.mscclppAmdMemChannelSelfTest(mode, nelem, 1, ctypes.byref(fails), rec) == 0
    code, flag, where, seen = list(rec)
    assert code == 1 and flag == 7 and seen == 0, list(rec)
    packets = nelem // 2 if unit == 16 else nelem
    assert where % unit == 0 and where < packets * unit, list(rec)
