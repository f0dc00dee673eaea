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
