"""The host channel API and the reference's device spellings:

* tests/cpp/test_fifo.hip -- the FIFO known-answer tests of test/unit/fifo_tests.cu:15-162 on the
  device FIFO with the host poller (10k pushes fst = snd = i, zero triggers, lap-wrap parity with the
  commit bit cleared, rejection of a non-power-of-two size);
* tests/cpp/test_channels.hip -- two processes building MemoryChannels and PortChannels with
  Communicator::connect / registerMemory / sendMemory / recvMemory / MemoryDevice2DeviceSemaphore /
  ProxyService, driven by kernels written with the reference's spellings (LL8/LL16 packet ping-pong
  of test/mp_unit/memory_channel_tests.cu:246-325, unpackPacket, put/get ping-pong, the proxy LL
  ping-pong of port_channel_tests.cu:337-446 with copyToPackets / copyFromPackets);
* tests/cpp/test_customized_allgather.hip -- a user AllGather plugged in through the C++ algorithm
  interface with the API sequence of the reference's plugin example (examples/customized-collective-
  algorithm/): PortChannels through ProxyService, reached through ncclAllGather, direct and
  graph-captured, exact.
Both C++ programs include the reference's header paths (include/mscclpp/*.hpp) and spell mscclpp::."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "bin")


def _run(name, args, timeout):
    env = dict(os.environ, MSCCLPP_AMD_SPIN_TIMEOUT_MS="10000")
    r = subprocess.run([os.path.join(BIN, name)] + args, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-4000:]
    return r.stdout


def test_fifo_rejects_non_power_of_two(built):
    assert "reject OK" in _run("test_fifo", ["cpu"], 60)


@pytest.mark.gpu
def test_fifo_known_answers_on_device(built):
    out = _run("test_fifo", ["gpu"], 120)
    for part in ("reject OK", "fifo OK", "zero OK", "wrap OK", "gpu OK"):
        assert part in out, out


@pytest.mark.gpu
def test_memory_and_port_channels_reference_spellings(built):
    out = _run("test_channels", ["gpu", str(1 << 20)], 200)
    assert "gpu OK" in out and "rank 0 OK" in out and "rank 1 OK" in out, out
    # the timed 1024-int ping-pongs (memory_channel_tests.cu:98-107), printed in framework.cc's form
    line = [x for x in out.splitlines() if x.startswith("PINGPONG_JSON ")]
    assert len(line) == 1 and "LL16 latency:" in out and "LL8 latency:" in out, out
    pp = json.loads(line[0].split(" ", 1)[1])
    assert pp["iters"] >= 100000 and 0 < pp["ll8_pingpong_us"] < 1000 and 0 < pp["ll16_pingpong_us"] < 1000, pp
    print(line[0])


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 4])
@pytest.mark.parametrize("mode", ["cached", "uncached", "direct"])
def test_customized_allgather_port_channels(built, n, mode):
    """PortChannel destinations: the example's hipMalloc receive
    buffer is exact and gets the one-time warning; a pool (uncached) receive buffer gets none; an
    uncached buffer from hipExtMallocWithFlags itself is accepted even under strict."""
    out = _run("test_customized_allgather", ["gpu", str(n), str(1 << 18), mode], 200)
    assert "gpu OK" in out and all(f"rank {r} OK" in out for r in range(n)), out
    assert ("is cached device memory" in out) == (mode == "cached"), out


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 4])
def test_port_channel_strict_refuses_cached_destination(built, n):
    """MSCCLPP_AMD_PORT_CHANNEL_DST=strict: a PortChannel into cached device memory is refused with
    ncclInvalidUsage and the reason in ncclGetLastError, on every rank and with no rank left waiting."""
    out = _run("test_customized_allgather", ["gpu", str(n), str(1 << 12), "refuse"], 120)
    assert "gpu OK" in out and all(f"rank {r} refused OK" in out for r in range(n)), out


@pytest.mark.gpu
def test_device_syncer_back_to_back(built):
    """DeviceSyncer.sync() called back to back by 128 workgroups for 3 x 20000 rounds (two
    barriers each): no arrival lost to the previous generation's reset (no spin-bound expiry) and
    every slot stored before a barrier is read after it."""
    out = _run("test_device_syncer", ["gpu", "128", "20000"], 100)
    assert "gpu OK" in out and "mismatches 0 timedOut 0" in out, out
