"""The reference's user-level setup written with its own spellings (tests/cpp/test_reference_setup.hip):
TcpBootstrap + Communicator(bootstrap) + EndpointConfig{transport, {DeviceType, id}} + GpuBuffer +
DeviceSyncer, on this library -- a PortChannel loopback on one rank (test/unit/local_channel_tests.cu),
the memory-channel tutorial's put / get / packet round between two processes meeting at "ip:port"
(examples/tutorials/03-memory-channel), a UniqueId made in the parent, and the Context / Endpoint /
SemaphoreStub ping-pong of examples/tutorials/01-basic-concepts in one process."""
import json
import os
import socket
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "bin", "test_reference_setup")


def _run(args, timeout=120):
    env = dict(os.environ, MSCCLPP_AMD_SPIN_TIMEOUT_MS="5000")
    try:
        r = subprocess.run([EXE] + args, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                           timeout=timeout, env=env)
    except subprocess.TimeoutExpired as e:  # say what the ranks printed last, not only that time ran out
        out = e.output.decode(errors="replace") if isinstance(e.output, bytes) else (e.output or "")
        raise AssertionError(f"{args[0]} timed out after {timeout} s; output tail:\n{out[-3000:]}\n"
                             f"{_other_processes()}") from None
    assert r.returncode == 0, r.stdout[-3000:] + "\n" + _other_processes()
    return r.stdout


def _other_processes():
    """The box's other python / test-binary processes (a leftover of an earlier test that still holds
    the GPU shows here)."""
    ps = subprocess.run(["ps", "-eo", "pid,ppid,etimes,stat,args"], stdout=subprocess.PIPE, text=True)
    keep = [x[:200] for x in ps.stdout.splitlines()[1:] if any(k in x for k in ("python", "tests/bin", "tools/"))]
    return "processes:\n" + "\n".join(keep)


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_port_channel_loopback_one_rank(built):
    out = _run(["local"])
    assert "local OK" in out
    rows = [json.loads(x.split(" ", 1)[1]) for x in out.splitlines() if x.startswith("LOCAL_JSON ")]
    assert [r["bytes"] for r in rows] == [1024, 1 << 20] and all(r["us_per_iter"] > 0 for r in rows), out
    print(rows)


def test_memory_channel_tutorial_ip_port(built):
    """examples/tutorials/03-memory-channel: put, get and putPackets/unpackPackets between two processes
    meeting at "ip:port", exact; then the tutorial's timing -- 1000 graph-captured launches per kernel
    at 1 KiB, 1 MiB and 128 MiB with its own log line (docs/tutorials/03-memory-channel.md:26-34
    publishes 344.8 GB/s put, 321.5 get, 131.7 put-packets at 128 MiB)."""
    out = _run(["pair", str(_free_port())], timeout=180)
    assert "rank 0 pair OK" in out and "rank 1 pair OK" in out and "pair OK" in out
    rows = [json.loads(x.split(" ", 1)[1]) for x in out.splitlines() if x.startswith("PAIR_JSON ")]
    assert [(r["kernel"], r["bytes"]) for r in rows] == [
        (k, b) for k in ("Bidir Put", "Bidir Get", "Bidir Put Packets") for b in (1024, 1 << 20, 128 << 20)], out
    assert all(r["us_per_iter"] > 0 for r in rows), rows
    print([x for x in out.splitlines() if "[Bidir" in x])


def test_port_channel_tutorial_graph_replays(built):
    """examples/tutorials/04-port-channel as written: 1000 graph-captured bidirectional putWithSignal
    iterations at 1 KiB, 1 MiB and 128 MiB, exact, with the tutorial's own `elapsed ms/iter, BW` line
    (docs/tutorials/04-port-channel.md:25 publishes 25.0 us/iter, 41.9 GB/s at 1 MiB)."""
    out = _run(["port", str(_free_port())])
    assert "rank 0 port OK" in out and "rank 1 port OK" in out, out
    rows = [json.loads(x.split(" ", 1)[1]) for x in out.splitlines() if x.startswith("PORT_JSON ")]
    assert [r["bytes"] for r in rows] == [1024, 1 << 20, 128 << 20], out
    assert all(r["us_per_iter"] > 0 for r in rows), rows
    print([x for x in out.splitlines() if "[Bidir PutWithSignal]" in x])


def test_unique_id_from_parent(built):
    out = _run(["uid"])
    assert "rank 0 uid OK" in out and "rank 1 uid OK" in out


def test_context_endpoints_ping_pong(built):
    out = _run(["context"])
    assert "context OK" in out, out


@pytest.mark.parametrize("plan", ["allreduce_packet.json", "allreduce.json"])
def test_executor_api_reference_plans(built, plan):
    """test/executor_test.cc's sequence on the reference's own 2-rank plans (fixtures)."""
    out = _run(["executor", os.path.join(ROOT, "tests", "golden", "plans", "ref", plan)])
    assert "rank 0 executor OK" in out and "rank 1 executor OK" in out, out


def test_host_utilities_errors_and_atomics(built):
    """test/unit/numa_tests.cc and utils_tests.cc as the reference writes them, the BaseError /
    CudaError hierarchy, and atomicStore / POLL_MAYBE_JAILBREAK(atomicLoad) between two blocks."""
    assert "utils OK" in _run(["utils"])
