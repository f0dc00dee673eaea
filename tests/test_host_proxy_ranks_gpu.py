"""The reference's host-proxy path (test/allgather_test_host_offloading.cu) and the PortChannel
all-to-all through ProxyService at 4 ranks, as spawned processes on this box's GPU: every copy stream
of a rank's connections must stay runnable while that rank's kernel spins for its peers' data (a
per-connection stream can share the spinning kernel's hardware queue -- HIP maps a process's streams
onto four -- which hung this run before the connections shared one copy stream)."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_host_offload_and_portchannel_four_ranks(built):
    import host_proxy_baseline as H

    r = H.run(4, 4096, timeout=110)
    assert r["correct"] is True and r["ranks"] == 4 and r["cores"] == 8
    for mode, row in r["portchannel_alltoall_1MiB"].items():
        assert row["correct"] is True, mode


def test_memory_channel_pingpong_two_ranks(built):
    """The reference's MemoryChannel packet ping-pong latency (memory_channel_tests.cu:98-107) through
    the library entry the bench line uses: both packet types correct over 1000 checked and 100k timed
    one-way hand-offs of 1024 ints, with a finite us/iter (two processes sharing this GPU)."""
    import host_proxy_baseline as H

    r = H.run(2, 4096, timeout=150)
    assert r["correct"] is True and r["pingpong_correct"] is True, r.get("pingpong")
    for name in ("ll16", "ll8"):
        row = r["pingpong"][name]
        assert row["error_record"] == [0, 0, 0, 0] and 0 < row["us_per_iter"] < 1000, (name, row)
    print("pingpong", r["pingpong"])
