"""The C++ algorithm plugin interface (include/mscclpp_amd/algorithm.hpp): AlgorithmCollection,
selectors, NativeAlgorithm context caching, AlgorithmCollectionBuilder (host-only checks), and a
user algorithm + selector registered before ncclCommInitRank reached through ncclAllGather /
ncclAllReduce in forked processes (the reference's examples/customized-collective-algorithm)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "bin", "test_algorithm_plugin")


def _run(args, timeout, forced=None):
    env = dict(os.environ, MSCCLPP_AMD_SPIN_TIMEOUT_MS="5000")
    env.pop("MSCCLPP_AMD_ALGO", None)
    if forced:
        env["MSCCLPP_AMD_ALGO"] = forced
    r = subprocess.run([EXE] + args, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=timeout,
                       env=env)
    assert r.returncode == 0, r.stdout[-3000:]
    return r.stdout


def test_plugin_host_logic(built):
    assert "cpu OK" in _run(["cpu"], 60)


def test_env_forced_algorithm(built):
    """MSCCLPP_AMD_ALGO (read once per process) forces the built-in selector's choice."""
    assert "forced OK" in _run(["cpu"], 60, forced="packet")


@pytest.mark.gpu
def test_plugin_user_algorithm_through_nccl_abi(built):
    out = _run(["gpu", "2"], 100)
    assert "gpu OK" in out and "rank 0 OK" in out and "rank 1 OK" in out
