"""The N>1 benchmark's bit-exact check can fail: two ranks sharing the GPU
(rehearsal), a fullmesh AllReduce whose reduce-scatter handshake is skipped on purpose
(MSCCLPP_AMD_DEBUG_SKIP_HANDSHAKE=1) must be reported as not bit-exact, and the same run without
the knob as bit-exact."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(extra_env):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(extra_env)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--algo", "fullmesh",
                        "--bytes", str(8 << 20), "--steps", "3", "--warmup", "1", "--no-extras"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line)


def test_skipped_handshake_is_caught(built):
    good = _bench({})
    assert good["correct"] is True and good["correct_bitexact"]["timed_last_step"] is True
    # the N>1 line is complete: roofline, the CPU sum and the host-proxy loop
    # at the job's world size, each with its cores
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(good["roofline"])
    assert good["cpu_baseline"]["cores"] >= 1 and "2-way sum" in good["cpu_baseline"]["sample"]
    hp = good["host_proxy_baseline"]
    assert hp.get("ranks") == 2 and hp.get("cores") == 4 and hp.get("correct") is True, hp
    bad = _bench({"MSCCLPP_AMD_DEBUG_SKIP_HANDSHAKE": "1"})
    assert bad["correct"] is False
    assert any(v is False for k, v in bad["correct_bitexact"].items() if k.startswith("fullmesh"))
