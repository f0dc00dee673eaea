"""torch.distributed's "nccl" backend on libmscclpp_amd.so (LD_PRELOAD), two ranks on one GPU:
all_reduce / all_gather_into_tensor / reduce_scatter_tensor / broadcast / barrier checked against
locally computed references (tools/torch_dist_check.py; the reference's test/torch/correctness_test.py
flow).  RCCL refuses two ranks on one device, so the run passing means the interposed library
carried every collective."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_torch_distributed_nccl_backend_on_mscclpp_amd(built):
    import mscclpp_amd as m

    import torch

    # a torch wheel that bundles its own HIP runtime must share it with this library: preload that
    # runtime first so libmscclpp_amd.so binds to it (one HIP runtime per process)
    bundled = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    preload = f"{bundled}:{m.LIB_PATH}" if os.path.exists(bundled) else m.LIB_PATH
    env = dict(os.environ, LD_PRELOAD=preload, MSCCLPP_AMD_SPIN_TIMEOUT_MS="10000")
    env.pop("MSCCLPP_AMD_NCCL_LIB_PATH", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29651", os.path.join(ROOT, "tools", "torch_dist_check.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=200)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, r.stdout[-4000:]
    res = json.loads(lines[-1])
    assert res["interposed"] and res["all_ranks_ok"], res
    assert len(res["checks"]) >= 30
