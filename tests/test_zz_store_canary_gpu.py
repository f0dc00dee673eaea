"""Runs last in the `-m gpu` session (file order): after every other GPU test has run in this
long-lived process, freshly allocated torch buffers must receive every store of a kernel, as seen
both by a copy-out and by every XCD's L2 (the lost-store failure of round 2)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_fresh_buffers_receive_every_store(built):
    import diag_lib

    ts = [torch.empty(1 << 18, dtype=torch.int32, device="cuda") for _ in range(128)]
    for i, t in enumerate(ts):
        t.fill_(7000 + i)
    torch.cuda.synchronize()
    bad = []
    for i, t in enumerate(ts):
        n = int((t.cpu() != 7000 + i).sum())
        xcd = diag_lib.xcd_compare(t, np.full(t.numel(), 7000 + i, dtype=np.int32).view(np.uint32))
        if n or any(v["bad"] for v in xcd.values()):
            bad.append((hex(t.data_ptr()), n, xcd))
    assert not bad, bad[:4]
