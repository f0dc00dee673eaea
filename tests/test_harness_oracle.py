"""CPU checks of the oracle's mscclpp-test allreduce2 restatement (oracle/ll_oracle.c
oracle_mscclpp_test_k2, test/mscclpp-test/allreduce_test.cu:841-943 on one node): the harness's
known answer (input = rank -> n(n-1)/2 everywhere, allreduce_test.cu:1172-1183) and the scratch
layout, against a plain-Python walk of the kernel's offsets for small cases."""
import numpy as np
import pytest

import oracle_lib as O


def _walk_k2(ins, nelems, flag):
    """Each rank s writes LLPacket {x, flag, y, flag} of its pairs into peer q's scratch at packet
    scratchBaseIndex + (s < q ? s : s - 1) * nPkts (:861-863, :876-880)."""
    n = len(ins)
    npk = nelems // 2
    base = 0 if flag & 1 else npk * (n - 1)
    scr = [np.zeros(2 * npk * (n - 1) * 4, np.uint32) for _ in range(n)]
    for s in range(n):
        for q in range(n):
            if q == s:
                continue
            slot = s if s < q else s - 1
            for i in range(npk):
                o = (base + slot * npk + i) * 4
                scr[q][o:o + 4] = [ins[s][2 * i], flag, ins[s][2 * i + 1], flag]
    outs = [(np.sum(np.stack([a.astype(np.int64) for a in ins]), axis=0) & 0xFFFFFFFF).astype(np.uint32)
            for _ in range(n)]
    return outs, scr


@pytest.mark.parametrize("n,nelems,flag", [(2, 8, 1), (3, 6, 2), (4, 16, 3), (8, 4, 4)])
def test_k2_oracle_matches_kernel_walk(n, nelems, flag):
    rng = np.random.default_rng(n * 100 + nelems)
    ins = [rng.integers(0, 2 ** 32, nelems, dtype=np.uint64).astype(np.uint32) for _ in range(n)]
    sb = 16 * nelems * (n - 1)
    got, scr = O.mscclpp_test_k2(ins, nelems, flag, sb)
    want, wscr = _walk_k2(ins, nelems, flag)
    for r in range(n):
        assert np.array_equal(got[r], want[r])
        assert np.array_equal(scr[r], wscr[r])


def test_k2_oracle_known_answer():
    n, nelems = 8, 1024
    ins = [np.full(nelems, r, np.uint32) for r in range(n)]
    got, _ = O.mscclpp_test_k2(ins, nelems, 1, 16 * nelems * (n - 1))
    assert all(np.all(g == n * (n - 1) // 2) for g in got)
