"""GPU parity of the mscclpp-test AllReduce kernels restated for gfx950 (SURVEY §8a row a16:
test/mscclpp-test/allreduce_test.cu allreduce2 / allreduce5 / allreduce6 / allreduce7), n ranks in one
process.

k2 / k6 / k7: outputs and the whole packet scratch image (harness layout, flag parity double buffering)
bit-exact against the oracle's restatement; k5 (in place, remote reads + gets): exact int32 sums.
Plus the harness's known answer (input = rank -> n(n-1)/2, allreduce_test.cu:1172-1183)."""
import numpy as np
import pytest
import torch

import oracle_lib as O

pytestmark = pytest.mark.gpu


def _rand_i32(n, count, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(-2 ** 31, 2 ** 31, count, dtype=np.int64).astype(np.int32) for _ in range(n)]


@pytest.mark.parametrize("kernel", ["k6", "k7", "k2"])
@pytest.mark.parametrize("n,count", [(2, 4096), (4, 8192), (8, 6144), (8, 65536), (3, 1536), (8, 16)])
def test_ll_test_kernels_bit_exact(built, kernel, n, count):
    import mscclpp_amd as m

    code = m.ALGO_NAMES[kernel]
    sb = m.scratch_required(code, n, count * 4, m.I32)
    # k6/k7: nPacket * 2 * 2 LLPackets; k2: nPacket * (n - 1) * 2 (allreduce_test.cu:1277-1286)
    assert sb == (8 * count * 4 if kernel != "k2" else 16 * count * (n - 1))
    oracle = O.mscclpp_test_k2 if kernel == "k2" else O.mscclpp_test_ll
    ranks = m.InProcessRanks(n, sb)
    for call, flag in enumerate((1, 2, 3)):
        ins = _rand_i32(n, count, 10 * call + n)
        dins = [torch.from_numpy(a).cuda() for a in ins]
        douts = [torch.zeros_like(d) for d in dins]
        ranks.all_reduce(dins, douts, code)
        torch.cuda.synchronize()
        assert ranks.errors() == [0] * n
        exp, scr = oracle([a.view(np.uint32) for a in ins], count, flag, sb)
        want = np.sum(np.stack([a.astype(np.int64) for a in ins]), axis=0).astype(np.uint32)  # wrapping
        for r in range(n):
            got = douts[r].cpu().numpy().view(np.uint32)
            assert np.array_equal(exp[r], want)
            assert np.array_equal(got, want), f"rank {r}"
        if call == 0:
            for r in range(n):
                img = ranks.scratch_tensor(r, sb).cpu().numpy().view(np.uint32)
                assert np.array_equal(img, scr[r]), f"scratch image of rank {r}"


def _describe_lost_words(buf, want, own, label):
    """A k5 result that differs from the sum: say which XCDs read which words wrong (a stale line in
    some XCDs' L2s vs words missing from memory), whether a second copy-out agrees, and whether the
    buffer lies in an address range this process's library allocations used before
    (m.ALLOC_HISTORY); written to gpurun_out/k5_lost_words.json."""
    import json
    import os

    import diag_lib
    import mscclpp_amd as m

    got = buf.cpu().numpy().view(np.uint32)
    bad = np.nonzero(got != want)[0]
    torch.cuda.synchronize()
    again = buf.cpu().numpy().view(np.uint32)
    lo, hi = buf.data_ptr(), buf.data_ptr() + buf.numel() * 4
    overlaps = [list(e[:3]) + [bool(e[3])] for e in m.ALLOC_HISTORY if e[1] < hi and lo < e[1] + e[2]]
    rep = {"case": label, "ptr": hex(lo), "bytes": hi - lo, "nbad": int(bad.size),
           "first": int(bad[0]), "last": int(bad[-1]),
           "bad_equal_own_input": int((got[bad] == own[bad]).sum()),
           "bad_4KiB_pages": sorted(set(int(i) * 4 // 4096 for i in bad))[:64],
           "second_copy_out_bad": int((again != want).sum()),
           "per_xcd": diag_lib.xcd_compare(buf, want),
           "library_allocs_overlapping": overlaps[-32:],
           "torch_reserved_bytes": int(torch.cuda.memory_reserved())}
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/k5_lost_words.json", "a") as f:
        f.write(json.dumps(rep) + "\n")
    return rep


def _run_k5(cases):
    """k5 (in place, remote reads + gets) cases [(n, count, seed, nblocks)], in this process."""
    import mscclpp_amd as m

    for n, count, seed, nb in cases:
        ranks = m.InProcessRanks(n, 1 << 16)
        for call in range(3):
            if seed is None:  # the harness known answer: input = rank
                ins = [np.full(count, r, dtype=np.int32) for r in range(n)]
            else:
                ins = _rand_i32(n, count, seed + call)
            bufs = [torch.from_numpy(a.copy()).cuda() for a in ins]
            ranks.all_reduce(bufs, bufs, m.ALGO_TEST_K5, nblocks=nb, nthreads=512 if nb else 0)
            torch.cuda.synchronize()
            assert ranks.errors() == [0] * n, f"n={n} count={count} call {call}: device errors"
            want = np.sum(np.stack([a.astype(np.int64) for a in ins]), axis=0).astype(np.uint32)
            for r in range(n):
                got = bufs[r].cpu().numpy().view(np.uint32)
                if not np.array_equal(got, want):
                    rep = _describe_lost_words(bufs[r], want, ins[r].view(np.uint32),
                                               f"n={n} count={count} call {call} rank {r}")
                    raise AssertionError(f"k5 result differs: {rep}")


@pytest.mark.parametrize("n,count", [(2, 4096), (4, 65536), (8, 8192), (8, 1 << 18), (5, 640)])
def test_k5_in_place(built, n, count):
    _run_k5([(n, count, 100, 24)])


def test_harness_kat(built):
    """allreduce_test.cu:1172-1183: every rank's input is its rank; every output is n(n-1)/2."""
    import mscclpp_amd as m

    n, count = 8, 1 << 14
    _run_k5([(n, count, None, 0)])  # k5 (in place), default launch shape
    for kernel in ("k6", "k7", "k2"):
        code = m.ALGO_NAMES[kernel]
        ranks = m.InProcessRanks(n, max(m.scratch_required(code, n, count * 4, m.I32), 1 << 16))
        ins = [torch.full((count,), r, dtype=torch.int32, device="cuda") for r in range(n)]
        outs = [torch.empty_like(t) for t in ins]
        ranks.all_reduce(ins, outs, code)
        torch.cuda.synchronize()
        assert ranks.errors() == [0] * n
        for o in outs:
            assert torch.all(o == n * (n - 1) // 2), kernel


def test_restrictions(built):
    """k5 runs in place; k2/k5/k7 are int32 kernels and k6 runs int32, or fp16 / fp32 SUM as the
    benchmark's allreduce2 (bf16 and fp16 MIN are refused); k6/k7 need bytes % (8 * n) == 0, k2 an
    even count."""
    import mscclpp_amd as m

    n = 4
    ranks = m.InProcessRanks(n, 1 << 20)
    a = [torch.zeros(1024, dtype=torch.int32, device="cuda") for _ in range(n)]
    b = [torch.zeros_like(t) for t in a]
    with pytest.raises(m.MscclppError):
        ranks.all_reduce(a, b, m.ALGO_TEST_K5)  # out of place
    f = [torch.zeros(1024, dtype=torch.float16, device="cuda") for _ in range(n)]
    bf = [torch.zeros(1024, dtype=torch.bfloat16, device="cuda") for _ in range(n)]
    with pytest.raises(m.MscclppError):
        ranks.all_reduce(bf, [torch.empty_like(t) for t in bf], m.ALGO_TEST_K6)
    with pytest.raises(m.MscclppError):
        ranks.all_reduce(f, [torch.empty_like(t) for t in f], m.ALGO_TEST_K6, op=m.MIN)
    with pytest.raises(m.MscclppError):
        ranks.all_reduce(f, [torch.empty_like(t) for t in f], m.ALGO_TEST_K7)
    odd = [torch.zeros(4 * n + 4, dtype=torch.int32, device="cuda") for _ in range(n)]
    with pytest.raises(m.MscclppError):
        ranks.all_reduce(odd, [torch.empty_like(t) for t in odd], m.ALGO_TEST_K6)
    with pytest.raises(m.MscclppError):
        ranks.all_reduce(f, [torch.empty_like(t) for t in f], m.ALGO_TEST_K2)
    odd2 = [torch.zeros(1023, dtype=torch.int32, device="cuda") for _ in range(n)]
    with pytest.raises(m.MscclppError):
        ranks.all_reduce(odd2, [torch.empty_like(t) for t in odd2], m.ALGO_TEST_K2)


@pytest.mark.parametrize("kernel", ["1", "2", "5", "6", "7", "rsag_zc"])
def test_harness_two_processes(built, tmp_path, kernel):
    """tools/allreduce_test_perf.py (the mscclpp-test runTest loop) with 2 ranks sharing cuda:0:
    graph-captured timing, the n(n-1)/2 data check and the JSONL perf rows."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "perf.jsonl"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str({"1": 29610, "5": 29611, "6": 29612, "7": 29613, "2": 29616}.get(kernel, 29614)),
           os.path.join(root, "tools", "allreduce_test_perf.py"), "-b", "64K", "-e", "1M", "-f", "4", "-k", kernel,
           "-w", "2", "-n", "5", "-G", "2", "-o", str(out)]
    env = dict(os.environ, MSCCLPP_AMD_SPIN_TIMEOUT_MS="5000")
    r = subprocess.run(cmd, cwd=root, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "Out of bounds values : 0 OK" in r.stdout
    rows = [json.loads(line) for line in out.read_text().splitlines()]
    assert [row["size"] for row in rows] == [64 << 10, 256 << 10, 1 << 20]
    assert all(row["ranks"] == 2 and row["time"] > 0 and row["busBw"] == pytest.approx(row["algBw"]) for row in rows)


def test_k1_large_chunks_two_processes(built, tmp_path):
    """allreduce1 at 64 MiB: copies long enough that the proxy runs ahead of its copy stream --
    every signal must carry its own token value (TokenWriter in proxy.cpp), or a waiter is released
    before the data queued ahead of a later signal has landed."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29615",
           os.path.join(root, "tools", "allreduce_test_perf.py"), "-b", "64M", "-e", "64M", "-k", "1",
           "-n", "2", "-G", "1"]
    r = subprocess.run(cmd, cwd=root, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "Out of bounds values : 0 OK" in r.stdout
