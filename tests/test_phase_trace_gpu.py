"""Phase trace of the collective kernels (SURVEY.md §5 "Tracing / profiling": the reference's NPKit
events, allreduce_packet.cu:20-49, npkit.hpp:16; here s_memrealtime stamps at phase boundaries,
mscclppAmdTraceSet): while a trace buffer is set, every workgroup of every rank view stamps each
phase boundary in order; the results stay bit-exact; with the buffer unset nothing is written."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("algo_name,count", [("fullmesh", 1 << 20), ("rsag", 300000), ("rsag_zc", 1 << 20),
                                             ("packet", 1 << 17), ("allpair", 4096)])
def test_phase_stamps_in_order_and_results_unchanged(built, algo_name, count):
    import mscclpp_amd as m

    torch.cuda.set_device(0)
    n = 4
    algo = m.ALGO_NAMES[algo_name]
    nbytes = count * 2
    sb = max(m.scratch_required(m.ALGO_PACKET, n, nbytes, m.F16), m.scratch_required(m.ALGO_ALLPAIR, n, nbytes, m.F16))
    ranks = m.InProcessRanks(n, sb, bulk_scratch_bytes=nbytes + (1 << 20))
    ins = [torch.randn(count, device="cuda").half() for _ in range(n)]
    ref = [torch.empty_like(a) for a in ins]
    ranks.all_reduce(ins, ref, algo)  # untraced
    torch.cuda.synchronize()
    outs = [torch.empty_like(a) for a in ins]
    with m.PhaseTrace() as tr:
        ranks.all_reduce(ins, outs, algo)
    assert ranks.errors() == [0] * n
    for r in range(n):  # the stamps change no result bit
        assert torch.equal(outs[r].view(torch.int16), ref[r].view(torch.int16))
    nev = len(m.TRACE_PHASES[algo_name]) + 1
    for r in range(n):
        st = tr.stamps(r)
        used = st[st[:, 0] != 0]
        assert used.shape[0] > 0
        assert np.all(used[:, :nev] > 0)  # every workgroup stamped every boundary
        assert np.all(np.diff(used[:, :nev].astype(np.int64), axis=1) >= 0)  # in order
        assert np.all(used[:, nev:] == 0)
        ph = tr.phases(algo_name, r)
        assert set(m.TRACE_PHASES[algo_name]) <= set(ph) and 0 < ph["kernel_span_us"] < 1e6
    # trace off: a further launch writes nothing into the (re-zeroed) buffer
    tr.buf.zero_()
    ranks.all_reduce(ins, outs, algo)
    torch.cuda.synchronize()
    assert int(tr.buf.abs().sum().item()) == 0


def test_trace_buffer_too_small_is_rejected(built):
    import mscclpp_amd as m

    buf = torch.zeros(16, dtype=torch.int64, device="cuda")
    assert m.lib().mscclppAmdTraceSet(buf.data_ptr(), 128) == 4
    assert m.lib().mscclppAmdTraceSet(None, 0) == 0
