"""Host side of the phase trace (mscclpp_amd.PhaseTrace.phases, CPU only): stamps laid out as the
kernels write them (buf[(view * 256 + workgroup) * 8 + event], 10 ns ticks) turn into per-phase
mean / max durations over the workgroups that stamped, and the buffer size matches the C ABI's
MSCCLPP_AMD_TRACE_BYTES."""
import re
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_phases_from_synthetic_stamps():
    import mscclpp_amd as m

    tr = m.PhaseTrace.__new__(m.PhaseTrace)  # no device buffer: fill the layout by hand
    tr.buf = torch.zeros(m.TRACE_BYTES // 8, dtype=torch.int64)
    st = tr.buf.view(m.MAX_RANKS, m.TRACE_BLOCKS, m.TRACE_EVENTS)
    # view 1, two workgroups of a zero-copy call: entry 1 us / 3 us, reduce_ag 10 / 20 us, exit 2 / 0 us
    st[1, 0, :4] = torch.tensor([1000, 1100, 2100, 2300])
    st[1, 5, :4] = torch.tensor([1050, 1350, 3350, 3350])
    ph = tr.phases("rsag_zc", view=1)
    assert ph["workgroups"] == 2
    assert ph["entry_handshake"] == {"mean_us": 2.0, "max_us": 3.0}
    assert ph["reduce_ag"] == {"mean_us": 15.0, "max_us": 20.0}
    assert ph["exit_handshake"] == {"mean_us": 1.0, "max_us": 2.0}
    assert ph["kernel_span_us"] == 23.5
    assert tr.phases("rsag_zc", view=0) == {}  # nothing stamped there


def test_trace_size_matches_the_c_abi():
    import mscclpp_amd as m

    h = open(os.path.join(ROOT, "include", "mscclpp_amd", "mscclpp_amd.h")).read()
    expr = re.search(r"#define MSCCLPP_AMD_TRACE_BYTES \(\(size_t\)MSCCLPP_AMD_MAX_RANKS \* (\d+) \* (\d+) \* (\d+)\)", h)
    assert expr, "MSCCLPP_AMD_TRACE_BYTES definition changed"
    blocks, events, word = (int(v) for v in expr.groups())
    assert (blocks, events, word) == (m.TRACE_BLOCKS, m.TRACE_EVENTS, 8)
    assert m.TRACE_BYTES == m.MAX_RANKS * blocks * events * word
