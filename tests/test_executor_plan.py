"""Execution plans on the CPU: the C++ lowering (mscclppAmdExecutionPlanDescribe) against the
oracle's independent restatement of execution_plan.cc, for every rank of every plan at several
message sizes; the oracle's simulated execution against exact integer sums (a known answer); and
the error paths (unsupported channels / operations, misaligned sizes, missing files)."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PLANS = os.path.join(ROOT, "tests", "golden", "plans")
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import executor_oracle as E  # noqa: E402

GENERATED = sorted(f for f in os.listdir(PLANS) if f.endswith(".json"))
REF_PLANS = "/root/reference/test/execution-files"
# The reference's own plan files (test/execution-files/allreduce*.json), committed as data fixtures
# (sha256 in tests/golden/plans/ref/SOURCE.txt) so that the GPU box, which has no /root/reference,
# can run them too.
REF_FIXTURES = os.path.join(PLANS, "ref")


def _nranks(doc):
    return len(doc["gpus"])


def _sizes(doc):
    g = doc["gpus"][0]
    c = max(g["input_chunks"], g["output_chunks"]) * doc.get("buffer_alignment", 16)
    return [c, c * 4, c * 1024, c * 1000 + c * 7]


def _check_plan(built, path):
    import mscclpp_amd as m

    with open(path) as f:
        doc = json.load(f)
    for rank in range(_nranks(doc)):
        plan = m.ExecutionPlan(path, rank)
        assert plan.name() == doc["name"] and plan.collective() == doc["collective"]
        assert plan.is_in_place() == doc["inplace"]
        for size in _sizes(doc):
            got = plan.describe(size, size)
            exp = E.RankPlan(doc, rank, size, size).describe()
            assert got == json.loads(json.dumps(exp)), (path, rank, size)


@pytest.mark.parametrize("fname", GENERATED)
def test_lowering_matches_oracle(built, fname):
    _check_plan(built, os.path.join(PLANS, fname))


@pytest.mark.parametrize("fname", ["allreduce_packet.json", "allreduce.json"])
def test_lowering_of_reference_plans(built, fname):
    """The reference's own plan files (the committed fixtures; where /root/reference exists, they
    must still be byte-identical to the files there)."""
    path = os.path.join(REF_FIXTURES, fname)
    if os.path.isdir(REF_PLANS):
        with open(path, "rb") as a, open(os.path.join(REF_PLANS, fname), "rb") as b:
            assert a.read() == b.read()
    _check_plan(built, path)


@pytest.mark.parametrize("fname", ["allreduce_packet.json", "allreduce.json"])
@pytest.mark.parametrize("dtype", ["i32", "u32"])
def test_oracle_known_answer_reference_plans(fname, dtype):
    test_oracle_known_answer(os.path.join("ref", fname), dtype)


@pytest.mark.parametrize("fname", GENERATED)
@pytest.mark.parametrize("dtype", ["i32", "u32"])
def test_oracle_known_answer(fname, dtype):
    """Integer sums are exact whatever the order: every rank must end with the plain sum."""
    with open(os.path.join(PLANS, fname)) as f:
        doc = json.load(f)
    n = _nranks(doc)
    eo = E.ExecutorOracle(doc, n)
    nbytes = _sizes(doc)[1] * 8
    rng = np.random.default_rng(5)
    npdt = np.int32 if dtype == "i32" else np.uint32
    for _ in range(3):
        ins = [rng.integers(0, 1 << 20, nbytes // 4).astype(npdt).view(np.uint8).copy() for _ in range(n)]
        exp = sum(a.view(npdt).astype(np.int64) for a in ins).astype(npdt)
        outs = ins if doc["inplace"] else [np.zeros_like(a) for a in ins]
        res = eo.execute(ins, outs, dtype)
        for r in range(n):
            got = res[r][0 if doc["inplace"] else 1].view(npdt)
            assert np.array_equal(got, exp)


def test_oracle_flag_and_double_scratch():
    """Consecutive calls alternate scratch halves (flag parity) and carry flag = call number."""
    with open(os.path.join(PLANS, "allreduce_pkt_n2.json")) as f:
        doc = json.load(f)
    eo = E.ExecutorOracle(doc, 2)
    ins = [np.arange(1024, dtype=np.int32).view(np.uint8).copy() for _ in range(2)]
    res1 = eo.execute([a.copy() for a in ins], [a.copy() for a in ins], "i32")
    half = res1[0][2].size // 2
    flags1 = res1[0][2][:half].view(np.uint32).reshape(-1, 4)[:, 1]
    assert set(np.unique(flags1)) <= {0, 1} and 1 in flags1
    res2 = eo.execute([a.copy() for a in ins], [a.copy() for a in ins], "i32")
    flags2 = res2[0][2][half:].view(np.uint32).reshape(-1, 4)[:, 1]
    assert 2 in flags2


def _write(tmp_path, doc, name="p.json"):
    p = tmp_path / name
    p.write_text(json.dumps(doc))
    return str(p)


def test_rejects_port_and_switch_channels(built, tmp_path):
    import mscclpp_amd as m

    with open(os.path.join(PLANS, "allreduce_rres_n2.json")) as f:
        doc = json.load(f)
    doc["gpus"][0]["channels"][0]["channel_type"] = "port"
    plan = m.ExecutionPlan(_write(tmp_path, doc), 0)
    with pytest.raises(m.MscclppError):
        plan.describe(4096, 4096)
    doc["gpus"][0]["channels"][0]["channel_type"] = "switch"
    plan = m.ExecutionPlan(_write(tmp_path, doc, "q.json"), 0)
    with pytest.raises(m.MscclppError):
        plan.describe(4096, 4096)


def test_rejects_multimem_ops(built, tmp_path):
    import mscclpp_amd as m

    with open(os.path.join(PLANS, "allreduce_rres_n2.json")) as f:
        doc = json.load(f)
    doc["gpus"][0]["threadblocks"][0]["ops"][3]["name"] = "glres"
    plan = m.ExecutionPlan(_write(tmp_path, doc), 0)
    with pytest.raises(m.MscclppError):
        plan.describe(4096, 4096)


def test_rejects_misaligned_and_out_of_range(built, tmp_path):
    import mscclpp_amd as m

    with open(os.path.join(PLANS, "allreduce_pkt_n2.json")) as f:
        doc = json.load(f)
    path = _write(tmp_path, doc)
    plan = m.ExecutionPlan(path, 0)
    with pytest.raises(m.MscclppError):
        plan.describe(1000, 1000)  # not a multiple of alignment * chunks
    doc["max_message_size"] = 4096
    plan = m.ExecutionPlan(_write(tmp_path, doc, "small.json"), 0)
    plan.describe(4096, 4096)
    with pytest.raises(m.MscclppError):
        plan.describe(8192, 8192)


def test_missing_or_malformed_file(built, tmp_path):
    import mscclpp_amd as m

    with pytest.raises(m.MscclppError):
        m.ExecutionPlan(str(tmp_path / "nope.json"), 0)
    bad = tmp_path / "bad.json"
    bad.write_text("{\"name\": \"x\", ")
    with pytest.raises(m.MscclppError):
        m.ExecutionPlan(str(bad), 0)


@pytest.mark.parametrize("fname", ["ref/allreduce_packet.json", "ref/allreduce.json", "allreduce_pkt_n4.json"])
@pytest.mark.parametrize("dtype,one", [("e4m3", 0x38), ("e5m2", 0x3C)])
def test_oracle_known_answer_fp8(fname, dtype, one):
    """OCP fp8 through a plan: inputs of small integers (exact in fp8, as are all their partial sums
    up to 8 ranks x 3), so every rank must end with the exact integer sum whatever the order."""
    import oracle_lib as O

    with open(os.path.join(PLANS, fname)) as f:
        doc = json.load(f)
    n = _nranks(doc)
    eo = E.ExecutorOracle(doc, n)
    nbytes = _sizes(doc)[1] * 8
    rng = np.random.default_rng(7)
    e5 = dtype == "e5m2"
    top = 2 if e5 else 4  # inputs in [0, top): every partial sum stays an integer fp8 holds exactly
    enc = {v: O.fp8_encode_sat(float(v), e5) for v in range(0, (top - 1) * n + 1)}
    assert enc[1] == one and all(O.fp8_decode(b, e5) == float(v) for v, b in enc.items())
    vals = rng.integers(0, top, size=(n, nbytes))
    ins = [np.array([enc[int(v)] for v in vals[r]], dtype=np.uint8) for r in range(n)]
    exp = np.array([enc[int(v)] for v in vals.sum(axis=0)], dtype=np.uint8)
    outs = ins if doc["inplace"] else [np.zeros_like(a) for a in ins]
    res = eo.execute([a.copy() for a in ins], [a.copy() for a in outs], dtype)
    for r in range(n):
        assert np.array_equal(res[r][0 if doc["inplace"] else 1], exp), r
