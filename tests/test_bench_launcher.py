"""bench.py's N-rank launcher and its input generator (CPU only; no GPU is touched).

`python bench.py --gpus N` without WORLD_SIZE must start N ranks with the torch.distributed.run
environment, and a --gpus that disagrees with WORLD_SIZE must fail.  The device
LCG of the N>1 benchmark must generate exactly the oracle's inputs (test/torch/correctness_test.py:
19-56), and the oracle's owner-sliced AllReduce must agree with its per-slice form."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _bench(args, env_extra=None, timeout=120):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 4])
def test_launcher_spawns_n_ranks(n):
    r = _bench(["--gpus", str(n), "--dry-run"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["master"] == "127.0.0.1" and int(d["port"]) > 0


def test_gpus_world_size_mismatch_fails():
    r = _bench(["--gpus", "8", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "disagrees" in r.stderr


def test_failing_rank_fails_the_launch():
    r = _bench(["--gpus", "2", "--dry-run"], {"BENCH_DRY_RUN_FAIL_RANK": "1"})
    assert r.returncode == 3


def test_device_lcg_matches_oracle():
    import bench
    import oracle_lib as O

    for rank, seq in ((0, 0), (3, 1), (7, 1)):
        t = bench.lcg_tensor(100003, rank, seq, torch.float16, "cpu")
        ref = O.lcg(O.F16, 100003, rank, seq)
        assert np.array_equal(t.view(torch.int16).numpy().view(np.uint16), ref)


def test_owned_allreduce_matches_sliced():
    import oracle_lib as O

    n, count = 8, (1 << 16) + 24
    ins = [O.lcg(O.F16, count, r, 1) for r in range(n)]
    nbytes = count * 2
    slice_w = ((nbytes + n - 1) // n + 15) // 16 * 4
    nw = (nbytes + 15) // 16 * 4
    for order in (0, 1):
        owned = O.allreduce_owned(O.F16, O.SUM, ins, nw, n * slice_w, slice_w, order)
        padded = []
        for a in ins:
            w = np.zeros(nw, np.uint32)
            w.view(np.uint8)[:nbytes] = a.view(np.uint8)
            padded.append(w)
        sliced = O.allreduce_sliced(O.F16, O.SUM, padded, nw, slice_w, order)[0]
        assert np.array_equal(owned, sliced)
    # interleaved ownership (rsag_pipeline): unit u owned by (u mod n*C) // C, ring order from the owner
    C = 64
    owned = O.allreduce_owned(O.F16, O.SUM, ins, nw, n * 4 * C, 4 * C, 1)
    padded = [np.pad(a.view(np.uint32), (0, nw - a.size // 2)) for a in ins]
    owner = ((np.arange(nw) // 4) % (n * C)) // C
    for o in range(n):
        seq = O.reduce_seq(O.F16, O.SUM, [padded[(o + k) % n] for k in range(n)])
        assert np.array_equal(owned[owner == o], seq[owner == o])


@pytest.mark.parametrize("n", [2, 4, 8])
def test_checker_expectations_per_algorithm(built, n):
    """bench.py's BitExactChecker against direct oracle calls (host logic only): the one-hop LL8
    result is per rank (own first), the two-hop LL16 result is the owners' everywhere, the bulk
    orders are own-then-ascending (fullmesh) and ring (rsag / zero-copy), and the pipeline's
    ownership interleaves slots of 4*C words (C = nblocks * nthreads * 4 units of 16 B)."""
    import bench
    import mscclpp_amd as m
    import oracle_lib as O

    S = 64 << 10
    chk = bench.BitExactChecker(n, S, m.F16)
    ins = [O.lcg(m.F16, S // 2, r, 1) for r in range(n)]
    half = m.scratch_required(m.ALGO_ALLPAIR, n, 16 << 10, m.F16) // 2
    ins16 = [O.lcg(m.F16, (16 << 10) // 2, r, 1) for r in range(n)]
    outs, _ = O.allreduce_allpairs(m.F16, O.SUM, ins16, (16 << 10) // 2, 1, half)
    for r in range(n):
        assert np.array_equal(chk.expected("allpair", 0, 0, 1, 16 << 10, r), outs[r][: (16 << 10) // 4])
    half = m.scratch_required(m.ALGO_PACKET, n, S, m.F16) // 2
    outs, _ = O.allreduce_packet(m.F16, O.SUM, ins, S // 2, 1, half)
    for r in range(n):
        assert np.array_equal(chk.expected("packet", 0, 0, 1, S, r), outs[r][: S // 4])
    nw = S // 4
    sw = ((S + n - 1) // n + 15) // 16 * 4
    words = [a.view(np.uint32) for a in ins]
    for algo, order in (("fullmesh", 0), ("rsag", 1), ("rsag_zc", 1)):
        exp = O.allreduce_sliced(m.F16, O.SUM, words, nw, sw, order)[0]
        assert np.array_equal(chk.expected(algo, 64, 512, 1, S, 0), exp[:nw]), algo
    nb, nt = 2, 64
    C = nb * nt * 4
    owner = ((np.arange(nw) // 4) % (n * C)) // C
    exp = np.zeros(nw, np.uint32)
    for o in range(n):
        seq = O.reduce_seq(m.F16, O.SUM, [words[(o + k) % n] for k in range(n)])
        exp[owner == o] = seq[owner == o]
    assert np.array_equal(chk.expected("rsag_pipeline", nb, nt, 1, S, 0), exp)


def _probe(put, getput):
    return {"allpairs_put_out_GBs": put, "allpairs_getput_GBs": getput}


@pytest.mark.parametrize("n", [2, 4, 8])
def test_multi_line_roofline_grades_the_spec_xgmi_ceiling(n):
    """the N>1 line's roofline peak is the all-pairs algbw ceiling of BASELINE.md §2,
    n * 153.6 / 2 GB/s (614.4 at n = 8), whatever the probe measured, and frac = the kernel's algbw /
    that peak (= wire bytes per rank / ((n-1) * 153.6)).  The probe of the kernel's own pattern moves
    to measured_ceiling / frac_of_measured; a frac_of_measured above 1 is flagged, with no slack."""
    import bench

    S, kern_ms = 48 << 20, 0.2
    algbw = S / (kern_ms * 1e-3) / 1e9
    wire_gbs = 2 * (n - 1) * S / n / (kern_ms * 1e-3) / 1e9
    peak = n * 153.6 / 2
    for algo, key in (("rsag_zc", "allpairs_getput_GBs"), ("fullmesh", "allpairs_put_out_GBs")):
        probe = _probe(2 * wire_gbs, 3 * wire_gbs)
        roof, xg = bench.multi_roofline(n, S, algo, kern_ms * 1.05e-3, kern_ms, probe, False)
        for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
            assert k in roof
        assert roof["peak"] == pytest.approx(peak, abs=0.05)
        assert roof["achieved"] == pytest.approx(algbw, rel=1e-3)
        assert roof["frac"] == pytest.approx(algbw / peak, rel=1e-3)
        assert roof["frac"] == pytest.approx(wire_gbs / ((n - 1) * 153.6), rel=1e-3)
        mc = probe[key] * n / (2 * (n - 1))
        assert roof["measured_ceiling"] == pytest.approx(mc, rel=1e-3)
        assert roof["frac_of_measured"] == pytest.approx(algbw / mc, rel=1e-3)
        assert xg["probe_consistent"] is True
        # a probe slower than the kernel itself: inconsistent, and the peak does not move
        roof, xg = bench.multi_roofline(n, S, algo, kern_ms * 1.05e-3, kern_ms, _probe(0.99 * wire_gbs, 0.99 * wire_gbs),
                                        False)
        assert roof["frac_of_measured"] > 1 and xg["probe_consistent"] is False
        assert roof["peak"] == pytest.approx(peak, abs=0.05)
    roof, xg = bench.multi_roofline(n, S, "fullmesh", 1e-4, 0.1, {"error": "no probe"}, True)
    assert xg["probe_consistent"] is False and "measured_ceiling" not in roof
    assert roof["frac"] == pytest.approx(S / 1e-4 / 1e9 / peak, rel=1e-3)
    assert bench.multi_roofline(8, S, "fullmesh", 1e-3, 1.0, {}, False)[0]["peak"] == pytest.approx(614.4)


class _FakeLib:
    """mscclppAmdSelectAlgo of the built-in table (host/tuning.cpp) for the winner_profile test."""

    def mscclppAmdSelectAlgo(self, n, size, dt):
        return 2 if size <= 16 << 10 or (n == 2 and size <= 1 << 20) else 1 if size <= 1 << 20 else 3


class _FakeM:
    def lib(self):
        return _FakeLib()

    def tuned_config(self, coll, n, size):
        return None

    def tuned_config_source(self, coll, n, size):
        return "reference"


@pytest.mark.parametrize("n", [2, 8])
def test_winner_profile_keeps_the_ll_range(n):
    """The profile bench.py loads before timing ncclAllReduce names the winner from the bucket size
    up and keeps the selector's choices below it, so only the headline size changes algorithm."""
    import bench

    S = 48 << 20
    prof = bench.winner_profile(_FakeM(), n, S, "AMD Instinct MI355X", "rsag_zc", 128, 512)
    (p,) = prof["profiles"]
    assert p["scale"] == n and prof["version"] == 1
    es = p["collectives"]["allreduce"]
    assert {k: v for k, v in es[-1].items() if k != "source"} == \
        {"message_size": S, "algorithm": "default_allreduce_rsag_zero_copy", "nblocks": 128, "nthreads": 512}
    assert es[-1]["source"].startswith("tuned") and es[0]["source"] == "reference"
    want = ["default_allreduce_allpair_packet"] + ([] if n == 2 else ["default_allreduce_packet"]) + \
        ["default_allreduce_fullmesh", "default_allreduce_rsag_zero_copy"]
    assert [e["algorithm"] for e in es] == want
    assert es[0]["message_size"] == 1


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "mscclpp_amd", "lib", "libmscclpp_amd.so")),
                    reason="library not built")
def test_loaded_winner_drives_the_library_selector(tmp_path):
    """Host only (no GPU call): after mscclppAmdTunedConfigLoad of winner_profile, the library's own
    selector -- what ncclAllReduce consults -- returns the winner and its launch shape at the bucket,
    and the built-in choices below it."""
    import bench
    import mscclpp_amd as m

    n, S = 8, 48 << 20
    before = {sz: m.lib().mscclppAmdSelectAlgo(n, sz, 0) for sz in (1024, 64 << 10, 4 << 20)}
    try:
        # no SKU: this container has no GPU to name one (bench.py passes the device's name)
        loaded = bench.load_winner(m, n, S, None, "rsag_zc", 128, 512)
        assert loaded[-1]["algorithm"] == "default_allreduce_rsag_zero_copy"
        assert m.tuned_config("allreduce", n, S) == ("default_allreduce_rsag_zero_copy", 128, 512)
        assert bench.SELECT_NAMES[m.lib().mscclppAmdSelectAlgo(n, S, 0)] == "rsag_zc"
        for sz, a in before.items():
            assert m.lib().mscclppAmdSelectAlgo(n, sz, 0) == a, sz
    finally:
        empty = tmp_path / "empty.json"
        empty.write_text('{"version": 1, "profiles": []}')
        m.load_tuned_config(str(empty))


def test_cpu_baselines_state_their_cores():
    """cpu_baseline objects (N=1 and N>1): value / unit / cores / kind / sample, cores = threads used."""
    import bench

    for d in (bench.cpu_baseline_sum(4, 1 << 20, 0.05, threads=3), bench.cpu_baseline_self_reduce(1 << 20, 0.05, 2)):
        assert set(d) >= {"value", "unit", "cores", "kind", "sample"} and d["value"] > 0
    assert bench.cpu_baseline_sum(8, 1 << 20, 0.05, threads=3)["cores"] == 3
    assert "8-way sum" in bench.cpu_baseline_sum(8, 1 << 20, 0.05, threads=2)["sample"]


def test_cpu_threaded_sum_matches_the_oracle():
    """The threaded sum computes exactly what the oracle's one-call form does."""
    import bench
    import oracle_lib as O

    nbytes, n = 1 << 20, 3
    ins = [O.lcg(O.F16, nbytes // 2, r, 0).view(np.uint32) for r in range(n)]
    want = O.reduce_seq(O.F16, O.SUM, ins)
    got = bench._threaded_sum_for_test(n, nbytes, threads=5)
    assert np.array_equal(got, want)


def _ring_output(bench, n, count, seq, order):
    """An AllReduce output of ring_tensor inputs summed in `order` per owner slice (CPU)."""
    out = torch.empty(count)
    se = bench.ring_slice_elems(n, count)
    for o in range(n):
        lo, hi = o * se, min(count, (o + 1) * se)
        if lo >= hi:
            continue
        ranks = [(o + k) % n for k in range(n)] if order == "ring" else list(range(n))
        acc = bench.ring_tensor(lo, hi - lo, ranks[0], seq, "cpu")
        for r in ranks[1:]:
            acc += bench.ring_tensor(lo, hi - lo, r, seq, "cpu")
        out[lo:hi] = acc
    return out


@pytest.mark.parametrize("n", [2, 4, 8])
def test_fp32_ring_check_tells_the_order_apart(n, monkeypatch):
    """the config-5 check (fp32 1 GiB rsag / rsag_zc) must catch a wrong sum order.
    Its inputs (ring_bits: random sign, 8 exponents, full mantissa) make the ring-order sum differ from
    the ascending-order sum on a large share of elements, the device-side check counts 0 mismatches
    only for the ring order, and the CPU-oracle sample agrees.  A small chunk exercises the chunking."""
    import bench

    monkeypatch.setattr(bench, "RING_CHUNK", 1000)
    count = n * 4096 + 36  # ragged last slice
    i = np.arange(5000, dtype=np.int64)
    assert np.array_equal(bench.ring_bits(i, 3, 1), bench.ring_bits(torch.from_numpy(i), 3, 1).numpy())
    good = _ring_output(bench, n, count, 1, "ring")
    wrong = _ring_output(bench, n, count, 1, "ascending")
    assert bench.ring_order_mismatches(good, n, 1) == 0
    bad = bench.ring_order_mismatches(wrong, n, 1)
    assert bench.ring_order_mismatches(good, n, 0) > count // 2  # another seq's inputs
    assert bench.ring_oracle_sample(good, n, 1, samples=3000)
    if n == 2:  # a + b == b + a in IEEE arithmetic: two ranks have one sum whatever the order
        assert bad == 0
        return
    assert bad > count // 8, bad  # slice 0's orders coincide; the others differ widely
    assert not bench.ring_oracle_sample(wrong, n, 1, samples=3000)


def test_extras_check_every_timed_size():
    """the N>1 extras check every LL sweep size (eager and graph-captured), LL16 at
    48 MiB and both fp32 1 GiB ring kernels before timing them, and all of it folds into `correct`."""
    import bench

    keys = set(bench.EXTRAS_CHECK_KEYS)
    for kb in bench.LL_SWEEP_KIB:
        assert f"ll_sweep:{kb}KiB" in keys and f"ll_graph:{kb}KiB" in keys
    assert {"ll16_48MiB", "fp32_1GiB_rsag", "fp32_1GiB_rsag_zc"} <= keys
    assert bench.LL_SWEEP_KIB[0] == 1 and bench.LL_SWEEP_KIB[-1] == 1024
    ok = {"correct_bitexact": {k: True for k in keys}, "device_error": 0}
    assert bench.extras_correct(ok, True)
    assert bench.extras_correct({"device_error": 0}, False)
    for k in ("ll_graph:64KiB", "fp32_1GiB_rsag_zc", "ll16_48MiB"):
        missing = {"correct_bitexact": {q: True for q in keys if q != k}, "device_error": 0}
        assert not bench.extras_correct(missing, True), k
        wrong = {"correct_bitexact": dict(ok["correct_bitexact"], **{k: False}), "device_error": 0}
        assert not bench.extras_correct(wrong, True), k
    assert not bench.extras_correct(dict(ok, fp32_1GiB_error="boom"), True)
    assert not bench.extras_correct(dict(ok, device_error=3), True)
    extra_false = {"correct_bitexact": dict(ok["correct_bitexact"], **{"crossover:4KiB:packet:0x0": False})}
    assert not bench.extras_correct(extra_false, True)
    assert bench.ll16_ceiling(8) == pytest.approx(307.2)


def test_pingpong_extras_labels():
    """The N=1 line's ping-pong extras: the two host-proxy ranks' LL16 / LL8
    latencies, labelled a shared-device figure on a 1-GPU box and one xGMI hop on a node; a failed
    host-proxy run leaves them null with the reason, never an exception."""
    import bench

    pp = {"ll16": {"us_per_iter": 2.6, "correct": True}, "ll8": {"us_per_iter": 2.4, "correct": True}}
    one = bench.pingpong_extras({"pingpong": pp, "pingpong_correct": True, "devices": [0]})
    assert one["ll16_pingpong_us"] == 2.6 and one["ll8_pingpong_us"] == 2.4 and one["pingpong_correct"] is True
    assert "shared-device" in one["pingpong_note"]
    two = bench.pingpong_extras({"pingpong": pp, "pingpong_correct": True, "devices": [0, 1]})
    assert "xGMI hop" in two["pingpong_note"] and two["pingpong_devices"] == [0, 1]
    bad = bench.pingpong_extras({"error": "boom"})
    assert bad["ll16_pingpong_us"] is None and "boom" in bad["pingpong_note"]
    assert bench.pingpong_extras(None)["ll8_pingpong_us"] is None
