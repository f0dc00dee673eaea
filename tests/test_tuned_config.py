"""The data-driven selector: the tuned-config store in the JSON format of the
reference's tuner (python/mscclpp_benchmark/tuning_config.py:37-200) -- profile matching by SKU and
scale, the bisect_left rule within a collective -- with the built-in table restating
algorithm_selector.cc:107-131 (AMD branch).  CPU only (no GPU: the SKU is unknown here, so only
profiles without a sku match)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import json, sys
sys.path.insert(0, {root!r})
import mscclpp_amd as m
out = {{}}
for n, size in ((8, 1024), (8, 16384), (8, 16385), (8, 1 << 20), (8, (1 << 20) + 1), (8, 48 << 20), (4, 48 << 20),
                (2, 4096), (2, 262144), (2, 262145), (2, 1 << 20), (2, 48 << 20), (4, 65536)):
    out[f"ar/{{n}}/{{size}}"] = m.tuned_config("allreduce", n, size)
    out[f"sel/{{n}}/{{size}}"] = m.lib().mscclppAmdSelectAlgo(n, size, 0)
    out[f"src/{{n}}/{{size}}"] = m.tuned_config_source("allreduce", n, size)
out["ag"] = m.tuned_config("allgather", 8, 1 << 20)
out["bcast"] = m.tuned_config("broadcast", 8, 1 << 20)
print(json.dumps(out))
"""


def _query(env_extra=None):
    env = dict(os.environ)
    env.pop("MSCCLPP_AMD_TUNED_CONFIG", None)
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, "-c", SCRIPT.format(root=ROOT)], capture_output=True, text=True, env=env,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_builtin_table_restates_the_amd_thresholds(built):
    q = _query()
    assert q["ar/8/1024"][0] == "default_allreduce_allpair_packet"
    assert q["ar/8/16384"][0] == "default_allreduce_allpair_packet"
    assert q["ar/8/16385"][0] == "default_allreduce_packet"
    assert q["ar/8/1048576"][0] == "default_allreduce_packet"
    assert q["ar/8/1048577"][0] == "default_allreduce_fullmesh"
    assert q["ar/8/50331648"] == ["default_allreduce_fullmesh", 0, 0]
    assert q["sel/8/1024"] == 2 and q["sel/8/16385"] == 1 and q["sel/8/50331648"] == 3
    assert q["ag"][0] == "default_allgather_fullmesh2"
    assert q["bcast"] is None
    # 2 ranks: one-hop LL8 over the whole LL range (the same bytes on the one link as LL16, one hop fewer)
    assert q["ar/2/262144"][0] == "default_allreduce_allpair_packet" and q["sel/2/262144"] == 2
    assert q["ar/2/262145"][0] == "default_allreduce_allpair_packet"
    assert q["ar/2/1048576"][0] == "default_allreduce_allpair_packet"
    assert q["ar/2/50331648"][0] == "default_allreduce_fullmesh"
    assert q["ar/4/65536"][0] == "default_allreduce_packet"  # other scales: the reference's thresholds
    # the defaults that came from fabric-free sweeps say so
    assert q["src/2/262144"] == "fabric-free" and q["src/2/1048576"] == "fabric-free"
    assert q["src/2/50331648"] == "reference"
    assert q["src/8/1024"] == "reference" and q["src/8/50331648"] == "reference"
    assert q["src/8/16385"] == "reference; grid fabric-free" and q["src/4/65536"] == "reference; grid fabric-free"


def test_user_profile_overrides_by_scale(built, tmp_path):
    cfg = {"version": 1, "profiles": [
        {"scale": 8, "collectives": {"allreduce": [
            {"message_size": 65536, "algorithm": "default_allreduce_packet", "nblocks": 56, "nthreads": 512},
            {"message_size": 1048577, "algorithm": "default_allreduce_rsag_zero_copy", "nblocks": 128,
             "nthreads": 512, "time_us": 150.0}]}},
        {"sku": "SOME_OTHER_GPU", "scale": 8, "collectives": {"allreduce": [
            {"message_size": 1, "algorithm": "default_allreduce_rsag"}]}}]}
    path = tmp_path / "tuned.json"
    path.write_text(json.dumps(cfg))
    q = _query({"MSCCLPP_AMD_TUNED_CONFIG": str(path)})
    # scale 8: the user profile (a smaller message than the first entry takes the first entry)
    assert q["ar/8/1024"] == ["default_allreduce_packet", 56, 512]
    assert q["ar/8/1048576"] == ["default_allreduce_packet", 56, 512]
    assert q["ar/8/50331648"] == ["default_allreduce_rsag_zero_copy", 128, 512]
    assert q["sel/8/50331648"] == 5
    assert q["src/8/50331648"] == "tuned" and q["src/2/4096"] == "fabric-free"  # a node table overrides
    # other scales: the built-in table
    assert q["ar/4/50331648"][0] == "default_allreduce_fullmesh" and q["sel/4/50331648"] == 3
    assert q["ar/2/4096"][0] == "default_allreduce_allpair_packet"
    # collectives the user profile does not name fall through to the built-in table
    assert q["ag"][0] == "default_allgather_fullmesh2"


def test_malformed_file_is_rejected(built, tmp_path):
    import mscclpp_amd as m

    bad = tmp_path / "bad.json"
    bad.write_text('{"profiles": [{"collectives": {"allreduce": [{"message_size": 0, "algorithm": "x"}]}}]}')
    assert m.lib().mscclppAmdTunedConfigLoad(os.fsencode(str(bad))) == 4
    assert m.lib().mscclppAmdTunedConfigLoad(os.fsencode(str(tmp_path / "missing.json"))) == 4


def test_bench_node_table_loads_and_selects(built, tmp_path):
    """bench.py --gpus N turns its crossover / bulk sweeps into one profile (tuned_config_table); the
    library must accept it and pick each measured winner from its size up to the next one."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    extras = {"selector_crossover": {"4KiB": {"best": "allpair:0x0"}, "16KiB": {"best": "allpair:0x0"},
                                     "32KiB": {"best": "packet:0x0"}, "1024KiB": {"best": "packet:0x0"},
                                     "2048KiB": {"best": "rsag_zc:64x512"}},
              "bulk_size_sweep": {"2MiB": {"best": "fullmesh:64x512"}, "64MiB": {"best": "rsag_zc:128x512"}}}
    table = b.node_tuned_table(8, None, extras, (48 << 20, "rsag_zc", 128, 512))
    entries = table["profiles"][0]["collectives"]["allreduce"]
    assert [e["message_size"] for e in entries] == [1, 32 << 10, 2 << 20, 48 << 20]  # runs collapsed
    assert entries[2]["algorithm"] == "default_allreduce_fullmesh"  # the bulk sweep's row wins a tie of sizes
    del table["profiles"][0]["sku"]  # no GPU here: only a profile without a sku can match
    path = tmp_path / "node.json"
    path.write_text(json.dumps(table))
    q = _query({"MSCCLPP_AMD_TUNED_CONFIG": str(path)})
    assert q["ar/8/1024"] == ["default_allreduce_allpair_packet", 0, 0]
    assert q["ar/8/16385"] == ["default_allreduce_allpair_packet", 0, 0]
    assert q["ar/8/1048576"] == ["default_allreduce_packet", 0, 0]
    assert q["ar/8/1048577"] == ["default_allreduce_packet", 0, 0]
    assert q["ar/8/50331648"] == ["default_allreduce_rsag_zero_copy", 128, 512]
    assert q["ar/4/50331648"][0] == "default_allreduce_fullmesh"  # other scales keep the built-in table
    assert q["src/8/50331648"].startswith("node (") and q["src/4/50331648"] == "reference"
