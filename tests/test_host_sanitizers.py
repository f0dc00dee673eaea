"""Host sanitizers (SURVEY.md §5 "Race detection / sanitizers": the reference runs none; the build
equivalent is ASan/TSan on the host code).  CPU only:

* the TCP bootstrap (mscclpp_amd/csrc/host/bootstrap.cpp: a root thread relaying all-gather /
  barrier / broadcast rounds and point-to-point messages into per-rank mailboxes) under
  ThreadSanitizer and under AddressSanitizer + UBSan, 8 ranks as threads of one process
  (tests/sanitize/bootstrap_stress.cpp);
* the CPU oracle (oracle/ll_oracle.c) built with AddressSanitizer + UBSan and driven through its
  golden-vector and fp8 known-answer tests.

GPU code is never sanitized here (the pool refuses GPU ASan); these builds contain no device code."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "build", "san")
HOST = os.path.join(ROOT, "mscclpp_amd", "csrc", "host")


def _runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


def _build_stress(flags, exe):
    os.makedirs(OUT, exist_ok=True)
    out = os.path.join(OUT, exe)
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, "-I" + HOST,
           os.path.join(HOST, "bootstrap.cpp"), os.path.join(ROOT, "tests", "sanitize", "bootstrap_stress.cpp"),
           "-o", out, "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    return out


@pytest.mark.skipif(_runtime("libtsan.so") is None, reason="no ThreadSanitizer runtime")
def test_bootstrap_under_thread_sanitizer():
    exe = _build_stress(["-fsanitize=thread"], "bootstrap_tsan")
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:exitcode=66")
    r = subprocess.run([exe, "8", "30"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "bootstrap stress OK" in r.stdout, r.stderr[-4000:]


@pytest.mark.skipif(_runtime("libasan.so") is None, reason="no AddressSanitizer runtime")
def test_bootstrap_under_address_and_ub_sanitizers():
    exe = _build_stress(["-fsanitize=address,undefined"], "bootstrap_asan")
    env = dict(os.environ, UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([exe, "8", "30"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "bootstrap stress OK" in r.stdout, r.stderr[-4000:]


@pytest.mark.skipif(_runtime("libasan.so") is None, reason="no AddressSanitizer runtime")
def test_oracle_under_address_and_ub_sanitizers():
    os.makedirs(OUT, exist_ok=True)
    so = os.path.join(OUT, "liboracle_asan.so")
    r = subprocess.run(["gcc", "-O1", "-g", "-std=c11", "-fPIC", "-shared", "-fsanitize=address,undefined",
                        "-fno-omit-frame-pointer", "-o", so, os.path.join(ROOT, "oracle", "ll_oracle.c"), "-lm"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, LD_PRELOAD=_runtime("libasan.so"), ASAN_OPTIONS="detect_leaks=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", MSCCLPP_AMD_ORACLE_SO=so)
    # the sanitized build is the one loaded
    probe = subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, 'tests'); import oracle_lib as O; "
                            "O.lcg(O.F16, 8, 0, 0); print(O._lib()._name if hasattr(O, '_lib') else O.ORACLE_SO)"],
                           cwd=ROOT, capture_output=True, text=True, env=env, timeout=120)
    assert probe.returncode == 0 and "liboracle_asan.so" in probe.stdout, probe.stderr[-2000:]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", "tests/test_oracle_golden.py",
                        "tests/test_fp8_oracle.py"], cwd=ROOT, capture_output=True, text=True, env=env, timeout=900)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
