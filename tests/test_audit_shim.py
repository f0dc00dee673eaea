"""LD_AUDIT redirect (reference: src/ext/nccl/audit-shim/audit_nccl.cc:9-17): a program that
dlopen()s librccl.so.1 / libnccl.so.2 resolves the NCCL symbols from libmscclpp_amd.so.  CPU only:
ncclGetVersion touches no device."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AUDIT = os.path.join(ROOT, "mscclpp_amd", "lib", "libmscclpp_amd_audit.so")
LIB = os.path.join(ROOT, "mscclpp_amd", "lib", "libmscclpp_amd.so")

PROBE = r"""
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdio.h>
int main(int argc, char** argv) {
  void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) { printf("ERR %s\n", dlerror()); return 2; }
  int (*gv)(int*) = (int (*)(int*))dlsym(h, "ncclGetVersion");
  if (!gv) { printf("ERR nosym\n"); return 3; }
  Dl_info info;
  dladdr((void*)gv, &info);
  int v = 0;
  int rc = gv(&v);
  printf("%s %d %d\n", info.dli_fname, rc, v);
  return 0;
}
"""


@pytest.fixture(scope="module")
def probe(tmp_path_factory, built):
    d = tmp_path_factory.mktemp("audit")
    src = d / "probe.c"
    src.write_text(PROBE)
    exe = d / "probe"
    subprocess.run(["gcc", "-o", str(exe), str(src), "-ldl"], check=True)
    assert os.path.exists(AUDIT), "audit library not built"
    return str(exe)


def _run(exe, name, **extra):
    env = dict(os.environ, LD_AUDIT=AUDIT, **extra)
    r = subprocess.run([exe, name], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=120)
    return r.returncode, r.stdout.strip().splitlines()[-1] if r.stdout.strip() else ""


@pytest.mark.parametrize("name", ["librccl.so.1", "librccl.so", "libnccl.so.2", "libnccl.so"])
def test_redirects_nccl_names(probe, name):
    rc, line = _run(probe, name)
    assert rc == 0, line
    path, res, ver = line.split()
    assert os.path.realpath(path) == os.path.realpath(LIB)
    assert int(res) == 0 and int(ver) > 0


def test_env_override_target(probe):
    rc, line = _run(probe, "librccl.so.1", MSCCLPP_AMD_NCCL_LIB=LIB)
    assert rc == 0, line
    assert os.path.realpath(line.split()[0]) == os.path.realpath(LIB)


def test_other_names_untouched(probe):
    # a library that is not NCCL is searched for normally (here: it does not exist at all)
    rc, line = _run(probe, "libnot_nccl_at_all.so")
    assert rc == 2 and line.startswith("ERR")
