"""Build libmscclpp_amd.so (HIP kernels for gfx950 + C++ host runtime) and the CPU oracle.

Everything is built in-tree so the shared objects travel to the GPU box with the repo snapshot:
    mscclpp_amd/lib/libmscclpp_amd.so   product library (C ABI: include/mscclpp_amd/*.h)
    mscclpp_amd/lib/libmscclpp_amd_audit.so  LD_AUDIT redirect of librccl/libnccl to the above
    oracle/liboracle.so                 CPU restatement used only by tests / smoke / bench baseline
    oracle/proxy_baseline               host-proxy CPU path (config 1 baseline), see oracle/
No cmake/ninja: plain hipcc / gcc invocations, parallel, incremental by mtime.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mscclpp_amd")
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
OBJDIR = os.path.join(ROOT, "build", "obj")
INCLUDE = os.path.join(ROOT, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
LIB = os.path.join(LIBDIR, "libmscclpp_amd.so")
ORACLE_LIB = os.path.join(ROOT, "oracle", "liboracle.so")
AUDIT_LIB = os.path.join(LIBDIR, "libmscclpp_amd_audit.so")


def _headers():
    return glob.glob(os.path.join(INCLUDE, "**", "*.h*"), recursive=True) + glob.glob(
        os.path.join(CSRC, "**", "*.h*"), recursive=True
    )


# MSCCLPP_AMD_FORCE_REBUILD=1: rebuild every artefact from its sources, whatever the timestamps
FORCE = os.environ.get("MSCCLPP_AMD_FORCE_REBUILD") == "1"
BUILT = []  # what this process compiled or linked (build_all's summary)


def _newer(target, deps):
    if FORCE or not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed: " + " ".join(cmd) + "\n" + r.stdout)
    out = cmd[cmd.index("-o") + 1] if "-o" in cmd else cmd[-1]
    BUILT.append(os.path.relpath(out, ROOT))
    return r.stdout


def _compile(src, hdrs):
    rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
    obj = os.path.join(OBJDIR, rel + ".o")
    if _newer(obj, [src] + hdrs):
        common = ["-O3", "-std=c++17", "-fPIC", "-I" + INCLUDE, "-I" + os.path.join(CSRC, "kernels"), "-Wall",
                  "-Wno-unused-function", "-Wno-unused-variable"]
        if src.endswith(".hip"):
            cmd = [HIPCC, "--offload-arch=" + ARCH, "-x", "hip"] + common + ["-c", src, "-o", obj]
        else:
            cmd = [HIPCC, "-D__HIP_PLATFORM_AMD__"] + common + ["-c", src, "-o", obj]
        _run(cmd)
    return obj


def build_library(verbose=False):
    os.makedirs(OBJDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    hdrs = _headers()
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")) + glob.glob(os.path.join(CSRC, "host", "*.cpp")))
    if not _newer(LIB, srcs + hdrs):
        return LIB  # up to date (also on the GPU box, where build/ does not travel)
    jobs = int(os.environ.get("MAX_JOBS", min(8, os.cpu_count() or 4)))
    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, 16))) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdrs), srcs))
    if _newer(LIB, objs):
        _run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB] + objs + ["-lpthread"])
        if verbose:
            print("linked", LIB)
    return LIB


def build_oracle():
    src = os.path.join(ROOT, "oracle", "ll_oracle.c")
    if _newer(ORACLE_LIB, [src]):
        _run(["gcc", "-O2", "-std=c11", "-fPIC", "-shared", "-o", ORACLE_LIB, src, "-lm"])
    return ORACLE_LIB


def build_audit():
    src = os.path.join(CSRC, "audit", "audit_nccl.c")
    os.makedirs(LIBDIR, exist_ok=True)
    if _newer(AUDIT_LIB, [src]):
        _run(["gcc", "-O2", "-std=c11", "-fPIC", "-shared", "-fvisibility=hidden", "-o", AUDIT_LIB, src, "-ldl"])
    return AUDIT_LIB


TESTBIN = os.path.join(ROOT, "tests", "bin")


def build_tests():
    """C++ test programs (tests/cpp/*.cpp) linked against the product library -> tests/bin/."""
    os.makedirs(TESTBIN, exist_ok=True)
    hdrs = _headers()
    outs = []
    srcs = sorted(glob.glob(os.path.join(ROOT, "tests", "cpp", "*.cpp")) +
                  glob.glob(os.path.join(ROOT, "tests", "cpp", "*.hip")))

    def one(src):
        exe = os.path.join(TESTBIN, os.path.splitext(os.path.basename(src))[0])
        if _newer(exe, [src, LIB] + hdrs):
            # .hip: test programs with device code of their own (kernels written against the
            # public device headers), compiled for gfx950
            lang = ["--offload-arch=" + ARCH, "-x", "hip"] if src.endswith(".hip") else ["-D__HIP_PLATFORM_AMD__"]
            _run([HIPCC] + lang + ["-O2", "-std=c++17", "-Wall", "-Wno-unused-variable", "-Wno-unused-parameter",
                                   "-I" + INCLUDE, src, "-o", exe, "-L" + LIBDIR, "-lmscclpp_amd",
                                   "-Wl,-rpath,$ORIGIN/../../mscclpp_amd/lib"])
        return exe

    with cf.ThreadPoolExecutor(max_workers=4) as ex:
        outs = list(ex.map(one, srcs))
    return outs


DIAG_LIB = os.path.join(TESTBIN, "libxcdprobe.so")
SR_DIAG_LIB = os.path.join(TESTBIN, "libselfreduce_diag.so")
LL_DIAG_LIB = os.path.join(TESTBIN, "libll_diag.so")


def build_diag():
    """Test diagnostics with device code -> tests/bin/: the per-XCD readback (tests/diag/xcd_probe.hip)
    and the self-reduce kernel with its shape / poll-miss entry (kernels/self_reduce.hip built with
    MSCCLPP_AMD_DIAG, symbols bound inside the library so it can sit beside the product one)."""
    os.makedirs(TESTBIN, exist_ok=True)
    src = os.path.join(ROOT, "tests", "diag", "xcd_probe.hip")
    if _newer(DIAG_LIB, [src]):
        _run([HIPCC, "--offload-arch=" + ARCH, "-O2", "-std=c++17", "-shared", "-fPIC", src, "-o", DIAG_LIB])
    for src, lib in (("self_reduce.hip", SR_DIAG_LIB), ("allreduce_ll.hip", LL_DIAG_LIB)):
        src = os.path.join(CSRC, "kernels", src)
        if _newer(lib, [src] + _headers()):
            _run([HIPCC, "--offload-arch=" + ARCH, "-x", "hip", "-O3", "-std=c++17", "-fPIC", "-shared",
                  "-DMSCCLPP_AMD_DIAG", "-I" + INCLUDE, "-I" + os.path.join(CSRC, "kernels"), "-Wl,-Bsymbolic", src,
                  "-o", lib])
    return DIAG_LIB


def build_all(verbose=False):
    """Builds what is out of date; returns a one-line summary of what was compiled or linked."""
    del BUILT[:]
    build_oracle()
    build_library(verbose=verbose)
    build_audit()
    build_tests()
    build_diag()
    ref = os.path.join(ROOT, "oracle", "build_ref.sh")
    ref_note = "oracle/_ref: skipped (no /root/reference)"
    if os.path.isdir("/root/reference") and os.path.exists(ref):
        # the reference-header harness (oracle/_ref) can only be built where /root/reference exists
        env = dict(os.environ, REF_FORCE="1") if FORCE else None
        r = subprocess.run(["bash", ref], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
        if verbose or r.returncode != 0:
            print(r.stdout, file=sys.stderr)
        if r.returncode != 0:
            raise RuntimeError("oracle/build_ref.sh failed:\n" + r.stdout)
        ref_note = "oracle/_ref: " + ("; ".join(x for x in r.stdout.splitlines() if x.startswith("built")) or "up to date")
    objs = sum(1 for b in BUILT if b.endswith(".o"))
    rest = [b for b in BUILT if not b.endswith(".o")]
    return (f"build: {objs} objects compiled, {len(rest)} artefacts linked ({', '.join(rest) or 'all up to date'}); "
            + ref_note)


if __name__ == "__main__":
    print(build_all(verbose=True))
