"""CPU check of the case tables in test_reference_kernel_gpu.py: every shape is one the reference kernels
take whole (allreduce2: 32-bit words per rank a multiple of 2 n, python/mscclpp_benchmark/allreduce.cu:
229-248; allreduce1: each rank's chunk a whole number of int4 vectors, :160-190), so a bad table entry
fails here instead of on the GPU box."""
import importlib.util
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def _cases():
    spec = importlib.util.spec_from_file_location("ref_gpu_cases", os.path.join(HERE, "test_reference_kernel_gpu.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_reference_kernel_case_shapes():
    t = _cases()
    for n, count, bpp, threads in t.CASES:
        assert 2 <= n <= 8 and count % (2 * n) == 0 and 1 <= bpp * (n - 1) <= 64 and threads % 64 == 0, (n, count)
    for kind, n, words, bpp, threads in t.TYPED_CASES:
        assert kind in ("f16", "f32") and 2 <= n <= 8 and words % (2 * n) == 0, (kind, n, words)
        assert 1 <= bpp * (n - 1) <= 64 and threads % 64 == 0
    for kind, n, words, nblocks, threads, ro in t.BENCH1_CASES:
        assert kind in ("i32", "f16", "f32") and 2 <= n <= 8 and words % n == 0 and (words // n) % 4 == 0
        assert 1 <= nblocks <= 16 and threads % 64 == 0 and nblocks * threads >= 2 * (n - 1) and ro in (0, 1)
