#!/usr/bin/env bash
# Build oracle/_ref/libref.so: the reference's own device headers (where they lie under
# /root/reference, nothing copied) driven by oracle/ref_harness.hip.  Test infrastructure only.
# Only possible where /root/reference exists; the built .so travels to the GPU box (it is
# git-ignored, not gpurun-ignored).
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
REF=${MSCCLPP_REFERENCE:-/root/reference}
OUT="$HERE/_ref"
mkdir -p "$OUT"
if [ ! -d "$REF/include/mscclpp" ]; then
  echo "reference tree not present: skipping oracle/_ref" >&2
  exit 0
fi
# -D__HIP_PLATFORM_AMD__ selects the reference's HIP branch (gpu_data_types.hpp:50)
if ! { [ "$OUT/libref.so" -nt "$HERE/ref_harness.hip" ] && [ "$OUT/libref.so" -nt "$HERE/build_ref.sh" ]; }; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -D__HIP_PLATFORM_AMD__ \
    -I"$REF/include" "$HERE/ref_harness.hip" -o "$OUT/libref.so"
  echo "built $OUT/libref.so"
fi
# The reference's python benchmark kernels (python/mscclpp_benchmark/allreduce.cu), a code object
# with TYPE=int, whose allreduce2 ref_harness.hip's refBench2* run as n ranks on one GPU.
BENCH_CU="$REF/python/mscclpp_benchmark/allreduce.cu"
if [ -f "$BENCH_CU" ] && ! { [ "$OUT/bench_allreduce_int.hsaco" -nt "$BENCH_CU" ] && \
    [ "$OUT/bench_allreduce_int.hsaco" -nt "$HERE/build_ref.sh" ]; }; then
  /opt/rocm/bin/hipcc --genco --offload-arch=gfx950 -O3 -std=c++17 -D__HIP_PLATFORM_AMD__ -DTYPE=int \
    -I"$REF/include" "$BENCH_CU" -o "$OUT/bench_allreduce_int.hsaco"
  echo "built $OUT/bench_allreduce_int.hsaco"
fi
