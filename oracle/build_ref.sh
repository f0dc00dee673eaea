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
# REF_FORCE=1 (MSCCLPP_AMD_FORCE_REBUILD=1 in mscclpp_amd/_build.py): rebuild whatever the timestamps
FORCE=${REF_FORCE:-0}
if [ "$FORCE" = 1 ] || ! { [ "$OUT/libref.so" -nt "$HERE/ref_harness.hip" ] && [ "$OUT/libref.so" -nt "$HERE/build_ref.sh" ]; }; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -D__HIP_PLATFORM_AMD__ \
    -I"$REF/include" "$HERE/ref_harness.hip" -o "$OUT/libref.so"
  echo "built $OUT/libref.so"
fi
# The reference's python benchmark kernels (python/mscclpp_benchmark/allreduce.cu), one code object
# per TYPE (int, float, __half), whose allreduce2 ref_harness.hip's refBench2* run as n ranks on one
# GPU.  int pins geometry, packet images and flags; float and __half also pin the order and the
# rounding of the sum (0 + peers ascending + own, unclipped, :257-264).
BENCH_CU="$REF/python/mscclpp_benchmark/allreduce.cu"
for spec in int:int float:float half:__half; do
  name=${spec%%:*}
  type=${spec#*:}
  obj="$OUT/bench_allreduce_$name.hsaco"
  if [ -f "$BENCH_CU" ] && { [ "$FORCE" = 1 ] || ! { [ "$obj" -nt "$BENCH_CU" ] && [ "$obj" -nt "$HERE/build_ref.sh" ]; }; }; then
    /opt/rocm/bin/hipcc --genco --offload-arch=gfx950 -O3 -std=c++17 -D__HIP_PLATFORM_AMD__ -DTYPE="$type" \
      -I"$REF/include" "$BENCH_CU" -o "$obj"
    echo "built $obj"
  fi
done
