#!/usr/bin/env bash
# rocprofv3 kernel trace + stats of the N>1 benchmark (a rehearsal on a one-GPU box: the ranks share
# the device): the dominant kernel's rocprof average beside the bench line's HIP-event kernel_us.
# Usage (from the repo root, on the box):  bash tools/profile_bench_multi.sh <tag> [ranks]
set -euo pipefail
TAG=${1:-r4}
N=${2:-2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_multi_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o bench --output-format csv -- \
  python3 "$ROOT/bench.py" --gpus "$N" --steps 20 --warmup 5 --no-cpu-baseline --no-extras > "$OUT/bench.log" 2>&1
tail -n 1 "$OUT/bench.log" > "$OUT/bench_line.json"
