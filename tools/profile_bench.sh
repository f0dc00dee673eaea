#!/usr/bin/env bash
# Profile bench.py (N=1) on the GPU box: kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in
# separate --pmc passes (MI355X_MICROARCH.md: TCC slots; never combined with other traces).
# Usage (from the repo root, on the box):  bash tools/profile_bench.sh <tag>
set -euo pipefail
TAG=${1:-r1}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o bench --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-extras > "$OUT/trace.log" 2>&1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/fetch" -o bench --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-extras > "$OUT/fetch.log" 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/write" -o bench --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-extras > "$OUT/write.log" 2>&1
python3 "$ROOT/tools/summarize_profile.py" "$OUT" "$TAG"
