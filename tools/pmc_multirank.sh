#!/usr/bin/env bash
# FETCH_SIZE / WRITE_SIZE of the multi-rank kernels (tools/inprocess_pmc_run.py), one --pmc pass each
# (MI355X_MICROARCH.md: counters in their own runs, never beside other traces).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_multirank
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/fetch" -o run --output-format csv -- \
  python3 "$ROOT/tools/inprocess_pmc_run.py" > "$OUT/fetch.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/write" -o run --output-format csv -- \
  python3 "$ROOT/tools/inprocess_pmc_run.py" > "$OUT/write.log" 2>&1
python3 "$ROOT/tools/summarize_pmc_multirank.py" "$OUT" "${1:-r3}"
