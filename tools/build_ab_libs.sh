#!/usr/bin/env bash
# Build libmscclpp_amd.so at each named commit into tools/ab_libs/<commit>/ for tools/portchannel_ab.py
# (the round-5 A/B that named the round-4 PortChannel regression).  Each commit is
# checked out into a throw-away git worktree under ${AB_TMP:-/tmp/ab} and built there with its own
# mscclpp_amd/_build.py; only the shared library is copied back.  tools/ab_libs/ is git-ignored (*.so)
# and gpurun-ignored: list it out of .gpurunignore for the GPU call that runs the A/B.
#   tools/build_ab_libs.sh 0078d72 7aa8f71 7dc0002
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
TMP=${AB_TMP:-/tmp/ab}
mkdir -p "$TMP"
for c in "$@"; do
  wt="$TMP/$c"
  [ -d "$wt" ] || git -C "$ROOT" worktree add -f "$wt" "$c" >/dev/null
  (cd "$wt" && MAX_JOBS=${MAX_JOBS:-8} python -c "from mscclpp_amd import _build; _build.build_library()")
  mkdir -p "$ROOT/tools/ab_libs/$c"
  cp "$wt/mscclpp_amd/lib/libmscclpp_amd.so" "$ROOT/tools/ab_libs/$c/"
  echo "built tools/ab_libs/$c/libmscclpp_amd.so"
done
