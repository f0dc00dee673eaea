#!/bin/bash
# One GPU-box session: each step runs under its own time limit and writes under gpurun_out/.
# A step that fails normally (exit 1 or 2: a failed test, a failed check) lets the next step run;
# a step that faults, aborts, crashes or times out (any other non-zero code) ends the session, so
# nothing more touches a GPU that may be in a bad state.
#   tools/gpu_session.sh "<name> <seconds> <command...>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
status=0
for spec in "$@"; do
  name=${spec%% *}
  rest=${spec#* }
  secs=${rest%% *}
  cmd=${rest#* }
  echo "[session $(date +%H:%M:%S)] $name (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
  rc=$?
  echo "[session $(date +%H:%M:%S)] $name rc=$rc"
  tail -n 3 "gpurun_out/$name.out"
  if [ $rc -ne 0 ]; then
    status=$rc
    if [ $rc -ne 1 ] && [ $rc -ne 2 ]; then
      echo "[session] $name ended with $rc: stopping here"
      tail -n 20 "gpurun_out/$name.err"
      exit $rc
    fi
  fi
done
exit $status
