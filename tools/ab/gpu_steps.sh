#!/bin/bash
# Run named GPU steps, each under its own time limit, logs under gpurun_out/$TAG.
# Usage: TAG=x bash tools/ab/gpu_steps.sh "name:timeout:command" ...
# A crash / time limit (rc >= 124) or a signal stops the script; an ordinary
# failure (rc 1-123) is reported and the next step runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-steps}
mkdir -p "$OUT"
export NERF_FRAME_REPORT="$OUT/frames"
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; t=${rest%%:*}; cmd=${rest#*:}
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -n 4 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ge 124 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
done
echo "== done"
