#!/bin/bash
# GPU round: tests -> smoke -> bench -> rocprof kernel trace. Every GPU step has
# its own time limit; a crash/timeout (exit >= 124 or signal) stops the script.
# Ordinary test failures (pytest exit 1) do not stop the later steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export NERF_FRAME_REPORT="$OUT/frames"
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 1 -a $rc -ne 5 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -q ${PYTEST_X--x} -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
[ "${SKIP_SMOKE:-0}" = 1 ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 900 python bench.py ${BENCH_ARGS:-}
if [ "${PROFILE:-1}" = 1 ]; then
  step rocprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench \
       -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gt ${PROF_ARGS:-}
fi
echo "== done"
