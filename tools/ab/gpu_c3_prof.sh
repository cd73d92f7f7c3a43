#!/bin/bash
# C3 kernel breakdown (rocprof kernel stats of the eager training step) and the
# kilonerf op tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3c3}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kilonerf.py -m gpu -q -x --timeout 120 --timeout-method thread > "$OUT/kn_tests.log" 2>&1 || exit $?
tail -n 1 "$OUT/kn_tests.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o c3 \
  -- python bench.py --config c3 --steps 30 --warmup 10 --train-launch eager > "$OUT/c3prof.log" 2>&1 || exit $?
tail -n 1 "$OUT/c3prof.log" | cut -c1-300
echo "== done"
