#!/bin/bash
# round 2: GPU tests, bench with the trained checkpoint, wide-kernel timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r2b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log
[ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python bench.py --precision f16x3w --no-fp32-run --no-cpu-baseline --no-c3 --steps 3 > $O/bench_x3w.log 2>&1 || exit $?
tail -c 1500 $O/bench_x3w.log
timeout -k 10 600 python bench.py --steps 5 > $O/bench.log 2>&1 || exit $?
tail -c 3000 $O/bench.log
