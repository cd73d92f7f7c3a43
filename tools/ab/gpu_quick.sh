#!/bin/bash
# quick loop: selected GPU test files ($TESTS), then a short bench ($BENCH_ARGS)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-quick}
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-300
