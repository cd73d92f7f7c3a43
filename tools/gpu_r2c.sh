#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r2c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -25 $O/pytest_gpu.log
[ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
timeout -k 10 400 python tools/mlp_ablate.py run 6 x3 x3_prio_hi x3_prio_lo x3_ldhi x3_ldhi_prio_lo x3_ilv1 x3_ilv3 > $O/ablate.log 2>&1 || exit $?
cat $O/ablate.log
