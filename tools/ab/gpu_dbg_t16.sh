#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/dbg_t16
mkdir -p $O
timeout -k 10 300 python -u tools/ab/dbg_wgrad_t16.py > $O/dbg.log 2>&1 || { tail -20 $O/dbg.log; exit 1; }
cat $O/dbg.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_train_mlp.py -q --maxfail 40 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -45 $O/pytest.log | grep -E "passed|failed|FAILED|Error" | head -45
exit 0
