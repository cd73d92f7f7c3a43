#!/bin/bash
# C3 loop: training-MLP GPU tests, the C3 bench line, a kernel-stats profile of it
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-c3}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_mlp.py tests/test_gpu_train.py tests/test_gpu_train_ops.py -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 5 > $O/c3.log 2>&1 || exit $?
tail -1 $O/c3.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c3 -- python bench.py --config c3 --steps 10 --warmup 3 > $O/c3prof.log 2>&1 || exit $?
echo done
