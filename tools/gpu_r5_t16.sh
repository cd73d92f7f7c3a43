#!/bin/bash
# round 5: the T16 training layout -- training MLP tests, gradient parity, C3 timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5_t16}
mkdir -p $O
NERF_FRAME_REPORT=$O/frames timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread \
  tests/test_gpu_train_mlp.py tests/test_gpu_train.py tests/test_gpu_train_ops.py > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for mode in 1 0 1; do
  NERF_TRAIN_T16=$mode timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 5 --train-launch eager > $O/c3_t16_$mode.log 2>&1 || exit $?
  echo "T16=$mode $(tail -1 $O/c3_t16_$mode.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
