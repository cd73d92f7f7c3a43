#!/bin/bash
# the weight gradients on a side stream (NERF_TRAIN_SIDE_WGRAD=1, default) vs in
# line (=0): C3 step times, eager and graph, interleaved twice; then the
# training tests with the side stream on
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-side}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread \
  tests/test_gpu_train_mlp.py tests/test_gpu_train.py tests/test_gpu_train_ops.py > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
  for side in 0 1; do
    for launch in eager graph; do
      NERF_TRAIN_SIDE_WGRAD=$side timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 5 \
        --train-launch $launch > $O/c3_${side}_${launch}_$rep.log 2>&1 || { tail -5 $O/c3_${side}_${launch}_$rep.log; exit 1; }
      echo "c3 rep $rep side $side $launch $(tail -1 $O/c3_${side}_${launch}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
    done
  done
done
