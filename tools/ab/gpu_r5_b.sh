#!/bin/bash
# round 5: buffer range-check probe, the lego.yaml eval frame (candidate dump),
# the C3-shape gradient test
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5_b}
mkdir -p $O
timeout -k 10 60 ./tools/probe/buffer_range > $O/probe.log 2>&1; rc=$?; cat $O/probe.log
[ $rc -ne 0 ] && exit $rc
NERF_FRAME_DUMP=$O/cand NERF_FRAME_REPORT=$O/frames timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_frames.py -k "yaml" tests/test_gpu_train.py -k "yaml or bench_shape" > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
exit $rc
