#!/bin/bash
# round 5: every whole-frame test (r0-r3, both precisions) with the tail check on
# the reference's own depths, candidate dumps for make_ref_frames.py --tail
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5_frames}
mkdir -p $O
NERF_FRAME_DUMP=$O/cand NERF_FRAME_REPORT=$O/frames timeout -k 10 900 python -u -m pytest -v --timeout 300 \
  --timeout-method thread tests/test_gpu_frames.py > $O/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed" $O/pytest.log | tail -12
exit $rc
