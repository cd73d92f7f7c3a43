#!/bin/bash
# round 5: ESS frames with the tail-given-reference-depths check, the perturbed
# interleaved C4 test, then a bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5_d}
mkdir -p $O
NERF_FRAME_DUMP=$O/cand NERF_FRAME_REPORT=$O/frames timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_frames.py tests/test_gpu_render.py -k "${K:-yaml or c4_frame16 or interleaved_perturbed}" > $O/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|passed|failed" $O/pytest.log | tail -12
[ $rc -ge 2 ] && exit $rc
timeout -k 10 900 python bench.py --steps 3 --no-fp32-run --no-cpu-baseline --no-gt --no-c3 > $O/bench.log 2>&1; rc2=$?
tail -c 3000 $O/bench.log
exit $rc2
