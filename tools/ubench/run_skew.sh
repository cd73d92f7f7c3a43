#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/ubench/run.sh base rot1 rot8 rot24 skew2 skew4 || exit $?
mkdir -p gpurun_out/ubench
timeout -k 10 300 python tools/mlp_ablate.py run 4 x3 x3_skew1 x3_skew2 x3_skew3 > gpurun_out/ubench/skew_ablate.log 2>&1; rc=$?
cat gpurun_out/ubench/skew_ablate.log | tail -8
exit $rc
