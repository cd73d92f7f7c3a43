#!/bin/bash
# round-2 closing pass: GPU tests, smoke, default bench + rocprof (gpu_check.sh),
# then the round-2 profiles (C2/C3 kernel stats, HBM bench, PMC) and the C3/C4 lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r2final
# schedule ablations of the shipped x3 kernel (tools/mlp_ablate.py build 0 <variants> first)
if ls nerf-rep_for_test_amd/build/abl/lib_x3.so > /dev/null 2>&1; then
  timeout -k 10 200 python tools/mlp_ablate.py run 30 ${ABL:-x3 x3_ord0 x3_ilv1 x3_ilv3 x3_ilv4 x3_nodma x3_noepi} > gpurun_out/r2final/ablate.log 2>&1 || exit $?
  cat gpurun_out/r2final/ablate.log
fi
TAG=r2final bash tools/gpu_check.sh || exit $?
bash tools/gpu_r2_prof.sh || exit $?
O=gpurun_out/r2final
timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 5 > $O/c3.log 2>&1 || exit $?
tail -1 $O/c3.log | cut -c1-200
timeout -k 10 400 python bench.py --config c4 --no-fp32-run > $O/c4.log 2>&1 || exit $?
tail -1 $O/c4.log | cut -c1-200
echo "final done"
