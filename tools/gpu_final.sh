#!/bin/bash
# Closing pass of a round: GPU tests, smoke, bench and its rocprof kernel trace
# (tools/gpu_check.sh), then the headline PMC passes (tools/pmc.sh defaults) and
# the C3 step's PMC passes. Stops at the first crash / time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${ROUND:-r4}
TAG=${R}_final PYTEST_X="" PROFILE=1 BENCH_ARGS="--steps 5" PROF_ARGS="--no-fp32-run" \
  bash tools/gpu_check.sh || exit $?
TAG=${R}_final_pmc BENCH_ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-fp32-run --no-gt --no-c3 --no-c4 --no-perturb" bash tools/pmc.sh || exit $?
TAG=${R}_final_pmc_c3 BENCH_ARGS="--config c3 --steps 10 --warmup 3 --train-launch eager" \
  PMC_GROUPS="FETCH_SIZE WRITE_SIZE__SQ_VALU_MFMA_BUSY_CYCLES__GRBM_GUI_ACTIVE__SQ_WAVE_CYCLES__SQ_BUSY_CYCLES" \
  bash tools/pmc.sh || exit $?
echo "== final done"
