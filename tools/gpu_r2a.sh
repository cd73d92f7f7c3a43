#!/bin/bash
# round 2, first GPU pass: parity report, GPU tests, smoke, bench (no profile)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r2a
timeout -k 10 300 python -u tools/parity_report.py --out gpurun_out/r2a/parity.json > gpurun_out/r2a/parity.log 2>&1 || exit $?
TAG=r2a PROFILE=0 BENCH_ARGS="--steps 5 --warmup 1" bash tools/gpu_check.sh
