#!/bin/bash
# run the act_lds microbenchmark variants (each under its own time limit)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/ubench
for v in "$@"; do
  timeout -k 10 60 ./tools/ubench/act_lds_$v > gpurun_out/ubench/$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"; cat gpurun_out/ubench/$v.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
