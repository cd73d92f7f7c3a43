#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/ubench
for v in "$@"; do
  timeout -k 10 60 ./tools/ubench/act_lds${UB:-2}_$v > gpurun_out/ubench/${UB:-2}_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"; tail -1 gpurun_out/ubench/${UB:-2}_$v.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
