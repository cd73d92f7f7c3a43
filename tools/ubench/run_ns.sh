#!/bin/bash
# one-wave-per-SIMD slice skeleton (tools/ubench/ns_wave.hip), each binary under its own limit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/ubench
for v in "$@"; do
  timeout -k 10 90 ./tools/ubench/ns_wave_$v > gpurun_out/ubench/ns_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"; cat gpurun_out/ubench/ns_$v.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
