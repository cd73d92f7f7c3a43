#!/bin/bash
# A/B of variant libraries (lib/libnerfhip_<v>.so, VARIANTS="v1 v2") on the fused
# training forward alone (tools/ab/time_train_fwd.py, fine-pass P), interleaved
# three times: inputs identical across libraries, so a variant that writes
# another layout is timed on the same data (the C3 step would feed it back).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for rep in 1 2 3; do for v in base ${VARIANTS:-}; do
  if [ $v = base ]; then unset NERFHIP_LIB; else export NERFHIP_LIB=$PWD/nerf-rep_for_test_amd/lib/libnerfhip_$v.so; fi
  echo "== $v $rep"; timeout -k 10 120 python tools/ab/time_train_fwd.py 196608 30 || exit 1
done; done
