#!/bin/bash
# training A/B on one box: the training GPU tests on the current library, then
# the fused-forward timing (tools/ab/time_train_fwd.py) and the C3 step for
# lib/libnerfhip_old.so (a build of the previous commit) and the current build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abtrain}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_mlp.py tests/test_gpu_train.py tests/test_gpu_frames.py -m gpu -q -x --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -n 1 "$OUT/tests.log"
for v in old new old new; do
  if [ $v = old ]; then export NERFHIP_LIB=$PWD/nerf-rep_for_test_amd/lib/libnerfhip_old.so; else unset NERFHIP_LIB; fi
  echo "== $v"
  timeout -k 10 120 python tools/ab/time_train_fwd.py 196608 20 2>&1 | tail -2 || exit $?
  timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 10 --train-launch eager > "$OUT/c3_$v.log" 2>&1 || exit $?
  grep -o '"ms_per_step": [0-9.]*' "$OUT/c3_$v.log"
done
