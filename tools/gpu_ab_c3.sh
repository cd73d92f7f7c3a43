#!/bin/bash
# training-kernel A/B on one box: tests of the current library, then the
# kernel bench and the C3 step for lib/libnerfhip_old.so and the current build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abc3}
mkdir -p "$OUT"
step() {
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-6} "$OUT/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step tests 600 python -u -m pytest tests/test_gpu_train_mlp.py tests/test_gpu_train.py -m gpu -q -x --timeout 120 --timeout-method thread ${PYTEST_K:-}
for v in old new a; do
  if [ $v = old ]; then export NERFHIP_LIB=$PWD/nerf-rep_for_test_amd/lib/libnerfhip_old.so; else unset NERFHIP_LIB; fi
  [ $v = a ] && export NERFHIP_LIB=$PWD/nerf-rep_for_test_amd/lib/libnerfhip_old.so
  step kbench_$v 300 python tools/train_kernels_bench.py
  step c3_$v 300 python bench.py --config c3 --steps 30 --warmup 10 --train-launch eager
done
echo "== done"
