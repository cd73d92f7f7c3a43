#!/bin/bash
# Correctness of the tree's library on the training tests, then the fused
# forward alone and the C3 step: tree library vs lib/libnerfhip_<v>.so
# (VARIANTS), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abq}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_mlp.py tests/test_gpu_train_ops.py -q -x --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
echo "pytest rc=$?"; tail -3 "$OUT/pytest.log"
for rep in 1 2; do for v in new ${VARIANTS:-prev}; do
  if [ $v = new ]; then unset NERFHIP_LIB; else export NERFHIP_LIB=$PWD/nerf-rep_for_test_amd/lib/libnerfhip_$v.so; fi
  timeout -k 10 120 python tools/ab/time_train_fwd.py 196608 30 > "$OUT/fwd_${v}_$rep.log" 2>&1 || exit 1
  echo "$v $rep fwd: $(grep 'train (' "$OUT/fwd_${v}_$rep.log")"
  timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 10 --train-launch graph > "$OUT/c3_${v}_$rep.log" 2>&1 || exit 1
  python -c "import json; d=json.loads(open('$OUT/c3_${v}_$rep.log').read().strip().splitlines()[-1]); print('$v rep $rep c3 ms/step', round(d['ms_per_step'],3))"
done; done
