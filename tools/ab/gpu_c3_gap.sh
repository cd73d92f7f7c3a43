#!/bin/bash
# Training tests on the tree's library, a kernel trace of the C3 step replayed
# as a HIP graph (kernel time vs wall time per step: the gaps between
# launches), then the C3 step of the tree's library against
# lib/libnerfhip_prev.so, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-c3gap}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_mlp.py tests/test_gpu_train_ops.py -q -x --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
echo "pytest rc=$?"; tail -2 "$OUT/pytest.log"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o k -- python bench.py --config c3 --steps 20 --warmup 5 --train-launch graph > "$OUT/b.log" 2>&1
echo "trace rc=$?"
for r in 1 2; do for v in new prev; do
  if [ $v = new ]; then unset NERFHIP_LIB; else export NERFHIP_LIB=$PWD/nerf-rep_for_test_amd/lib/libnerfhip_prev.so; fi
  timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 10 --train-launch graph > "$OUT/c3_${v}_$r.log" 2>&1 || exit 1
  python -c "import json; d=json.loads(open('$OUT/c3_${v}_$r.log').read().strip().splitlines()[-1]); print('$v', $r, round(d['ms_per_step'],3))"
done; done
