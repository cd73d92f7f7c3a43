#!/bin/bash
# A/B of variant libraries (NERFHIP_LIB=lib/libnerfhip_<v>.so, VARIANTS="v1 v2")
# against the tree's library: the kernel alone at the C3 fine size
# (tools/train_kernels_bench.py) and the whole C3 step, interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abw}
mkdir -p "$OUT"
VARIANTS=${VARIANTS:-wv2}
for rep in 1 2; do
  for v in base $VARIANTS; do
    if [ $v = base ]; then unset NERFHIP_LIB; else export NERFHIP_LIB=$PWD/nerf-rep_for_test_amd/lib/libnerfhip_$v.so; fi
    echo "== $v rep $rep"
    timeout -k 10 200 python tools/train_kernels_bench.py > "$OUT/kbench_${v}_$rep.log" 2>&1 || exit $?
    grep "wgrad" "$OUT/kbench_${v}_$rep.log" | head -3
    timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 10 --train-launch graph > "$OUT/c3_${v}_$rep.log" 2>&1 || exit $?
    python -c "import json,sys; d=json.loads(open('$OUT/c3_${v}_$rep.log').read().strip().splitlines()[-1]); print('c3 ms/step', round(d['ms_per_step'],3))"
  done
done
