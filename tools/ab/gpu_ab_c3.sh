#!/bin/bash
# A/B of variant libraries (NERFHIP_LIB=lib/libnerfhip_<v>.so, VARIANTS="v1 v2")
# against the tree's library on the C3 step: bench.py --config c3 (graph),
# interleaved REPS times, then one rocprofv3 kernel-stats pass per library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abc3}
mkdir -p "$OUT"
VARIANTS=${VARIANTS:-}
for rep in $(seq 1 ${REPS:-2}); do
  for v in base $VARIANTS; do
    if [ $v = base ]; then unset NERFHIP_LIB; else export NERFHIP_LIB=$PWD/nerf-rep_for_test_amd/lib/libnerfhip_$v.so; fi
    timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 10 --train-launch graph > "$OUT/c3_${v}_$rep.log" 2>&1 || exit $?
    python -c "import json; d=json.loads(open('$OUT/c3_${v}_$rep.log').read().strip().splitlines()[-1]); print('$v rep $rep c3 ms/step', round(d['ms_per_step'],3))"
  done
done
if [ "${PROF:-1}" = 1 ]; then
  for v in base $VARIANTS; do
    if [ $v = base ]; then unset NERFHIP_LIB; else export NERFHIP_LIB=$PWD/nerf-rep_for_test_amd/lib/libnerfhip_$v.so; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$v" -o k \
      -- python bench.py --config c3 --steps 10 --warmup 3 --train-launch eager > "$OUT/prof_$v.log" 2>&1 || exit $?
  done
fi
echo done
