#!/bin/bash
# The C4 frame (bench.py --config c4) for the tree's library and
# lib/libnerfhip_<v>.so (VARIANTS), interleaved REPS times on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abc4}
mkdir -p "$OUT"
ARGS="--config c4 --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-fp32-run"
for rep in $(seq 1 ${REPS:-2}); do for v in new ${VARIANTS:-prev}; do
  if [ $v = new ]; then unset NERFHIP_LIB; else export NERFHIP_LIB=$PWD/nerf-rep_for_test_amd/lib/libnerfhip_$v.so; fi
  timeout -k 10 300 python bench.py $ARGS > "$OUT/c4_${v}_$rep.log" 2>&1 || exit 1
  python -c "import json; d=json.loads([l for l in open('$OUT/c4_${v}_$rep.log') if l.startswith('{')][-1]); print('$v', $rep, round(d['value'],4), 'Mrays/s', round(d['ms_per_step'],2), 'ms/frame', d['parity_vs_reference_frame'].get('max_abs_err_rgb_map'), d['parity_vs_reference_frame'].get('grid_final_equal'))"
done; done
