#!/bin/bash
# Render tests on the tree's library, then the headline frame (bench.py, no
# sub-records) for the tree's library and lib/libnerfhip_<v>.so (VARIANTS),
# interleaved REPS times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abh}
mkdir -p "$OUT"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -q -x --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  echo "pytest rc=$?"; tail -2 "$OUT/pytest.log"
fi
ARGS="--steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-fp32-run --no-gt --no-c3 --no-c4 --no-perturb"
for rep in $(seq 1 ${REPS:-3}); do for v in new ${VARIANTS:-prev}; do
  if [ $v = new ]; then unset NERFHIP_LIB; else export NERFHIP_LIB=$PWD/nerf-rep_for_test_amd/lib/libnerfhip_$v.so; fi
  timeout -k 10 300 python bench.py $ARGS > "$OUT/h_${v}_$rep.log" 2>&1 || exit 1
  python -c "import json; d=json.loads([l for l in open('$OUT/h_${v}_$rep.log') if l.startswith('{')][-1]); r=d['roofline']; print('$v', $rep, round(d['value'],4), 'Mrays/s', round(r['avg_launch_ms'],2), 'ms/launch', round(r['frac'],4))"
done; done
