#!/bin/bash
# Round 6: the sample-major T16 tile (one 16-B store per lane and tile in the
# fused training kernels; the weight gradient's owner waves transpose) -- the
# training GPU tests, then C3 against the previous library (make in a checkout
# of the last commit -> lib/libnerfhip_old.so, NERFHIP_LIB), alternating, and a
# kernel trace of each; then the fine d z enqueued before / after its
# side-stream weight gradients (NERF_TRAIN_DZ_FIRST).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-t16s}
mkdir -p $O
timeout -k 10 300 python -u tools/ab/dbg_wgrad_t16.py > $O/dbg.log 2>&1 || { tail -20 $O/dbg.log; exit 1; }
grep -c "bad 0 " $O/dbg.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_train_mlp.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
ms() { grep '^{' $1 | tail -1 | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])'; }
for v in old new old new; do
  if [ $v = old ]; then L="NERFHIP_LIB=nerf-rep_for_test_amd/lib/libnerfhip_old.so"; else L=""; fi
  env $L timeout -k 10 200 python bench.py --config c3 --steps 60 --warmup 10 --train-launch graph > $O/c3_$v.log 2>&1 || { tail -5 $O/c3_$v.log; exit 1; }
  echo "== c3 graph $v $(ms $O/c3_$v.log)"
done
for v in old new; do
  if [ $v = old ]; then L="NERFHIP_LIB=nerf-rep_for_test_amd/lib/libnerfhip_old.so"; else L=""; fi
  env $L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k_$v -o k -- python bench.py --config c3 --steps 20 --warmup 5 --train-launch eager > $O/k_$v.log 2>&1 || { tail -5 $O/k_$v.log; exit 1; }
  echo "== kernels $v (eager $(ms $O/k_$v.log) ms)"
  python - $O/k_$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(f'{r["Name"][:60]:60s} {r["Calls"]:>5s} {float(r["AverageNs"])/1e3:8.1f} us')
PY
done
for dz in 0 1 0 1; do
  NERF_TRAIN_DZ_FIRST=$dz timeout -k 10 200 python bench.py --config c3 --steps 60 --warmup 10 --train-launch graph > $O/dz$dz.log 2>&1 || { tail -5 $O/dz$dz.log; exit 1; }
  echo "== dz_first=$dz $(ms $O/dz$dz.log)"
done
