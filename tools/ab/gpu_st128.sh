#!/bin/bash
# Round 6 study: (1) the fused training kernels' row stores as one 16-B store
# per tile (timing-only build NERF_ABL_NOSTORE=4: make variant V=st128) against
# the shipped b32 stores, per-kernel C3 times from a rocprofv3 kernel trace of
# eager steps; (2) the fine node's d z enqueued before / after its side-stream
# weight gradients (NERF_TRAIN_DZ_FIRST), the graph step's ms.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-st128}
mkdir -p $O
for v in base st128 base st128; do
  if [ $v = base ]; then L=""; else L="NERFHIP_LIB=nerf-rep_for_test_amd/lib/libnerfhip_$v.so"; fi
  d=$O/${v}_$RANDOM
  env $L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o k -- python bench.py --config c3 --steps 20 --warmup 5 --train-launch eager > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  echo "== $v $(grep '^{' $d.log | tail -1 | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  python - $d <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:6]:
    print(f'{r["Name"][:60]:60s} {r["Calls"]:>5s} {float(r["AverageNs"])/1e3:8.1f} us')
PY
done
for dz in 1 0 1 0; do
  NERF_TRAIN_DZ_FIRST=$dz timeout -k 10 200 python bench.py --config c3 --steps 60 --warmup 10 --train-launch graph > $O/dz$dz.log 2>&1 || { tail -5 $O/dz$dz.log; exit 1; }
  echo "== dz_first=$dz $(grep '^{' $O/dz$dz.log | tail -1 | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
