#!/bin/bash
# per-kernel C3 times of study builds (make variant V=<v> ...): one rocprofv3
# kernel trace of 20 eager steps per library (timing only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-c3k}
mkdir -p $O
for v in base ${VARIANTS:-}; do
  if [ $v = base ]; then L=""; else L="NERFHIP_LIB=nerf-rep_for_test_amd/lib/libnerfhip_$v.so"; fi
  env $L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o k -- python bench.py --config c3 --steps 20 --warmup 5 --train-launch eager > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
  echo "== $v $(grep '^{' $O/$v.log | tail -1 | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  python - $O/$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:6]:
    print(f'{r["Name"][:60]:60s} {r["Calls"]:>5s} {float(r["AverageNs"])/1e3:8.1f} us')
PY
done
