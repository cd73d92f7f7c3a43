#!/bin/bash
# PMC passes over the x3 MLP kernel alone (tools/mlp_ablate.py run on prebuilt
# variants), one counter group per rocprofv3 run, each under its own limit.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-x3pmc}
mkdir -p "$OUT"
V=${VARIANT:-x3}
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
i=0
for grp in ${PMC_GROUPS}; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc ${grp//__/ } --kernel-trace --output-format csv -d "$OUT/p$i" -o pmc \
      -- python tools/mlp_ablate.py run 2 $V > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
