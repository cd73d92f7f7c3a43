#!/bin/bash
# PMC passes for the bench workload (one counter group per rocprofv3 run;
# PMC_SCRIPT=<script> profiles another python entry point, with BENCH_ARGS as its arguments).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
ARGS=${BENCH_ARGS---steps 1 --warmup 0 --no-cpu-baseline --no-fp32-run --no-gt --no-c3 --no-c4}
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
i=0
for grp in ${PMC_GROUPS:-FETCH_SIZE WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES__GRBM_GUI_ACTIVE__SQ_WAVE_CYCLES__SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT__SQ_INSTS_LDS__SQ_INSTS_VALU_MFMA_F32}; do
  i=$((i+1))
  echo "== pass $i: $grp"
  # a group is counters joined by "__" (one env word); rocprofv3 takes them space-separated
  timeout -k 10 600 rocprofv3 --pmc ${grp//__/ } --kernel-trace --output-format csv -d "$OUT/p$i" -o pmc \
      -- python ${PMC_SCRIPT:-bench.py} $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?; echo "rc=$rc"; tail -2 "$OUT/p$i.log"
  if [ $rc -ne 0 ]; then echo "STOP"; exit $rc; fi
done
