#!/bin/bash
# SQ counters of the C3 training kernels (one pass; eager step)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3c3pmc}
mkdir -p "$OUT"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d "$OUT/p1" -o pmc -- python bench.py --config c3 --steps 10 --warmup 3 --train-launch eager > "$OUT/p1.log" 2>&1 || exit $?
echo "== done"
