#!/bin/bash
# SQ stall breakdown of the weight-gradient kernel alone (tools/train_kernels_bench.py
# at the C3 fine size), one counter group per rocprofv3 pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-wpmc}
mkdir -p "$OUT"
i=0
for grp in ${PMC_GROUPS:-SQ_WAVE_CYCLES__SQ_WAIT_ANY__SQ_WAIT_INST_ANY__SQ_ACTIVE_INST_ANY__SQ_ACTIVE_INST_VALU__SQ_ACTIVE_INST_LDS__SQ_ACTIVE_INST_MISC__SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES__GRBM_GUI_ACTIVE__SQ_BUSY_CYCLES__SQ_INSTS_VALU__SQ_INSTS_LDS__SQ_INSTS_VMEM__SQ_LDS_BANK_CONFLICT__SQ_INSTS_SALU}; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -s KILL 120 rocprofv3 --pmc ${grp//__/ } --kernel-trace --output-format csv -d "$OUT/p$i" -o pmc \
      -- python tools/train_kernels_bench.py > "$OUT/p$i.log" 2>&1
  rc=$?; echo "rc=$rc"; tail -2 "$OUT/p$i.log"
  if [ $rc -ne 0 ]; then echo "STOP"; exit $rc; fi
done
