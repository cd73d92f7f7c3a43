#!/bin/bash
# round 5, C3 after the self-split weight gradient: wgrad ablations (make variant
# V=wabl1 / wabl2 VFLAGS=-DNERF_WGRAD_ABL=1 / 2), the step's kernel trace, and
# the PMC passes tools/pmc_step_summary.py reduces to profiles/r5_c3_pmc_summary.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5_c3}
mkdir -p $O
for v in base wabl1 wabl2; do
  if [ $v = base ]; then L=""; else L="NERFHIP_LIB=nerf-rep_for_test_amd/lib/libnerfhip_$v.so"; fi
  env $L timeout -k 10 120 python tools/wgrad_layout_bench.py > $O/wl_$v.log 2>&1 || { cat $O/wl_$v.log; exit 1; }
  echo "== $v"; grep us $O/wl_$v.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o c3 -- python bench.py --config c3 --steps 25 --warmup 5 --train-launch eager > $O/c3_trace.log 2>&1 || { tail -5 $O/c3_trace.log; exit 1; }
tail -1 $O/c3_trace.log | cut -c1-300
TAG=${TAG:-r5_c3}/pmc BENCH_ARGS="--config c3 --steps 10 --warmup 3 --train-launch eager" \
  PMC_GROUPS="FETCH_SIZE WRITE_SIZE__SQ_VALU_MFMA_BUSY_CYCLES__GRBM_GUI_ACTIVE__SQ_WAVE_CYCLES__SQ_BUSY_CYCLES" \
  bash tools/pmc.sh
