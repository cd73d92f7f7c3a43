#!/bin/bash
# timing-only ablations of the batched weight-gradient kernel (make variant
# V=wabl<n> VFLAGS=-DNERF_WGRAD_ABL=<n>): 1 = no MFMAs, 2 = no operand stream,
# 3 = no mid-step barrier, 4 = no step barrier (3 and 4 race: timing only);
# the shipped kernel first and last
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${TAG:-wabl}
mkdir -p $O
for v in base ${VARIANTS:-wabl1 wabl2} base; do
  if [ $v = base ]; then L=""; else L="NERFHIP_LIB=nerf-rep_for_test_amd/lib/libnerfhip_$v.so"; fi
  env $L timeout -k 10 120 python tools/wgrad_layout_bench.py > $O/$v.log 2>&1 || { cat $O/$v.log; exit 1; }
  echo "== $v"; grep -E "us" $O/$v.log
done
