#!/bin/bash
# timing-only ablations of the weight-gradient kernel (libraries built from
# temporary patches: 1 = no MFMAs, 2 = no LDS-DMA issue, 3 = no FP16 split)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/wabl
for v in base abl1 abl2 abl3; do
  if [ $v = base ]; then unset NERFHIP_LIB; else export NERFHIP_LIB=$PWD/nerf-rep_for_test_amd/lib/libnerfhip_$v.so; fi
  echo "== $v"
  timeout -k 10 200 python tools/train_kernels_bench.py > gpurun_out/wabl/$v.log 2>&1 || exit $?
  grep "wgrad" gpurun_out/wabl/$v.log
done
