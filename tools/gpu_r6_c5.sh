#!/bin/bash
# Round 6 re-run of tools/gpu_r5_c5.sh on the final library. C5 (BASELINE configs[4]) on one GPU: every one of the 200 lego test poses timed
# in turn, then PSNR / SSIM over all 200 ground-truth views (data/lego/test_all.npz,
# tools/pack_lego.py --splits test --test-stride 1; pushed for this call only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6_c5}
mkdir -p $O
timeout -k 10 900 python bench.py --config c5 --all-poses --steps 200 --warmup 2 --no-cpu-baseline \
  --gt-path data/lego/test_all.npz > $O/c5.log 2>&1; rc=$?
tail -c 1500 $O/c5.log
exit $rc
