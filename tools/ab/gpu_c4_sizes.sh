#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/c4_sizes
mkdir -p $O
for sg in 8 16; do
  timeout -k 10 300 python tools/ab/c4_launch_sizes.py $sg > $O/s$sg.log 2>&1 || { tail -5 $O/s$sg.log; exit 1; }
  grep -v amdgpu.ids $O/s$sg.log
done
