#!/bin/bash
# Round-6 closing pass: tools/gpu_final.sh (GPU tests, smoke, bench, rocprof
# kernel stats, headline and C3 PMC passes), then the C3 graph step's kernel
# trace (tools/ab/gpu_c3_trace.sh -> tools/ab/c3_timeline.py). Stops at the
# first crash / time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUND=r6 bash tools/gpu_final.sh || exit $?
TAG=r6_final_c3trace bash tools/ab/gpu_c3_trace.sh || exit $?
python tools/ab/c3_timeline.py gpurun_out/r6_final_c3trace/prof > gpurun_out/r6_final_c3trace/timeline.txt 2>&1
echo "== r6 final done"
