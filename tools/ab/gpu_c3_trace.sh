#!/bin/bash
# kernel trace of the C3 graph step (timeline of one step: tools/ab/c3_timeline.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-c3trace}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o k -- python bench.py --config c3 --steps 20 --warmup 5 --train-launch ${LAUNCH:-graph} > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
