#!/bin/bash
# kernel trace of C4 frames (timeline per frame: tools/ab/c4_timeline.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-c4trace}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o k -- python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-fp32-run ${ARGS:-} > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
python tools/ab/c4_timeline.py $O/prof > $O/timeline.txt 2>&1
tail -1 $O/bench.log | cut -c1-200
