#!/bin/bash
# round 2 profiles: rocprof kernel stats of the C2 bench and the C3 step, HBM
# micro-bench of the byte-moving kernels, PMC passes of the C2 frame
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r2prof
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o c2 -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-run --no-gt --no-c3 > $O/c2.log 2>&1 || exit $?
tail -c 400 $O/c2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o c3 -- python bench.py --config c3 --steps 10 --warmup 3 > $O/c3.log 2>&1 || exit $?
timeout -k 10 300 python tools/hbm_bench.py $O/hbm.json > $O/hbm.log 2>&1 || exit $?
tail -20 $O/hbm.log
TAG=r2prof/pmc bash tools/pmc.sh > $O/pmc.log 2>&1 || exit $?
tail -5 $O/pmc.log
