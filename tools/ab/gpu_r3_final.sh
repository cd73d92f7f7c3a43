#!/bin/bash
# Round-3 closing pass on one box: GPU tests, smoke, default bench, rocprof
# kernel stats (tools/gpu_check.sh), then the C5 test-set bench, the HBM
# micro-benchmarks and one FETCH_SIZE pass over them (the random-gather
# kernels' real HBM traffic). Each GPU step has its own time limit; a failure
# stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
TAG=${TAG:-r3final} bash tools/gpu_check.sh || exit $?
OUT=gpurun_out/${TAG:-r3final}
timeout -k 10 300 python bench.py --config c5 --steps 25 --warmup 1 --no-fp32-run > "$OUT/c5.log" 2>&1 || exit $?
tail -n 1 "$OUT/c5.log" | cut -c1-400
timeout -k 10 300 python tools/hbm_bench.py "$OUT/hbm.json" > "$OUT/hbm.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/hbm_pmc" -o pmc \
  -- python tools/hbm_bench.py > "$OUT/hbm_pmc.log" 2>&1 || exit $?
echo "== done"
