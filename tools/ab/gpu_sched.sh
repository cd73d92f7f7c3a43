#!/bin/bash
# Round 6: the x3 kernels built with other LLVM scheduling strategies
# (make variant V=ilp / mclause), headline frame interleaved with the shipped
# build, then the C3 step for each (timing only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
TAG=sched/h REPS=3 STEPS=10 VARIANTS="ilp mclause" bash tools/ab/ab_headline.sh || exit 1
O=gpurun_out/sched
for v in new ilp mclause; do
  if [ $v = new ]; then L=""; else L="NERFHIP_LIB=$PWD/nerf-rep_for_test_amd/lib/libnerfhip_$v.so"; fi
  env $L timeout -k 10 200 python bench.py --config c3 --steps 60 --warmup 10 --train-launch graph > $O/c3_$v.log 2>&1 || { tail -5 $O/c3_$v.log; exit 1; }
  echo "== c3 $v $(grep '^{' $O/c3_$v.log | tail -1 | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
