#!/bin/bash
# N > 1 rehearsal on a one-GPU box: bench.py under torch.distributed.run with
# 2 ranks sharing the device over gloo (NERF_DIST_BACKEND=gloo), default config
# (C2 frame sharding + the C4 sub-record) and C3 (data-parallel all-reduce).
# Checks the multi-rank code path end to end (collectives, barriers, max over
# ranks, rank-0 JSON); RCCL itself needs one GPU per rank (the driver's runs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp NERF_DIST_BACKEND=gloo
OUT=gpurun_out/${TAG:-dist2}
mkdir -p "$OUT"
run() {  # name timeout args...
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port ${PORT:-29533} bench.py --gpus 2 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
run c2 600 --steps 2 --warmup 1 --no-fp32-run
run c3 300 --config c3 --steps 5 --warmup 3
echo "== done"
