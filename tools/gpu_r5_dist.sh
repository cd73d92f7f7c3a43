#!/bin/bash
# Multi-GPU readiness without the hardware: bench.py's sharded frames at world
# 2 / 4 / 8 as ranks over gloo sharing the box's one GPU (NERF_DIST_BACKEND=gloo),
# each run's per-rank shard report (owned pixels / chunks, replayed grid-update
# chunks, MLP launches and sizes per frame). Timing is not the point: 8 ranks
# share one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5_dist}
mkdir -p $O
port=29611
for cfg in c2 c4; do
  for W in 2 4 8; do
    port=$((port+1))
    NERF_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus $W --config $cfg --steps 2 --warmup 1 \
      --no-cpu-baseline --no-gt --no-fp32-run > $O/${cfg}_w$W.log 2>&1 || { tail -20 $O/${cfg}_w$W.log; exit 1; }
    echo "== $cfg world $W"; tail -1 $O/${cfg}_w$W.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); [print(r) for r in d.get("shards", [])]'
  done
done
