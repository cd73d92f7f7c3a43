#!/bin/bash
# Round 6: the fine network's side-stream weight gradients leave L CUs free for
# the main stream's coarse backward chain (NERF_TRAIN_SIDE_WGRAD_LEAVE_CUS),
# C3 graph step, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${TAG:-leave_cus}
mkdir -p $O
ms() { grep '^{' $1 | tail -1 | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])'; }
for L in ${LS:-0 16 32 64 0 16 32 64}; do
  NERF_TRAIN_SIDE_WGRAD_LEAVE_CUS=$L timeout -k 10 200 python bench.py --config c3 --steps 60 --warmup 10 --train-launch graph > $O/l$L.log 2>&1 || { tail -5 $O/l$L.log; exit 1; }
  echo "== leave $L: $(ms $O/l$L.log)"
done
