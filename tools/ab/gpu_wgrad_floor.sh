#!/bin/bash
# Round 6: the batched weight gradient's K split per tile (NERF_WGRAD_COST_FLOOR:
# a light tile's assumed cost floor; 512 = the equal split), C3 graph step,
# interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${TAG:-wgrad_floor}
mkdir -p $O
for rep in 1 2; do for f in 512 384 448 640 320; do
  NERF_WGRAD_COST_FLOOR=$f timeout -k 10 200 python bench.py --config c3 --steps 60 --warmup 10 --train-launch graph > $O/f${f}_$rep.log 2>&1 || { tail -5 $O/f${f}_$rep.log; exit 1; }
  echo "== floor $f rep $rep $(grep '^{' $O/f${f}_$rep.log | tail -1 | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done; done
