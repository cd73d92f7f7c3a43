#!/bin/bash
# The driver's multi-GPU command form on a one-GPU box: `python bench.py --gpus N`
# self-launching N ranks (gloo rehearsal: the ranks share the GPU; the shard
# structure, collectives, barriers and max-over-ranks are the real ones). Stops
# at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r6_selflaunch}
mkdir -p $O
for n in 2 4; do
  NERF_DIST_BACKEND=gloo timeout -k 10 420 python bench.py --gpus $n --steps 2 --warmup 1 > $O/bench_gpus$n.log 2>&1 || { echo "n=$n failed"; tail -5 $O/bench_gpus$n.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$O/bench_gpus$n.log') if l.startswith('{')][-1]); print($n, d['n_gpus'], round(d['value'],3), [r['pixels'] for r in d['shards']], d['c4_ess_ert']['value'] > 0, 'c3' in str(d.keys()))"
done
python bench.py --gpus 2 > $O/bench_rccl_gpus2.log 2>&1; echo "rccl --gpus 2 on one GPU: rc=$? (2 expected)"
