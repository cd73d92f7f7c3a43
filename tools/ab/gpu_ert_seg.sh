#!/bin/bash
# Round 6: the C4 frame's ERT depth-segment length (bench.py --ert-segment),
# interleaved: 8 (shipped), 4, 6, 12.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${TAG:-ert_seg}
mkdir -p $O
for rep in 1 2; do for sg in 8 4 6 12; do
  timeout -k 10 300 python bench.py --config c4 --ert-segment $sg --steps 5 --warmup 1 --no-cpu-baseline --no-fp32-run > $O/s${sg}_$rep.log 2>&1 || { tail -5 $O/s${sg}_$rep.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$O/s${sg}_$rep.log') if l.startswith('{')][-1]); e=d.get('ert_compaction',{}); print('seg $sg rep $rep', round(d['value'],4), 'Mrays/s', round(d['ms_per_step'],2), 'ms', e.get('evaluated_fraction'), d['parity_vs_reference_frame'].get('grid_final_equal'))"
done; done
