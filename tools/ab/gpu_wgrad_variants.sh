#!/bin/bash
# weight-gradient study builds (make variant V=<v> VFLAGS=...): each variant's
# results bit for bit against the shipped build, launch times interleaved twice,
# then C3 step times interleaved for the variants in C3VARS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-wvar}
mkdir -p $O
VARS=${VARIANTS:-sp1 sp2}
lib() { [ "$1" = base ] && echo "" || echo "NERFHIP_LIB=nerf-rep_for_test_amd/lib/libnerfhip_$1.so"; }
for rep in 1 2; do
  for v in base $VARS; do
    env $(lib $v) WGRAD_DUMP=$O/$v.pt timeout -k 10 120 python tools/wgrad_layout_bench.py > $O/wl_${v}_$rep.log 2>&1 || { cat $O/wl_${v}_$rep.log; exit 1; }
    echo "$rep $v $(grep 'block layout' $O/wl_${v}_$rep.log)"
  done
done
python - "$O" $VARS <<'PY' || exit 1
import sys, torch
a = torch.load(sys.argv[1] + "/base.pt", weights_only=True)
ok = True
for v in sys.argv[2:]:
    b = torch.load(f"{sys.argv[1]}/{v}.pt", weights_only=True)
    bad = [i for i, (x, y) in enumerate(zip(a, b)) if not torch.equal(x, y)]
    print(v, "bitwise equal" if not bad else f"DIFFER at {bad}")
    ok = ok and not bad
sys.exit(0 if ok else 1)
PY
for rep in 1 2; do
  for v in base ${C3VARS:-}; do
    env $(lib $v) timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 5 --train-launch eager > $O/c3_${v}_$rep.log 2>&1 || { tail -5 $O/c3_${v}_$rep.log; exit 1; }
    echo "c3 $rep $v $(tail -1 $O/c3_${v}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
