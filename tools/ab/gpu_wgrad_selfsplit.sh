#!/bin/bash
# self-split weight-gradient kernel vs round 4's per-wave split (make variant
# V=ss0 VFLAGS=-DNERF_WGRAD_SELFSPLIT=0 at commit 5e5efee; the form is removed
# since): results bit for bit, launch times,
# C3 step times interleaved, then the training-MLP tests on the shipped build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-wss}
mkdir -p $O
OLD=NERFHIP_LIB=nerf-rep_for_test_amd/lib/libnerfhip_ss0.so
WGRAD_DUMP=$O/new.pt timeout -k 10 120 python tools/wgrad_layout_bench.py > $O/wl_new.log 2>&1 || { cat $O/wl_new.log; exit 1; }
env $OLD WGRAD_DUMP=$O/old.pt timeout -k 10 120 python tools/wgrad_layout_bench.py > $O/wl_old.log 2>&1 || { cat $O/wl_old.log; exit 1; }
python - "$O" <<'PY' || exit 1
import sys, torch
a = torch.load(sys.argv[1] + "/new.pt", weights_only=True)
b = torch.load(sys.argv[1] + "/old.pt", weights_only=True)
assert len(a) == len(b)
bad = [i for i, (x, y) in enumerate(zip(a, b)) if not torch.equal(x, y)]
print("self-split vs per-wave split:", "bitwise equal" if not bad else f"DIFFER at {bad}", len(a), "tensors")
sys.exit(1 if bad else 0)
PY
echo "== new"; grep us $O/wl_new.log; echo "== old"; grep us $O/wl_old.log
for v in new old new old; do
  if [ $v = old ]; then L=$OLD; else L=""; fi
  env $L timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 5 --train-launch eager > $O/c3_$v.log 2>&1 || { tail -5 $O/c3_$v.log; exit 1; }
  echo "c3 $v $(tail -1 $O/c3_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread \
  tests/test_gpu_train_mlp.py tests/test_gpu_train.py > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
exit $rc
