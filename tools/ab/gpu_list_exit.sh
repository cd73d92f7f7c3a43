#!/bin/bash
# Round 6: idle workgroups of the list MLP leave before the weight prologue --
# the GPU suite, C4 against the previous library, and the launch sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-list_exit}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TAG=list_exit/c4 REPS=4 STEPS=5 bash tools/ab/ab_c4.sh || exit 1
timeout -k 10 300 python tools/ab/c4_launch_sizes.py 8 > $O/sizes.log 2>&1 || { tail -5 $O/sizes.log; exit 1; }
grep -v amdgpu.ids $O/sizes.log
