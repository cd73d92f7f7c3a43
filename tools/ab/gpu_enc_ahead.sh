#!/bin/bash
# Round 6: the next tile's xyz encoding in the views layer's MFMA shadows
# (NERF_X3_ENC_AHEAD) -- the GPU suite, then the headline frame and the C4 frame
# against the previous library (lib/libnerfhip_prev.so), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-enc_ahead}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TAG=enc_ahead/h REPS=4 STEPS=10 bash tools/ab/ab_headline.sh || exit 1
TAG=enc_ahead/c4 REPS=3 STEPS=5 bash tools/ab/ab_c4.sh || exit 1
