#!/bin/bash
# Timing-only ablation of the fused training forward's activation stores
# (tools/ab/time_train_fwd.py) against two libraries built from temporary patches
# of csrc/mlp_x3.hip (not kept in the tree): libnerfhip_nostore.so, whose
# ActStore::pair returns at once (no stores), and libnerfhip_zerorec.so, whose
# rows_rsrc gives zero-record descriptors (stores issued, dropped by the range
# check). Build each with the Makefile's flags from the patched file and link
# it with the other objects of build/.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/abl2
for v in base nostore zerorec base nostore zerorec; do
  if [ $v = base ]; then unset NERFHIP_LIB; else export NERFHIP_LIB=$PWD/nerf-rep_for_test_amd/lib/libnerfhip_$v.so; fi
  echo "== $v"; timeout -k 10 120 python tools/ab/time_train_fwd.py 196608 20 2>&1 | tail -3 || exit $?
done
