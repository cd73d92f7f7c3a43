#!/bin/bash
# Timing-only A/B of the training layer kernel (x3_layer_kernel): builds whole
# libraries with its C stores (X3L_ABL_NOSTORE) or B loads (X3L_ABL_NOLOAD)
# dropped by a zero-record buffer descriptor, then (run) times the 8-layer
# forward / dgrad chains of tools/ic_chunk_bench.py with each (NERFHIP_LIB);
# X3L_ABL_NOWAIT drops the tile-end vmcnt(0) (the store drain overlaps the next
# tile; the first two slices of a tile may then read unlanded weights).
#   bash tools/layer_ablate.sh build      # CPU
#   bash tools/layer_ablate.sh run        # GPU
set -u
cd "$(dirname "$0")/.."
P=nerf-rep_for_test_amd
OUT=$P/build/abl
if [ "${1:-run}" = build ]; then
  mkdir -p $OUT
  for v in ${VARIANTS:-NOSTORE NOLOAD NOWAIT}; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off \
      -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -shared -DX3L_ABL_$v \
      $P/csrc/runtime.hip $P/csrc/render_kernels.hip $P/csrc/mlp_fused.hip $P/csrc/mlp_x3.hip \
      $P/csrc/train_kernels.hip $P/csrc/kilonerf_ops.hip -o $OUT/libnerfhip_$v.so &
  done
  wait
  ls -la $OUT
else
  for r in 1 2; do
    for v in base ${VARIANTS:-NOSTORE NOLOAD NOWAIT}; do
      lib=$P/lib/libnerfhip.so; [ $v != base ] && lib=$OUT/libnerfhip_$v.so
      echo "$v $(NERFHIP_LIB=$lib timeout -k 10 120 python tools/ic_chunk_bench.py 1 2>/dev/null | tail -1)"
    done
  done
fi
