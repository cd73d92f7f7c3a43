#!/bin/bash
# store_pattern.hip: time and TCC write requests of three activation-store layouts
set -u
cd "$(dirname "$0")"
OUT=${OUT:-../../gpurun_out/store_pattern}
mkdir -p "$OUT"
export TMPDIR=/tmp
for m in 0 1 2; do for a in 0 2; do
  timeout -k 5 60 ./store_pattern $m $a 50 || exit 1
done; done | tee "$OUT/time.log"
for m in 0 1 2; do for a in 0 2; do
  timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-trace \
    --output-format csv -d "$OUT/p_${m}_${a}" -o pmc -- ./store_pattern $m $a 5 > "$OUT/p_${m}_${a}.log" 2>&1 || exit 1
done; done
echo ok
