#!/bin/bash
# T16 stores: nt (aux 2, shipped) vs the default cache policy (aux 0), C3 interleaved;
# then the C3 kernel stats of the shipped build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5_aux}
mkdir -p $O
for rep in 1 2; do
  for v in base aux0; do
    if [ $v = base ]; then L=""; else L="NERFHIP_LIB=nerf-rep_for_test_amd/lib/libnerfhip_$v.so"; fi
    env $L timeout -k 10 300 python bench.py --config c3 --steps 30 --warmup 5 --train-launch eager > $O/c3_${v}_$rep.log 2>&1 || exit $?
    echo "$v rep $rep $(tail -1 $O/c3_${v}_$rep.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c3 -- python bench.py --config c3 --steps 20 --warmup 5 --train-launch eager > $O/prof.log 2>&1 || exit $?
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-4 {} | head -14'
