#!/bin/bash
# Round 6: the x3 kernels' head block in LDS with the bias / density-weight lane
# groups padded to 68 floats (no 2-way bank conflict on the epilogue's bias
# reads) -- the GPU suite, then the headline frame against the previous library
# (lib/libnerfhip_prev.so), interleaved, and one PMC pass of the LDS counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-headpad}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TAG=headpad/ab REPS=4 STEPS=10 bash tools/ab/ab_headline.sh || exit 1
for v in new prev; do
  if [ $v = new ]; then L=""; else L="NERFHIP_LIB=$PWD/nerf-rep_for_test_amd/lib/libnerfhip_prev.so"; fi
  env $L timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_$v -o p -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32-run --no-gt --no-c3 --no-c4 --no-perturb > $O/pmc_$v.log 2>&1 || { tail -5 $O/pmc_$v.log; exit 1; }
  python - $O/pmc_$v $v <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
s = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(f)):
    if "mlp_x3_kernel" in r["Kernel_Name"]:
        s[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print(sys.argv[2], {k: s[k] for k in s})
PY
done
