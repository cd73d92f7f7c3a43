#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/ubench/run.sh base now now2 small4 small16 || exit $?
for v in base now2 now; do
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/ubench/pmc_$v -o p -- ./tools/ubench/act_lds_$v > gpurun_out/ubench/pmc_$v.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob
for v in ("base", "now2", "now"):
    cs = glob.glob(f"gpurun_out/ubench/pmc_{v}/**/*counter_collection.csv", recursive=True)
    ks = glob.glob(f"gpurun_out/ubench/pmc_{v}/**/*kernel_trace.csv", recursive=True)
    if not cs:
        print(v, "no counter csv", glob.glob(f"gpurun_out/ubench/pmc_{v}/**/*", recursive=True)); continue
    rows = list(csv.DictReader(open(cs[0])))
    for r in rows:
        if r.get("Counter_Name") == "GRBM_GUI_ACTIVE":
            print(v, r.get("Dispatch_Id"), r["Counter_Name"], r["Counter_Value"])
    if ks:
        for r in csv.DictReader(open(ks[0])):
            print(v, "dispatch", r.get("Dispatch_Id"), "ns", int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
PY
