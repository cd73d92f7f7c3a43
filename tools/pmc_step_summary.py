"""Reduce rocprofv3 PMC passes over a C3 run (tools/pmc.sh with BENCH_ARGS
"--config c3 ...") to HBM bytes per TRAINING STEP, per kernel.

    python tools/pmc_step_summary.py gpurun_out/<tag> profiles/<round>_c3_pmc_summary.json

Steps = the number of adam_kernel dispatches (one per step). FETCH_SIZE is
doubled (gfx950, MI355X_MICROARCH.md HBM section), WRITE_SIZE taken as is.
bench.py's c3 record reads "hbm_bytes_per_step" into roofline.traffic.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(root, out):
    tot = defaultdict(lambda: defaultdict(float))
    for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"].split("(")[0].replace("void ", "")
                tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
                if r["Counter_Name"] == "WRITE_SIZE" and "adam_kernel" in name:
                    tot["_steps"]["n"] += 1
    steps = int(tot.pop("_steps")["n"])
    kernels = {}
    for k, c in tot.items():
        fb = 2.0 * c.get("FETCH_SIZE", 0.0) * 1024 / steps
        wb = c.get("WRITE_SIZE", 0.0) * 1024 / steps
        e = {"fetch_bytes_per_step": fb, "write_bytes_per_step": wb,
             "hbm_bytes_per_step": fb + wb}
        if c.get("GRBM_GUI_ACTIVE"):
            e["mfma_busy_frac"] = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / 1024 / (
                c["GRBM_GUI_ACTIVE"] / 8)
        kernels[k] = e
    doc = {"source": "rocprofv3 --pmc (FETCH_SIZE; WRITE_SIZE + SQ counters) over "
                     "bench.py --config c3 (eager steps)",
           "units": "bytes per training step (fetch corrected x2, gfx950)", "steps": steps,
           "workload": {"config": "c3", "N_rays": 1024, "N_samples": 64, "N_importance": 128},
           "hbm_bytes_per_step": sum(e["hbm_bytes_per_step"] for e in kernels.values()),
           "kernels": kernels}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    print(f"{steps} steps, {doc['hbm_bytes_per_step'] / 1e9:.3f} GB per step")


if __name__ == "__main__":
    main(*sys.argv[1:3])
