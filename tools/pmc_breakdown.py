"""Per-wave instruction mix and cycle shares of one kernel from rocprofv3 PMC
passes (tools/pmc.sh with SQ counter groups; one group per pass).

    python tools/pmc_breakdown.py gpurun_out/<tag> mlp_x3_kernel profiles/<out>.json

SQ_INSTS_* / SQ_WAVES: instructions issued per wave. SQ_WAIT_ANY,
SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_* over SQ_WAVE_CYCLES: the share of a wave's
resident cycles spent waiting on anything / on an instruction dependency
(s_waitcnt), or issuing an instruction of that class (the SQ counts them per
wave per 4-cycle quantum on gfx9; the ratios are what is read here).
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): MFMA-busy share
of the kernel's cycles (MI355X_MICROARCH.md)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(root, kernel, out):
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel in row["Kernel_Name"]:
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    mean = {k: sum(v) / len(v) for k, v in vals.items()}
    waves = mean.get("SQ_WAVES")
    doc = {"kernel": kernel, "source": root, "means_per_launch": mean, "per_wave": {},
           "share_of_wave_cycles": {}}
    if waves:
        for k, v in mean.items():
            if k.startswith("SQ_INSTS") or k.startswith("SQ_INST_CYCLES"):
                doc["per_wave"][k] = v / waves
    wc = mean.get("SQ_WAVE_CYCLES")
    if wc:
        for k, v in mean.items():
            if k.startswith("SQ_WAIT") or k.startswith("SQ_ACTIVE_INST") or k == "SQ_BUSY_CYCLES":
                doc["share_of_wave_cycles"][k] = v / wc
    if mean.get("SQ_VALU_MFMA_BUSY_CYCLES") and mean.get("GRBM_GUI_ACTIVE"):
        doc["mfma_busy_frac"] = mean["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (mean["GRBM_GUI_ACTIVE"] / 8)
    if mean.get("SQ_INSTS_LDS") and mean.get("SQ_LDS_BANK_CONFLICT") is not None:
        doc["lds_bank_conflict_cycles_per_lds_inst"] = mean["SQ_LDS_BANK_CONFLICT"] / mean["SQ_INSTS_LDS"]
    with open(out, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    print(json.dumps({k: doc[k] for k in ("per_wave", "share_of_wave_cycles")}, indent=1))
    print("mfma_busy_frac", doc.get("mfma_busy_frac"))


if __name__ == "__main__":
    main(*sys.argv[1:4])
