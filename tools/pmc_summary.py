"""Reduce rocprofv3 PMC passes (tools/pmc.sh) to a per-kernel, per-launch summary.

    python tools/pmc_summary.py gpurun_out/<tag> profiles/<round>_pmc_summary.json \
        --workload H=800 W=800 N_samples=64 N_importance=128

Each pass directory p<i>/ holds pmc_counter_collection.csv (one row per
dispatch x counter). FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE
counts half the bytes of 16-B-per-lane streaming reads (glds and global_load
alike), so it is doubled (MI355X_MICROARCH.md, HBM section). WRITE_SIZE is
exact for 16-B-per-lane stores. bench.py reads the MLP entry's
``hbm_bytes_per_launch`` into roofline.traffic when the workload matches.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict

SHORT = {"mlp_fused_kernel": "mlp_fused", "mlp_x3_kernel": "mlp_x3", "composite_kernel": "composite",
         "composite_ert_kernel": "composite_ert", "sample_fine_kernel": "sample_fine",
         "rays_kernel": "rays", "coarse_kernel": "coarse", "ess_kernel": "ess",
         "grid_update_kernel": "grid_update",
         # C3 (the training step)
         "mlp_x3_train_kernel": "mlp_x3_train", "mlp_x3_bwd_kernel": "mlp_x3_bwd",
         "x3_wgrad_batch_kernel": "x3_wgrad_batch", "sum_partials_kernel": "sum_partials",
         "adam_kernel": "adam", "composite_train_fwd_kernel": "composite_train_fwd",
         "composite_train_bwd_kernel": "composite_train_bwd",
         "sample_pdf_bwd_kernel": "sample_pdf_bwd", "x3_pack": "x3_pack",
         "freq_encode_fm_backward_sum": "freq_encode_bwd_sum"}


def short(name):
    for k, v in SHORT.items():
        if k in name:
            return v
    return None


def collect(root):
    per = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [value per dispatch]
    meta = defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                if k is None:
                    continue
                per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                meta[k].update(grid=int(row["Grid_Size"]), wg=int(row["Workgroup_Size"]),
                               vgpr=int(row["VGPR_Count"]), lds=int(row["LDS_Block_Size"]))
    return per, meta


def summarise(per, meta):
    out = {}
    for k, counters in per.items():
        e = {"launches": max(len(v) for v in counters.values()), **meta[k]}
        mean = {c: sum(v) / len(v) for c, v in counters.items()}
        if "FETCH_SIZE" in mean:
            e["fetch_bytes_raw"] = mean["FETCH_SIZE"] * 1024
            e["fetch_bytes_corrected"] = 2 * e["fetch_bytes_raw"]
        if "WRITE_SIZE" in mean:
            e["write_bytes"] = mean["WRITE_SIZE"] * 1024
        if "fetch_bytes_corrected" in e and "write_bytes" in e:
            e["hbm_bytes_per_launch"] = e["fetch_bytes_corrected"] + e["write_bytes"]
        for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
                  "SQ_BUSY_CU_CYCLES", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT",
                  "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_VALU_MFMA_F32"):
            if c in mean:
                e[c] = mean[c]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in e and e.get("GRBM_GUI_ACTIVE"):
            # MFMA-busy share of the kernel's cycles: the counter sums over the
            # 1024 SIMDs, GRBM_GUI_ACTIVE over the 8 XCDs (MI355X_MICROARCH.md)
            e["mfma_busy_frac"] = (e["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024.0
                                   / (e["GRBM_GUI_ACTIVE"] / 8.0))
        out[k] = e
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("out")
    ap.add_argument("--workload", nargs="*", default=[])
    a = ap.parse_args()
    per, meta = collect(a.root)
    wl = {}
    for kv in a.workload:
        k, v = kv.split("=")
        wl[k] = int(v)
    doc = {"source": "rocprofv3 --pmc (one counter group per pass) over bench.py",
           "units": "bytes and counter values are means per launch; fetch corrected x2 (gfx950)",
           "workload": wl, "kernels": summarise(per, meta)}
    with open(a.out, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    print(json.dumps(doc["kernels"].get("mlp_fused", {}), indent=1))


if __name__ == "__main__":
    main()
